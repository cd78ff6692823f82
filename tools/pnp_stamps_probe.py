import sys
sys.path.insert(0, '.')
from visualodometry_amd import _lib, pnp
from visualodometry_amd.synthetic import pnp_case
ctx = _lib.context(0)
X, uv, K, _, _ = pnp_case(1000, 5)
for _ in range(3):
    pnp.pnp_ransac(X, uv, K, 1.0, ctx=ctx)
