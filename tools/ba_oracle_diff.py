"""Diagnostic: relative differences of a BA run (HIP) against the C oracle, per iteration.
    python tools/ba_oracle_diff.py [cfg] [iters]   (VO_LIB_PATH selects the library build)"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import cref  # noqa: E402
from visualodometry_amd import _lib  # noqa: E402
from visualodometry_amd.ba import BASession  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
p = make_ba_config(cfg)
ctx = _lib.context(0)
R = cref.BAProblemRef(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0)
for it in range(1, iters + 1):
    s = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0, ctx)
    s.set_state(p.poses_cw, p.points)
    rc, costs = s.run(it)
    P, X = s.get_state()
    n, Pr, Xr, cr = R.solve(p.poses_cw, p.points, it, nthreads=8)
    rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())
    print(f"{cfg} iters {it}: cost rel {np.abs(costs - cr).max() / np.abs(cr).max():.3e} "
          f"last cost rel {abs(costs[-1] - cr[-1]) / abs(cr[-1]):.3e} dP rel {rel(P - p.poses_cw, Pr - p.poses_cw):.3e} "
          f"X rel {rel(X, Xr):.3e}")
