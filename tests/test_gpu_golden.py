"""The committed golden fixtures replayed through the HIP path (C-ABI, libvo_hip.so).

``tests/golden/*.npz`` pin the oracle (tests/test_oracle_*.py); here the product path
must reproduce the same vectors: matcher indices, fp32 distance bits and ratio-test
pairs bit-exact, and the BA step's reduced system, pose update and
cost trajectory within the north-star 1e-5 relative bar.
"""

import numpy as np
import pytest

from tests.conftest import GOLDEN
from visualodometry_amd import _lib, matcher
from visualodometry_amd.ba import BASession

pytestmark = pytest.mark.gpu
REL = 1e-5


@pytest.fixture(scope="module")
def ctx():
    return _lib.Context(0)


def test_golden_sift_512_hip(ctx):
    g = np.load(GOLDEN / "match_sift_512.npz")
    d0, d1 = g["des0"].astype(np.float32), g["des1"].astype(np.float32)
    idx, dist = matcher.match_knn2(d0, d1, ctx=ctx)
    np.testing.assert_array_equal(idx, g["idx"])
    np.testing.assert_array_equal(np.asarray(dist, np.float32).view(np.uint32), g["dist"].view(np.uint32))
    np.testing.assert_array_equal(matcher.match_knn2_ratio(d0, d1, ctx=ctx), g["pairs"])


@pytest.mark.parametrize("case", ["ties", "n1_eq_1", "n1_eq_2", "many_to_one", "sqrt_collision"])
def test_golden_kats_hip(ctx, case):
    g = np.load(GOLDEN / "match_kat.npz")
    a, b = g[f"{case}_des0"], g[f"{case}_des1"]
    idx, dist = matcher.match_knn2(a, b, ctx=ctx)
    np.testing.assert_array_equal(idx, g[f"{case}_idx"])
    np.testing.assert_array_equal(np.asarray(dist, np.float32), g[f"{case}_dist"])
    np.testing.assert_array_equal(matcher.match_knn2_ratio(a, b, ctx=ctx), g[f"{case}_pairs"])


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def test_golden_ba_small_hip(ctx):
    g = np.load(GOLDEN / "ba_small.npz")
    N, nf, lam = g["poses_cw"].shape[0], int(g["n_fixed"]), float(g["lam"])
    s = BASession(g["K"], g["point_ptr"], g["obs_cam"], g["obs_uv"], N, nf, lam, ctx)
    s.set_state(g["poses_cw"], g["points"])
    rc, S, b, dc, cost = s.gn_step()
    assert rc == _lib.VO_OK
    assert _rel(S, g["S"]) < 1e-9
    assert _rel(dc, g["dc"]) < REL
    np.testing.assert_allclose(cost, g["cost0"], rtol=1e-10)
    s2 = BASession(g["K"], g["point_ptr"], g["obs_cam"], g["obs_uv"], N, nf, lam, ctx)
    s2.set_state(g["poses_cw"], g["points"])
    rc, costs = s2.run(len(g["costs"]) - 1)
    assert rc == _lib.VO_OK
    np.testing.assert_allclose(costs, g["costs"], rtol=REL)
