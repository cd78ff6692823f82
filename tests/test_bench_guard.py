"""bench.py's untimed BA parity guard (CPU): a session that reproduces the C oracle passes, one
whose results are off by more than the north-star 1e-5 (or that fails) is rejected, so a
wrong-result build cannot print a GN-iters/s number."""
import numpy as np

import bench
from oracle import cref
from visualodometry_amd import _lib
from visualodometry_amd.synthetic import make_ba_problem


class FakeSession:
    """Stands in for BASession: returns the oracle's own results, optionally perturbed."""

    def __init__(self, p, lam, scale=0.0, rc=_lib.VO_OK):
        self.p, self.lam, self.scale, self.rc = p, lam, scale, rc

    def set_state(self, poses, points):
        # a sharded session holds only its landmarks; the fake solves the whole window
        self.start = (self.p.poses_cw.copy(), self.p.points.copy())

    def run(self, iters):
        p = self.p
        R = cref.BAProblemRef(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, self.lam)
        _, self.P, self.X, c = R.solve(self.start[0], self.start[1], iters, nthreads=2)
        self.X = self.X * (1.0 + self.scale)
        return self.rc, np.asarray(c)

    def get_state(self):
        return self.P, self.X


def test_guard_accepts_oracle_and_rejects_drift():
    p = make_ba_problem(6, 200, 9)
    L = p.points.shape[0]
    ok = bench.ba_parity_guard(FakeSession(p, 1.0), p, p.points, 0, L, 1.0)
    assert ok["ok"] and max(ok["rel_err"].values()) < 1e-12
    bad = bench.ba_parity_guard(FakeSession(p, 1.0, scale=1e-4), p, p.points, 0, L, 1.0)
    assert not bad["ok"] and bad["rel_err"]["points"] > 1e-5
    failed = bench.ba_parity_guard(FakeSession(p, 1.0, rc=_lib.VO_ERR_NOT_SPD), p, p.points, 0, L, 1.0)
    assert not failed["ok"]


def test_guard_checks_this_ranks_shard():
    p = make_ba_problem(6, 200, 9)
    L = p.points.shape[0]
    s = FakeSession(p, 1.0)

    class Shard(FakeSession):
        def get_state(self):
            P, X = super().get_state()
            return P, X[50:120]

    g = bench.ba_parity_guard(Shard(p, 1.0), p, p.points[50:120], 50, 120, 1.0)
    assert g["ok"]
    g = bench.ba_parity_guard(Shard(p, 1.0), p, p.points[50:120], 60, 130, 1.0)
    assert not g["ok"]
    del s, L
