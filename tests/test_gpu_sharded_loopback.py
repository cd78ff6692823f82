"""The landmark-sharded BA data path on one device (in-process loopback communicator).

RCCL refuses two ranks on one GPU, so the N > 1 path of ``vo_comm_init`` + ``vo_ba_run``
cannot run on a one-GPU box.  ``vo_comm_init_loopback`` puts N contexts of one process
(one host thread each) in a group whose all-reduces go through host memory in rank
order; everything else is the production path: per-rank plans over the rank's landmark
shard (``shard.py``), the min all-reduce of the profile envelope at setup, the damping on
rank 0 only, the per-iteration sum of [S | b | cost], the replicated dense solve and the
per-shard back substitution.  The result must match the unsharded run.
"""

import threading

import numpy as np
import pytest

from visualodometry_amd import _lib
from visualodometry_amd.ba import BASession
from visualodometry_amd.shard import shard
from visualodometry_amd.synthetic import make_ba_config

pytestmark = pytest.mark.gpu


def _unsharded(p, iters, lam):
    s = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, lam, _lib.Context(0))
    s.set_state(p.poses_cw, p.points)
    rc, costs = s.run(iters)
    poses, pts = s.get_state()
    return rc, costs, poses, pts


def _sharded(p, nranks, iters, lam, group):
    out = [None] * nranks
    errors = []

    def worker(r):
        try:
            ctx = _lib.Context(0)
            _lib.comm_init_loopback(ctx, nranks, r, group)
            (p0, p1), ptr, cam, uv, pts = shard(p.point_ptr, p.obs_cam, p.obs_uv, p.points, nranks, r)
            s = BASession(p.K, ptr, cam, uv, p.n_poses, p.n_fixed, lam, ctx)
            s.set_state(p.poses_cw, pts)
            rc, costs = s.run(iters)
            poses, q = s.get_state()
            out[r] = (p0, p1, rc, costs, poses, q)
        except Exception as e:  # surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "loopback group deadlocked"
    if errors:
        raise errors[0]
    return out


@pytest.mark.parametrize("cfg,nranks", [("cfg2", 2), ("cfg2", 3), ("cfg3", 2), ("cfg3", 4), ("cfg3", 8),
                                        ("cfg4", 2), ("cfg4", 4), ("cfg4", 8)])
def test_sharded_matches_unsharded(cfg, nranks):
    p = make_ba_config(cfg)
    iters, lam = (3 if cfg == "cfg4" else 5), 1.0  # cfg4 = BASELINE config 4, 100 x 200k
    rc0, c0, P0, X0 = _unsharded(p, iters, lam)
    res = _sharded(p, nranks, iters, lam, f"vo-loopback-{cfg}-{nranks}".encode())
    # every rank solved the same reduced system: identical poses and cost trajectories
    for r in range(1, nranks):
        assert res[r][2] == res[0][2]
        np.testing.assert_array_equal(res[r][3], res[0][3])
        np.testing.assert_array_equal(res[r][4], res[0][4])
    assert res[0][2] == rc0
    # against the unsharded run: only the summation order of S, b and the cost differs
    np.testing.assert_allclose(res[0][3], c0, rtol=1e-9)
    np.testing.assert_allclose(res[0][4], P0, rtol=1e-8, atol=1e-10)
    X = np.concatenate([q for (_, _, _, _, _, q) in res])
    assert X.shape == X0.shape
    np.testing.assert_allclose(X, X0, rtol=1e-8, atol=1e-10)
    for r, (p0, p1, *_rest) in enumerate(res):
        assert p1 - p0 == res[r][5].shape[0]


def test_loopback_one_rank_is_neutral():
    p = make_ba_config("cfg2")
    _, c0, P0, X0 = _unsharded(p, 3, 1.0)
    res = _sharded(p, 1, 3, 1.0, b"vo-loopback-single")
    np.testing.assert_array_equal(res[0][3], c0)
    np.testing.assert_array_equal(res[0][4], P0)
    np.testing.assert_array_equal(res[0][5], X0)


def test_one_invalid_shard_fails_every_rank():
    """Only rank 1's shard is invalid (an observation of a camera outside the window):
    every rank's vo_ba_setup fails with VO_ERR_ARG -- none is left waiting in a
    collective."""
    p = make_ba_config("cfg2")
    nranks = 2
    codes = [None] * nranks

    def worker(r):
        ctx = _lib.Context(0)
        _lib.comm_init_loopback(ctx, nranks, r, b"vo-loopback-invalid")
        (_p0, _p1), ptr, cam, uv, _pts = shard(p.point_ptr, p.obs_cam, p.obs_uv, p.points, nranks, r)
        cam = cam.copy()
        if r == 1:
            cam[0] = p.n_poses + 3
        try:
            BASession(p.K, ptr, cam, uv, p.n_poses, p.n_fixed, 1.0, ctx)
            codes[r] = 0
        except _lib.VoError as e:
            codes[r] = e.code

    th = [threading.Thread(target=worker, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a rank is stuck in a collective"
    assert codes == [_lib.VO_ERR_ARG] * nranks
