"""GPU parity of the BA Gauss-Newton step (vo_ba_*) against the CPU oracles.

Tolerances (north star): residual costs and pose/point updates within 1e-5
relative; the fp64 kernels actually agree to ~1e-10 (different summation
order only), which the tighter asserts below document.
"""

import numpy as np
import pytest

from oracle import ba_ref, cref
from visualodometry_amd import _lib
from visualodometry_amd._lib import VoError
from visualodometry_amd.ba import BASession, BAWindow, SlidingWindowBA
from visualodometry_amd.synthetic import make_ba_config, make_ba_problem

pytestmark = pytest.mark.gpu

# chunks per segment of the default one-wave K1 plan (BAEngine::wave_chunks): six while the
# segments fit one round (cfg3), three for windows of several rounds (cfg4)
WAVE_CHUNKS = {"cfg3": 6, "cfg4": 3}
REL = 1e-5  # north-star tolerance for residuals and pose updates


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def _session(p, ctx, lam=1.0):
    s = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, lam, ctx)
    s.set_state(p.poses_cw, p.points)
    return s


@pytest.mark.parametrize("lam", [0.0, 1.0])
def test_step_matches_numpy_oracle(ctx, lam):
    p = make_ba_problem(8, 300, 21)
    s = _session(p, ctx, lam)
    rc, S, b, dc, cost = s.gn_step()
    assert rc == _lib.VO_OK
    st = ba_ref.BAState.from_poses(p.poses_cw, p.points)
    struct = ba_ref.BAStructure(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_fixed, p.n_poses)
    ref = ba_ref.gn_step(st, struct, lam)
    assert abs(cost - ref.system.cost) <= 1e-12 * ref.system.cost
    assert _rel(S, ref.system.S) < 1e-11
    assert _rel(b, ref.system.b) < 1e-10
    assert _rel(dc, ref.dc) < 1e-8
    P, X = s.get_state()
    assert _rel(P, ref.state.poses_cw()) < 1e-10
    assert _rel(X, ref.state.X) < 1e-8


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_run_matches_c_oracle(ctx, cfg):
    p = make_ba_config(cfg)
    iters = 5
    s = _session(p, ctx)
    st = s.plan_stats()
    if cfg == "cfg3":  # the default plan: six-chunk segments, one round
        assert st["chunks"] == WAVE_CHUNKS["cfg3"] * st["segments"] and st["segments"] <= 256, st
    rc, costs = s.run(iters)
    assert rc == _lib.VO_OK
    P, X = s.get_state()
    R = cref.BAProblemRef(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0)
    n, Pr, Xr, cr = R.solve(p.poses_cw, p.points, iters, nthreads=8)
    assert n == iters
    np.testing.assert_allclose(costs, cr, rtol=REL)
    assert _rel(costs, cr) < 1e-9
    assert _rel(P, Pr) < REL
    assert _rel(X, Xr) < REL
    # pose updates (relative to the start) within 1e-5 relative
    dP, dPr = P - p.poses_cw, Pr - p.poses_cw
    assert _rel(dP, dPr) < REL


def test_cfg4_matches_c_oracle(ctx):
    """100 poses x 200k landmarks: the profile (225 KB) exceeds LDS; the banded K3 streams
    it through its LDS rings.  K1 is the default one-wave K1 (three chunks of one first-camera
    group per segment: 4.6k workgroups of three waves, nine rounds)."""
    p = make_ba_config("cfg4")
    s = _session(p, ctx)
    st = s.plan_stats()
    assert st["profile_blocks"] * 288 > 150 * 1024
    assert st["band_solver"] == 1
    assert st["seg_obs"] == 1 and st["chunks"] == WAVE_CHUNKS["cfg4"] * st["segments"], st
    rc, costs = s.run(3)
    assert rc == _lib.VO_OK
    R = cref.BAProblemRef(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0)
    n, Pr, Xr, cr = R.solve(p.poses_cw, p.points, 3, nthreads=8)
    np.testing.assert_allclose(costs, cr, rtol=REL)
    P, X = s.get_state()
    assert _rel(P, Pr) < REL and _rel(X, Xr) < REL


@pytest.mark.parametrize("cfg", ["cfg3", "cfg4"])
def test_four_wave_k1_matches_c_oracle(ctx, cfg):
    """The four-wave K1 (multi-chunk segments, one 256-lane workgroup walking them; reached
    through the testing switch vo_ba_testing_k1_four_wave) against the C oracle, and against the
    default one-wave K1 to rounding (the summation order differs)."""
    p = make_ba_config(cfg)
    iters = 3
    R = cref.BAProblemRef(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0)
    n, Pr, Xr, cr = R.solve(p.poses_cw, p.points, iters, nthreads=8)
    out = []
    for four in (True, False):
        _lib.ba_testing_k1(ctx, -1 if four else 0)
        try:
            s = _session(p, ctx)
            st = s.plan_stats()
            assert (st["seg_obs"] > 1 and st["segments"] < st["chunks"]) == four, st
            rc, costs = s.run(iters)
            assert rc == _lib.VO_OK
            P, X = s.get_state()
        finally:
            _lib.ba_testing_k1(ctx, 0)
        np.testing.assert_allclose(costs, cr, rtol=REL)
        assert _rel(P, Pr) < REL and _rel(X, Xr) < REL
        out.append((costs, P, X))
    assert _rel(out[0][0], out[1][0]) < 1e-9
    assert _rel(out[0][1], out[1][1]) < 1e-8


@pytest.mark.parametrize("cfg,nch", [("cfg2", 2), ("cfg3", 2), ("cfg3", 3), ("cfg4", 2), ("cfg4", 3), ("cfg2", 6),
                                     ("cfg3", 6)])
def test_group_segment_k1_matches_c_oracle(ctx, cfg, nch):
    """The one-wave K1 with nch chunks of one first-camera group per segment (testing switch
    vo_ba_testing_k1(ctx, nch)): the segment's waves sum their slot blocks in LDS in chunk order
    into one slab row per segment slot.  Against the C oracle, the one-chunk plan to rounding,
    and bitwise reproducible."""
    p = make_ba_config(cfg)
    iters = 3
    R = cref.BAProblemRef(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0)
    n, Pr, Xr, cr = R.solve(p.poses_cw, p.points, iters, nthreads=8)
    out = []
    for variant in (nch, nch, 1):
        _lib.ba_testing_k1(ctx, variant)
        try:
            s = _session(p, ctx)
            st = s.plan_stats()
            assert st["seg_obs"] == 1 and st["chunks"] == variant * st["segments"], st
            rc, costs = s.run(iters)
            assert rc == _lib.VO_OK
            P, X = s.get_state()
        finally:
            _lib.ba_testing_k1(ctx, 0)
        np.testing.assert_allclose(costs, cr, rtol=REL)
        assert _rel(P, Pr) < REL and _rel(X, Xr) < REL
        out.append((costs, P, X, st["slab_blocks"]))
    for a_, b_ in zip(out[0][:3], out[1][:3]):
        np.testing.assert_array_equal(a_, b_)
    assert _rel(out[0][0], out[2][0]) < 1e-9
    assert out[0][3] < 0.6 * out[2][3]  # slab rows: one per segment slot


def test_deterministic_bitwise(ctx):
    p = make_ba_config("cfg2")
    out = []
    for _ in range(2):
        s = _session(p, ctx)
        rc, costs = s.run(4)
        P, X = s.get_state()
        out.append((costs, P, X))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


def test_reserve_then_window_equals_plain(ctx):
    """vo_ba_reserve pre-sizes the context (a synthetic window set up twice, then dropped): the
    next window's results are bitwise those of a context that never reserved, the reserved
    context holds no problem, and a window larger than the reservation still runs."""
    p = make_ba_config("cfg2")
    ref_s = _session(p, ctx)
    rc0, c0 = ref_s.run(4)
    P0, X0 = ref_s.get_state()
    fresh = _lib.Context(ctx.device)
    _lib.ba_reserve(fresh, p.n_poses, p.n_points, p.n_obs, p.n_fixed)
    with pytest.raises(VoError):  # no problem after a reservation
        _lib.check(fresh.lib.vo_ba_run(fresh.handle, 0, 1, None), "vo_ba_run")
    s = _session(p, fresh)
    rc1, c1 = s.run(4)
    P1, X1 = s.get_state()
    assert rc0 == rc1 == _lib.VO_OK
    np.testing.assert_array_equal(c0, c1)
    np.testing.assert_array_equal(P0, P1)
    np.testing.assert_array_equal(X0, X1)
    big = make_ba_config("cfg3")  # larger than the reservation: grows
    s = _session(big, fresh)
    rc2, c2 = s.run(2)
    assert rc2 == _lib.VO_OK and np.all(np.isfinite(c2))
    with pytest.raises(VoError):
        _lib.ba_reserve(fresh, 1, 10, 20, 0)  # bad sizes
    fresh.close()


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "tiny"])
def test_fused_reduce_equals_split_launches(ctx, cfg):
    """One rank runs K2 inside the banded K3's launch (reducer workgroups hand the reduced
    system to the solver workgroup); the split layout of N > 1 ranks launches K2 on its own.
    Same sums in the same order: the runs agree bit for bit, and the fused one is the default."""
    p = make_ba_problem(4, 160, 35, max_track=2) if cfg == "tiny" else make_ba_config(cfg)
    out = []
    for split in (False, True):
        _lib.ba_split_reduce(ctx, split)
        try:
            _lib.profile_enable(ctx, True)
            s = _session(p, ctx)
            rc, costs = s.run(3)
            assert rc == _lib.VO_OK
            P, X = s.get_state()
            prof = _lib.profile_read(ctx)
            _lib.profile_enable(ctx, False)
        finally:
            _lib.ba_split_reduce(ctx, False)
        assert ("ba_reduce" in prof) == split
        assert s.plan_stats()["band_solver"] == 1
        out.append((costs, P, X))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


def test_fused_handoff_stress(ctx):
    """The fused launch's solver reads its reducers' columns without an acquire fence (sc1 loads
    after its own poll of each column's counter).  A stale line anywhere would change the bits:
    60 GN iterations of cfg3 (60 launches, each with 178 reducers spread over every XCD) must
    equal the split launches (K2 on its own, read after a kernel boundary) bit for bit, cost by
    cost, and the state after them."""
    p = make_ba_config("cfg3")
    out = []
    for split in (False, True):
        _lib.ba_split_reduce(ctx, split)
        try:
            s = _session(p, ctx)
            rc, costs = s.run(60)
            assert rc == _lib.VO_OK
            out.append((costs,) + s.get_state())
        finally:
            _lib.ba_split_reduce(ctx, False)
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


def test_split_layout_equals_ring(ctx):
    """cfg4's window (F = 98, too large for one workgroup's LDS) on the split layout (one
    workgroup per side, each side's columns in its own CU's LDS, three global-memory hand-offs per
    launch) and on the ring layout (one workgroup, factor records in global memory): the same
    arithmetic in the same order, so the same bits over 30 GN iterations (30 launches, each
    workgroup pair possibly on two XCDs), cost by cost, and the state after them."""
    p = make_ba_config("cfg4")
    out = []
    for no_split in (False, True):
        _lib.ba_testing_no_split(ctx, no_split)
        try:
            s = _session(p, ctx)
            assert s.plan_stats()["band_mode"] == ("ring" if no_split else "split")
            rc, costs = s.run(30)
            assert rc == _lib.VO_OK
            out.append((costs,) + s.get_state())
        finally:
            _lib.ba_testing_no_split(ctx, False)
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("n_poses,max_track,mode", [(50, 8, "full"), (100, 8, "split"), (100, 4, "full"),
                                                    (140, 6, "split"), (200, 8, "ring")])
def test_band_layout_modes(ctx, n_poses, max_track, mode):
    """The banded K3's layouts by window size (one workgroup with every column in LDS; one
    workgroup per side; the ring with records in global memory): one GN step against the numpy
    oracle's dense Cholesky."""
    p = make_ba_problem(n_poses, 30 * n_poses, 5 + n_poses, max_track=max_track)
    s = _step_vs_oracle(ctx, p)
    assert s.plan_stats()["band_mode"] == mode


def test_run_in_pieces_equals_one_run(ctx):
    p = make_ba_config("cfg2")
    s1 = _session(p, ctx)
    s1.run(4)
    P1, X1 = s1.get_state()
    s2 = _session(p, ctx)
    s2.run_async(2)
    s2.run_async(2)
    s2.synchronize()
    P2, X2 = s2.get_state()
    np.testing.assert_array_equal(P1, P2)
    np.testing.assert_array_equal(X1, X2)


def test_degenerate_landmarks_frozen(ctx):
    """1-observation landmarks, landmarks seen only by fixed cameras and duplicate
    (landmark, camera) observations, checked against the oracle."""
    p = make_ba_problem(6, 120, 31)
    pp, cam, uv = list(p.point_ptr), p.obs_cam.copy(), p.obs_uv.copy()
    L = p.n_points
    # landmark 0: keep only its first observation
    keep = np.ones(cam.size, bool)
    keep[pp[0] + 1 : pp[1]] = False
    # landmark 1: duplicate its first observation (same camera twice)
    dup_idx = pp[1]
    cam2 = np.insert(cam[keep], 1, cam[dup_idx])
    uv2 = np.insert(uv[keep], 1, uv[dup_idx] + 0.5, axis=0)
    counts = np.diff(np.array(pp))
    counts[0] = 1
    counts[1] += 1
    ptr2 = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    # landmark 2: move all observations to fixed cameras 0/1
    cam2[ptr2[2] : ptr2[3]] = np.arange(ptr2[3] - ptr2[2]) % 2
    s = BASession(p.K, ptr2, cam2, uv2, p.n_poses, 2, 0.0, ctx)  # no damping: 1-obs V is singular
    s.set_state(p.poses_cw, p.points)
    rc, S, b, dc, cost = s.gn_step()
    assert rc == _lib.VO_OK
    st = ba_ref.BAState.from_poses(p.poses_cw, p.points)
    struct = ba_ref.BAStructure(p.K, ptr2, cam2, uv2, 2, p.n_poses)
    ref = ba_ref.gn_step(st, struct, 0.0)
    assert not ref.system.valid[0]
    assert _rel(S, ref.system.S) < 1e-11
    assert _rel(dc, ref.dc) < 1e-8
    P, X = s.get_state()
    assert _rel(X, ref.state.X) < 1e-8
    np.testing.assert_array_equal(X[0], p.points[0])  # frozen landmark unchanged
    assert L == X.shape[0]


def test_not_spd_reported(ctx):
    """A free camera with no observations and no damping: S is singular."""
    p = make_ba_problem(6, 100, 41)
    cam = p.obs_cam.copy()
    cam[cam == 5] = 4
    s = BASession(p.K, p.point_ptr, cam, p.obs_uv, p.n_poses, 2, 0.0, ctx)
    s.set_state(p.poses_cw, p.points)
    rc, costs = s.run(3)
    assert rc == _lib.VO_ERR_NOT_SPD
    assert np.isfinite(costs[0]) and np.isnan(costs[1:]).all()
    P, X = s.get_state()
    np.testing.assert_array_equal(P, _pose_round(p.poses_cw))
    np.testing.assert_array_equal(X, p.points)


def test_fused_reduce_after_failed_solve(ctx):
    """A failed (not SPD) fused launch still counts every reducer and gives the count back:
    the next window on the same context runs the fused launch to the split launches' bits."""
    p = make_ba_problem(6, 100, 41)
    cam = p.obs_cam.copy()
    cam[cam == 5] = 4
    bad = BASession(p.K, p.point_ptr, cam, p.obs_uv, p.n_poses, 2, 0.0, ctx)
    bad.set_state(p.poses_cw, p.points)
    assert bad.run(3)[0] == _lib.VO_ERR_NOT_SPD
    q = make_ba_config("cfg2")
    out = []
    for split in (False, True):
        _lib.ba_split_reduce(ctx, split)
        try:
            s = _session(q, ctx)
            rc, costs = s.run(2)
            assert rc == _lib.VO_OK
            out.append((costs,) + tuple(s.get_state()))
        finally:
            _lib.ba_split_reduce(ctx, False)
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


def _fused_equals_split(ctx, q, iters=2):
    out = []
    for split in (False, True):
        _lib.ba_split_reduce(ctx, split)
        try:
            s = _session(q, ctx)
            rc, costs = s.run(iters)
            assert rc == _lib.VO_OK
            out.append((costs,) + tuple(s.get_state()))
        finally:
            _lib.ba_split_reduce(ctx, False)
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


def test_fused_reduce_timeout_fails_loudly_and_recovers(ctx):
    """The fused launch's bounded wait (csrc/ba_band.hip band_wait_reduced): with one reducer
    workgroup left out of every launch (test switch) the solver gives up, vo_ba_run fails with
    VO_ERR_HIP naming the timeout, and the state stays at the failed iteration's linearisation
    point.  The host re-zeroes the reducer counter, so the next window on the same context runs
    the fused launch to the split launches' bits."""
    p = make_ba_config("cfg2")
    s = _session(p, ctx)
    assert s.plan_stats()["band_solver"] == 1
    _lib.ba_testing_drop_reducers(ctx, 1)
    try:
        with pytest.raises(_lib.VoError, match="timed out"):
            s.run(2)
    finally:
        _lib.ba_testing_drop_reducers(ctx, 0)
    P, X = s.get_state()
    np.testing.assert_array_equal(P, _pose_round(p.poses_cw))
    np.testing.assert_array_equal(X, p.points)
    _fused_equals_split(ctx, p)


def test_fused_reduce_timeout_after_failed_solve(ctx):
    """A timeout in a launch whose earlier iteration already failed (not SPD) is still recorded
    (ADVICE r3): the launches after the failure count their reducers, the host re-zeroes the
    counter on any failed status, and the next window is exact."""
    p = make_ba_problem(6, 100, 41)
    cam = p.obs_cam.copy()
    cam[cam == 5] = 4
    bad = BASession(p.K, p.point_ptr, cam, p.obs_uv, p.n_poses, 2, 0.0, ctx)
    bad.set_state(p.poses_cw, p.points)
    if bad.plan_stats()["band_solver"] != 1:
        pytest.skip("window not on the banded solver")
    _lib.ba_testing_drop_reducers(ctx, 1)
    try:
        with pytest.raises(_lib.VoError, match="timed out"):
            bad.run(3)
    finally:
        _lib.ba_testing_drop_reducers(ctx, 0)
    # a not-SPD run without the switch: its later launches count every reducer
    bad.set_state(p.poses_cw, p.points)
    assert bad.run(3)[0] == _lib.VO_ERR_NOT_SPD
    _fused_equals_split(ctx, make_ba_config("cfg2"))


def _pose_round(P):
    from visualodometry_amd.ba import poses_to_rt, rt_to_poses

    return rt_to_poses(poses_to_rt(P))


def test_all_fixed_and_empty(ctx):
    p = make_ba_problem(4, 50, 51)
    s = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, 4, 4, 1.0, ctx)  # F = 0
    s.set_state(p.poses_cw, p.points)
    rc, costs = s.run(2)
    assert rc == _lib.VO_OK
    struct = ba_ref.BAStructure(p.K, p.point_ptr, p.obs_cam, p.obs_uv, 4, 4)
    st, cr = ba_ref.solve(ba_ref.BAState.from_poses(p.poses_cw, p.points), struct, 2, 1.0)
    np.testing.assert_allclose(costs, cr, rtol=1e-9)
    ba = SlidingWindowBA(p.K, iters=2)
    res = ba.optimize(BAWindow(p.poses_cw, p.points[:0], p.obs_uv[:0], p.obs_cam[:0],
                               p.obs_cam[:0], 2))
    assert res.status == "skipped"


def test_sliding_window_api(ctx):
    p = make_ba_problem(10, 400, 61)
    obs_pt = p.obs_point()
    perm = np.random.default_rng(0).permutation(obs_pt.size)  # any observation order
    w = BAWindow(p.poses_cw, p.points, p.obs_uv[perm], p.obs_cam[perm], obs_pt[perm], 2)
    res = SlidingWindowBA(p.K, iters=4, lam=1.0).optimize(w)
    assert res.status == "ok"
    struct = ba_ref.BAStructure(p.K, p.point_ptr, p.obs_cam, p.obs_uv, 2, p.n_poses)
    st, cr = ba_ref.solve(ba_ref.BAState.from_poses(p.poses_cw, p.points), struct, 4, 1.0)
    np.testing.assert_allclose(res.cost_per_iter, cr, rtol=1e-8)
    assert _rel(res.poses_cw, st.poses_cw()) < REL
    assert _rel(res.points, st.X) < REL


def _step_vs_oracle(ctx, p, lam=1.0):
    s = _session(p, ctx, lam)
    rc, S, b, dc, cost = s.gn_step()
    assert rc == _lib.VO_OK
    st = ba_ref.BAState.from_poses(p.poses_cw, p.points)
    struct = ba_ref.BAStructure(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_fixed, p.n_poses)
    ref = ba_ref.gn_step(st, struct, lam)
    assert _rel(S, ref.system.S) < 1e-11
    assert _rel(dc, ref.dc) < 1e-8
    P, X = s.get_state()
    assert _rel(P, ref.state.poses_cw()) < 1e-10
    assert _rel(X, ref.state.X) < 1e-8
    return s


@pytest.mark.parametrize("n_poses,max_track", [(3, 2), (4, 2), (6, 8), (12, 3), (16, 8), (18, 8),
                                               (23, 8), (40, 10), (61, 4)])
def test_band_solver_shapes(ctx, n_poses, max_track):
    """The banded K3 over one-sided (F < 2w + 2) and two-sided splits, odd and even F,
    bandwidths 1..9: one GN step against the numpy oracle's dense Cholesky."""
    p = make_ba_problem(n_poses, 40 * n_poses, 31 + n_poses, max_track=max_track)
    s = _step_vs_oracle(ctx, p)
    assert s.plan_stats()["band_solver"] == 1


def _add_far_landmark(p, cams):
    """One extra landmark seen by the given (far apart) cameras: a wide / non-monotone
    profile row."""
    from visualodometry_amd.synthetic import BAProblemData

    X = p.points[:1] * 0.0 + np.array([[0.5, 0.2, 60.0]])
    uv = []
    for c in cams:
        T = p.poses_cw[c]
        pc = T[:3, :3] @ X[0] + T[:3, 3]
        q = p.K @ pc
        uv.append(q[:2] / q[2])
    ptr = np.append(p.point_ptr, p.point_ptr[-1] + len(cams))
    return BAProblemData(
        **{**p.__dict__, "points": np.vstack([p.points, X]), "point_ptr": ptr,
           "obs_cam": np.append(p.obs_cam, cams).astype(p.obs_cam.dtype),
           "obs_uv": np.vstack([p.obs_uv, np.array(uv, dtype=p.obs_uv.dtype)])})


def test_wide_profile_uses_profile_solver(ctx):
    """A landmark linking keyframes 2 and 19 makes the bandwidth 17 > 9: the profile solver
    (any envelope) takes the window."""
    p = _add_far_landmark(make_ba_problem(20, 800, 41), [2, 19])
    s = _step_vs_oracle(ctx, p)
    assert s.plan_stats()["band_solver"] == 0


def test_non_monotone_profile_band_solver(ctx):
    """A landmark linking keyframes 2 and 11 of a short-track window: first[] is not
    monotone and the bandwidth 9 still fits the banded K3 (zeros inside the band)."""
    p = _add_far_landmark(make_ba_problem(12, 500, 43, max_track=3), [2, 11])
    s = _step_vs_oracle(ctx, p)
    assert s.plan_stats()["band_solver"] == 1


def test_two_sessions_on_one_context(ctx):
    """A second setup on the same context replaces the first problem: the first
    session's calls fail with VO_ERR_STATE instead of reading the other problem's sizes
    (ADVICE r1)."""
    p2 = make_ba_config("cfg2")
    small = make_ba_problem(6, 80, 5)
    s1 = _session(small, ctx)
    s2 = _session(p2, ctx)
    for call in (lambda: s1.get_state(), lambda: s1.run(1), lambda: s1.gn_step(),
                 lambda: s1.set_state(small.poses_cw, small.points), lambda: s1.run_async(1)):
        with pytest.raises(VoError) as e:
            call()
        assert e.value.code == _lib.VO_ERR_STATE
    rc, costs = s2.run(2)  # the current session is unaffected
    assert rc == _lib.VO_OK and np.all(np.isfinite(costs))
    s1b = _session(small, ctx)  # a fresh setup of the first problem works again
    rc, _ = s1b.run(1)
    assert rc == _lib.VO_OK
    with pytest.raises(VoError):
        s2.get_state()


@pytest.mark.parametrize("cfg,variant", [("cfg3", 0), ("cfg3", 2), ("cfg4", 0), ("cfg4", 3), ("cfg4", -1)])
def test_slide_takes_groups_over_and_matches_scratch(ctx, cfg, variant):
    """Consecutive keyframe windows on one context: each vo_ba_setup takes the unchanged
    first-camera groups of the previous window's plan over (chunk images copied on the
    device, not rebuilt or uploaded), and every result is bitwise the one of a setup from
    scratch (an unrelated window set up in between), which also matches the C oracle.  Every
    K1 variant: the default, the one-wave K1 with segments of several chunks, and the four-wave
    K1's multi-chunk segments (with its repacking to one round; its packing target depends on
    the window alone, ADVICE r4, so the slid plan is the scratch plan)."""
    four = variant < 0
    from visualodometry_amd.synthetic import make_ba_slide

    ws = make_ba_slide(cfg, 3)
    other = make_ba_problem(8, 200, 11)
    iters = 2
    inc = []
    reused, prev_so = 0, None
    _lib.ba_testing_k1(ctx, variant)
    try:
        for i, w in enumerate(ws):
            s = _session(w, ctx)
            st = s.plan_stats()
            assert (st["seg_obs"] > 1) == four, st
            # groups are taken over from a plan of the same packing target (seg_obs, on a
            # fixed grid: consecutive windows usually share it)
            if i and st["seg_obs"] == prev_so:
                assert st["reused_chunks"] >= 0.6 * st["chunks"], st
            reused += st["reused_chunks"]
            prev_so = st["seg_obs"]
            rc, costs = s.run(iters)
            assert rc == _lib.VO_OK
            inc.append((costs, *s.get_state()))
        for w, (costs, P, X) in zip(ws, inc):
            _session(other, ctx).run(1)
            s = _session(w, ctx)
            assert s.plan_stats()["reused_chunks"] == 0
            rc, c2 = s.run(iters)
            P2, X2 = s.get_state()
            np.testing.assert_array_equal(c2, costs)
            np.testing.assert_array_equal(P2, P)
            np.testing.assert_array_equal(X2, X)
    finally:
        _lib.ba_testing_k1(ctx, 0)
    assert reused > 0
    w = ws[-1]
    R = cref.BAProblemRef(w.K, w.point_ptr, w.obs_cam, w.obs_uv, w.n_poses, w.n_fixed, 1.0)
    n, Pr, Xr, cr = R.solve(w.poses_cw, w.points, iters, nthreads=8)
    np.testing.assert_allclose(inc[-1][0], cr, rtol=REL)
    assert _rel(inc[-1][1], Pr) < REL
