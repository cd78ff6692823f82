"""GPU parity of PnP-RANSAC (vo_pnp_ransac) against the oracle (reference
``src/modules/vo.py:135-141``; oracle/pnp_ref.py).

Success flags and inlier masks (the reference uses the inlier indices,
``vo.py:206-209``) must be identical; rvec/tvec within 1e-5 relative (the north_star
floating-point tolerance).  The kernel keeps the oracle's operation order without FMA
contraction, but the SVD rotations, hypot/log/pow/sin/cos and the order of the
refinement's sums still round differently, so the synthetic cases keep the planted
outliers far (>= 25 px) from the thresholds.
"""

import numpy as np
import pytest

from oracle import pnp_ref as P
from visualodometry_amd import _lib, pnp
from visualodometry_amd.synthetic import pnp_case

pytestmark = pytest.mark.gpu


def _check(got, ref):
    ok, rv, tv, mask = got
    rok, rrv, rtv, rmask, _ = ref
    assert ok == rok
    np.testing.assert_array_equal(mask, rmask)
    if ok:
        np.testing.assert_allclose(rv, rrv, rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(tv, rtv, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("n,seed", [(6, 0), (12, 1), (100, 2), (600, 3), (2000, 4)])
@pytest.mark.parametrize("thr", [1.0, 2.0, 4.0])  # the reference's per-dataset pnp_reproj_err
def test_matches_oracle(ctx, n, seed, thr):
    X, uv, K, T, out = pnp_case(n, seed, noise_px=0.3, outlier_frac=0.2 if n > 12 else 0.0)
    _check(pnp.pnp_ransac(X, uv, K, thr, ctx=ctx), P.solve_pnp_ransac(X, uv, K, thr))


@pytest.mark.parametrize("iters,conf", [(1, 0.99), (20, 0.5), (300, 0.999)])
def test_iterations_and_confidence(ctx, iters, conf):
    X, uv, K, T, out = pnp_case(400, 9, noise_px=0.3, outlier_frac=0.45)
    _check(pnp.pnp_ransac(X, uv, K, 2.0, iters, conf, ctx=ctx),
           P.solve_pnp_ransac(X, uv, K, 2.0, iters, conf))


def test_drop_in_signature(ctx):
    X, uv, K, T, out = pnp_case(800, 5, noise_px=0.3, outlier_frac=0.3)
    ok, rvec, tvec, inliers = pnp.solvePnPRansac(X, uv, K, None, reprojectionError=1.0, ctx=ctx)
    rok, rrv, rtv, rmask, _ = P.solve_pnp_ransac(X, uv, K, 1.0)
    assert ok and rvec.shape == (3, 1) and tvec.shape == (3, 1)
    assert inliers.dtype == np.int32 and inliers.shape[1] == 1
    np.testing.assert_array_equal(inliers[:, 0], np.flatnonzero(rmask))
    assert not out[inliers[:, 0]].any()
    np.testing.assert_allclose(rvec[:, 0], rrv, rtol=1e-5, atol=1e-8)
    R = P.rodrigues_to_mat(rvec[:, 0][None])[0]
    assert np.abs(R - T[:3, :3]).max() < 2e-3


def test_edge_cases(ctx):
    X, uv, K, T, _ = pnp_case(5, 4, noise_px=0.0, outlier_frac=0.0)
    _check(pnp.pnp_ransac(X, uv, K, 1.0, ctx=ctx), P.solve_pnp_ransac(X, uv, K, 1.0))  # EPnP on all 5
    ok, rv, tv, mask = pnp.pnp_ransac(X[:4], uv[:4], K, 1.0, ctx=ctx)
    assert not ok and not mask.any()
    ok, rv, tv, mask = pnp.pnp_ransac(np.zeros((0, 3)), np.zeros((0, 2)), K, 1.0, ctx=ctx)
    assert not ok and mask.shape == (0,)
    ok, rvec, tvec, inliers = pnp.solvePnPRansac(X[:3], uv[:3], K, None, ctx=ctx)
    assert not ok and inliers is None
    rng = np.random.default_rng(5)  # pure noise: no model has more than 4 inliers
    Xn = (rng.uniform(-5, 5, (50, 3)) + [0, 0, 20]).astype(np.float32)
    un = rng.uniform(0, 1000, (50, 2)).astype(np.float32)
    _check(pnp.pnp_ransac(Xn, un, K, 0.5, ctx=ctx), P.solve_pnp_ransac(Xn, un, K, 0.5))
    with pytest.raises(ValueError):
        pnp.solvePnPRansac(X, uv, K, np.ones(5), ctx=ctx)


def test_batch_matches_single_calls(ctx):
    sizes = [0, 3, 5, 6, 250, 1000, 17, 600]
    cases = [pnp_case(max(n, 1), 20 + i, noise_px=0.3, outlier_frac=0.25 if n > 20 else 0.0)
             for i, n in enumerate(sizes)]
    Xs = [c[0][:n] for c, n in zip(cases, sizes)]
    Us = [c[1][:n] for c, n in zip(cases, sizes)]
    K = cases[0][2]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    dX = _lib.DeviceArray.from_numpy(ctx, np.concatenate(Xs))
    dU = _lib.DeviceArray.from_numpy(ctx, np.concatenate(Us))
    dP = _lib.DeviceArray(ctx, (len(sizes), 6), np.float64)
    dM = _lib.DeviceArray(ctx, (int(off[-1]),), np.uint8)
    dS = _lib.DeviceArray(ctx, (len(sizes), 2), np.int32)
    for rep in range(2):  # the second call reuses the cached subsets
        pnp.pnp_ransac_device(dX, dU, off, K, 2.0, dP, dM, dS, ctx=ctx)
        pose, mask, st = dP.numpy(), dM.numpy().astype(bool), dS.numpy()
        for f, n in enumerate(sizes):
            ref = P.solve_pnp_ransac(Xs[f], Us[f], K, 2.0)
            got = (bool(st[f, 0]), pose[f, :3], pose[f, 3:], mask[off[f]:off[f + 1]])
            _check(got, ref)
            assert st[f, 1] == ref[3].sum()


def test_large_frame_properties(ctx):
    """20k correspondences: outliers rejected, pose recovered (size-independent checks)."""
    X, uv, K, T, out = pnp_case(20_000, 31, noise_px=0.3, outlier_frac=0.3)
    ok, rv, tv, mask = pnp.pnp_ransac(X, uv, K, 2.0, ctx=ctx)
    assert ok and not (mask & out).any() and mask.sum() > 0.8 * (~out).sum()
    R = P.rodrigues_to_mat(rv[None])[0]
    assert np.abs(R - T[:3, :3]).max() < 1e-3 and np.abs(tv - T[:3, 3]).max() < 0.02


def _run_batch(ctx, Xs, Us, K, thr=2.0):
    sizes = [len(x) for x in Xs]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    dX = _lib.DeviceArray.from_numpy(ctx, np.concatenate(Xs).reshape(-1, 3))
    dU = _lib.DeviceArray.from_numpy(ctx, np.concatenate(Us).reshape(-1, 2))
    dP = _lib.DeviceArray(ctx, (len(sizes), 6), np.float64)
    dM = _lib.DeviceArray(ctx, (max(int(off[-1]), 1),), np.uint8)
    dS = _lib.DeviceArray(ctx, (len(sizes), 2), np.int32)
    pnp.pnp_ransac_device(dX, dU, off, K, thr, dP, dM, dS, ctx=ctx)
    return off, dP.numpy(), dM.numpy()[: off[-1]].astype(bool), dS.numpy()


def _split_cases(count, n_max, seed0, big=None):
    """Frames of mixed sizes and outlier fractions: some stop the serial loop within a few
    hypotheses, some run all 100 (60 % outliers, pure noise).  big: {frame: points} for frames
    past the scoring kernel's 1024-point register path."""
    rng = np.random.default_rng(seed0)
    fracs = [0.0, 0.1, 0.25, 0.45, 0.6]
    Xs, Us = [], []
    for i in range(count):
        n = [0, 5, 6][i] if i < 3 else int(rng.integers(8, n_max))
        n = (big or {}).get(i, n)
        X, uv, K, _, _ = pnp_case(max(n, 1), seed0 + i, noise_px=0.3, outlier_frac=fracs[i % 5] if n > 20 else 0.0)
        if i == 3:  # pure noise: no model has more than 4 inliers
            uv = rng.uniform(0, 1000, uv.shape).astype(np.float32)
        Xs.append(X[:n])
        Us.append(uv[:n])
    return Xs, Us, K


@pytest.mark.parametrize("h1", [1, 5, 16, 40])
def test_split_replay_matches_all_at_once(ctx, h1):
    """pnp_run's split (the first h1 hypotheses of every frame, the RANSAC replay, the rest
    only for the frames whose serial loop goes on): the same bits as solving all hypotheses
    at once, and the oracle's masks and poses."""
    Xs, Us, K = _split_cases(24, 700, 300)
    try:
        _lib.pnp_testing_split(ctx, -1)
        off, pose0, mask0, st0 = _run_batch(ctx, Xs, Us, K)
        assert _lib.pnp_testing_last_split(ctx) == (100, 0)
        _lib.pnp_testing_split(ctx, h1)
        off, pose1, mask1, st1 = _run_batch(ctx, Xs, Us, K)
        got_h1, tail = _lib.pnp_testing_last_split(ctx)
    finally:
        _lib.pnp_testing_split(ctx, 0)
    assert got_h1 == h1 and 0 < tail < len(Xs) - 3
    np.testing.assert_array_equal(pose1, pose0)
    np.testing.assert_array_equal(mask1, mask0)
    np.testing.assert_array_equal(st1, st0)
    for f in range(len(Xs)) if h1 == 16 else range(0, len(Xs), 4):
        ref = P.solve_pnp_ransac(Xs[f], Us[f], K, 2.0)
        _check((bool(st1[f, 0]), pose1[f, :3], pose1[f, 3:], mask1[off[f]:off[f + 1]]), ref)


@pytest.mark.parametrize("h1", [3, 16])
def test_split_replay_large_frames(ctx, h1):
    """The split with frames beyond the scoring kernel's register path (> 1024 points: counts
    from the global-memory loop, no incremental replay) and beyond pnp_final's LDS stage
    (> 1024 inliers): the bits of the all-at-once run, and the oracle's results."""
    sizes, fracs = [1025, 2600, 900, 4000, 1500, 60], [0.1, 0.45, 0.25, 0.05, 0.6, 0.0]
    Xs, Us = [], []
    for i, (n, fr) in enumerate(zip(sizes, fracs)):
        X, uv, K, _, _ = pnp_case(n, 500 + i, noise_px=0.3, outlier_frac=fr)
        Xs.append(X)
        Us.append(uv)
    try:
        _lib.pnp_testing_split(ctx, -1)
        _, pose0, mask0, st0 = _run_batch(ctx, Xs, Us, K)
        _lib.pnp_testing_split(ctx, h1)
        off, pose1, mask1, st1 = _run_batch(ctx, Xs, Us, K)
        assert _lib.pnp_testing_last_split(ctx)[0] == h1
    finally:
        _lib.pnp_testing_split(ctx, 0)
    assert st1[3, 1] > 1024  # the 4000-point frame's inliers exceed the LDS stage
    np.testing.assert_array_equal(pose1, pose0)
    np.testing.assert_array_equal(mask1, mask0)
    np.testing.assert_array_equal(st1, st0)
    for f in (0, 4):
        ref = P.solve_pnp_ransac(Xs[f], Us[f], K, 2.0)
        _check((bool(st1[f, 0]), pose1[f, :3], pose1[f, 3:], mask1[off[f]:off[f + 1]]), ref)


def test_group_kernel_equals_lane_kernel(ctx):
    """The lane-group hypothesis kernel (single frames: EPnP's 12 x 12 Jacobi SVD spread over a
    group's lanes in the index-sum step order, the beta kinds on separate lanes) and the
    one-lane-per-hypothesis kernel (the serial sweep): the same bits in every pose, mask and
    count of one batch of mixed frames (1025-4000-point frames included)."""
    Xs, Us, K = _split_cases(40, 700, 700, big={7: 1025, 19: 4000})
    out = []
    try:
        for mode in (1, -1):
            _lib.pnp_testing_group(ctx, mode)
            out.append(_run_batch(ctx, Xs, Us, K))
    finally:
        _lib.pnp_testing_group(ctx, 0)
    for a, b in zip(out[0][1:], out[1][1:]):
        np.testing.assert_array_equal(a, b)


def test_split_auto_large_batch(ctx):
    """A batch of more hypotheses than one wave per SIMD holds splits by itself; the results
    are the bits of the all-at-once run."""
    Xs, Us, K = _split_cases(1100, 120, 900, big={9: 1500, 21: 3000, 33: 1100})
    try:
        _lib.pnp_testing_split(ctx, -1)
        _, pose0, mask0, st0 = _run_batch(ctx, Xs, Us, K)
        _lib.pnp_testing_split(ctx, 0)
        off, pose1, mask1, st1 = _run_batch(ctx, Xs, Us, K)
        h1, tail = _lib.pnp_testing_last_split(ctx)
    finally:
        _lib.pnp_testing_split(ctx, 0)
    assert 16 <= h1 < 100 and tail > 0
    np.testing.assert_array_equal(pose1, pose0)
    np.testing.assert_array_equal(mask1, mask0)
    np.testing.assert_array_equal(st1, st0)
    for f in range(0, 40, 3):
        ref = P.solve_pnp_ransac(Xs[f], Us[f], K, 2.0)
        _check((bool(st1[f, 0]), pose1[f, :3], pose1[f, 3:], mask1[off[f]:off[f + 1]]), ref)
