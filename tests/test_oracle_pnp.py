"""Pins the PnP-RANSAC oracle (oracle/pnp_ref.py), which restates the reference's
``cv2.solvePnPRansac`` call (``src/modules/vo.py:135-141``).  OpenCV is absent, so the
pins are known answers: the cv::RNG recurrence against its closed form, the library's
host subset generator against the oracle's, the Jacobi SVD against LAPACK, EPnP's exact
recovery of noise-free poses, planted outliers rejected, and the refined pose at the
least-squares optimum.  Against OpenCV itself: parity unpinned."""

import math

import numpy as np
import pytest

from oracle import pnp_ref as P
from visualodometry_amd import pnp
from visualodometry_amd.synthetic import pnp_case


def test_rng_matches_multiply_with_carry_closed_form():
    # MWC with base b = 2^32 and multiplier a is the LCG z -> z * b^-1 mod (a b - 1)
    a, b = P.CV_RNG_COEFF, 1 << 32
    m = a * b - 1
    binv = pow(b, -1, m)
    r = P.CvRNG()
    r.next()
    z1 = r.state
    for k in range(1, 200):  # the state is congruent mod m (it may exceed m by a carry)
        assert r.state % m == (z1 * pow(binv, k - 1, m)) % m
        r.next()


def test_library_subsets_equal_oracle_subsets():
    for count in (6, 7, 11, 100, 1000, 4097):
        np.testing.assert_array_equal(pnp.ransac_subsets(count, 100), P.ransac_subsets(count, 100))
        s = P.ransac_subsets(count, 100)
        assert all(len(set(row)) == 5 for row in s) and s.min() >= 0 and s.max() < count


def test_update_num_iters_known_values():
    # log(0.01) / log(1 - 0.8^5) = 11.66 -> 12
    assert P.update_num_iters(0.99, 0.2, 5, 100) == 12
    assert P.update_num_iters(0.99, 0.0, 5, 100) == 0  # every point an inlier: stop now
    assert P.update_num_iters(0.99, 0.9, 5, 100) == 100  # needs more than the cap
    assert P.update_num_iters(0.99, 0.5, 5, 100) == 100  # 145 > the cap
    assert P.update_num_iters(0.99, 0.5, 5, 200) == round(math.log(0.01) / math.log(1 - 0.5 ** 5))


def test_jacobi_svd_matches_lapack():
    rng = np.random.default_rng(0)
    for n in (3, 12):
        A = rng.normal(size=(8, n, n))
        A = A @ np.swapaxes(A, 1, 2)
        w, U, Vt, deg = P.svd_of(A)
        assert not deg.any()
        np.testing.assert_allclose(w, np.linalg.svd(A)[1], rtol=1e-12, atol=1e-12 * w.max())
        np.testing.assert_allclose(U * w[:, None, :] @ Vt, A, atol=1e-12 * np.abs(A).max())
        np.testing.assert_allclose(np.swapaxes(U, 1, 2) @ U, np.broadcast_to(np.eye(n), A.shape), atol=1e-12)


def test_epnp_recovers_noise_free_pose():
    for seed in range(5):
        X, uv, K, T, _ = pnp_case(40, seed, noise_px=0.0, outlier_frac=0.0)
        idx = np.stack([np.random.default_rng(seed * 100 + k).choice(40, 5, replace=False) for k in range(16)])
        R, t, ok = P.epnp(X[idx].astype(np.float64), uv[idx].astype(np.float64), K)
        assert ok.all()
        # uv are float32-rounded exact projections: the pose is recovered to ~1e-6
        np.testing.assert_allclose(R, np.broadcast_to(T[:3, :3], R.shape), atol=1e-4)
        np.testing.assert_allclose(t, np.broadcast_to(T[:3, 3], t.shape), atol=1e-3 * (1 + np.abs(T[:3, 3]).max()))


def test_rodrigues_round_trip():
    rng = np.random.default_rng(1)
    r = rng.normal(0, 1.0, (50, 3))
    r[0] = 0.0
    r[1] = [np.pi - 1e-9, 0, 0]
    R = P.rodrigues_to_mat(r)
    np.testing.assert_allclose(np.swapaxes(R, 1, 2) @ R, np.broadcast_to(np.eye(3), R.shape), atol=1e-14)
    back = P.rodrigues_to_vec(R)
    ok = np.linalg.norm(r, axis=1) < np.pi - 1e-6
    np.testing.assert_allclose(back[ok], r[ok], atol=1e-12)


@pytest.mark.parametrize("seed,thr,frac", [(0, 1.0, 0.25), (1, 4.0, 0.4), (2, 2.0, 0.1)])
def test_ransac_rejects_planted_outliers(seed, thr, frac):
    X, uv, K, T, out = pnp_case(600, seed, noise_px=0.3, outlier_frac=frac)
    ok, rv, tv, mask, d = P.solve_pnp_ransac(X, uv, K, thr)
    assert ok
    assert not (mask & out).any()  # outliers are >= 25 px off
    assert mask.sum() >= 0.6 * (~out).sum()
    R = P.rodrigues_to_mat(rv[None])[0]
    assert np.abs(R - T[:3, :3]).max() < 2e-3 and np.abs(tv - T[:3, 3]).max() < 0.05
    # the refined pose is the least-squares optimum over the inliers: zero gradient
    A, g, cost = P._normal_eq(R, tv, X[mask].astype(np.float64), uv[mask].astype(np.float64), K)
    step = np.linalg.solve(A, g)
    assert np.abs(step).max() < 1e-7


def test_niters_early_exit_and_first_best():
    X, uv, K, T, out = pnp_case(500, 3, noise_px=0.2, outlier_frac=0.1)
    ok, rv, tv, mask, d = P.solve_pnp_ransac(X, uv, K, 2.0)
    assert ok and d["iters_run"] < 100
    counts = np.where(d["valid"], d["counts"], 0)[: d["iters_run"]]
    # the best model is the FIRST one with the maximum count over the iterations run
    assert d["best"] == int(np.argmax(counts))


def test_five_points_and_too_few():
    X, uv, K, T, _ = pnp_case(5, 4, noise_px=0.0, outlier_frac=0.0)
    ok, rv, tv, mask, _ = P.solve_pnp_ransac(X, uv, K, 1.0)
    assert ok and mask.all()
    np.testing.assert_allclose(P.rodrigues_to_mat(rv[None])[0], T[:3, :3], atol=1e-4)
    ok, *_ = P.solve_pnp_ransac(X[:4], uv[:4], K, 1.0)
    assert not ok


def test_all_outliers_fail():
    rng = np.random.default_rng(5)
    X = rng.uniform(-5, 5, (50, 3)).astype(np.float32) + np.float32([0, 0, 20])
    uv = rng.uniform(0, 1000, (50, 2)).astype(np.float32)
    ok, rv, tv, mask, _ = P.solve_pnp_ransac(X, uv, np.array([[700.0, 0, 600], [0, 700, 180], [0, 0, 1]]), 0.5)
    assert not ok and not mask.any()
