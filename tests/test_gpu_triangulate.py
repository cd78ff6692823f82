"""GPU parity of triangulation (vo_triangulate) against the oracle (reference
``src/modules/frontend.py:115-148``; oracle/triangulate_ref.py).

Masks (the inlier indices) must be identical; the float32 points within 1e-5
relative (the north_star tolerance for floating point).  The two solve the 4x4 DLT
with different SVD algorithms (one-sided Jacobi on the GPU, LAPACK in the oracle), so
the float32 homogeneous vectors can differ in the last bit; the synthetic cases keep
every point far from the reprojection and depth thresholds.
"""

import numpy as np
import pytest

from oracle import triangulate_ref as tr
from visualodometry_amd import triangulate
from visualodometry_amd.synthetic import triangulation_case

pytestmark = pytest.mark.gpu


class Cfg:
    def __init__(self, min_depth=0.001, max_reproj_err=6.0):
        self.min_depth = min_depth
        self.max_reproj_err = max_reproj_err


@pytest.mark.parametrize("n,seed", [(1, 0), (37, 1), (1000, 2), (4000, 3)])
@pytest.mark.parametrize("max_err", [2.0, 5.0, 6.0, 10.0])  # the reference's per-dataset values
def test_matches_oracle(n, seed, max_err):
    T1, T2, p1, p2, K, X, kind = triangulation_case(n, seed)
    got, gmask = triangulate.triangulate_all(T1, T2, p1, p2, K, 0.001, max_err)
    ref, rmask = tr.all_points(T1, T2, p1, p2, K, 0.001, max_err)
    np.testing.assert_array_equal(gmask, rmask)
    assert got.dtype == np.float32
    np.testing.assert_allclose(got[kind != 2], ref[kind != 2], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-4)


def test_drop_in_signature_and_values():
    T1, T2, p1, p2, K, X, kind = triangulation_case(3000, 7)
    cfg = Cfg(0.001, 5.0)
    got, gmask = triangulate.triangulate_points(T1, T2, p1, p2, K, cfg)
    ref, rmask = tr.triangulate_points(T1, T2, p1, p2, K, cfg.min_depth, cfg.max_reproj_err)
    np.testing.assert_array_equal(gmask, rmask)
    np.testing.assert_array_equal(gmask, kind == 0)
    assert gmask.dtype == bool and got.shape == ref.shape == (int(gmask.sum()), 3)
    np.testing.assert_allclose(got, ref, rtol=1e-5)


def test_empty():
    pts, mask = triangulate.triangulate_points(np.eye(4), np.eye(4), np.zeros((0, 2)), np.zeros((0, 2)),
                                               np.eye(3), Cfg())
    assert pts.shape == (0, 3) and mask.shape == (0,) and mask.dtype == bool


def test_large_batch_recovers_inliers():
    """200k points: the inlier set and the recovered geometry (size-independent checks)."""
    T1, T2, p1, p2, K, X, kind = triangulation_case(200_000, 11)
    got, gmask = triangulate.triangulate_all(T1, T2, p1, p2, K, 0.001, 6.0)
    np.testing.assert_array_equal(gmask, kind == 0)
    err = np.linalg.norm(got[kind == 0] - X[kind == 0], axis=1) / np.linalg.norm(X[kind == 0], axis=1)
    assert np.median(err) < 0.05  # 0.5 px noise over a 1 m baseline
