"""Known-answer pins of the triangulation oracle (reference ``frontend.py:115-148``).

OpenCV is absent and the reference ships no fixtures, so the restatement of
``cv2.triangulatePoints`` + ``cv2.projectPoints`` is pinned by construction:
noise-free points are recovered, the projection is the pinhole model, and the two
filters reject exactly the planted outliers and points behind the camera.
"""

import numpy as np

from oracle import triangulate_ref as tr
from visualodometry_amd.synthetic import triangulation_case


def test_noise_free_points_are_recovered():
    T1, T2, p1, p2, K, X, kind = triangulation_case(400, 0, noise_px=0.0, outlier_frac=0.0, behind_frac=0.0)
    pts, mask = tr.triangulate_points(T1, T2, p1, p2, K, 0.001, 6.0)
    assert mask.all()
    # float32 image points quantise the rays: ~1e-7 relative per coordinate, amplified by depth/baseline
    np.testing.assert_allclose(pts, X, rtol=2e-3, atol=1e-3)
    assert pts.dtype == np.float32


def test_projection_is_the_pinhole_model():
    rng = np.random.default_rng(1)
    K = np.array([[718.856, 0.0, 607.1928], [0.0, 718.856, 185.2157], [0.0, 0.0, 1.0]])
    th = rng.normal(0, 0.1, 3)
    from visualodometry_amd.synthetic import so3_exp
    R, t = so3_exp(th), rng.normal(0, 1, 3)
    M = (rng.normal(0, 5, (100, 3)) + np.array([0, 0, 20])).astype(np.float32)
    uv = tr.project_points(M, R, t, K)
    Xc = (R @ M.astype(np.float64).T).T + t
    ref = (K @ Xc.T).T
    np.testing.assert_allclose(uv, ref[:, :2] / ref[:, 2:3], rtol=1e-6)
    assert uv.dtype == np.float32


def test_filters_reject_outliers_and_points_behind():
    T1, T2, p1, p2, K, X, kind = triangulation_case(2000, 2)
    for max_err in (2.0, 5.0, 6.0, 10.0):  # the reference's per-dataset values (config.py)
        pts, mask = tr.triangulate_points(T1, T2, p1, p2, K, 0.001, max_err)
        np.testing.assert_array_equal(mask, kind == 0)
        assert pts.shape == (int((kind == 0).sum()), 3)


def test_dlt_vector_is_the_null_direction():
    T1, T2, p1, p2, K, X, kind = triangulation_case(50, 3)
    P1, P2 = tr.projection_matrices(T1, T2, K)
    h = tr.dlt_points4d(P1, P2, p1, p2).astype(np.float64)
    assert np.allclose(np.linalg.norm(h, axis=0), 1.0, atol=1e-6)
    good = kind != 1  # consistent correspondences reproject onto their camera-1 point
    q1 = P1 @ h[:, good]
    np.testing.assert_allclose(q1[:2] / q1[2], p1[good].T, atol=2.0)


def test_empty_input():
    T1 = T2 = np.eye(4)
    K = np.eye(3)
    pts, mask = tr.triangulate_points(T1, T2, np.zeros((0, 2)), np.zeros((0, 2)), K, 0.001, 6.0)
    assert pts.shape == (0, 3) and mask.shape == (0,) and mask.dtype == bool
