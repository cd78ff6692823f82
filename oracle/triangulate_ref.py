"""CPU oracle for triangulation -- TEST INFRASTRUCTURE ONLY.

Imported by ``tests/`` and the ``cpu_baseline`` leg of ``bench.py``; never by the
product path.

Restates ``triangulate_points`` of the reference (``src/modules/frontend.py:115-148``)
with the arithmetic of the OpenCV calls it makes (``opencv-python==4.12.0.88``,
``uv.lock:742-743``; OpenCV is absent from this image, so this follows its published
source):

* ``cv2.triangulatePoints(P1, P2, pts1.T, pts2.T)`` (``frontend.py:130``) -- for each
  point the 4x4 DLT matrix, in double, row ``2j`` = ``x_j * P_j[2] - P_j[0]`` and row
  ``2j+1`` = ``y_j * P_j[2] - P_j[1]`` (OpenCV ``icvTriangulatePoints``), its SVD, and the
  right singular vector of the smallest singular value (last row of V^T) as the
  homogeneous point.  The output has the type of the image points: float32 for the
  reference's keypoints (``frontend.py:59``, ``vo.py:266-272``).
* ``pts4d[:3] / pts4d[3]`` in float32 (``frontend.py:131``).
* depth of the point in camera 2 > ``min_depth`` (``frontend.py:134-135``).
* ``cv2.projectPoints(pts3d, R2, t2, K, None)`` (``frontend.py:139``) -- OpenCV's
  ``cvProjectPoints2Internal`` in double with no distortion: ``X = R M + t`` summed left
  to right, ``z = 1/Z``, ``x = X z``, ``u = x fx + cx`` (the distortion factors are exactly
  1 and 0 then), stored as float32 like the object points.
* reprojection error ``norm(proj - pts2)`` in float32 (``frontend.py:140``) below
  ``max_reproj_err`` (``frontend.py:143``).

Parity pin: OpenCV cannot run here and the reference has no tests or fixtures
(SURVEY.md §8c), so this restatement is pinned by known-answer cases
(``tests/test_oracle_triangulate.py``): noise-free points are recovered, points
behind the camera and gross outliers are rejected, and the projection equals the
pinhole model.  Against OpenCV itself it is **parity unpinned**.
"""

from __future__ import annotations

import numpy as np


def projection_matrices(T_cw1, T_cw2, K):
    """``P = K @ T_cw[:3, :]`` as the reference forms it (``frontend.py:127-128``)."""
    K = np.asarray(K, dtype=np.float64)
    return K @ np.asarray(T_cw1, dtype=np.float64)[:3, :], K @ np.asarray(T_cw2, dtype=np.float64)[:3, :]


def dlt_points4d(P1, P2, pts1, pts2) -> np.ndarray:
    """``cv2.triangulatePoints`` for float32 image points -> (4, N) float32."""
    p1 = np.asarray(pts1, dtype=np.float32).reshape(-1, 2).astype(np.float64)
    p2 = np.asarray(pts2, dtype=np.float32).reshape(-1, 2).astype(np.float64)
    n = p1.shape[0]
    A = np.empty((n, 4, 4))
    for j, (P, p) in enumerate(((P1, p1), (P2, p2))):
        A[:, 2 * j] = p[:, :1] * P[2][None, :] - P[0][None, :]
        A[:, 2 * j + 1] = p[:, 1:2] * P[2][None, :] - P[1][None, :]
    if n == 0:
        return np.zeros((4, 0), dtype=np.float32)
    _, _, vt = np.linalg.svd(A)
    return vt[:, 3, :].T.astype(np.float32)


def project_points(pts3d, R, t, K) -> np.ndarray:
    """``cv2.projectPoints(pts3d, R, t, K, None)`` for float32 object points -> (N, 2) f32."""
    M = np.asarray(pts3d, dtype=np.float32).reshape(-1, 3).astype(np.float64)
    R = np.asarray(R, dtype=np.float64).reshape(3, 3)
    t = np.asarray(t, dtype=np.float64).reshape(3)
    K = np.asarray(K, dtype=np.float64)
    X, Y, Z = M[:, 0], M[:, 1], M[:, 2]
    x = R[0, 0] * X + R[0, 1] * Y + R[0, 2] * Z + t[0]
    y = R[1, 0] * X + R[1, 1] * Y + R[1, 2] * Z + t[1]
    z = R[2, 0] * X + R[2, 1] * Y + R[2, 2] * Z + t[2]
    with np.errstate(divide="ignore"):
        zi = np.where(z != 0, 1.0 / np.where(z != 0, z, 1.0), 1.0)
    x = x * zi
    y = y * zi
    u = x * K[0, 0] + K[0, 2]
    v = y * K[1, 1] + K[1, 2]
    return np.stack([u, v], axis=1).astype(np.float32)


def triangulate_points(T_cw1, T_cw2, pts1, pts2, K, min_depth: float, max_reproj_err: float):
    """The reference's ``triangulate_points`` (``frontend.py:115-148``) ->
    (pts3d[mask] float32 (M, 3), mask (N,) bool)."""
    pts1 = np.asarray(pts1, dtype=np.float32).reshape(-1, 2)
    pts2 = np.asarray(pts2, dtype=np.float32).reshape(-1, 2)
    if len(pts1) == 0:
        return np.empty((0, 3)), np.zeros(0, dtype=bool)
    P1, P2 = projection_matrices(T_cw1, T_cw2, K)
    pts4d = dlt_points4d(P1, P2, pts1, pts2)
    pts3d = (pts4d[:3] / pts4d[3]).T
    T2 = np.asarray(T_cw2, dtype=np.float64)
    pts3d_c2 = (T2[:3, :3] @ pts3d.T + T2[:3, 3:4]).T
    mask_pos_depth = pts3d_c2[:, 2] > min_depth
    proj = project_points(pts3d, T2[:3, :3], T2[:3, 3], K)
    err2 = np.linalg.norm(proj.reshape(-1, 2) - pts2, axis=1)
    mask = mask_pos_depth & (err2 < max_reproj_err)
    return pts3d[mask], mask


def all_points(T_cw1, T_cw2, pts1, pts2, K, min_depth: float, max_reproj_err: float):
    """(pts3d of every input (N, 3) float32, mask (N,) bool) -- the unfiltered form the
    GPU entry point returns."""
    pts1 = np.asarray(pts1, dtype=np.float32).reshape(-1, 2)
    if len(pts1) == 0:
        return np.zeros((0, 3), dtype=np.float32), np.zeros(0, dtype=bool)
    P1, P2 = projection_matrices(T_cw1, T_cw2, K)
    pts4d = dlt_points4d(P1, P2, pts1, pts2)
    pts3d = (pts4d[:3] / pts4d[3]).T
    _, mask = triangulate_points(T_cw1, T_cw2, pts1, pts2, K, min_depth, max_reproj_err)
    return pts3d, mask
