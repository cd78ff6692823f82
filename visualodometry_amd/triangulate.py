"""Two-view triangulation on the MI355X.

:func:`triangulate_points` has the signature and return values of the reference's
``triangulate_points`` (``src/modules/frontend.py:115-148``): ``(T_cw1, T_cw2, pts1,
pts2, K, config) -> (pts3d[mask] float32 (M, 3), mask (N,) bool)``.  The projection
matrices ``K @ T_cw[:3, :]`` are formed here with numpy exactly as the reference
forms them (``:127-128``); the DLT + SVD, the float32 dehomogenisation, the depth test
and the ``cv2.projectPoints`` reprojection filter run in ``vo_triangulate``
(``csrc/tri.hip``).  Fails loudly without the HIP library (no CPU fallback).
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, ptr


def _mats(T_cw1, T_cw2, K):
    K = np.asarray(K, dtype=np.float64)
    T1 = np.asarray(T_cw1, dtype=np.float64)
    T2 = np.asarray(T_cw2, dtype=np.float64)
    P1 = np.ascontiguousarray(K @ T1[:3, :])  # frontend.py:127-128
    P2 = np.ascontiguousarray(K @ T2[:3, :])
    return P1, P2, np.ascontiguousarray(T2[:3, :]), np.ascontiguousarray(K)


def triangulate_all(T_cw1, T_cw2, pts1, pts2, K, min_depth: float, max_reproj_err: float,
                    ctx: _lib.Context | None = None):
    """Every point's float32 triangulation (N, 3) and the keep mask (N,) bool."""
    ctx = ctx or _lib.context()
    p1 = np.ascontiguousarray(np.asarray(pts1, dtype=np.float32).reshape(-1, 2))
    p2 = np.ascontiguousarray(np.asarray(pts2, dtype=np.float32).reshape(-1, 2))
    if p1.shape != p2.shape:
        raise ValueError("pts1 and pts2 must have the same shape (N, 2)")
    n = p1.shape[0]
    out = np.empty((n, 3), dtype=np.float32)
    mask = np.empty(n, dtype=np.uint8)
    P1, P2, T2, Km = _mats(T_cw1, T_cw2, K)
    check(ctx.lib.vo_triangulate(ctx.handle, ptr(P1, C.c_double), ptr(P2, C.c_double), ptr(T2, C.c_double),
                                 ptr(Km, C.c_double), ptr(p1, C.c_float), ptr(p2, C.c_float), n,
                                 float(min_depth), float(max_reproj_err), ptr(out, C.c_float),
                                 ptr(mask, C.c_uint8)), "vo_triangulate")
    return out, mask.astype(bool)


def triangulate_points(T_cw1, T_cw2, pts1, pts2, K, config, ctx: _lib.Context | None = None):
    """Drop-in for the reference's ``triangulate_points`` (``frontend.py:115-148``)."""
    if len(pts1) == 0:
        return np.empty((0, 3)), np.zeros(0, dtype=bool)  # frontend.py:123-124
    pts3d, mask = triangulate_all(T_cw1, T_cw2, pts1, pts2, K, config.min_depth, config.max_reproj_err, ctx)
    return pts3d[mask], mask


def triangulate_device(T_cw1, T_cw2, d_pts1: _lib.DeviceArray, d_pts2: _lib.DeviceArray, K,
                       min_depth: float, max_reproj_err: float, d_out: _lib.DeviceArray,
                       d_mask: _lib.DeviceArray, ctx: _lib.Context | None = None) -> None:
    """Points and outputs resident in HBM (``vo_triangulate_async``); enqueued, not synchronised."""
    ctx = ctx or d_pts1.ctx
    n = d_pts1.shape[0]
    P1, P2, T2, Km = _mats(T_cw1, T_cw2, K)
    check(ctx.lib.vo_triangulate_async(ctx.handle, ptr(P1, C.c_double), ptr(P2, C.c_double),
                                       ptr(T2, C.c_double), ptr(Km, C.c_double), C.c_void_p(d_pts1.ptr),
                                       C.c_void_p(d_pts2.ptr), n, float(min_depth), float(max_reproj_err),
                                       C.c_void_p(d_out.ptr), C.c_void_p(d_mask.ptr)), "vo_triangulate_async")
