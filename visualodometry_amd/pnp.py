"""PnP-RANSAC on the MI355X.

:func:`solvePnPRansac` has the call signature and return values of
``cv2.solvePnPRansac`` as the reference's tracking step uses it
(``src/modules/vo.py:135-141``): ``(objectPoints, imagePoints, cameraMatrix,
distCoeffs, reprojectionError=...) -> (retval, rvec (3,1), tvec (3,1), inliers (k,1)
int32 or None)``.  RANSAC with OpenCV's subsets and bookkeeping, EPnP per hypothesis
and the refinement run in ``vo_pnp_ransac`` (``csrc/pnp.hip``); the restatement it is
checked against is ``oracle/pnp_ref.py``.  Fails loudly without the HIP library (no CPU
fallback).  Only the configuration the reference uses is accepted: no distortion
(``None`` or all zeros), ``SOLVEPNP_ITERATIVE``, no extrinsic guess.
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, ptr

SOLVEPNP_ITERATIVE = 0


def _points(objpts, imgpts):
    X = np.ascontiguousarray(np.asarray(objpts, dtype=np.float32).reshape(-1, 3))
    uv = np.ascontiguousarray(np.asarray(imgpts, dtype=np.float32).reshape(-1, 2))
    if X.shape[0] != uv.shape[0]:
        raise ValueError(f"{X.shape[0]} object points but {uv.shape[0]} image points")
    return X, uv


def pnp_ransac(objpts, imgpts, K, reproj_err: float = 8.0, iterations: int = 100,
               confidence: float = 0.99, ctx: _lib.Context | None = None):
    """-> (success bool, rvec (3,), tvec (3,), inlier mask (n,) bool)."""
    ctx = ctx or _lib.context()
    X, uv = _points(objpts, imgpts)
    n = X.shape[0]
    Km = np.ascontiguousarray(np.asarray(K, dtype=np.float64).reshape(3, 3))
    rvec = np.zeros(3)
    tvec = np.zeros(3)
    mask = np.zeros(max(n, 1), dtype=np.uint8)
    ok = C.c_int32(0)
    check(ctx.lib.vo_pnp_ransac(ctx.handle, ptr(X, C.c_float), ptr(uv, C.c_float), n, ptr(Km, C.c_double),
                                int(iterations), float(reproj_err), float(confidence), ptr(rvec, C.c_double),
                                ptr(tvec, C.c_double), ptr(mask, C.c_uint8), C.byref(ok)), "vo_pnp_ransac")
    return bool(ok.value), rvec, tvec, mask[:n].astype(bool)


def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs=None, rvec=None, tvec=None,
                   useExtrinsicGuess=False, iterationsCount=100, reprojectionError=8.0, confidence=0.99,
                   inliers=None, flags=SOLVEPNP_ITERATIVE, ctx: _lib.Context | None = None):
    """Drop-in for ``cv2.solvePnPRansac`` in the reference's tracking step (``vo.py:135-141``)."""
    if distCoeffs is not None and np.any(np.asarray(distCoeffs) != 0):
        raise ValueError("solvePnPRansac (MI355X): lens distortion is not supported")
    if useExtrinsicGuess or flags != SOLVEPNP_ITERATIVE:
        raise ValueError("solvePnPRansac (MI355X): only SOLVEPNP_ITERATIVE without extrinsic guess")
    ok, rv, tv, mask = pnp_ransac(objectPoints, imagePoints, cameraMatrix, reprojectionError,
                                  iterationsCount, confidence, ctx)
    if not ok:
        return False, rv.reshape(3, 1), tv.reshape(3, 1), None
    return True, rv.reshape(3, 1), tv.reshape(3, 1), np.flatnonzero(mask).astype(np.int32).reshape(-1, 1)


def ransac_subsets(count: int, iterations: int) -> np.ndarray:
    """The cv::RNG((uint64)-1) subsets the library draws for ``count`` points (host only)."""
    out = np.empty((iterations, 5), dtype=np.int32)
    check(_lib.load().vo_pnp_subsets(int(count), int(iterations), ptr(out, C.c_int32)), "vo_pnp_subsets")
    return out


def pnp_ransac_device(d_X: _lib.DeviceArray, d_uv: _lib.DeviceArray, offsets, K, reproj_err: float,
                      d_pose: _lib.DeviceArray, d_mask: _lib.DeviceArray, d_status: _lib.DeviceArray,
                      iterations: int = 100, confidence: float = 0.99,
                      ctx: _lib.Context | None = None) -> None:
    """A batch of frames resident in HBM (``vo_pnp_ransac_batch_async``); enqueued, not
    synchronised.  ``offsets`` (host, batch+1) delimit each frame's points."""
    ctx = ctx or d_X.ctx
    off = np.ascontiguousarray(np.asarray(offsets, dtype=np.int32))
    Km = np.ascontiguousarray(np.asarray(K, dtype=np.float64).reshape(3, 3))
    batch = off.size - 1
    check(ctx.lib.vo_pnp_ransac_batch_async(ctx.handle, C.c_void_p(d_X.ptr), C.c_void_p(d_uv.ptr),
                                            ptr(off, C.c_int32), batch, ptr(Km, C.c_double), int(iterations),
                                            float(reproj_err), float(confidence), C.c_void_p(d_pose.ptr),
                                            C.c_void_p(d_mask.ptr), C.c_void_p(d_status.ptr)),
          "vo_pnp_ransac_batch_async")
