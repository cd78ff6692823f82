"""Brute-force descriptor matching on MI355X (knn k=2 + Lowe ratio test).

Drop-in for the SIFT branch of ``FeatureFrontend.match_frames``
(reference ``src/modules/frontend.py:86-111``): the reference calls
``cv2.BFMatcher(cv2.NORM_L2, crossCheck=False).knnMatch(des0, des1, k=2)``
(``:34``, ``:101``) and keeps ``[m.queryIdx, m.trainIdx]`` when
``m.distance < 0.75 * n.distance`` (``:103-109``).  Here both steps run in
``libvo_hip.so`` (``vo_match_knn2_ratio``); see DESIGN.md §Matcher for the
exact semantics and the one documented divergence (no pair passing the test
returns shape ``(0, 2)``, not the reference's ``(0,)``).
"""

from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import C, check, ptr

RATIO_THRESH = 0.75  # frontend.py:104


def _as_des(d) -> np.ndarray:
    if hasattr(d, "detach"):  # torch tensor, possibly on the GPU (frontend.py:92-95)
        d = d.detach().cpu().numpy()
    d = np.asarray(d)
    if d.ndim == 3 and d.shape[0] == 1:  # (1, N, D) feature-dict layout (frontend.py:71)
        d = d[0]
    if d.ndim != 2:
        raise ValueError(f"descriptors must be (N, D), got shape {d.shape}")
    return np.ascontiguousarray(d, dtype=np.float32)


class _QueryTags:
    """Tags for the library's cached query side (``vo_match_knn2_ratio_q`` / ``_dev``).

    A descriptor object gets a tag while it is the cached query: the cache holds a strong
    reference to it, so neither the object nor its memory can be recycled under the same
    identity, and torch tensors carry a version counter that every in-place write bumps.  A
    numpy array has no such counter (a write could go unnoticed), so it is never cached."""

    def __init__(self):
        self.obj, self.version, self.tag, self.next = None, None, 0, 1

    def tag_for(self, d) -> int:
        version = getattr(d, "_version", None)
        if version is None:
            return 0
        if d is not self.obj or version != self.version:
            self.obj, self.version, self.tag = d, version, self.next
            self.next += 1
        return self.tag


def _tensor_2d(d):
    """A torch tensor as its (N, D) float32 contiguous view (the feature dict's (1, N, D))."""
    if d.dim() == 3 and d.shape[0] == 1:
        d = d[0]
    if d.dim() != 2:
        raise ValueError(f"descriptors must be (N, D), got shape {tuple(d.shape)}")
    return d.detach().float().contiguous()


def match_knn2_ratio(des0, des1, ratio: float = RATIO_THRESH, ctx: _lib.Context | None = None,
                     kind: int | None = None, cache_query: bool = False) -> np.ndarray:
    """Ratio-test matches as an ``int64`` array ``(M, 2)`` of (query, train), ascending query.

    ``kind`` (``DESC_SIFT`` / ``DESC_FLOAT``) is a hint for this call only: the context's own
    hint (:func:`set_descriptor_kind`) is restored afterwards.  Results never depend on it.

    ``cache_query``: ``des0`` is the keyframe side the reference matches every frame against
    (``vo.py:64-65``): the library keeps its device copy and packed rows across calls while the
    same unmodified torch tensor comes back.  Torch tensors already on the GPU are read in place
    (``vo_match_knn2_ratio_dev``: no descriptor crosses PCIe); results never depend on either."""
    ctx = ctx or _lib.context()
    dev = None if getattr(ctx, "_foreign_tensors", False) else _gpu_tensors(des0, des1, ctx)
    if dev is not None:
        a, b = dev
        n0, n1, dim = a.shape[0], b.shape[0], a.shape[1]
    else:
        a, b = _as_des(des0), _as_des(des1)
        n0, n1, dim = a.shape[0], b.shape[0], a.shape[1]
    if n0 == 0 or n1 == 0:  # frontend.py:97-98
        return np.empty((0, 2), dtype=np.int64)
    if dim != b.shape[1]:
        raise ValueError(f"descriptor dims differ: {dim} vs {b.shape[1]}")
    tag = _tags(ctx).tag_for(des0) if cache_query else 0
    out = np.empty((n0, 2), dtype=np.int32)
    cnt = np.zeros(1, dtype=np.int32)
    prior = getattr(ctx, "desc_kind", DESC_AUTO)
    scoped = kind is not None and kind != prior
    if scoped:
        check(ctx.lib.vo_match_hint(ctx.handle, int(kind)), "vo_match_hint")
    try:
        if dev is not None:
            import torch

            torch.cuda.current_stream(a.device).synchronize()  # the tensors' producer is done
            rc = ctx.lib.vo_match_knn2_ratio_dev(
                ctx.handle, C.c_void_p(a.data_ptr()), n0, C.c_uint64(tag), C.c_void_p(b.data_ptr()), n1, dim,
                float(ratio), ptr(out, C.c_int32), ptr(cnt, C.c_int32))
            if rc == _lib.VO_ERR_ARG and n0 and n1:
                # torch's device memory is not this library's HIP runtime's (the library refuses
                # such pointers before any launch): the host path from here on
                ctx._foreign_tensors = True
                return match_knn2_ratio(des0.detach().cpu(), des1.detach().cpu(), ratio, ctx, kind, False)
            check(rc, "vo_match_knn2_ratio_dev")
        elif tag:
            check(ctx.lib.vo_match_knn2_ratio_q(
                ctx.handle, ptr(a, C.c_float), n0, C.c_uint64(tag), ptr(b, C.c_float), n1, dim, float(ratio),
                ptr(out, C.c_int32), ptr(cnt, C.c_int32)), "vo_match_knn2_ratio_q")
        else:
            check(ctx.lib.vo_match_knn2_ratio(
                ctx.handle, ptr(a, C.c_float), n0, ptr(b, C.c_float), n1, dim, float(ratio),
                ptr(out, C.c_int32), ptr(cnt, C.c_int32)), "vo_match_knn2_ratio")
    finally:
        if scoped:
            check(ctx.lib.vo_match_hint(ctx.handle, int(prior)), "vo_match_hint")
    return out[: int(cnt[0])].astype(np.int64)


def _tags(ctx) -> _QueryTags:
    t = getattr(ctx, "_query_tags", None)
    if t is None:
        t = ctx._query_tags = _QueryTags()
    return t


def _gpu_tensors(des0, des1, ctx):
    """Both descriptor sets as (N, D) float32 torch tensors on the context's GPU, or None (host
    path): only tensors torch already holds on ``cuda:<ctx.device>`` qualify."""
    if not (hasattr(des0, "is_cuda") and hasattr(des1, "is_cuda")):
        return None
    if not (des0.is_cuda and des1.is_cuda):
        return None
    if des0.device.index != ctx.device or des1.device.index != ctx.device:
        return None
    return _tensor_2d(des0), _tensor_2d(des1)


def match_knn2(des0, des1, ctx: _lib.Context | None = None):
    """knnMatch(k=2) alone: ``idx (n0, 2) int32`` (-1 = none), ``dist (n0, 2) float32``."""
    a, b = _as_des(des0), _as_des(des1)
    n0 = a.shape[0]
    idx = np.full((n0, 2), -1, dtype=np.int32)
    dist = np.full((n0, 2), np.finfo(np.float32).max, dtype=np.float32)
    if n0 == 0:
        return idx, dist
    if b.shape[0] and a.shape[1] != b.shape[1]:
        raise ValueError(f"descriptor dims differ: {a.shape[1]} vs {b.shape[1]}")
    ctx = ctx or _lib.context()
    check(
        ctx.lib.vo_match_knn2(
            ctx.handle, ptr(a, C.c_float), n0, ptr(b, C.c_float), b.shape[0], a.shape[1],
            ptr(idx, C.c_int32), ptr(dist, C.c_float),
        ),
        "vo_match_knn2",
    )
    return idx, dist


def match_batch_device(des0: _lib.DeviceArray, des1: _lib.DeviceArray, ratio: float = RATIO_THRESH,
                       out: _lib.DeviceArray | None = None, ctx: _lib.Context | None = None):
    """Batched frame pairs already resident in HBM.

    ``des0`` (B, n0, D) and ``des1`` (B, n1, D) float32 :class:`DeviceArray`;
    returns the (B, n0) int32 :class:`DeviceArray` of kept train indices
    (-1 = rejected).  Enqueued on the library stream; call :func:`synchronize`.
    """
    if len(des0.shape) != 3 or len(des1.shape) != 3 or des0.shape[0] != des1.shape[0] \
            or des0.shape[2] != des1.shape[2]:
        raise ValueError("expected (B, n0, D) and (B, n1, D)")
    if des0.dtype != np.float32 or des1.dtype != np.float32:
        raise ValueError("expected float32 descriptors")
    B, n0, D = des0.shape
    ctx = ctx or des0.ctx
    if out is None:
        out = _lib.DeviceArray(ctx, (B, n0), np.int32)
    check(
        ctx.lib.vo_match_batch_async(
            ctx.handle, C.c_void_p(des0.ptr), C.c_void_p(des1.ptr), B, n0, des1.shape[1], D,
            float(ratio), C.c_void_p(out.ptr),
        ),
        "vo_match_batch_async",
    )
    return out


DESC_AUTO, DESC_SIFT, DESC_FLOAT = 0, 1, 2  # vo_match_hint kinds (include/vo_hip.h)


def set_descriptor_kind(kind: int, ctx: _lib.Context | None = None) -> None:
    """``vo_match_hint``: which descriptors later calls on ``ctx`` expect (results never
    depend on it).  ``DESC_SIFT`` leaves the float shortlist unlaunched (the drop-in sets it
    for the reference's SIFT extractor); ``DESC_AUTO`` launches both paths' kernels."""
    ctx = ctx or _lib.context()
    check(ctx.lib.vo_match_hint(ctx.handle, int(kind)), "vo_match_hint")
    ctx.desc_kind = int(kind)  # restored by match_knn2_ratio after a per-call hint


def synchronize(ctx: _lib.Context | None = None) -> None:
    ctx = ctx or _lib.context()
    check(ctx.lib.vo_synchronize(ctx.handle), "vo_synchronize")
