"""SIFT keypoint detection on the MI355X (detection half).

:func:`detect` runs the scale space, the DoG extrema and ``adjustLocalExtrema`` of OpenCV's
SIFT (reference ``cv2.SIFT_create(...).detectAndCompute`` at
``src/modules/frontend.py:27-32,55``) in ``vo_sift_detect`` (``csrc/sift.hip``); the
restatement it is checked against is ``oracle/sift_ref.py``.  Orientation assignment and
descriptors are not part of it yet.  Fails loudly without the HIP library (no CPU
fallback).
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, ptr


def layout(h: int, w: int, n_layers: int = 3) -> dict:
    """The pitched pyramid layout of ``vo_sift_layout`` (host only)."""
    out = np.zeros(3 + 5 * 32, dtype=np.int64)
    n = check(_lib.load().vo_sift_layout(int(h), int(w), int(n_layers), ptr(out, C.c_int64), out.size),
              "vo_sift_layout")
    v = out[:n]
    n_oct = int(v[0])
    octs = v[3:3 + 5 * n_oct].reshape(n_oct, 5)
    return {"n_octaves": n_oct, "g_floats": int(v[1]), "d_floats": int(v[2]),
            "octaves": [dict(h=int(a), w=int(b), pitch=int(c), g_off=int(d), d_off=int(e)) for a, b, c, d, e in octs]}


def detect(gray, contrast: float = 0.04, edge: float = 10.0, sigma: float = 1.6, n_layers: int = 3,
           capacity: int = 1 << 16, ctx: _lib.Context | None = None) -> dict:
    """DoG keypoints of a uint8 image in (octave, level, row, column) order: the dict of
    ``oracle/sift_ref.detect`` (pt, size, response, octave word, xi, index)."""
    ctx = ctx or _lib.context()
    img = np.ascontiguousarray(np.asarray(gray, dtype=np.uint8))
    if img.ndim != 2:
        raise ValueError("detect: a single-channel (h, w) uint8 image is expected")
    h, w = img.shape
    kf = np.zeros((capacity, 8), np.float32)
    ki = np.zeros((capacity, 8), np.int32)
    cnt = C.c_int32(0)
    check(ctx.lib.vo_sift_detect(ctx.handle, ptr(img, C.c_uint8), h, w, float(contrast), float(edge), float(sigma),
                                 int(n_layers), int(capacity), ptr(kf, C.c_float), ptr(ki, C.c_int32), C.byref(cnt)),
          "vo_sift_detect")
    if cnt.value > capacity:
        raise RuntimeError(f"vo_sift_detect found {cnt.value} keypoints, capacity {capacity}")
    k = cnt.value
    kf, ki = kf[:k], ki[:k]
    word = ki[:, 1].astype(np.int64)
    word = (word & ~255) | (((word & 255) - 1) & 255)  # first octave -1 (doubled image)
    half = np.float32(0.5)
    return {"pt": (kf[:, :2] * half).astype(np.float32), "size": (kf[:, 2] * half).astype(np.float32),
            "response": kf[:, 3].copy(), "octave": word.astype(np.int32), "xi": kf[:, 4].copy(),
            "index": np.stack([ki[:, 1] & 255, ki[:, 3], ki[:, 4], ki[:, 5]], 1).astype(np.int32)}


def pyramid(gray, sigma: float = 1.6, n_layers: int = 3, ctx: _lib.Context | None = None):
    """(Gaussian levels, DoG levels) per octave of one image, as lists of float32 arrays."""
    ctx = ctx or _lib.context()
    img = np.ascontiguousarray(np.asarray(gray, dtype=np.uint8))
    h, w = img.shape
    L = layout(h, w, n_layers)
    g = np.zeros(L["g_floats"], np.float32)
    d = np.zeros(L["d_floats"], np.float32)
    check(ctx.lib.vo_sift_pyramid(ctx.handle, ptr(img, C.c_uint8), h, w, float(sigma), int(n_layers),
                                  ptr(g, C.c_float), g.size, ptr(d, C.c_float), d.size), "vo_sift_pyramid")
    G, D = [], []
    for o in L["octaves"]:
        oh, ow, op = o["h"], o["w"], o["pitch"]
        lv = oh * op
        G.append([g[o["g_off"] + i * lv:o["g_off"] + (i + 1) * lv].reshape(oh, op)[:, :ow] for i in range(n_layers + 3)])
        D.append([d[o["d_off"] + i * lv:o["d_off"] + (i + 1) * lv].reshape(oh, op)[:, :ow] for i in range(n_layers + 2)])
    return G, D


def detect_device(d_imgs: _lib.DeviceArray, contrast: float, edge: float, sigma: float, n_layers: int,
                  d_kpf: _lib.DeviceArray, d_kpi: _lib.DeviceArray, d_count: _lib.DeviceArray,
                  ctx: _lib.Context | None = None) -> None:
    """A batch of (batch, h, w) uint8 images in HBM (``vo_sift_detect_batch_async``); enqueued."""
    ctx = ctx or d_imgs.ctx
    b, h, w = d_imgs.shape
    check(ctx.lib.vo_sift_detect_batch_async(ctx.handle, C.c_void_p(d_imgs.ptr), b, h, w, float(contrast),
                                             float(edge), float(sigma), int(n_layers), int(d_kpf.shape[0]),
                                             C.c_void_p(d_kpf.ptr), C.c_void_p(d_kpi.ptr), C.c_void_p(d_count.ptr)),
          "vo_sift_detect_batch_async")
