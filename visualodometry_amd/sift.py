"""SIFT on the MI355X: ``cv2.SIFT_create(...).detectAndCompute``.

Reference: ``src/modules/frontend.py:27-32`` creates the extractor, ``:55`` calls
``detectAndCompute(gray, None)`` and ``:59-60`` keeps ``k.pt`` and the float32 descriptors.

* :func:`detect_and_compute` / :class:`SIFT` (``SIFT_create``): the whole call in
  ``vo_sift_detect_and_compute`` (``csrc/sift.hip`` + ``csrc/sift_desc.hip``): scale space,
  extrema, orientation, removeDuplicatedSorted, retainBest(nfeatures), descriptors.
* :func:`detect`: the refined extrema alone (``vo_sift_detect``), for parity.

The restatement both are checked against is ``oracle/sift_ref.py``.  Fails loudly without
the HIP library (no CPU fallback).
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


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4"), ("image", "<i4"), ("reserved", "<i4")])  # vo_sift_keypoint


def _kp_dict(kp: np.ndarray, desc: np.ndarray) -> dict:
    return {"pt": np.stack([kp["x"], kp["y"]], 1).astype(np.float32).reshape(-1, 2),
            "size": kp["size"].copy(), "angle": kp["angle"].copy(), "response": kp["response"].copy(),
            "octave": kp["octave"].copy(), "descriptors": desc}


def detect_and_compute(gray, nfeatures: int = 0, contrast: float = 0.04, edge: float = 10.0, sigma: float = 1.6,
                       n_layers: int = 3, capacity: int = 1 << 15, ctx: _lib.Context | None = None) -> dict:
    """``SIFT_create(nfeatures, n_layers, contrast, edge, sigma).detectAndCompute(gray, None)``
    -> dict: pt (N, 2), size, angle, response, octave, descriptors (N, 128) float32, in the
    order of ``oracle/sift_ref.detect_and_compute``."""
    kp, desc = _detect_and_compute_records(gray, nfeatures, contrast, edge, sigma, n_layers, capacity, ctx)
    return _kp_dict(kp, desc)


def _detect_and_compute_records(gray, nfeatures: int, contrast: float, edge: float, sigma: float, n_layers: int,
                                capacity: int, ctx: _lib.Context | None) -> tuple:
    """``vo_sift_detect_and_compute`` -> (the N KP_DTYPE records, descriptors (N, 128) float32)."""
    ctx = ctx or _lib.context()
    img = np.ascontiguousarray(np.asarray(gray, dtype=np.uint8))
    if img.ndim != 2:
        raise ValueError("detect_and_compute: a single-channel (h, w) uint8 image is expected")
    h, w = img.shape
    # unzeroed outputs (the call writes the first `count` entries; a zeroed 17 MB pair cost
    # milliseconds per call once the allocator serves it from the heap), compact copies returned
    kp = np.empty(capacity, KP_DTYPE)
    desc = np.empty((capacity, 128), np.float32)
    cnt = C.c_int32(0)
    check(ctx.lib.vo_sift_detect_and_compute(ctx.handle, ptr(img, C.c_uint8), h, w, int(nfeatures), float(contrast),
                                             float(edge), float(sigma), int(n_layers), int(capacity),
                                             kp.ctypes.data_as(C.c_void_p), ptr(desc, C.c_float), C.byref(cnt)),
          "vo_sift_detect_and_compute")
    n = cnt.value
    return kp[:n], desc[:n].copy()


def detect_and_compute_torch(gray, nfeatures: int, contrast: float, edge: float, sigma: float, n_layers: int = 3,
                             device=None, ctx: _lib.Context | None = None):
    """``detect_and_compute`` with its outputs in torch tensors on the GPU, as
    ``FeatureFrontend.process_image`` keeps them (``frontend.py:59-67``: ``k.pt`` and the
    descriptors, moved to ``config.device``): ``vo_sift_detect_and_compute_dev`` writes them
    into torch's memory and only the count crosses PCIe.  Returns ``(pts (N, 2), desc (N, 128))``
    float32 tensors (same values as :func:`detect_and_compute`), or None when the library refuses
    torch's memory (another HIP runtime instance in the process) or the output would not fit:
    the caller takes the host path then."""
    import torch

    ctx = ctx or _lib.context()
    img = np.ascontiguousarray(np.asarray(gray, dtype=np.uint8))
    if img.ndim != 2:
        raise ValueError("detect_and_compute_torch: a single-channel (h, w) uint8 image is expected")
    h, w = img.shape
    device = torch.device(device) if device is not None else torch.device("cuda", ctx.device)
    # retainBest keeps every keypoint tied with the nfeatures-th response: a little headroom
    cap = nfeatures + nfeatures // 4 + 64 if nfeatures > 0 else 1 << 15
    kp = torch.empty((cap, 8), dtype=torch.float32, device=device)
    desc = torch.empty((cap, 128), dtype=torch.float32, device=device)
    torch.cuda.current_stream(device).synchronize()  # memory torch's stream may still be using
    cnt = C.c_int32(0)
    rc = ctx.lib.vo_sift_detect_and_compute_dev(ctx.handle, ptr(img, C.c_uint8), h, w, int(nfeatures),
                                                float(contrast), float(edge), float(sigma), int(n_layers), int(cap),
                                                C.c_void_p(kp.data_ptr()), C.c_void_p(desc.data_ptr()),
                                                C.byref(cnt))
    if rc == _lib.VO_ERR_ARG:
        return None
    check(rc, "vo_sift_detect_and_compute_dev")
    n = cnt.value
    return kp[:n, :2].contiguous(), desc[:n]


def detect_and_compute_device(d_imgs: _lib.DeviceArray, nfeatures: int, contrast: float, edge: float, sigma: float,
                              n_layers: int, d_kp: _lib.DeviceArray, d_desc: _lib.DeviceArray,
                              d_counts: _lib.DeviceArray, ctx: _lib.Context | None = None) -> None:
    """A batch of (batch, h, w) uint8 images in HBM (``vo_sift_detect_and_compute_batch_async``):
    d_kp (batch, capacity, 8) 32-byte keypoint records, d_desc (batch, capacity, 128) float32,
    d_counts (batch,) int32; enqueued."""
    ctx = ctx or d_imgs.ctx
    b, h, w = d_imgs.shape
    cap = int(d_kp.shape[1])
    if d_kp.shape[0] != b or d_desc.shape[:2] != (b, cap) or d_counts.shape[0] != b:
        raise ValueError("detect_and_compute_device: output shapes do not match the batch")
    check(ctx.lib.vo_sift_detect_and_compute_batch_async(
        ctx.handle, C.c_void_p(d_imgs.ptr), b, h, w, int(nfeatures), float(contrast), float(edge), float(sigma),
        int(n_layers), cap, C.c_void_p(d_kp.ptr), C.c_void_p(d_desc.ptr), C.c_void_p(d_counts.ptr)),
        "vo_sift_detect_and_compute_batch_async")


def unpack_device_keypoints(raw: np.ndarray) -> np.ndarray:
    """(…, 8) 32-bit words copied back from a device keypoint buffer -> KP_DTYPE records."""
    return np.ascontiguousarray(raw).view(KP_DTYPE).reshape(raw.shape[:-1])


def _load_keypoint_module():
    """``lib/_vo_keypoints.so`` (``csrc/kp_objects.c``, built beside libvo_hip.so): the C
    KeyPoint type and its bulk builder.  Required, like the HIP library: a missing build fails
    here rather than falling back to a per-object Python loop."""
    import importlib.machinery
    import importlib.util
    from pathlib import Path
    path = Path(__file__).resolve().parent / "lib" / "_vo_keypoints.so"
    if not path.exists():
        raise ImportError(f"{path} is missing: run `make -C visualodometry_amd/csrc` "
                          "(or __graft_entry__.build())")
    name = __name__.rsplit(".", 1)[0] + "._vo_keypoints"
    spec = importlib.util.spec_from_loader(name, importlib.machinery.ExtensionFileLoader(name, str(path)))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


_kpmod = _load_keypoint_module()

#: ``cv2.KeyPoint``'s Python surface (``frontend.py:59`` reads ``k.pt``):
#: ``KeyPoint(x, y, size, angle=-1, response=0, octave=0, class_id=-1)``; ``pt`` is a fresh
#: ``(x, y)`` tuple per read and the float fields are float32-stored, as in OpenCV.
KeyPoint = _kpmod.KeyPoint


def _keypoints(records: np.ndarray) -> tuple:
    """KeyPoint objects of ``vo_sift_keypoint`` records (KP_DTYPE), in one C loop."""
    if records.dtype != KP_DTYPE:
        raise ValueError(f"_keypoints: KP_DTYPE records expected, got {records.dtype}")
    return _kpmod.build(np.ascontiguousarray(records))


class SIFT:
    """``cv2.SIFT`` as the reference uses it: ``SIFT_create(nfeatures=..., contrastThreshold=...,
    edgeThreshold=..., sigma=...)`` then ``detectAndCompute(gray, None) -> (keypoints,
    descriptors)`` (``frontend.py:27-32,55``); descriptors is None when nothing is found, as in
    OpenCV's Python binding."""

    def __init__(self, nfeatures: int = 0, nOctaveLayers: int = 3, contrastThreshold: float = 0.04,
                 edgeThreshold: float = 10.0, sigma: float = 1.6, ctx: _lib.Context | None = None):
        self.nfeatures = int(nfeatures)
        self.n_layers = int(nOctaveLayers)
        self.contrast = float(contrastThreshold)
        self.edge = float(edgeThreshold)
        self.sigma = float(sigma)
        self._ctx = ctx

    def detectAndCompute(self, image, mask=None, descriptors=None, useProvidedKeypoints=False):
        if mask is not None or useProvidedKeypoints:
            raise NotImplementedError("SIFT.detectAndCompute: masks and provided keypoints are not supported")
        kp, desc = _detect_and_compute_records(image, self.nfeatures, self.contrast, self.edge, self.sigma,
                                               self.n_layers, 1 << 15, self._ctx or _lib.context())
        return _keypoints(kp), (desc if len(kp) else None)


def SIFT_create(nfeatures: int = 0, nOctaveLayers: int = 3, contrastThreshold: float = 0.04,
                edgeThreshold: float = 10.0, sigma: float = 1.6, **kw) -> SIFT:
    """``cv2.SIFT_create`` (keyword names as the reference passes them, ``frontend.py:27-32``)."""
    return SIFT(nfeatures, nOctaveLayers, contrastThreshold, edgeThreshold, sigma, **kw)
