"""Where the single-image SIFT drop-in call (SIFT_create(4000, 0.02, 2.0, 1.6).detectAndCompute
on a textured KITTI-sized image) spends its time, medians in ms:

  c_call_ms          vo_sift_detect_and_compute alone (upload, pipeline, count sync, download)
  c_call_pinned_ms   the same call with page-locked image and output buffers
  dict_ms            sift.detect_and_compute (the C call plus the compact numpy copies)
  dropin_ms          SIFT.detectAndCompute (the above plus the KeyPoint objects)
  keypoints_ms       sift._keypoints alone on the same result (the C KeyPoint object build)
"""
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib, sift  # noqa: E402
from visualodometry_amd.synthetic import sift_scene  # noqa: E402


def timed(fn, reps=30, warm=3):
    for _ in range(warm):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return float(np.median(t)) * 1e3


torch.zeros(1, device="cuda")
ctx = _lib.context(0)
img = np.ascontiguousarray(sift_scene(376, 1241, seed=200, texture=12.0))
args = (4000, 0.02, 2.0, 1.6, 3)
cap = 1 << 15
kp = np.empty(cap, sift.KP_DTYPE)
desc = np.empty((cap, 128), np.float32)
cnt = C.c_int32(0)


def c_call():
    rc = ctx.lib.vo_sift_detect_and_compute(ctx.handle, img.ctypes.data_as(C.POINTER(C.c_uint8)), 376, 1241,
                                            args[0], args[1], args[2], args[3], args[4], cap,
                                            kp.ctypes.data_as(C.c_void_p), desc.ctypes.data_as(C.POINTER(C.c_float)),
                                            C.byref(cnt))
    assert rc == 0


def pinned(shape, dtype):

    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    t = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    return t, t.numpy().view(dtype).reshape(shape)


_hold = []


def c_call_pinned():
    if not _hold:
        _hold.extend([pinned((cap,), sift.KP_DTYPE), pinned((cap, 128), np.float32), pinned(img.shape, np.uint8)])
        _hold[2][1][...] = img
    pk, pd, pi = _hold[0][1], _hold[1][1], _hold[2][1]
    rc = ctx.lib.vo_sift_detect_and_compute(ctx.handle, pi.ctypes.data_as(C.POINTER(C.c_uint8)), 376, 1241,
                                            args[0], args[1], args[2], args[3], args[4], cap,
                                            pk.ctypes.data_as(C.c_void_p), pd.ctypes.data_as(C.POINTER(C.c_float)),
                                            C.byref(cnt))
    assert rc == 0


det = sift.SIFT_create(nfeatures=4000, contrastThreshold=0.02, edgeThreshold=2.0, sigma=1.6, ctx=ctx)
recs, _ = sift._detect_and_compute_records(img, *args, cap, ctx)
out = {"keypoints": int(len(recs)),
       "c_call_ms": timed(c_call),
       "c_call_pinned_ms": timed(c_call_pinned),
       "dict_ms": timed(lambda: sift.detect_and_compute(img, *args[:4], n_layers=3, ctx=ctx)),
       "dropin_ms": timed(lambda: det.detectAndCompute(img, None)),
       "keypoints_ms": timed(lambda: sift._keypoints(recs))}
print(json.dumps(out))
