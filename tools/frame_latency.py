"""Per-frame latency of the reference's per-frame calls through the drop-in, torch first on the
GPU as the reference's frontend does (frontend.py:3, :66-67): what process_frame pays per call.

  process_image_gpu   FeatureFrontend.process_image hook: one textured KITTI-size image, SIFT
                      nfeatures 4000; k.pt and descriptors written into torch's GPU memory
  process_image_host  the same through SIFT.detectAndCompute + the reference's body (host
                      keypoint objects, descriptors to host, then torch copies them back)
  match_gpu_cached    match_frames hook: keyframe (4000 x 128) vs frame (4000 x 128) GPU tensors,
                      the keyframe's packed rows cached (every frame after a keyframe's first)
  match_gpu_uncached  the same with a fresh keyframe every call
  match_host          numpy descriptors through vo_match_knn2_ratio (no cache)
  match_host_cached   numpy descriptors, the keyframe side as a CPU torch tensor (cached, _q)
  pnp                 pnp_ransac, 1000 correspondences (vo.py:135-141)
Medians in ms; one JSON line."""
import json
import sys
import time
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
dev = torch.device("cuda")
torch.ones(8, device=dev).sum().item()  # torch's HIP runtime first

from visualodometry_amd import _lib, matcher, pnp, sift  # noqa: E402
from visualodometry_amd.dropin import hooks  # noqa: E402
from visualodometry_amd.synthetic import pnp_case, sift_like_pair, sift_scene  # noqa: E402


def timed(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return float(np.median(t)) * 1e3


ctx = _lib.context(0)
out = {}
img = sift_scene(376, 1241, seed=200, texture=12.0)
det = sift.SIFT_create(nfeatures=4000, contrastThreshold=0.02, edgeThreshold=2.0, sigma=1.6)
fe = SimpleNamespace(extractor=det, device=dev)


def reference_body(self, im):  # frontend.py:51-75 with the drop-in's SIFT object as the extractor
    kps, des = self.extractor.detectAndCompute(im, None)
    pts = np.array([k.pt for k in kps], dtype=np.float32)
    des = np.array(des, dtype=np.float32)
    return {"keypoints": torch.from_numpy(pts).unsqueeze(0).to(dev),
            "descriptors": torch.from_numpy(des).unsqueeze(0).to(dev),
            "image_size": torch.tensor([(im.shape[1], im.shape[0])]).to(dev)}


pi = hooks._wrap_process_image(reference_body)
f = pi(fe, img)
out["process_image_gpu_in_place"] = bool(f["descriptors"].is_cuda) and not getattr(ctx, "_foreign_tensors", False)
out["keypoints"] = int(f["keypoints"].shape[1])
out["process_image_gpu_ms"] = timed(lambda: pi(fe, img), reps=10)
out["process_image_host_ms"] = timed(lambda: reference_body(fe, img), reps=10)
_lib.profile_enable(ctx, True)
for _ in range(5):
    pi(fe, img)
prof = _lib.profile_read(ctx)
_lib.profile_enable(ctx, False)
out["process_image_kernel_us"] = {k: round(v[0] / v[1] * 1e3, 2) for k, v in prof.items()}
out["process_image_kernel_launches"] = {k: v[1] // 5 for k, v in prof.items()}
d0, d1 = sift_like_pair(4000, 4000, 7)
t0, t1 = torch.from_numpy(d0)[None].to(dev), torch.from_numpy(d1)[None].to(dev)
fr = SimpleNamespace(conf=SimpleNamespace(extractor_type="sift", match_on_gpu=True))
mf = hooks._wrap_match_frames(lambda self, a, b: None)
out["match_gpu_cached_ms"] = timed(lambda: mf(fr, {"descriptors": t0}, {"descriptors": t1}))
out["match_gpu_uncached_ms"] = timed(lambda: mf(fr, {"descriptors": t0.clone()}, {"descriptors": t1}))
out["match_host_ms"] = timed(lambda: matcher.match_knn2_ratio(d0, d1, ctx=ctx, kind=matcher.DESC_SIFT))
c0 = torch.from_numpy(d0)
out["match_host_cached_ms"] = timed(lambda: matcher.match_knn2_ratio(c0, d1, ctx=ctx, kind=matcher.DESC_SIFT,
                                                                     cache_query=True))
X, uv, Kp, _, _ = pnp_case(1000, 5)
out["pnp_ms"] = timed(lambda: pnp.pnp_ransac(X, uv, Kp, 1.0, ctx=ctx))
_lib.profile_enable(ctx, True)
for _ in range(10):
    pnp.pnp_ransac(X, uv, Kp, 1.0, ctx=ctx)
prof = _lib.profile_read(ctx)
_lib.profile_enable(ctx, False)
out["pnp_kernel_us"] = {k: round(v[0] / v[1] * 1e3, 2) for k, v in prof.items()}
print(json.dumps(out))
