"""Diagnostic: one-image SIFT detectAndCompute calls (the drop-in's per-frame call), for a
kernel trace of the single-image path: ``rocprofv3 --kernel-trace -- python3 tools/sift_single.py``."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib, sift  # noqa: E402
from visualodometry_amd.synthetic import sift_scene  # noqa: E402

ctx = _lib.context(0)
img = sift_scene(376, 1241, seed=200, texture=12.0)
det = sift.SIFT_create(nfeatures=4000, contrastThreshold=0.02, edgeThreshold=2.0, sigma=1.6, ctx=ctx)
for _ in range(3):
    det.detectAndCompute(img, None)
t = []
for _ in range(10):
    t0 = time.perf_counter()
    kp, des = det.detectAndCompute(img, None)
    t.append(time.perf_counter() - t0)
print("keypoints", len(kp), "ms per call (min / median)", round(min(t) * 1e3, 3), round(sorted(t)[5] * 1e3, 3))
