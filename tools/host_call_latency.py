"""Per-call latency of the host-buffer entry points (the reference's per-frame calls),
PCIe transfers and host-side marshalling included: what `process_frame` pays per call,
beside the device-resident throughput lines of bench.py.

  matcher   match_knn2_ratio, one KITTI frame pair (4000 x 4000 x 128 SIFT-like)
  sift      SIFT_create(4000, 0.02, 2.0, 1.6).detectAndCompute on a textured KITTI image
  tri       triangulate_all, 2000 correspondences
  pnp       pnp_ransac, 1000 correspondences
  ba        SlidingWindowBA.optimize of the cfg3 window, 10 GN iterations (setup included)
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib, matcher, pnp, sift, triangulate  # noqa: E402
from visualodometry_amd.ba import BAWindow, SlidingWindowBA  # noqa: E402
from visualodometry_amd.synthetic import (make_ba_config, pnp_case, sift_like_pair, sift_scene,  # noqa: E402
                                          triangulation_case)


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
d0, d1 = sift_like_pair(4000, 4000, 7)
out["matcher_ms"] = timed(lambda: matcher.match_knn2_ratio(d0, d1, ctx=ctx))
img = sift_scene(376, 1241, seed=200, texture=12.0)
det = sift.SIFT_create(nfeatures=4000, contrastThreshold=0.02, edgeThreshold=2.0, sigma=1.6, ctx=ctx)
out["sift_ms"] = timed(lambda: det.detectAndCompute(img, None), reps=10)
T1, T2, q1, q2, K, _, _ = triangulation_case(2000, 3)
out["tri_ms"] = timed(lambda: triangulate.triangulate_all(T1, T2, q1, q2, K, 0.001, 6.0, ctx))
X, uv, Kp, _, _ = pnp_case(1000, 5)
out["pnp_ms"] = timed(lambda: pnp.pnp_ransac(X, uv, Kp, 1.0, ctx=ctx))
p = make_ba_config("cfg3")
obs_pt = np.repeat(np.arange(p.n_points), np.diff(p.point_ptr))
win = BAWindow(p.poses_cw, p.points, p.obs_uv, p.obs_cam, obs_pt, p.n_fixed)
ba = SlidingWindowBA(p.K, iters=10, lam=1.0, device=0)
out["ba_cfg3_10iters_ms"] = timed(lambda: ba.optimize(win), reps=5, warm=1)
print(json.dumps(out))
