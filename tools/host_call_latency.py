"""Per-call latency of the host-buffer entry points (the reference's per-frame calls),
PCIe transfers and host-side marshalling included: what `process_frame` pays per call,
beside the device-resident throughput lines of bench.py.

  matcher   match_knn2_ratio, one KITTI frame pair (4000 x 4000 x 128 SIFT-like)
  sift      SIFT_create(4000, 0.02, 2.0, 1.6).detectAndCompute on a textured KITTI image
  tri       triangulate_all, 2000 correspondences
  pnp       pnp_ransac, 1000 correspondences
  ba        SlidingWindowBA.optimize of a cfg3-sized window, 10 GN iterations (setup included):
            from scratch (ba_cfg3_scratch_ms: an unrelated window set up before each call, so
            nothing is taken over), the same window again and again (ba_cfg3_10iters_ms: every
            first-camera group taken over at the same camera), and a drive's consecutive windows,
            one keyframe apart, as the reference's loop calls it (vo.py:252-288; each setup takes
            the unchanged groups of the last plan over: ba_cfg3_slide_ms), medians; the slid
            windows from scratch beside them (ba_cfg3_slide_windows_scratch_ms)
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib, matcher, pnp, sift, triangulate  # noqa: E402
from visualodometry_amd.ba import BAWindow, SlidingWindowBA  # noqa: E402
from visualodometry_amd.synthetic import (make_ba_config, make_ba_problem, make_ba_slide, pnp_case,  # noqa: E402
                                          sift_like_pair, sift_scene, triangulation_case)


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
obs_pt = np.repeat(np.arange(p.n_points, dtype=np.int32), np.diff(p.point_ptr))
win = BAWindow(p.poses_cw, p.points, p.obs_uv, p.obs_cam, obs_pt, p.n_fixed)
ba = SlidingWindowBA(p.K, iters=10, lam=1.0, device=0)
out["ba_cfg3_10iters_ms"] = timed(lambda: ba.optimize(win), reps=5, warm=1)
small = make_ba_problem(8, 200, 11)
small_win = BAWindow(small.poses_cw, small.points, small.obs_uv, small.obs_cam,
                     np.repeat(np.arange(small.n_points, dtype=np.int32), np.diff(small.point_ptr)), small.n_fixed)


def scratch_call(w):
    ba.optimize(small_win)  # untimed: the next setup has nothing to take over
    t0 = time.perf_counter()
    ba.optimize(w)
    return time.perf_counter() - t0


out["ba_cfg3_scratch_ms"] = float(np.median([scratch_call(win) for _ in range(12)][2:])) * 1e3
slides = []
for w in make_ba_slide("cfg3", 18):
    slides.append(BAWindow(w.poses_cw, w.points, w.obs_uv, w.obs_cam,
                           np.repeat(np.arange(w.n_points, dtype=np.int32), np.diff(w.point_ptr)), w.n_fixed))
ba.optimize(slides[0])
ba.optimize(slides[1])
t = []
for w in slides[2:]:
    t0 = time.perf_counter()
    ba.optimize(w)
    t.append(time.perf_counter() - t0)
out["ba_cfg3_slide_ms"] = float(np.median(t)) * 1e3
st = np.zeros(11, dtype=np.int64)  # the last slid window's plan (before the scratch calls below)
ctx.lib.vo_ba_plan_stats(ctx.handle, _lib.ptr(st, _lib.C.c_int64), 11)
out["ba_cfg3_slide_last"] = {"chunks": int(st[0]), "reused_chunks": int(st[9]), "reused_groups": int(st[8])}
out["ba_cfg3_slide_windows_scratch_ms"] = float(np.median([scratch_call(w) for w in slides[2:]])) * 1e3
print(json.dumps(out))
