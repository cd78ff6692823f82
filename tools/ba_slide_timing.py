"""Per-call host timing of SlidingWindowBA.optimize on consecutive cfg3 windows (the reference's
keyframe loop, vo.py:252-288) and on the same window from scratch, step by step: grouping,
setup (plan + uploads), set_state, 10 GN iterations, get_state.  Run it against a
-DVO_PLAN_TIMING build (VO_LIB_PATH) to get the setup's sections on stderr.
Usage on the GPU box: python tools/ba_slide_timing.py [n_slides] > out.json"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib  # noqa: E402
from visualodometry_amd.ba import BASession, BAWindow, group_window  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config, make_ba_slide  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
ctx = _lib.context(0)
steps = ["csr", "setup", "set_state", "run10", "get_state", "total"]


def call(w, log):
    obs_pt = np.repeat(np.arange(w.n_points, dtype=np.int32), np.diff(w.point_ptr))
    win = BAWindow(w.poses_cw, w.points, w.obs_uv, w.obs_cam, obs_pt, w.n_fixed)
    t0 = time.perf_counter()
    point_ptr, obs_cam, obs_uv = group_window(w.n_points, win)
    t1 = time.perf_counter()
    s = BASession(w.K, point_ptr, obs_cam, obs_uv, w.n_poses, w.n_fixed, 1.0, ctx)
    t2 = time.perf_counter()
    s.set_state(w.poses_cw, w.points)
    t3 = time.perf_counter()
    s.run(10)
    t4 = time.perf_counter()
    s.get_state()
    t5 = time.perf_counter()
    for k, v in zip(steps, [t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t5 - t0]):
        log[k].append(v * 1e3)
    return s.plan_stats()


out = {}
p = make_ba_config("cfg3")
log = {k: [] for k in steps}
for _ in range(n):
    sys.stderr.write("-- scratch\n")
    call(p, log)
out["scratch"] = {k: round(float(np.median(v[2:])), 3) for k, v in log.items()}
ws = make_ba_slide("cfg3", n + 2)
log = {k: [] for k in steps}
st = None
for w in ws:
    sys.stderr.write("-- slide\n")
    st = call(w, log)
out["slide"] = {k: round(float(np.median(v[2:])), 3) for k, v in log.items()}
out["slide_last_plan"] = st
# the same windows from scratch: an unrelated window set up before each (nothing to take over)
from visualodometry_amd.synthetic import make_ba_problem  # noqa: E402

other = make_ba_problem(8, 200, 11)
log = {k: [] for k in steps}
for w in ws:
    sys.stderr.write("-- slide windows from scratch\n")
    BASession(other.K, other.point_ptr, other.obs_cam, other.obs_uv, other.n_poses, other.n_fixed, 1.0, ctx)
    call(w, log)
out["slide_windows_scratch"] = {k: round(float(np.median(v[2:])), 3) for k, v in log.items()}
print(json.dumps(out))
