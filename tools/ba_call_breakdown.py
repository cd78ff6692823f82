"""Per-keyframe cost of SlidingWindowBA.optimize split into its steps (cfg3 window):
host planning alone (vo_ba_plan_probe), setup (plan + upload), set_state, 10 GN
iterations, get_state.  Medians over repeated calls; run on the GPU box."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib  # noqa: E402
from visualodometry_amd.ba import BASession, BAWindow, group_window, plan_probe  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
p = make_ba_config(cfg)
ctx = _lib.context(0)
obs_pt = np.repeat(np.arange(p.n_points), np.diff(p.point_ptr))
win = BAWindow(p.poses_cw, p.points, p.obs_uv, p.obs_cam, obs_pt, p.n_fixed)  # grouped, as the hooks build it
t = {k: [] for k in ["csr", "plan_only", "setup", "set_state", "run10", "get_state", "total"]}
for r in range(12):
    t0 = time.perf_counter()
    point_ptr, obs_cam, obs_uv = group_window(p.n_points, win)
    t1 = time.perf_counter()
    s = BASession(p.K, point_ptr, obs_cam, obs_uv, p.n_poses, p.n_fixed, 1.0, ctx)
    t2 = time.perf_counter()
    s.set_state(p.poses_cw, p.points)
    t3 = time.perf_counter()
    s.run(10)
    t4 = time.perf_counter()
    s.get_state()
    t5 = time.perf_counter()
    plan_probe(p.K, point_ptr, obs_cam, obs_uv, p.n_poses, p.n_fixed, 1024)
    t6 = time.perf_counter()
    for k, v in zip(["csr", "setup", "set_state", "run10", "get_state", "total", "plan_only"],
                    [t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t5 - t0, t6 - t5]):
        t[k].append(v * 1e3)
print(json.dumps({k: round(float(np.median(v[2:])), 3) for k, v in t.items()}))
