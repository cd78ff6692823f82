"""Diagnostic: host sections of the first and later cfg3 keyframe setups on one context
(vo_ba_plan_stats setup_us), with the wall time of each setup call and of context creation;
`reserve` as second argument first calls vo_ba_reserve for the window's size (what
SlidingWindowBA does at VO construction).  Prints one JSON line."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib  # noqa: E402
from visualodometry_amd.ba import BASession  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
reserve = len(sys.argv) > 2 and sys.argv[2] == "reserve"
p = make_ba_config(cfg)
t0 = time.perf_counter()
ctx = _lib.context(0)
t_ctx = time.perf_counter() - t0
out = {"config": cfg, "context_ms": t_ctx * 1e3, "setups": []}
if reserve:
    t0 = time.perf_counter()
    _lib.ba_reserve(ctx, p.n_poses, p.n_points, p.n_obs, p.n_fixed)
    out["reserve_ms"] = (time.perf_counter() - t0) * 1e3
for i in range(3):
    t0 = time.perf_counter()
    s = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0, ctx)
    t1 = time.perf_counter()
    s.set_state(p.poses_cw, p.points)
    rc, costs = s.run(10)
    t2 = time.perf_counter()
    st = s.plan_stats()
    out["setups"].append({"setup_ms": (t1 - t0) * 1e3, "set_state_run10_ms": (t2 - t1) * 1e3,
                          "setup_us": st["setup_us"], "setup_us_sum": sum(st["setup_us"].values())})
print(json.dumps(out))
