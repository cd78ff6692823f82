"""Step-by-step host timing of one BA keyframe call (cfg3-sized windows), three ways: from
scratch (an unrelated window set up before each call: nothing taken over), the same window
repeated (every group taken over), and consecutive slid windows.  Steps: grouping (csr), the
Python preparation of the problem struct (prep), the vo_ba_setup call itself (setup), the wait
for the uploads it enqueued (upload_wait: a stream sync right after setup, measured on its own),
set_state, 10 GN iterations with the cost readback (run10), get_state.  Medians; GPU box only.
Usage: python tools/ba_call_steps.py > out.json"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib  # noqa: E402
from visualodometry_amd._lib import C, check  # noqa: E402
from visualodometry_amd.ba import BASession, BAWindow, _problem_struct, group_window  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config, make_ba_problem, make_ba_slide  # noqa: E402

ctx = _lib.context(0)
steps = ["csr", "prep", "setup", "upload_wait", "set_state", "run10", "get_state", "total"]
small = make_ba_problem(8, 200, 11)


def call(w, log, sync_after_setup):
    obs_pt = np.repeat(np.arange(w.n_points, dtype=np.int32), np.diff(w.point_ptr))
    win = BAWindow(w.poses_cw, w.points, w.obs_uv, w.obs_cam, obs_pt, w.n_fixed)
    t = [time.perf_counter()]
    point_ptr, obs_cam, obs_uv = group_window(w.n_points, win)
    t.append(time.perf_counter())
    pp = np.ascontiguousarray(point_ptr, dtype=np.int32)
    oc = np.ascontiguousarray(obs_cam, dtype=np.int32)
    uv = np.ascontiguousarray(obs_uv, dtype=np.float32).reshape(-1, 2)
    prob = _problem_struct(w.K, pp, oc, uv, w.n_poses, w.n_fixed, 1.0)
    sid = C.c_uint64(0)
    t.append(time.perf_counter())
    check(ctx.lib.vo_ba_setup(ctx.handle, C.byref(prob), C.byref(sid)), "setup")
    t.append(time.perf_counter())
    if sync_after_setup:
        check(ctx.lib.vo_synchronize(ctx.handle), "sync")
    t.append(time.perf_counter())
    s = BASession.__new__(BASession)
    s.ctx, s.session, s.n_poses, s.n_points, s.n_fixed, s._prob = ctx, int(sid.value), w.n_poses, w.n_points, \
        w.n_fixed, prob
    s.set_state(w.poses_cw, w.points)
    t.append(time.perf_counter())
    s.run(10)
    t.append(time.perf_counter())
    s.get_state()
    t.append(time.perf_counter())
    d = np.diff(t)
    for k, v in zip(steps, list(d) + [t[-1] - t[0]]):
        log[k].append(v * 1e3)
    for k, v in s.plan_stats().get("setup_us", {}).items():  # the setup's own sections (us)
        log.setdefault("setup_us." + k, []).append(v)


out = {}
p = make_ba_config("cfg3")
ws = make_ba_slide("cfg3", 16)
for sync in (False, True):
    tag = "_synced" if sync else ""
    log = {k: [] for k in steps}
    for _ in range(12):
        BASession(small.K, small.point_ptr, small.obs_cam, small.obs_uv, small.n_poses, small.n_fixed, 1.0, ctx)
        call(p, log, sync)
    out["scratch" + tag] = {k: round(float(np.median(v[2:])), 3) for k, v in log.items()}
    log = {k: [] for k in steps}
    for _ in range(12):
        call(p, log, sync)
    out["repeat" + tag] = {k: round(float(np.median(v[2:])), 3) for k, v in log.items()}
    log = {k: [] for k in steps}
    for w in ws:
        call(w, log, sync)
    out["slide" + tag] = {k: round(float(np.median(v[2:])), 3) for k, v in log.items()}
print(json.dumps(out))
