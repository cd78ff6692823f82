"""Projected N-rank GN-iteration time of the landmark-sharded BA from measured kernels.

For N in (1, 2, 4, 8), every rank's shard of the window (``visualodometry_amd.shard``)
is set up alone on this one GPU and timed with the HIP-event profiler: K1 (ba_lin, its
1/N of the observations), K2 (ba_reduce) and K3 (ba_solve, replicated on every rank in
the real run).  The projection is max_r K1 + max_r K2 + K3(full window) + one all-reduce
of the reduced system, whose time is NOT measured here (RCCL needs one GPU per rank): it
is reported separately as bytes and left as a term.  Usage on the GPU box:
    python tools/shard_projection.py [cfg4|cfg3] > out.json
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from visualodometry_amd import _lib  # noqa: E402
from visualodometry_amd.ba import BASession  # noqa: E402
from visualodometry_amd.shard import shard  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
ITERS = 20
p = make_ba_config(cfg)
ctx = _lib.Context(0)
# K2 as a launch of its own, as on N > 1 ranks (the all-reduce sits between K2 and K3); one
# rank runs K2 inside K3's launch: "fused_1rank_us" below
_lib.ba_split_reduce(ctx, True)


def timed(ptr, cam, uv, pts):
    s = BASession(p.K, ptr, cam, uv, p.n_poses, p.n_fixed, 1.0, ctx)
    s.set_state(p.poses_cw, pts)
    s.run_async(3)
    s.synchronize()
    _lib.profile_enable(ctx, True)
    s.run_async(ITERS)
    s.synchronize()
    prof = _lib.profile_read(ctx)
    _lib.profile_enable(ctx, False)
    return {k: v[0] / v[1] * 1e3 for k, v in prof.items()}, s.plan_stats()


full, st = timed(p.point_ptr, p.obs_cam, p.obs_uv, p.points)
_lib.ba_split_reduce(ctx, False)
fused, _ = timed(p.point_ptr, p.obs_cam, p.obs_uv, p.points)
_lib.ba_split_reduce(ctx, True)
out = {"config": cfg, "full_us": full, "fused_1rank_us": fused, "reduced_system_bytes": int(st["profile_blocks"] * 288 + 48 * (p.n_poses - p.n_fixed) + 8),
       "ranks": {}}
for n in (1, 2, 4, 8):
    k1 = k2 = 0.0
    for r in range(n):
        _, ptr, cam, uv, pts = shard(p.point_ptr, p.obs_cam, p.obs_uv, p.points, n, r)
        t, _ = timed(ptr, cam, uv, pts)
        k1, k2 = max(k1, t["ba_lin"]), max(k2, t["ba_reduce"])
    step = k1 + k2 + full["ba_solve"]
    out["ranks"][n] = {"k1_max_us": k1, "k2_max_us": k2, "k3_us": full["ba_solve"],
                       "step_us_without_allreduce": step,
                       "speedup_vs_1_without_allreduce": None}
base = out["ranks"][1]["step_us_without_allreduce"]
for n, v in out["ranks"].items():
    v["speedup_vs_1_without_allreduce"] = base / v["step_us_without_allreduce"]
print(json.dumps(out, indent=1))
