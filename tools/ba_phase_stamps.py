"""Diagnostic: per-phase shader-cycle shares of the BA K1 kernel (stamped build).

Run on the GPU box: ``VO_BA_STAMPS=1 python tools/ba_phase_stamps.py [cfg]``.
Phase shares come from a separate stamped instantiation of K1; read the shares,
not the absolute time (the stamps themselves perturb the schedule).
"""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("VO_LIB_PATH", str(Path(__file__).resolve().parents[1] / "visualodometry_amd" / "lib" /
                                         "libvo_hip_stamps.so"))

from visualodometry_amd import _lib  # noqa: E402
from visualodometry_amd.ba import BASession  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config  # noqa: E402

PHASES = ["load", "backsub", "lin_obs", "reduce", "eliminate", "schur_pairs", "write(rhs)", "schur_cams(U)", "-", "-",
          "n_obs", "n_te", "n_pts", "n_pairs", "n_slots", "n_cams"]
NPH = len(PHASES)
K3 = ["k3_setup", "k3_side_chol", "k3_backsub", "k3_tail", "k3_side_barrier", "k3_side_midbar", "k3_merge",
      "k3_separator", "k3_side_tasks", "k3_side_panel"]

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
p = make_ba_config(cfg)
ctx = _lib.context(0)
s = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0, ctx)
s.set_state(p.poses_cw, p.points)
s.run_async(3)
s.synchronize()
out = np.zeros(len(PHASES) + len(K3), dtype=np.uint64)
n = _lib.check(ctx.lib.vo_ba_debug_stamps(ctx.handle, out.ctypes.data_as(_lib.C.POINTER(_lib.C.c_uint64)),
                                           len(out)))
tot = float(out[:8].sum())
print(cfg, s.plan_stats())
for k in range(min(n, 8)):
    print(f"{PHASES[k]:18s} {int(out[k]):14d} cycles (sum over WGs)  {100 * out[k] / tot:5.1f} %")
t3 = float(out[len(PHASES):].sum())
for k in range(len(PHASES), n):
    print(f"{K3[k - len(PHASES)]:18s} {int(out[k]):14d} cycles (one WG)  {100 * out[k] / max(t3, 1):5.1f} %")

# per-workgroup timeline of the last K1 launch (start/end absolute stamps)
st_ = s.plan_stats()
nseg = st_["chunks"] if st_["seg_obs"] == 1 else st_["segments"]  # rows: chunks of the one-wave K1
raw = np.zeros(nseg * NPH, dtype=np.uint64)
k = ctx.lib.vo_ba_debug_stamps(ctx.handle, raw.ctypes.data_as(_lib.C.POINTER(_lib.C.c_uint64)), -raw.size)
if k > 0:
    r = raw[:k].reshape(-1, NPH).astype(np.int64)
    xcc = r[:, 15] >> 24  # the stamping lane's XCD (s_memtime counts per XCD)
    r[:, 15] &= 0xFFFFFF
    t0, t1 = r[:, 8], r[:, 9]
    dur = t1 - t0
    t0 = t0.copy()
    t1 = t1.copy()
    for x in np.unique(xcc):  # times relative to each XCD's first start
        m = xcc == x
        b = t0[m].min()
        t0[m] -= b
        t1[m] -= b
    base = 0
    print(f"K1 workgroups: {len(r)} over {len(np.unique(xcc))} XCDs; per XCD (start spread, end of last) cyc:",
          [(int(t0[xcc == x].max()), int(t1[xcc == x].max())) for x in np.unique(xcc)])
    print(f"  duration min/median/p90/max: {dur.min()} {int(np.median(dur))} {int(np.percentile(dur, 90))} {dur.max()}")
    order = np.argsort(t0)
    print("  first 5 starts", (t0[order[:5]] - base).tolist(), " last 5 starts", (t0[order[-5:]] - base).tolist())
    slow = np.argsort(dur)[-5:]
    print("  slowest segments", slow.tolist(), dur[slow].tolist())
    if len(sys.argv) > 2:  # per-segment rows for cost-model fitting: duration, phases, counts
        np.savetxt(sys.argv[2], np.column_stack([dur, r[:, :8], r[:, 10:16]]), fmt="%d",
                   header="dur " + " ".join(PHASES[:8]) + " " + " ".join(PHASES[10:16]))
