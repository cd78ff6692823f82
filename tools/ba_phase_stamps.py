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
os.environ.setdefault("VO_BA_STAMPS", "1")

from visualodometry_amd import _lib  # noqa: E402
from visualodometry_amd.ba import BASession  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config  # noqa: E402

PHASES = ["load", "backsub", "lin_obs", "reduce", "eliminate", "schur_pairs", "write", "schur_cams", "unused"]
K3 = ["k3_setup", "k3_factor(rest)", "k3_backsub", "k3_tail", "k3_data", "k3_chol", "k3_panel", "k3_trail", "k3_barrier"]

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
tot = float(out[: len(PHASES)].sum())
print(cfg, s.plan_stats())
for k in range(min(n, len(PHASES))):
    print(f"{PHASES[k]:18s} {int(out[k]):14d} cycles (sum over WGs)  {100 * out[k] / tot:5.1f} %")
t3 = float(out[len(PHASES):].sum())
for k in range(len(PHASES), n):
    print(f"{K3[k - len(PHASES)]:18s} {int(out[k]):14d} cycles (one WG)  {100 * out[k] / max(t3, 1):5.1f} %")
