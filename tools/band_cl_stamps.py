"""Diagnostic: per-role cycles of the critical-lane K3 (stamped build, lane 0 of each wave).

Build the stamped library first (CPU container):
  make -C visualodometry_amd/csrc OUT=../lib/libvo_hip_stamps.so OBJDIR=../lib/obj_stamps \
       EXTRA=-DVO_BA_STAMPS=1 ../lib/libvo_hip_stamps.so
then on the GPU box: ``python tools/band_cl_stamps.py [cfg]``.  Slot 30 collects the time
between a role's steps (loop overhead); per-step figures divide by the side's step count.
"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("VO_LIB_PATH", str(ROOT / "visualodometry_amd" / "lib" / "libvo_hip_stamps.so"))

from visualodometry_amd import _lib  # noqa: E402
from visualodometry_amd.ba import BASession, plan_probe  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config  # noqa: E402

NK1 = 16
PH = {0: "prologue", 8: "vmcnt drain", 9: "sync", 10: "BS1", 11: "BS1 sync", 12: "BS2", 13: "BS2 sync",
      14: "tail", 16: "G pass", 17: "C pivots+pub", 18: "C lazy wait", 19: "C lazy+solve", 20: "C next wait",
      21: "C next", 22: "F wait", 23: "F work", 24: "T wait", 25: "T work", 26: "merge barrier",
      27: "merge", 28: "phase S (top)", 29: "G set 0 (bot)", 30: "loop"}
WAVES = ["T chain", "B chain", "T trail1", "B trail1", "T fwd", "B fwd", "T trail2", "B trail2"]

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
p = make_ba_config(cfg)
pr = plan_probe(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1024)
ctx = _lib.context(0)
s = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0, ctx)
s.set_state(p.poses_cw, p.points)
s.run_async(3)
s.synchronize()
out = np.zeros(NK1 + 256, dtype=np.uint64)
n = _lib.check(ctx.lib.vo_ba_debug_stamps(ctx.handle, out.ctypes.data_as(_lib.C.POINTER(_lib.C.c_uint64)),
                                           len(out)), "stamps")
st = out[NK1:].reshape(8, 32).astype(np.int64)
m, sp, nb = pr["band_top_rows"], pr["band_separator_rows"], pr["band_bottom_rows"]
print(cfg, "F", pr["free_poses"], "m/s/nb", m, sp, nb, "stamps read", n)
print(f"{'phase':16s}" + "".join(f"{w:>10s}" for w in WAVES))
for i, ph in PH.items():
    print(f"{ph:16s}" + "".join(f"{int(st[w, i]):10d}" for w in range(8)))
print(f"{'total':16s}" + "".join(f"{int(st[w, :].sum()):10d}" for w in range(8)))
steps = m + sp
print("per step (top, %d steps): " % steps + " ".join(f"{PH[i]}={st[0, i] / steps:.0f}" for i in range(17, 22)))
