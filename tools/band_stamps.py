"""Diagnostic: per-phase cycles of the banded K3 (stamped build, lane 0 of each wave).

Build the stamped library first (CPU container):
  make -C visualodometry_amd/csrc OUT=../lib/libvo_hip_stamps.so OBJDIR=../lib/obj_stamps \
       EXTRA=-DVO_BA_STAMPS=1 ../lib/libvo_hip_stamps.so
then on the GPU box: ``python tools/band_stamps.py [cfg]``.  Values are the last K3
launch's; stamps perturb the schedule a little, read shares and per-step figures.
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

NK1 = 16  # K1 phase slots precede the K3 stamps
PH = ["prologue", "A: pre", "A: barrier", "A: post/helper", "merge", "B: pre", "B: barrier", "B: post/helper",
      "vmcnt drain", "sync", "BS1", "BS1 sync", "BS2", "BS2 sync", "tail", "wait reducers",
      "G pass", "c: D bcast", "c: chol6", "c: fwd6", "ld: dma issue", "ld: dma wait", "c: post loads", "c: post fma", "f: loads", "f: fwd6", "bs: 2 steps", "f: rmw"]
WAVES = ["T chain", "B chain", "T trail", "B trail", "T load", "B load", "T fwd", "B fwd"]

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
p = make_ba_config(cfg)
pr = plan_probe(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1024)
ctx = _lib.context(0)
s = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0, ctx)
s.set_state(p.poses_cw, p.points)
s.run_async(3)
s.synchronize()
NRED_MAX = 600
out = np.zeros(NK1 + 256 + 8 + 4 * NRED_MAX, dtype=np.uint64)
n = _lib.check(ctx.lib.vo_ba_debug_stamps(ctx.handle, out.ctypes.data_as(_lib.C.POINTER(_lib.C.c_uint64)),
                                           len(out)), "stamps")
st = out[NK1:NK1 + 256].reshape(8, 32).astype(np.int64)
rt = out[NK1 + 256:].astype(np.int64)
m, sp, nb = pr["band_top_rows"], pr["band_separator_rows"], pr["band_bottom_rows"]
print(cfg, "F", pr["free_poses"], "m/s/nb", m, sp, nb, "stamps read", n)
print(f"{'phase':16s}" + "".join(f"{w:>15s}" for w in WAVES))
for i, ph in enumerate(PH):
    print(f"{ph:16s}" + "".join(f"{int(st[w, i]):15d}" for w in range(8)))
print(f"{'total':16s}" + "".join(f"{int(st[w, :28].sum()):15d}" for w in range(8)))
pa = max(m, nb)
print("phase A per step (top chain): pre %.0f barrier %.0f post %.0f" % tuple(st[0, 1:4] / max(pa, 1)))
for wv, name in [(2, "trail"), (4, "load"), (6, "fwd")]:
    print("phase A per step (top %s): barrier %.0f work %.0f" % ((name,) + tuple(st[wv, 2:4] / max(pa, 1))))
if sp:
    print("phase B per step (top chain): pre %.0f barrier %.0f post %.0f" % tuple(st[0, 5:8] / sp))
    print("BS1 per step %.0f, BS2 per step (top) %.0f (bottom) %.0f" % (st[0, 10] / sp, st[0, 12] / max(m, 1),
                                                                   st[1, 12] / max(nb + sp, 1)))

if n > NK1 + 256:  # fused launch: realtime stamps (100 MHz ticks) of the solver and each reducer
    nred = (n - NK1 - 256 - 8) // 4 - 1
    t0 = rt[0]
    red = rt[8:8 + 4 * nred].reshape(nred, 4) - t0
    print("fused launch, realtime from the solver's start (ns): solver poll done %d, prologue done %d" %
          ((rt[1] - t0) * 10, (rt[2] - t0) * 10))
    for j, name in enumerate(["reducer start", "loads in", "stored+drained", "counted"]):
        v = red[:, j] * 10
        print("%-16s min %6d  p50 %6d  p90 %6d  max %6d" % (name, v.min(), np.median(v), np.percentile(v, 90), v.max()))
    print("reducer spans (ns): loads %d, store+drain %d, count %d (medians)" %
          (np.median(red[:, 1] - red[:, 0]) * 10, np.median(red[:, 2] - red[:, 1]) * 10,
           np.median(red[:, 3] - red[:, 2]) * 10))
