"""Writes a cfg-sized slide sequence for tools/plan_bench.cpp, builds and runs it (host only).
Usage: python tools/plan_bench.py [cfg] [n_windows] [reps]"""
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from visualodometry_amd.synthetic import make_ba_slide  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
nwin = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
exe = Path(tempfile.gettempdir()) / "plan_bench"
subprocess.run(["g++", "-O3", "-std=c++17", "-pthread", str(ROOT / "tools" / "plan_bench.cpp"),
                str(ROOT / "visualodometry_amd" / "csrc" / "ba_plan.cpp"), "-o", str(exe)] +
               (["-DVO_PLAN_TIMING"] if "--timing" in sys.argv else []), check=True)
ws = make_ba_slide(cfg, nwin)
with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
    np.array([len(ws)], np.int32).tofile(f)
    for w in ws:
        np.array([w.poses_cw.shape[0], w.points.shape[0], w.obs_cam.size, w.n_fixed], np.int32).tofile(f)
        np.asarray(w.point_ptr, np.int32).tofile(f)
        np.asarray(w.obs_cam, np.int32).tofile(f)
        np.asarray(w.obs_uv, np.float32).tofile(f)
    path = f.name
for so, sc in [(1, 3), (1, 1)]:
    out = subprocess.run([str(exe), path, str(so), str(sc), str(reps)], capture_output=True, text=True, check=True)
    print(cfg, f"seg_obs={so} seg_chunks={sc}", out.stdout.strip())
    if out.stderr:
        sys.stderr.write(out.stderr[-3000:])
