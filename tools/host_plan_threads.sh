#!/bin/bash
# Host-only: the BA planner's sections (tools/plan_bench.cpp, -DVO_PLAN_TIMING) on cfg3 slide
# windows at 1, 4, 8 and 16 planner threads, on whatever host runs it (no GPU used).
# Usage: gpurun --timeout 600 -- bash tools/host_plan_threads.sh [tag]
set -euo pipefail
TAG=${1:-planthr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
python3 - <<'PY'
import sys
import numpy as np
sys.path.insert(0, ".")
from visualodometry_amd.synthetic import make_ba_slide
ws = make_ba_slide("cfg3", 6)
with open("/tmp/pb_cfg3.bin", "wb") as f:
    np.array([len(ws)], np.int32).tofile(f)
    for w in ws:
        np.array([w.poses_cw.shape[0], w.points.shape[0], w.obs_cam.size, w.n_fixed], np.int32).tofile(f)
        np.asarray(w.point_ptr, np.int32).tofile(f)
        np.asarray(w.obs_cam, np.int32).tofile(f)
        np.asarray(w.obs_uv, np.float32).tofile(f)
PY
for T in 1 4 8 16; do
  g++ -O3 -std=c++17 -pthread -DVO_PLAN_TIMING -DVO_PLAN_MAX_THREADS=$T tools/plan_bench.cpp \
    visualodometry_amd/csrc/ba_plan.cpp -o /tmp/pbt$T
  timeout -k 10 120 /tmp/pbt$T /tmp/pb_cfg3.bin 1 3 5 > $OUT/t$T.json 2> $OUT/t$T.sections
done
echo done
