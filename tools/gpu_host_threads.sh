#!/bin/bash
# Per-call host timing of cfg3 scratch / slid windows with the planner capped at 4, 8 and 16 threads
# (lib/libvo_hip_t4.so, lib/libvo_hip_t8.so, the product library), alternating, plus the setup's
# sections (-DVO_PLAN_TIMING build).  Usage: gpurun --timeout 900 -- bash tools/gpu_host_threads.sh [tag]
set -euo pipefail
TAG=${1:-hostthr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for T in 4 8 16; do
    LIB=visualodometry_amd/lib/libvo_hip_t$T.so
    [ $T = 16 ] && LIB=visualodometry_amd/lib/libvo_hip.so
    VO_LIB_PATH=$LIB timeout -k 10 300 python tools/ba_slide_timing.py 12 > $OUT/t${T}_$rep.json 2> $OUT/t${T}_$rep.err
  done
done
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_ptiming.so timeout -k 10 300 python tools/ba_slide_timing.py 8 \
  > $OUT/sections.json 2> $OUT/sections.err
echo done
