#!/bin/bash
# BA GPU tests, then the per-call host timing of cfg3 scratch and slid windows (three runs of the
# product library, one of a -DVO_PLAN_TIMING build for the setup's sections), host_call_latency.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_host_ab.sh [tag]
set -euo pipefail
TAG=${1:-hostab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_sharded_loopback.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_ba.log 2>&1
for rep in 1 2 3; do
  timeout -k 10 300 python tools/ba_slide_timing.py 12 > $OUT/spin_$rep.json 2> $OUT/spin_$rep.err
done
timeout -k 10 300 python tools/host_call_latency.py > $OUT/host_latency.json 2> $OUT/host_latency.err
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_ptiming.so timeout -k 10 300 python tools/ba_slide_timing.py 8 \
  > $OUT/sections.json 2> $OUT/sections.err
echo done
