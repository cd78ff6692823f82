#!/bin/bash
# BA GPU tests, then the host call A/B: the product library (planner workers poll during a plan)
# against a -DVO_PLAN_SESSION_SPIN=0 build (lib/libvo_hip_nospin.so), alternating, plus the cfg3 /
# cfg4 bench lines.  Usage: gpurun --timeout 1200 -- bash tools/gpu_host_ab.sh [tag]
set -euo pipefail
TAG=${1:-hostab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_sharded_loopback.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_ba.log 2>&1
for rep in 1 2 3; do
  timeout -k 10 300 python tools/ba_slide_timing.py 12 > $OUT/spin_$rep.json 2> $OUT/spin_$rep.err
  VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_nospin.so timeout -k 10 300 python tools/ba_slide_timing.py 12 > $OUT/nospin_$rep.json 2> $OUT/nospin_$rep.err
done
timeout -k 10 300 python tools/host_call_latency.py > $OUT/host_latency.json 2> $OUT/host_latency.err
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_ptiming.so timeout -k 10 300 python tools/ba_slide_timing.py 8 \
  > $OUT/sections.json 2> $OUT/sections.err
timeout -k 10 120 python bench.py --no-matcher --no-cpu-baseline > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err
timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
echo done
