#!/bin/bash
# BA correctness after planner / setup changes, then the per-call breakdown (timing build).
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_sharded_loopback.py tests/test_gpu_dropin.py tests/test_gpu_golden.py tests/test_gpu_reference_trace.py > $OUT/plan_tests.log 2>&1
timeout -k 10 120 python tools/ba_call_breakdown.py > $OUT/breakdown.json 2>&1
VO_LIB_PATH=$PWD/visualodometry_amd/lib/libvo_hip_timing.so timeout -k 10 120 python tools/ba_call_breakdown.py > $OUT/breakdown_t.json 2> $OUT/breakdown_t.err
timeout -k 10 200 python tools/host_call_latency.py > $OUT/host_latency.json 2>&1
echo done
