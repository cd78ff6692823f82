#!/bin/bash
# BA: GPU tests, cfg3 bench line without the matcher, stamped K1 phases of cfg3, the host call
# breakdown and latency.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > $OUT/k1v_tests.log 2>&1
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --steps 300 --warmup 30 > $OUT/k1v_bench_a.json 2> $OUT/k1v_bench_a.err
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > $OUT/k1v_stamps_cfg3.txt 2>&1
timeout -k 10 200 python tools/ba_call_breakdown.py cfg3 > $OUT/k1v_breakdown.json 2> $OUT/k1v_breakdown.err
timeout -k 10 300 python tools/host_call_latency.py > $OUT/k1v_host_latency.json 2> $OUT/k1v_host_latency.err
echo done
