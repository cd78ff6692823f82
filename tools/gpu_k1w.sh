#!/bin/bash
# One-wave K1: BA GPU tests, cfg3/cfg4 bench lines without the matcher, stamped K1 phases.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_golden.py tests/test_gpu_sharded_loopback.py -x -q --timeout 200 --timeout-method thread > $OUT/k1w_tests.log 2>&1
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --steps 200 --warmup 20 > $OUT/k1w_bench.json 2> $OUT/k1w_bench.err
timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 > $OUT/k1w_bench_cfg4.json 2> $OUT/k1w_bench_cfg4.err
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 $OUT/k1w_seg_cfg3.txt > $OUT/k1w_stamps_cfg3.txt 2>&1
timeout -k 10 300 python tools/host_call_latency.py > $OUT/k1w_host_latency.json 2> $OUT/k1w_host_latency.err
echo done
