#!/bin/bash
# Critical-lane K3 iteration: BA GPU tests, cfg3/cfg2 bench lines without the matcher, the
# stamped per-role cycles, a kernel-trace profile.  Each GPU step has its own limit.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $OUT/k3cl_tests.log 2>&1
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --steps 200 --warmup 20 > $OUT/k3cl_bench.json 2> $OUT/k3cl_bench.err
timeout -k 10 200 python bench.py --config cfg2 --no-matcher --no-cpu-baseline --steps 200 --warmup 20 > $OUT/k3cl_bench_cfg2.json 2> $OUT/k3cl_bench_cfg2.err
timeout -k 10 120 python tools/band_cl_stamps.py cfg3 > $OUT/cl_stamps_cfg3.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/k3cl_trace -o run --output-format csv \
  -- python3 $ROOT/bench.py --no-matcher --no-cpu-baseline --steps 200 --warmup 20 > $OUT/k3cl_trace.json 2> $OUT/k3cl_trace.err
echo done
