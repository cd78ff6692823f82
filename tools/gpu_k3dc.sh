#!/bin/bash
# K3 chain iteration: BA GPU tests, cfg3/cfg4 bench lines without the matcher, a kernel-trace
# profile.  Each GPU step has its own limit.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $OUT/k3dc_tests.log 2>&1
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --steps 200 --warmup 20 > $OUT/k3dc_bench.json 2> $OUT/k3dc_bench.err
timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 100 --warmup 10 > $OUT/k3dc_bench_cfg4.json 2> $OUT/k3dc_bench_cfg4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/k3dc_trace -o run --output-format csv \
  -- python3 $ROOT/bench.py --no-matcher --no-cpu-baseline --steps 200 --warmup 20 > $OUT/k3dc_trace.json 2> $OUT/k3dc_trace.err
echo done
