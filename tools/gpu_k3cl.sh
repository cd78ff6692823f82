#!/bin/bash
# Critical-lane K3 iteration: the step microbenchmark, the BA GPU tests, a cfg3 bench line
# without the matcher and a kernel-trace profile of it.  Each GPU step has its own limit.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 5 60 ./tools/microbench/k3_crit > $OUT/k3_crit.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $OUT/k3cl_tests.log 2>&1
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --steps 200 --warmup 20 > $OUT/k3cl_bench.json 2> $OUT/k3cl_bench.err
timeout -k 10 200 python bench.py --config cfg2 --no-matcher --no-cpu-baseline --steps 200 --warmup 20 > $OUT/k3cl_bench_cfg2.json 2> $OUT/k3cl_bench_cfg2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/k3cl_trace -o run --output-format csv \
  -- python3 $ROOT/bench.py --no-matcher --no-cpu-baseline --steps 200 --warmup 20 > $OUT/k3cl_trace.json 2> $OUT/k3cl_trace.err
echo done
