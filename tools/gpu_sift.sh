#!/bin/bash
# SIFT bring-up: the SIFT GPU tests, smoke, the bench line and a rocprofv3 kernel trace of
# the bench.  Each step has its own limit; the chain stops at the first failure.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_sift.py -x -v --timeout 300 --timeout-method thread > gpurun_out/sift_pytest.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/sift_trace -o run --output-format csv \
  -- python3 $ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_trace.json 2> gpurun_out/bench_trace.err
echo ok
