#!/bin/bash
# BA GPU tests + cfg3 / cfg4 BA bench lines + the K3 stamps of cfg3 (stamped build).
# Usage: gpurun --timeout 900 -- bash tools/gpu_ba_quick.sh [tag]
set -euo pipefail
TAG=${1:-baq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_sharded_loopback.py tests/test_gpu_golden.py tests/test_gpu_reference_trace.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_ba.log 2>&1
for rep in 1 2; do
  timeout -k 10 120 python bench.py --no-matcher --no-cpu-baseline > $OUT/bench_cfg3_$rep.json 2> $OUT/bench_cfg3_$rep.err
done
timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/k3_stamps_cfg3.txt 2>&1
timeout -k 10 300 python tools/host_call_latency.py > $OUT/host_latency.json 2> $OUT/host_latency.err
timeout -k 10 300 python tools/ba_call_steps.py > $OUT/call_steps.json 2> $OUT/call_steps.err
echo done
