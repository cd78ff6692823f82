#!/bin/bash
# Bench lines only (cfg3 with the matcher / front-end legs, cfg4 BA), no tests, no profiler.
# Usage: gpurun --timeout 600 -- bash tools/gpu_bench.sh [tag]
set -euo pipefail
TAG=${1:-bench}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
echo done
