#!/bin/bash
# BA parity tests, K3 phase stamps, BA-only bench lines for cfg3 and cfg4 (one GPU call).
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_sharded_loopback.py > $OUT/ba_tests.log 2>&1
timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/stamps_cfg3.txt 2>&1
timeout -k 10 120 python tools/band_stamps.py cfg4 > $OUT/stamps_cfg4.txt 2>&1
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --config cfg4 --steps 50 --warmup 5 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
echo done
