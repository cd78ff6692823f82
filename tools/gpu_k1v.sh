#!/bin/bash
# BA: GPU tests, cfg3 (one-wave K1) twice and cfg4 (four-wave K1) bench lines without the
# matcher, stamped K1 phases of cfg3.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_golden.py tests/test_gpu_sharded_loopback.py -x -q --timeout 200 --timeout-method thread > $OUT/k1v_tests.log 2>&1
for v in a b; do
  timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --steps 300 --warmup 30 > $OUT/k1v_bench_$v.json 2> $OUT/k1v_bench_$v.err
done
timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 > $OUT/k1v_bench_cfg4.json 2> $OUT/k1v_bench_cfg4.err
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > $OUT/k1v_stamps_cfg3.txt 2>&1
echo done
