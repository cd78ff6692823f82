#!/bin/bash
# BA build variants (VO_LIB_PATH): BA GPU tests on the default, cfg3 bench lines without the
# matcher (default twice), cfg4, stamps.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_golden.py tests/test_gpu_sharded_loopback.py -x -q --timeout 200 --timeout-method thread > $OUT/k1v_tests.log 2>&1
for v in default c12 c15 c30 default; do
  if [ $v = default ]; then L=visualodometry_amd/lib/libvo_hip.so; else L=visualodometry_amd/lib/libvo_hip_$v.so; fi
  VO_LIB_PATH=$L timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --steps 300 --warmup 30 > $OUT/k1v_bench_$v.json 2> $OUT/k1v_bench_$v.err
done
timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 > $OUT/k1v_bench_cfg4.json 2> $OUT/k1v_bench_cfg4.err
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > $OUT/k1v_stamps_cfg3.txt 2>&1
echo done
