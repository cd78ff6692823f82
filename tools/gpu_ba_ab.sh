#!/bin/bash
# A/B of two builds of the library on the BA-only bench (cfg3, cfg4), parity tests on the default build.
# usage: bash tools/gpu_ba_ab.sh <alt .so path>
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
ALT=$1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba.py > $OUT/ab_tests.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline > $OUT/ab_def_cfg3_$r.json 2> $OUT/ab.err
  VO_LIB_PATH=$ALT timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline > $OUT/ab_alt_cfg3_$r.json 2>> $OUT/ab.err
done
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --config cfg4 --steps 50 --warmup 5 > $OUT/ab_def_cfg4.json 2>> $OUT/ab.err
VO_LIB_PATH=$ALT timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --config cfg4 --steps 50 --warmup 5 > $OUT/ab_alt_cfg4.json 2>> $OUT/ab.err
echo done
