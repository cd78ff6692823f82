#!/bin/bash
# Matcher A/B: parity tests on the default build, then the bench's matcher lines for the
# default build and an alternative one.  usage: bash tools/gpu_match_ab.sh <alt .so>
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_match.py tests/test_gpu_golden.py > $OUT/mab_tests.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/mab_def_$r.json 2> $OUT/mab.err
  VO_LIB_PATH=$1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/mab_alt_$r.json 2>> $OUT/mab.err
done
echo done
