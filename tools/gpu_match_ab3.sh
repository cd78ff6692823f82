#!/bin/bash
# Matcher parity tests on the default build, then alternating int8 bench lines of the default
# build and candidate builds.  usage: bash tools/gpu_match_ab3.sh <candidate .so> [...]
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_match.py > gpurun_out/mab3_tests.log 2>&1
for r in 1 2 3; do
  timeout -k 10 120 python tools/match_only.py > gpurun_out/mab3_def_$r.txt 2>&1
  i=0
  for L in "$@"; do
    VO_LIB_PATH=$L timeout -k 10 120 python tools/match_only.py > gpurun_out/mab3_${i}_$r.txt 2>&1
    i=$((i+1))
  done
done
echo done
