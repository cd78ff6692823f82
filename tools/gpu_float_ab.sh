#!/bin/bash
# Matcher parity tests on the default build, then alternating float-path bench lines of two
# builds.  usage: bash tools/gpu_float_ab.sh <baseline .so> <candidate .so>
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_match.py > gpurun_out/fab_tests.log 2>&1
for r in 1 2 3; do
  VO_LIB_PATH=$1 timeout -k 10 120 python tools/match_float_only.py > gpurun_out/fab_a_$r.json 2>> gpurun_out/fab.err
  VO_LIB_PATH=$2 timeout -k 10 120 python tools/match_float_only.py > gpurun_out/fab_b_$r.json 2>> gpurun_out/fab.err
done
echo done
