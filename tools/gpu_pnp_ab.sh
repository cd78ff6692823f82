#!/bin/bash
# PnP parity tests on the default build, then alternating PnP bench lines of two or more builds.
# usage: bash tools/gpu_pnp_ab.sh <baseline .so> <candidate .so> [<candidate .so> ...]
# outputs: gpurun_out/pnp_ab_<a|b|c|...>_<round>.json
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pnp.py tests/test_gpu_reference_trace.py > gpurun_out/pnp_ab_tests.log 2>&1
tags=(a b c d e f)
for r in 1 2 3; do
  i=0
  for lib in "$@"; do
    VO_LIB_PATH=$lib timeout -k 10 120 python tools/pnp_only.py > gpurun_out/pnp_ab_${tags[$i]}_$r.json 2>> gpurun_out/pnp_ab.err
    i=$((i + 1))
  done
done
echo done
