#!/bin/bash
# PnP parity tests on the default build, then alternating PnP bench lines of two builds.
# usage: bash tools/gpu_pnp_ab.sh <baseline .so> <candidate .so>
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pnp.py tests/test_gpu_reference_trace.py > gpurun_out/pnp_ab_tests.log 2>&1
for r in 1 2 3; do
  VO_LIB_PATH=$1 timeout -k 10 120 python tools/pnp_only.py > gpurun_out/pnp_ab_a_$r.json 2>> gpurun_out/pnp_ab.err
  VO_LIB_PATH=$2 timeout -k 10 120 python tools/pnp_only.py > gpurun_out/pnp_ab_b_$r.json 2>> gpurun_out/pnp_ab.err
done
echo done
