#!/bin/bash
# int8 matcher: split-count variants (tuning builds libvo_hip_W<n>.so with
# EXTRA=-DVO_MATCH_WGS_PER_CU=<n>), parity then timing against the default build.
set -euo pipefail
mkdir -p gpurun_out
L=$PWD/visualodometry_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_match.py > gpurun_out/sp_t_def.txt 2>&1
for v in W3 W4; do VO_LIB_PATH=$L/libvo_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_match.py > gpurun_out/sp_t_$v.txt 2>&1; done
for r in 1 2; do
  echo "def $(timeout -k 10 120 python tools/match_only.py)"
  for v in W3 W4; do echo "$v $(VO_LIB_PATH=$L/libvo_hip_$v.so timeout -k 10 120 python tools/match_only.py)"; done
done > gpurun_out/sp_time.txt 2>&1
