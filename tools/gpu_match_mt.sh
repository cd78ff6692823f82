#!/bin/bash
# int8 matcher: M tiles per wave / workgroups per CU variants (tuning builds), parity then timing.
set -euo pipefail
mkdir -p gpurun_out
L=$PWD/visualodometry_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_match.py tests/test_gpu_golden.py > gpurun_out/mt_t_A.txt 2>&1
for v in B C D; do VO_LIB_PATH=$L/libvo_hip_mt$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_match.py > gpurun_out/mt_t_$v.txt 2>&1; done
for r in 1 2; do
  echo "A $(timeout -k 10 120 python tools/match_only.py)"
  for v in B C D; do echo "$v $(VO_LIB_PATH=$L/libvo_hip_mt$v.so timeout -k 10 120 python tools/match_only.py)"; done
done > gpurun_out/mt_time.txt 2>&1
