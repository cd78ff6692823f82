#!/bin/bash
# cfg4 parity on the copy-chain variants (diagnosis)
set -uo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for v in c100 c30 default; do
  if [ $v = default ]; then L=visualodometry_amd/lib/libvo_hip.so; else L=visualodometry_amd/lib/libvo_hip_$v.so; fi
  VO_LIB_PATH=$L timeout -k 10 200 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 120 --timeout-method thread -k "cfg4 or run_matches" > $OUT/k1c4_$v.log 2>&1
  echo "$v rc=$?"
done
