#!/bin/bash
# Re-rank phase costs from timing-only builds (libvo_hip_rx<n>.so, EXTRA=-DVO_RERANK_EXP=<n>).
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
L=$ROOT/visualodometry_amd/lib
for v in def rx1 rx4 rx5; do
  lib=$L/libvo_hip.so; [ $v != def ] && lib=$L/libvo_hip_$v.so
  VO_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/rx_$v -o run --output-format csv \
    -- python3 $ROOT/tools/match_float_time.py > gpurun_out/rx_$v.log 2>&1
done
echo ok
