#!/bin/bash
# int8 sweep timing-only builds (libvo_hip_me<n>.so, EXTRA=-DVO_MATCH_EXP=<n>): kernel averages.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
L=$ROOT/visualodometry_amd/lib
for v in def me1 me2; do
  lib=$L/libvo_hip.so; [ $v != def ] && lib=$L/libvo_hip_$v.so
  VO_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/me_$v -o run --output-format csv \
    -- python3 $ROOT/tools/match_only.py > gpurun_out/me_$v.log 2>&1
done
echo ok
