#!/bin/bash
# Re-rank pipeline depth (tuning builds libvo_hip_rd<n>.so, EXTRA=-DVO_RERANK_DEPTH=<n>): parity, then
# rocprofv3 kernel averages of each build.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
L=$ROOT/visualodometry_amd/lib
VO_LIB_PATH=$L/libvo_hip_rd6.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_match.py > gpurun_out/rd_t.txt 2>&1
for v in def rd4 rd6; do
  lib=$L/libvo_hip.so; [ $v != def ] && lib=$L/libvo_hip_$v.so
  VO_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/rd_$v -o run --output-format csv \
    -- python3 $ROOT/tools/match_float_time.py > gpurun_out/rd_$v.log 2>&1
done
echo ok
