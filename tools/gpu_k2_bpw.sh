#!/bin/bash
# K2 profile blocks per workgroup (tuning builds libvo_hip_rb<n>.so, EXTRA=-DVO_RED_BLOCKS_PER_WG=<n>):
# BA parity on one variant, then rocprofv3 kernel averages of each build.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
L=$ROOT/visualodometry_amd/lib
VO_LIB_PATH=$L/libvo_hip_rb4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba.py > gpurun_out/rb_t.txt 2>&1
for v in def rb2 rb4 rb8; do
  lib=$L/libvo_hip.so; [ $v != def ] && lib=$L/libvo_hip_$v.so
  VO_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/rb_$v -o run --output-format csv \
    -- python3 $ROOT/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-matcher > gpurun_out/rb_$v.json 2>&1
done
echo ok
