#!/bin/bash
# GPU session for the split band layout: the BA GPU tests (split-vs-ring bitwise, layout modes,
# every cfg4 test on the split layout), K3 stamps at cfg3 and cfg4, and cfg3 / cfg4 bench lines
# alternating a base library and the product (three rounds).
# Usage: gpurun --timeout 1200 -- bash tools/gpu_split.sh tag base_name
set -euo pipefail
TAG=$1
BASE=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
VO_LIB_PATH=$L/libvo_hip_stamps.so timeout -k 10 120 python tools/band_stamps.py cfg4 > $OUT/stamps_cfg4.txt 2>&1
VO_LIB_PATH=$L/libvo_hip_stamps.so timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/stamps_cfg3.txt 2>&1
for rep in 1 2 3; do
  for n in $BASE prod; do
    LIB=$L/libvo_hip_$n.so; [ $n = prod ] && LIB=$L/libvo_hip.so
    VO_LIB_PATH=$LIB timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 \
      > $OUT/cfg4_${n}_$rep.json 2> $OUT/cfg4_${n}_$rep.err
    VO_LIB_PATH=$LIB timeout -k 10 120 python bench.py --no-matcher --no-cpu-baseline > $OUT/cfg3_${n}_$rep.json 2> $OUT/cfg3_${n}_$rep.err
  done
done
echo done
