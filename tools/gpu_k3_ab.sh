#!/bin/bash
# Same-box A/B of K3 builds: the BA GPU tests on the product library, stamps of two stamped
# builds (lib/libvo_hip_<stampsA|stampsB>.so), then cfg3 bench lines alternating between a
# baseline library and the product library, three rounds.
# Usage: gpurun --timeout 900 -- bash tools/gpu_k3_ab.sh tag base_name [stampsA stampsB]
set -euo pipefail
TAG=$1
BASE=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/visualodometry_amd/lib
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
fi
if [ -n "${3:-}" ]; then
  VO_LIB_PATH=$L/libvo_hip_$3.so timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/stamps_$3.txt 2>&1
  VO_LIB_PATH=$L/libvo_hip_$4.so timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/stamps_$4.txt 2>&1
fi
for rep in 1 2 3; do
  for n in $BASE prod; do
    LIB=$L/libvo_hip_$n.so
    [ $n = prod ] && LIB=$L/libvo_hip.so
    VO_LIB_PATH=$LIB timeout -k 10 120 python bench.py --no-matcher --no-cpu-baseline > $OUT/cfg3_${n}_$rep.json 2> $OUT/cfg3_${n}_$rep.err
  done
done
if [ -n "${CFG4:-}" ]; then
  for rep in 1 2; do
    for n in $BASE prod; do
      LIB=$L/libvo_hip_$n.so
      [ $n = prod ] && LIB=$L/libvo_hip.so
      VO_LIB_PATH=$LIB timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 \
        > $OUT/cfg4_${n}_$rep.json 2> $OUT/cfg4_${n}_$rep.err
    done
  done
fi
echo done
