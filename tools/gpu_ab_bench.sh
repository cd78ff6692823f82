#!/bin/bash
# Same-box A/B of tuning builds (lib/libvo_hip_<name>.so) against the product library: the BA GPU
# tests on each variant, then cfg3 and cfg4 BA bench lines alternating, two rounds.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_ab_bench.sh tag name1 [name2 ...]
# (NO_TESTS=1: bench lines only, e.g. for a variant whose plan shape the tests do not expect)
set -euo pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for n in "$@"; do
  [ -n "${NO_TESTS:-}" ] && break
  VO_LIB_PATH=$PWD/visualodometry_amd/lib/libvo_hip_$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py \
    -x -q --timeout 120 --timeout-method thread > $OUT/tests_$n.log 2>&1
done
for rep in 1 2; do
  for n in prod "$@"; do
    LIB=$PWD/visualodometry_amd/lib/libvo_hip_$n.so
    [ $n = prod ] && LIB=$PWD/visualodometry_amd/lib/libvo_hip.so
    VO_LIB_PATH=$LIB timeout -k 10 120 python bench.py --no-matcher --no-cpu-baseline > $OUT/cfg3_${n}_$rep.json 2> $OUT/cfg3_${n}_$rep.err
    VO_LIB_PATH=$LIB timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 \
      > $OUT/cfg4_${n}_$rep.json 2> $OUT/cfg4_${n}_$rep.err
  done
done
echo done
