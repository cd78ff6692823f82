#!/bin/bash
# BA-only cfg3 bench lines for several builds, alternating (usage: bash tools/gpu_ba_variants_bench.sh a.so b.so ...).
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline > $OUT/vb_default_$r.json 2>> $OUT/vb.err
  for so in "$@"; do
    n=$(basename $so .so)
    VO_LIB_PATH=$PWD/$so timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline > $OUT/vb_${n}_$r.json 2>> $OUT/vb.err
  done
done
echo done
