#!/bin/bash
# A/B/C of library builds on the BA-only bench (cfg3), alternating runs in one session, plus cfg4
# once each.  usage: bash tools/gpu_ba_abc.sh <lib> [<lib> ...]   (results: gpurun_out/abc_*.json)
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
for r in 1 2 3; do
  i=0
  for L in "$@"; do
    VO_LIB_PATH=$L timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline > $OUT/abc_${i}_cfg3_$r.json 2>> $OUT/abc.err
    i=$((i+1))
  done
done
i=0
for L in "$@"; do
  VO_LIB_PATH=$L timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --config cfg4 --steps 50 --warmup 5 > $OUT/abc_${i}_cfg4.json 2>> $OUT/abc.err
  i=$((i+1))
done
echo done
