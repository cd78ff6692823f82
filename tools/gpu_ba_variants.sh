#!/bin/bash
# BA build variants (VO_LIB_PATH, built beside the product by make EXTRA=...): cfg3 bench lines
# without the matcher, the default first and last.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for v in default "$@" default2; do
  case $v in default|default2) L=visualodometry_amd/lib/libvo_hip.so ;; *) L=visualodometry_amd/lib/libvo_hip_$v.so ;; esac
  VO_LIB_PATH=$L timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --steps 300 --warmup 30 > $OUT/var_bench_$v.json 2> $OUT/var_bench_$v.err
done
echo done
