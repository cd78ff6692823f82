#!/bin/bash
# Host-call A/B of tuning builds (lib/libvo_hip_<name>.so) against the product library,
# alternating, three rounds: tools/ba_call_steps.py per variant.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_host_variants.sh tag name1 name2 ...
set -euo pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  timeout -k 10 300 python tools/ba_call_steps.py > $OUT/prod_$rep.json 2> $OUT/prod_$rep.err
  for n in "$@"; do
    VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_$n.so timeout -k 10 300 python tools/ba_call_steps.py > $OUT/${n}_$rep.json 2> $OUT/${n}_$rep.err
  done
done
echo done
