#!/bin/bash
# A/B of two matcher builds (visualodometry_amd/lib/var_<name>) in one session: int8 and
# float bench lines, alternating.
set -euo pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    VO_LIB_PATH=$PWD/visualodometry_amd/lib/var_$v/libvo_hip.so timeout -k 10 300 python tools/match_only.py > gpurun_out/ab_${v}_i8_$r.txt 2>/dev/null
    VO_LIB_PATH=$PWD/visualodometry_amd/lib/var_$v/libvo_hip.so timeout -k 10 300 python tools/match_float_only.py > gpurun_out/ab_${v}_f32_$r.json 2>/dev/null
  done
done
echo ok
