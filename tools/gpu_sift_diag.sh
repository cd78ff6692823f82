#!/bin/bash
# Timing-only descriptor diagnostics: the SIFT bench line with the default library and with
# variant builds (visualodometry_amd/lib/var_<name>) whose results are NOT correct, twice each.
set -euo pipefail
mkdir -p gpurun_out

for r in 1 2; do
  timeout -k 10 300 python tools/sift_only.py > gpurun_out/sdiag_base_$r.json
  for v in "$@"; do
    VO_LIB_PATH=$PWD/visualodometry_amd/lib/var_$v/libvo_hip.so timeout -k 10 300 python tools/sift_only.py --no-check > gpurun_out/sdiag_${v}_$r.json
  done
done
echo ok
