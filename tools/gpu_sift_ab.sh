#!/bin/bash
# A/B of SIFT builds (visualodometry_amd/lib/var_<name>): parity tests once per build, the
# SIFT bench line twice, alternating.
set -euo pipefail
mkdir -p gpurun_out
for v in "$@"; do
  VO_LIB_PATH=$PWD/visualodometry_amd/lib/var_$v/libvo_hip.so timeout -k 10 300 python -m pytest tests/test_gpu_sift.py -x -q > gpurun_out/sab_${v}_pytest.log 2>&1
done
for r in 1 2; do
  for v in "$@"; do
    VO_LIB_PATH=$PWD/visualodometry_amd/lib/var_$v/libvo_hip.so timeout -k 10 300 python tools/sift_only.py > gpurun_out/sab_${v}_$r.json 2>/dev/null
  done
done
echo ok
