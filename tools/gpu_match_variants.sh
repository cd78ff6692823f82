#!/bin/bash
# Matcher build variants (tools/build_variants.sh output under lib/var_*): parity + bench each.
set -euo pipefail
mkdir -p gpurun_out
for v in "$@"; do
  VO_LIB_PATH=$PWD/visualodometry_amd/lib/var_$v/libvo_hip.so timeout -k 10 300 python -m pytest tests/test_gpu_match.py -x -q > gpurun_out/mv_${v}_pytest.log 2>&1
  VO_LIB_PATH=$PWD/visualodometry_amd/lib/var_$v/libvo_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/mv_$v.json 2> gpurun_out/mv_$v.err
done
echo ok
