#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out
for v in 64 32; do
  export VO_LIB_PATH=$(pwd)/visualodometry_amd/lib/v$v/libvo_hip.so
  timeout -k 10 300 python -m pytest tests/test_gpu_ba.py -x -q > gpurun_out/c${v}_pytest.log 2>&1
  for s in 512 768 1024 2048; do
    VO_BA_SEGMENTS=$s timeout -k 10 300 python bench.py --no-cpu-baseline --no-matcher > gpurun_out/c${v}_$s.json 2> gpurun_out/c${v}_$s.err
  done
done
echo ok
