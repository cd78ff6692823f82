#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_ba.py -x -q > gpurun_out/sw_pytest.log 2>&1
for s in 512 1024 2048; do
  VO_BA_SEGMENTS=$s timeout -k 10 300 python bench.py --no-cpu-baseline --no-matcher > gpurun_out/sw_$s.json 2> gpurun_out/sw_$s.err
done
VO_BA_STAMPS=1 timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > gpurun_out/sw_stamps.txt 2>&1
echo ok
