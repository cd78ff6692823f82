#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_match.py -x -q > gpurun_out/ms_pytest.log 2>&1
for w in 2 4 8 16; do
  VO_MATCH_WGS_PER_CU=$w timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/ms_$w.json 2> gpurun_out/ms_$w.err
done
echo ok
