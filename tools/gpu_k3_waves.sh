#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out
for nw in 4 2 1; do
  VO_K3_WAVES=$nw timeout -k 10 300 python -m pytest tests/test_gpu_ba.py -x -q > gpurun_out/w${nw}_pytest.log 2>&1
  VO_K3_WAVES=$nw timeout -k 10 300 python bench.py --no-cpu-baseline --no-matcher > gpurun_out/w${nw}_bench.json 2> gpurun_out/w${nw}_bench.err
  VO_K3_WAVES=$nw VO_BA_STAMPS=1 timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > gpurun_out/w${nw}_stamps.txt 2>&1
done
echo ok
