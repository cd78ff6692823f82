#!/bin/bash
# K3 iteration loop: BA parity tests, BA bench line, per-wave K3 stamps.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ba.py tests/test_gpu_dropin.py tests/test_gpu_comm.py -x -q > gpurun_out/k3_pytest.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-matcher > gpurun_out/k3_bench.json 2> gpurun_out/k3_bench.err
for w in 0 1 2 3; do
  VO_K3_STAMP_WAVE=$w VO_BA_STAMPS=1 timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > gpurun_out/k3w_$w.txt 2>&1
done
echo ok
