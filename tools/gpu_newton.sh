#!/bin/bash
# K3 with and without the Newton step after v_rsq_f64 (precision + speed)
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_ba.py tests/test_gpu_dropin.py -x -q > gpurun_out/nw1_pytest.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-matcher > gpurun_out/nw1_bench.json 2> gpurun_out/nw1_bench.err
VO_BA_STAMPS=1 timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > gpurun_out/nw1_stamps.txt 2>&1
cp visualodometry_amd/lib/libvo_hip.so /tmp/keep.so
cp visualodometry_amd/lib/libvo_hip_nonewton.so visualodometry_amd/lib/libvo_hip.so
timeout -k 10 300 python -m pytest tests/test_gpu_ba.py -q > gpurun_out/nw0_pytest.log 2>&1 || true
timeout -k 10 300 python bench.py --no-cpu-baseline --no-matcher > gpurun_out/nw0_bench.json 2> gpurun_out/nw0_bench.err
cp /tmp/keep.so visualodometry_amd/lib/libvo_hip.so
echo ok
