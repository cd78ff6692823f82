#!/bin/bash
# PnP iteration: the PnP GPU tests, then the batch sweep (256 .. 4096 frames per call).
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_pnp.py -x -q > gpurun_out/pnp_pytest.log 2>&1
timeout -k 10 600 python tools/pnp_batch_sweep.py > gpurun_out/pnp_sweep.txt 2> gpurun_out/pnp_sweep.err
echo ok
