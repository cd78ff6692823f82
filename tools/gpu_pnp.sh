#!/bin/bash
# PnP bring-up on the GPU: parity tests, then the rest of the GPU suite.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pnp_pytest.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo ok
