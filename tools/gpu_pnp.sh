#!/bin/bash
# Bring-up of the new rows on the GPU: PnP and SIFT parity tests, then the whole GPU suite,
# smoke and one bench line.  Each step has its own limit; the chain stops at the first failure.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pnp_pytest.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sift.py -x -v --timeout 120 --timeout-method thread > gpurun_out/sift_pytest.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo ok
