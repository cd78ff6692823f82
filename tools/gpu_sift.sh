#!/bin/bash
# SIFT detectAndCompute bring-up: the SIFT GPU tests alone, then smoke.  Each step has its own
# limit; the chain stops at the first failure.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sift.py -x -v --timeout 300 --timeout-method thread > gpurun_out/sift_pytest.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo ok
