#!/bin/bash
# SIFT kernel iteration: the SIFT GPU tests, then the SIFT bench line alone.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sift.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sift_pytest.log 2>&1
timeout -k 10 300 python tools/sift_only.py > gpurun_out/sift_bench.json 2> gpurun_out/sift_bench.err
echo ok
