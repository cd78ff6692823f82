#!/bin/bash
# SIFT parity tests and the SIFT bench line with the default library, then the bench line of
# each variant build given (visualodometry_amd/lib/var_<name>, parity tests first).
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sift.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sift_pytest.log 2>&1
timeout -k 10 300 python tools/sift_only.py > gpurun_out/sift_new.json
if [ $# -gt 0 ]; then bash tools/gpu_sift_ab.sh "$@"; fi
echo ok
