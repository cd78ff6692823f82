#!/bin/bash
# GPU parity tests + one bench line (no profiler).  Usage: gpurun -- bash tools/gpu_check.sh [pytest args]
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo done
