#!/bin/bash
# Matcher iteration: parity tests, the float-path bench line and the int8 bench line.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_match.py -x -q > gpurun_out/mf_pytest.log 2>&1
timeout -k 10 300 python tools/match_float_only.py > gpurun_out/mf.json 2> gpurun_out/mf.err
timeout -k 10 300 python tools/match_only.py > gpurun_out/mi.txt 2> gpurun_out/mi.err
echo ok
