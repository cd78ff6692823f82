#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_match.py tests/test_gpu_dropin.py -x -q > gpurun_out/mq_pytest.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/mq.json 2> gpurun_out/mq.err
echo ok
