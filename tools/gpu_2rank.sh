#!/bin/bash
# Rehearsal of the N > 1 bench path on a one-GPU box: 2 ranks pinned to device 0.
set -uo pipefail
mkdir -p gpurun_out
export VO_BENCH_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 2 > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err
echo "rc=$?"
