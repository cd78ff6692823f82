#!/bin/bash
# Host-call latency and the setup's sections (product library: vo_ba_plan_stats), and the
# landmark-shard projections.  Usage: gpurun --timeout 900 -- bash tools/gpu_host.sh [tag]
set -euo pipefail
TAG=${1:-host}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/host_call_latency.py > $OUT/host_latency.json 2> $OUT/host_latency.err
timeout -k 10 300 python tools/ba_slide_timing.py 12 > $OUT/slide_timing.json 2> $OUT/slide_timing.err
timeout -k 10 300 python tools/shard_projection.py cfg3 > $OUT/shard_projection_cfg3.json 2> $OUT/shard_projection_cfg3.err
timeout -k 10 300 python tools/shard_projection.py cfg4 > $OUT/shard_projection_cfg4.json 2> $OUT/shard_projection_cfg4.err
echo done
