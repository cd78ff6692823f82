#!/bin/bash
# Copies one tools/gpu_round.sh session's outputs from gpurun_out/ into profiles/<tag>_*
# (and the PMC traffic files, keyed to the build they measured, to profiles/traffic_cfg{3,4}.json).
# Usage: bash tools/archive_round.sh r06m
set -euo pipefail
T=$1
G=gpurun_out
P=profiles
cp $G/${T}_trace/run_kernel_stats.csv $P/${T}_kernel_stats.csv
cp $G/${T}_trace/run_domain_stats.csv $P/${T}_domain_stats.csv
cp $G/bench_trace.json $P/${T}_bench_under_rocprof.json
cp $G/bench_final.json $P/${T}_bench.json
cp $G/bench_cfg4.json $P/${T}_bench_cfg4.json
cp $G/pytest_gpu.log $P/${T}_pytest_gpu.log
cp $G/smoke.log $P/${T}_smoke.log
cp $G/mfma_busy.json $P/${T}_mfma_busy.json
cp $G/host_latency.json $P/${T}_host_latency.json
cp $G/frame_latency.json $P/${T}_frame_latency.json
for c in cfg3 cfg4; do
  cp $G/shard_projection_$c.json $P/${T}_shard_projection_$c.json
  cp $G/${T}_fetch_$c/run_counter_collection.csv $P/${T}_pmc_fetch_size_$c.csv
  cp $G/${T}_write_$c/run_counter_collection.csv $P/${T}_pmc_write_size_$c.csv
  cp $G/traffic_$c.json $P/traffic_$c.json
done
echo archived $T
