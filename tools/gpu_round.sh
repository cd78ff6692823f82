#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace stats and the two PMC
# traffic passes.  Each GPU step has its own time limit; the chain stops at the first failure.
# Usage (from the build container): gpurun --timeout 1500 -- bash tools/gpu_round.sh r01
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/${TAG}_trace -o run --output-format csv \
  -- python3 $ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/bench_trace.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $ROOT/$OUT/${TAG}_fetch -o run --output-format csv \
  -- python3 $ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $ROOT/$OUT/${TAG}_write -o run --output-format csv \
  -- python3 $ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_write.json 2> $OUT/bench_write.err
python tools/pmc_traffic.py $OUT/${TAG}_fetch/run_counter_collection.csv \
  $OUT/${TAG}_write/run_counter_collection.csv -o $OUT/traffic.json > /dev/null
timeout -k 10 600 python bench.py --traffic-json $OUT/traffic.json > $OUT/bench_final.json 2> $OUT/bench_final.err
timeout -k 10 300 python tools/shard_projection.py cfg3 > $OUT/shard_projection_cfg3.json 2> $OUT/shard_projection_cfg3.err
timeout -k 10 300 python tools/shard_projection.py cfg4 > $OUT/shard_projection_cfg4.json 2> $OUT/shard_projection_cfg4.err
timeout -k 10 300 python tools/host_call_latency.py > $OUT/host_latency.json 2> $OUT/host_latency.err
timeout -k 10 300 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
echo done
