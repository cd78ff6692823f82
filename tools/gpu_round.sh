#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace stats, the PMC traffic
# passes of cfg3 and cfg4 (keyed to this build: tools/pmc_traffic.py), the matcher MFMA-busy
# pass, and the final bench lines with the matching traffic.  Each GPU step has its own time
# limit; the chain stops at the first failure.
# Usage (from the build container): gpurun --timeout 1500 -- bash tools/gpu_round.sh r06 [notest]
set -euo pipefail
TAG=${1:-r04}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
if [ "${2:-}" != "notest" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/${TAG}_trace -o run --output-format csv \
  -- python3 $ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/bench_trace.err
for CFG in cfg3 cfg4; do
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $ROOT/$OUT/${TAG}_fetch_$CFG -o run --output-format csv \
    -- python3 $ROOT/bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_fetch_$CFG.json 2> $OUT/bench_fetch_$CFG.err
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $ROOT/$OUT/${TAG}_write_$CFG -o run --output-format csv \
    -- python3 $ROOT/bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_write_$CFG.json 2> $OUT/bench_write_$CFG.err
  python tools/pmc_traffic.py $OUT/${TAG}_fetch_$CFG/run_counter_collection.csv \
    $OUT/${TAG}_write_$CFG/run_counter_collection.csv --config $CFG -o $OUT/traffic_$CFG.json > /dev/null
done
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $ROOT/$OUT/${TAG}_mfma_i8 -o run --output-format csv -- python3 $ROOT/tools/match_only.py > $OUT/mfma_i8.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $ROOT/$OUT/${TAG}_mfma_f -o run --output-format csv -- python3 $ROOT/tools/match_float_only.py > $OUT/mfma_f.log 2>&1
python tools/mfma_busy.py $OUT/${TAG}_mfma_i8/run_counter_collection.csv $OUT/${TAG}_mfma_f/run_counter_collection.csv \
  -o $OUT/mfma_busy.json > /dev/null
timeout -k 10 600 python bench.py --traffic-json $OUT/traffic_cfg3.json > $OUT/bench_final.json 2> $OUT/bench_final.err
timeout -k 10 300 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 \
  --traffic-json $OUT/traffic_cfg4.json > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
timeout -k 10 300 python tools/shard_projection.py cfg3 > $OUT/shard_projection_cfg3.json 2> $OUT/shard_projection_cfg3.err
timeout -k 10 300 python tools/shard_projection.py cfg4 > $OUT/shard_projection_cfg4.json 2> $OUT/shard_projection_cfg4.err
timeout -k 10 300 python tools/host_call_latency.py > $OUT/host_latency.json 2> $OUT/host_latency.err
timeout -k 10 180 python tools/frame_latency.py > $OUT/frame_latency.json 2> $OUT/frame_latency.err
echo done
