#!/bin/bash
# PMC FETCH/WRITE passes of the BA-only bench at cfg4 (separate passes), then per-kernel traffic.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $ROOT/$OUT/c4_fetch -o run --output-format csv \
  -- python3 $ROOT/bench.py --no-matcher --no-cpu-baseline --config cfg4 --steps 10 --warmup 2 > $OUT/c4_fetch.json 2> $OUT/c4_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $ROOT/$OUT/c4_write -o run --output-format csv \
  -- python3 $ROOT/bench.py --no-matcher --no-cpu-baseline --config cfg4 --steps 10 --warmup 2 > $OUT/c4_write.json 2> $OUT/c4_write.err
python tools/pmc_traffic.py $OUT/c4_fetch/run_counter_collection.csv $OUT/c4_write/run_counter_collection.csv -o $OUT/traffic_cfg4.json > /dev/null
echo done
