#!/bin/bash
# LDS counters of the BA kernels (cfg3 bench, BA only): bank-conflict cycles against LDS activity.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d $ROOT/gpurun_out/ba_lds -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-matcher > gpurun_out/ba_lds.log 2>&1
python3 tools/pmc_summary.py gpurun_out/ba_lds/run_counter_collection.csv -o gpurun_out/ba_lds.csv
echo ok
