#!/bin/bash
# Float re-rank counters (one --pmc pass each), on tools/match_float_time.py.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS \
  -d $ROOT/gpurun_out/rr_pmc1 -o run --output-format csv -- python3 $ROOT/tools/match_float_time.py > gpurun_out/rr_pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM \
  -d $ROOT/gpurun_out/rr_pmc2 -o run --output-format csv -- python3 $ROOT/tools/match_float_time.py > gpurun_out/rr_pmc2.log 2>&1
python3 tools/pmc_summary.py gpurun_out/rr_pmc1/run_counter_collection.csv -o gpurun_out/rr_pmc1.csv
python3 tools/pmc_summary.py gpurun_out/rr_pmc2/run_counter_collection.csv -o gpurun_out/rr_pmc2.csv
echo ok
