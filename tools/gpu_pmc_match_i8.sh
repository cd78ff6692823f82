#!/bin/bash
# int8 matcher counters (two --pmc passes) and its kernel-trace average, on tools/match_only.py.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/i8_trace -o run --output-format csv \
  -- python3 $ROOT/tools/match_only.py > gpurun_out/i8_trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  -d $ROOT/gpurun_out/i8_pmc1 -o run --output-format csv -- python3 $ROOT/tools/match_only.py > gpurun_out/i8_pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM \
  -d $ROOT/gpurun_out/i8_pmc2 -o run --output-format csv -- python3 $ROOT/tools/match_only.py > gpurun_out/i8_pmc2.log 2>&1
python3 tools/pmc_summary.py gpurun_out/i8_pmc1/run_counter_collection.csv -o gpurun_out/i8_pmc1.csv
python3 tools/pmc_summary.py gpurun_out/i8_pmc2/run_counter_collection.csv -o gpurun_out/i8_pmc2.csv
echo ok
