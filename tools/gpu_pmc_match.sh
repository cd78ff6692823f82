#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  -d $ROOT/gpurun_out/pmc_m1 -o run --output-format csv -- python3 $ROOT/tools/match_only.py > gpurun_out/pmc_m1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU \
  -d $ROOT/gpurun_out/pmc_m2 -o run --output-format csv -- python3 $ROOT/tools/match_only.py > gpurun_out/pmc_m2.log 2>&1
echo ok
