#!/bin/bash
# K1 stall profile (cfg3 bench, BA only): wave cycles against busy / waiting / VALU / LDS
# activity, LDS bank conflicts.  Two passes (each within the per-pass counter limits).
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS \
  -d $ROOT/gpurun_out/k1_pmc_a -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-matcher > gpurun_out/k1_pmc_a.log 2>&1
python3 tools/pmc_summary.py gpurun_out/k1_pmc_a/run_counter_collection.csv -o gpurun_out/k1_pmc_a.csv
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  -d $ROOT/gpurun_out/k1_pmc_b -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-matcher > gpurun_out/k1_pmc_b.log 2>&1
python3 tools/pmc_summary.py gpurun_out/k1_pmc_b/run_counter_collection.csv -o gpurun_out/k1_pmc_b.csv
echo ok
