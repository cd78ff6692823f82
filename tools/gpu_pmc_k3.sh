#!/bin/bash
# SQ counters for the BA kernels (two --pmc passes, no tracing domains).
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU \
  -d $ROOT/gpurun_out/pmc_k3a -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-matcher > gpurun_out/pmc_k3a.json 2> gpurun_out/pmc_k3a.err
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC \
  -d $ROOT/gpurun_out/pmc_k3b -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-matcher > gpurun_out/pmc_k3b.json 2> gpurun_out/pmc_k3b.err
echo ok
