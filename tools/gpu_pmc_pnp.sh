#!/bin/bash
# PMC passes on the PnP bench leg (tools/pnp_only.py): issue/stall split, instruction mix,
# and the instruction-cache counters (pnp_hyp's code object is 252 KB).
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES \
  -d $ROOT/gpurun_out/pmc_p1 -o run --output-format csv -- python3 $ROOT/tools/pnp_only.py > gpurun_out/pmc_p1.log 2>&1
[ -n "${NO_ICACHE:-}" ] || timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES \
  -d $ROOT/gpurun_out/pmc_p2 -o run --output-format csv -- python3 $ROOT/tools/pnp_only.py > gpurun_out/pmc_p2.log 2>&1
echo ok
