#!/bin/bash
# K3 LDS bank conflicts by role: the default build and the timing-only builds without the
# trailing (1), forward-substitution (2) or loader (3) wave (libvo_hip_exp<n>.so, EXTRA=-DVO_BA_EXP=<n>).
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
L=$ROOT/visualodometry_amd/lib
for v in def exp1 exp2 exp3; do
  lib=$L/libvo_hip.so; [ $v != def ] && lib=$L/libvo_hip_$v.so
  VO_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
    -d $ROOT/gpurun_out/k3lds_$v -o run --output-format csv -- python3 $ROOT/tools/ba_only.py > gpurun_out/k3lds_$v.log 2>&1
  python3 tools/pmc_summary.py gpurun_out/k3lds_$v/run_counter_collection.csv -o gpurun_out/k3lds_$v.csv
done
echo ok
