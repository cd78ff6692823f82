#!/bin/bash
# Host-call timing (tools/gpu_host_ab.sh) plus the K1 and K3 phase stamps of the cfg3 window
# (stamped build lib/libvo_hip_stamps.so).  Usage: gpurun --timeout 1200 -- bash tools/gpu_diag.sh [tag]
set -euo pipefail
TAG=${1:-diag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_host_ab.sh $TAG
timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 $OUT/k1_rows_cfg3.txt > $OUT/k1_stamps_cfg3.txt 2>&1
timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/k3_stamps_cfg3.txt 2>&1
echo done
