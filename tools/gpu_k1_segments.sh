#!/bin/bash
# Per-segment K1 durations and work counts (cost-model fitting), cfg3 and cfg4.
set -euo pipefail
mkdir -p gpurun_out
VO_BA_STAMPS=1 timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 gpurun_out/k1seg_cfg3.txt > gpurun_out/k1seg_cfg3.log 2>&1
VO_BA_STAMPS=1 timeout -k 10 300 python tools/ba_phase_stamps.py cfg4 gpurun_out/k1seg_cfg4.txt > gpurun_out/k1seg_cfg4.log 2>&1
echo ok
