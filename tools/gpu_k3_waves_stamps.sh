#!/bin/bash
# K3 sub-phase stamps from each of the four waves' point of view.
set -euo pipefail
mkdir -p gpurun_out
for w in 0 1 2 3; do
  VO_K3_STAMP_WAVE=$w VO_BA_STAMPS=1 timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > gpurun_out/k3w_$w.txt 2>&1
done
echo ok
