#!/bin/bash
# K3 role experiments (timing only, results wrong): per-wave stamps of builds with one helper
# role switched off.  Build first (CPU container), e = 0 (none), 1 (trail), 2 (fwd), 3 (loader):
#   for e in 0 1 2 3; do make -C visualodometry_amd/csrc OUT=../lib/libvo_hip_exp$e.so \
#     OBJDIR=../lib/obj_exp$e EXTRA="-DVO_BA_STAMPS=1 -DVO_BA_EXP=$e" ../lib/libvo_hip_exp$e.so; done
set -euo pipefail
mkdir -p gpurun_out
for e in 0 1 2 3; do
  VO_LIB_PATH=$PWD/visualodometry_amd/lib/libvo_hip_exp$e.so timeout -k 10 120 python tools/band_stamps.py cfg3 > gpurun_out/exp$e.txt 2>&1
done
echo ok
