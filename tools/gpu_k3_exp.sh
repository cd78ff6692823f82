set -euo pipefail
mkdir -p gpurun_out
for e in 0 1 2 3; do
  VO_LIB_PATH=$PWD/visualodometry_amd/lib/libvo_hip_exp$e.so timeout -k 10 120 python tools/band_stamps.py cfg3 > gpurun_out/exp$e.txt 2>&1
done
echo ok
