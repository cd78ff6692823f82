set -euo pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  VO_LIB_PATH=$PWD/visualodometry_amd/lib/libvo_hip_head.so timeout -k 10 120 python tools/match_only.py > gpurun_out/mab_head_$r.txt 2>&1
  timeout -k 10 120 python tools/match_only.py > gpurun_out/mab_new_$r.txt 2>&1
done
echo done
