# Same-box A/B of SIFT library builds: bash tools/gpu_sift_ab.sh <out> <lib name> <lib name> ...
set -euo pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
L=$PWD/visualodometry_amd/lib
for round in 1 2; do
  for lib in "$@"; do
    VO_LIB_PATH=$L/$lib timeout -k 10 240 python tools/sift_ab.py > $OUT/${lib}_$round.json 2> $OUT/${lib}_$round.err
    tail -1 $OUT/${lib}_$round.json
  done
done
echo done
