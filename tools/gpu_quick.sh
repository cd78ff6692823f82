#!/bin/bash
# Small GPU session: BA, matcher and torch-coexistence GPU tests, K3 stamps of the stamped build,
# the cold-setup diagnostic, per-frame latencies, and cfg3 A/B bench lines (base vs product).
# Usage: gpurun --timeout 900 -- bash tools/gpu_quick.sh tag base_name
set -euo pipefail
TAG=$1
BASE=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/visualodometry_amd/lib
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_match.py tests/test_gpu_torch_coexist.py \
    -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
fi
if [ -f $L/libvo_hip_stamps.so ]; then
  VO_LIB_PATH=$L/libvo_hip_stamps.so timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/stamps.txt 2>&1
fi
timeout -k 10 120 python tools/cold_setup.py cfg3 > $OUT/cold_setup.json 2> $OUT/cold_setup.err
timeout -k 10 120 python tools/cold_setup.py cfg3 reserve > $OUT/cold_setup_reserve.json 2> $OUT/cold_setup_reserve.err
timeout -k 10 180 python tools/frame_latency.py > $OUT/frame_latency.json 2> $OUT/frame_latency.err
for rep in 1 2 3; do
  for n in $BASE prod; do
    LIB=$L/libvo_hip_$n.so
    [ $n = prod ] && LIB=$L/libvo_hip.so
    VO_LIB_PATH=$LIB timeout -k 10 120 python bench.py --no-matcher --no-cpu-baseline > $OUT/cfg3_${n}_$rep.json 2> $OUT/cfg3_${n}_$rep.err
  done
done
echo done
