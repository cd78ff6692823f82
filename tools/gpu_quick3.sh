#!/bin/bash
# GPU session for round-6 changes: the product's BA / matcher / PnP / torch-coexistence GPU tests,
# K3 stamps, per-frame latencies, cfg3 bench lines alternating base / product / tuning variants
# (three rounds), cfg4 lines product / variants (two rounds), the PnP leg base / product, and the
# BA GPU tests on each variant (no -x: a variant's plan shape may differ from the one the tests
# assert).
# Usage: gpurun --timeout 1200 -- bash tools/gpu_quick3.sh tag base_name [variant ...]
set -euo pipefail
TAG=$1
BASE=$2
shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/visualodometry_amd/lib
lib() { if [ $1 = prod ]; then echo $L/libvo_hip.so; else echo $L/libvo_hip_$1.so; fi; }
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_match.py tests/test_gpu_pnp.py \
    tests/test_gpu_torch_coexist.py -x -q --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1
fi
if [ -f $L/libvo_hip_stamps.so ]; then
  VO_LIB_PATH=$L/libvo_hip_stamps.so timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/stamps.txt 2>&1
fi
timeout -k 10 180 python tools/frame_latency.py > $OUT/frame_latency.json 2> $OUT/frame_latency.err
for rep in 1 2 3; do
  for n in $BASE prod "$@"; do
    VO_LIB_PATH=$(lib $n) timeout -k 10 120 python bench.py --no-matcher --no-cpu-baseline > $OUT/cfg3_${n}_$rep.json 2> $OUT/cfg3_${n}_$rep.err
  done
done
for rep in 1 2; do
  for n in prod "$@"; do
    VO_LIB_PATH=$(lib $n) timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 \
      > $OUT/cfg4_${n}_$rep.json 2> $OUT/cfg4_${n}_$rep.err
  done
done
for n in $BASE prod; do
  VO_LIB_PATH=$(lib $n) timeout -k 10 200 python tools/pnp_only.py > $OUT/pnp_${n}.json 2> $OUT/pnp_${n}.err
done
for n in "$@"; do
  VO_LIB_PATH=$(lib $n) timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py -q --timeout 120 \
    --timeout-method thread > $OUT/tests_$n.log 2>&1 || echo "variant $n: tests failed (see log)"
done
echo done
