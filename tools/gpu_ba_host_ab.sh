#!/bin/bash
# Host-side A/B of two library builds on the per-keyframe BA call (cfg3): BA parity tests on
# the alternative build, then tools/ba_call_breakdown.py alternately on each.
# usage: bash tools/gpu_ba_host_ab.sh <alt .so path>
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
ALT=$1
VO_LIB_PATH=$ALT timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_dropin.py tests/test_gpu_sharded_loopback.py > $OUT/hab_tests.log 2>&1
for r in 1 2 3; do
  timeout -k 10 120 python tools/ba_call_breakdown.py cfg3 > $OUT/hab_def_$r.json 2> $OUT/hab.err
  VO_LIB_PATH=$ALT timeout -k 10 120 python tools/ba_call_breakdown.py cfg3 > $OUT/hab_alt_$r.json 2>> $OUT/hab.err
done
echo done
