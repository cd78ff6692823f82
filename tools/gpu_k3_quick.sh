#!/bin/bash
# K3 iteration: BA parity tests, BA-only bench lines (cfg3, cfg4), coarse and fine K3 stamps (cfg3).
# Build first (CPU container): make -C visualodometry_amd/csrc, plus the two stamped libraries
# (EXTRA=-DVO_BA_STAMPS=1 -> libvo_hip_stamps.so, =2 -> libvo_hip_stamps2.so).
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_sharded_loopback.py > $OUT/ba_tests.log 2>&1
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --config cfg4 --steps 50 --warmup 5 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/st1.txt 2>&1
VO_LIB_PATH=$PWD/visualodometry_amd/lib/libvo_hip_stamps2.so timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/st2.txt 2>&1
echo done
