#!/bin/bash
# BA iteration: BA parity tests, BA-only bench lines (cfg3, cfg4), K1 phase stamps and K3 coarse
# stamps (cfg3, from the stamped build libvo_hip_stamps.so: make EXTRA=-DVO_BA_STAMPS=1).
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_sharded_loopback.py tests/test_gpu_golden.py tests/test_gpu_reference_trace.py > $OUT/ba_tests.log 2>&1
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --config cfg4 --steps 50 --warmup 5 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
VO_LIB_PATH=$PWD/visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > $OUT/k1st.txt 2>&1
VO_LIB_PATH=$PWD/visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/band_stamps.py cfg3 > $OUT/st1.txt 2>&1
VO_LIB_PATH=$PWD/visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/band_stamps.py cfg4 > $OUT/st4.txt 2>&1
echo done
