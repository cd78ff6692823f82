#!/bin/bash
# One-wave K1 with NW segments (waves) per workgroup (VO_BA_K1_WAVES): BA GPU tests at 2 and 6,
# cfg3 bench lines for 1, 2, 3, 6 and 1 again, stamped K1 with per-XCD dispatch spread.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > $OUT/k1nw_tests1.log 2>&1
VO_BA_K1_WAVES=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 200 --timeout-method thread > $OUT/k1nw_tests2.log 2>&1
VO_BA_K1_WAVES=6 timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 200 --timeout-method thread -k "oracle or determin" > $OUT/k1nw_tests6.log 2>&1
for nw in 1 2 3 6 1; do
  VO_BA_K1_WAVES=$nw timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --steps 300 --warmup 30 > $OUT/k1nw_bench_$nw.json 2> $OUT/k1nw_bench_$nw.err
done
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > $OUT/k1nw_stamps_cfg3.txt 2>&1
echo done
# cfg4 on the one-wave K1 (nine rounds of one-chunk segments) against the four-wave default
VO_BA_WAVE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 200 --timeout-method thread -k "cfg4" > $OUT/k1nw_cfg4wave_tests.log 2>&1
for w in 1 0; do
  VO_BA_WAVE=$w timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 > $OUT/k1nw_cfg4_wave$w.json 2> $OUT/k1nw_cfg4_wave$w.err
done
echo done2
timeout -k 10 300 python tools/host_call_latency.py > $OUT/k1nw_host_latency.json 2> $OUT/k1nw_host_latency.err
echo done3
