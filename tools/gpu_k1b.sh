#!/bin/bash
# Measurements of the held-back branch r04-k1-unverified, built beside the product as
# lib/libvo_hip_k1b.so (VO_LIB_PATH): BA parity tests, cfg3 lines against the product library,
# K1 waves per workgroup, cfg4 on the one-wave K1, host call latency.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
K=visualodometry_amd/lib/libvo_hip_k1b.so
VO_LIB_PATH=$K timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 200 --timeout-method thread > $OUT/k1b_tests.log 2>&1
echo tests-ok
timeout -k 10 150 python bench.py --no-matcher --no-cpu-baseline --steps 300 --warmup 30 > $OUT/k1b_bench_main.json 2> $OUT/k1b_bench_main.err
for nw in 1 2 3 6; do
  VO_LIB_PATH=$K VO_BA_K1_WAVES=$nw timeout -k 10 150 python bench.py --no-matcher --no-cpu-baseline --steps 300 --warmup 30 > $OUT/k1b_bench_$nw.json 2> $OUT/k1b_bench_$nw.err
done
timeout -k 10 150 python bench.py --no-matcher --no-cpu-baseline --steps 300 --warmup 30 > $OUT/k1b_bench_main2.json 2> $OUT/k1b_bench_main2.err
VO_LIB_PATH=$K timeout -k 10 200 python tools/host_call_latency.py > $OUT/k1b_host_latency.json 2> $OUT/k1b_host_latency.err
VO_LIB_PATH=$K VO_BA_WAVE=1 timeout -k 10 150 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 30 --warmup 3 > $OUT/k1b_cfg4_wave1.json 2> $OUT/k1b_cfg4_wave1.err
echo done
