#!/bin/bash
# Slide-stable plan: BA GPU tests (take-over == scratch), drop-in/trace replays, K1 with the
# group-partitioned plan (bench without the matcher), per-call host latency, K1 phase stamps.
set -euo pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_golden.py tests/test_gpu_dropin.py tests/test_gpu_reference_trace.py -x -q --timeout 120 --timeout-method thread > $OUT/slide_tests.log 2>&1
timeout -k 10 200 python bench.py --no-matcher --no-cpu-baseline --steps 200 --warmup 20 > $OUT/slide_bench.json 2> $OUT/slide_bench.err
timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 100 --warmup 10 > $OUT/slide_bench_cfg4.json 2> $OUT/slide_bench_cfg4.err
timeout -k 10 300 python tools/host_call_latency.py > $OUT/slide_host_latency.json 2> $OUT/slide_host_latency.err
timeout -k 10 200 python tools/ba_call_breakdown.py cfg3 > $OUT/slide_breakdown.json 2> $OUT/slide_breakdown.err
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 $OUT/slide_seg_cfg3.txt > $OUT/slide_stamps_cfg3.txt 2>&1
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/ba_phase_stamps.py cfg4 > $OUT/slide_stamps_cfg4.txt 2>&1
echo done
