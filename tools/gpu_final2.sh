#!/bin/bash
# Round-4 second session: the evidence chain of tools/gpu_round.sh for this build (tests, smoke,
# rocprofv3 stats, PMC traffic of cfg3 and cfg4, final bench lines, host latency; the MFMA-busy
# passes of the unchanged matchers are not repeated), then the K1 waves-per-workgroup lines.
set -euo pipefail
TAG=${1:-r04e}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo tests-ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/${TAG}_trace -o run --output-format csv \
  -- python3 $ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/bench_trace.err
for CFG in cfg3 cfg4; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $ROOT/$OUT/${TAG}_fetch_$CFG -o run --output-format csv \
    -- python3 $ROOT/bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_fetch_$CFG.json 2> $OUT/bench_fetch_$CFG.err
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $ROOT/$OUT/${TAG}_write_$CFG -o run --output-format csv \
    -- python3 $ROOT/bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_write_$CFG.json 2> $OUT/bench_write_$CFG.err
  python tools/pmc_traffic.py $OUT/${TAG}_fetch_$CFG/run_counter_collection.csv \
    $OUT/${TAG}_write_$CFG/run_counter_collection.csv --config $CFG -o $OUT/traffic_$CFG.json > /dev/null
done
echo pmc-ok
timeout -k 10 400 python bench.py --traffic-json $OUT/traffic_cfg3.json > $OUT/bench_final.json 2> $OUT/bench_final.err
timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 \
  --traffic-json $OUT/traffic_cfg4.json > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
timeout -k 10 200 python tools/host_call_latency.py > $OUT/host_latency.json 2> $OUT/host_latency.err
timeout -k 10 200 python tools/ba_call_breakdown.py cfg3 > $OUT/call_breakdown.json 2> $OUT/call_breakdown.err
echo evidence-ok
VO_LIB_PATH=visualodometry_amd/lib/libvo_hip_stamps.so timeout -k 10 120 python tools/ba_phase_stamps.py cfg3 > $OUT/k1_stamps_cfg3.txt 2>&1
VO_BA_K1_WAVES=2 timeout -k 10 200 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 120 --timeout-method thread -k "oracle or determin" > $OUT/k1nw_tests2.log 2>&1
for nw in 2 3 6 1; do
  VO_BA_K1_WAVES=$nw timeout -k 10 150 python bench.py --no-matcher --no-cpu-baseline --steps 300 --warmup 30 > $OUT/k1nw_bench_$nw.json 2> $OUT/k1nw_bench_$nw.err
done
VO_BA_WAVE=1 timeout -k 10 150 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 30 --warmup 3 > $OUT/k1nw_cfg4_wave1.json 2> $OUT/k1nw_cfg4_wave1.err
echo done
