set -euo pipefail
OUT=gpurun_out/q13
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/visualodometry_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_sift.py tests/test_gpu_golden.py tests/test_gpu_torch_coexist.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 180 python tools/frame_latency.py > $OUT/frame_latency.json 2> $OUT/frame_latency.err
for rep in 1 2; do
  for n in c1 prod; do
    LIB=$L/libvo_hip_$n.so; [ $n = prod ] && LIB=$L/libvo_hip.so
    VO_LIB_PATH=$LIB timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_${n}_$rep.json 2> $OUT/bench_${n}_$rep.err
  done
done
echo done
