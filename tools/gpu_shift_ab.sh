set -euo pipefail
OUT=gpurun_out/q14
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/visualodometry_amd/lib
for n in shift1 shift2; do
  VO_LIB_PATH=$L/libvo_hip_$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 200 --timeout-method thread -k "cfg4 or split or layout" > $OUT/tests_$n.log 2>&1
done
for rep in 1 2 3; do
  for n in prod shift1 shift2; do
    LIB=$L/libvo_hip_$n.so; [ $n = prod ] && LIB=$L/libvo_hip.so
    VO_LIB_PATH=$LIB timeout -k 10 200 python bench.py --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 \
      > $OUT/cfg4_${n}_$rep.json 2> $OUT/cfg4_${n}_$rep.err
  done
done
echo done
