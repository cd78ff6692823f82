set -euo pipefail
OUT=gpurun_out/${1:-q17}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sift.py tests/test_gpu_golden.py tests/test_gpu_torch_coexist.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
timeout -k 10 200 python tools/sift_dropin_breakdown.py > $OUT/breakdown.json 2> $OUT/breakdown.err
cat $OUT/breakdown.json
timeout -k 10 300 python tools/host_call_latency.py > $OUT/host_latency.json 2> $OUT/host_latency.err
cat $OUT/host_latency.json

cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o sift -- python3 $GRAFT_REPO_ROOT/tools/sift_single.py > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
echo prof done
