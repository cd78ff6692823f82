#!/bin/bash
# The one-wave K1 with 1, 2, 3 chunks per segment (testing switch through bench.py --k1):
# BA GPU tests, then cfg3 and cfg4 bench lines per variant, alternating.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_k1_group.sh [tag]
set -euo pipefail
TAG=${1:-k1g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_sharded_loopback.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_ba.log 2>&1
for rep in 1 2; do
  for v in 1 2 3; do
    timeout -k 10 120 python bench.py --k1 $v --no-matcher --no-cpu-baseline > $OUT/cfg3_v${v}_$rep.json 2> $OUT/cfg3_v${v}_$rep.err
    timeout -k 10 200 python bench.py --k1 $v --config cfg4 --no-matcher --no-cpu-baseline --steps 50 --warmup 5 > $OUT/cfg4_v${v}_$rep.json 2> $OUT/cfg4_v${v}_$rep.err
  done
done
echo done
