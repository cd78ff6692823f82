#!/bin/bash
# BA kernel build variants (visualodometry_amd/lib/var_<name>): BA bench line each (no parity).
set -euo pipefail
mkdir -p gpurun_out
for v in "$@"; do
  VO_LIB_PATH=$PWD/visualodometry_amd/lib/var_$v/libvo_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-matcher --steps 100 > gpurun_out/bv_$v.json 2> gpurun_out/bv_$v.err || echo "variant $v failed"
done
echo ok
