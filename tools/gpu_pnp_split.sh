#!/bin/bash
# PnP parity tests, then the PnP bench leg at several first-phase sizes h1 (tools/pnp_only.py).
set -euo pipefail
mkdir -p gpurun_out/pnp_split
[ -n "${NO_TESTS:-}" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pnp.py tests/test_gpu_reference_trace.py > gpurun_out/pnp_split/tests.log 2>&1
H_LIST="${H_LIST:--1 0 48 56 64}"
for h in $H_LIST; do
  timeout -k 10 120 python tools/pnp_only.py $h > gpurun_out/pnp_split/h$h.json 2>> gpurun_out/pnp_split/err.log
done
echo done
