#!/bin/bash
# Summary of tools/gpu_k3_quick.sh output.
tail -1 gpurun_out/ba_tests.log
python - <<'PY'
import json
for c in ("cfg3", "cfg4"):
    d = json.loads(open(f"gpurun_out/bench_{c}.json").read().strip().splitlines()[-1])
    print(c, round(d["value"]), {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
tail -6 gpurun_out/st1.txt
grep -E "c: |ld: " gpurun_out/st2.txt | awk '{printf "%s %s %s ", $1, $2, $3; print int($4/28), int($5/28)}'
