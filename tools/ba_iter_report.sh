#!/bin/bash
# Summary of tools/gpu_ba_iter.sh output.
tail -1 gpurun_out/ba_tests.log
python - <<'PY'
import json
for c in ("cfg3", "cfg4"):
    d = json.loads(open(f"gpurun_out/bench_{c}.json").read().strip().splitlines()[-1])
    print(c, round(d["value"]), {k: v["avg_us"] for k, v in d["kernels"].items()})
PY
grep -E "^(load|backsub|lin_obs|reduce|eliminate|schur|write)|duration" gpurun_out/k1st.txt
tail -6 gpurun_out/st1.txt
