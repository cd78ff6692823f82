#!/bin/bash
tail -1 gpurun_out/k3_pytest.log
python -c "
import json; d=json.loads(open('gpurun_out/k3_bench.json').read().strip().splitlines()[-1]); print(round(d['value']), {k:v['avg_us'] for k,v in d['kernels'].items()})"
for w in 0 1 2 3; do echo "wave $w: $(grep k3_ gpurun_out/k3w_$w.txt | awk '{printf "%s=%s ", $1, $2}')"; done
