"""Summarises tools/gpu_ab_bench.sh: per variant and config, GN-iters/s and the kernels' HIP-event
microseconds (median over rounds)."""
import collections
import glob
import json
import statistics
import sys

rows = collections.defaultdict(list)
for f in sorted(glob.glob(f"{sys.argv[1]}/cfg*_*.json")):
    cfg, name = f.split("/")[-1].rsplit("_", 1)[0].split("_", 1)
    d = json.load(open(f))
    rows[(cfg, name)].append((d["value"], {k: v["avg_us"] for k, v in d.get("kernels", {}).items()}))
for (cfg, name), v in sorted(rows.items()):
    ks = {k: round(statistics.median(x[1][k] for x in v), 2) for k in v[0][1]}
    print(cfg, name, round(statistics.median(x[0] for x in v), 1), ks)
