"""Summarises tools/gpu_host_variants.sh: per variant and mode, the call total and setup medians."""
import collections
import glob
import json
import statistics
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/*_*.json"):
    name = f.split("/")[-1].rsplit("_", 1)[0]
    d = json.load(open(f))
    for mode in ("scratch", "repeat", "slide"):
        rows[name][mode].append((d[mode]["total"], d[mode]["setup"]))
for name, modes in sorted(rows.items()):
    print(name, {m: (round(statistics.median(t for t, _ in v), 3), round(statistics.median(s for _, s in v), 3))
                 for m, v in modes.items()})
