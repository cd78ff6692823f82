"""Summarises a tools/gpu_host_ab.sh run: per-call totals and the setup's median sections."""
import collections
import glob
import json
import re
import statistics
import sys

d0 = sys.argv[1]
for f in sorted(glob.glob(f"{d0}/spin_*.json")) + [f"{d0}/host_latency.json"]:
    d = json.load(open(f))
    if "scratch" in d:
        print(f.split("/")[-1], "scratch", d["scratch"]["total"], d["scratch"]["setup"], "slide", d["slide"]["total"],
              d["slide"]["setup"], "slide windows from scratch", d.get("slide_windows_scratch", {}).get("total"),
              d.get("slide_windows_scratch", {}).get("setup"))
    else:
        print(f.split("/")[-1], d["ba_cfg3_10iters_ms"], d["ba_cfg3_slide_ms"])
secs = collections.defaultdict(lambda: collections.defaultdict(list))
mode = None
for line in open(f"{d0}/sections.err"):
    line = line.rstrip()
    if line.startswith("-- "):
        mode = line[3:]
        continue
    m = re.match(r"\s+(.+?)\s+([\d.]+) ms", line)
    if m and mode:
        secs[mode][m.group(1)].append(float(m.group(2)))
for mode, d in secs.items():
    print(mode, {k: round(statistics.median(v[2:]), 3) for k, v in d.items()})
