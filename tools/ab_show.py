"""Prints value and per-kernel averages of every bench line in a directory (A/B runs)."""
import json
import sys
from pathlib import Path

for f in sorted(Path(sys.argv[1]).glob("*.json")):
    try:
        d = json.loads(f.read_text().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f.name, "unreadable", e)
        continue
    if "value" not in d:
        print(f.name, json.dumps(d)[:300])
        continue
    k = {n: v["avg_us"] for n, v in d.get("kernels", {}).items()}
    reg = d.get("timed_regions", {}).get("value")
    print(f"{f.name:28s} {d['value']:10.1f}  {k}  {[round(x) for x in reg] if reg else ''}")
