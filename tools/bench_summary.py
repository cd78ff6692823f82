"""One line per bench JSON: value, kernel averages (HIP events), slab rows, parity guard."""
import glob
import json
import sys

for f in sorted(sum((glob.glob(a) for a in sys.argv[1:]), [])):
    try:
        d = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    print(f.split("/")[-1], round(d["value"], 1), {k: v["avg_us"] for k, v in d["kernels"].items()},
          d["config"]["plan"]["slab_blocks"], d["parity_guard"]["ok"])
