"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Follows /opt/skills/guides/MI355X_MICROARCH.md §HBM: the counters are in KB
(x1024), and on gfx950 FETCH_SIZE tallies exactly half the bytes of a wide
coalesced read, so reads are doubled.  The two counters cannot share a pass
(TCC slots), hence two runs of the same command.

    python tools/pmc_traffic.py FETCH_DIR/run_counter_collection.csv \
        WRITE_DIR/run_counter_collection.csv --config cfg3 -o profiles/traffic_cfg3.json

The output is keyed (``_key``): the configuration and damping of the profiled bench.py run,
the source digests of the BA and matcher kernels (bench.source_digest) and the launches per
kernel.  bench.py attaches a figure only to a timed run with the same key.  Per-launch values
are medians over the dispatches (the parity guard's odd launches do not move them).
"""

import argparse
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

# first match wins: "fpack_kernel" before "pack_kernel"; the int8 sweep is attributed by
# its template argument (match_kernel<2> = the D = 128 SIFT workload of the bench line;
# the float line's match_kernel<4> only checks the flag and exits)
SHORT = [("ba_lin_wave_kernel", "ba_lin"), ("ba_lin_kernel", "ba_lin"), ("ba_reduce_kernel", "ba_reduce"), ("ba_band_kernel", "ba_solve"),
         ("ba_solve_kernel", "ba_solve"), ("ba_solve2_kernel", "ba_solve"),
         ("fpack_kernel", "match_fpack"), ("fsweep_kernel", "match_f32"), ("frerank_kernel", "match_rerank"),
         ("pack_kernel", "match_pack"), ("match_kernel<2>", "match_i8"), ("match_kernel", "match_i8_other_d"),
         ("merge_kernel", "match_merge"), ("no_train_kernel", "match_none"), ("compact_kernel", "match_compact")]


def short_name(kernel: str):
    for key, s in SHORT:
        if key in kernel.replace(" ", ""):
            return s
    return None


def per_launch(path: str, counter: str):
    acc = defaultdict(float)  # (short, dispatch) -> value (summed over counter instances)
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            s = short_name(row["Kernel_Name"])
            if s:
                acc[(s, row["Dispatch_Id"])] += float(row["Counter_Value"])
    out = defaultdict(list)
    for (s, _), v in acc.items():
        out[s].append(v)
    med = {}
    for s, v in out.items():
        v = sorted(v)
        med[s] = v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2])
    return med, {s: len(v) for s, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--config", default="cfg3", help="bench.py --config of the profiled runs")
    ap.add_argument("--lam", type=float, default=1.0, help="bench.py --lam of the profiled runs")
    ap.add_argument("--gpus", type=int, default=1)
    a = ap.parse_args()
    fetch, nf = per_launch(a.fetch_csv, "FETCH_SIZE")
    write, nw = per_launch(a.write_csv, "WRITE_SIZE")
    res = {"_method": "bytes/launch = (2*median FETCH_SIZE + median WRITE_SIZE) * 1024 over the dispatches, "
                      "gfx950 FETCH_SIZE half-count correction per MI355X_MICROARCH.md; separate --pmc passes",
           "_key": {"config": a.config, "lam": a.lam, "gpus": a.gpus,
                    "digest": {g: bench.source_digest(g) for g in bench.TRAFFIC_SOURCES},
                    "launches": {s: min(nf.get(s, 0), nw.get(s, 0)) for s in set(nf) | set(nw)}},
           "_raw_kb": {}}
    for s in sorted(set(fetch) | set(write)):
        fk, wk = fetch.get(s, 0.0), write.get(s, 0.0)
        res[s] = (2 * fk + wk) * 1024
        res["_raw_kb"][s] = {"FETCH_SIZE": fk, "WRITE_SIZE": wk, "launches": [nf.get(s, 0), nw.get(s, 0)]}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
