"""Per-kernel summary of one rocprofv3 --pmc pass: launches and the mean counter value per
launch (KB, raw, before the gfx950 FETCH_SIZE correction applied by tools/pmc_traffic.py).

    python tools/pmc_summary.py gpurun_out/r01_fetch/run_counter_collection.csv \
        -o profiles/r01_pmc_fetch_size.csv
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("counter_csv")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    acc = defaultdict(float)  # (kernel, counter, dispatch) -> value summed over instances
    with open(a.counter_csv, newline="") as f:
        for row in csv.DictReader(f):
            acc[(row["Kernel_Name"], row["Counter_Name"], row["Dispatch_Id"])] += float(row["Counter_Value"])
    per = defaultdict(list)
    for (k, c, _), v in acc.items():
        per[(k, c)].append(v)
    with open(a.out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_MINIMAL)
        w.writerow(["kernel", "counter", "launches", "mean_value_kb"])
        for (k, c), vs in sorted(per.items()):
            w.writerow([k, c, len(vs), f"{sum(vs) / len(vs):.3f}"])


if __name__ == "__main__":
    main()
