"""MFMA-busy summary of the matcher sweeps from one rocprofv3 --pmc pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE ...
    python tools/mfma_busy.py PMC_DIR/run_counter_collection.csv [more.csv] -o profiles/r04_mfma_busy.json

Per kernel (median over dispatches, counter instances summed per dispatch):
  kernel_cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs' GPU-busy cycles; MI355X_MICROARCH.md
                  "DVFS give-back"), i.e. the dispatch's length in shader cycles;
  mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs x kernel_cycles): the fraction of all
                  SIMD-cycles of the dispatch in which a matrix core was busy;
  mfma_per_valu  = SQ_INSTS_MFMA / SQ_INSTS_VALU.
"""
import argparse
import csv
import json
from collections import defaultdict

N_SIMD = 256 * 4
KEEP = ("match_kernel", "fsweep_kernel", "frerank_kernel", "pack_kernel", "fpack_kernel", "merge_kernel")


def short(name: str) -> str:
    n = name.replace(" ", "")
    for key, s in (("match_kernel<2>", "match_i8 (match_kernel<2>)"), ("fsweep_kernel<1", "fsweep<1>"),
                   ("fsweep_kernel<2", "fsweep<2>"), ("frerank_kernel", "frerank"), ("fpack_kernel", "fpack"),
                   ("pack_kernel", "pack"), ("merge_kernel", "merge")):
        if key in n:
            return s
    return n.split("(")[0]


def median(v):
    v = sorted(v)
    return v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    acc = defaultdict(float)  # (kernel, counter, file, dispatch) -> value
    for path in a.csv:
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if not any(k in row["Kernel_Name"] for k in KEEP):
                    continue
                acc[(short(row["Kernel_Name"]), row["Counter_Name"], path, row["Dispatch_Id"])] += \
                    float(row["Counter_Value"])
    per = defaultdict(lambda: defaultdict(list))
    for (k, c, _, _), v in acc.items():
        per[k][c].append(v)
    out = {"_method": __doc__.strip().splitlines()[0] + " -- see tools/mfma_busy.py", "kernels": {}}
    for k, cs in sorted(per.items()):
        m = {c: median(v) for c, v in cs.items()}
        r = {c: m[c] for c in sorted(m)}
        r["dispatches"] = max(len(v) for v in cs.values())
        cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if cyc > 0:
            r["kernel_cycles"] = cyc
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                r["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * cyc)
        if m.get("SQ_INSTS_VALU"):
            r["mfma_per_valu"] = m.get("SQ_INSTS_MFMA", 0.0) / m["SQ_INSTS_VALU"]
        out["kernels"][k] = r
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
