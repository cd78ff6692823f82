"""The PnP bench line alone (bench.bench_pnp) with per-kernel HIP-event averages, for A/B runs of
library builds (VO_LIB_PATH)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from visualodometry_amd import _lib  # noqa: E402

ctx = _lib.context(0)
if len(sys.argv) > 1:  # h1 for vo_pnp_testing_split (0 auto, -1 all hypotheses at once)
    _lib.pnp_testing_split(ctx, int(sys.argv[1]))
r = bench.bench_pnp(ctx)
r.pop("cpu_baseline", None)
print(json.dumps({"value": r["value"], "kernel_us": r["kernel_us"], "split": r.get("split"),
                  "roofline_frac": r["roofline"]["frac"], "single_frame_ms": r.get("single_frame_ms")}))
