"""PnP-RANSAC throughput against the frames per call (bench.bench_pnp), for choosing the
bench batch: pnp_hyp runs one thread per (frame, hypothesis), so small batches leave
SIMDs idle."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from visualodometry_amd import _lib  # noqa: E402

ctx = _lib.context(0)
for b in (256, 1024, 2048, 4096):
    r = bench.bench_pnp(ctx, batch=b, calls=10)
    print(json.dumps({"batch": b, "frames_per_s": r["value"], "kernel_us": r["kernel_us"],
                      "frac": r["roofline"]["frac"]}), flush=True)
