"""The SIFT bench line alone (bench.bench_sift) with per-kernel HIP-event averages; for
quick GPU iterations on the SIFT kernels.  --no-check skips the parity guard (timing-only
diagnostic builds)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from visualodometry_amd import _lib  # noqa: E402

ctx = _lib.context(0)
r = bench.bench_sift(ctx, check="--no-check" not in sys.argv)
r.pop("cpu_baseline", None)
print(json.dumps(r))
