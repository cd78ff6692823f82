"""Runs the batched matcher (bench.py's secondary workload) a few times: profiling driver."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from visualodometry_amd import _lib  # noqa: E402

ctx = _lib.context(0)
print(bench.bench_matcher(ctx, calls=5, warmup=1)["value"])
