"""The float-path matcher bench line alone (bench.bench_matcher_float), for quick GPU
iterations on the fp32 sweep."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from visualodometry_amd import _lib  # noqa: E402

ctx = _lib.context(0)
r = bench.bench_matcher_float(ctx)
print(json.dumps(r))
