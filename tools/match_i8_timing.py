"""The int8 matcher bench line (bench.bench_matcher, with its oracle guard) for same-box A/B of
tuning builds (VO_LIB_PATH): prints the rate and the kernels' HIP-event microseconds."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from visualodometry_amd import _lib  # noqa: E402

r = bench.bench_matcher(_lib.context(0), calls=10, warmup=2)
print(json.dumps({"value": r["value"], "kernel_us": r["kernel_us"]}))
