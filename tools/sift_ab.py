"""A/B timing of one SIFT library build (VO_LIB_PATH selects it): the single-image host call
(vo_sift_detect_and_compute, median ms) and the 8-image device batch (bench.bench_sift,
images/s and per-phase kernel us); one JSON line."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from tools import sift_dropin_breakdown as B  # noqa: E402  (times the single call at import)

r = bench.bench_sift(B.ctx, check=False)
print(json.dumps({"lib": str(B._lib.LIB_PATH), "single_c_call_ms": B.out["c_call_ms"], "batch_images_s": r["value"],
                  "batch_kernel_us": r["kernel_us"]}))
