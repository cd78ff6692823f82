"""Distribution of descriptor window sizes (OpenCV calcSIFTDescriptor radius and square
window length) over the keypoints the SIFT bench keeps on its first image."""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib, sift  # noqa: E402
from visualodometry_amd.synthetic import sift_scene  # noqa: E402

ctx = _lib.context(0)
img = sift_scene(376, 1241, seed=200, texture=12.0)
kps, _ = sift.SIFT_create(nfeatures=4000, contrastThreshold=0.02, edgeThreshold=2.0, sigma=1.6,
                          ctx=ctx).detectAndCompute(img, None)
octv = np.array([((k.octave & 255) ^ 128) - 128 for k in kps])
size = np.array([k.size for k in kps], np.float64)
o = octv + 1                                  # octave index of the upsampled pyramid
scl = size * 2.0 / (2.0 ** o) * 0.5
radius = np.rint(3.0 * scl * np.sqrt(2.0) * 5 * 0.5)
length = (2 * radius + 1) ** 2
print(json.dumps({"n": len(kps), "octaves": np.bincount(o).tolist(),
                  "radius_pct": np.percentile(radius, [10, 50, 90, 99]).tolist(),
                  "len_mean": float(length.mean()), "len_sum": float(length.sum())}))
