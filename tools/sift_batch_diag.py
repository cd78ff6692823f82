"""Diagnostic: device-batch SIFT against the oracle per image with a flat image in the batch
(VO_LIB_PATH picks the build): refined extrema counts per image and per octave, and the
full detectAndCompute counts."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import sift_ref as S  # noqa: E402
from visualodometry_amd import _lib, sift  # noqa: E402
from visualodometry_amd.synthetic import sift_scene  # noqa: E402

ctx = _lib.context(0)
a, c = sift_scene(188, 620, seed=21, n_blobs=100), sift_scene(188, 620, seed=22, n_blobs=100)
for name, imgs in (("a_flat90_c", [a, np.full((188, 620), 90, np.uint8), c]),
                   ("a_flat0_c", [a, np.zeros((188, 620), np.uint8), c]),
                   ("a_c_flat90", [a, c, np.full((188, 620), 90, np.uint8)]),
                   ("a_c", [a, c])):
    imgs = np.stack(imgs)
    cap = 1 << 15
    dI = _lib.DeviceArray.from_numpy(ctx, imgs)
    dF = _lib.DeviceArray(ctx, (cap, 8), np.float32)
    dK = _lib.DeviceArray(ctx, (cap, 8), np.int32)
    dC = _lib.DeviceArray(ctx, (1,), np.int32)
    sift.detect_device(dI, 0.02, 2.0, 1.6, 3, dF, dK, dC, ctx=ctx)
    n = int(dC.numpy()[0])
    K = dK.numpy()[:n]
    for b in range(len(imgs)):
        ref = S.detect(imgs[b], 0.02, 2.0, 1.6)
        sel = K[:, 0] == b
        oct_got = np.bincount(K[sel, 1] & 255, minlength=10)[:10].tolist()
        oct_ref = np.bincount((np.asarray(ref["octave"]) & 255 + 1) & 255, minlength=10)[:10].tolist() if len(ref["pt"]) else []
        print(name, "img", b, "refined", int(sel.sum()), "oracle", len(ref["pt"]), "by octave got", oct_got, flush=True)
