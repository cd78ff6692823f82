"""The SIFT orientation kernel's math (csrc/sift_math.h: exp32f, fastAtan2, the correctly
rounded sqrt; sift_orient_kernel's sample loop and per-bin order), compiled for the host
by ``sift_host_check`` and run on CPU, against ``oracle.sift_ref.orientation_hist``:
bitwise equal histograms for every extremum of a scene."""

import subprocess
from pathlib import Path

import numpy as np
import pytest

from oracle import sift_ref as S
from visualodometry_amd.synthetic import sift_scene

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "visualodometry_amd" / "lib" / "sift_host_check"


@pytest.fixture(scope="module")
def exe():
    if not EXE.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "visualodometry_amd" / "csrc"), "../lib/sift_host_check"],
                       check=True)
    return EXE


def test_orientation_hist_host_build_matches_oracle(exe, tmp_path):
    img = sift_scene(188, 620, seed=11, n_blobs=150)
    pyr = S.gaussian_pyramid(img)
    det = S.detect(img, 0.02, 2.0, 1.6)
    groups = {}
    for i in range(len(det["pt"])):
        o, layer, r, c = (int(v) for v in det["index"][i])
        scl = np.float32(np.float32(np.float32(det["size"][i] * np.float32(2)) * np.float32(0.5)) / np.float32(1 << o))
        groups.setdefault((o, layer), []).append((r, c, scl))
    checked = 0
    for (o, layer), items in groups.items():
        G = pyr[o][layer]
        fi, fo = tmp_path / "in", tmp_path / "out"
        with open(fi, "wb") as f:
            np.array(G.shape, np.int32).tofile(f)
            G.astype(np.float32).tofile(f)
            np.array([len(items)], np.int32).tofile(f)
            for r, c, s in items:
                np.array([r, c], np.int32).tofile(f)
                np.array([s], np.float32).tofile(f)
        subprocess.run([str(exe), str(fi), str(fo)], check=True)
        H = np.fromfile(fo, np.float32).reshape(-1, 36)
        for q, (r, c, s) in enumerate(items):
            h, _ = S.orientation_hist(G, c, r, S.cv_round(float(S.SIFT_ORI_RADIUS * s)),
                                      np.float32(S.SIFT_ORI_SIG_FCTR * s))
            np.testing.assert_array_equal(H[q], h)
            checked += 1
    assert checked > 100


def test_keypoint_objects_carry_the_record_fields():
    """detectAndCompute's bulk KeyPoint builder (sift._keypoints) gives the same Python values
    and types as the per-keypoint cv2-style constructor, for every field the reference reads."""
    from visualodometry_amd.sift import KP_DTYPE, KeyPoint, _keypoints, _kp_dict
    rng = np.random.default_rng(5)
    kp = np.zeros(257, KP_DTYPE)
    for f in ("x", "y", "size", "angle", "response"):
        kp[f] = rng.random(kp.size, dtype=np.float32) * 1000
    kp["octave"] = rng.integers(-(1 << 20), 1 << 20, kp.size)
    r = _kp_dict(kp, np.zeros((kp.size, 128), np.float32))
    got = _keypoints(r)
    assert isinstance(got, tuple) and len(got) == kp.size
    for k, rec in zip(got, kp):
        ref = KeyPoint(rec["x"], rec["y"], rec["size"], rec["angle"], rec["response"], rec["octave"])
        for f in ("pt", "size", "angle", "response", "octave", "class_id"):
            assert getattr(k, f) == getattr(ref, f) and type(getattr(k, f)) is type(getattr(ref, f)), f
        assert type(k.pt[0]) is float and type(k.pt[1]) is float
    assert _keypoints(_kp_dict(kp[:0], np.zeros((0, 128), np.float32))) == ()
