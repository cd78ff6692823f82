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
    """detectAndCompute's bulk KeyPoint builder (sift._keypoints, csrc/kp_objects.c) gives the
    record's float32 fields as Python floats and its octave as an int, with cv2.KeyPoint's
    attribute surface (pt a fresh tuple per read, writable fields, class_id -1)."""
    from visualodometry_amd.sift import KP_DTYPE, KeyPoint, _keypoints
    rng = np.random.default_rng(5)
    kp = np.zeros(257, KP_DTYPE)
    for f in ("x", "y", "size", "angle", "response"):
        kp[f] = rng.random(kp.size, dtype=np.float32) * 1000
    kp["octave"] = rng.integers(-(1 << 20), 1 << 20, kp.size)
    got = _keypoints(kp)
    assert isinstance(got, tuple) and len(got) == kp.size
    for k, rec in zip(got, kp):
        assert type(k) is KeyPoint
        assert k.pt == (float(rec["x"]), float(rec["y"]))
        assert type(k.pt[0]) is float and type(k.pt[1]) is float
        for f in ("size", "angle", "response"):
            assert type(getattr(k, f)) is float and getattr(k, f) == float(rec[f]), f
        assert type(k.octave) is int and k.octave == int(rec["octave"])
        assert k.class_id == -1
        ref = KeyPoint(rec["x"], rec["y"], rec["size"], rec["angle"], rec["response"], rec["octave"])
        assert (ref.pt, ref.size, ref.angle, ref.response, ref.octave, ref.class_id) == \
            (k.pt, k.size, k.angle, k.response, k.octave, k.class_id)
    assert _keypoints(kp[:0]) == ()
    # the non-contiguous slice of a wider buffer is packed first
    assert [k.octave for k in _keypoints(kp[::2])] == kp["octave"][::2].tolist()


def test_keypoint_object_surface():
    """cv2.KeyPoint's constructor defaults and writable attributes."""
    from visualodometry_amd.sift import KeyPoint, _keypoints
    k = KeyPoint(1.5, 2.5, 3.0)
    assert (k.pt, k.size, k.angle, k.response, k.octave, k.class_id) == ((1.5, 2.5), 3.0, -1.0, 0.0, 0, -1)
    k.pt = (4, 5)
    k.angle = 90.25
    k.octave = 7
    assert (k.pt, k.angle, k.octave) == ((4.0, 5.0), 90.25, 7)
    assert KeyPoint(x=1, y=2, size=3, octave=5, class_id=2).class_id == 2
    with pytest.raises(TypeError):
        k.pt = (1.0,)
    with pytest.raises(ValueError):
        _keypoints(np.zeros(10, np.uint8))
    assert "KeyPoint(pt=(4, 5)" in repr(k)
