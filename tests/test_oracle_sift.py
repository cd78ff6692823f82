"""Pins the SIFT detection oracle (oracle/sift_ref.py; reference SIFT at
``src/modules/frontend.py:27-32,55``).  OpenCV is absent, so against it the oracle is
parity unpinned; these are its known answers."""

import math

import numpy as np
import pytest

from oracle import sift_ref as S
from visualodometry_amd.synthetic import sift_scene


@pytest.mark.parametrize("sigma", [0.8, 1.2489996, 1.2262735, 1.5450077, 1.9465878, 2.4525316, 3.0900907])
def test_gaussian_taps(sigma):
    k = S.gaussian_kernel(sigma)
    n = S.cv_round(sigma * 8 + 1) | 1
    assert k.size == n and k.dtype == np.float32
    np.testing.assert_array_equal(k, k[::-1])  # symmetric by construction
    x = np.arange(n) - (n - 1) / 2
    ref = np.exp(-x * x / (2 * sigma * sigma))
    np.testing.assert_allclose(k, ref / ref.sum(), rtol=2e-7, atol=1e-9)


def test_octave_sigmas_compose():
    sig = S.octave_sigmas(1.6, 3)
    total = [1.6]
    for s in sig[1:]:
        total.append(math.sqrt(total[-1] ** 2 + s ** 2))
    np.testing.assert_allclose(total, [1.6 * 2 ** (i / 3) for i in range(6)], rtol=1e-12)


def test_blur_constant_and_impulse():
    c = np.full((40, 50), 100.0, np.float32)
    np.testing.assert_allclose(S.blur(c, 1.6), c, rtol=1e-6)
    imp = np.zeros((41, 41), np.float32)
    imp[20, 20] = 1.0
    k = S.gaussian_kernel(1.6)
    r = k.size // 2
    out = S.blur(imp, 1.6)
    np.testing.assert_array_equal(out[20 - r:21 + r, 20 - r:21 + r], np.outer(k, k).astype(np.float32))
    assert out.sum() == pytest.approx(1.0, rel=1e-6)


def test_reflect101_border():
    np.testing.assert_array_equal(S.reflect101(np.arange(-3, 8), 5), [3, 2, 1, 0, 1, 2, 3, 4, 3, 2, 1])


def test_upsample_is_exact_linear_interpolation():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (7, 9)).astype(np.float32)
    up = S.upsample2(img).astype(np.float64)
    src = img.astype(np.float64)
    def axis(n):
        d = np.arange(2 * n)
        f = (d + 0.5) / 2 - 0.5
        s = np.floor(f)
        w1 = f - s
        s = s.astype(int)
        w1[(s < 0) | (s + 1 >= n)] = 0
        s0 = np.clip(s, 0, n - 1)
        s0[s + 1 >= n] = n - 1
        return s0, np.clip(s + 1, 0, n - 1), 1 - w1, w1
    x0, x1, a0, a1 = axis(9)
    y0, y1, b0, b1 = axis(7)
    rows = src[:, x0] * a0 + src[:, x1] * a1
    ref = rows[y0] * b0[:, None] + rows[y1] * b1[:, None]
    np.testing.assert_array_equal(up, ref)  # multiples of 1/16: exact in float32
    assert up[0, 0] == src[0, 0] and up[-1, -1] == src[-1, -1]


def test_single_blob_is_found_at_its_centre_and_scale():
    h, w = 96, 128
    yy, xx = np.mgrid[0:h, 0:w]
    for s_blob, cy, cx in ((3.0, 47.3, 60.6), (5.0, 50.0, 70.0)):
        im = 100 + 120 * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s_blob ** 2))
        kp = S.detect(np.rint(im).astype(np.uint8), contrast=0.04, edge=10.0)
        d = np.hypot(kp["pt"][:, 0] - cx, kp["pt"][:, 1] - cy)
        j = int(np.argmin(d))
        assert d[j] < 0.5
        # DoG extrema of a blob sit at sigma ~ s_blob * sqrt(2)/..: size = 2 sigma_kp in image px
        assert 1.0 * s_blob < kp["size"][j] < 4.0 * s_blob
        assert kp["response"][j] > 0.04 / 3


def test_scene_detection_is_ordered_and_consistent():
    img = sift_scene(120, 200, seed=3, n_blobs=60, n_boxes=10)
    kp = S.detect(img, contrast=0.02, edge=2.0)  # the KITTI SIFT config (config.py)
    assert len(kp["pt"]) > 10
    idx = kp["index"]
    assert np.all(np.diff(idx[:, 0]) >= 0)  # octave order
    o = (kp["octave"] & 255).astype(np.int8)  # OpenCV's octave word: first octave -1
    np.testing.assert_array_equal(o + 1, idx[:, 0])
    assert np.all((kp["octave"] >> 8 & 255) == idx[:, 1])
    assert np.all(np.abs(kp["xi"]) < 0.5)


# ---- orientation / descriptors / keypoint filtering (oracle known answers) ---------------

def test_exp32f_and_fast_atan2_accuracy():
    x = np.linspace(-40, 0, 20001).astype(np.float32)
    ref = np.exp(x.astype(np.float64))
    assert np.max(np.abs(S.exp32f(x) - ref) / ref) < 2e-6
    rng = np.random.default_rng(0)
    y, xx = rng.normal(size=(2, 5000)).astype(np.float32)
    a = S.fast_atan2(y, xx)
    ref = np.degrees(np.arctan2(y, xx)) % 360
    err = np.abs(a - ref)
    assert np.max(np.minimum(err, 360 - err)) < 0.01  # OpenCV documents ~0.3 deg; this is tighter
    assert np.all((a >= 0) & (a <= 360))


def test_orientation_of_ramps():
    x = np.arange(64, dtype=np.float32)
    ramp = np.tile(2 * x, (64, 1)).astype(np.float32)
    h, m = S.orientation_hist(ramp, 32, 32, 8, 3.0)
    assert S.orientation_peaks(h, m) == [0.0]  # 360 - 0 snaps to 0
    h, m = S.orientation_hist(np.ascontiguousarray(ramp.T), 32, 32, 8, 3.0)
    assert S.orientation_peaks(h, m) == [90.0]  # dy = I(y-1) - I(y+1) < 0: gradient at 270
    h, m = S.orientation_hist(np.full((32, 32), 5, np.float32), 16, 16, 6, 2.0)
    assert m == 0 and S.orientation_peaks(h, m) == []


def test_descriptor_known_answers():
    x = np.arange(64, dtype=np.float32)
    ramp = np.tile(2 * x, (64, 1)).astype(np.float32)
    d = S.descriptor(ramp, 32.0, 32.0, 0.0, 2.0).reshape(16, 8)
    assert d[:, 1:].sum() == 0 and np.all(d[:, 0] > 0)        # every vote in orientation bin 0
    assert np.array_equal(d[:, 0].reshape(4, 4), d[:, 0].reshape(4, 4).T)  # symmetric window
    assert S.descriptor(np.full((64, 64), 7, np.float32), 32.0, 32.0, 10.0, 2.0).sum() == 0
    # rotating the window by 90 degrees on the transposed ramp gives the same descriptor
    d90 = S.descriptor(np.ascontiguousarray(ramp.T), 32.0, 32.0, 270.0, 2.0).reshape(16, 8)
    assert d90[:, 1:].sum() == 0 and np.abs(d90[:, 0] - d[:, 0]).max() <= 1


def test_detect_and_compute_filtering():
    img = sift_scene(188, 620, seed=3, n_blobs=150)
    full = S.detect_and_compute(img, 0, 0.02, 2.0, 1.6, with_descriptors=False)
    n = len(full["pt"])
    assert n > 100
    keys = list(zip(full["pt"][:, 0], full["pt"][:, 1], -full["size"], full["angle"]))
    assert keys == sorted(keys) and len(set(keys)) == n  # sorted, no duplicates
    cut = S.detect_and_compute(img, n // 3, 0.02, 2.0, 1.6, with_descriptors=False)
    thr = np.sort(full["response"])[::-1][n // 3 - 1]
    assert len(cut["pt"]) >= n // 3
    assert np.all(cut["response"] >= thr)
    assert np.sum(full["response"] >= thr) == len(cut["pt"])  # every tie at the boundary kept
    big = S.detect_and_compute(img, 10 * n, 0.02, 2.0, 1.6, with_descriptors=False)
    assert len(big["pt"]) == n
    # orientation duplicates share the extremum: same pt/size, different angles
    pts = {(a, b) for a, b in full["pt"]}
    assert len(pts) < n
