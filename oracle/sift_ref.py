"""CPU oracle for SIFT keypoint detection -- TEST INFRASTRUCTURE ONLY.

Imported by ``tests/`` and the ``cpu_baseline`` leg of ``bench.py``; never by the product
path.

Restates the detection half of ``cv2.SIFT_create(nfeatures, contrastThreshold,
edgeThreshold, sigma).detectAndCompute(gray, None)`` as the reference calls it
(``src/modules/frontend.py:27-32,55``; OpenCV 4.12 ``features2d/src/sift.dispatch.cpp`` and
``sift.simd.hpp``; cv2 is absent here, so this follows its published source):

* ``createInitialImage`` with ``firstOctave = -1``: the uint8 image as float32 (scale 1),
  doubled by ``resize(INTER_LINEAR)`` (exact here: weights 3/4 and 1/4 on integers), then
  ``GaussianBlur`` with ``sig_diff = sqrtf(max(sigma^2 - 4 * 0.5^2, 0.01))``;
* ``buildGaussianPyramid``: ``nOctaves = cvRound(log2(min(w2, h2)) - 2) + 1`` octaves of
  ``nOctaveLayers + 3`` levels, level i blurred from level i-1 with
  ``sig[i] = sqrt(s_i^2 - s_{i-1}^2)``, ``s_i = sigma k^i``, ``k = 2^(1/nOctaveLayers)``; an
  octave starts from level ``nOctaveLayers`` of the previous one, every other pixel
  (``INTER_NEAREST`` at scale 1/2);
* ``buildDoGPyramid``: ``D_i = G_{i+1} - G_i`` in float32;
* ``findScaleSpaceExtrema`` up to (not including) the orientation histogram: pixels at
  least ``SIFT_IMG_BORDER = 5`` from the edge of DoG levels 1..nOctaveLayers with
  ``|v| > floor(0.5 contrastThreshold / nOctaveLayers * 255)`` that are >= (maxima) or <=
  (minima) all 26 neighbours; ``adjustLocalExtrema``: at most 5 Newton steps on the 3x3x3
  quadratic fit (float32 central differences, ``Matx33f::solve`` by Cramer's rule with the
  determinant in float), moves by ``cvRound`` of the offset, the contrast test
  ``|contr| * nOctaveLayers >= contrastThreshold`` and the edge test
  ``det > 0 and tr^2 edgeThreshold < (edgeThreshold + 1)^2 det``; the keypoint's position,
  size, octave word and response as OpenCV packs them (then scaled by 1/2 for the doubled
  first octave).

Build-defined (OpenCV's float GaussianBlur runs SIMD kernels whose summation order and
FMA use depend on the CPU it runs on, so no order is "the" reference):

* ``GaussianBlur`` = a row pass then a column pass, each ``s = sum_j k_j x_{i-r+j}`` summed
  left to right in float32 without FMA, BORDER_REFLECT_101; the taps are those of
  ``getGaussianKernel(cvRound(8 sigma + 1) | 1, sigma, CV_32F)`` (:func:`gaussian_kernel`);
* keypoints come out in (octave, level, row, column) order; OpenCV's order after its
  parallel gather, ``removeDuplicatedSorted`` and ``retainBest`` is implementation-defined.
* Orientation assignment (which may duplicate a keypoint per histogram peak), the
  ``nfeatures`` cut and the descriptors are not part of this row yet.

Parity pin: OpenCV cannot run here and the reference has no fixtures, so against OpenCV
this is **parity unpinned**.  It is pinned by known answers (``tests/test_oracle_sift.py``):
the Gaussian taps against the closed form, blur of a constant image (identity) and of an
impulse (the separable kernel), the doubling being exact, and a synthetic blob detected at
its centre with the scale of its sigma.
"""

from __future__ import annotations

import math

import numpy as np

SIFT_IMG_BORDER = 5
SIFT_MAX_INTERP_STEPS = 5
SIFT_INIT_SIGMA = 0.5
FIRST_OCTAVE = -1


def cv_round(x: float) -> int:
    """cvRound: round half to even (the SSE conversion OpenCV uses)."""
    return int(np.rint(x))


def gaussian_kernel(sigma: float) -> np.ndarray:
    """``getGaussianKernel(cvRound(sigma*4*2+1)|1, sigma, CV_32F)`` for float images, i.e.
    OpenCV 4's ``getGaussianKernelBitExact`` (imgproc/smooth.dispatch.cpp): the left half
    ``exp(x^2 * (-0.125 / sigma^2))`` at x = 1-n, 3-n, ... (doubled coordinates), the sum
    ``2 * sum(left) + 1``, taps ``left * (1 / sum)`` mirrored, the centre ``1 / sum``; cast to
    float32.  OpenCV evaluates it in softdouble; libm ``exp`` here (parity unpinned)."""
    n = cv_round(sigma * 4 * 2 + 1) | 1
    scale2x = -0.125 / (sigma * sigma)
    n2 = (n - 1) // 2
    vals = []
    total = 0.0
    x = 1 - n
    for _ in range(n2):
        t = math.exp(float(x * x) * scale2x)
        vals.append(t)
        total += t
        x += 2
    total *= 2.0
    total += 1.0
    if n % 2 == 0:
        total += 1.0
    mul1 = 1.0 / total
    k = np.empty(n)
    for i in range(n2):
        k[i] = k[n - 1 - i] = vals[i] * mul1
    k[n2:n - n2] = mul1
    return k.astype(np.float32)


def reflect101(idx: np.ndarray, n: int) -> np.ndarray:
    """BORDER_REFLECT_101 index map (gfedcb|abcdefgh|gfedcba)."""
    if n == 1:
        return np.zeros_like(idx)
    idx = np.abs(idx)
    period = 2 * n - 2
    idx = idx % period
    return np.where(idx >= n, period - idx, idx)


def blur(img: np.ndarray, sigma: float) -> np.ndarray:
    """Separable Gaussian in float32: row pass, then column pass, left-to-right sums."""
    k = gaussian_kernel(sigma)
    r = k.size // 2
    img = np.asarray(img, dtype=np.float32)
    h, w = img.shape
    cols = reflect101(np.arange(-r, w + r), w)
    tmp = np.zeros((h, w), np.float32)
    for j in range(k.size):
        tmp = tmp + k[j] * img[:, cols[j:j + w]]
    rows = reflect101(np.arange(-r, h + r), h)
    out = np.zeros((h, w), np.float32)
    for j in range(k.size):
        out = out + k[j] * tmp[rows[j:j + h], :]
    return out


def upsample2(img: np.ndarray) -> np.ndarray:
    """``resize(2x, INTER_LINEAR)`` of a float image: source coordinate (d + 0.5)/2 - 0.5,
    clamped at the borders.  Every product and sum is exact for integer pixel values."""
    img = np.asarray(img, dtype=np.float32)
    h, w = img.shape

    def axis_weights(n_src):
        d = np.arange(2 * n_src)
        f = (d + 0.5) * 0.5 - 0.5
        s = np.floor(f).astype(np.int64)
        f = (f - s).astype(np.float32)
        lo = s < 0
        hi = s + 1 >= n_src
        s0 = np.clip(s, 0, n_src - 1)
        s1 = np.clip(s + 1, 0, n_src - 1)
        f = np.where(lo | hi, np.float32(0), f)
        s0 = np.where(hi, n_src - 1, s0)
        return s0, s1, (np.float32(1) - f).astype(np.float32), f

    x0, x1, ax0, ax1 = axis_weights(w)
    y0, y1, ay0, ay1 = axis_weights(h)
    rows = img[:, x0] * ax0 + img[:, x1] * ax1
    return (rows[y0, :] * ay0[:, None] + rows[y1, :] * ay1[:, None]).astype(np.float32)


def octave_sigmas(sigma: float, n_layers: int) -> list[float]:
    sig = [sigma]
    k = 2.0 ** (1.0 / n_layers)
    for i in range(1, n_layers + 3):
        prev = k ** (i - 1) * sigma
        total = prev * k
        sig.append(math.sqrt(total * total - prev * prev))
    return sig


def n_octaves(h2: int, w2: int) -> int:
    return cv_round(math.log(min(h2, w2)) / math.log(2.0) - 2) - FIRST_OCTAVE


def gaussian_pyramid(gray: np.ndarray, sigma: float = 1.6, n_layers: int = 3):
    """-> list over octaves of (n_layers + 3) float32 levels."""
    base = upsample2(np.asarray(gray, dtype=np.uint8).astype(np.float32))
    sig_diff = float(np.sqrt(np.float32(max(np.float32(sigma) * np.float32(sigma) -
                                            np.float32(SIFT_INIT_SIGMA * SIFT_INIT_SIGMA * 4), np.float32(0.01)))))
    g0 = blur(base, sig_diff)
    sig = octave_sigmas(sigma, n_layers)
    pyr = []
    for o in range(n_octaves(*base.shape)):
        src = pyr[o - 1][n_layers] if o else None  # resize(src, (w/2, h/2), INTER_NEAREST)
        levels = [g0 if o == 0 else src[:(src.shape[0] // 2) * 2:2, :(src.shape[1] // 2) * 2:2].copy()]
        for i in range(1, n_layers + 3):
            levels.append(blur(levels[-1], sig[i]))
        pyr.append(levels)
    return pyr


def dog_pyramid(pyr):
    return [[(lv[i + 1] - lv[i]).astype(np.float32) for i in range(len(lv) - 1)] for lv in pyr]


def _solve3(H, b):
    """``Matx33f::solve(DECOMP_LU)`` for 3x3: Cramer's rule, float32, zeros if det == 0."""
    f = np.float32
    a = [[f(v) for v in row] for row in H]
    b = [f(v) for v in b]
    det = f(a[0][0] * (a[1][1] * a[2][2] - a[2][1] * a[1][2]) - a[0][1] * (a[1][0] * a[2][2] - a[2][0] * a[1][2]) +
            a[0][2] * (a[1][0] * a[2][1] - a[2][0] * a[1][1]))
    if det == 0:
        return [f(0), f(0), f(0)]
    d = f(1) / det
    x0 = d * (b[0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) - a[0][1] * (b[1] * a[2][2] - a[1][2] * b[2]) +
              a[0][2] * (b[1] * a[2][1] - a[1][1] * b[2]))
    x1 = d * (a[0][0] * (b[1] * a[2][2] - a[1][2] * b[2]) - b[0] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
              a[0][2] * (a[1][0] * b[2] - b[1] * a[2][0]))
    x2 = d * (a[0][0] * (a[1][1] * b[2] - b[1] * a[2][1]) - a[0][1] * (a[1][0] * b[2] - b[1] * a[2][0]) +
              b[0] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]))
    return [f(x0), f(x1), f(x2)]


def adjust_local_extremum(dog, o, layer, r, c, n_layers, contrast, edge, sigma):
    """``adjustLocalExtrema`` -> keypoint tuple or None (float32 arithmetic throughout)."""
    f = np.float32
    img_scale = f(1.0) / f(255)
    deriv_scale = img_scale * f(0.5)
    second = img_scale
    cross = img_scale * f(0.25)
    xi = xr = xc = f(0)
    i = 0
    while i < SIFT_MAX_INTERP_STEPS:
        img, prev, nxt = dog[o][layer], dog[o][layer - 1], dog[o][layer + 1]
        dD = [(img[r, c + 1] - img[r, c - 1]) * deriv_scale, (img[r + 1, c] - img[r - 1, c]) * deriv_scale,
              (nxt[r, c] - prev[r, c]) * deriv_scale]
        v2 = img[r, c] * f(2)
        dxx = (img[r, c + 1] + img[r, c - 1] - v2) * second
        dyy = (img[r + 1, c] + img[r - 1, c] - v2) * second
        dss = (nxt[r, c] + prev[r, c] - v2) * second
        dxy = (img[r + 1, c + 1] - img[r + 1, c - 1] - img[r - 1, c + 1] + img[r - 1, c - 1]) * cross
        dxs = (nxt[r, c + 1] - nxt[r, c - 1] - prev[r, c + 1] + prev[r, c - 1]) * cross
        dys = (nxt[r + 1, c] - nxt[r - 1, c] - prev[r + 1, c] + prev[r - 1, c]) * cross
        X = _solve3([[dxx, dxy, dxs], [dxy, dyy, dys], [dxs, dys, dss]], dD)
        xi, xr, xc = -X[2], -X[1], -X[0]
        if abs(xi) < 0.5 and abs(xr) < 0.5 and abs(xc) < 0.5:
            break
        lim = f(2147483647 // 3)  # (float)(INT_MAX / 3)
        if abs(xi) > lim or abs(xr) > lim or abs(xc) > lim:
            return None
        c += cv_round(float(xc))
        r += cv_round(float(xr))
        layer += cv_round(float(xi))
        if (layer < 1 or layer > n_layers or c < SIFT_IMG_BORDER or c >= img.shape[1] - SIFT_IMG_BORDER or
                r < SIFT_IMG_BORDER or r >= img.shape[0] - SIFT_IMG_BORDER):
            return None
        i += 1
    if i >= SIFT_MAX_INTERP_STEPS:
        return None
    img, prev, nxt = dog[o][layer], dog[o][layer - 1], dog[o][layer + 1]
    dD = [(img[r, c + 1] - img[r, c - 1]) * deriv_scale, (img[r + 1, c] - img[r - 1, c]) * deriv_scale,
          (nxt[r, c] - prev[r, c]) * deriv_scale]
    t = f(f(dD[0] * xc + dD[1] * xr) + dD[2] * xi)
    contr = f(img[r, c] * img_scale + t * f(0.5))
    if abs(contr) * f(n_layers) < f(contrast):
        return None
    v2 = img[r, c] * f(2)
    dxx = (img[r, c + 1] + img[r, c - 1] - v2) * second
    dyy = (img[r + 1, c] + img[r - 1, c] - v2) * second
    dxy = (img[r + 1, c + 1] - img[r + 1, c - 1] - img[r - 1, c + 1] + img[r - 1, c - 1]) * cross
    tr = f(dxx + dyy)
    det = f(dxx * dyy - dxy * dxy)
    e = f(edge)
    if det <= 0 or tr * tr * e >= (e + f(1)) * (e + f(1)) * det:
        return None
    scale = f(1 << o)
    x = f(f(c) + xc) * scale
    y = f(f(r) + xr) * scale
    octave_word = o + (layer << 8) + (cv_round((float(xi) + 0.5) * 255) << 16)  # double, as in C
    size = f(sigma) * f(2.0 ** float(f(layer + xi) / f(n_layers))) * scale * f(2)
    return (o, layer, r, c, float(x), float(y), octave_word, float(size), float(abs(contr)), float(xi))


def detect(gray: np.ndarray, contrast: float = 0.04, edge: float = 10.0, sigma: float = 1.6, n_layers: int = 3):
    """DoG keypoints of ``gray`` before orientation assignment, in (octave, level, row, column)
    order -> dict of arrays: pt (k, 2) float32 in input-image pixels, size, response,
    octave (OpenCV's packed word with the first octave at -1), level, xi, and the
    (octave index, level, row, column) of the extremum after refinement."""
    pyr = gaussian_pyramid(gray, sigma, n_layers)
    dog = dog_pyramid(pyr)
    thr = math.floor(0.5 * contrast / n_layers * 255)
    out = []
    for o in range(len(dog)):
        for layer in range(1, n_layers + 1):
            img, prev, nxt = dog[o][layer], dog[o][layer - 1], dog[o][layer + 1]
            h, w = img.shape
            if h <= 2 * SIFT_IMG_BORDER or w <= 2 * SIFT_IMG_BORDER:
                continue
            cands = extrema_mask(prev, img, nxt, thr)
            for r, c in zip(*np.nonzero(cands)):
                kp = adjust_local_extremum(dog, o, layer, int(r), int(c), n_layers, contrast, edge, sigma)
                if kp is not None:
                    out.append(kp)
    return _pack(out)


def extrema_mask(prev, img, nxt, thr) -> np.ndarray:
    """Candidates of one DoG level: border 5, |v| > thr, >= / <= all 26 neighbours."""
    h, w = img.shape
    b = SIFT_IMG_BORDER
    v = img[b:h - b, b:w - b]
    big = np.abs(v) > np.float32(thr)
    is_max = big & (v > 0)
    is_min = big & (v < 0)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            for k, L in enumerate((prev, img, nxt)):
                if k == 1 and dy == 0 and dx == 0:
                    continue
                nb = L[b + dy:h - b + dy, b + dx:w - b + dx]
                is_max &= v >= nb
                is_min &= v <= nb
    m = np.zeros((h, w), dtype=bool)
    m[b:h - b, b:w - b] = is_max | is_min
    return m


def _pack(kps):
    n = len(kps)
    a = np.array(kps, dtype=np.float64).reshape(n, 10)
    half = np.float32(0.5)  # firstOctave = -1: back to input-image pixels
    oct_word = a[:, 6].astype(np.int64)
    o = oct_word & 255
    oct_word = (oct_word & ~255) | ((o + FIRST_OCTAVE) & 255)
    return {
        "pt": (a[:, 4:6].astype(np.float32) * half).astype(np.float32),
        "size": (a[:, 7].astype(np.float32) * half).astype(np.float32),
        "response": a[:, 8].astype(np.float32),
        "octave": oct_word.astype(np.int32),
        "xi": a[:, 9].astype(np.float32),
        "index": a[:, :4].astype(np.int32),  # (octave, level, row, column)
    }
