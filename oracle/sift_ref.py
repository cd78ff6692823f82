"""CPU oracle for SIFT detectAndCompute -- TEST INFRASTRUCTURE ONLY.

Imported by ``tests/`` and the ``cpu_baseline`` leg of ``bench.py``; never by the product
path.

Restates ``cv2.SIFT_create(nfeatures, contrastThreshold,
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
* Orientation assignment, the keypoint filtering and the descriptors: see the section
  further down (``detect_and_compute``).

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


# ---------------------------------------------------------------------------------------
# Orientation, keypoint filtering and descriptors (the rest of detectAndCompute).
#
# OpenCV 4.12 sift.simd.hpp / sift.dispatch.cpp / keypoint.cpp, restated:
#
# * ``calcOrientationHist``: 36-bin histogram over a (2 radius + 1)^2 window of the Gaussian
#   level the extremum was refined on, radius = cvRound(4.5 scl), sigma = 1.5 scl with
#   scl = size / 2 / 2^octave; samples strictly inside the image (1 .. rows-2); dx, dy
#   central differences; weight exp32f((i^2 + j^2) * -1 / (2 sigma^2)); bin
#   cvRound(n / 360 * angle) wrapped; ``temphist[bin] += w * mag`` in sample order;
#   [1 4 6 4 1] / 16 circular smoothing; every local peak >= 0.8 max gives a keypoint with
#   the parabolically interpolated angle ``360 - 10 * bin`` (0 when within FLT_EPSILON of
#   360).
# * ``removeDuplicatedSorted``: sort by (x asc, y asc, size desc, angle asc, response desc,
#   octave desc), drop entries equal to the kept predecessor in (x, y, size, angle).
# * ``retainBest(nfeatures)``: when more than nfeatures remain, keep every keypoint whose
#   response is >= the nfeatures-th largest response (ties at the boundary are all kept).
# * ``calcSIFTDescriptor`` (d = 4, n = 8): the window rotated by the keypoint angle,
#   hist_width = 3 scl, radius = cvRound(hist_width * sqrt2 * (d + 1) / 2) clipped to the
#   image diagonal; trilinear votes of exp32f-weighted magnitudes into a (d+2)^2 (n+2)
#   histogram in sample order; orientation wrap; L2 norm, clip at 0.2 * norm, renormalise to
#   512 and saturate_cast<uchar> (round half to even, clamp 0..255), stored as float32.
#
# Build-defined where OpenCV's result depends on the CPU it runs on: OpenCV's SIMD paths of
# exp32f / fastAtan2 / magnitude / the histogram smoothing / the norm sums use FMA where
# the CPU has it, so this file (and csrc/sift.hip) follows the scalar fallback of each
# routine with no FMA; cosf / sinf are ``(float)cos((double)x)``; the keypoint size's
# ``powf(2, e)`` is ``(float)pow(2.0, (double)e)``.  retainBest's nth_element / partition
# leave an implementation-defined order: the output here is the removeDuplicatedSorted
# order, filtered.  Against OpenCV itself this is parity unpinned (cv2 absent).
# ---------------------------------------------------------------------------------------

SIFT_ORI_HIST_BINS = 36
SIFT_ORI_SIG_FCTR = np.float32(1.5)
SIFT_ORI_RADIUS = np.float32(3 * 1.5)
SIFT_ORI_PEAK_RATIO = np.float32(0.8)
SIFT_DESCR_WIDTH = 4
SIFT_DESCR_HIST_BINS = 8
SIFT_DESCR_SCL_FCTR = np.float32(3.0)
SIFT_DESCR_MAG_THR = np.float32(0.2)
SIFT_INT_DESCR_FCTR = np.float32(512.0)
FLT_EPSILON = np.float32(1.1920928955078125e-07)

_f = np.float32

# cv::hal::exp32f (core/src/mathfuncs_core.simd.hpp), scalar path
EXPTAB_SCALE = 6
EXPPOLY_32F_A0 = .9670371139572337719125840413672004409288e-2
EXP_TAB = np.array([2.0 ** (j / 64.0) * EXPPOLY_32F_A0 for j in range(64)], dtype=np.float64).astype(np.float32)
EXP_A4 = _f(1.000000000000002438532970795181890933776 / EXPPOLY_32F_A0)
EXP_A3 = _f(.6931471805521448196800669615864773144641 / EXPPOLY_32F_A0)
EXP_A2 = _f(.2402265109513301490103372422686535526573 / EXPPOLY_32F_A0)
EXP_A1 = _f(.5550339366753125211915322047004666939128e-1 / EXPPOLY_32F_A0)
EXP_PRESCALE = _f(1.4426950408889634073599246810019 * (1 << EXPTAB_SCALE))
EXP_POSTSCALE = _f(1.0 / (1 << EXPTAB_SCALE))
_EXP_MAX = 3000.0 * (1 << EXPTAB_SCALE)
EXP_MINVAL = _f(-_EXP_MAX / (1.4426950408889634073599246810019 * (1 << EXPTAB_SCALE)))
EXP_MAXVAL = _f(_EXP_MAX / (1.4426950408889634073599246810019 * (1 << EXPTAB_SCALE)))


def exp32f(x: np.ndarray) -> np.ndarray:
    """``cv::hal::exp32f`` scalar loop: clamp, scale by 64/ln2, split into cvRound integer and
    fraction, 2^(int>>6) from the exponent bits times the 64-entry table times a quartic."""
    x0 = np.minimum(np.maximum(np.asarray(x, _f), EXP_MINVAL), EXP_MAXVAL)
    x0 = (x0 * EXP_PRESCALE).astype(_f)
    xi = np.rint(x0).astype(np.int32)  # saturate_cast<int>(float) = cvRound
    x0 = ((x0 - xi.astype(_f)) * EXP_POSTSCALE).astype(_f)
    t = (xi >> EXPTAB_SCALE) + 127
    t = np.where((t & ~255) == 0, t, np.where(t < 0, 0, 255)).astype(np.int32)
    buf = (t.astype(np.uint32) << np.uint32(23)).view(np.float32)
    poly = ((((x0 + EXP_A1) * x0 + EXP_A2) * x0 + EXP_A3) * x0 + EXP_A4).astype(_f)
    return ((buf * EXP_TAB[xi & 63]).astype(_f) * poly).astype(_f)


_RAD2DEG = _f(180 / math.pi)
ATAN_P1 = _f(_f(0.9997878412794807) * _RAD2DEG)
ATAN_P3 = _f(_f(-0.3258083974640975) * _RAD2DEG)
ATAN_P5 = _f(_f(0.1555786518463281) * _RAD2DEG)
ATAN_P7 = _f(_f(-0.04432655554792128) * _RAD2DEG)
_DBL_EPS_F = _f(2.220446049250313e-16)


def fast_atan2(y: np.ndarray, x: np.ndarray) -> np.ndarray:
    """``cv::fastAtan2`` in degrees (core/src/mathfuncs_core.simd.hpp ``atan_f32``)."""
    y = np.asarray(y, _f)
    x = np.asarray(x, _f)
    ax, ay = np.abs(x), np.abs(y)
    ge = ax >= ay
    num = np.where(ge, ay, ax)
    den = (np.where(ge, ax, ay) + _DBL_EPS_F).astype(_f)
    c = (num / den).astype(_f)
    c2 = (c * c).astype(_f)
    a = ((((ATAN_P7 * c2 + ATAN_P5) * c2 + ATAN_P3) * c2 + ATAN_P1) * c).astype(_f)
    a = np.where(ge, a, _f(90) - a).astype(_f)
    a = np.where(x < 0, _f(180) - a, a).astype(_f)
    return np.where(y < 0, _f(360) - a, a).astype(_f)


def magnitude(x: np.ndarray, y: np.ndarray) -> np.ndarray:
    x = np.asarray(x, _f)
    y = np.asarray(y, _f)
    return np.sqrt((x * x + y * y).astype(_f)).astype(_f)


def cos_sin_deg(ori: float) -> tuple:
    """cosf / sinf of ``ori * (float)(CV_PI/180)`` as ``(float)cos((double)x)``."""
    a = float(_f(ori) * _f(math.pi / 180))
    return _f(math.cos(a)), _f(math.sin(a))


def orientation_hist(img: np.ndarray, px: int, py: int, radius: int, sigma, n: int = SIFT_ORI_HIST_BINS):
    """``calcOrientationHist`` -> (smoothed hist (n,) float32, max)."""
    rows, cols = img.shape
    sigma = _f(sigma)
    expf_scale = _f(-1) / ((_f(2) * sigma) * sigma)
    ii, jj = np.meshgrid(np.arange(-radius, radius + 1), np.arange(-radius, radius + 1), indexing="ij")
    y = py + ii
    x = px + jj
    ok = (y > 0) & (y < rows - 1) & (x > 0) & (x < cols - 1)
    ii, jj, y, x = ii[ok], jj[ok], y[ok], x[ok]  # row-major sample order
    dx = (img[y, x + 1] - img[y, x - 1]).astype(_f)
    dy = (img[y - 1, x] - img[y + 1, x]).astype(_f)
    W = ((ii * ii + jj * jj).astype(_f) * expf_scale).astype(_f)
    W = exp32f(W)
    ori = fast_atan2(dy, dx)
    mag = magnitude(dx, dy)
    bins = np.rint((_f(n) / _f(360)) * ori).astype(np.int64)
    bins = np.where(bins >= n, bins - n, bins)
    bins = np.where(bins < 0, bins + n, bins)
    temp = np.zeros(n, _f)
    np.add.at(temp, bins, (W * mag).astype(_f))  # sequential, in sample order
    tp = np.concatenate([temp[-2:], temp, temp[:2]])
    hist = ((tp[0:n] + tp[4:n + 4]) * _f(1 / 16) + (tp[1:n + 1] + tp[3:n + 3]) * _f(4 / 16) +
            tp[2:n + 2] * _f(6 / 16)).astype(_f)
    return hist, _f(hist.max())


def orientation_peaks(hist: np.ndarray, omax) -> list:
    """Angles (degrees, float32) of the histogram peaks >= 0.8 max, in bin order."""
    n = hist.size
    mag_thr = _f(_f(omax) * SIFT_ORI_PEAK_RATIO)
    out = []
    for j in range(n):
        l, r2 = (j - 1) if j > 0 else n - 1, (j + 1) if j < n - 1 else 0
        if hist[j] > hist[l] and hist[j] > hist[r2] and hist[j] >= mag_thr:
            b = _f(_f(j) + (_f(0.5) * (hist[l] - hist[r2])) / ((hist[l] - _f(2) * hist[j]) + hist[r2]))
            b = _f(n) + b if b < 0 else (b - _f(n) if b >= n else b)
            angle = _f(_f(360) - _f(_f(360.0 / n) * _f(b)))
            if abs(angle - _f(360)) < FLT_EPSILON:
                angle = _f(0)
            out.append(angle)
    return out


def descriptor(img: np.ndarray, x: float, y: float, ori, scl, d: int = SIFT_DESCR_WIDTH,
               n: int = SIFT_DESCR_HIST_BINS) -> np.ndarray:
    """``calcSIFTDescriptor`` -> (d*d*n,) float32 holding integers 0..255."""
    rows, cols = img.shape
    ptx, pty = cv_round(float(x)), cv_round(float(y))
    ori = _f(ori)
    cos_t, sin_t = cos_sin_deg(ori)
    bins_per_rad = _f(n) / _f(360)
    exp_scale = _f(-1) / _f(d * d * 0.5)
    hist_width = _f(SIFT_DESCR_SCL_FCTR * _f(scl))
    radius = cv_round(float(_f(_f(_f(hist_width * _f(1.4142135623730951)) * _f(d + 1)) * _f(0.5))))
    radius = min(radius, int(math.sqrt(float(cols) * cols + float(rows) * rows)))
    cos_t = _f(cos_t / hist_width)
    sin_t = _f(sin_t / hist_width)
    ii, jj = np.meshgrid(np.arange(-radius, radius + 1), np.arange(-radius, radius + 1), indexing="ij")
    ii, jj = ii.ravel(), jj.ravel()
    fi, fj = ii.astype(_f), jj.astype(_f)
    c_rot = (fj * cos_t - fi * sin_t).astype(_f)
    r_rot = (fj * sin_t + fi * cos_t).astype(_f)
    half = _f(d // 2)
    rbin = ((r_rot + half) - _f(0.5)).astype(_f)
    cbin = ((c_rot + half) - _f(0.5)).astype(_f)
    r = pty + ii
    c = ptx + jj
    ok = ((rbin > -1) & (rbin < d) & (cbin > -1) & (cbin < d) & (r > 0) & (r < rows - 1) & (c > 0) & (c < cols - 1))
    r, c, rbin, cbin, c_rot, r_rot = r[ok], c[ok], rbin[ok], cbin[ok], c_rot[ok], r_rot[ok]
    dx = (img[r, c + 1] - img[r, c - 1]).astype(_f)
    dy = (img[r - 1, c] - img[r + 1, c]).astype(_f)
    W = ((c_rot * c_rot + r_rot * r_rot) * exp_scale).astype(_f)
    Ori = fast_atan2(dy, dx)
    Mag = magnitude(dx, dy)
    W = exp32f(W)
    obin = ((Ori - ori) * bins_per_rad).astype(_f)
    mag = (Mag * W).astype(_f)
    r0 = np.floor(rbin).astype(np.int64)
    c0 = np.floor(cbin).astype(np.int64)
    o0 = np.floor(obin).astype(np.int64)
    rb = (rbin - r0.astype(_f)).astype(_f)
    cb = (cbin - c0.astype(_f)).astype(_f)
    ob = (obin - o0.astype(_f)).astype(_f)
    o0 = np.where(o0 < 0, o0 + n, o0)
    o0 = np.where(o0 >= n, o0 - n, o0)
    v_r1 = (mag * rb).astype(_f)
    v_r0 = (mag - v_r1).astype(_f)
    v_rc11 = (v_r1 * cb).astype(_f)
    v_rc10 = (v_r1 - v_rc11).astype(_f)
    v_rc01 = (v_r0 * cb).astype(_f)
    v_rc00 = (v_r0 - v_rc01).astype(_f)
    v = {}
    for key, base in (("11", v_rc11), ("10", v_rc10), ("01", v_rc01), ("00", v_rc00)):
        v[key + "1"] = (base * ob).astype(_f)
        v[key + "0"] = (base - v[key + "1"]).astype(_f)
    idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0
    s1, s2 = n + 2, (d + 2) * (n + 2)
    order = [(0, "000"), (1, "001"), (s1, "010"), (s1 + 1, "011"), (s2, "100"), (s2 + 1, "101"),
             (s2 + s1, "110"), (s2 + s1 + 1, "111")]
    tgt = np.stack([idx + off for off, _ in order], 1).ravel()  # sample-major: sample order per bin
    val = np.stack([v[k] for _, k in order], 1).ravel()
    hist = np.zeros((d + 2) * (d + 2) * (n + 2), _f)
    np.add.at(hist, tgt, val)
    raw = np.empty(d * d * n, _f)
    for i in range(d):
        for j in range(d):
            b = ((i + 1) * (d + 2) + (j + 1)) * (n + 2)
            hist[b] = _f(hist[b] + hist[b + n])
            hist[b + 1] = _f(hist[b + 1] + hist[b + n + 1])
            raw[(i * d + j) * n:(i * d + j + 1) * n] = hist[b:b + n]
    nrm2 = _f(0)
    for k in range(raw.size):
        nrm2 = _f(nrm2 + _f(raw[k] * raw[k]))
    thr = _f(_f(np.sqrt(nrm2)) * SIFT_DESCR_MAG_THR)
    raw = np.minimum(raw, thr)
    nrm2 = _f(0)
    for k in range(raw.size):
        nrm2 = _f(nrm2 + _f(raw[k] * raw[k]))
    nrm2 = _f(SIFT_INT_DESCR_FCTR / max(_f(np.sqrt(nrm2)), FLT_EPSILON))
    return np.clip(np.rint((raw * nrm2).astype(_f)), 0, 255).astype(_f)


def _sort_key(k):
    # KeyPoint12_LessThan: x asc, y asc, size desc, angle asc, response desc, octave desc
    return (k["x"], k["y"], -k["size"], k["angle"], -k["response"], -k["octave"])


def detect_and_compute(gray: np.ndarray, nfeatures: int = 0, contrast: float = 0.04, edge: float = 10.0,
                       sigma: float = 1.6, n_layers: int = 3, with_descriptors: bool = True) -> dict:
    """``SIFT_create(nfeatures, nOctaveLayers, contrastThreshold, edgeThreshold, sigma)
    .detectAndCompute(gray, None)`` -> dict: pt (N, 2), size, angle, response, octave (as
    cv::KeyPoint holds them) and descriptors (N, 128) float32."""
    pyr = gaussian_pyramid(gray, sigma, n_layers)
    det = detect(gray, contrast, edge, sigma, n_layers)
    kps = []
    for i in range(len(det["pt"])):
        o, layer, r, c = (int(v) for v in det["index"][i])
        size2 = _f(det["size"][i] * _f(2))  # back to doubled-image units (exact)
        scl_octv = _f(_f(size2 * _f(0.5)) / _f(1 << o))
        hist, omax = orientation_hist(pyr[o][layer], c, r, cv_round(float(SIFT_ORI_RADIUS * scl_octv)),
                                      _f(SIFT_ORI_SIG_FCTR * scl_octv))
        word = int(det["octave"][i])
        word_pre = (word & ~255) | (((word & 255) + 1) & 255)
        for ang in orientation_peaks(hist, omax):
            kps.append(dict(x=_f(det["pt"][i, 0] * _f(2)), y=_f(det["pt"][i, 1] * _f(2)), size=size2, angle=ang,
                            response=_f(det["response"][i]), octave=word_pre, o=o, layer=layer))
    kps.sort(key=_sort_key)
    uniq = []
    for k in kps:  # removeDuplicatedSorted
        if uniq and (uniq[-1]["x"] == k["x"] and uniq[-1]["y"] == k["y"] and uniq[-1]["size"] == k["size"] and
                     uniq[-1]["angle"] == k["angle"]):
            continue
        uniq.append(k)
    if nfeatures > 0 and len(uniq) > nfeatures:  # retainBest
        t = np.sort(np.array([k["response"] for k in uniq], _f))[::-1][nfeatures - 1]
        uniq = [k for k in uniq if k["response"] >= t]
    N = len(uniq)
    desc = np.zeros((N, SIFT_DESCR_WIDTH ** 2 * SIFT_DESCR_HIST_BINS), _f)
    if with_descriptors:
        for i, k in enumerate(uniq):
            # calcDescriptors: the octave's image, pt and size in octave pixels (exact scalings)
            s = _f(1.0 / (1 << k["o"]))
            ang = _f(_f(360) - k["angle"])
            if abs(ang - _f(360)) < FLT_EPSILON:
                ang = _f(0)
            desc[i] = descriptor(pyr[k["o"]][k["layer"]], _f(k["x"] * s), _f(k["y"] * s), ang,
                                 _f(_f(k["size"] * s) * _f(0.5)))
    half = _f(0.5)
    octs = np.array([(k["octave"] & ~255) | (((k["octave"] & 255) + FIRST_OCTAVE) & 255) for k in uniq], np.int64)
    return {
        "pt": np.array([[k["x"] * half, k["y"] * half] for k in uniq], _f).reshape(N, 2),
        "size": np.array([k["size"] * half for k in uniq], _f),
        "angle": np.array([k["angle"] for k in uniq], _f),
        "response": np.array([k["response"] for k in uniq], _f),
        "octave": octs.astype(np.int32),
        "descriptors": desc,
    }
