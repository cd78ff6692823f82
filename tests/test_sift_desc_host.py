"""Host emulation of sift_desc_kernel's phase 2 (csrc/sift_desc.hip) against the oracle.

The kernel gives each interior (cell, orientation slot) bin of the 4 x 4 x 8 descriptor a
lane that walks the bounding box of its cell's rotated footprint in window order.  This
test restates that walk in float32 numpy and checks that it reproduces
``oracle.sift_ref.descriptor`` bit for bit (no sample missed, none counted twice, the
per-bin order kept), on keypoints of every angle quadrant and scale.
"""

import math

import numpy as np

from oracle import sift_ref as S
from visualodometry_amd.synthetic import sift_scene

f = np.float32


def emulate(img, x, y, ori, scl, d=4, n=8):
    rows, cols = img.shape
    px, py = S.cv_round(float(x)), S.cv_round(float(y))
    ori = f(ori)
    cos0, sin0 = S.cos_sin_deg(ori)
    bins_per_rad = f(n) / f(360)
    exp_scale = f(-1) / f(d * d * 0.5)
    hw = f(f(3) * f(scl))
    radius = S.cv_round(float(f(f(f(hw * f(1.4142135623730951)) * f(d + 1)) * f(0.5))))
    radius = min(radius, int(math.sqrt(float(cols) * cols + float(rows) * rows)))
    cos_t, sin_t = f(cos0 / hw), f(sin0 / hw)

    def geom(i, j):
        c_rot = f(f(f(j) * cos_t) - f(f(i) * sin_t))
        r_rot = f(f(f(j) * sin_t) + f(f(i) * cos_t))
        return c_rot, r_rot, f(f(r_rot + f(2)) - f(0.5)), f(f(c_rot + f(2)) - f(0.5))

    # phase 1: per-sample (magnitude * weight, obin)
    samp = {}
    for i in range(-radius, radius + 1):
        for j in range(-radius, radius + 1):
            c_rot, r_rot, rbin, cbin = geom(i, j)
            r, c = py + i, px + j
            if rbin > -1 and rbin < d and cbin > -1 and cbin < d and 0 < r < rows - 1 and 0 < c < cols - 1:
                dx = f(img[r, c + 1] - img[r, c - 1])
                dy = f(img[r - 1, c] - img[r + 1, c])
                w = S.exp32f(np.array([f(f(f(c_rot * c_rot) + f(r_rot * r_rot)) * exp_scale)]))[0]
                Ori = S.fast_atan2(np.array([dy]), np.array([dx]))[0]
                Mag = S.magnitude(np.array([dx]), np.array([dy]))[0]
                samp[(i, j)] = (f(Mag * w), f(f(Ori - ori) * bins_per_rad))
    h10 = np.zeros(160, f)
    for lane in range(160):
        q, O = divmod(lane, 10)
        Rc, Cc = q // 4 + 1, q % 4 + 1
        ii_, jj_ = [], []
        for cr in (0, 1):
            for cc in (0, 1):
                u = f(hw * f(f(Rc) - f(3.5) + f(2 * cr)))
                v = f(hw * f(f(Cc) - f(3.5) + f(2 * cc)))
                ii_.append(f(f(u * cos0) - f(v * sin0)))
                jj_.append(f(f(u * sin0) + f(v * cos0)))
        i0, i1 = max(-radius, math.floor(min(ii_)) - 1), min(radius, math.ceil(max(ii_)) + 1)
        j0, j1 = max(-radius, math.floor(min(jj_)) - 1), min(radius, math.ceil(max(jj_)) + 1)
        acc = f(0)
        for i in range(i0, i1 + 1):
            for j in range(j0, j1 + 1):
                if (i, j) not in samp:
                    continue
                _, _, rbin, cbin = geom(i, j)
                r0, c0 = math.floor(rbin), math.floor(cbin)
                dr, dc = Rc - 1 - r0, Cc - 1 - c0
                if dr not in (0, 1) or dc not in (0, 1):
                    continue
                mag, obin = samp[(i, j)]
                o0 = math.floor(obin)
                ob = f(obin - f(o0))
                o0 = o0 + n if o0 < 0 else o0
                o0 = o0 - n if o0 >= n else o0
                dO = O - o0
                if dO not in (0, 1):
                    continue
                rb, cb = f(rbin - f(r0)), f(cbin - f(c0))
                v_r1 = f(mag * rb)
                vr = v_r1 if dr else f(mag - v_r1)
                v_c1 = f(vr * cb)
                vc = v_c1 if dc else f(vr - v_c1)
                v_o1 = f(vc * ob)
                acc = f(acc + (v_o1 if dO else f(vc - v_o1)))
        h10[lane] = acc
    raw = np.empty(128, f)
    for t in range(128):
        q, k = divmod(t, 8)
        v = h10[q * 10 + k]
        raw[t] = f(v + h10[q * 10 + k + 8]) if k < 2 else v
    nrm2 = f(0)
    for v in raw:
        nrm2 = f(nrm2 + f(v * v))
    thr = f(f(np.sqrt(nrm2)) * f(0.2))
    raw = np.minimum(raw, thr)
    nrm2 = f(0)
    for v in raw:
        nrm2 = f(nrm2 + f(v * v))
    nrm2 = f(f(512) / max(f(np.sqrt(nrm2)), S.FLT_EPSILON))
    return np.clip(np.rint((raw * nrm2).astype(f)), 0, 255).astype(f)


def test_bin_lane_walk_matches_oracle():
    img = S.gaussian_pyramid(sift_scene(120, 160, seed=4, n_blobs=30, n_boxes=8))[0][2]
    rng = np.random.default_rng(0)
    for t in range(8):
        x, y = f(rng.uniform(8, img.shape[1] - 8)), f(rng.uniform(8, img.shape[0] - 8))
        ori = f(45 * t + rng.uniform(0, 45))  # every octant
        scl = f(rng.uniform(1.8, 3.6))
        ref = S.descriptor(img, x, y, ori, scl)
        got = emulate(img, x, y, ori, scl)
        assert np.array_equal(got, ref), (t, np.nonzero(got != ref))
    # a window clipped by the image border
    ref = S.descriptor(img, f(3.2), f(4.7), f(123.0), f(3.5))
    assert np.array_equal(emulate(img, f(3.2), f(4.7), f(123.0), f(3.5)), ref)
