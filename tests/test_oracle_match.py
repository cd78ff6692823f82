"""The matcher oracle (numpy + C restatements) against its golden vectors and KATs.

Parity pin: cv2 is absent and the reference has no fixtures, so
the oracle is pinned by the hand-built known-answer cases below (OpenCV
BFMatcher(NORM_L2).knnMatch(k=2) semantics: strict-'<' insertion, lower train
index on ties, sqrtf distances, double ratio compare at 0.75) and by the two
independent restatements agreeing bit for bit.
"""

import numpy as np
import pytest

from oracle import match_ref
from tests.conftest import GOLDEN
from visualodometry_amd.synthetic import sift_like_pair, superpoint_like_pair


def test_golden_sift_512():
    g = np.load(GOLDEN / "match_sift_512.npz")
    d0, d1 = g["des0"].astype(np.float32), g["des1"].astype(np.float32)
    for idx, dist in (match_ref.knn2_int(d0, d1), match_ref.knn2_c(d0, d1, nthreads=4)):
        np.testing.assert_array_equal(idx, g["idx"])
        np.testing.assert_array_equal(dist.view(np.uint32), g["dist"].view(np.uint32))
    np.testing.assert_array_equal(match_ref.match_int(d0, d1), g["pairs"])


@pytest.mark.parametrize("case", ["ties", "n1_eq_1", "n1_eq_2", "many_to_one", "sqrt_collision"])
def test_golden_kats(case):
    g = np.load(GOLDEN / "match_kat.npz")
    a, b = g[f"{case}_des0"], g[f"{case}_des1"]
    for idx, dist in (match_ref.knn2_int(a, b), match_ref.knn2_c(a, b)):
        np.testing.assert_array_equal(idx, g[f"{case}_idx"])
        np.testing.assert_array_equal(dist, g[f"{case}_dist"])
    np.testing.assert_array_equal(match_ref.match_int(a, b), g[f"{case}_pairs"])


def test_kat_semantics():
    g = np.load(GOLDEN / "match_kat.npz")
    # ties: each query matches its own copy first, then the copy 6 rows later
    np.testing.assert_array_equal(g["ties_idx"][:, 0], np.arange(6))
    np.testing.assert_array_equal(g["ties_idx"][:, 1], np.arange(6) + 6)
    assert g["ties_pairs"].shape == (0, 2)  # 0 < 0.75 * 0 is false
    assert (g["n1_eq_1_idx"][:, 1] == -1).all() and g["n1_eq_1_pairs"].shape == (0, 2)
    assert (g["many_to_one_pairs"][:, 1] == 0).all() and len(g["many_to_one_pairs"]) == 5
    # sqrt collision: train 1 (d2 = n + 1) beats train 3 (d2 = n) on the lower index
    np.testing.assert_array_equal(g["sqrt_collision_idx"][0], [1, 3])


def test_brute_force_definition_small():
    """Both restatements equal a literal O(n0 n1) sort on (sqrtf(d2), j)."""
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (20, 16)).astype(np.float32)
    b = rng.integers(0, 256, (30, 16)).astype(np.float32)
    b[5] = b[7]  # exact duplicate train rows
    idx, dist = match_ref.knn2_int(a, b)
    for i in range(len(a)):
        d = [np.sqrt(np.float32(((a[i].astype(np.int64) - b[j].astype(np.int64)) ** 2).sum())) for j in range(len(b))]
        order = sorted(range(len(b)), key=lambda j: (d[j], j))
        assert list(idx[i]) == order[:2]
        assert list(dist[i]) == [d[order[0]], d[order[1]]]


def test_empty_inputs():
    d = np.zeros((3, 128), np.float32)
    e = np.zeros((0, 128), np.float32)
    assert match_ref.match_int(e, d).shape == (0, 2)
    assert match_ref.match_c(d, e).shape == (0, 2)


def test_numpy_and_c_agree_sift_and_float():
    d0, d1 = sift_like_pair(300, 350, 12)
    i1, s1 = match_ref.knn2_int(d0, d1)
    i2, s2 = match_ref.knn2_c(d0, d1, nthreads=4)
    np.testing.assert_array_equal(i1, i2)
    np.testing.assert_array_equal(s1, s2)
    # float descriptors: the C oracle defines the fp32 fmaf-chain path; its indices
    # agree with an exact float64 ranking wherever the ranking is not a near tie
    f0, f1 = superpoint_like_pair(100, 150, 13)
    ic, sc = match_ref.knn2_c(f0, f1)
    d = np.sqrt(((f0[:, None, :].astype(np.float64) - f1[None, :, :]) ** 2).sum(-1))
    best = np.argsort(d, axis=1, kind="stable")[:, :2]
    gap = np.take_along_axis(d, best, 1)
    clear = (gap[:, 1] - gap[:, 0]) > 1e-5
    np.testing.assert_array_equal(ic[clear, 0], best[clear, 0])
