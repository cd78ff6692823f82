"""CPU oracle for the descriptor matcher -- TEST INFRASTRUCTURE ONLY.

Imported by ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline``
leg of ``bench.py``; never by the product path.

Two restatements of the reference's SIFT matching path
(``src/modules/frontend.py:86-111``: ``cv2.BFMatcher(cv2.NORM_L2,
crossCheck=False).knnMatch(des0, des1, k=2)`` + the 0.75 ratio loop):

* :func:`knn2_int` -- numpy, for integer-valued (OpenCV SIFT) descriptors:
  exact int64 squared distances, float32 ``sqrt`` (correctly rounded, as
  ``std::sqrt(float)`` in OpenCV's ``batchDistL2_32f``), then the two
  smallest keys ``(dist, j)`` per row -- OpenCV's insertion scan with strict
  ``<`` keeps the lower train index on equal distances.
* :func:`knn2_c` -- the C restatement ``oracle/match_ref.c`` (insertion scan
  as written in OpenCV's ``batchDistance``; k-ordered ``fmaf`` chain for the
  squared distance), used for float descriptors and as the timed CPU baseline.

Parity pin: ``cv2`` is absent from this image and the reference ships no
fixtures, so the pin is the hand-built known-answer suite
in ``tests/test_oracle_match.py`` plus agreement of the two restatements.
"""

from __future__ import annotations

import numpy as np

from . import cref

RATIO_THRESH = 0.75  # frontend.py:104


def knn2_int(des0: np.ndarray, des1: np.ndarray):
    """Top-2 ``(idx (n0,2) int32, dist (n0,2) float32)`` for integer-valued descriptors."""
    a = np.asarray(des0)
    b = np.asarray(des1)
    n0, n1 = a.shape[0], b.shape[0]
    idx = np.full((n0, 2), -1, dtype=np.int32)
    dist = np.full((n0, 2), np.finfo(np.float32).max, dtype=np.float32)
    if n0 == 0 or n1 == 0:
        return idx, dist
    ai = a.astype(np.int64)
    bi = b.astype(np.int64)
    d2 = (ai * ai).sum(1)[:, None] + (bi * bi).sum(1)[None, :] - 2 * (ai @ bi.T)
    s = np.sqrt(d2.astype(np.float32))  # exact below 2^24; IEEE sqrt is correctly rounded
    k = min(2, n1)
    order = np.argsort(s, axis=1, kind="stable")[:, :k]  # stable: equal s keeps lower j
    idx[:, :k] = order
    dist[:, :k] = np.take_along_axis(s, order, axis=1)
    return idx, dist


def ratio_filter(idx: np.ndarray, dist: np.ndarray, ratio: float = RATIO_THRESH) -> np.ndarray:
    """frontend.py:105-111 -> (M, 2) int64 pairs in ascending query order."""
    keep = (idx[:, 1] >= 0) & (dist[:, 0].astype(np.float64) < ratio * dist[:, 1].astype(np.float64))
    q = np.nonzero(keep)[0]
    return np.stack([q, idx[q, 0]], axis=1).astype(np.int64).reshape(-1, 2)


def match_int(des0, des1, ratio: float = RATIO_THRESH) -> np.ndarray:
    if len(des0) == 0 or len(des1) == 0:
        return np.empty((0, 2), dtype=np.int64)
    return ratio_filter(*knn2_int(des0, des1), ratio)


def knn2_c(des0: np.ndarray, des1: np.ndarray, nthreads: int = 1):
    return cref.knn2(des0, des1, nthreads)


def match_c(des0, des1, ratio: float = RATIO_THRESH, nthreads: int = 1) -> np.ndarray:
    if len(des0) == 0 or len(des1) == 0:
        return np.empty((0, 2), dtype=np.int64)
    return ratio_filter(*cref.knn2(des0, des1, nthreads), ratio)
