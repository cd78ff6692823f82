"""Array-backed map store and trajectory evaluation.

:class:`MapStore` replaces the reference's ``map_points`` dict
(``src/modules/vo.py:17``: ``{pt_id: (3,) float32}``, filled at ``vo.py:281`` and pruned
to the newest 20 000 ids by ``_prune_map``, ``vo.py:35-47``).  It keeps the dict
interface the reference's loops use (``pid in map_points`` at ``vo.py:123``,
``map_points[pid]`` at ``vo.py:127/130``, assignment at ``vo.py:281``, ``del`` in
``_prune_map``, ``.items()`` at ``vo.py:349``) and adds vectorised ``contains``/
``gather``/``scatter`` over id arrays, which the keyframe window uses to feed the BA
and PnP C-ABI without per-point Python loops.

Storage: ids are handed out in increasing order (``next_pt_id``, ``vo.py:282``) and only
the newest ``capacity`` of them are alive after a prune, so a point lives in ring slot
``id % slots`` of float32 ``(slots, 3)`` coordinates with the owning id beside it
(``slots`` = 2 x capacity leaves room for one keyframe's worth of new points between
prunes).  A slot whose owner id differs from the requested one is a miss.

:func:`ate` is the absolute trajectory error after a similarity alignment (Umeyama),
on the ground-truth columns the reference loads (``dataset_loader.py:60``:
``poses[:, [3, 11]]``, the x and z translation of KITTI/Parking poses).
"""

from __future__ import annotations

from collections.abc import MutableMapping

import numpy as np

MAX_POINTS = 20000  # vo.py:38


class MapStore(MutableMapping):
    """Drop-in for the ``map_points`` dict, ring-buffered by id."""

    def __init__(self, capacity: int = MAX_POINTS, slots: int | None = None):
        self.capacity = int(capacity)
        self.slots = int(slots or 2 * self.capacity)
        self.xyz = np.zeros((self.slots, 3), dtype=np.float32)
        self.owner = np.full(self.slots, -1, dtype=np.int64)
        self._n = 0

    # --- dict interface (the reference's per-point loops)
    def __getitem__(self, pid):
        pid = int(pid)
        s = pid % self.slots
        if pid < 0 or self.owner[s] != pid:
            raise KeyError(pid)
        return self.xyz[s].copy()

    def __setitem__(self, pid, value):
        pid = int(pid)
        if pid < 0:
            raise KeyError(pid)
        s = pid % self.slots
        old = int(self.owner[s])
        if old != pid:
            if old >= 0:
                raise OverflowError(f"map store slot of id {pid} still holds id {old}: more than "
                                    f"{self.slots} live points (prune first)")
            self._n += 1
            self.owner[s] = pid
        self.xyz[s] = np.asarray(value, dtype=np.float32).reshape(3)

    def __delitem__(self, pid):
        pid = int(pid)
        s = pid % self.slots
        if pid < 0 or self.owner[s] != pid:
            raise KeyError(pid)
        self.owner[s] = -1
        self._n -= 1

    def __contains__(self, pid) -> bool:
        try:
            pid = int(pid)
        except (TypeError, ValueError):
            return False
        return pid >= 0 and self.owner[pid % self.slots] == pid

    def __iter__(self):
        live = self.owner[self.owner >= 0]
        return iter(np.sort(live).tolist())  # insertion order == id order, as the dict

    def __len__(self) -> int:
        return self._n

    # one vectorised pass instead of MutableMapping's per-key __getitem__ (the reference's
    # per-frame ``for pid, pt in self.map_points.items()``, vo.py:349, over up to 20k points);
    # keys() stays Mapping's KeysView (O(1) containment through __contains__, set operations)
    def values(self):
        return list(self.arrays()[1])

    def items(self):
        ids, xyz = self.arrays()
        return list(zip(ids.tolist(), xyz))

    # --- vectorised access
    def contains(self, ids) -> np.ndarray:
        ids = np.asarray(ids, dtype=np.int64)
        ok = ids >= 0
        return ok & (self.owner[np.where(ok, ids, 0) % self.slots] == ids)

    def gather(self, ids) -> np.ndarray:
        """(k, 3) float32 coordinates of ``ids`` (KeyError if one is absent)."""
        ids = np.asarray(ids, dtype=np.int64)
        if not self.contains(ids).all():
            raise KeyError(ids[~self.contains(ids)][:5].tolist())
        return self.xyz[ids % self.slots].copy()

    def scatter(self, ids, xyz) -> None:
        """Overwrite the coordinates of existing ``ids``."""
        ids = np.asarray(ids, dtype=np.int64)
        if not self.contains(ids).all():
            raise KeyError(ids[~self.contains(ids)][:5].tolist())
        self.xyz[ids % self.slots] = np.asarray(xyz, dtype=np.float32).reshape(-1, 3)

    def insert(self, first_id: int, xyz) -> np.ndarray:
        """Add points with ids ``first_id, first_id + 1, ...``; returns the ids."""
        xyz = np.asarray(xyz, dtype=np.float32).reshape(-1, 3)
        ids = np.arange(first_id, first_id + xyz.shape[0], dtype=np.int64)
        for pid, x in zip(ids, xyz):
            self[pid] = x
        return ids

    def prune_below(self, threshold_id: int) -> int:
        """Drop every id < ``threshold_id`` (``_prune_map``); returns how many."""
        dead = (self.owner >= 0) & (self.owner < threshold_id)
        k = int(dead.sum())
        self.owner[dead] = -1
        self._n -= k
        return k

    def arrays(self):
        """(ids ascending, (k, 3) float32) of every live point."""
        ids = np.sort(self.owner[self.owner >= 0])
        return ids, self.xyz[ids % self.slots].copy()


def umeyama(src: np.ndarray, dst: np.ndarray, with_scale: bool = True):
    """Similarity (s, R, t) minimising ||dst - (s R src + t)||^2 over point pairs (n, d)."""
    src = np.asarray(src, dtype=np.float64)
    dst = np.asarray(dst, dtype=np.float64)
    n, d = src.shape
    mu_s, mu_d = src.mean(0), dst.mean(0)
    xs, xd = src - mu_s, dst - mu_d
    cov = xd.T @ xs / n
    U, D, Vt = np.linalg.svd(cov)
    S = np.eye(d)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[-1, -1] = -1
    R = U @ S @ Vt
    var_s = (xs * xs).sum() / n
    s = float(np.trace(np.diag(D) @ S) / var_s) if with_scale and var_s > 0 else 1.0
    t = mu_d - s * R @ mu_s
    return s, R, t


def ate(est: np.ndarray, gt: np.ndarray, with_scale: bool = True) -> dict:
    """Absolute trajectory error of ``est`` against ``gt`` (both (n, d) positions, e.g. the
    (x, z) columns of KITTI ground truth, ``dataset_loader.py:60``) after a similarity
    (monocular VO has no metric scale) or rigid alignment."""
    est = np.asarray(est, dtype=np.float64)
    gt = np.asarray(gt, dtype=np.float64)
    if est.shape != gt.shape or est.ndim != 2 or est.shape[0] < 2:
        raise ValueError(f"ate: need two (n >= 2, d) arrays, got {est.shape} and {gt.shape}")
    s, R, t = umeyama(est, gt, with_scale)
    aligned = s * est @ R.T + t
    err = np.linalg.norm(aligned - gt, axis=1)
    return {"rmse": float(np.sqrt(np.mean(err ** 2))), "mean": float(err.mean()),
            "median": float(np.median(err)), "max": float(err.max()), "scale": s, "R": R, "t": t,
            "aligned": aligned}


def trajectory_xz(trajectory) -> np.ndarray:
    """The reference's ``vo.trajectory`` (list of camera positions ``T_wc[:3, 3]``,
    ``vo.py:327``) as (n, 2) x/z columns, the layout of its ground truth."""
    tr = np.asarray(trajectory, dtype=np.float64).reshape(-1, 3)
    return tr[:, [0, 2]]
