"""ctypes binding of the C oracle ``oracle/build/liboracle.so`` -- TEST INFRASTRUCTURE ONLY.

Built by ``make -C oracle`` (called from ``__graft_entry__.build()``).
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "liboracle.so"
_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        lib = C.CDLL(str(LIB))
        P = C.c_void_p
        lib.oracle_knn2.argtypes = [P, C.c_int, P, C.c_int, C.c_int, P, P, C.c_int]
        lib.oracle_knn2.restype = None
        lib.oracle_ba_step.argtypes = [C.c_int, C.c_int, C.c_int] + [C.c_double] * 5 + [P] * 9 + [C.c_int]
        lib.oracle_ba_step.restype = C.c_int
        lib.oracle_ba_solve.argtypes = ([C.c_int, C.c_int, C.c_int] + [C.c_double] * 5 + [P] * 5
                                        + [C.c_int, P, C.c_int])
        lib.oracle_ba_solve.restype = C.c_int
        lib.oracle_ba_cost.argtypes = [C.c_int] + [C.c_double] * 4 + [P] * 5 + [C.c_int]
        lib.oracle_ba_cost.restype = C.c_double
        _lib = lib
    return _lib


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def default_threads() -> int:
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def knn2(des0, des1, nthreads: int = 1):
    a = np.ascontiguousarray(des0, dtype=np.float32)
    b = np.ascontiguousarray(des1, dtype=np.float32)
    n0 = a.shape[0]
    idx = np.full((n0, 2), -1, dtype=np.int32)
    dist = np.full((n0, 2), np.finfo(np.float32).max, dtype=np.float32)
    if n0 and b.shape[0]:
        load().oracle_knn2(_p(a), n0, _p(b), b.shape[0], a.shape[1], _p(idx), _p(dist), nthreads)
    return idx, dist


def _rt(poses_cw):
    P = np.asarray(poses_cw, dtype=np.float64)
    out = np.empty((P.shape[0], 12))
    out[:, :9] = P[:, :3, :3].reshape(-1, 9)
    out[:, 9:] = P[:, :3, 3]
    return out


def _poses(rt):
    T = np.tile(np.eye(4), (rt.shape[0], 1, 1))
    T[:, :3, :3] = rt[:, :9].reshape(-1, 3, 3)
    T[:, :3, 3] = rt[:, 9:]
    return T


class BAProblemRef:
    """Structure of a BA window for the C oracle (same layout as the C-ABI)."""

    def __init__(self, K, point_ptr, obs_cam, obs_uv, n_poses, n_fixed=2, lam=0.0):
        self.K = np.asarray(K, dtype=np.float64)
        self.point_ptr = np.ascontiguousarray(point_ptr, dtype=np.int32)
        self.obs_cam = np.ascontiguousarray(obs_cam, dtype=np.int32)
        self.obs_uv = np.ascontiguousarray(obs_uv, dtype=np.float32)
        self.n_poses = int(n_poses)
        self.n_fixed = int(n_fixed)
        self.lam = float(lam)

    @property
    def n_points(self):
        return self.point_ptr.size - 1

    def _k(self):
        K = self.K
        return K[0, 0], K[1, 1], K[0, 2], K[1, 2]

    def step(self, poses_cw, points, nthreads: int = 1, want_system: bool = True):
        """One GN step: returns (ok, poses, points, cost, S, b, dc)."""
        rt = _rt(poses_cw)
        X = np.ascontiguousarray(points, dtype=np.float64).copy()
        F = self.n_poses - self.n_fixed
        S = np.empty((6 * F, 6 * F)) if want_system else None
        b = np.empty(6 * F) if want_system else None
        dc = np.zeros(6 * F)
        cost = np.zeros(1)
        ok = load().oracle_ba_step(
            self.n_poses, self.n_points, self.n_fixed, *self._k(), self.lam, _p(self.point_ptr),
            _p(self.obs_cam), _p(self.obs_uv), _p(rt), _p(X), _p(cost), _p(S), _p(b), _p(dc), nthreads)
        return bool(ok), _poses(rt), X, float(cost[0]), S, b, dc

    def solve(self, poses_cw, points, iters: int, nthreads: int = 1):
        rt = _rt(poses_cw)
        X = np.ascontiguousarray(points, dtype=np.float64).copy()
        costs = np.full(iters + 1, np.nan)
        n = load().oracle_ba_solve(
            self.n_poses, self.n_points, self.n_fixed, *self._k(), self.lam, _p(self.point_ptr),
            _p(self.obs_cam), _p(self.obs_uv), _p(rt), _p(X), iters, _p(costs), nthreads)
        return n, _poses(rt), X, costs

    def cost(self, poses_cw, points, nthreads: int = 1) -> float:
        rt = _rt(poses_cw)
        X = np.ascontiguousarray(points, dtype=np.float64)
        return load().oracle_ba_cost(self.n_points, *self._k(), _p(self.point_ptr), _p(self.obs_cam),
                                     _p(self.obs_uv), _p(rt), _p(X), nthreads)
