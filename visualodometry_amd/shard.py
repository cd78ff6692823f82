"""Landmark sharding of a BA window across ranks (one process per GPU).

Each rank owns a contiguous run of whole landmarks (and all of their
observations), balanced by observation count; every rank keeps all cameras.
The per-rank partial reduced camera systems are summed by one RCCL
all-reduce per Gauss-Newton iteration inside ``libvo_hip.so``
(``vo_comm_init``).
"""

from __future__ import annotations

import numpy as np


def shard_bounds(point_ptr: np.ndarray, nranks: int) -> np.ndarray:
    """Landmark boundaries (nranks+1,) splitting the observations evenly."""
    point_ptr = np.asarray(point_ptr, dtype=np.int64)
    M = int(point_ptr[-1])
    targets = (np.arange(1, nranks) * M) // max(nranks, 1)
    cuts = np.searchsorted(point_ptr, targets, side="left")
    return np.concatenate([[0], cuts, [point_ptr.size - 1]]).astype(np.int64)


def shard(point_ptr, obs_cam, obs_uv, points, nranks: int, rank: int):
    """This rank's landmark shard: (point range, point_ptr, obs_cam, obs_uv, points)."""
    b = shard_bounds(point_ptr, nranks)
    p0, p1 = int(b[rank]), int(b[rank + 1])
    o0, o1 = int(point_ptr[p0]), int(point_ptr[p1])
    ptr = (np.asarray(point_ptr[p0 : p1 + 1], dtype=np.int64) - o0).astype(np.int32)
    return (p0, p1), ptr, np.asarray(obs_cam)[o0:o1], np.asarray(obs_uv)[o0:o1], np.asarray(points)[p0:p1]
