"""Sliding-window bundle adjustment on MI355X (Gauss-Newton with Schur complement).

The reference has no BA: ``pyceres``/``pycolmap`` are declared
(``pyproject.toml:11-12``) but never imported, and pose comes only from
``cv2.solvePnPRansac`` (``src/modules/vo.py:135-141``).  This module is the
build-defined BA API of SURVEY.md §8b, meant to be called from the keyframe
hook ``VisualOdometry._create_keyframe`` (``src/modules/vo.py:252-288``):

    ba = SlidingWindowBA(K, cfg)
    result = ba.optimize(window)        # never raises on a degenerate window

Model (identical to ``oracle/ba_ref.py``): residual ``pi(K (R_cw X + t_cw)) - uv``
with the no-distortion pinhole of ``frontend.py:139``, cost ``sum ||r||^2``,
left se(3) pose increments, the first ``n_fixed`` poses fixed, pure GN.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import BAProblemC, C, VoError, check, ptr


@dataclass
class BAWindow:
    """Keyframe window handed to :meth:`SlidingWindowBA.optimize`.

    ``obs_pt`` gives the landmark of each observation in any order; it is
    grouped by landmark (CSR) before the C-ABI call.
    """

    poses_cw: np.ndarray  # (N,4,4) float64, world -> camera
    points: np.ndarray  # (L,3) float64
    obs_uv: np.ndarray  # (M,2) float32 pixels
    obs_cam: np.ndarray  # (M,) int
    obs_pt: np.ndarray  # (M,) int
    n_fixed: int = 2


@dataclass
class BAResult:
    poses_cw: np.ndarray
    points: np.ndarray
    cost_per_iter: np.ndarray = field(default_factory=lambda: np.zeros(0))
    status: str = "ok"  # "ok" | "not_spd" | "skipped"
    message: str = ""


def poses_to_rt(poses_cw: np.ndarray) -> np.ndarray:
    """(N,4,4) -> (N,12) = R row-major, t (the C-ABI pose layout)."""
    P = np.asarray(poses_cw, dtype=np.float64)
    out = np.empty((P.shape[0], 12))
    out[:, :9] = P[:, :3, :3].reshape(-1, 9)
    out[:, 9:] = P[:, :3, 3]
    return out


def rt_to_poses(rt: np.ndarray) -> np.ndarray:
    T = np.tile(np.eye(4), (rt.shape[0], 1, 1))
    T[:, :3, :3] = rt[:, :9].reshape(-1, 3, 3)
    T[:, :3, 3] = rt[:, 9:]
    return T


def _as_index32(obs_pt) -> np.ndarray:
    """obs_pt as contiguous int32, checked in its own (wider) type first: an int64 index of
    2^31 or more, or a large negative one, must not wrap into [0, n_points)."""
    a = np.asarray(obs_pt).reshape(-1)
    if a.dtype != np.int32 and a.size:
        if not np.issubdtype(a.dtype, np.integer):
            raise ValueError("obs_pt must be integer")
        if int(a.min()) < 0 or int(a.max()) > np.iinfo(np.int32).max:
            raise ValueError("obs_pt out of range")
    return np.ascontiguousarray(a, dtype=np.int32)


def csr_from_obs_pt(n_points: int, obs_pt: np.ndarray):
    """Stable grouping of observations by landmark -> (order, point_ptr)
    (``vo_ba_group_by_point``: one counting sort on the host)."""
    obs_pt = _as_index32(obs_pt)
    order = np.empty(obs_pt.size, dtype=np.int32)
    ptr_ = np.empty(int(n_points) + 1, dtype=np.int32)
    rc = _lib.load().vo_ba_group_by_point(int(n_points), obs_pt.size, ptr(obs_pt, C.c_int32),
                                          ptr(order, C.c_int32), ptr(ptr_, C.c_int32))
    if rc != _lib.VO_OK:
        raise ValueError("obs_pt out of range")
    return order, ptr_


def group_window(n_points: int, window: "BAWindow"):
    """The window's observations grouped by landmark -> (point_ptr, obs_cam, obs_uv).
    Windows built landmark by landmark (dropin/hooks.py ``KeyframeWindow.build``) are
    already grouped: their arrays pass through unchanged; others are reordered by
    ``csr_from_obs_pt``."""
    obs_pt = _as_index32(window.obs_pt)
    obs_cam = np.asarray(window.obs_cam)
    obs_uv = np.asarray(window.obs_uv, dtype=np.float32).reshape(-1, 2)
    point_ptr = np.empty(int(n_points) + 1, dtype=np.int32)
    # order == NULL: one pass that checks the grouping and fills point_ptr
    rc = _lib.load().vo_ba_group_by_point(int(n_points), obs_pt.size, ptr(obs_pt, C.c_int32), None,
                                          ptr(point_ptr, C.c_int32))
    if rc == _lib.VO_OK:
        return point_ptr, obs_cam, obs_uv
    if rc != 1:
        raise ValueError("obs_pt out of range")
    order, point_ptr = csr_from_obs_pt(n_points, obs_pt)
    return point_ptr, obs_cam[order], obs_uv[order]


def _problem_struct(K, point_ptr, obs_cam, obs_uv, n_poses, n_fixed, lam):
    K = np.asarray(K, dtype=np.float64)
    prob = BAProblemC()
    prob.n_poses = int(n_poses)
    prob.n_points = point_ptr.size - 1
    prob.n_obs = obs_cam.size
    prob.n_fixed = int(n_fixed)
    prob.fx, prob.fy, prob.cx, prob.cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    prob.lam = float(lam)
    prob.point_ptr = ptr(point_ptr, C.c_int32)
    prob.obs_cam = ptr(obs_cam, C.c_int32)
    prob.obs_uv = ptr(obs_uv, C.c_float)
    return prob


def plan_probe(K, point_ptr, obs_cam, obs_uv, n_poses: int, n_fixed: int = 2,
               target_segments: int = 512) -> dict:
    """Host-only static plan statistics (no device needed): ``vo_ba_plan_probe``."""
    point_ptr = np.ascontiguousarray(point_ptr, dtype=np.int32)
    obs_cam = np.ascontiguousarray(obs_cam, dtype=np.int32)
    obs_uv = np.ascontiguousarray(obs_uv, dtype=np.float32).reshape(-1, 2)
    prob = _problem_struct(K, point_ptr, obs_cam, obs_uv, n_poses, n_fixed, 0.0)
    out = np.zeros(14, dtype=np.int64)
    n = check(_lib.load().vo_ba_plan_probe(C.byref(prob), int(target_segments),
                                           ptr(out, C.c_int64), 14), "vo_ba_plan_probe")
    keys = ["chunks", "segments", "slab_blocks", "profile_blocks", "track_entries",
            "max_chunk_pairs", "max_segment_slots", "max_segment_cameras", "free_poses",
            "max_row_span", "band_solver", "band_top_rows", "band_separator_rows", "band_bottom_rows"]
    return dict(zip(keys[:n], out[:n].tolist()))


def plan_digest(K, point_ptr, obs_cam, obs_uv, n_poses: int, n_fixed: int = 2, target_segments: int = 512) -> int:
    """Host-only 64-bit digest of the whole static plan (``vo_ba_plan_digest``): pins the
    planner's output, and with it every kernel's summation order."""
    point_ptr = np.ascontiguousarray(point_ptr, dtype=np.int32)
    obs_cam = np.ascontiguousarray(obs_cam, dtype=np.int32)
    obs_uv = np.ascontiguousarray(obs_uv, dtype=np.float32).reshape(-1, 2)
    prob = _problem_struct(K, point_ptr, obs_cam, obs_uv, n_poses, n_fixed, 0.0)
    d = C.c_uint64(0)
    check(_lib.load().vo_ba_plan_digest(C.byref(prob), int(target_segments), C.byref(d)), "vo_ba_plan_digest")
    return int(d.value)


def plan_slide_digest(K, prev, cur, seg_obs: int, seg_chunks: int = 1) -> tuple:
    """Host-only (test): ``(digest, reused_chunks)`` of the plan of window ``cur`` packed for
    ``seg_obs`` observations per segment (1: the one-wave K1's plan of ``seg_chunks`` chunks per
    segment), built from scratch (``prev`` None) or by taking over
    the unchanged first-camera groups of ``prev``'s plan, as ``vo_ba_setup`` does on a slide
    (``vo_ba_testing_plan_slide``).  Windows: ``(point_ptr, obs_cam, obs_uv, n_poses, n_fixed)``."""
    keep = []

    def struct(w):
        pp, oc, uv, n, nf = w
        a = (np.ascontiguousarray(pp, dtype=np.int32), np.ascontiguousarray(oc, dtype=np.int32),
             np.ascontiguousarray(uv, dtype=np.float32).reshape(-1, 2))
        keep.append(a)
        return _problem_struct(K, a[0], a[1], a[2], n, nf, 0.0)

    pc = struct(cur)
    pv = struct(prev) if prev is not None else None
    d = C.c_uint64(0)
    r = C.c_int64(0)
    check(_lib.load().vo_ba_testing_plan_slide(C.byref(pv) if pv is not None else None, C.byref(pc), int(seg_obs),
                                               int(seg_chunks), C.byref(d), C.byref(r)), "vo_ba_testing_plan_slide")
    return int(d.value), int(r.value)


class BASession:
    """A BA problem resident on one device (structure + state in HBM).

    Thin wrapper of the ``vo_ba_*`` C-ABI: ``setup`` uploads the structure and
    builds the static plan, ``set_state``/``get_state`` move poses and points,
    ``run`` performs GN iterations on the device-resident state.
    """

    def __init__(self, K, point_ptr, obs_cam, obs_uv, n_poses: int, n_fixed: int = 2,
                 lam: float = 0.0, ctx: _lib.Context | None = None):
        self.ctx = ctx or _lib.context()
        self.point_ptr = np.ascontiguousarray(point_ptr, dtype=np.int32)
        self.obs_cam = np.ascontiguousarray(obs_cam, dtype=np.int32)
        self.obs_uv = np.ascontiguousarray(obs_uv, dtype=np.float32).reshape(-1, 2)
        self.n_poses = int(n_poses)
        self.n_points = self.point_ptr.size - 1
        self.n_fixed = int(n_fixed)
        prob = _problem_struct(K, self.point_ptr, self.obs_cam, self.obs_uv, self.n_poses,
                               self.n_fixed, lam)
        self._prob = prob
        sid = C.c_uint64(0)
        check(self.ctx.lib.vo_ba_setup(self.ctx.handle, C.byref(prob), C.byref(sid)), "vo_ba_setup")
        # the problem's id on this context: a later setup on the same context (another
        # session) makes every call below fail with VO_ERR_STATE instead of misreading
        self.session = int(sid.value)

    def set_state(self, poses_cw: np.ndarray, points: np.ndarray) -> None:
        rt = np.ascontiguousarray(poses_to_rt(poses_cw))
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
        if rt.shape[0] != self.n_poses or pts.shape[0] != self.n_points:
            raise ValueError("state shape does not match the problem")
        check(self.ctx.lib.vo_ba_set_state(self.ctx.handle, self.session, ptr(rt, C.c_double),
                                           ptr(pts, C.c_double)),
              "vo_ba_set_state")

    def get_state(self):
        rt = np.empty((self.n_poses, 12))
        pts = np.empty((self.n_points, 3))
        check(self.ctx.lib.vo_ba_get_state(self.ctx.handle, self.session, ptr(rt, C.c_double),
                                           ptr(pts, C.c_double)),
              "vo_ba_get_state")
        return rt_to_poses(rt), pts

    def run(self, iters: int):
        """``iters`` GN iterations; returns (status_code, costs[iters+1])."""
        costs = np.empty(iters + 1)
        rc = self.ctx.lib.vo_ba_run(self.ctx.handle, self.session, int(iters), ptr(costs, C.c_double))
        if rc not in (_lib.VO_OK, _lib.VO_ERR_NOT_SPD):
            check(rc, "vo_ba_run")
        return rc, costs

    def run_async(self, iters: int) -> None:
        check(self.ctx.lib.vo_ba_run_async(self.ctx.handle, self.session, int(iters)), "vo_ba_run_async")

    def synchronize(self) -> None:
        check(self.ctx.lib.vo_synchronize(self.ctx.handle), "vo_synchronize")

    def gn_step(self):
        """One GN step exporting (rc, S dense, b, dc, cost-before-step)."""
        F = self.n_poses - self.n_fixed
        S = np.empty((6 * F, 6 * F))
        b = np.empty(6 * F)
        dc = np.empty(6 * F)
        cost = np.empty(1)
        rc = self.ctx.lib.vo_ba_gn_step(self.ctx.handle, self.session, ptr(S, C.c_double), ptr(b, C.c_double),
                                           ptr(dc, C.c_double), ptr(cost, C.c_double))
        if rc not in (_lib.VO_OK, _lib.VO_ERR_NOT_SPD):
            check(rc, "vo_ba_gn_step")
        return rc, S, b, dc, float(cost[0])

    SETUP_SECTIONS = ["sync", "order", "segments", "lists_images", "plan_rest", "plan_checks", "images",
                      "profile", "uploads", "buffers", "band_tables", "attributes"]

    def plan_stats(self) -> dict:
        out = np.zeros(24, dtype=np.int64)
        n = check(self.ctx.lib.vo_ba_plan_stats(self.ctx.handle, ptr(out, C.c_int64), 24), "stats")
        keys = ["chunks", "segments", "slab_blocks", "reduced_blocks", "profile_blocks",
                "track_entries", "algorithmic_bytes_per_iter", "band_solver", "reused_groups",
                "reused_chunks", "seg_obs"]
        st = dict(zip(keys[:n], out[:n].tolist()))
        if n > 11:  # the last setup's host sections (ns)
            st["setup_us"] = {k: round(v / 1e3, 1) for k, v in zip(self.SETUP_SECTIONS, out[11:23].tolist())}
        if n > 23:  # the banded K3's layout
            st["band_mode"] = ["none", "full", "ring", "split"][int(out[23])]
        return st


class SlidingWindowBA:
    """``SlidingWindowBA(K, cfg).optimize(window) -> BAResult``.

    ``cfg`` may be a ``VOConfig`` carrying ``ba_iters`` / ``ba_lambda``; any
    missing knob takes the keyword default.  Degenerate windows come back with
    ``status != "ok"`` instead of raising, so ``process_frame`` keeps the
    reference's print-and-continue failure style (``vo.py:240-245``).
    """

    def __init__(self, K, cfg=None, *, iters: int = 10, lam: float = 0.0, device: int | None = None):
        self.K = np.asarray(K, dtype=np.float64)
        self.iters = int(getattr(cfg, "ba_iters", iters))
        self.lam = float(getattr(cfg, "ba_lambda", lam))
        self.device = device

    def reserve(self, n_poses: int, n_points: int, obs_per_point: float = 5.0, n_fixed: int = 2) -> None:
        """Pre-size the device context for windows of up to about ``n_poses`` keyframes and
        ``n_points`` landmarks (``vo_ba_reserve``), once, before the drive's first keyframe:
        the first :meth:`optimize` then allocates nothing and faults in no page."""
        n_points = max(1, int(n_points))
        n_obs = max(2 * n_points, int(round(obs_per_point * n_points)))
        _lib.ba_reserve(_lib.context(self.device), max(2, int(n_poses)), n_points, n_obs, int(n_fixed))

    def optimize(self, window: BAWindow) -> BAResult:
        poses = np.asarray(window.poses_cw, dtype=np.float64)
        pts = np.asarray(window.points, dtype=np.float64).reshape(-1, 3)
        n_fixed = min(int(window.n_fixed), poses.shape[0])
        if poses.shape[0] == 0 or pts.shape[0] == 0 or np.asarray(window.obs_cam).size == 0 \
                or poses.shape[0] <= n_fixed:
            return BAResult(poses.copy(), pts.copy(), np.zeros(0), "skipped", "empty window")
        point_ptr, obs_cam, obs_uv = group_window(pts.shape[0], window)
        ctx = _lib.context(self.device)
        try:
            sess = BASession(self.K, point_ptr, obs_cam, obs_uv, poses.shape[0], n_fixed, self.lam, ctx)
            sess.set_state(poses, pts)
            rc, costs = sess.run(self.iters)
            P, X = sess.get_state()
        except VoError as e:
            if e.code == _lib.VO_ERR_ARG:
                return BAResult(poses.copy(), pts.copy(), np.zeros(0), "skipped", str(e))
            raise
        status = "ok" if rc == _lib.VO_OK else "not_spd"
        return BAResult(P, X, costs, status)
