"""CPU oracle for the sliding-window bundle-adjustment Gauss-Newton step.

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` -- never by the product path.

PARITY STATUS: the reference repository contains **no bundle adjustment**
(``pyceres``/``pycolmap`` are declared in ``pyproject.toml:11-12`` but never
imported).  There is therefore no reference output to pin
against; parity with the reference is *unpinned* for BA.  This restatement
is instead pinned by (tests/test_oracle_ba.py):

* finite-difference checks of its Jacobians,
* equality of the Schur-complement step with a direct solve of the full
  (cameras + points) normal equations,
* convergence to the same optimum as ``scipy.optimize.least_squares`` on
  the same residual, and to ground truth on noise-free problems.

What it follows from the reference:

* the projection model of ``src/modules/frontend.py:128-140``: pinhole
  ``K`` with no distortion (``cv2.projectPoints(pts3d, R2, t2, K, None)``),
* the pose convention of ``src/modules/vo.py:98-101,260-261``: cameras are
  stored as ``T_cw`` (world -> camera) when projecting.

Build-defined problem:

* residual ``r = pi(K (R_cw X + t_cw)) - uv``, cost ``sum ||r||^2``,
* left se(3) increment ``T_cw <- exp(delta^) T_cw``, ``delta = (rho, phi)``,
* the first ``n_fixed`` poses are held fixed (gauge),
* optional Levenberg damping ``lambda * I`` on every camera and point block,
* a landmark whose 3x3 block fails the pivot test of :func:`point_block_valid`
  is frozen for that iteration (no contribution to S/b, zero update).
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import scipy.linalg

PIVOT_REL_EPS = 1e-12  # relative pivot threshold of the 3x3 point blocks
EXP_TAYLOR_THETA = 1e-4  # below this rotation angle the exp map uses its series


def skew(v: np.ndarray) -> np.ndarray:
    """Batched cross-product matrix (...,3) -> (...,3,3)."""
    k = np.zeros(v.shape[:-1] + (3, 3))
    k[..., 0, 1], k[..., 0, 2] = -v[..., 2], v[..., 1]
    k[..., 1, 0], k[..., 1, 2] = v[..., 2], -v[..., 0]
    k[..., 2, 0], k[..., 2, 1] = -v[..., 1], v[..., 0]
    return k


def se3_exp(delta: np.ndarray):
    """exp of se(3) twists (...,6) = (rho, phi) -> (R (...,3,3), t (...,3))."""
    rho, phi = delta[..., :3], delta[..., 3:]
    th2 = np.sum(phi * phi, axis=-1)
    th = np.sqrt(th2)
    small = th < EXP_TAYLOR_THETA
    ths = np.where(small, 1.0, th)
    A = np.where(small, 1.0 - th2 / 6.0, np.sin(ths) / ths)
    B = np.where(small, 0.5 - th2 / 24.0, (1.0 - np.cos(ths)) / ths**2)
    C = np.where(small, 1.0 / 6.0 - th2 / 120.0, (ths - np.sin(ths)) / ths**3)
    P = skew(phi)
    P2 = P @ P
    eye = np.broadcast_to(np.eye(3), P.shape)
    R = eye + A[..., None, None] * P + B[..., None, None] * P2
    V = eye + B[..., None, None] * P + C[..., None, None] * P2
    return R, np.einsum("...ij,...j->...i", V, rho)


@dataclass
class BAState:
    R: np.ndarray  # (N,3,3) R_cw
    t: np.ndarray  # (N,3) t_cw
    X: np.ndarray  # (L,3)

    @staticmethod
    def from_poses(poses_cw: np.ndarray, points: np.ndarray) -> "BAState":
        return BAState(
            poses_cw[:, :3, :3].copy(), poses_cw[:, :3, 3].copy(), points.astype(np.float64).copy()
        )

    def poses_cw(self) -> np.ndarray:
        T = np.tile(np.eye(4), (self.R.shape[0], 1, 1))
        T[:, :3, :3] = self.R
        T[:, :3, 3] = self.t
        return T

    def copy(self) -> "BAState":
        return BAState(self.R.copy(), self.t.copy(), self.X.copy())


@dataclass
class BAStructure:
    K: np.ndarray
    point_ptr: np.ndarray
    obs_cam: np.ndarray
    obs_uv: np.ndarray
    n_fixed: int
    n_poses: int
    obs_pt: np.ndarray = field(init=False)

    def __post_init__(self):
        counts = np.diff(self.point_ptr)
        self.obs_pt = np.repeat(np.arange(counts.size), counts)

    @property
    def n_points(self) -> int:
        return self.point_ptr.size - 1

    @property
    def n_free(self) -> int:
        return max(self.n_poses - self.n_fixed, 0)


def residuals(st: BAState, s: BAStructure):
    """Reprojection residuals r (M,2) and camera-frame points p_c (M,3)."""
    fx, fy, cx, cy = s.K[0, 0], s.K[1, 1], s.K[0, 2], s.K[1, 2]
    pc = np.einsum("mij,mj->mi", st.R[s.obs_cam], st.X[s.obs_pt]) + st.t[s.obs_cam]
    u = fx * pc[:, 0] / pc[:, 2] + cx
    v = fy * pc[:, 1] / pc[:, 2] + cy
    uv = s.obs_uv.astype(np.float64)
    return np.stack([u - uv[:, 0], v - uv[:, 1]], -1), pc


def jacobians(st: BAState, s: BAStructure, pc: np.ndarray):
    """J_pose (M,2,6) w.r.t. the left twist (rho, phi); J_point (M,2,3)."""
    fx, fy = s.K[0, 0], s.K[1, 1]
    iz = 1.0 / pc[:, 2]
    Jproj = np.zeros((pc.shape[0], 2, 3))
    Jproj[:, 0, 0] = fx * iz
    Jproj[:, 0, 2] = -fx * pc[:, 0] * iz * iz
    Jproj[:, 1, 1] = fy * iz
    Jproj[:, 1, 2] = -fy * pc[:, 1] * iz * iz
    dpc = np.concatenate([np.broadcast_to(np.eye(3), pc.shape[:1] + (3, 3)), -skew(pc)], -1)
    return Jproj @ dpc, Jproj @ st.R[s.obs_cam]


def point_block_valid(V: np.ndarray) -> np.ndarray:
    """Pivot test of the 3x3 Cholesky of each point block V (L,3,3).

    Same operation order as the HIP kernel (DESIGN.md §BA "frozen landmarks").
    """
    eps = PIVOT_REL_EPS * (V[:, 0, 0] + V[:, 1, 1] + V[:, 2, 2])
    v00 = V[:, 0, 0]
    ok = v00 > eps
    l00 = np.sqrt(np.where(ok, v00, 1.0))
    l10 = V[:, 0, 1] / l00
    l20 = V[:, 0, 2] / l00
    d1 = V[:, 1, 1] - l10 * l10
    ok &= d1 > eps
    l11 = np.sqrt(np.where(ok, d1, 1.0))
    l21 = (V[:, 1, 2] - l20 * l10) / l11
    d2 = V[:, 2, 2] - l20 * l20 - l21 * l21
    ok &= d2 > eps
    return ok


@dataclass
class GNSystem:
    S: np.ndarray  # (6N',6N') reduced camera matrix
    b: np.ndarray  # (6N',)
    cost: float
    Vinv: np.ndarray  # (L,3,3) (zero for frozen landmarks)
    g_p: np.ndarray  # (L,3)
    W: np.ndarray  # (M,6,3) J_pose^T J_point per observation
    valid: np.ndarray  # (L,) bool
    r: np.ndarray  # (M,2)


def build_system(st: BAState, s: BAStructure, lam: float = 0.0) -> GNSystem:
    """Linearise and eliminate the points: S = U - W V^-1 W^T, b = -g_c + W V^-1 g_p."""
    r, pc = residuals(st, s)
    Jc, Jp = jacobians(st, s, pc)
    M, L, nf, NF = s.obs_cam.size, s.n_points, s.n_fixed, s.n_free
    free = s.obs_cam >= nf
    fidx = s.obs_cam - nf

    V = np.zeros((L, 3, 3))
    np.add.at(V, s.obs_pt, np.einsum("mki,mkj->mij", Jp, Jp))
    V += lam * np.eye(3)
    g_p = np.zeros((L, 3))
    np.add.at(g_p, s.obs_pt, np.einsum("mki,mk->mi", Jp, r))
    valid = point_block_valid(V)
    Vinv = np.zeros_like(V)
    Vinv[valid] = np.linalg.inv(V[valid])

    n = 6 * NF
    S = np.zeros((n, n))
    b = np.zeros(n)
    U = np.einsum("mki,mkj->mij", Jc, Jc)
    gc = np.einsum("mki,mk->mi", Jc, r)
    W = np.einsum("mki,mkj->mij", Jc, Jp)
    of = np.nonzero(free & valid[s.obs_pt])[0]  # frozen landmarks leave the system
    if of.size:
        f6 = 6 * fidx[of]
        rows = f6[:, None, None] + np.arange(6)[None, :, None]
        cols = f6[:, None, None] + np.arange(6)[None, None, :]
        S += np.bincount((rows * n + cols).ravel(), weights=U[of].ravel(),
                         minlength=n * n).reshape(n, n)
        b -= np.bincount((f6[:, None] + np.arange(6)).ravel(), weights=gc[of].ravel(),
                         minlength=n)
    if NF:
        S += lam * np.eye(n)

    # Schur correction: every ordered pair (o, o') of free observations of a
    # valid landmark adds -W_o V^-1 W_o'^T at block (cam o, cam o').
    use = free & valid[s.obs_pt]
    counts = np.bincount(s.obs_pt[use], minlength=L)
    starts = np.zeros(L + 1, dtype=np.int64)
    starts[1:] = np.cumsum(counts)
    order = np.nonzero(use)[0]  # already grouped by point (CSR order)
    Y = np.einsum("mij,mjk->mik", W, Vinv[s.obs_pt])  # W V^-1
    np.add.at(b, (6 * fidx[order, None] + np.arange(6)).ravel(),
              np.einsum("mij,mj->mi", Y[order], g_p[s.obs_pt[order]]).ravel())
    pa, pb = [], []
    for k in np.unique(counts[counts > 0]):
        pts_k = np.nonzero(counts == k)[0]
        base = starts[pts_k]
        ii, jj = np.meshgrid(np.arange(k), np.arange(k), indexing="ij")
        pa.append((base[:, None] + ii.ravel()[None, :]).ravel())
        pb.append((base[:, None] + jj.ravel()[None, :]).ravel())
    if pa:
        oa = order[np.concatenate(pa)]
        ob = order[np.concatenate(pb)]
        blocks = np.einsum("pij,pkj->pik", Y[oa], W[ob])  # (P,6,6)
        rows = 6 * fidx[oa][:, None, None] + np.arange(6)[None, :, None]
        cols = 6 * fidx[ob][:, None, None] + np.arange(6)[None, None, :]
        flat = (rows * n + cols).ravel()
        S -= np.bincount(flat, weights=blocks.ravel(), minlength=n * n).reshape(n, n)
    return GNSystem(S, b, float(np.sum(r * r)), Vinv, g_p, W, valid, r)


def solve_reduced(S: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Dense Cholesky solve of S dc = b (raises LinAlgError if not SPD)."""
    if S.size == 0:
        return np.zeros(0)
    c = scipy.linalg.cho_factor(S, lower=True, check_finite=True)
    return scipy.linalg.cho_solve(c, b)


def back_substitute(sys_: GNSystem, s: BAStructure, dc: np.ndarray) -> np.ndarray:
    """dp = V^-1 (-g_p - sum_o W_o^T dc_cam(o)) per landmark (zero if frozen)."""
    nf = s.n_fixed
    acc = -sys_.g_p.copy()
    free = s.obs_cam >= nf
    dcam = np.zeros((s.obs_cam.size, 6))
    dcam[free] = dc.reshape(-1, 6)[s.obs_cam[free] - nf]
    np.add.at(acc, s.obs_pt, -np.einsum("mij,mi->mj", sys_.W, dcam))
    dp = np.einsum("lij,lj->li", sys_.Vinv, acc)
    dp[~sys_.valid] = 0.0
    return dp


def apply_update(st: BAState, s: BAStructure, dc: np.ndarray, dp: np.ndarray) -> BAState:
    out = st.copy()
    nf = s.n_fixed
    if dc.size:
        Rd, td = se3_exp(dc.reshape(-1, 6))
        out.R[nf:] = Rd @ st.R[nf:]
        out.t[nf:] = np.einsum("nij,nj->ni", Rd, st.t[nf:]) + td
    out.X = st.X + dp
    return out


@dataclass
class GNStep:
    system: GNSystem
    dc: np.ndarray
    dp: np.ndarray
    state: BAState  # state after the update


def gn_step(st: BAState, s: BAStructure, lam: float = 0.0) -> GNStep:
    sys_ = build_system(st, s, lam)
    dc = solve_reduced(sys_.S, sys_.b)
    dp = back_substitute(sys_, s, dc)
    return GNStep(sys_, dc, dp, apply_update(st, s, dc, dp))


def cost(st: BAState, s: BAStructure) -> float:
    r, _ = residuals(st, s)
    return float(np.sum(r * r))


def solve(st: BAState, s: BAStructure, iters: int, lam: float = 0.0):
    """Pure GN: ``iters`` steps, all accepted; returns (state, costs[iters+1])."""
    costs = []
    for _ in range(iters):
        step = gn_step(st, s, lam)
        costs.append(step.system.cost)
        st = step.state
    costs.append(cost(st, s))
    return st, np.array(costs)


def full_system_step(st: BAState, s: BAStructure, lam: float = 0.0):
    """Reference step by solving the FULL normal equations (no Schur); tiny problems only."""
    r, pc = residuals(st, s)
    Jc, Jp = jacobians(st, s, pc)
    nf, NF, L = s.n_fixed, s.n_free, s.n_points
    n = 6 * NF + 3 * L
    J = np.zeros((2 * r.shape[0], n))
    for o in range(r.shape[0]):
        c, p = s.obs_cam[o], s.obs_pt[o]
        if c >= nf:
            J[2 * o : 2 * o + 2, 6 * (c - nf) : 6 * (c - nf) + 6] = Jc[o]
        J[2 * o : 2 * o + 2, 6 * NF + 3 * p : 6 * NF + 3 * p + 3] = Jp[o]
    H = J.T @ J + lam * np.eye(n)
    g = J.T @ r.ravel()
    d = np.linalg.solve(H, -g)
    return d[: 6 * NF], d[6 * NF :].reshape(L, 3)
