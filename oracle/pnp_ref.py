"""CPU oracle for PnP-RANSAC -- TEST INFRASTRUCTURE ONLY.

Imported by ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py``; never by the product path.

Restates the tracking step of the reference, ``cv2.solvePnPRansac(pnp_3d, pnp_2d, K,
None, reprojectionError=cfg.pnp_reproj_err)`` (``src/modules/vo.py:135-141``; defaults
``iterationsCount=100``, ``confidence=0.99``, ``flags=SOLVEPNP_ITERATIVE``), with the
arithmetic of OpenCV 4.12 (``opencv-python==4.12.0.88``, ``uv.lock:742-743``; OpenCV is
absent from this image, so this follows its published source, module by module):

* ``solvePnPRansac`` (calib3d/solvepnp.cpp): the minimal solver is EPnP on
  ``model_points = 5`` correspondences; with exactly 5 points EPnP runs once on all of
  them; fewer than 5 is a failure here (OpenCV would switch to P3P at 4).
* ``RANSACPointSetRegistrator::run`` / ``getSubset`` (calib3d/ptsetreg.cpp): a
  ``cv::RNG((uint64)-1)`` multiply-with-carry stream, subsets of 5 distinct indices
  drawn with ``rng.uniform(0, count)`` (redrawn on a repeat), a model replaces the best
  one only if its inlier count is ``> max(best, model_points - 1)``, and
  ``niters = RANSACUpdateNumIters(confidence, (count - good) / count, 5, niters)``.
* ``PnPRansacCallback::computeError``: ``projectPoints`` of the float32 object points
  with the model's ``rvec``/``tvec`` into float32, error ``dx*dx + dy*dy`` in float32,
  inlier iff ``err <= (float)(thr*thr)``.
* ``epnp::compute_pose`` (calib3d/epnp.cpp): control points from the centroid and PCA,
  barycentric coordinates, the 2n x 12 matrix M, the four right singular vectors of
  ``M^T M`` with the smallest singular values, the three beta approximations each
  refined by 5 Gauss-Newton steps (Householder ``qr_solve``), and the pose with the
  smallest mean reprojection error.  Every SVD is ``JacobiSVDImpl_`` (core/lapack.cpp):
  one-sided Jacobi on the rows of A^T with ``eps = 10 DBL_EPSILON``, at most
  ``max(m, 30)`` sweeps, singular values sorted descending by selection sort.
* ``Rodrigues`` (calib3d/calibration.cpp) in both directions.

Build-defined, documented divergences (no OpenCV to pin against):

* ``hypot(p, beta)`` in the Jacobi rotation is ``sqrt(p*p + beta*beta)``: only correctly
  rounded operations, so the GPU reproduces it bit for bit (libm hypot differs in the last
  ulp between libraries).  This matters: with 5 points ``M^T M`` has a two-dimensional
  null space whose computed basis is decided by rounding, and one ulp in one rotation
  changes individual EPnP hypotheses completely (tests/test_pnp_host_math.py).
* ``cvSolve(L, rho, CV_SVD)`` (least squares on 6 x {3,4,5} systems) uses the same
  Householder ``qr_solve`` as the Gauss-Newton steps: the same least-squares solution
  for full column rank.
* The image points enter EPnP as pixels; OpenCV round-trips them through
  ``undistortPoints`` with zero distortion, which is the identity up to float32 rounding.
* A subset whose ``M^T M`` has a singular value ``<= DBL_MIN`` (degenerate: repeated
  points) yields no model; OpenCV would complete the basis with random vectors.
* The final refinement on the RANSAC inliers is a Levenberg-Marquardt on the left
  se(3) increment of the RANSAC pose, with CvLevMarq's schedule (lambda = 10^-3
  initially, /10 on an accepted step, x10 and retry on a rejected one, damping
  ``diag(J^T J) (1 + lambda)``, at most 20 accepted steps, stop once
  ``||delta|| <= FLT_EPSILON (1 + ||t||)``).  OpenCV restarts SOLVEPNP_ITERATIVE from
  its own DLT initialisation; both converge to the least-squares pose.
* The returned inliers are those of the best RANSAC model (as OpenCV does).

Parity pin: the reference has no tests or fixtures and OpenCV cannot run here
(SURVEY.md §8c), so against OpenCV this restatement is **parity unpinned**.  It is
pinned by known answers (``tests/test_oracle_pnp.py``): the RNG stream against its
closed form, EPnP's exact recovery of noise-free poses, the SVD against numpy, planted
outliers rejected, and the refined pose at the least-squares optimum (zero gradient).
"""

from __future__ import annotations

import math

import numpy as np

MASK64 = (1 << 64) - 1
CV_RNG_COEFF = 4164903690
DBL_EPSILON = float(np.finfo(np.float64).eps)
DBL_MIN = float(np.finfo(np.float64).tiny)
FLT_EPSILON = float(np.finfo(np.float32).eps)
MODEL_POINTS = 5
LM_MAX_ITERS = 20
LM_LAMBDA_LG10_INIT = -3


# --------------------------------------------------------------------------- RNG
class CvRNG:
    """``cv::RNG`` (core/rand.cpp): ``state = (uint32)state * 4164903690 + (state >> 32)``."""

    def __init__(self, state: int = MASK64):
        self.state = state if state else 0xFFFFFFFF

    def next(self) -> int:
        s = self.state
        self.state = ((s & 0xFFFFFFFF) * CV_RNG_COEFF + (s >> 32)) & MASK64
        return self.state & 0xFFFFFFFF

    def uniform(self, a: int, b: int) -> int:
        return a if a == b else self.next() % (b - a) + a


def ransac_subsets(count: int, iters: int, model_points: int = MODEL_POINTS) -> np.ndarray:
    """The subsets ``getSubset`` draws for iterations 0..iters-1 (ptsetreg.cpp) -> (iters, 5).

    The draws do not depend on the models, so all of them can be made up front."""
    rng = CvRNG()
    out = np.empty((iters, model_points), dtype=np.int32)
    for it in range(iters):
        idx: list[int] = []
        for _ in range(model_points):
            j = rng.uniform(0, count)
            while j in idx:
                j = rng.uniform(0, count)
            idx.append(j)
        out[it] = idx
    return out


def update_num_iters(p: float, ep: float, model_points: int, max_iters: int) -> int:
    """``RANSACUpdateNumIters`` (ptsetreg.cpp)."""
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, DBL_MIN)
    denom = 1.0 - math.pow(1.0 - ep, model_points)
    if denom < DBL_MIN:
        return 0
    num = math.log(num)
    denom = math.log(denom)
    if denom >= 0 or -num >= max_iters * (-denom):
        return max_iters
    return int(np.rint(num / denom))


# --------------------------------------------------------------------------- SVD
def _seqsum(x: np.ndarray) -> np.ndarray:
    """Left-to-right sum over the last axis (the loop order of the C code)."""
    return np.cumsum(x, axis=-1)[..., -1]


def jacobi_svd(At: np.ndarray, want_vt: bool = True):
    """``JacobiSVDImpl_`` (core/lapack.cpp) on a batch of row sets ``At`` (B, n, m).

    Returns (W (B, n) descending, U^T rows (B, n, m) = the rotated rows scaled by 1/W,
    Vt (B, n, n), degenerate (B,) bool -- some W <= DBL_MIN)."""
    A = np.array(At, dtype=np.float64, copy=True)
    B, n, m = A.shape
    eps = DBL_EPSILON * 10
    W = _seqsum(A * A)
    Vt = np.broadcast_to(np.eye(n), (B, n, n)).copy()
    for _ in range(max(m, 30)):
        changed = np.zeros(B, dtype=bool)
        for i in range(n - 1):
            for j in range(i + 1, n):
                Ai, Aj = A[:, i], A[:, j]
                a, b = W[:, i], W[:, j]
                p = _seqsum(Ai * Aj)
                rot = ~(np.abs(p) <= eps * np.sqrt(a * b))
                if not rot.any():
                    continue
                with np.errstate(divide="ignore", invalid="ignore"):
                    p = p * 2
                    beta = a - b
                    gamma = np.sqrt(p * p + beta * beta)  # hypot from correctly rounded ops only
                    neg = beta < 0
                    delta = (gamma - beta) * 0.5
                    s_n = np.sqrt(delta / gamma)
                    c_n = p / (gamma * s_n * 2)
                    c_p = np.sqrt((gamma + beta) / (gamma * 2))
                    s_p = p / (gamma * c_p * 2)
                c = np.where(neg, c_n, c_p)[:, None]
                s = np.where(neg, s_n, s_p)[:, None]
                t0 = c * Ai + s * Aj
                t1 = -s * Ai + c * Aj
                r = rot[:, None]
                A[:, i] = np.where(r, t0, Ai)
                A[:, j] = np.where(r, t1, Aj)
                W[:, i] = np.where(rot, _seqsum(t0 * t0), a)
                W[:, j] = np.where(rot, _seqsum(t1 * t1), b)
                Vi, Vj = Vt[:, i].copy(), Vt[:, j].copy()
                Vt[:, i] = np.where(r, c * Vi + s * Vj, Vi)
                Vt[:, j] = np.where(r, -s * Vi + c * Vj, Vj)
                changed |= rot
        if not changed.any():
            break
    W = np.sqrt(_seqsum(A * A))
    ar = np.arange(B)
    for i in range(n - 1):  # selection sort, descending (first maximum wins)
        jsel = np.full(B, i)
        for k in range(i + 1, n):
            jsel = np.where(W[ar, jsel] < W[:, k], k, jsel)
        sw = jsel != i
        if sw.any():
            b_ = ar[sw]
            jj = jsel[sw]
            W[b_, i], W[b_, jj] = W[b_, jj], W[b_, i].copy()
            Ai, Aj = A[b_, i].copy(), A[b_, jj].copy()
            A[b_, i], A[b_, jj] = Aj, Ai
            Vi, Vj = Vt[b_, i].copy(), Vt[b_, jj].copy()
            Vt[b_, i], Vt[b_, jj] = Vj, Vi
    degenerate = np.any(W <= DBL_MIN, axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        s = 1.0 / W
    U = A * s[:, :, None]
    return W, U, Vt, degenerate


def svd_of(src: np.ndarray):
    """``cv::SVD::compute`` of square matrices (B, n, n): JacobiSVD on A^T's rows.
    Returns (w, U (columns = left vectors), Vt, degenerate)."""
    W, Ut, Vt, deg = jacobi_svd(np.swapaxes(src, -1, -2))
    return W, np.swapaxes(Ut, -1, -2), Vt, deg


# --------------------------------------------------------------------------- EPnP
def qr_solve(A: np.ndarray, b: np.ndarray, X: np.ndarray) -> np.ndarray:
    """``epnp::qr_solve``: Householder least squares, batched (B, nr, nc), (B, nr).

    Rows where a column is all zero keep their previous ``X`` (the C code returns early)."""
    A = A.copy()
    b = b.copy()
    B, nr, nc = A.shape
    A1 = np.zeros((B, nc))
    A2 = np.zeros((B, nc))
    ok = np.ones(B, dtype=bool)
    for k in range(nc):
        eta = np.abs(A[:, k, k])
        for i in range(k + 1, nr):
            eta = np.maximum(eta, np.abs(A[:, i, k]))
        ok &= eta != 0
        with np.errstate(divide="ignore", invalid="ignore"):
            inv_eta = 1.0 / eta
            sum2 = np.zeros(B)
            for i in range(k, nr):
                A[:, i, k] = A[:, i, k] * inv_eta
                sum2 = sum2 + A[:, i, k] * A[:, i, k]
            sigma = np.sqrt(sum2)
            sigma = np.where(A[:, k, k] < 0, -sigma, sigma)
            A[:, k, k] = A[:, k, k] + sigma
            A1[:, k] = sigma * A[:, k, k]
            A2[:, k] = -eta * sigma
            for j in range(k + 1, nc):
                s = np.zeros(B)
                for i in range(k, nr):
                    s = s + A[:, i, k] * A[:, i, j]
                tau = s / A1[:, k]
                for i in range(k, nr):
                    A[:, i, j] = A[:, i, j] - tau * A[:, i, k]
    with np.errstate(divide="ignore", invalid="ignore"):
        for j in range(nc):
            tau = np.zeros(B)
            for i in range(j, nr):
                tau = tau + A[:, i, j] * b[:, i]
            tau = tau / A1[:, j]
            for i in range(j, nr):
                b[:, i] = b[:, i] - tau * A[:, i, j]
        Xn = np.empty((B, nc))
        Xn[:, nc - 1] = b[:, nc - 1] / A2[:, nc - 1]
        for i in range(nc - 2, -1, -1):
            s = np.zeros(B)
            for j in range(i + 1, nc):
                s = s + A[:, i, j] * Xn[:, j]
            Xn[:, i] = (b[:, i] - s) / A2[:, i]
    return np.where(ok[:, None], Xn, X)


_PAIRS = ((0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3))


def _dot3(a, b):
    return a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1] + a[..., 2] * b[..., 2]


def epnp(pws: np.ndarray, us: np.ndarray, K: np.ndarray):
    """``epnp::compute_pose`` batched: pws (B, n, 3), us (B, n, 2) -> (R (B,3,3), t (B,3), ok (B,))."""
    pws = np.asarray(pws, dtype=np.float64)
    us = np.asarray(us, dtype=np.float64)
    B, n, _ = pws.shape
    fu, fv, uc, vc = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
    # choose_control_points
    c0 = np.zeros((B, 3))
    for i in range(n):
        c0 = c0 + pws[:, i]
    c0 = c0 / n
    PW0 = pws - c0[:, None, :]
    PtP = np.zeros((B, 3, 3))
    for i in range(n):
        PtP = PtP + PW0[:, i, :, None] * PW0[:, i, None, :]
    dc, uc_t_cols, _, deg0 = svd_of(PtP)
    uct = np.swapaxes(uc_t_cols, -1, -2)  # rows = left singular vectors (CV_SVD_U_T)
    cws = np.empty((B, 4, 3))
    cws[:, 0] = c0
    for i in range(1, 4):
        k = np.sqrt(dc[:, i - 1] / n)
        cws[:, i] = c0 + k[:, None] * uct[:, i - 1]
    # compute_barycentric_coordinates (cvInvert(CC, CV_SVD))
    CC = np.empty((B, 3, 3))
    for i in range(3):
        for j in range(1, 4):
            CC[:, i, j - 1] = cws[:, j, i] - cws[:, 0, i]
    w, U, Vt, deg1 = svd_of(CC)
    with np.errstate(divide="ignore"):
        CCi = np.einsum("bki,bk,bjk->bij", Vt, 1.0 / w, U)
    d = pws - cws[:, None, 0, :]
    alphas = np.empty((B, n, 4))
    for j in range(3):
        alphas[:, :, 1 + j] = CCi[:, j, 0, None] * d[:, :, 0] + CCi[:, j, 1, None] * d[:, :, 1] + \
            CCi[:, j, 2, None] * d[:, :, 2]
    alphas[:, :, 0] = 1.0 - alphas[:, :, 1] - alphas[:, :, 2] - alphas[:, :, 3]
    # fill_M
    M = np.zeros((B, 2 * n, 12))
    for i in range(n):
        for c in range(4):
            a = alphas[:, i, c]
            M[:, 2 * i, 3 * c] = a * fu
            M[:, 2 * i, 3 * c + 2] = a * (uc - us[:, i, 0])
            M[:, 2 * i + 1, 3 * c + 1] = a * fv
            M[:, 2 * i + 1, 3 * c + 2] = a * (vc - us[:, i, 1])
    MtM = np.zeros((B, 12, 12))
    for r in range(2 * n):
        MtM = MtM + M[:, r, :, None] * M[:, r, None, :]
    _, ut_cols, _, deg2 = svd_of(MtM)
    ut = np.swapaxes(ut_cols, -1, -2)
    v = [ut[:, 11 - i] for i in range(4)]  # compute_L_6x10: v[i] = ut + 12 (11 - i)
    dv = np.empty((B, 4, 6, 3))
    for i in range(4):
        for jj, (a, b) in enumerate(_PAIRS):
            dv[:, i, jj] = v[i][:, 3 * a:3 * a + 3] - v[i][:, 3 * b:3 * b + 3]
    L = np.empty((B, 6, 10))
    for i in range(6):
        d0, d1, d2, d3 = dv[:, 0, i], dv[:, 1, i], dv[:, 2, i], dv[:, 3, i]
        L[:, i, 0] = _dot3(d0, d0)
        L[:, i, 1] = 2.0 * _dot3(d0, d1)
        L[:, i, 2] = _dot3(d1, d1)
        L[:, i, 3] = 2.0 * _dot3(d0, d2)
        L[:, i, 4] = 2.0 * _dot3(d1, d2)
        L[:, i, 5] = _dot3(d2, d2)
        L[:, i, 6] = 2.0 * _dot3(d0, d3)
        L[:, i, 7] = 2.0 * _dot3(d1, d3)
        L[:, i, 8] = 2.0 * _dot3(d2, d3)
        L[:, i, 9] = _dot3(d3, d3)
    rho = np.empty((B, 6))
    for jj, (a, b) in enumerate(_PAIRS):
        e = cws[:, a] - cws[:, b]
        rho[:, jj] = _dot3(e, e)

    def gauss_newton(betas):
        x = np.zeros((B, 4))
        for _ in range(5):
            Aj = np.empty((B, 6, 4))
            bj = np.empty((B, 6))
            b0, b1, b2, b3 = betas[:, 0], betas[:, 1], betas[:, 2], betas[:, 3]
            for i in range(6):
                l = L[:, i]
                Aj[:, i, 0] = 2 * l[:, 0] * b0 + l[:, 1] * b1 + l[:, 3] * b2 + l[:, 6] * b3
                Aj[:, i, 1] = l[:, 1] * b0 + 2 * l[:, 2] * b1 + l[:, 4] * b2 + l[:, 7] * b3
                Aj[:, i, 2] = l[:, 3] * b0 + l[:, 4] * b1 + 2 * l[:, 5] * b2 + l[:, 8] * b3
                Aj[:, i, 3] = l[:, 6] * b0 + l[:, 7] * b1 + l[:, 8] * b2 + 2 * l[:, 9] * b3
                bj[:, i] = rho[:, i] - (l[:, 0] * b0 * b0 + l[:, 1] * b0 * b1 + l[:, 2] * b1 * b1 +
                                        l[:, 3] * b0 * b2 + l[:, 4] * b1 * b2 + l[:, 5] * b2 * b2 +
                                        l[:, 6] * b0 * b3 + l[:, 7] * b1 * b3 + l[:, 8] * b2 * b3 +
                                        l[:, 9] * b3 * b3)
            x = qr_solve(Aj, bj, x)
            betas = betas + x
        return betas

    def compute_R_and_t(betas):
        ccs = np.zeros((B, 4, 3))
        for i in range(4):
            for j in range(4):
                ccs[:, j] = ccs[:, j] + betas[:, i, None] * v[i][:, 3 * j:3 * j + 3]
        pcs = alphas[:, :, 0, None] * ccs[:, None, 0] + alphas[:, :, 1, None] * ccs[:, None, 1] + \
            alphas[:, :, 2, None] * ccs[:, None, 2] + alphas[:, :, 3, None] * ccs[:, None, 3]
        flip = pcs[:, 0, 2] < 0.0  # solve_for_sign
        pcs = np.where(flip[:, None, None], -pcs, pcs)
        # estimate_R_and_t
        pc0 = np.zeros((B, 3))
        pw0 = np.zeros((B, 3))
        for i in range(n):
            pc0 = pc0 + pcs[:, i]
            pw0 = pw0 + pws[:, i]
        pc0 = pc0 / n
        pw0 = pw0 / n
        abt = np.zeros((B, 3, 3))
        for i in range(n):
            abt = abt + (pcs[:, i] - pc0)[:, :, None] * (pws[:, i] - pw0)[:, None, :]
        _, Uab, Vtab, _ = svd_of(abt)
        R = np.einsum("bik,bkj->bij", Uab, Vtab)  # R[i][j] = dot(U row i, V row j) = (U V^T)_ij
        det = (R[:, 0, 0] * R[:, 1, 1] * R[:, 2, 2] + R[:, 0, 1] * R[:, 1, 2] * R[:, 2, 0] +
               R[:, 0, 2] * R[:, 1, 0] * R[:, 2, 1] - R[:, 0, 2] * R[:, 1, 1] * R[:, 2, 0] -
               R[:, 0, 1] * R[:, 1, 0] * R[:, 2, 2] - R[:, 0, 0] * R[:, 1, 2] * R[:, 2, 1])
        R[:, 2] = np.where((det < 0)[:, None], -R[:, 2], R[:, 2])
        t = pc0 - np.stack([_dot3(R[:, 0], pw0), _dot3(R[:, 1], pw0), _dot3(R[:, 2], pw0)], 1)
        # reprojection_error
        Xc = _dot3(R[:, None, 0], pws) + t[:, None, 0]
        Yc = _dot3(R[:, None, 1], pws) + t[:, None, 1]
        with np.errstate(divide="ignore", invalid="ignore"):
            inv_Zc = 1.0 / (_dot3(R[:, None, 2], pws) + t[:, None, 2])
        ue = uc + fu * Xc * inv_Zc
        ve = vc + fv * Yc * inv_Zc
        du, dvv = us[:, :, 0] - ue, us[:, :, 1] - ve
        err = np.zeros(B)
        for i in range(n):
            err = err + np.sqrt(du[:, i] * du[:, i] + dvv[:, i] * dvv[:, i])
        return R, t, err / n

    def approx_betas(cols, kind):
        Ls = L[:, :, cols]
        x = qr_solve(Ls, rho, np.zeros((B, len(cols))))
        be = np.zeros((B, 4))
        with np.errstate(divide="ignore", invalid="ignore"):
            if kind == 1:
                neg = x[:, 0] < 0
                be[:, 0] = np.sqrt(np.where(neg, -x[:, 0], x[:, 0]))
                sg = np.where(neg, -1.0, 1.0)
                be[:, 1] = sg * x[:, 1] / be[:, 0]
                be[:, 2] = sg * x[:, 2] / be[:, 0]
                be[:, 3] = sg * x[:, 3] / be[:, 0]
            else:
                neg = x[:, 0] < 0
                be[:, 0] = np.sqrt(np.where(neg, -x[:, 0], x[:, 0]))
                be[:, 1] = np.where(neg, np.where(x[:, 2] < 0, np.sqrt(-x[:, 2]), 0.0),
                                    np.where(x[:, 2] > 0, np.sqrt(x[:, 2]), 0.0))
                be[:, 0] = np.where(x[:, 1] < 0, -be[:, 0], be[:, 0])
                if kind == 3:
                    be[:, 2] = x[:, 3] / be[:, 0]
        return be

    sols = []
    for cols, kind in (([0, 1, 3, 6], 1), ([0, 1, 2], 2), ([0, 1, 2, 3, 4], 3)):
        betas = gauss_newton(approx_betas(cols, kind))
        sols.append(compute_R_and_t(betas))
    (R1, t1, e1), (R2, t2, e2), (R3, t3, e3) = sols
    N = np.where(e2 < e1, 2, 1)
    eN = np.where(N == 2, e2, e1)
    N = np.where(e3 < eN, 3, N)
    R = np.where((N == 1)[:, None, None], R1, np.where((N == 2)[:, None, None], R2, R3))
    t = np.where((N == 1)[:, None], t1, np.where((N == 2)[:, None], t2, t3))
    ok = ~(deg0 | deg1 | deg2) & np.all(np.isfinite(R), axis=(1, 2)) & np.all(np.isfinite(t), axis=1)
    return R, t, ok


# --------------------------------------------------------------------------- Rodrigues
def rodrigues_to_vec(R: np.ndarray) -> np.ndarray:
    """``Rodrigues`` matrix -> vector (calibration.cpp), batched (B, 3, 3) -> (B, 3).

    OpenCV first replaces R by ``U Vt`` of its SVD; for a rotation whose columns are
    orthogonal to ``10 DBL_EPSILON`` (every R produced here) JacobiSVD makes no rotation
    and ``U Vt`` is R with unit columns."""
    R = np.asarray(R, dtype=np.float64)
    R = R / np.sqrt(_seqsum(np.swapaxes(R, -1, -2) ** 2))[:, None, :]
    rx = R[:, 2, 1] - R[:, 1, 2]
    ry = R[:, 0, 2] - R[:, 2, 0]
    rz = R[:, 1, 0] - R[:, 0, 1]
    s = np.sqrt((rx * rx + ry * ry + rz * rz) * 0.25)
    c = (R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2] - 1) * 0.5
    c = np.clip(c, -1.0, 1.0)
    theta = np.array([math.acos(x) for x in c])  # libm acos, as OpenCV's std::acos
    out = np.empty((R.shape[0], 3))
    for b in range(R.shape[0]):
        if s[b] < 1e-5:
            if c[b] > 0:
                out[b] = 0.0
            else:
                r0 = math.sqrt(max((R[b, 0, 0] + 1) * 0.5, 0.0))
                r1 = math.sqrt(max((R[b, 1, 1] + 1) * 0.5, 0.0)) * (-1.0 if R[b, 0, 1] < 0 else 1.0)
                r2 = math.sqrt(max((R[b, 2, 2] + 1) * 0.5, 0.0)) * (-1.0 if R[b, 0, 2] < 0 else 1.0)
                if abs(r0) < abs(r1) and abs(r0) < abs(r2) and (R[b, 1, 2] > 0) != (r1 * r2 > 0):
                    r2 = -r2
                th = theta[b] / math.sqrt(r0 * r0 + r1 * r1 + r2 * r2)
                out[b] = (r0 * th, r1 * th, r2 * th)
        else:
            vth = 1 / (2 * s[b])
            vth *= theta[b]
            out[b] = (rx[b] * vth, ry[b] * vth, rz[b] * vth)
    return out


def rodrigues_to_mat(r: np.ndarray) -> np.ndarray:
    """``Rodrigues`` vector -> matrix, batched (B, 3) -> (B, 3, 3)."""
    r = np.asarray(r, dtype=np.float64).reshape(-1, 3)
    theta = np.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2])
    out = np.broadcast_to(np.eye(3), (r.shape[0], 3, 3)).copy()
    nz = theta >= DBL_EPSILON
    if nz.any():
        th = theta[nz]
        c = np.array([math.cos(x) for x in th])  # libm, as OpenCV
        s = np.array([math.sin(x) for x in th])
        c1 = 1.0 - c
        u = r[nz] * (1.0 / th)[:, None]
        x, y, z = u[:, 0], u[:, 1], u[:, 2]
        rrt = np.stack([x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z], 1).reshape(-1, 3, 3)
        zero = np.zeros_like(x)
        rx = np.stack([zero, -z, y, z, zero, -x, -y, x, zero], 1).reshape(-1, 3, 3)
        out[nz] = c[:, None, None] * np.eye(3) + c1[:, None, None] * rrt + s[:, None, None] * rx
    return out


# --------------------------------------------------------------------------- scoring
def project_f32(R: np.ndarray, t: np.ndarray, X32: np.ndarray, K: np.ndarray) -> np.ndarray:
    """``projectPoints`` of float32 object points with (R, t) -> float32 (B, n, 2)
    (cvProjectPoints2Internal, no distortion: X = R M + t left to right, z = 1/Z)."""
    M = np.asarray(X32, dtype=np.float32).astype(np.float64)
    X, Y, Z = M[..., 0], M[..., 1], M[..., 2]
    R = R[:, None]
    t = t[:, None]
    x = R[..., 0, 0] * X + R[..., 0, 1] * Y + R[..., 0, 2] * Z + t[..., 0]
    y = R[..., 1, 0] * X + R[..., 1, 1] * Y + R[..., 1, 2] * Z + t[..., 1]
    z = R[..., 2, 0] * X + R[..., 2, 1] * Y + R[..., 2, 2] * Z + t[..., 2]
    with np.errstate(divide="ignore"):
        zi = np.where(z != 0, 1.0 / np.where(z != 0, z, 1.0), 1.0)
    u = (x * zi) * K[0, 0] + K[0, 2]
    v = (y * zi) * K[1, 1] + K[1, 2]
    return np.stack([u, v], -1).astype(np.float32)


def reproj_err2(R, t, X32, uv32, K) -> np.ndarray:
    """``computeError``: float32 ``dx*dx + dy*dy`` per point (B, n)."""
    P = project_f32(R, t, X32, K)
    d = np.asarray(uv32, dtype=np.float32)[None] - P
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]).astype(np.float32)


# --------------------------------------------------------------------------- refinement
def _skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def _se3_exp(d):
    rho, phi = d[:3], d[3:]
    th = math.sqrt(float(phi @ phi))
    K_ = _skew(phi)
    if th < 1e-4:
        R = np.eye(3) + K_ + 0.5 * K_ @ K_
        V = np.eye(3) + 0.5 * K_ + K_ @ K_ / 6.0
    else:
        a = math.sin(th) / th
        b = (1 - math.cos(th)) / (th * th)
        c = (th - math.sin(th)) / (th * th * th)
        R = np.eye(3) + a * K_ + b * K_ @ K_
        V = np.eye(3) + b * K_ + c * K_ @ K_
    return R, V @ rho


def _normal_eq(R, t, X, uv, K):
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    pc = X @ R.T + t
    zi = 1.0 / pc[:, 2]
    u = fx * pc[:, 0] * zi + cx
    v = fy * pc[:, 1] * zi + cy
    r = np.stack([u - uv[:, 0], v - uv[:, 1]], 1)
    n = X.shape[0]
    Jp = np.zeros((n, 2, 3))
    Jp[:, 0, 0] = fx * zi
    Jp[:, 0, 2] = -fx * pc[:, 0] * zi * zi
    Jp[:, 1, 1] = fy * zi
    Jp[:, 1, 2] = -fy * pc[:, 1] * zi * zi
    J = np.zeros((n, 2, 6))
    J[:, :, :3] = Jp
    sk = np.zeros((n, 3, 3))
    sk[:, 0, 1], sk[:, 0, 2] = -pc[:, 2], pc[:, 1]
    sk[:, 1, 0], sk[:, 1, 2] = pc[:, 2], -pc[:, 0]
    sk[:, 2, 0], sk[:, 2, 1] = -pc[:, 1], pc[:, 0]
    J[:, :, 3:] = -Jp @ sk
    A = np.einsum("nki,nkj->ij", J, J)
    g = np.einsum("nki,nk->i", J, r)
    return A, g, float(np.sum(r * r))


def refine_lm(R, t, X, uv, K):
    """Levenberg-Marquardt on the reprojection error of (X, uv) (float64), left se(3)
    increment, CvLevMarq's lambda schedule.  -> (R, t)."""
    R = np.array(R, dtype=np.float64)
    t = np.array(t, dtype=np.float64)
    X = np.asarray(X, dtype=np.float64)
    uv = np.asarray(uv, dtype=np.float64)
    A, g, cost = _normal_eq(R, t, X, uv, K)
    lg = LM_LAMBDA_LG10_INIT
    accepted = 0
    while accepted < LM_MAX_ITERS:
        lam = 10.0 ** lg
        An = A.copy()
        An[np.diag_indices(6)] *= 1.0 + lam
        try:
            delta = -np.linalg.solve(An, g)
        except np.linalg.LinAlgError:
            break
        dR, dt = _se3_exp(delta)
        Rn, tn = dR @ R, dR @ t + dt
        An2, gn, costn = _normal_eq(Rn, tn, X, uv, K)
        if costn <= cost:
            small = float(np.sqrt(delta @ delta)) <= FLT_EPSILON * (1.0 + float(np.sqrt(t @ t)))
            R, t, A, g, cost = Rn, tn, An2, gn, costn
            lg = max(lg - 1, -16)
            accepted += 1
            if small:
                break
        else:
            lg += 1
            if lg > 16:
                break
    return R, t


# --------------------------------------------------------------------------- driver
def solve_pnp_ransac(opoints, ipoints, K, reproj_err: float = 8.0, iterations: int = 100,
                     confidence: float = 0.99):
    """``cv2.solvePnPRansac(opoints, ipoints, K, None, reprojectionError=...)`` ->
    (success, rvec (3,), tvec (3,), inlier mask (n,) bool, details dict)."""
    X32 = np.ascontiguousarray(np.asarray(opoints, dtype=np.float32).reshape(-1, 3))
    uv32 = np.ascontiguousarray(np.asarray(ipoints, dtype=np.float32).reshape(-1, 2))
    K = np.asarray(K, dtype=np.float64)
    n = X32.shape[0]
    fail = (False, np.zeros(3), np.zeros(3), np.zeros(n, dtype=bool), {})
    if n < MODEL_POINTS:
        return fail
    if n == MODEL_POINTS:
        R, t, ok = epnp(X32[None].astype(np.float64), uv32[None].astype(np.float64), K)
        if not ok[0]:
            return fail
        return True, rodrigues_to_vec(R)[0], t[0], np.ones(n, dtype=bool), {}
    subsets = ransac_subsets(n, iterations)
    R, t, ok = epnp(X32[subsets].astype(np.float64), uv32[subsets].astype(np.float64), K)
    # the model is stored as (rvec, tvec) and projectPoints turns rvec back into R
    rv = rodrigues_to_vec(np.where(ok[:, None, None], R, np.eye(3)))
    Rm = rodrigues_to_mat(rv)
    err = reproj_err2(Rm, t, X32, uv32, K)
    thr = np.float32(reproj_err * reproj_err)
    inl = err <= thr
    counts = inl.sum(axis=1)
    niters = max(iterations, 1)
    best, max_good = -1, 0
    it = 0
    while it < niters:
        if ok[it]:
            good = int(counts[it])
            if good > max(max_good, MODEL_POINTS - 1):
                best, max_good = it, good
                niters = update_num_iters(confidence, (n - good) / n, MODEL_POINTS, niters)
        it += 1
    if best < 0:
        return fail
    mask = inl[best]
    Rr, tr = refine_lm(Rm[best], t[best], X32[mask], uv32[mask], K)
    rvec = rodrigues_to_vec(Rr[None])[0]
    return True, rvec, tr, mask, {"best": best, "counts": counts, "valid": ok, "iters_run": it,
                                  "R_models": Rm, "t_models": t, "R": Rr, "t": tr}
