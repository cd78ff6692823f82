"""Seeded synthetic inputs for the matcher and the sliding-window BA.

The reference ships no fixtures or data, so every workload
in tests and bench.py is generated here from a fixed seed, following the
generator spec of SURVEY.md §8(d):

* BA: KITTI intrinsics (``src/modules/dataset_loader.py:52-54``), a forward
  trajectory of 1 m per pose with a yaw random walk, landmarks drawn in the
  frustum of their first camera at depth U[5, 50] m, contiguous tracks of
  U{2..8} poses clipped to visibility, 1 px pixel noise, and an initial guess
  perturbed by 0.01 rad / 0.05 m per pose and 2 % of depth per point.
* Matcher: SIFT-like descriptors (integers 0..255 stored as float32, the
  layout ``FeatureFrontend.process_image`` produces at
  ``src/modules/frontend.py:59-67``) and SuperPoint-like L2-normalised
  float32 descriptors.

Pose convention: ``T_cw`` (world -> camera), as the reference projects with
``T_cw = inv(T_wc)`` (``src/modules/vo.py:260-261``).
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

KITTI_K = np.array(
    [[718.856, 0.0, 607.1928], [0.0, 718.856, 185.2157], [0.0, 0.0, 1.0]]
)
KITTI_WH = (1241, 376)

# (n_poses, n_points, seed) of the BASELINE.json BA configs
BA_CONFIGS = {
    "cfg2": (20, 5_000, 2),
    "cfg3": (50, 20_000, 3),
    "cfg4": (100, 200_000, 4),
}


@dataclass
class BAProblemData:
    """A BA window in the layout of the C-ABI (``include/vo_hip.h``).

    ``obs_*`` are CSR-ordered by point: observations of point ``p`` are
    ``point_ptr[p]:point_ptr[p+1]``.
    """

    K: np.ndarray  # (3,3) f64
    poses_cw: np.ndarray  # (N,4,4) f64 initial guess
    points: np.ndarray  # (L,3) f64 initial guess
    point_ptr: np.ndarray  # (L+1,) i32
    obs_cam: np.ndarray  # (M,) i32
    obs_uv: np.ndarray  # (M,2) f32
    n_fixed: int
    poses_true: np.ndarray  # (N,4,4)
    points_true: np.ndarray  # (L,3)

    @property
    def n_poses(self) -> int:
        return self.poses_cw.shape[0]

    @property
    def n_points(self) -> int:
        return self.points.shape[0]

    @property
    def n_obs(self) -> int:
        return self.obs_cam.shape[0]

    def obs_point(self) -> np.ndarray:
        """Point index of each observation (expanded CSR)."""
        return np.repeat(
            np.arange(self.n_points, dtype=np.int32), np.diff(self.point_ptr)
        )


def so3_exp(phi: np.ndarray) -> np.ndarray:
    """Rodrigues for a batch of axis-angle vectors (...,3) -> (...,3,3)."""
    phi = np.asarray(phi, dtype=np.float64)
    th = np.linalg.norm(phi, axis=-1)[..., None, None]
    k = np.zeros(phi.shape[:-1] + (3, 3))
    k[..., 0, 1], k[..., 0, 2] = -phi[..., 2], phi[..., 1]
    k[..., 1, 0], k[..., 1, 2] = phi[..., 2], -phi[..., 0]
    k[..., 2, 0], k[..., 2, 1] = -phi[..., 1], phi[..., 0]
    small = th < 1e-8
    ths = np.where(small, 1.0, th)
    a = np.where(small, 1.0, np.sin(ths) / ths)
    b = np.where(small, 0.5, (1.0 - np.cos(ths)) / ths**2)
    eye = np.broadcast_to(np.eye(3), k.shape)
    return eye + a * k + b * (k @ k)


def make_ba_problem(
    n_poses: int,
    n_points: int,
    seed: int,
    *,
    noise_px: float = 1.0,
    n_fixed: int = 2,
    rot_perturb: float = 0.01,
    trans_perturb: float = 0.05,
    point_perturb: float = 0.02,
    max_track: int = 8,
) -> BAProblemData:
    """Synthetic sliding-window BA problem."""
    rng = np.random.default_rng(seed)
    K = KITTI_K.copy()
    W, H = KITTI_WH
    Kinv = np.linalg.inv(K)

    # --- trajectory: T_wc, 1 m forward per pose along the camera z axis
    yaw = np.cumsum(np.concatenate([[0.0], rng.normal(0.0, 0.01, n_poses - 1)]))
    R_wc = so3_exp(np.stack([np.zeros(n_poses), yaw, np.zeros(n_poses)], -1))
    pos = np.zeros((n_poses, 3))
    for i in range(1, n_poses):
        pos[i] = pos[i - 1] + R_wc[i] @ np.array([0.0, 0.0, 1.0])
    R_cw = np.transpose(R_wc, (0, 2, 1))
    t_cw = -np.einsum("nij,nj->ni", R_cw, pos)
    poses_true = np.tile(np.eye(4), (n_poses, 1, 1))
    poses_true[:, :3, :3] = R_cw
    poses_true[:, :3, 3] = t_cw

    # --- landmarks: first camera sorted (landmarks are created in keyframe order)
    first = np.sort(rng.integers(0, n_poses - 1, n_points))
    want = rng.integers(2, max_track + 1, n_points)
    pts = np.empty((n_points, 3))
    tracks_len = np.empty(n_points, dtype=np.int64)
    todo = np.arange(n_points)
    for _attempt in range(64):
        if todo.size == 0:
            break
        f = first[todo]
        u = rng.uniform(0.0, W, todo.size)
        v = rng.uniform(0.0, H, todo.size)
        d = rng.uniform(5.0, 50.0, todo.size)
        ray = (Kinv @ np.stack([u, v, np.ones_like(u)])).T * d[:, None]
        X = np.einsum("nij,nj->ni", R_wc[f], ray) + pos[f]
        # visibility run along the following cameras
        length = np.ones(todo.size, dtype=np.int64)
        alive = np.ones(todo.size, dtype=bool)
        for s in range(1, max_track):
            cam = f + s
            ok = alive & (cam < n_poses) & (s < want[todo])
            camc = np.minimum(cam, n_poses - 1)
            pc = np.einsum("nij,nj->ni", R_cw[camc], X) + t_cw[camc]
            z = pc[:, 2]
            zs = np.where(z > 1e-6, z, 1.0)
            uu = K[0, 0] * pc[:, 0] / zs + K[0, 2]
            vv = K[1, 1] * pc[:, 1] / zs + K[1, 2]
            vis = (z > 0.5) & (uu >= 0) & (uu < W) & (vv >= 0) & (vv < H)
            ok &= vis
            length += ok
            alive &= ok
        good = length >= 2
        pts[todo[good]] = X[good]
        tracks_len[todo[good]] = length[good]
        todo = todo[~good]
    if todo.size:
        raise RuntimeError("could not place all landmarks with track >= 2")

    point_ptr = np.zeros(n_points + 1, dtype=np.int64)
    point_ptr[1:] = np.cumsum(tracks_len)
    M = int(point_ptr[-1])
    obs_pt = np.repeat(np.arange(n_points), tracks_len)
    obs_cam = first[obs_pt] + (np.arange(M) - point_ptr[obs_pt])
    pc = np.einsum("nij,nj->ni", R_cw[obs_cam], pts[obs_pt]) + t_cw[obs_cam]
    uv = np.stack(
        [K[0, 0] * pc[:, 0] / pc[:, 2] + K[0, 2], K[1, 1] * pc[:, 1] / pc[:, 2] + K[1, 2]],
        -1,
    )
    uv = uv + rng.normal(0.0, noise_px, uv.shape)

    # --- initial guess
    poses0 = poses_true.copy()
    nf = min(n_fixed, n_poses)
    dR = so3_exp(rng.normal(0.0, rot_perturb, (n_poses, 3)))
    dt = rng.normal(0.0, trans_perturb, (n_poses, 3))
    poses0[nf:, :3, :3] = dR[nf:] @ poses_true[nf:, :3, :3]
    poses0[nf:, :3, 3] = poses_true[nf:, :3, 3] + dt[nf:]
    depth = np.einsum("nj,nj->n", R_cw[first][:, 2, :], pts) + t_cw[first][:, 2]
    points0 = pts + rng.normal(0.0, 1.0, pts.shape) * (point_perturb * depth)[:, None]

    return BAProblemData(
        K=K,
        poses_cw=poses0,
        points=points0,
        point_ptr=point_ptr.astype(np.int32),
        obs_cam=obs_cam.astype(np.int32),
        obs_uv=uv.astype(np.float32),
        n_fixed=nf,
        poses_true=poses_true,
        points_true=pts,
    )


def make_ba_config(name: str, **kw) -> BAProblemData:
    n, l, seed = BA_CONFIGS[name]
    return make_ba_problem(n, l, seed, **kw)


def make_ba_slide(name: str, n_windows: int, **kw) -> list:
    """``n_windows`` windows of config ``name``'s size sliding one keyframe at a time along one
    drive: window j holds poses j .. j + n - 1 of a drive of n + n_windows - 1 poses and every
    landmark seen there by two or more of them (its observations outside clipped), in the
    drive's landmark order -- what the reference's loop hands its BA per keyframe
    (``vo.py:252-288``; the drop-in's ``KeyframeWindow.build``).  The drive's landmark density
    per pose is the config's, so each window is the config's size give or take its edges."""
    n, l, seed = BA_CONFIGS[name]
    n_drive = n + n_windows - 1
    d = make_ba_problem(n_drive, int(round(l * n_drive / n)), seed, **kw)
    obs_pt = np.repeat(np.arange(d.points.shape[0]), np.diff(d.point_ptr))
    out = []
    for j in range(n_windows):
        inw = (d.obs_cam >= j) & (d.obs_cam < j + n)
        cnt = np.bincount(obs_pt[inw], minlength=d.points.shape[0])
        keep_pt = cnt >= 2
        sel = inw & keep_pt[obs_pt]
        pts_idx = np.flatnonzero(keep_pt)
        point_ptr = np.zeros(pts_idx.size + 1, np.int64)
        point_ptr[1:] = np.cumsum(cnt[pts_idx])
        out.append(BAProblemData(
            K=d.K,
            poses_cw=d.poses_cw[j:j + n].copy(),
            points=d.points[pts_idx].copy(),
            point_ptr=point_ptr.astype(np.int32),
            obs_cam=(d.obs_cam[sel] - j).astype(np.int32),
            obs_uv=d.obs_uv[sel].copy(),
            n_fixed=d.n_fixed,
            poses_true=d.poses_true[j:j + n].copy(),
            points_true=d.points_true[pts_idx].copy(),
        ))
    return out


def sift_like_descriptors(n: int, rng: np.random.Generator, dim: int = 128) -> np.ndarray:
    """Integer-valued 0..255 float32 descriptors with ~40 % zeros (SIFT-like).

    OpenCV SIFT writes ``saturate_cast<uchar>`` values into its CV_32F
    descriptor, which ``process_image`` casts to float32 (frontend.py:60).
    """
    mag = rng.gamma(1.5, 40.0, (n, dim))
    mag[rng.random((n, dim)) < 0.4] = 0.0
    return np.clip(np.rint(mag), 0, 255).astype(np.float32)


def sift_like_pair(n0: int, n1: int, seed: int, dim: int = 128, overlap: float = 0.6):
    """Two descriptor sets where a fraction of set-1 rows are noisy copies of set-0 rows."""
    rng = np.random.default_rng(seed)
    d0 = sift_like_descriptors(n0, rng, dim)
    d1 = sift_like_descriptors(n1, rng, dim)
    k = int(min(n0, n1) * overlap)
    src = rng.choice(n0, k, replace=False)
    dst = rng.choice(n1, k, replace=False)
    noisy = d0[src] + rng.normal(0.0, 6.0, (k, dim))
    d1[dst] = np.clip(np.rint(noisy), 0, 255).astype(np.float32)
    return d0, d1


def superpoint_like_pair(n0: int, n1: int, seed: int, dim: int = 256, overlap: float = 0.6):
    """L2-normalised float32 descriptor sets (SuperPoint-like, D=256)."""
    rng = np.random.default_rng(seed)
    d0 = rng.standard_normal((n0, dim)).astype(np.float32)
    d1 = rng.standard_normal((n1, dim)).astype(np.float32)
    k = int(min(n0, n1) * overlap)
    src = rng.choice(n0, k, replace=False)
    dst = rng.choice(n1, k, replace=False)
    d1[dst] = d0[src] + 0.3 * rng.standard_normal((k, dim)).astype(np.float32)
    d0 /= np.linalg.norm(d0, axis=1, keepdims=True)
    d1 /= np.linalg.norm(d1, axis=1, keepdims=True)
    return d0.astype(np.float32), d1.astype(np.float32)


def triangulation_case(n: int, seed: int, noise_px: float = 0.5, outlier_frac: float = 0.1,
                       behind_frac: float = 0.05):
    """Two-view triangulation input of the reference's shape (``vo.py:266-275``): KITTI K,
    camera 2 one metre ahead of camera 1 with a small yaw, points in front of both, image
    points float32 with ``noise_px`` noise.  A fraction of the correspondences are gross
    outliers (camera 2 point moved by 30-100 px) and a fraction lie behind both cameras.
    Cases sit far from the reference's thresholds (reprojection error << 2 px for
    inliers, >> 10 px for outliers) so that masks are comparable exactly.

    Returns (T_cw1, T_cw2, pts1 (n,2) f32, pts2 (n,2) f32, K, X (n,3) f64, kind (n,) int:
    0 inlier, 1 outlier, 2 behind).
    """
    rng = np.random.default_rng(seed)
    K = np.array([[718.856, 0.0, 607.1928], [0.0, 718.856, 185.2157], [0.0, 0.0, 1.0]])
    T_cw1 = np.eye(4)
    yaw = rng.normal(0.0, 0.02)
    R = so3_exp(np.array([0.0, yaw, 0.0]))
    C2 = np.array([rng.normal(0, 0.05), rng.normal(0, 0.02), 1.0])  # camera 2 centre (world)
    T_cw2 = np.eye(4)
    T_cw2[:3, :3] = R.T
    T_cw2[:3, 3] = -R.T @ C2
    kind = np.zeros(n, dtype=np.int64)
    u = rng.permutation(n)
    n_out, n_beh = int(outlier_frac * n), int(behind_frac * n)
    kind[u[:n_out]] = 1
    kind[u[n_out:n_out + n_beh]] = 2
    depth = rng.uniform(5.0, 50.0, n)
    # keep >= 150 px from the epipole of the forward motion (enough parallax)
    e1 = K @ C2
    e1 = e1[:2] / e1[2]
    px = np.empty((n, 2))
    filled = 0
    while filled < n:
        c = np.stack([rng.uniform(50, 1190, 4 * n), rng.uniform(30, 345, 4 * n)], 1)
        c = c[np.linalg.norm(c - e1, axis=1) > 150.0][: n - filled]
        px[filled:filled + len(c)] = c
        filled += len(c)
    ray = np.linalg.solve(K, np.concatenate([px, np.ones((n, 1))], 1).T).T
    X = ray * depth[:, None]
    X[kind == 2] *= -1.0  # behind both cameras
    def proj(T, Xw):
        Xc = (T[:3, :3] @ Xw.T).T + T[:3, 3]
        q = (K @ Xc.T).T
        return q[:, :2] / q[:, 2:3]
    p1 = proj(T_cw1, X) + rng.normal(0, noise_px, (n, 2))
    p2 = proj(T_cw2, X) + rng.normal(0, noise_px, (n, 2))
    # outliers: moved 30-100 px across the epipolar line of their camera-1 point
    R21 = T_cw2[:3, :3]
    t21 = T_cw2[:3, 3]
    tx = np.array([[0, -t21[2], t21[1]], [t21[2], 0, -t21[0]], [-t21[1], t21[0], 0]])
    Ki = np.linalg.inv(K)
    Fm = Ki.T @ tx @ R21 @ Ki
    lines = (Fm @ np.concatenate([p1, np.ones((n, 1))], 1).T).T
    nrm = lines[:, :2] / np.linalg.norm(lines[:, :2], axis=1, keepdims=True)
    d = rng.uniform(30, 100, n) * np.where(rng.random(n) < 0.5, -1.0, 1.0)
    p2[kind == 1] += (nrm * d[:, None])[kind == 1]
    return T_cw1, T_cw2, p1.astype(np.float32), p2.astype(np.float32), K, X, kind


def pnp_case(n: int, seed: int, noise_px: float = 0.3, outlier_frac: float = 0.25):
    """A tracking-step input of the reference's shape (``vo.py:129-141``): ``n`` map points
    (float32, as ``map_points`` holds them, ``vo.py:281``) seen by a camera with KITTI K
    at a random pose, their float32 keypoints with ``noise_px`` noise, and a fraction of
    gross outliers (keypoint moved 25-200 px).  Points sit 5-50 m in front of the camera.

    Returns (X (n,3) f32, uv (n,2) f32, K, T_cw (4,4), is_outlier (n,) bool)."""
    rng = np.random.default_rng(seed)
    K = KITTI_K.copy()
    W, H = KITTI_WH
    px = np.stack([rng.uniform(20, W - 20, n), rng.uniform(20, H - 20, n)], 1)
    depth = rng.uniform(5.0, 50.0, n)
    ray = np.linalg.solve(K, np.concatenate([px, np.ones((n, 1))], 1).T).T
    Xc = ray * depth[:, None]
    R = so3_exp(rng.normal(0, 0.2, 3))
    t = rng.normal(0, 2.0, 3)
    T_cw = np.eye(4)
    T_cw[:3, :3] = R
    T_cw[:3, 3] = t
    Xw = (R.T @ (Xc - t).T).T
    X32 = Xw.astype(np.float32)
    pc = (R @ X32.astype(np.float64).T).T + t
    q = (K @ pc.T).T
    uv = q[:, :2] / q[:, 2:3] + rng.normal(0, noise_px, (n, 2))
    out = np.zeros(n, dtype=bool)
    out[rng.permutation(n)[: int(outlier_frac * n)]] = True
    ang = rng.uniform(0, 2 * np.pi, n)
    mag = rng.uniform(25, 200, n)
    uv[out] += np.stack([np.cos(ang), np.sin(ang)], 1)[out] * mag[out, None]
    return X32, uv.astype(np.float32), K, T_cw, out


def sift_scene(h: int = 376, w: int = 1241, seed: int = 0, n_blobs: int = 400, n_boxes: int = 60,
               texture: float = 0.0) -> np.ndarray:
    """A uint8 grayscale image of KITTI's size (``image_0``, ``dataset_loader.py:63``) with
    SIFT-detectable structure: a smooth vertical gradient, Gaussian blobs of 2-10 px
    sigma (light and dark), axis-aligned boxes (edges and corners) and 2 gray levels of
    noise.  ``texture`` > 0 adds cubic value noise at 3, 6 and 12 px scales of that
    amplitude (gray levels): at 12 a KITTI-size image has ~7.8k SIFT keypoints at the
    reference's KITTI settings, so its ``nfeatures = 4000`` cut binds as on real frames."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    im = 70.0 + 60.0 * yy / h
    for _ in range(n_boxes):
        y0, x0 = rng.integers(0, max(h - 10, 1)), rng.integers(0, max(w - 10, 1))
        bh, bw = rng.integers(8, 60), rng.integers(8, 120)
        im[y0:y0 + bh, x0:x0 + bw] += rng.uniform(-50, 50)
    for _ in range(n_blobs):
        cy, cx, s = rng.uniform(0, h), rng.uniform(0, w), rng.uniform(2, 10)
        r = int(4 * s)
        y0, y1 = max(int(cy) - r, 0), min(int(cy) + r + 1, h)
        x0, x1 = max(int(cx) - r, 0), min(int(cx) + r + 1, w)
        g = np.exp(-((yy[y0:y1, x0:x1] - cy) ** 2 + (xx[y0:y1, x0:x1] - cx) ** 2) / (2 * s * s))
        im[y0:y1, x0:x1] += rng.choice([-1.0, 1.0]) * rng.uniform(40, 90) * g
    im += rng.normal(0, 2.0, im.shape)
    if texture > 0:
        from scipy.ndimage import zoom

        trng = np.random.default_rng(seed + 99)
        for sc in (3, 6, 12):
            g = trng.normal(0, 1, (h // sc + 2, w // sc + 2))
            im += texture * zoom(g, sc, order=3)[:h, :w]
    return np.clip(np.rint(im), 0, 255).astype(np.uint8)
