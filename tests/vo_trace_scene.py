"""Deterministic synthetic VO sequence for the reference-trace fixtures (test infrastructure).

A KITTI-like drive (camera ``image_0`` intrinsics, 1241 x 376, forward motion with a slow
yaw) through a corridor of landmarks.  Each frame's "SIFT output" is the projection of the
visible landmarks plus noise and their per-landmark descriptors (integers 0..255, as
OpenCV's SIFT produces, with a small per-observation perturbation), plus distractors.

``tests/golden/make_reference_trace.py`` feeds these frames to the reference's own
``VisualOdometry`` (cv2 replaced by oracle-backed stubs) and records its calls; the GPU
test ``tests/test_gpu_reference_trace.py`` regenerates the same frames here to replay the
recorded calls through the HIP path.  Everything is seeded: the same numpy produces the
same frames on the build container and the GPU box.
"""

from __future__ import annotations

import numpy as np

K_KITTI = np.array([[7.18856e02, 0, 6.071928e02], [0, 7.18856e02, 1.852157e02], [0, 0, 1]])
W, H = 1241, 376


def _rot_y(a: float) -> np.ndarray:
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])


class TraceScene:
    def __init__(self, n_frames: int = 36, n_landmarks: int = 9000, seed: int = 7, max_features: int = 1400,
                 n_distractors: int = 80, noise_px: float = 0.25, speed: float = 1.2):
        self.n_frames, self.seed = n_frames, seed
        self.max_features, self.n_distractors, self.noise_px = max_features, n_distractors, noise_px
        rng = np.random.default_rng(seed)
        L = n_landmarks
        z_far = 12.0 + speed * n_frames + 60.0
        self.X = np.stack([rng.uniform(-25, 25, L), rng.uniform(-4, 2.5, L), rng.uniform(4, z_far, L)], 1)
        # SIFT-like integer descriptors: sparse, heavy-tailed, clipped to 0..255
        d = rng.gamma(0.6, 30.0, (L, 128))
        d[rng.random((L, 128)) < 0.35] = 0.0
        self.des = np.clip(np.rint(d), 0, 255).astype(np.int16)
        self.prio = rng.permutation(L)  # deterministic visibility priority
        # camera -> world poses: forward along +z, slow yaw and a small lateral sway
        self.T_wc = []
        for f in range(n_frames):
            T = np.eye(4)
            T[:3, :3] = _rot_y(0.06 * np.sin(f / 9.0))
            T[:3, 3] = (0.8 * np.sin(f / 11.0), 0.0, speed * f)
            self.T_wc.append(T)
        self.kp_frame: dict[tuple, int] = {}

    def frame(self, f: int):
        """-> (keypoints (N, 2) float32, descriptors (N, 128) float32, landmark id per row or -1)."""
        rng = np.random.default_rng((self.seed, f))
        T_cw = np.linalg.inv(self.T_wc[f])
        Xc = self.X @ T_cw[:3, :3].T + T_cw[:3, 3]
        z = Xc[:, 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = K_KITTI[0, 0] * Xc[:, 0] / z + K_KITTI[0, 2]
            v = K_KITTI[1, 1] * Xc[:, 1] / z + K_KITTI[1, 2]
        vis = (z > 2.0) & (u > 4) & (u < W - 4) & (v > 4) & (v < H - 4)
        ids = self.prio[np.isin(self.prio, np.flatnonzero(vis))][: self.max_features]
        uv = np.stack([u[ids], v[ids]], 1) + rng.normal(0.0, self.noise_px, (ids.size, 2))
        des = self.des[ids] + rng.integers(-2, 3, (ids.size, 128))
        nd = self.n_distractors
        uv_d = np.stack([rng.uniform(4, W - 4, nd), rng.uniform(4, H - 4, nd)], 1)
        des_d = np.clip(np.rint(rng.gamma(0.6, 30.0, (nd, 128))), 0, 255)
        uv = np.concatenate([uv, uv_d]).astype(np.float32)
        des = np.clip(np.concatenate([des, des_d]), 0, 255).astype(np.float32)
        lm = np.concatenate([ids, -np.ones(nd, np.int64)])
        order = rng.permutation(uv.shape[0])
        uv, des, lm = uv[order], des[order], lm[order]
        for p in uv:
            self.kp_frame[(float(p[0]), float(p[1]))] = f
        return uv, des, lm

    def frame_of(self, uv) -> int:
        """The frame a keypoint array came from (every keypoint frame() returned is registered)."""
        for p in np.asarray(uv, np.float32).reshape(-1, 2)[:8]:
            f = self.kp_frame.get((float(p[0]), float(p[1])))
            if f is not None:
                return f
        raise KeyError("keypoints of an unknown frame")

    def relative_pose(self, f_ref: int, f_cur: int):
        """(R, t unit) with X_cur = R X_ref + t, as cv2.recoverPose returns it."""
        T = np.linalg.inv(self.T_wc[f_cur]) @ self.T_wc[f_ref]
        t = T[:3, 3]
        return T[:3, :3].copy(), (t / np.linalg.norm(t)).reshape(3, 1)
