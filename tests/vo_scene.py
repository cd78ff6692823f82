"""Synthetic keyframe sequence and a test double of the reference VO state (tests only).

``FakeVO`` carries the attributes the keyframe hook reads and writes
(``map_points``, ``next_pt_id``, ``T_wc``, ``keyframe``, ``cfg``, ``K``,
``last_pos`` -- reference ``src/modules/vo.py:15-29``) and a
``_create_keyframe`` with the reference's observable effect (``vo.py:252-288``):
new ids for matched keypoints without one, the keyframe replaced, old ids pruned.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from visualodometry_amd.synthetic import KITTI_K, KITTI_WH


@dataclass
class Cfg:
    ba_enabled: bool = True
    ba_window: int = 50
    ba_fixed: int = 2
    ba_iters: int = 10
    ba_lambda: float = 1.0
    extractor_type: str = "sift"
    match_on_gpu: bool = True


class FakeVO:
    def __init__(self, cfg, K=KITTI_K, tri_noise=0.05, seed=0):
        self.cfg, self.K = cfg, np.asarray(K, np.float64)
        self.map_points, self.next_pt_id = {}, 0
        self.T_wc, self.keyframe, self.last_pos = np.eye(4), None, np.zeros(3)
        self.truth = {}  # id -> true landmark index (test bookkeeping)
        self.rng = np.random.default_rng(seed)
        self.tri_noise = tri_noise
        self.scene = None

    def _create_keyframe(self, curr_feats, curr_ids, ref_indices, curr_indices):
        no_id = curr_ids[curr_indices] == -1
        rows = np.nonzero(no_id)[0]
        valid = self.rng.random(rows.size) < 0.9
        for r, ok in zip(rows, valid):
            if ok:
                lm = curr_feats["lm"][curr_indices[r]]
                X = self.scene.X[lm] + self.rng.normal(0, self.tri_noise, 3)
                self.map_points[self.next_pt_id] = X.astype(np.float32)
                self.truth[self.next_pt_id] = lm
                curr_ids[curr_indices[r]] = self.next_pt_id
                self.next_pt_id += 1
        self.keyframe = {"feats": curr_feats, "ids": curr_ids, "T_wc": self.T_wc.copy()}

    def _reset_system(self):
        self.map_points, self.keyframe = {}, None


class Scene:
    """Forward-moving camera (1 m/keyframe) and landmarks in front of it."""

    def __init__(self, n_kf=12, n_pts=600, seed=1, noise_px=0.5):
        rng = np.random.default_rng(seed)
        self.n_kf = n_kf
        self.T_wc = np.tile(np.eye(4), (n_kf, 1, 1))
        yaw = np.cumsum(rng.normal(0, 0.01, n_kf))
        for k in range(n_kf):
            c, s = np.cos(yaw[k]), np.sin(yaw[k])
            self.T_wc[k, :3, :3] = [[c, 0, s], [0, 1, 0], [-s, 0, c]]
            self.T_wc[k, 2, 3] = float(k)
        self.X = np.stack([rng.uniform(-15, 15, n_pts), rng.uniform(-3, 3, n_pts),
                           rng.uniform(6, 40 + n_kf, n_pts)], 1)
        self.rng, self.noise = rng, noise_px

    def keypoints(self, k):
        T_cw = np.linalg.inv(self.T_wc[k])
        pc = self.X @ T_cw[:3, :3].T + T_cw[:3, 3]
        z = pc[:, 2]
        uv = (pc[:, :2] / np.maximum(z, 1e-9)[:, None]) * [KITTI_K[0, 0], KITTI_K[1, 1]] + [KITTI_K[0, 2], KITTI_K[1, 2]]
        vis = (z > 1) & (uv[:, 0] >= 0) & (uv[:, 0] < KITTI_WH[0]) & (uv[:, 1] >= 0) & (uv[:, 1] < KITTI_WH[1])
        lm = self.rng.permutation(np.nonzero(vis)[0])
        uv = uv[lm] + self.rng.normal(0, self.noise, (lm.size, 2))
        return {"keypoints": uv[None].astype(np.float32), "descriptors": None, "lm": lm}


def drive(vo, scene, create_keyframe, pose_noise=0.02, seed=5):
    """Feed keyframes 1..n-1 through ``create_keyframe`` (the hook or the plain double)."""
    rng = np.random.default_rng(seed)
    vo.scene = scene
    f0 = scene.keypoints(0)
    vo.keyframe = {"feats": f0, "ids": np.full(f0["lm"].size, -1), "T_wc": scene.T_wc[0].copy()}
    for k in range(1, scene.n_kf):
        prev = vo.keyframe
        cur = scene.keypoints(k)
        pos = {lm: i for i, lm in enumerate(cur["lm"])}
        ref_idx = np.array([i for i, lm in enumerate(prev["feats"]["lm"]) if lm in pos], int)
        cur_idx = np.array([pos[prev["feats"]["lm"][i]] for i in ref_idx], int)
        curr_ids = np.full(cur["lm"].size, -1)
        carried = prev["ids"][ref_idx]
        ok = (carried >= 0) & np.array([c in vo.map_points for c in carried], bool)
        curr_ids[cur_idx[ok]] = carried[ok]  # PnP inliers carry the id (vo.py:206-210)
        T = scene.T_wc[k].copy()
        if k >= 2:
            T[:3, 3] += rng.normal(0, pose_noise, 3)
        vo.T_wc = T
        create_keyframe(vo, cur, curr_ids, ref_idx, cur_idx)
