"""Runtime hooks that put the MI355X matcher and BA under the reference's VO loop.

Nothing of the reference is copied: :func:`install` patches methods of the
reference's own classes and names of its modules once they are imported (cv2 etc.
are the caller's environment):

* ``FeatureFrontend.__init__`` (reference ``src/modules/frontend.py:10-34``): with the SIFT
  extractor and ``cfg.sift_on_gpu`` (default on), ``self.extractor`` becomes
  :func:`visualodometry_amd.sift.SIFT_create` with the same nfeatures / contrast / edge /
  sigma, so ``process_image`` (``:51-75``) runs detectAndCompute on the MI355X.
* ``FeatureFrontend.match_frames`` (reference ``src/modules/frontend.py:78-113``),
  SIFT branch -> :func:`visualodometry_amd.matcher.match_knn2_ratio`.  The
  LightGlue branch (``:80-84``) is left to the original method.
* ``triangulate_points`` (``src/modules/frontend.py:115-148``, imported by name into
  ``vo.py``) -> :func:`visualodometry_amd.triangulate.triangulate_points` in both
  modules (``cfg.triangulate_on_gpu``, default on).
* ``VisualOdometry._create_keyframe`` (``src/modules/vo.py:252-288``) is wrapped:
  the original triangulates and rotates the keyframe, then
  :class:`KeyframeWindow` records the new keyframe and, if ``cfg.ba_enabled``,
  runs :class:`~visualodometry_amd.ba.SlidingWindowBA` on the last
  ``cfg.ba_window`` keyframes and writes poses and map points back
  (SURVEY.md §8a row a11).

The reference keeps only the current keyframe's observation of a freshly
triangulated point (``vo.py:277-284``); the window also records the previous
keyframe's observation of it (the other ray of the triangulation), which is
what makes a two-keyframe landmark constrain BA at all.
"""

from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field

import numpy as np

from ..ba import BAResult, BAWindow, SlidingWindowBA
from ..mapstore import MAX_POINTS, MapStore


def _np(x) -> np.ndarray:
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def _keypoints(feats: dict) -> np.ndarray:
    kp = _np(feats["keypoints"])
    return kp[0] if kp.ndim == 3 else kp


@dataclass
class KeyframeRecord:
    T_wc: np.ndarray  # (4,4) f64 camera -> world (the reference's pose storage, vo.py:19)
    uv: np.ndarray  # (N,2) f32 keypoints
    ids: np.ndarray  # (N,) int landmark id per keypoint, -1 if none
    extra_uv: list = field(default_factory=list)  # observations added after the keyframe was made
    extra_ids: list = field(default_factory=list)


class KeyframeWindow:
    """The last ``size`` keyframes and their landmark observations.

    ``max_track`` caps the observations of one landmark to its most recent
    keyframes: the BA planner handles at most 10 free cameras per landmark
    (DESIGN.md §BA layout).
    """

    def __init__(self, size: int = 50, n_fixed: int = 2, max_track: int = 10):
        self.size = int(size)
        self.n_fixed = int(n_fixed)
        self.max_track = int(max_track)
        self.frames: deque[KeyframeRecord] = deque(maxlen=self.size)

    def reset(self) -> None:
        self.frames.clear()

    def add(self, T_wc, uv, ids, prev_uv=None, prev_ids=None) -> None:
        """Append a keyframe; ``prev_uv/prev_ids`` are new observations of the previous keyframe."""
        if prev_ids is not None and len(prev_ids) and self.frames:
            last = self.frames[-1]
            last.extra_uv.append(np.asarray(prev_uv, np.float32).reshape(-1, 2))
            last.extra_ids.append(np.asarray(prev_ids, np.int64))
        self.frames.append(KeyframeRecord(np.array(T_wc, np.float64), np.asarray(uv, np.float32).reshape(-1, 2),
                                          np.array(ids, np.int64)))

    def observations(self, map_points: dict):
        """-> (obs_kf, obs_uv, obs_id) of every window observation of a landmark still in the map."""
        kf, uv, pid = [], [], []
        for k, fr in enumerate(self.frames):
            us = [fr.uv] + fr.extra_uv
            ids = [fr.ids] + fr.extra_ids
            u = np.concatenate(us)
            i = np.concatenate(ids)
            if isinstance(map_points, MapStore):
                keep = map_points.contains(i)
            else:
                keep = (i >= 0) & np.fromiter((int(x) in map_points for x in i), bool, i.size)
            kf.append(np.full(int(keep.sum()), k, np.int32))
            uv.append(u[keep])
            pid.append(i[keep])
        if not kf:
            return np.zeros(0, np.int32), np.zeros((0, 2), np.float32), np.zeros(0, np.int64)
        return np.concatenate(kf), np.concatenate(uv), np.concatenate(pid)

    def build(self, map_points: dict):
        """-> (BAWindow, landmark ids) or (None, None) if the window has nothing to adjust."""
        if len(self.frames) <= self.n_fixed:
            return None, None
        kf, uv, pid = self.observations(map_points)
        if pid.size == 0:
            return None, None
        # group by landmark, newest keyframe first; rank the distinct keyframes of each landmark
        order = np.lexsort((-kf, pid))
        kf, uv, pid = kf[order], uv[order], pid[order]
        new_pt = np.r_[True, pid[1:] != pid[:-1]]
        new_kf = new_pt | np.r_[True, kf[1:] != kf[:-1]]
        grp = np.cumsum(new_pt) - 1
        c = np.cumsum(new_kf)
        kf_rank = c - c[new_pt][grp]  # 0 = newest keyframe of this landmark
        keep = kf_rank < self.max_track
        kf, uv, pid, grp, new_kf = kf[keep], uv[keep], pid[keep], grp[keep], new_kf[keep]
        ids = pid[new_pt[keep]]  # the newest keyframe of every landmark is always kept
        n_kf = np.bincount(grp, weights=new_kf, minlength=ids.size)
        inv = grp
        good = n_kf >= 2  # a landmark needs two distinct keyframes to be constrained
        if not good.any():
            return None, None
        sel = good[inv]
        kf, uv, inv = kf[sel], uv[sel], inv[sel]
        remap = -np.ones(ids.size, np.int64)
        remap[good] = np.arange(int(good.sum()))
        lm_ids = ids[good]
        if isinstance(map_points, MapStore):
            points = map_points.gather(lm_ids).astype(np.float64)
        else:
            points = np.stack([np.asarray(map_points[int(i)], np.float64).reshape(3) for i in lm_ids])
        poses_cw = np.stack([np.linalg.inv(fr.T_wc) for fr in self.frames])
        w = BAWindow(poses_cw=poses_cw, points=points, obs_uv=uv.astype(np.float32), obs_cam=kf.astype(np.int32),
                     obs_pt=remap[inv].astype(np.int32), n_fixed=self.n_fixed)
        return w, lm_ids

    def write_back(self, res: BAResult, lm_ids, map_points: dict) -> None:
        for fr, P in zip(self.frames, res.poses_cw):
            fr.T_wc = np.linalg.inv(P)
        if isinstance(map_points, MapStore):
            map_points.scatter(lm_ids, res.points)
            return
        for i, X in zip(lm_ids, res.points):
            old = map_points[int(i)]
            map_points[int(i)] = np.asarray(X, dtype=np.asarray(old).dtype).reshape(np.shape(old))


def _wrap_create_keyframe(orig):
    def _create_keyframe(self, curr_feats, curr_ids, ref_indices, curr_indices):
        cfg = self.cfg
        win = getattr(self, "_vo_amd_window", None)
        if win is None:
            win = KeyframeWindow(getattr(cfg, "ba_window", 50), getattr(cfg, "ba_fixed", 2))
            self._vo_amd_window = win
        prev = self.keyframe
        if prev is not None and not win.frames:  # the window starts at the keyframe before the first
            win.add(prev["T_wc"], _keypoints(prev["feats"]), prev["ids"])
        first_new = self.next_pt_id
        ref_indices = np.asarray(ref_indices)
        curr_indices = np.asarray(curr_indices)
        no_id = curr_ids[curr_indices] == -1
        orig(self, curr_feats, curr_ids, ref_indices, curr_indices)
        # the previous keyframe saw every newly triangulated point (vo.py:265-284)
        cand = curr_indices[no_id]
        new_ids = curr_ids[cand]
        # a current keypoint matched by several reference keypoints (no cross-check,
        # frontend.py:34) had its id overwritten in the loop: its other ray is ambiguous
        uniq, cnt = np.unique(cand, return_counts=True)
        is_new = (new_ids >= first_new) & np.isin(cand, uniq[cnt == 1])
        prev_uv = _keypoints(prev["feats"])[ref_indices[no_id][is_new]] if prev is not None else None
        win.add(self.T_wc, _keypoints(curr_feats), curr_ids, prev_uv, new_ids[is_new])
        if getattr(cfg, "ba_enabled", False):
            self._vo_amd_last_ba = run_window_ba(self, win)

    _create_keyframe._vo_amd_wrapped = orig
    return _create_keyframe


def run_window_ba(vo, win: KeyframeWindow):
    """Adjust the window and write poses/points back into the VO state; never raises on bad windows."""
    window, lm_ids = win.build(vo.map_points)
    if window is None:
        return None
    cfg = vo.cfg
    ba = getattr(vo, "_vo_amd_ba", None)
    if ba is None:
        ba = SlidingWindowBA(vo.K, cfg)
        vo._vo_amd_ba = ba
    res = ba.optimize(window)
    if res.status != "ok" or not np.all(np.isfinite(res.cost_per_iter)) or \
            res.cost_per_iter[-1] > res.cost_per_iter[0]:
        print(f"BA: window rejected ({res.status} {res.message})")
        return res
    win.write_back(res, lm_ids, vo.map_points)
    T_wc = win.frames[-1].T_wc.copy()
    vo.T_wc = T_wc
    vo.keyframe["T_wc"] = T_wc.copy()
    vo.last_pos = T_wc[:3, 3].copy()
    return res


def _use_map_store(vo) -> None:
    if getattr(vo.cfg, "map_store_arrays", True) and not isinstance(vo.map_points, MapStore):
        store = MapStore()
        for pid, X in vo.map_points.items():
            store[pid] = X
        vo.map_points = store


def _wrap_init(orig):
    def __init__(self, *args, **kw):  # VisualOdometry(K, config), vo.py:9
        orig(self, *args, **kw)
        _PNP_ON_GPU[0] = bool(getattr(self.cfg, "pnp_on_gpu", True))
        _use_map_store(self)
        if getattr(self.cfg, "ba_enabled", False):
            # the BA context pre-sized for a full window (ba_window keyframes, the map's
            # MAX_POINTS cap, vo.py:38) now, so no keyframe call of the drive pays for it
            self._vo_amd_ba = SlidingWindowBA(self.K, self.cfg)
            self._vo_amd_ba.reserve(getattr(self.cfg, "ba_window", 50), MAX_POINTS,
                                    n_fixed=getattr(self.cfg, "ba_fixed", 2))

    __init__._vo_amd_wrapped = orig
    return __init__


def _wrap_prune(orig):
    def _prune_map(self):
        if isinstance(self.map_points, MapStore):
            self.map_points.prune_below(self.next_pt_id - MAX_POINTS)  # vo.py:38-47
        else:
            orig(self)

    _prune_map._vo_amd_wrapped = orig
    return _prune_map


def _wrap_reset(orig):
    def _reset_system(self):
        orig(self)
        _use_map_store(self)
        win = getattr(self, "_vo_amd_window", None)
        if win is not None:
            win.reset()

    _reset_system._vo_amd_wrapped = orig
    return _reset_system


_PNP_ON_GPU = [True]  # set from the VO config at construction (cfg.pnp_on_gpu)


def _wrap_frontend_init(orig):
    from .. import sift

    def __init__(self, config, *args, **kw):  # FeatureFrontend(config), frontend.py:10
        orig(self, config, *args, **kw)
        if getattr(config, "extractor_type", None) == "sift" and getattr(config, "sift_on_gpu", True):
            self.extractor = sift.SIFT_create(nfeatures=config.sift_n_features,
                                              contrastThreshold=config.sift_contrast_threshold,
                                              edgeThreshold=config.sift_edge_threshold, sigma=config.sift_sigma)

    __init__._vo_amd_wrapped = orig
    return __init__


def _wrap_process_image(orig):
    from .. import sift

    def process_image(self, img):  # FeatureFrontend.process_image, frontend.py:36-75
        ext = getattr(self, "extractor", None)
        dev = getattr(self, "device", None)
        if isinstance(ext, sift.SIFT) and getattr(dev, "type", None) == "cuda" and np.ndim(img) == 2:
            # the SIFT branch (:51-75) keeps k.pt and the descriptors and moves both to the GPU:
            # the kernels write them into torch's memory there, no keypoint objects on the host
            import torch

            r = sift.detect_and_compute_torch(img, ext.nfeatures, ext.contrast, ext.edge, ext.sigma, ext.n_layers,
                                              device=dev, ctx=ext._ctx or None)
            if r is not None:
                pts, des = r
                return {
                    "keypoints": pts.unsqueeze(0),  # (1, N, 2)
                    "descriptors": des.unsqueeze(0),  # (1, N, 128)
                    "image_size": torch.tensor([(img.shape[1], img.shape[0])]).to(dev),
                }
        return orig(self, img)

    process_image._vo_amd_wrapped = orig
    return process_image


def _wrap_match_frames(orig):
    from .. import matcher

    def match_frames(self, feats0, feats1):
        if getattr(self.conf, "extractor_type", None) == "sift" and getattr(self.conf, "match_on_gpu", True):
            # SIFT integers: the int8 path only, hinted for this call (the context's own hint,
            # which other users of the context may rely on, is restored afterwards)
            # feats0 is the keyframe's (vo.py:64-65): its packed rows stay cached across frames
            return matcher.match_knn2_ratio(feats0["descriptors"], feats1["descriptors"],
                                            kind=matcher.DESC_SIFT, cache_query=True)
        return orig(self, feats0, feats1)

    match_frames._vo_amd_wrapped = orig
    return match_frames


def _wrap_triangulate(orig):
    from .. import triangulate

    def triangulate_points(T_cw1, T_cw2, pts1, pts2, K, config):
        if getattr(config, "triangulate_on_gpu", True):
            return triangulate.triangulate_points(T_cw1, T_cw2, pts1, pts2, K, config)
        return orig(T_cw1, T_cw2, pts1, pts2, K, config)

    triangulate_points._vo_amd_wrapped = orig
    return triangulate_points


class Cv2Proxy:
    """Stands in for the ``cv2`` module inside ``modules.vo``: ``solvePnPRansac`` runs on
    the MI355X, every other attribute is the real cv2's."""

    def __init__(self, real, enabled=lambda: True):
        self._vo_amd_real = real
        self._enabled = enabled

    def __getattr__(self, name):
        return getattr(self._vo_amd_real, name)

    def solvePnPRansac(self, objectPoints, imagePoints, cameraMatrix, distCoeffs=None, *args, **kw):
        if self._enabled():
            from .. import pnp

            return pnp.solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, *args, **kw)
        return self._vo_amd_real.solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, *args, **kw)


def install(frontend_cls=None, vo_cls=None) -> None:
    """Patch the reference classes (imported from ``modules.*`` when not given). Idempotent.

    ``triangulate_points`` (``frontend.py:115``) is a module function that ``vo.py``
    imports by name (``vo.py:6``), so it is replaced in both modules.
    """
    import sys

    if frontend_cls is None:
        from modules.frontend import FeatureFrontend as frontend_cls  # the reference's module
    if vo_cls is None:
        from modules.vo import VisualOdometry as vo_cls
    for name in dict.fromkeys((frontend_cls.__module__, vo_cls.__module__)):
        mod = sys.modules.get(name)
        f = getattr(mod, "triangulate_points", None) if mod is not None else None
        if f is not None and not hasattr(f, "_vo_amd_wrapped"):
            mod.triangulate_points = _wrap_triangulate(f)
    if not hasattr(frontend_cls.__init__, "_vo_amd_wrapped"):
        frontend_cls.__init__ = _wrap_frontend_init(frontend_cls.__init__)
    if not hasattr(frontend_cls.match_frames, "_vo_amd_wrapped"):
        frontend_cls.match_frames = _wrap_match_frames(frontend_cls.match_frames)
    pi = getattr(frontend_cls, "process_image", None)
    if pi is not None and not hasattr(pi, "_vo_amd_wrapped"):
        frontend_cls.process_image = _wrap_process_image(pi)
    if not hasattr(vo_cls._create_keyframe, "_vo_amd_wrapped"):
        vo_cls._create_keyframe = _wrap_create_keyframe(vo_cls._create_keyframe)
    if not hasattr(vo_cls._reset_system, "_vo_amd_wrapped"):
        vo_cls._reset_system = _wrap_reset(vo_cls._reset_system)
    if not hasattr(vo_cls.__init__, "_vo_amd_wrapped"):
        vo_cls.__init__ = _wrap_init(vo_cls.__init__)
    if hasattr(vo_cls, "_prune_map") and not hasattr(vo_cls._prune_map, "_vo_amd_wrapped"):
        vo_cls._prune_map = _wrap_prune(vo_cls._prune_map)
    vo_mod = sys.modules.get(vo_cls.__module__)
    real_cv2 = getattr(vo_mod, "cv2", None) if vo_mod is not None else None
    if real_cv2 is not None and not isinstance(real_cv2, Cv2Proxy):
        vo_mod.cv2 = Cv2Proxy(real_cv2, lambda: _PNP_ON_GPU[0])
