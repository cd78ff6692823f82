"""Drop-in hooks on CPU: window assembly, write-back, method patching."""

import types

import numpy as np
import pytest

from oracle import ba_ref
from tests.vo_scene import Cfg, FakeVO, Scene, drive
from visualodometry_amd import _lib
from visualodometry_amd.ba import BAResult, csr_from_obs_pt
from visualodometry_amd import sift
from visualodometry_amd.dropin import hooks


class OracleBA:
    """Stands in for SlidingWindowBA on CPU: the numpy oracle, same window contract."""

    def __init__(self, K, iters=10, lam=1.0):
        self.K, self.iters, self.lam = K, iters, lam
        self.windows = []

    def optimize(self, w):
        self.windows.append(w)
        order, ptr = csr_from_obs_pt(w.points.shape[0], w.obs_pt)
        s = ba_ref.BAStructure(self.K, ptr, w.obs_cam[order], w.obs_uv[order], w.n_fixed, w.poses_cw.shape[0])
        st, costs = ba_ref.solve(ba_ref.BAState.from_poses(w.poses_cw, w.points), s, self.iters, self.lam)
        return BAResult(st.poses_cw(), st.X, costs, "ok")


def _hooked(vo_cls):
    return hooks._wrap_create_keyframe(vo_cls._create_keyframe)


def test_window_observations_match_the_scene():
    scene = Scene(n_kf=8, n_pts=500)
    vo = FakeVO(Cfg(ba_enabled=False))
    drive(vo, scene, _hooked(FakeVO))
    win = vo._vo_amd_window
    assert len(win.frames) == 8  # the keyframe before the first hook call is included
    w, lm_ids = win.build(vo.map_points)
    assert w.poses_cw.shape == (8, 4, 4) and w.points.shape[0] == lm_ids.size
    # every observation is the (noisy) projection of the true landmark behind its id
    for o in range(w.obs_cam.size):
        k, i = w.obs_cam[o], lm_ids[w.obs_pt[o]]
        T_cw = np.linalg.inv(scene.T_wc[k])
        pc = T_cw[:3, :3] @ scene.X[vo.truth[int(i)]] + T_cw[:3, 3]
        uv = pc[:2] / pc[2] * [vo.K[0, 0], vo.K[1, 1]] + [vo.K[0, 2], vo.K[1, 2]]
        assert np.abs(w.obs_uv[o] - uv).max() < 5.0, (k, i)
    # each landmark seen in >= 2 distinct keyframes, <= max_track, and the triangulating
    # previous keyframe contributes its ray
    for j in range(lm_ids.size):
        kfs = np.unique(w.obs_cam[w.obs_pt == j])
        assert 2 <= kfs.size <= win.max_track
    assert np.all(w.poses_cw[:, 3, 3] == 1)


def test_two_view_landmarks_get_the_previous_keyframe_ray():
    scene = Scene(n_kf=3, n_pts=300)
    vo = FakeVO(Cfg(ba_enabled=False))
    drive(vo, scene, _hooked(FakeVO))
    w, lm_ids = vo._vo_amd_window.build(vo.map_points)
    # points created at keyframe 1 are observed by keyframes 0 and 1
    born1 = [j for j, i in enumerate(lm_ids) if i < 10]
    assert born1
    for j in born1:
        assert set(w.obs_cam[w.obs_pt == j]) >= {0, 1}


def test_ba_hook_reduces_error_and_writes_back():
    scene = Scene(n_kf=10, n_pts=600)
    vo = FakeVO(Cfg(ba_enabled=True))
    vo._vo_amd_ba = OracleBA(vo.K, iters=8, lam=1.0)
    drive(vo, scene, _hooked(FakeVO), pose_noise=0.05)
    assert len(vo._vo_amd_ba.windows) == 8  # the first call has only the 2 fixed keyframes
    res = vo._vo_amd_last_ba
    assert res.status == "ok" and res.cost_per_iter[-1] < res.cost_per_iter[0]
    # state written back: VO pose == last window pose, keyframe pose too
    last = vo._vo_amd_window.frames[-1].T_wc
    np.testing.assert_array_equal(vo.T_wc, last)
    np.testing.assert_array_equal(vo.keyframe["T_wc"], last)
    # positions of the adjusted keyframes are closer to the truth than the noisy inputs
    err = [np.linalg.norm(fr.T_wc[:3, 3] - scene.T_wc[k, :3, 3]) for k, fr in enumerate(vo._vo_amd_window.frames)]
    assert np.mean(err[2:]) < 0.05
    assert all(isinstance(v, np.ndarray) and v.dtype == np.float32 for v in vo.map_points.values())


def test_window_slides_and_resets():
    scene = Scene(n_kf=9, n_pts=400)
    vo = FakeVO(Cfg(ba_enabled=False, ba_window=4))
    drive(vo, scene, _hooked(FakeVO))
    assert len(vo._vo_amd_window.frames) == 4
    hooks._wrap_reset(FakeVO._reset_system)(vo)
    assert len(vo._vo_amd_window.frames) == 0
    assert vo._vo_amd_window.build(vo.map_points) == (None, None)


def test_max_track_caps_distinct_keyframes():
    win = hooks.KeyframeWindow(size=20, n_fixed=2, max_track=3)
    mp = {7: np.zeros(3), 8: np.ones(3)}
    for k in range(6):
        win.add(np.eye(4), [[k, k], [k, -k]], [7, 8 if k < 1 else -1])
    w, ids = win.build(mp)
    assert list(ids) == [7]  # landmark 8 is seen once
    assert sorted(w.obs_cam.tolist()) == [3, 4, 5]


class _Front:
    def __init__(self, kind):
        self.conf = Cfg(extractor_type=kind)

    def match_frames(self, f0, f1):
        return "original"

    def process_image(self, img):
        return "original"


def test_match_frames_routing():
    patched = hooks._wrap_match_frames(_Front.match_frames)
    assert patched(_Front("superpoint"), {}, {}) == "original"
    from tests.conftest import gpu_available

    if gpu_available():
        pytest.skip("GPU present: routing covered by the GPU tests")
    d = {"descriptors": np.zeros((1, 5, 128), np.float32)}
    with pytest.raises(_lib.VoError):  # the SIFT branch goes to the HIP library, never a CPU path
        patched(_Front("sift"), d, d)


def test_frontend_init_swaps_in_the_gpu_sift():
    class FrontSift:
        def __init__(self, config):
            self.conf = config
            self.extractor = "cv2.SIFT"

    patched = hooks._wrap_frontend_init(FrontSift.__init__)
    cfg = types.SimpleNamespace(extractor_type="sift", sift_n_features=4000, sift_contrast_threshold=0.02,
                                sift_edge_threshold=2.0,
                                sift_sigma=1.6)
    f = FrontSift.__new__(FrontSift)
    patched(f, cfg)
    from visualodometry_amd import sift

    assert isinstance(f.extractor, sift.SIFT)
    assert (f.extractor.nfeatures, f.extractor.contrast, f.extractor.edge, f.extractor.sigma) == (4000, 0.02, 2.0, 1.6)
    f = FrontSift.__new__(FrontSift)
    patched(f, types.SimpleNamespace(extractor_type="sift", sift_on_gpu=False))
    assert f.extractor == "cv2.SIFT"
    f = FrontSift.__new__(FrontSift)
    patched(f, types.SimpleNamespace(extractor_type="superpoint"))
    assert f.extractor == "cv2.SIFT"


def test_process_image_routing():
    """The process_image hook takes the GPU-tensor path only for the drop-in's SIFT extractor
    on a CUDA device and a single-channel image; everything else runs the reference's body."""
    import types

    patched = hooks._wrap_process_image(_Front.process_image)
    f = _Front("sift")
    assert patched(f, np.zeros((4, 4), np.uint8)) == "original"  # extractor is not the drop-in's
    f.extractor = sift.SIFT_create(nfeatures=10)
    f.device = types.SimpleNamespace(type="cpu")
    assert patched(f, np.zeros((4, 4), np.uint8)) == "original"  # torch on the CPU
    f.device = types.SimpleNamespace(type="cuda")
    assert patched(f, np.zeros((4, 4, 3), np.uint8)) == "original"  # colour: the reference converts it


def test_install_is_idempotent():
    class F(_Front):
        pass

    class V(FakeVO):
        pass

    hooks.install(F, V)
    m1, k1, p1 = F.match_frames, V._create_keyframe, F.process_image
    hooks.install(F, V)
    assert F.match_frames is m1 and V._create_keyframe is k1 and F.process_image is p1
    assert V._create_keyframe._vo_amd_wrapped is FakeVO._create_keyframe


def test_env_switches(monkeypatch):
    import sys

    from tests.conftest import ROOT

    sys.path.insert(0, str(ROOT / "visualodometry_amd" / "dropin"))
    from config.config import get_config

    monkeypatch.setenv("VO_AMD_EXTRACTOR", "sift")
    monkeypatch.setenv("VO_AMD_BA", "1")
    c = get_config("kitti")
    assert c.extractor_type == "sift" and c.ba_enabled and c.sift_n_features == 4000


def test_install_patches_triangulate_points_in_both_modules():
    """``vo.py`` imports ``triangulate_points`` by name (vo.py:6): install() replaces it in
    the frontend module and in the VO module; with ``triangulate_on_gpu`` off the
    original runs, otherwise the HIP library (no CPU path)."""
    import sys
    import types

    calls = []

    def orig(T1, T2, p1, p2, K, cfg):
        calls.append(1)
        return "orig"

    fm, vm = types.ModuleType("_fake_frontend_mod"), types.ModuleType("_fake_vo_mod")
    fm.triangulate_points = orig
    vm.triangulate_points = orig
    F = type("F", (_Front,), {"__module__": fm.__name__})
    V = type("V", (FakeVO,), {"__module__": vm.__name__})
    sys.modules[fm.__name__], sys.modules[vm.__name__] = fm, vm
    try:
        hooks.install(F, V)
        hooks.install(F, V)  # idempotent
        for m in (fm, vm):
            assert m.triangulate_points._vo_amd_wrapped is orig
            off = types.SimpleNamespace(triangulate_on_gpu=False)
            assert m.triangulate_points(None, None, [], [], None, off) == "orig"
        on = types.SimpleNamespace(triangulate_on_gpu=True, min_depth=0.001, max_reproj_err=6.0)
        # empty input returns before touching the device, as the reference does
        pts, mask = fm.triangulate_points(np.eye(4), np.eye(4), np.zeros((0, 2)), np.zeros((0, 2)), np.eye(3), on)
        assert pts.shape == (0, 3) and mask.shape == (0,)
        with pytest.raises(_lib.VoError):  # a real call needs the HIP device: never a CPU path
            fm.triangulate_points(np.eye(4), np.eye(4), np.ones((3, 2)), np.ones((3, 2)), np.eye(3), on)
    finally:
        del sys.modules[fm.__name__], sys.modules[vm.__name__]
