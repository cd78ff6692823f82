"""Drop-in hooks end to end on the MI355X: keyframe hook -> HIP BA, SIFT branch -> HIP matcher."""

import copy

import numpy as np
import pytest

from oracle import match_ref
from tests.test_dropin_hooks import OracleBA, _Front
from tests.vo_scene import Cfg, FakeVO, Scene, drive
from visualodometry_amd.dropin import hooks
from visualodometry_amd.synthetic import sift_like_pair

pytestmark = pytest.mark.gpu


def test_keyframe_hook_hip_ba_matches_oracle(ctx):
    scene = Scene(n_kf=10, n_pts=600)
    cfg = Cfg(ba_enabled=True, ba_iters=8, ba_lambda=1.0)
    gpu = FakeVO(cfg)
    cpu = FakeVO(copy.deepcopy(cfg))
    cpu._vo_amd_ba = OracleBA(cpu.K, iters=8, lam=1.0)
    drive(gpu, Scene(n_kf=10, n_pts=600), hooks._wrap_create_keyframe(FakeVO._create_keyframe), pose_noise=0.05)
    drive(cpu, scene, hooks._wrap_create_keyframe(FakeVO._create_keyframe), pose_noise=0.05)
    rg, rc = gpu._vo_amd_last_ba, cpu._vo_amd_last_ba
    assert rg.status == "ok"
    np.testing.assert_allclose(rg.cost_per_iter, rc.cost_per_iter, rtol=1e-5)
    np.testing.assert_allclose(gpu.T_wc, cpu.T_wc, rtol=1e-5, atol=1e-8)
    ids = sorted(cpu.map_points)
    assert ids == sorted(gpu.map_points)
    a = np.stack([gpu.map_points[i] for i in ids]).astype(np.float64)
    b = np.stack([cpu.map_points[i] for i in ids]).astype(np.float64)
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5)


def test_patched_match_frames_uses_hip_matcher(ctx):
    d0, d1 = sift_like_pair(700, 800, 4)
    patched = hooks._wrap_match_frames(_Front.match_frames)
    got = patched(_Front("sift"), {"descriptors": d0[None]}, {"descriptors": d1[None]})
    np.testing.assert_array_equal(got, match_ref.match_int(d0, d1))
    assert got.dtype == np.int64 and got.shape[1] == 2
