"""Drop-in config vs the reference snapshot; host-side BA planner invariants."""

import dataclasses
import json
import sys

import numpy as np
import pytest

from tests.conftest import GOLDEN, ROOT
from visualodometry_amd import _lib
from visualodometry_amd.ba import csr_from_obs_pt, plan_probe
from visualodometry_amd.synthetic import KITTI_K, make_ba_config, make_ba_problem

sys.path.insert(0, str(ROOT / "visualodometry_amd" / "dropin"))
from config.config import VOConfig, get_config  # noqa: E402

REF = json.loads((GOLDEN / "reference_config.json").read_text())


@pytest.mark.parametrize("dataset", ["kitti", "malaga", "parking", "own", "unknown"])
def test_get_config_matches_reference(dataset):
    ours = dataclasses.asdict(get_config(dataset))
    for k, v in REF["get_config"][dataset].items():
        assert ours[k] == v, (dataset, k)


def test_defaults_match_and_ba_is_off():
    ours = dataclasses.asdict(VOConfig())
    for k, v in REF["VOConfig_defaults"].items():
        assert ours[k] == v
    assert ours["ba_enabled"] is False


def test_sift_extension_applies_the_unreachable_branch():
    c = get_config("kitti", extractor_type="sift")
    assert c.extractor_type == "sift" and c.sift_n_features == 4000
    assert get_config("kitti").sift_n_features == REF["get_config"]["kitti"]["sift_n_features"]


def test_synthetic_uses_the_reference_kitti_K():
    np.testing.assert_array_equal(KITTI_K, np.array(REF["K"]["kitti"]))


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg4"])
def test_plan_limits(cfg):
    p = make_ba_config(cfg)
    st = plan_probe(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 512)
    assert st["track_entries"] == p.n_obs  # synthetic windows have no duplicate (landmark, camera)
    assert st["max_chunk_pairs"] <= 1024
    assert st["max_segment_slots"] <= 64 and st["max_segment_cameras"] <= 32
    assert 1 <= st["segments"] <= st["chunks"]


def test_plan_rejects_too_wide_landmark():
    p = make_ba_problem(16, 10, 3)
    L = p.n_points
    cams = np.concatenate([p.obs_cam, np.arange(16, dtype=np.int32)])  # landmark L sees 16 cameras
    uv = np.concatenate([p.obs_uv, np.zeros((16, 2), np.float32)])
    ptr = np.concatenate([p.point_ptr, [p.point_ptr[-1] + 16]]).astype(np.int32)
    with pytest.raises(_lib.VoError) as e:
        plan_probe(p.K, ptr, cams, uv, 16, 2)
    assert e.value.code == _lib.VO_ERR_ARG and "too wide" in str(e.value)
    assert L == p.n_points


def test_csr_from_obs_pt_is_stable():
    obs_pt = np.array([2, 0, 1, 0, 2, 2])
    order, ptr = csr_from_obs_pt(3, obs_pt)
    np.testing.assert_array_equal(order, [1, 3, 2, 0, 4, 5])
    np.testing.assert_array_equal(ptr, [0, 2, 3, 6])


def test_plan_digests_pinned():
    """The static BA plan (chunks, segments, slab layout, pair lists, profile, K3 tables)
    is bitwise the one recorded in tests/golden/plan_digests.json: planner changes must
    not move any kernel's summation order (tests/golden/make_plan_digests.py)."""
    import json
    import sys

    from tests.conftest import ROOT

    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import make_plan_digests

    want = json.loads((ROOT / "tests" / "golden" / "plan_digests.json").read_text())
    assert make_plan_digests.digests() == want


def test_plan_digest_independent_of_concurrent_planners():
    """Plans built by several host threads at once (one takes the persistent planner pool,
    the others start their own threads: ba_plan.cpp PlanPool) are the same plan as one
    built alone -- the parallel planner writes disjoint, precomputed ranges only."""
    from concurrent.futures import ThreadPoolExecutor

    from visualodometry_amd.ba import plan_digest

    p = make_ba_config("cfg3")
    alone = plan_digest(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1024)
    with ThreadPoolExecutor(4) as ex:
        got = list(ex.map(lambda _: plan_digest(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1024),
                          range(8)))
    assert got == [alone] * 8


def test_csr_from_obs_pt_rejects_out_of_range():
    with pytest.raises(ValueError):
        csr_from_obs_pt(3, np.array([0, 3]))
    with pytest.raises(ValueError):
        csr_from_obs_pt(3, np.array([-1, 0]))


def test_group_window_passes_grouped_windows_through():
    """Windows built landmark by landmark keep their arrays; others are reordered stably."""
    from visualodometry_amd.ba import BAWindow, group_window

    obs_pt = np.array([0, 0, 1, 2, 2, 2])
    cam = np.arange(6, dtype=np.int32)
    uv = np.arange(12, dtype=np.float32).reshape(6, 2)
    w = BAWindow(np.zeros((3, 4, 4)), np.zeros((3, 3)), uv, cam, obs_pt, 1)
    ptr_, cam2, uv2 = group_window(3, w)
    np.testing.assert_array_equal(ptr_, [0, 2, 3, 6])
    assert cam2 is w.obs_cam or np.shares_memory(cam2, w.obs_cam)
    perm = np.array([3, 0, 5, 2, 1, 4])
    w2 = BAWindow(np.zeros((3, 4, 4)), np.zeros((3, 3)), uv[perm], cam[perm], obs_pt[perm], 1)
    ptr2, cam3, uv3 = group_window(3, w2)
    np.testing.assert_array_equal(ptr2, [0, 2, 3, 6])
    np.testing.assert_array_equal(cam3, [0, 1, 2, 3, 5, 4])  # stable within a landmark
    np.testing.assert_array_equal(uv3, uv[[0, 1, 2, 3, 5, 4]])


def test_group_by_point_grouped_check():
    """vo_ba_group_by_point with order == NULL: point_ptr of an already grouped window
    (empty landmarks included), 1 for an ungrouped one, VO_ERR_ARG out of range."""
    import ctypes as C

    from visualodometry_amd import _lib
    from visualodometry_amd._lib import ptr

    lib = _lib.load()

    def call(n_points, obs_pt):
        x = np.ascontiguousarray(obs_pt, dtype=np.int32)
        pp = np.full(n_points + 1, -7, dtype=np.int32)
        return lib.vo_ba_group_by_point(n_points, x.size, ptr(x, C.c_int32), None, ptr(pp, C.c_int32)), pp

    rc, pp = call(6, [1, 1, 3, 3, 3])
    assert rc == _lib.VO_OK
    np.testing.assert_array_equal(pp, [0, 0, 2, 2, 5, 5, 5])
    rc, pp = call(3, [])
    assert rc == _lib.VO_OK
    np.testing.assert_array_equal(pp, [0, 0, 0, 0])
    assert call(3, [0, 2, 1])[0] == 1
    assert call(3, [0, 3])[0] == _lib.VO_ERR_ARG
    assert call(3, [-1, 0])[0] == _lib.VO_ERR_ARG
    rng = np.random.default_rng(3)
    obs_pt = np.sort(rng.integers(0, 500, 4000))
    rc, pp = call(500, obs_pt)
    assert rc == _lib.VO_OK
    np.testing.assert_array_equal(pp[1:], np.cumsum(np.bincount(obs_pt, minlength=500)))


def test_plan_in_forked_child():
    """A child forked after the planner pool started (its threads do not survive fork)
    still plans, and gets the same plan."""
    import os
    import signal

    from visualodometry_amd.ba import plan_digest

    p = make_ba_config("cfg2")
    d0 = plan_digest(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1024)
    pid = os.fork()
    if pid == 0:  # child: exit status says whether it matched; an alarm ends a hang
        signal.alarm(60)
        try:
            d1 = plan_digest(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1024)
            os._exit(0 if d1 == d0 else 3)
        except BaseException:
            os._exit(4)
    _, status = os.waitpid(pid, 0)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0


def test_plan_input_errors_report_the_first_violation():
    """The planner's argument checks (run inside its first parallel pass) name the lowest
    non-monotone landmark offset, else the lowest out-of-range camera, whatever the thread
    split: the messages a serial scan gives."""
    from visualodometry_amd._lib import VoError
    from visualodometry_amd.ba import plan_digest

    p = make_ba_config("cfg3")  # 20k landmarks: the first pass runs on several threads
    ptr0, cam0 = p.point_ptr.copy(), p.obs_cam.copy()

    def err(point_ptr, obs_cam):
        with pytest.raises(VoError) as e:
            plan_digest(p.K, point_ptr, obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1024)
        return str(e.value)

    cam = cam0.copy()
    cam[[70000, 9000, 50000]] = [p.n_poses, -1, 99]
    assert "obs_cam[9000]=-1 out of range" in err(ptr0, cam)
    ptr = ptr0.copy()
    ptr[[17001, 4001]] = ptr[[17001, 4001]] + 10**6  # breaks monotonicity at 17001 and 4001
    assert "point_ptr not monotone at 4001" in err(ptr, cam)
    assert "point_ptr not monotone at 4001" in err(ptr, cam0)


def _win(p):
    return (p.point_ptr, p.obs_cam, p.obs_uv, p.poses_cw.shape[0], p.n_fixed)


def test_slide_plan_equals_scratch_plan():
    """A window's plan built by taking over the previous window's unchanged first-camera
    groups (what vo_ba_setup does on every keyframe, the window having slid by one) is the
    from-scratch plan of that window byte for byte, and takes most of the chunks over."""
    from visualodometry_amd.ba import plan_slide_digest
    from visualodometry_amd.synthetic import make_ba_slide

    ws = make_ba_slide("cfg3", 3)
    so = -(-ws[0].obs_cam.size // 671)
    for a, b in zip(ws, ws[1:]):
        d_inc, reused = plan_slide_digest(a.K, _win(a), _win(b), so)
        d_new, none = plan_slide_digest(a.K, None, _win(b), so)
        st = plan_probe(b.K, b.point_ptr, b.obs_cam, b.obs_uv, b.poses_cw.shape[0], b.n_fixed,
                        -(-b.obs_cam.size // so))
        assert d_inc == d_new and none == 0
        assert reused >= 0.7 * st["chunks"], (reused, st["chunks"])


@pytest.mark.parametrize("seg_chunks", [1, 3])
def test_wave_plan_slide_equals_scratch_plan(seg_chunks):
    """The one-wave K1's plans (one or three chunks per segment; padded segments of one
    first-camera group) taken over on a slide equal the scratch plans byte for byte."""
    from visualodometry_amd.ba import plan_slide_digest
    from visualodometry_amd.synthetic import make_ba_slide

    ws = make_ba_slide("cfg3", 3)
    for a, b in zip(ws, ws[1:]):
        d_inc, reused = plan_slide_digest(a.K, _win(a), _win(b), 1, seg_chunks)
        d_new, none = plan_slide_digest(a.K, None, _win(b), 1, seg_chunks)
        assert d_inc == d_new and none == 0 and reused > 1000
    d1 = plan_slide_digest(ws[0].K, None, _win(ws[1]), 1, 1)[0]
    d3 = plan_slide_digest(ws[0].K, None, _win(ws[1]), 1, 3)[0]
    assert d1 != d3  # three chunks per segment: another plan


def test_grown_and_repeated_window_plans_equal_scratch():
    """A window that grew by one keyframe (no eviction: groups keep their cameras) and the
    same window again take groups over at the same camera; the plans equal scratch plans."""
    from visualodometry_amd.ba import plan_slide_digest

    p = make_ba_problem(30, 3000, 5)
    obs_pt = np.repeat(np.arange(p.n_points), np.diff(p.point_ptr))
    inw = p.obs_cam < 29
    cnt = np.bincount(obs_pt[inw], minlength=p.n_points)
    keep = cnt >= 2
    sel = inw & keep[obs_pt]
    ptr = np.concatenate([[0], np.cumsum(cnt[keep])]).astype(np.int32)
    small = (ptr, p.obs_cam[sel], p.obs_uv[sel], 29, p.n_fixed)
    full = _win(p)
    for prev, cur in ((small, full), (full, full)):
        d_inc, reused = plan_slide_digest(p.K, prev, cur, 40)
        d_new, _ = plan_slide_digest(p.K, None, cur, 40)
        assert d_inc == d_new and reused > 0


def test_slide_plan_with_changed_groups():
    """Groups whose landmarks changed (an observation moved, a landmark's track cut, the
    fixed/free boundary) are repacked; the rest taken over; still the scratch plan."""
    from visualodometry_amd.ba import plan_slide_digest
    from visualodometry_amd.synthetic import make_ba_slide

    a, b = make_ba_slide("cfg2", 2)
    so = 37
    _, base = plan_slide_digest(a.K, _win(a), _win(b), so)
    uv = b.obs_uv.copy()
    mid = b.obs_cam.size // 2
    uv[mid, 0] += np.float32(0.25)  # one observation of a middle group moved
    ptr = b.point_ptr.copy()
    cam = b.obs_cam.copy()
    wb = (ptr, cam, uv, b.poses_cw.shape[0], b.n_fixed)
    d_inc, reused = plan_slide_digest(a.K, _win(a), wb, so)
    d_new, _ = plan_slide_digest(a.K, None, wb, so)
    assert d_inc == d_new
    assert 0 < reused < base
    # different n_fixed or seg_obs: nothing is taken over (and still the scratch plan)
    wf = (ptr, cam, uv, b.poses_cw.shape[0], b.n_fixed + 1)
    d_inc, reused = plan_slide_digest(a.K, _win(a), wf, so)
    assert reused == 0 and d_inc == plan_slide_digest(a.K, None, wf, so)[0]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_group_window_grouped_fast_path_matches_counting(seed):
    """The grouped path's offsets (first observations stored from the back, running minimum)
    equal a plain count + prefix sum, with landmarks of no observation at the ends and inside;
    an out-of-range entry is reported whether or not the rest is grouped."""
    from visualodometry_amd.ba import BAWindow, group_window

    rng = np.random.default_rng(seed)
    n_points = 400
    counts = rng.integers(0, 4, n_points)
    counts[:3] = 0
    counts[-5:] = 0
    obs_pt = np.repeat(np.arange(n_points), counts).astype(np.int32)
    m = obs_pt.size
    w = BAWindow(np.zeros((3, 4, 4)), np.zeros((n_points, 3)), np.zeros((m, 2), np.float32),
                 np.zeros(m, np.int32), obs_pt, 1)
    ptr_, _, _ = group_window(n_points, w)
    np.testing.assert_array_equal(ptr_, np.concatenate([[0], np.cumsum(counts)]))
    bad = obs_pt.copy()
    bad[m // 2] = n_points  # out of range in the middle of a grouped run (ends in range)
    with pytest.raises(ValueError):
        group_window(n_points, BAWindow(w.poses_cw, w.points, w.obs_uv, w.obs_cam, bad, 1))
    bad[m // 2] = -1
    with pytest.raises(ValueError):
        group_window(n_points, BAWindow(w.poses_cw, w.points, w.obs_uv, w.obs_cam, bad, 1))
    empty = BAWindow(w.poses_cw, w.points, w.obs_uv[:0], w.obs_cam[:0], obs_pt[:0], 1)
    np.testing.assert_array_equal(group_window(n_points, empty)[0], np.zeros(n_points + 1))
