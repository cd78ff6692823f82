"""The one-wave K1's Schur lanes (csrc/ba.hip ba_lin_wave_kernel) walked on the host over the
planner's chunk images (``ba_plan_check``, csrc/ba_plan_check.cpp): every pair of every active
slot summed exactly once per row, aligned butterfly groups inside one 64-lane pass, diagonal
slots carrying exactly their camera's track entries (U and b summed by their lanes), and, with
one chunk per segment, every slab row and rhs entry written.  No GPU needed."""

import os
import subprocess
import tempfile
from pathlib import Path

import numpy as np
import pytest

from visualodometry_amd.synthetic import make_ba_config, make_ba_problem

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "visualodometry_amd" / "lib" / "ba_plan_check"


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", str(ROOT / "visualodometry_amd" / "csrc"), "../lib/ba_plan_check"],
                   check=True)
    return EXE


def check(exe, p, seg_obs, seg_chunks=1):
    with tempfile.TemporaryDirectory() as d:
        fi = os.path.join(d, "in")
        with open(fi, "wb") as f:
            np.array([p.n_poses, len(p.point_ptr) - 1, len(p.obs_cam), p.n_fixed, seg_obs], np.int32).tofile(f)
            np.asarray(p.point_ptr, np.int32).tofile(f)
            np.asarray(p.obs_cam, np.int32).tofile(f)
            np.asarray(p.obs_uv, np.float32).tofile(f)
        out = subprocess.run([str(exe), fi, str(seg_chunks)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr
    return [int(v) for v in out.stdout.split()[1:]]


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_one_chunk_segments(exe, cfg):
    chunks, segs, passes, chain = check(exe, make_ba_config(cfg), 1)
    assert chunks == segs


@pytest.mark.parametrize("seg_obs", [1, 120, 1000])
def test_small_windows(exe, seg_obs):
    for n, L, seed in [(8, 200, 11), (30, 3000, 11), (12, 800, 5)]:
        check(exe, make_ba_problem(n, L, seed), seg_obs)


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
@pytest.mark.parametrize("seg_chunks", [2, 3])
def test_group_segments(exe, cfg, seg_chunks):
    """Wave plans of several chunks per segment: every segment exactly seg_chunks chunks of one
    first-camera group (empty chunks pad a group's last segment), the union of its chunks'
    active slots and cameras covers its window, and fewer segment slots (slab rows) than the
    one-chunk plan's."""
    p = make_ba_config(cfg)
    chunks, segs, _, _ = check(exe, p, 1, seg_chunks)
    assert chunks == seg_chunks * segs
    c1, s1, _, _ = check(exe, p, 1, 1)
    assert segs < s1 and chunks < c1 * 1.2


def test_group_segments_small_windows(exe):
    for n, L, seed in [(8, 200, 11), (30, 3000, 11), (12, 800, 5), (3, 40, 2)]:
        for sc in (2, 3):
            check(exe, make_ba_problem(n, L, seed), 1, sc)


def test_multi_chunk_segments(exe):
    chunks, segs, _, _ = check(exe, make_ba_config("cfg3"), 400)
    assert segs < chunks
