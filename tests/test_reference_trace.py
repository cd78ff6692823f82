"""The reference's own VO loop, recorded (tests/golden/reference_trace.npz), against the oracle.

``tests/golden/make_reference_trace.py`` ran the reference's unmodified ``VisualOdometry``
over the synthetic drive of ``tests/vo_trace_scene.py`` (cv2 stubbed with the oracle's
arithmetic) and, separately, ``src/main.py`` unchanged through the drop-in hooks; the two
trajectories came out bit-identical (stored side by side).  Here, on CPU, the oracle's
vectorised restatements of the reference's Python glue must reproduce what that glue
produced: the ratio loop of ``frontend.py:97-111`` (``match_ref.match_int``) and the
triangulation filters of ``frontend.py:124-148`` (``triangulate_ref.triangulate_points``).
``tests/test_gpu_reference_trace.py`` replays the same calls through the HIP path.
"""

import json

import numpy as np
import pytest

from oracle import match_ref, triangulate_ref
from tests.conftest import GOLDEN
from tests.vo_trace_scene import TraceScene


@pytest.fixture(scope="module")
def trace():
    g = dict(np.load(GOLDEN / "reference_trace.npz"))
    return g, TraceScene(**json.loads(str(g["scene"])))


def test_dropin_trajectory_equals_reference(trace):
    g, _ = trace
    assert g["T_wc"].shape[0] == g["T_wc_dropin"].shape[0] > 0
    np.testing.assert_array_equal(g["T_wc_dropin"], g["T_wc"])
    assert int(g["n_tri_calls"]) >= 3 and int(g["n_pnp_calls"]) >= 10 and int(g["n_win_calls"]) >= 1


def test_ratio_loop_matches_oracle(trace):
    g, scene = trace
    off = np.concatenate([[0], np.cumsum(np.maximum(g["match_len"], 0))])
    frames = {}
    for i, (fa, fb) in enumerate(g["match_frames"]):
        for f in (fa, fb):
            if f not in frames:
                frames[f] = scene.frame(int(f))
        ref = g["matches"][off[i]:off[i + 1]].astype(np.int64)
        got = match_ref.match_int(frames[fa][1], frames[fb][1])
        np.testing.assert_array_equal(got, ref)


def test_triangulation_glue_matches_oracle(trace):
    g, _ = trace
    for i in range(int(g["n_tri"])):
        t = {k[len(f"tri{i}_"):]: v for k, v in g.items() if k.startswith(f"tri{i}_")}
        pts, mask = triangulate_ref.triangulate_points(t["T1"], t["T2"], t["p1"], t["p2"], g["K"],
                                                       float(t["min_depth"]), float(t["max_err"]))
        np.testing.assert_array_equal(mask, t["mask"])
        np.testing.assert_array_equal(pts, t["pts"])
