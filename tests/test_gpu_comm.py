"""RCCL communicator plumbing on one device: a 1-rank communicator changes nothing."""

import numpy as np
import pytest

from visualodometry_amd import _lib
from visualodometry_amd.ba import BASession
from visualodometry_amd.synthetic import make_ba_config

pytestmark = pytest.mark.gpu


def test_single_rank_comm_is_bitwise_neutral(ctx):
    p = make_ba_config("cfg2")
    s = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0, ctx)
    s.set_state(p.poses_cw, p.points)
    rc, c0 = s.run(4)
    P0, X0 = s.get_state()
    assert rc == _lib.VO_OK
    # a separate context with a 1-rank RCCL communicator (all-reduces become identities)
    c2 = _lib.Context(0)
    _lib.comm_init(c2, 1, 0, _lib.comm_unique_id())
    s2 = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0, c2)
    s2.set_state(p.poses_cw, p.points)
    rc2, c1 = s2.run(4)
    P1, X1 = s2.get_state()
    assert rc2 == _lib.VO_OK
    np.testing.assert_array_equal(c0, c1)
    np.testing.assert_array_equal(P0, P1)
    np.testing.assert_array_equal(X0, X1)
