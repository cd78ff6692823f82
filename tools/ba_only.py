"""Runs the cfg3 BA window for a few GN iterations without any result check: a driver for
counter passes over timing-only builds (VO_LIB_PATH)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib  # noqa: E402
from visualodometry_amd.ba import BASession  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
p = make_ba_config(cfg)
ctx = _lib.context(0)
s = BASession(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0, ctx)
s.set_state(p.poses_cw, p.points)
s.run_async(20)
s.synchronize()
print("ok")
