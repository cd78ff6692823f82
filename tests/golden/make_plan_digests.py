"""Writes tests/golden/plan_digests.json: vo_ba_plan_digest of the synthetic BA windows at
several segment targets.  A planner rewrite must reproduce these exactly (the plan fixes
every kernel's summation order); a deliberate plan change regenerates them.  Round 4 packs
every first-camera group on its own (a segment boundary at each group start: the
slide-stable plan that a window's next plan can take groups over from, ba_plan.cpp), and
the one-wave K1 balances each chunk's Schur lanes over passes of 64; target 2**30 is the
engine's (segments of one chunk).
Usage: python tests/golden/make_plan_digests.py"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from visualodometry_amd.ba import plan_digest  # noqa: E402
from visualodometry_amd.synthetic import make_ba_config, make_ba_problem  # noqa: E402

CASES = [("cfg2", 1024), ("cfg3", 1024), ("cfg3", 256), ("cfg3", 4096), ("small_8x200", 64), ("small_30x3000", 512),
         ("cfg3", 1 << 30), ("cfg4", 1 << 30)]


def problem(name):
    if name.startswith("small_"):
        n, L = (int(v) for v in name[6:].split("x"))
        return make_ba_problem(n, L, 11)
    return make_ba_config(name)


def digests():
    out = {}
    for name, tgt in CASES:
        p = problem(name)
        out[f"{name}@{tgt}"] = format(plan_digest(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, tgt),
                                      "016x")
    return out


if __name__ == "__main__":
    (ROOT / "tests" / "golden" / "plan_digests.json").write_text(json.dumps(digests(), indent=1) + "\n")
