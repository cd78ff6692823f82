"""Regenerates the committed golden fixtures in tests/golden/ (run in the build container).

* ``reference_config.json`` -- ``get_config(d)`` for every dataset and the
  hardcoded intrinsics, captured by importing the reference's own importable
  modules (``src/config/config.py:49-104``, ``src/modules/dataset_loader.py:
  52-54, 85-87``) with ``src/`` on ``sys.path``.  Only data is stored.
* ``match_sift_512.npz`` -- a seeded SIFT-like 512 x 512 x 128 frame pair with
  the knn-2 + ratio-test outputs of BOTH matcher restatements (numpy and C),
  which must agree before the fixture is written.
* ``match_kat.npz`` -- hand-built known-answer cases (ties, N1 < 2, duplicates,
  many-to-one, a sqrtf collision) with their expected outputs.
* ``ba_small.npz`` -- a seeded 8-pose x 120-landmark window, one GN step of the
  numpy oracle (S, b, dc, cost) and the 6-iteration cost trajectory, checked
  against the C oracle before writing.

Usage: ``python tests/golden/make_golden.py`` from the repo root.
"""

from __future__ import annotations

import dataclasses
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
OUT = Path(__file__).resolve().parent
REF_SRC = Path("/root/reference/src")


def reference_config():
    if not REF_SRC.exists():
        print("reference not present; keeping the committed reference_config.json")
        return
    sys.dont_write_bytecode = True  # never write into the read-only reference tree
    sys.path.insert(0, str(REF_SRC))
    import config.config as rc  # noqa: E402  (the reference's own module)
    import modules.dataset_loader as rd  # noqa: E402

    cfgs = {d: dataclasses.asdict(rc.get_config(d)) for d in ["kitti", "malaga", "parking", "own", "unknown"]}
    defaults = dataclasses.asdict(rc.VOConfig())
    K = {
        "kitti": rd.KittiDataset(Path("/nonexistent")).K.tolist(),
        "malaga": rd.MalagaDataset(Path("/nonexistent")).K.tolist(),
    }
    sys.path.remove(str(REF_SRC))
    sys.dont_write_bytecode = False
    out = {"source": "cteufel13/VisualOdometry src/config/config.py, src/modules/dataset_loader.py",
           "VOConfig_defaults": defaults, "get_config": cfgs, "K": K}
    (OUT / "reference_config.json").write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print("wrote reference_config.json")


def match_fixtures():
    from oracle import match_ref
    from visualodometry_amd.synthetic import sift_like_pair

    d0, d1 = sift_like_pair(512, 512, 0)
    i_np, s_np = match_ref.knn2_int(d0, d1)
    i_c, s_c = match_ref.knn2_c(d0, d1, nthreads=4)
    assert np.array_equal(i_np, i_c) and np.array_equal(s_np.view(np.uint32), s_c.view(np.uint32))
    pairs = match_ref.ratio_filter(i_np, s_np)
    np.savez_compressed(OUT / "match_sift_512.npz", des0=d0.astype(np.uint8), des1=d1.astype(np.uint8),
                        idx=i_np, dist=s_np, pairs=pairs)
    print("wrote match_sift_512.npz", pairs.shape)

    cases = {}
    rng = np.random.default_rng(7)
    base = rng.integers(0, 256, (6, 128)).astype(np.float32)
    cases["ties"] = (base.copy(), np.concatenate([base, base, base]))
    cases["n1_eq_1"] = (base.copy(), base[:1].copy())
    cases["n1_eq_2"] = (base.copy(), base[:2].copy())
    d1 = rng.integers(0, 256, (40, 128)).astype(np.float32)
    many = np.repeat(d1[:1], 5, axis=0)
    many[:, 0] = np.clip(many[:, 0] + np.arange(5), 0, 255)
    cases["many_to_one"] = (many, d1)
    # sqrtf collision: d2 = n and n+1 with sqrtf(n) == sqrtf(n+1); the lower train
    # index must win although its d2 is larger (OpenCV compares sqrt distances)
    n = next(c for c in range(4_200_000, 8_000_000, 7) if np.sqrt(np.float32(c)) == np.sqrt(np.float32(c + 1)))

    def vec(target):
        v = np.zeros(128, np.int64)
        rem, k = target, 0
        while rem > 0:
            x = int(min(255, np.floor(np.sqrt(rem))))
            v[k], rem, k = x, rem - x * x, k + 1
        return rng.permutation(v).astype(np.float32)

    far = vec(n + 4000)
    cases["sqrt_collision"] = (np.zeros((1, 128), np.float32), np.stack([far, vec(n + 1), far, vec(n), far]))
    arrays = {}
    for name, (a, b) in cases.items():
        ia, sa = match_ref.knn2_int(a, b)
        ic, sc = match_ref.knn2_c(a, b)
        assert np.array_equal(ia, ic) and np.array_equal(sa, sc), name
        arrays[f"{name}_des0"] = a
        arrays[f"{name}_des1"] = b
        arrays[f"{name}_idx"] = ia
        arrays[f"{name}_dist"] = sa
        arrays[f"{name}_pairs"] = match_ref.ratio_filter(ia, sa)
    np.savez_compressed(OUT / "match_kat.npz", **arrays)
    print("wrote match_kat.npz", sorted(cases))


def ba_fixture():
    from oracle import ba_ref, cref
    from visualodometry_amd.synthetic import make_ba_problem

    p = make_ba_problem(8, 120, 21)
    lam = 1.0
    s = ba_ref.BAStructure(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_fixed, p.n_poses)
    st0 = ba_ref.BAState.from_poses(p.poses_cw, p.points)
    step = ba_ref.gn_step(st0, s, lam)
    _, costs = ba_ref.solve(st0, s, 6, lam)
    R = cref.BAProblemRef(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, lam)
    ok, P1, X1, c0, S, b, dc = R.step(p.poses_cw, p.points)
    assert ok and abs(c0 - step.system.cost) < 1e-9 * c0
    assert np.abs(S - step.system.S).max() < 1e-9 * np.abs(S).max()
    assert np.abs(dc - step.dc).max() < 1e-7 * np.abs(dc).max()
    np.savez_compressed(
        OUT / "ba_small.npz", K=p.K, poses_cw=p.poses_cw, points=p.points, point_ptr=p.point_ptr,
        obs_cam=p.obs_cam, obs_uv=p.obs_uv, n_fixed=p.n_fixed, lam=lam, S=step.system.S,
        b=step.system.b, dc=step.dc, dp=step.dp, cost0=step.system.cost, costs=costs,
        poses_after=step.state.poses_cw(), points_after=step.state.X)
    print("wrote ba_small.npz", costs)


if __name__ == "__main__":
    reference_config()
    match_fixtures()
    ba_fixture()
