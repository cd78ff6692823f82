"""Reference-trace fixtures: the reference's OWN Python VO loop, recorded (build container only).

The reference (``/root/reference/src``) needs cv2, rerun, lightglue and tyro, none of which
is installed here.  This script puts stand-ins for them in ``sys.modules`` -- their
arithmetic is the oracle's (``oracle/match_ref.py`` knnMatch, ``oracle/triangulate_ref.py``
triangulatePoints / projectPoints, ``oracle/pnp_ref.py`` solvePnPRansac / Rodrigues), the
essential-matrix initialisation (out of scope) returns the scene's true relative
pose -- and drives the reference's unmodified classes over the synthetic drive of
``tests/vo_trace_scene.py`` twice, each run in its own process:

* ``reference``: ``modules.vo.VisualOdometry`` exactly as written, KITTI config with the
  SIFT extractor (``config.py:51-67``).  Every ``match_frames`` result (the reference's own
  ratio loop, ``frontend.py:97-111``), every ``triangulate_points`` call (its own
  dehomogenisation / depth / reprojection glue, ``frontend.py:124-148``), every
  ``cv2.solvePnPRansac`` call with the inputs ``vo.py:120-141`` assembled, and the pose after
  every frame are recorded.
* ``dropin``: the reference's ``src/main.py`` run unchanged through the drop-in
  (``visualodometry_amd.dropin.run``: drop-in config with ``VO_AMD_EXTRACTOR=sift``,
  ``hooks.install()`` -- MapStore, Cv2Proxy, the matcher / triangulation / PnP hooks and
  the keyframe window on the real classes), with the product's HIP entry points routed to
  the same oracle arithmetic (no GPU here).

The two trajectories must agree bit for bit; ``tests/golden/reference_trace.npz`` keeps the
reference run's calls, which ``tests/test_gpu_reference_trace.py`` replays through the HIP
path on the GPU box (the reference itself never travels).

    python tests/golden/make_reference_trace.py            # both runs, compare, write the npz
    python tests/golden/make_reference_trace.py --check    # both runs, compare with the npz
    python tests/golden/make_reference_trace.py --long     # the long drive (below)

``--long`` drives the same three runs over a 1300-frame drive (``SCENE_LONG``), long enough
for the BA hook's ``KeyframeWindow`` to reach its full 50 keyframes (``vo.py:252-288``,
``_prune_map``'s 20 000 cap at ``vo.py:35-47`` binding), and writes
``tests/golden/reference_trace_long.npz``: the three trajectories (reference, drop-in,
drop-in with BA), the keyframe-window sizes of every BA call, and two windows with the C
oracle's solutions (the last full-size window and a mid-size one).  ``tests/test_ate.py``
computes the ATE of each trajectory on the drive's ground truth;
``tests/test_gpu_reference_trace.py`` replays the two windows through the HIP path.
"""

from __future__ import annotations

import builtins
import json
import os
import runpy
import subprocess
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
REF_SRC = Path("/root/reference/src")
LONG = os.environ.get("VO_TRACE_LONG") == "1"
OUT = ROOT / "tests" / "golden" / ("reference_trace_long.npz" if LONG else "reference_trace.npz")
# the long drive keeps the short one's landmark density along a 5x longer corridor
SCENE = (dict(n_frames=1300, n_landmarks=104000, seed=11, max_features=1400, n_distractors=80, noise_px=0.25,
              speed=1.2) if LONG else
         dict(n_frames=60, n_landmarks=9000, seed=7, max_features=1400, n_distractors=80, noise_px=0.25, speed=1.2))
MAX_TRI, MAX_PNP, MAX_WIN = (0, 0, 8) if LONG else (4, 6, 2)  # calls kept in the fixture


class _Any:
    """rerun / lightglue stand-in: every attribute and call is a no-op returning itself."""

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return self

    def __call__(self, *a, **k):
        return self


def _anymodule(name):
    m = types.ModuleType(name)

    def getattr_(attr):
        if attr.startswith("__"):
            raise AttributeError(attr)
        return _Any()

    m.__getattr__ = getattr_
    return m


class _KeyPoint:
    __slots__ = ("pt",)

    def __init__(self, x, y):
        self.pt = (x, y)


class _DMatch:
    __slots__ = ("queryIdx", "trainIdx", "distance")

    def __init__(self, q, t, d):
        self.queryIdx, self.trainIdx, self.distance = q, t, d


def make_cv2(scene, rec):
    """A ``cv2`` module whose arithmetic is the oracle's."""
    from oracle import match_ref, pnp_ref, triangulate_ref

    cv2 = types.ModuleType("cv2")
    cv2.NORM_L2, cv2.RANSAC, cv2.IMREAD_GRAYSCALE, cv2.COLOR_BGR2GRAY = 4, 8, 0, 6

    class SIFT:
        def __init__(self, **kw):
            self.kw = kw

        def detectAndCompute(self, gray, mask):
            f = int(gray[0, 0]) + 256 * int(gray[0, 1])
            uv, des, _ = scene.frame(f)
            return [_KeyPoint(float(x), float(y)) for x, y in uv], des

    class BFMatcher:
        def __init__(self, norm=4, crossCheck=False):
            assert norm == 4 and not crossCheck

        def knnMatch(self, des0, des1, k=2):
            idx, dist = match_ref.knn2_int(np.asarray(des0, np.float32), np.asarray(des1, np.float32))
            return [[_DMatch(i, int(idx[i, j]), float(dist[i, j])) for j in range(2) if idx[i, j] >= 0]
                    for i in range(idx.shape[0])]

    def imread(path, flags=0):
        f = int(Path(path).stem)
        return np.array([[f % 256, f // 256]], np.uint8)

    def findEssentialMat(p0, p1, K, method=8, prob=0.999, threshold=1.0):
        return np.eye(3), np.ones((len(p0), 1), np.uint8)

    def recoverPose(E, p0, p1, K):
        R, t = scene.relative_pose(scene.frame_of(p0), scene.frame_of(p1))
        return len(p0), R, t, np.full((len(p0), 1), 255, np.uint8)

    def solvePnPRansac(obj, img, K, dist=None, reprojectionError=8.0, iterationsCount=100, confidence=0.99, **kw):
        X = np.asarray(obj, np.float32).reshape(-1, 3)
        uv = np.asarray(img, np.float32).reshape(-1, 2)
        ok, rv, tv, mask, _ = pnp_ref.solve_pnp_ransac(X, uv, K, reprojectionError, iterationsCount, confidence)
        inl = np.flatnonzero(mask).astype(np.int32).reshape(-1, 1) if ok else None
        rec["pnp"].append(dict(X=X, uv=uv, thr=float(reprojectionError), ok=bool(ok), rvec=np.asarray(rv, float),
                               tvec=np.asarray(tv, float), inl=np.asarray(mask, bool)))
        return bool(ok), np.asarray(rv, float).reshape(3, 1), np.asarray(tv, float).reshape(3, 1), inl

    def Rodrigues(src):
        src = np.asarray(src, np.float64)
        if src.size == 3:
            return pnp_ref.rodrigues_to_mat(src.reshape(1, 3))[0], None
        return pnp_ref.rodrigues_to_vec(src.reshape(1, 3, 3))[0].reshape(3, 1), None

    def triangulatePoints(P1, P2, p1T, p2T):
        return triangulate_ref.dlt_points4d(P1, P2, np.asarray(p1T).T, np.asarray(p2T).T)

    def projectPoints(X, R, t, K, dist):
        assert dist is None
        return triangulate_ref.project_points(X, R, t, K).reshape(-1, 1, 2), None

    for name, f in list(locals().items()):
        if callable(f) and not name.startswith("_") and name not in ("make_cv2",):
            setattr(cv2, name, f)
    cv2.SIFT_create = lambda **kw: SIFT(**kw)
    return cv2


def install_stubs(scene, rec, data_dir=None):
    sys.modules["cv2"] = make_cv2(scene, rec)
    sys.modules["rerun"] = _anymodule("rerun")
    sys.modules["lightglue"] = _anymodule("lightglue")
    tyro = types.ModuleType("tyro")
    tyro.cli = lambda cls: cls(dataset="kitti", path=Path(data_dir), sequence="05")
    sys.modules["tyro"] = tyro


def _record_frontend(rec, scene, frontend_cls, vo_mod):
    mf = frontend_cls.match_frames

    def match_frames(self, f0, f1):
        m = mf(self, f0, f1)
        k0, k1 = f0["keypoints"][0].cpu().numpy(), f1["keypoints"][0].cpu().numpy()
        rec["match"].append((scene.frame_of(k0), scene.frame_of(k1), np.asarray(m)))
        return m

    frontend_cls.match_frames = match_frames
    tp = vo_mod.triangulate_points

    def triangulate_points(T1, T2, p1, p2, K, cfg):
        pts, mask = tp(T1, T2, p1, p2, K, cfg)
        rec["tri"].append(dict(T1=np.asarray(T1, float), T2=np.asarray(T2, float), p1=np.asarray(p1, np.float32),
                               p2=np.asarray(p2, np.float32), mask=np.asarray(mask, bool), pts=np.asarray(pts),
                               min_depth=float(cfg.min_depth), max_err=float(cfg.max_reproj_err)))
        return pts, mask

    vo_mod.triangulate_points = triangulate_points


def _record_poses(rec, vo_cls):
    pf = vo_cls.process_frame

    def process_frame(self, img):
        pf(self, img)
        rec["T_wc"].append(np.array(self.T_wc, float))

    vo_cls.process_frame = process_frame


def run_reference(out_path: str) -> None:
    """The reference's VisualOdometry, unmodified, over the scene."""
    sys.dont_write_bytecode = True
    sys.path[:0] = [str(REF_SRC), str(ROOT)]
    from tests.vo_trace_scene import K_KITTI, TraceScene

    scene = TraceScene(**SCENE)
    rec = {"match": [], "tri": [], "pnp": [], "T_wc": []}
    install_stubs(scene, rec)
    from config.config import get_config
    import modules.frontend as fe
    import modules.vo as vo_mod

    cfg = get_config("kitti")
    # the reference applies its SIFT overrides only when the extractor is already SIFT
    # (config.py:51-67; its default is superpoint): select SIFT and apply them as written
    cfg.extractor_type = "sift"
    for k, v in dict(sift_n_features=4000, sift_contrast_threshold=0.02, sift_edge_threshold=2.0,
                     max_reproj_err=5.0, pnp_reproj_err=1.0, turn_smoothing=0.2, trans_smoothing=0.4).items():
        setattr(cfg, k, v)
    _record_frontend(rec, scene, fe.FeatureFrontend, vo_mod)
    _record_poses(rec, vo_mod.VisualOdometry)
    vo = vo_mod.VisualOdometry(K_KITTI, cfg)
    cv2 = sys.modules["cv2"]
    for f in range(scene.n_frames):
        vo.process_frame(cv2.imread(f"{f:06d}.png"))
    _save_run(out_path, rec, len(vo.map_points), cfg)


def run_dropin(out_path: str, ba: bool = False) -> None:
    """The reference's src/main.py, unchanged, through the drop-in; HIP calls -> oracle.
    With ``ba`` the sliding-window BA hook is on (``VO_AMD_BA=1``); its windows and the
    oracle's solutions of them are recorded."""
    sys.dont_write_bytecode = True
    from tests.vo_trace_scene import TraceScene  # noqa: E402  (ROOT is on sys.path: see main)

    scene = TraceScene(**SCENE)
    rec = {"match": [], "tri": [], "pnp": [], "T_wc": []}
    data = Path(tempfile.mkdtemp(prefix="vo_trace_"))
    img_dir = data / "kitti" / "05" / "image_0"
    img_dir.mkdir(parents=True)
    for f in range(scene.n_frames):
        (img_dir / f"{f:06d}.png").write_bytes(b"")
    install_stubs(scene, rec, data)
    builtins.input = lambda *a, **k: ""
    os.environ["VO_AMD_EXTRACTOR"] = "sift"
    if ba:
        os.environ["VO_AMD_BA"] = "1"
    # the product's HIP entry points -> the oracle's arithmetic (no GPU in this container)
    from oracle import match_ref, triangulate_ref
    from visualodometry_amd import matcher, pnp, sift, triangulate

    matcher.match_knn2_ratio = lambda d0, d1, ratio=0.75, ctx=None, **kw: match_ref.match_int(
        matcher._as_des(d0), matcher._as_des(d1), ratio)
    triangulate.triangulate_points = lambda T1, T2, p1, p2, K, cfg, ctx=None: triangulate_ref.triangulate_points(
        T1, T2, p1, p2, K, cfg.min_depth, cfg.max_reproj_err)
    pnp.solvePnPRansac = sys.modules["cv2"].solvePnPRansac
    sift.SIFT_create = sys.modules["cv2"].SIFT_create
    rec["win"] = []
    from visualodometry_amd import ba as ba_mod

    def optimize(self, window):  # SlidingWindowBA.optimize on the C oracle
        from oracle import cref

        poses = np.asarray(window.poses_cw, np.float64)
        pts = np.asarray(window.points, np.float64).reshape(-1, 3)
        order, ptr_ = ba_mod.csr_from_obs_pt(pts.shape[0], window.obs_pt)
        cam = np.asarray(window.obs_cam, np.int32)[order]
        uv = np.asarray(window.obs_uv, np.float32).reshape(-1, 2)[order]
        R = cref.BAProblemRef(self.K, ptr_, cam, uv, poses.shape[0], int(window.n_fixed), self.lam)
        _, P, X, costs = R.solve(poses, pts, self.iters)
        rec["win"].append(dict(poses=poses, points=pts, obs_uv=np.asarray(window.obs_uv, np.float32),
                               obs_cam=np.asarray(window.obs_cam, np.int32), obs_pt=np.asarray(window.obs_pt, np.int32),
                               n_fixed=int(window.n_fixed), iters=self.iters, lam=self.lam, P=P, X=X, costs=costs))
        return ba_mod.BAResult(P, X, costs, "ok")

    ba_mod.SlidingWindowBA.optimize = optimize
    ba_mod.SlidingWindowBA.reserve = lambda self, *a, **k: None  # no device here
    # visualodometry_amd.dropin.run.main, with recording wrappers added after install()
    main_py = REF_SRC / "main.py"
    sys.path[:0] = [str(ROOT / "visualodometry_amd" / "dropin"), str(REF_SRC)]
    from visualodometry_amd.dropin import hooks

    hooks.install()
    import modules.frontend as fe
    import modules.vo as vo_mod

    _record_frontend(rec, scene, fe.FeatureFrontend, vo_mod)
    _record_poses(rec, vo_mod.VisualOdometry)
    n_map = []
    init = vo_mod.VisualOdometry.__init__

    def __init__(self, *a, **k):
        init(self, *a, **k)
        n_map.append(self)

    vo_mod.VisualOdometry.__init__ = __init__
    sys.argv = [str(main_py)]
    runpy.run_path(str(main_py), run_name="__main__")
    vo = n_map[0]
    assert type(vo.map_points).__name__ == "MapStore" and type(vo_mod.cv2).__name__ == "Cv2Proxy"
    _save_run(out_path, rec, len(vo.map_points), vo.cfg)


def _save_run(path, rec, n_map, cfg) -> None:
    out = {"T_wc": np.stack(rec["T_wc"]), "n_map": np.int64(n_map)}
    out["match_frames"] = np.array([(a, b) for a, b, _ in rec["match"]], np.int32).reshape(-1, 2)
    out["match_len"] = np.array([m.shape[0] if m.ndim == 2 else -1 for _, _, m in rec["match"]], np.int32)
    out["match_ndim"] = np.array([m.ndim for _, _, m in rec["match"]], np.int32)
    ms = [m.reshape(-1, 2) for _, _, m in rec["match"]]
    out["matches"] = (np.concatenate(ms) if ms else np.zeros((0, 2))).astype(np.int16)
    for i, t in enumerate(rec["tri"][:MAX_TRI]):
        for k, v in t.items():
            out[f"tri{i}_{k}"] = np.asarray(v)
    out["n_tri"] = np.int64(min(len(rec["tri"]), MAX_TRI))
    out["n_tri_calls"] = np.int64(len(rec["tri"]))
    wins = rec.get("win", [])
    out["win_sizes"] = np.array([[t["poses"].shape[0], t["points"].shape[0], t["obs_uv"].shape[0]] for t in wins],
                                np.int64).reshape(-1, 3)
    if LONG and wins:
        # the last window of the largest size, the window closest to half that size, then six
        # more spread evenly over the drive's calls; beyond the first two, the landmark positions
        # are stored as float32 (the map's own type, vo.py:281: exact) and the oracle's solution
        # X as float32 (the replay's bar is 1e-5 relative), to keep the fixture small
        n = out["win_sizes"][:, 0]
        full = int(np.flatnonzero(n == n.max())[-1])
        mid = int(np.argmin(np.abs(n - n.max() / 2)))
        idx = [full, mid]
        for j in np.linspace(0, len(wins) - 1, 8).round().astype(int):
            if int(j) not in idx and len(idx) < MAX_WIN:
                idx.append(int(j))
        sel = []
        for r, j in enumerate(idx):
            t = dict(wins[j])
            if r >= 2:
                assert np.array_equal(t["points"].astype(np.float32).astype(np.float64), t["points"])
                t["points"] = t["points"].astype(np.float32)
                t["X"] = t["X"].astype(np.float32)
            sel.append(t)
        wins = sel
        out["win_index"] = np.array(idx, np.int64)
    if LONG:
        out["matches"] = np.zeros((0, 2), np.int16)  # the long fixture keeps trajectories and windows only
    for i, t in enumerate(wins[:MAX_WIN]):
        for k, v in t.items():
            out[f"win{i}_{k}"] = np.asarray(v)
    out["n_win"] = np.int64(min(len(wins), MAX_WIN))
    out["n_win_calls"] = np.int64(len(rec.get("win", [])))
    for i, t in enumerate(rec["pnp"][:MAX_PNP]):
        for k, v in t.items():
            out[f"pnp{i}_{k}"] = np.asarray(v)
    out["n_pnp"] = np.int64(min(len(rec["pnp"]), MAX_PNP))
    out["n_pnp_calls"] = np.int64(len(rec["pnp"]))
    out["K"] = np.array([[7.18856e02, 0, 6.071928e02], [0, 7.18856e02, 1.852157e02], [0, 0, 1]])
    out["scene"] = np.array(json.dumps(SCENE))
    np.savez_compressed(path, **out)


def _run(mode: str, path: str) -> None:
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", PYTHONPATH=str(ROOT), VO_TRACE_LONG="1" if LONG else "0")
    return subprocess.Popen([sys.executable, __file__, f"--{mode}", path], env=env, stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)


def _wait(mode: str, proc) -> None:
    out, err = proc.communicate(timeout=3600)
    if proc.returncode != 0:
        raise SystemExit(f"{mode} run failed:\n{out[-3000:]}\n{err[-3000:]}")


def compare(a: dict, b: dict) -> list[str]:
    """Differences between two runs' records (empty = bit-identical)."""
    bad = []
    for k in ("T_wc", "match_frames", "match_len", "matches", "n_map", "n_tri_calls", "n_pnp_calls"):
        if not np.array_equal(a[k], b[k]):
            bad.append(k)
    return bad


def main() -> None:
    if "--long" in sys.argv and not LONG:  # re-read the module constants in long mode
        os.environ["VO_TRACE_LONG"] = "1"
        sys.argv.remove("--long")
        r = subprocess.run([sys.executable, __file__] + sys.argv[1:], env=dict(os.environ))
        raise SystemExit(r.returncode)
    if not REF_SRC.exists():
        raise SystemExit(f"{REF_SRC} is absent: the fixtures are generated in the build container")
    if len(sys.argv) > 2 and sys.argv[1] in ("--reference", "--dropin", "--dropin_ba"):
        sys.path.insert(0, str(ROOT))
        if sys.argv[1] == "--reference":
            run_reference(sys.argv[2])
        else:
            run_dropin(sys.argv[2], ba=sys.argv[1] == "--dropin_ba")
        return
    check = "--check" in sys.argv
    with tempfile.TemporaryDirectory() as td:
        pr, pd, pb = (os.path.join(td, f"{n}.npz") for n in ("ref", "dropin", "dropin_ba"))
        runs = [(m, _run(m, p)) for m, p in (("reference", pr), ("dropin", pd), ("dropin_ba", pb))]  # in parallel
        for m, proc in runs:
            _wait(m, proc)
        a, b, c = dict(np.load(pr)), dict(np.load(pd)), dict(np.load(pb))
        diff = compare(a, b)
        ref_quirk = int((a["match_ndim"] == 1).sum())
        print(f"frames {a['T_wc'].shape[0]}, match calls {len(a['match_len'])} (empty-result quirk {ref_quirk}), "
              f"triangulations {int(a['n_tri_calls'])}, PnP calls {int(a['n_pnp_calls'])}, map points {int(a['n_map'])}")
        if diff:
            raise SystemExit(f"reference and drop-in runs differ in: {diff}")
        print("reference run == drop-in run (trajectory, matches, call counts, map size): bit-identical")
        print(f"drop-in run with BA: {int(c['n_win_calls'])} keyframe windows adjusted")
        # the fixture: the reference run's calls plus the BA run's windows and trajectory
        for k, v in c.items():
            if k.startswith("win") or k in ("n_win", "n_win_calls"):
                a[k] = v
        if LONG:
            print("BA window sizes (poses, landmarks, observations):", c["win_sizes"].tolist())
        a["T_wc_ba"] = c["T_wc"]
        a["T_wc_dropin"] = b["T_wc"]
        if check:
            g = dict(np.load(OUT))
            diff = compare(a, g)
            if diff:
                raise SystemExit(f"reference run differs from {OUT.name} in: {diff}")
            print(f"{OUT.name} reproduced")
        else:
            np.savez_compressed(OUT, **a)
            print(f"wrote {OUT} ({OUT.stat().st_size} bytes)")


if __name__ == "__main__":
    main()
