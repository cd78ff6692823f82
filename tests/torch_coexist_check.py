"""Run as its own process by tests/test_gpu_torch_coexist.py: torch first, on the GPU, as
the reference's FeatureFrontend does (frontend.py:3, :66-67), then libvo_hip.so in the
same process (torch ships its own libamdhip64 under the same SONAME).  Each product call
is checked against the oracle; exit 0 and a final "OK" line on success, "SKIP: ..." when
torch has no GPU here."""

import sys
from pathlib import Path
from types import SimpleNamespace

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

if not torch.cuda.is_available():
    print("SKIP: torch sees no GPU")
    sys.exit(0)
dev = torch.device("cuda")
probe = torch.arange(1024, device=dev, dtype=torch.float32) * 2.0  # torch's HIP runtime is live
torch.cuda.synchronize()

from oracle import cref, match_ref, sift_ref  # noqa: E402
from visualodometry_amd import _lib, sift  # noqa: E402
from visualodometry_amd.ba import BAWindow, SlidingWindowBA  # noqa: E402
from visualodometry_amd.dropin import hooks  # noqa: E402
from visualodometry_amd.synthetic import make_ba_problem, sift_like_pair, sift_scene  # noqa: E402

lib = _lib.load()
print("libvo_hip:", _lib.LIB_PATH)

# match_frames through the hook, descriptors as (1, N, 128) torch tensors on the GPU
d0, d1 = sift_like_pair(700, 800, 3)
feats0 = {"descriptors": torch.from_numpy(d0)[None].to(dev)}
feats1 = {"descriptors": torch.from_numpy(d1)[None].to(dev)}
frontend = SimpleNamespace(conf=SimpleNamespace(extractor_type="sift", match_on_gpu=True))
match_frames = hooks._wrap_match_frames(lambda self, a, b: None)
got = match_frames(frontend, feats0, feats1)
assert np.array_equal(got, match_ref.match_int(d0, d1)), "match_frames mismatch vs oracle"
print("match_frames ok", got.shape)
# the keyframe side stays cached across frames (the same GPU tensor), read in place from
# torch's device memory unless the library refused it (another HIP runtime instance)
_, d2 = sift_like_pair(700, 650, 4)
feats2 = {"descriptors": torch.from_numpy(d2)[None].to(dev)}
got = match_frames(frontend, feats0, feats2)
assert np.array_equal(got, match_ref.match_int(d0, d2)), "match_frames (cached keyframe) mismatch vs oracle"
feats0["descriptors"][0, 3] = feats0["descriptors"][0, 7]  # in place on the GPU: a new version
m0 = feats0["descriptors"][0].cpu().numpy()
got = match_frames(frontend, feats0, feats1)
assert np.array_equal(got, match_ref.match_int(m0, d1)), "match_frames (modified keyframe) mismatch vs oracle"
print("match_frames cached ok; device tensors read in place:", not getattr(_lib.context(), "_foreign_tensors", False))

# one sliding-window BA optimize against the C oracle
p = make_ba_problem(10, 400, 11)
obs_pt = np.repeat(np.arange(p.points.shape[0]), np.diff(p.point_ptr))
res = SlidingWindowBA(p.K, iters=4, lam=1.0).optimize(
    BAWindow(p.poses_cw, p.points, p.obs_uv, p.obs_cam, obs_pt, p.n_fixed))
assert res.status == "ok", res.message
R = cref.BAProblemRef(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, 1.0)
_, Pr, Xr, cr = R.solve(p.poses_cw, p.points, 4)
rel = np.abs(res.poses_cw - Pr).max() / np.abs(Pr).max()
assert rel < 1e-5 and np.allclose(res.cost_per_iter, cr, rtol=1e-5), f"BA mismatch rel={rel}"
print("SlidingWindowBA ok", rel)

# process_image through the hook: the SIFT kernels write k.pt and the descriptors into torch's
# GPU memory (frontend.py:51-75 keeps only those); the same values as the host entry point's
img_pi = sift_scene(150, 260, seed=5, n_blobs=60, n_boxes=12)
fe = SimpleNamespace(extractor=sift.SIFT_create(nfeatures=300, contrastThreshold=0.02, edgeThreshold=2.0, sigma=1.6),
                     device=dev)
process_image = hooks._wrap_process_image(lambda self, im: None)
feats_pi = process_image(fe, img_pi)
ref_pi = sift.detect_and_compute(img_pi, 300, 0.02, 2.0, 1.6)
if feats_pi is None:  # the library refused torch's memory: the reference body ran (here a stub)
    print("process_image: torch memory refused, host path")
else:
    assert feats_pi["keypoints"].shape == (1, ref_pi["pt"].shape[0], 2) and feats_pi["keypoints"].is_cuda
    assert np.array_equal(feats_pi["keypoints"][0].cpu().numpy(), ref_pi["pt"]), "process_image keypoints mismatch"
    assert np.array_equal(feats_pi["descriptors"][0].cpu().numpy(), ref_pi["descriptors"]), "process_image descriptors"
    got = match_frames(frontend, feats_pi, feats_pi)
    assert np.array_equal(got, match_ref.match_int(ref_pi["descriptors"], ref_pi["descriptors"])), "match on GPU feats"
    print("process_image ok", feats_pi["keypoints"].shape)

# SIFT detectAndCompute (the SIFT_create drop-in) against the oracle
img = sift_scene(120, 200, seed=2, n_blobs=40, n_boxes=10)
kp, des = sift.SIFT_create(nfeatures=0, contrastThreshold=0.02, edgeThreshold=2.0, sigma=1.6).detectAndCompute(img, None)
kr = sift_ref.detect_and_compute(img, 0, 0.02, 2.0, 1.6)
pts = np.array([k.pt for k in kp], np.float32).reshape(-1, 2)
assert pts.shape[0] == kr["pt"].shape[0] and np.array_equal(pts, kr["pt"]), "SIFT keypoints mismatch"
assert np.array_equal(des, kr["descriptors"]), "SIFT descriptors mismatch"
print("SIFT ok", pts.shape[0])

# torch still works in the same process
assert torch.equal((probe / 2.0).cpu(), torch.arange(1024, dtype=torch.float32))
print("OK")
