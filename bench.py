#!/usr/bin/env python3
"""Benchmark: BA Gauss-Newton iterations/s on the 50-pose x 20k-landmark window.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1
it is launched by ``torch.distributed.run`` (one rank per GPU).  A *step* is
one full GN iteration of the synthetic cfg3 window (BASELINE.json configs[2]:
50 poses x 20k landmarks, ~83k observations, seed 3): fused back-substitution
+ linearisation + Schur accumulation (K1), slab reduction (K2), [RCCL
all-reduce of the reduced camera system when N > 1], dense pose solve + pose
update (K3).  Inputs are resident in HBM before timing starts.  N > 1 shards
the SAME window's landmarks across ranks (strong scaling, one all-reduce per
iteration).  Rank 0 prints ONE JSON line.

Also reported in that line: the per-kernel HIP-event durations measured on
the library stream over the timed region, the roofline of the dominant
kernel, the CPU baseline (the C oracle, timed on this host's cores) and, at
N = 1, the secondary metric "descriptor-match Mpairs/sec" (SIFT-like 4000 x
4000 x 128 frame pairs, batched, int8 MFMA path) with its own roofline.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
I8_PEAK_TOPS = 5000.0  # dense int8 MFMA = 2x the 2.5 PF dense bf16 rate (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)
METRIC = "BA GN-iters/sec at 50 poses×20k landmarks; descriptor-match Mpairs/sec"


def ba_kernel_bytes(kind: str, n_poses: int, n_points: int, n_obs: int, n_free: int,
                    prof_blocks: int) -> float:
    """Algorithmic HBM bytes per launch."""
    if kind == "ba_lin":
        # obs (uv f32x2 + camera i32 + track-entry i32), points read + written + CSR
        # offset, old + new poses
        return 16.0 * n_obs + (24 + 24 + 4) * n_points + 2 * 96 * n_poses
    if kind == "ba_reduce":
        return 36 * 8.0 * prof_blocks + 6 * 8.0 * n_free
    if kind == "ba_solve":
        return 36 * 8.0 * prof_blocks + 2 * 6 * 8.0 * n_free + 2 * 96 * n_poses
    return 0.0


# Source files whose code a kernel group's PMC traffic depends on: a traffic file records their
# digest (tools/pmc_traffic.py), and bench.py attaches its figures only to a run of the same
# sources, configuration and kernel set (a stale file would describe another build).
TRAFFIC_SOURCES = {
    "ba": ["ba.hip", "ba_band.hip", "ba_band.h", "ba_math.h", "ba_reduce.h", "ba_plan.cpp", "ba_plan.h",
           "vo_common.h", "vo_ctx.h", "Makefile"],
    "match": ["match.hip", "match_bf16.hip", "match_short.h", "vo_common.h", "vo_ctx.h", "Makefile"],
}


def source_digest(group: str) -> str:
    import hashlib

    h = hashlib.sha256()
    src = ROOT / "visualodometry_amd" / "csrc"
    for f in TRAFFIC_SOURCES[group]:
        h.update(f.encode())
        h.update((src / f).read_bytes())
    return h.hexdigest()[:16]


def traffic_for(path, config: str, lam: float, world: int, group: str, kernels):
    """PMC traffic per launch for `kernels` (short names) from a tools/pmc_traffic.py file, or
    (None, reason) when the file was counted on another build (source digest), configuration,
    damping, rank count or kernel set than the timed run."""
    if not path or not Path(path).exists():
        return {}, f"no traffic file {path}"
    t = json.loads(Path(path).read_text())
    key = t.get("_key")
    if not key:
        return {}, f"{path}: no build/config key (pre-r04 format)"
    want = {"config": config, "lam": lam, "gpus": world, "digest": source_digest(group)}
    got = {"config": key.get("config"), "lam": key.get("lam"), "gpus": key.get("gpus"),
           "digest": key.get("digest", {}).get(group)}
    if got != want:
        return {}, f"{path}: counted on {got}, timed run is {want}"
    # kernels launched on every counted step (a cost-only K2 of the parity guard launches once)
    seen = {k for k, n in key.get("launches", {}).items() if n >= 5}
    if group == "ba":
        timed = {k for k in kernels if k.startswith("ba_")}
        counted = {k for k in seen if k.startswith("ba_")}
        if timed != counted:
            return {}, f"{path}: counted kernel set {sorted(counted)} != timed {sorted(timed)}"
    missing = [k for k in kernels if k not in seen]
    if missing:
        return {}, f"{path}: kernels {missing} not in the counted run ({sorted(seen)})"
    return {k: t[k] for k in kernels if k in t}, None


def host_cores():
    """Host cores this process may use: its CPU affinity, capped by a cgroup CPU quota
    (on the GPU box the job's share of a larger machine).  Returns (threads, note)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    threads = min(n, quota) if quota else n
    note = f"{threads} threads = every core this job may use (affinity {n}"
    note += f", cgroup quota {quota}" if quota else ""
    note += f"; os.cpu_count() {os.cpu_count()})"
    return threads, note


def cpu_baseline_ba(p, lam: float, budget_s: float = 3.0):
    from oracle import cref

    threads, note = host_cores()
    R = cref.BAProblemRef(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, lam)
    poses, pts = p.poses_cw, p.points
    ok, poses, pts, *_ = R.step(poses, pts, threads, want_system=False)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        ok, poses, pts, *_ = R.step(poses, pts, threads, want_system=False)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= budget_s or n >= 2000:
            break
    return {"value": n / dt, "unit": "GN-iters/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ba_ref.c (OpenMP Schur accumulation into a dense S, Cholesky over its envelope) on the same cfg3 "
                      f"window: {n} GN iterations in {dt:.2f} s; {note}"}


def ba_parity_guard(sess, p, pts, p0: int, p1: int, lam: float, iters: int = 2, tol: float = 1e-5) -> dict:
    """Untimed check of the timed build: reset the session to the window's start state, run
    ``iters`` GN iterations and compare costs, poses and this rank's landmarks with the C
    oracle (oracle/ba_ref.c) on the whole window, relative max-norm error <= ``tol``
    (north_star's 1e-5).  On N ranks every rank runs the collective iterations and checks its
    own landmark shard."""
    from oracle import cref
    from visualodometry_amd import _lib

    def rel(a, b):
        return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))

    sess.set_state(p.poses_cw, pts)
    rc, costs = sess.run(iters)
    P, X = sess.get_state()
    R = cref.BAProblemRef(p.K, p.point_ptr, p.obs_cam, p.obs_uv, p.n_poses, p.n_fixed, lam)
    _, Pr, Xr, cr = R.solve(p.poses_cw, p.points, iters, nthreads=host_cores()[0])
    err = {"cost": rel(np.asarray(costs), np.asarray(cr)), "poses": rel(P, Pr), "points": rel(X, Xr[p0:p1])}
    ok = rc == _lib.VO_OK and all(np.isfinite(v) and v <= tol for v in err.values())
    return {"ok": bool(ok), "iters": iters, "tol": tol, "rel_err": err, "checker": "oracle/ba_ref.c"}


def bench_matcher(ctx, batch: int = 16, n: int = 4000, calls: int = 20, warmup: int = 3, traffic_path=None):
    from visualodometry_amd import _lib, matcher
    from visualodometry_amd.synthetic import sift_like_pair

    pairs = [sift_like_pair(n, n, 1000 + b) for b in range(batch)]
    # the drop-in's hint for the reference's SIFT extractor (hooks.match_frames): the int8
    # sweep only; results do not depend on it (float values would take the exact sweep)
    matcher.set_descriptor_kind(matcher.DESC_SIFT, ctx)
    a = _lib.DeviceArray.from_numpy(ctx, np.stack([q[0] for q in pairs]))
    b = _lib.DeviceArray.from_numpy(ctx, np.stack([q[1] for q in pairs]))
    out = _lib.DeviceArray(ctx, (batch, n), np.int32)
    for _ in range(warmup):
        matcher.match_batch_device(a, b, out=out, ctx=ctx)
    matcher.synchronize(ctx)
    # the value: back-to-back calls with no per-kernel events
    t0 = time.perf_counter()
    for _ in range(calls):
        matcher.match_batch_device(a, b, out=out, ctx=ctx)
    matcher.synchronize(ctx)
    dt = time.perf_counter() - t0
    # per-kernel averages: a second region with HIP events around every launch
    _lib.profile_enable(ctx, True)
    for _ in range(calls):
        matcher.match_batch_device(a, b, out=out, ctx=ctx)
    matcher.synchronize(ctx)
    prof = _lib.profile_read(ctx)
    _lib.profile_enable(ctx, False)
    # parity guard on frame pair 0 against the oracle (not timed)
    from oracle import match_ref

    ref = match_ref.match_int(*pairs[0])
    got = out.numpy()[0]
    kept = np.nonzero(got >= 0)[0]
    assert np.array_equal(np.stack([kept, got[kept]], 1), ref), "matcher parity guard failed"

    pairs_total = batch * n * n * calls
    ms_i8, cnt_i8 = prof.get("match_i8", (0.0, 1))
    avg_s = ms_i8 / max(cnt_i8, 1) / 1e3
    tops = 2.0 * 128 * batch * n * n / avg_s / 1e12 if avg_s > 0 else 0.0
    kern = {k: round(v[0] / v[1] * 1e3, 2) for k, v in prof.items()}
    traffic, why = traffic_for(traffic_path, "cfg3", 1.0, 1, "match", ["match_i8"])
    res = {
        "metric": "descriptor-match Mpairs/sec",
        "value": pairs_total / dt / 1e6,
        "unit": "Mpairs/s",
        "dtype": "i8",
        "config": {"workload": f"SIFT-like (integers 0..255 as f32) {n} x {n} x 128, "
                               f"{batch} frame pairs per call, knn2 + ratio 0.75", "calls": calls},
        "kernel_us": kern,
        "roofline": {"bound": "mfma", "kernel": "match_i8", "achieved": tops, "peak": I8_PEAK_TOPS,
                     "unit": "TFLOP/s", "frac": tops / I8_PEAK_TOPS, "traffic": traffic.get("match_i8"),
                     "traffic_note": why,
                     "note": "int8 ops (2*128 per pair) per match_i8 launch / its HIP-event duration"},
    }
    # CPU baseline: C oracle on a bounded sample of query rows
    from oracle import cref

    threads, note = host_cores()
    rows = 1000
    t0 = time.perf_counter()
    cref.knn2(pairs[0][0][:rows], pairs[0][1], threads)
    cdt = time.perf_counter() - t0
    res["cpu_baseline"] = {"value": rows * n / cdt / 1e6, "unit": "Mpairs/s", "cores": threads,
                           "kind": "port",
                           "sample": f"oracle/match_ref.c knn2 on {rows} x {n} x 128 of frame pair 0; {note}"}
    return res


def bench_matcher_float(ctx, batch: int = 16, n: int = 2048, dim: int = 256, calls: int = 10, warmup: int = 2,
                        traffic_path=None):
    """BASELINE config 5's matcher: SuperPoint-like L2-normalised float32 descriptors (not
    integer-valued: the bf16 MFMA shortlist + exact fp32 re-rank, bit-exact with the
    k-ordered fmaf chain), 2048 x 2048 x 256 per frame pair, knn2 + ratio
    0.75, frame pairs resident in HBM."""
    from oracle import match_ref
    from visualodometry_amd import _lib, matcher
    from visualodometry_amd.synthetic import superpoint_like_pair

    pairs = [superpoint_like_pair(n, n, 2000 + b, dim=dim) for b in range(batch)]
    matcher.set_descriptor_kind(matcher.DESC_FLOAT, ctx)
    a = _lib.DeviceArray.from_numpy(ctx, np.stack([q[0] for q in pairs]))
    b = _lib.DeviceArray.from_numpy(ctx, np.stack([q[1] for q in pairs]))
    out = _lib.DeviceArray(ctx, (batch, n), np.int32)
    for _ in range(warmup):
        matcher.match_batch_device(a, b, out=out, ctx=ctx)
    matcher.synchronize(ctx)
    t0 = time.perf_counter()
    for _ in range(calls):
        matcher.match_batch_device(a, b, out=out, ctx=ctx)
    matcher.synchronize(ctx)
    dt = time.perf_counter() - t0
    _lib.profile_enable(ctx, True)
    for _ in range(calls):
        matcher.match_batch_device(a, b, out=out, ctx=ctx)
    matcher.synchronize(ctx)
    prof = _lib.profile_read(ctx)
    _lib.profile_enable(ctx, False)
    threads, note = host_cores()
    ref = match_ref.match_c(pairs[0][0], pairs[0][1], nthreads=threads)
    got = out.numpy()[0]
    kept = np.nonzero(got >= 0)[0]
    assert np.array_equal(np.stack([kept, got[kept]], 1), ref), "float matcher parity guard failed"
    kern = {k: round(v[0] / v[1] * 1e3, 2) for k, v in prof.items()}
    ms_f, cnt_f = prof.get("match_f32", (0.0, 1))  # both bf16 MFMA sweeps of a call
    avg_s = ms_f / max(cnt_f, 1) / 1e3
    # algorithmic flops: ONE contraction of 2 flops per (pair, k); the second sweep recomputes
    # the first's products (it marks the shortlist), so it is time, not credited work
    tfl = 2.0 * dim * batch * n * n / avg_s / 1e12 if avg_s > 0 else 0.0
    traffic, why = traffic_for(traffic_path, "cfg3", 1.0, 1, "match", ["match_f32"])
    res = {
        "metric": "descriptor-match Mpairs/sec (float path)",
        "value": batch * n * n * calls / dt / 1e6,
        "unit": "Mpairs/s",
        "dtype": "f32",
        "config": {"workload": f"SuperPoint-like L2-normalised float32 {n} x {n} x {dim}, {batch} frame pairs "
                               "per call, knn2 + ratio 0.75 (BASELINE config 5 matcher)", "calls": calls},
        "kernel_us": kern,
        "roofline": {"bound": "mfma", "kernel": "match_f32 (fsweep<1> + fsweep<2>, bf16 MFMA)", "achieved": tfl,
                     "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tfl / BF16_MFMA_PEAK_TFLOPS,
                     "traffic": traffic.get("match_f32"), "traffic_note": why,
                     "issued_tflops": 2.0 * tfl,
                     "note": "algorithmic flops (2 per pair and dimension, one contraction) / the summed HIP-event "
                             "duration of both sweeps (fsweep<2> recomputes fsweep<1>'s products: issued_tflops "
                             "counts both); the exact fp32 re-rank of the shortlisted candidates is "
                             "kernel_us.match_rerank"},
    }
    rows = 256
    t0 = time.perf_counter()
    match_ref.knn2_c(pairs[0][0][:rows], pairs[0][1], threads)
    cdt = time.perf_counter() - t0
    res["cpu_baseline"] = {"value": rows * n / cdt / 1e6, "unit": "Mpairs/s", "cores": threads, "kind": "port",
                           "sample": f"oracle/match_ref.c knn2 on {rows} x {n} x {dim} of frame pair 0; {note}"}
    return res


FP32_VECTOR_PEAK_TFLOPS = 157.3  # 256 CUs x 4 SIMDs x 64 FLOP/clk (FMA, 16 lanes x 2, packed x2) x 2.4 GHz
FP64_VECTOR_PEAK_TFLOPS = 78.6  # 256 CUs x 4 SIMDs x 32 FLOP/clk (4-cycle wave64 fp64 FMA) x 2.4 GHz
TRI_FLOPS_PER_POINT = 2892      # DLT 32 + 5 Jacobi sweeps (typical; a wave stops once converged) x 6 pairs x ~92 + ~100


def bench_triangulate(ctx, n: int = 1_000_000, calls: int = 200, warmup: int = 3):
    """device-resident triangulation throughput (points/s)."""
    from visualodometry_amd import _lib, triangulate
    from visualodometry_amd.synthetic import triangulation_case

    T1, T2, p1, p2, K, X, kind = triangulation_case(n, 5)
    d1 = _lib.DeviceArray.from_numpy(ctx, p1)
    d2 = _lib.DeviceArray.from_numpy(ctx, p2)
    out = _lib.DeviceArray(ctx, (n, 3), np.float32)
    msk = _lib.DeviceArray(ctx, (n,), np.uint8)
    run = lambda: triangulate.triangulate_device(T1, T2, d1, d2, K, 0.001, 6.0, out, msk, ctx)  # noqa: E731
    for _ in range(warmup):
        run()
    _lib.load().vo_synchronize(ctx.handle)
    t0 = time.perf_counter()
    for _ in range(calls):
        run()
    _lib.load().vo_synchronize(ctx.handle)
    dt = time.perf_counter() - t0
    _lib.profile_enable(ctx, True)
    for _ in range(calls):
        run()
    prof = _lib.profile_read(ctx)
    _lib.profile_enable(ctx, False)
    ms, cnt = prof.get("triangulate", (0.0, 1))
    avg_s = ms / max(cnt, 1) / 1e3
    # parity guard against the oracle on a slice (not timed)
    from oracle import triangulate_ref as tr

    got_m = msk.numpy()[:20000].astype(bool)
    _, ref_m = tr.all_points(T1, T2, p1[:20000], p2[:20000], K, 0.001, 6.0)
    assert np.array_equal(got_m, ref_m), "triangulation parity guard failed"
    gflops = TRI_FLOPS_PER_POINT * n / avg_s / 1e12 if avg_s > 0 else 0.0
    res = {
        "metric": "triangulated points/sec",
        "value": n * calls / dt,
        "unit": "points/s",
        "dtype": "f64",
        "config": {"workload": f"two-view DLT + depth + reprojection filter, {n} correspondences per call, "
                               "KITTI K, float32 image points (reference frontend.py:115-148)", "calls": calls},
        "kernel_us": round(avg_s * 1e6, 2),
        "roofline": {"bound": "valu-fp64", "achieved": gflops, "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": gflops / FP64_VECTOR_PEAK_TFLOPS,
                     "hbm_gbs": 29.0 * n / avg_s / 1e9 if avg_s > 0 else 0.0,
                     "note": f"~{TRI_FLOPS_PER_POINT} fp64 flops per point at 5 Jacobi sweeps (the loop stops when "
                             "the wave has converged) and 29 HBM bytes per point"},
    }
    t0 = time.perf_counter()
    rows = 100_000
    tr.all_points(T1, T2, p1[:rows], p2[:rows], K, 0.001, 6.0)
    cdt = time.perf_counter() - t0
    res["cpu_baseline"] = {"value": rows / cdt, "unit": "points/s", "cores": 1, "kind": "port",
                           "sample": f"oracle/triangulate_ref.py (numpy, batched LAPACK SVD) on {rows} points"}
    return res


PNP_FLOPS_PER_HYP = 68_000  # EPnP: 12x12 Jacobi SVD (431 pair checks x ~26 + 314 rotations x ~135 flops,
                            # counted on this workload with the oracle), M^T M 2.9k, 3x3 SVDs ~5k, betas ~6k
PNP_FLOPS_PER_EVAL = 40     # scoring: R X + t, 1/z, pixel, float32 error (fp64 + fp32 ops) per point x hypothesis


def bench_pnp(ctx, batch: int = 1024, n: int = 1000, calls: int = 20, warmup: int = 3, thr: float = 1.0):
    """device-resident PnP-RANSAC throughput (frames/s), batched frames."""
    from oracle import pnp_ref
    from visualodometry_amd import _lib, pnp
    from visualodometry_amd.synthetic import pnp_case

    cases = [pnp_case(n, 100 + f, noise_px=0.3, outlier_frac=0.25) for f in range(batch)]
    K = cases[0][2]
    off = np.arange(batch + 1, dtype=np.int32) * n
    dX = _lib.DeviceArray.from_numpy(ctx, np.concatenate([c[0] for c in cases]))
    dU = _lib.DeviceArray.from_numpy(ctx, np.concatenate([c[1] for c in cases]))
    dP = _lib.DeviceArray(ctx, (batch, 6), np.float64)
    dM = _lib.DeviceArray(ctx, (batch * n,), np.uint8)
    dS = _lib.DeviceArray(ctx, (batch, 2), np.int32)
    H = 100  # RANSAC iterations per frame (cv2.solvePnPRansac's default, vo.py:135-141)
    run = lambda: pnp.pnp_ransac_device(dX, dU, off, K, thr, dP, dM, dS, iterations=H, ctx=ctx)  # noqa: E731
    for _ in range(warmup):
        run()
    _lib.load().vo_synchronize(ctx.handle)
    t0 = time.perf_counter()
    for _ in range(calls):
        run()
    _lib.load().vo_synchronize(ctx.handle)
    dt = time.perf_counter() - t0
    _lib.profile_enable(ctx, True)
    for _ in range(calls):
        run()
    prof = _lib.profile_read(ctx)
    _lib.profile_enable(ctx, False)
    kern = {k: round(v[0] / v[1] * 1e3, 2) for k, v in prof.items() if k.startswith("pnp")}
    # parity guard on frame 0 against the oracle (not timed)
    ref = pnp_ref.solve_pnp_ransac(cases[0][0], cases[0][1], K, thr)
    st = dS.numpy()
    assert st[0, 0] == 1 and np.array_equal(dM.numpy()[:n].astype(bool), ref[3]), "PnP parity guard failed"
    assert np.allclose(dP.numpy()[0, :3], ref[1], rtol=1e-5, atol=1e-8), "PnP parity guard failed (rvec)"
    # hypotheses solved per call: the first h1 of every frame, the rest only for the frames
    # whose serial RANSAC loop had not stopped by then (pnp_run; both launches timed)
    h1, tail = _lib.pnp_testing_last_split(ctx)
    hyp_s = (kern.get("pnp_hyp", 0.0) + kern.get("pnp_hyp_tail", 0.0)) / 1e6
    hyps = batch * h1 + tail * (H - h1)
    tfl = PNP_FLOPS_PER_HYP * hyps / hyp_s / 1e12 if hyp_s > 0 else 0.0
    res = {
        "metric": "PnP-RANSAC frames/sec",
        "value": batch * calls / dt,
        "unit": "frames/s",
        "dtype": "f64",
        "config": {"workload": f"cv2.solvePnPRansac contract (reference vo.py:135-141): {batch} frames x {n} "
                               f"float32 2D-3D correspondences (25% gross outliers, 0.3 px noise), KITTI K, "
                               f"{H} iterations, confidence 0.99, reprojectionError {thr} (KITTI config)",
                   "calls": calls},
        "kernel_us": kern,
        "roofline": {"bound": "valu-fp64", "kernel": "pnp_hyp", "achieved": tfl, "peak": FP64_VECTOR_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": tfl / FP64_VECTOR_PEAK_TFLOPS,
                     "note": f"~{PNP_FLOPS_PER_HYP} fp64 flops per EPnP hypothesis x {hyps} hypotheses per call "
                             f"/ the HIP-event duration of pnp_hyp (+ pnp_hyp_tail): the first {h1} hypotheses of "
                             f"every frame, the other {H - h1} for the {tail} frames whose serial loop had not "
                             "stopped by then"},
        "split": {"h1": h1, "tail_frames": tail},
    }
    # single-frame latency through the host-buffer entry point (the reference's per-frame call)
    X0, U0 = cases[0][0], cases[0][1]
    for _ in range(3):
        pnp.pnp_ransac(X0, U0, K, thr, ctx=ctx)
    t0 = time.perf_counter()
    for _ in range(20):
        pnp.pnp_ransac(X0, U0, K, thr, ctx=ctx)
    res["single_frame_ms"] = (time.perf_counter() - t0) / 20 * 1e3
    frames = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 3.0 and frames < batch:
        pnp_ref.solve_pnp_ransac(cases[frames][0], cases[frames][1], K, thr)
        frames += 1
    cdt = time.perf_counter() - t0
    res["cpu_baseline"] = {"value": frames / cdt, "unit": "frames/s", "cores": 1, "kind": "port",
                           "sample": f"oracle/pnp_ref.py (numpy, hypotheses batched; early exit as OpenCV) on "
                                     f"{frames} of the frames"}
    return res


def sift_bytes_per_image(h: int, w: int, n_layers: int = 3) -> float:
    """Algorithmic HBM bytes of one image's detection: the uint8 read and
    float32 write of the doubled image; per octave level 0 (blur or downsample: 4 B read + 4 B
    written per pixel), n_layers + 2 blurred levels (4 B read, G and DoG written: 12 B) and
    the extrema pass (3 DoG levels read per candidate level: 36 B)."""
    from visualodometry_amd import sift

    L = sift.layout(h, w, n_layers)
    total = h * w + 4.0 * 4 * h * w
    for o in L["octaves"]:
        px = o["h"] * o["w"]
        total += px * (8 + 12 * (n_layers + 2) + 12 * n_layers)
    return total


def bench_sift(ctx, batch: int = 8, h: int = 376, w: int = 1241, calls: int = 10, warmup: int = 2,
               nfeatures: int = 4000, contrast: float = 0.02, edge: float = 2.0, cap: int = 16384,
               check: bool = True):
    """device-resident SIFT detectAndCompute (pyramid, extrema, orientation,
    removeDuplicatedSorted, retainBest, descriptors), images/s, with the reference's KITTI
    settings (config.py:64-66)."""
    from oracle import sift_ref
    from visualodometry_amd import _lib, sift
    from visualodometry_amd.synthetic import sift_scene

    imgs = np.stack([sift_scene(h, w, seed=200 + b, texture=12.0) for b in range(batch)])
    dI = _lib.DeviceArray.from_numpy(ctx, imgs)
    dK = _lib.DeviceArray(ctx, (batch, cap, 8), np.int32)
    dD = _lib.DeviceArray(ctx, (batch, cap, 128), np.float32)
    dC = _lib.DeviceArray(ctx, (batch,), np.int32)
    run = lambda: sift.detect_and_compute_device(dI, nfeatures, contrast, edge, 1.6, 3, dK, dD, dC,  # noqa: E731
                                                 ctx=ctx)
    for _ in range(warmup):
        run()
    _lib.load().vo_synchronize(ctx.handle)
    t0 = time.perf_counter()
    for _ in range(calls):
        run()
    _lib.load().vo_synchronize(ctx.handle)
    dt = time.perf_counter() - t0
    _lib.profile_enable(ctx, True)
    for _ in range(calls):
        run()
    prof = _lib.profile_read(ctx)
    _lib.profile_enable(ctx, False)
    kern = {k: round(v[0] / v[1] * 1e3, 2) for k, v in prof.items() if k.startswith("sift")}
    counts = dC.numpy()
    assert np.all(counts >= 0), "SIFT capacity overflow"
    # parity guard against the oracle on image 0 of the batch (not timed; check=False only for
    # the timing-only diagnostic builds of tools/gpu_sift_diag.sh)
    if check:
        ref = sift_ref.detect_and_compute(imgs[0], nfeatures, contrast, edge, 1.6)
        K0 = sift.unpack_device_keypoints(dK.numpy()[0, :counts[0]])
        D0 = dD.numpy()[0, :counts[0]]
        assert counts[0] == len(ref["pt"]) and np.array_equal(K0["x"], ref["pt"][:, 0]) and \
            np.array_equal(K0["angle"], ref["angle"]) and np.array_equal(D0, ref["descriptors"]), \
            "SIFT parity guard failed"
    nbytes = sift_bytes_per_image(h, w) * batch
    pyr_s = kern.get("sift_pyramid", 0.0) / 1e6
    ext_s = kern.get("sift_extrema", 0.0) / 1e6
    gbs = nbytes / (pyr_s + ext_s) / 1e9 if pyr_s + ext_s > 0 else 0.0
    res = {
        "metric": "SIFT detectAndCompute images/sec",
        "value": batch * calls / dt,
        "unit": "images/s",
        "dtype": "f32",
        "config": {"workload": f"{batch} synthetic textured {w}x{h} uint8 images per call (KITTI image_0 size), "
                               f"SIFT_create(nfeatures={nfeatures}, contrastThreshold={contrast}, "
                               f"edgeThreshold={edge}, sigma=1.6) (reference KITTI SIFT config): pyramid, "
                               "extrema, orientation, duplicate removal, retainBest, 128-d descriptors",
                   "calls": calls, "keypoints_per_image": [int(c) for c in counts]},
        "kernel_us": kern,
        "roofline": {"bound": "hbm", "kernel": "sift_pyramid+sift_extrema", "achieved": gbs, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "bytes_per_call": nbytes,
                     "note": "algorithmic bytes (bench.sift_bytes_per_image) / the summed HIP-event spans of "
                             "the pyramid and extrema launches (launch gaps included); orientation, selection "
                             "and descriptors are reported in kernel_us"},
    }
    t0 = time.perf_counter()
    sift_ref.detect_and_compute(imgs[1], nfeatures, contrast, edge, 1.6)
    res["cpu_baseline"] = {"value": 1.0 / (time.perf_counter() - t0), "unit": "images/s", "cores": 1,
                           "kind": "port", "sample": "oracle/sift_ref.py detect_and_compute (numpy) on image 1"}
    return res


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)  # ~7 ms at cfg3: the clocks settle before the timed region
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--lam", type=float, default=1.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-matcher", action="store_true")
    ap.add_argument("--k1", type=int, default=0,
                    help="tuning: K1 variant through the testing switch vo_ba_testing_k1 (0 = the product "
                         "default, -1 four-wave K1, n = 1..3 one-wave K1 with n chunks per segment)")
    ap.add_argument("--traffic-json", default=None,
                    help="per-kernel HBM bytes per launch from rocprofv3 --pmc passes of this build and config "
                         "(tools/pmc_traffic.py; default profiles/traffic_<config>.json); attached only when its "
                         "key (source digest, config, lambda, ranks, kernel set) matches the timed run; the timed "
                         "run itself is never profiled")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    from visualodometry_amd import _lib
    from visualodometry_amd.ba import BASession
    from visualodometry_amd.shard import shard
    from visualodometry_amd.synthetic import BA_CONFIGS, make_ba_config

    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)  # control plane only

    # VO_BENCH_DEVICE pins every rank to one device (rehearsing N > 1 on a one-GPU box)
    ctx = _lib.context(int(os.environ.get("VO_BENCH_DEVICE", local)))
    if world > 1:
        uid = [_lib.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        _lib.comm_init(ctx, world, rank, uid[0])

    if args.k1:
        _lib.ba_testing_k1(ctx, args.k1)
    p = make_ba_config(args.config)
    (p0, p1), ptr, cam, uv, pts = shard(p.point_ptr, p.obs_cam, p.obs_uv, p.points, world, rank)
    reserve_ms = None
    # the VO's construction-time reservation (SlidingWindowBA.reserve): setup_us is a warm first
    # call (an older tuning library without the entry point skips it)
    if world == 1 and getattr(ctx.lib, "vo_ba_reserve", None) is not None:
        t0 = time.perf_counter()
        _lib.ba_reserve(ctx, p.n_poses, p.n_points, p.n_obs, p.n_fixed)
        reserve_ms = (time.perf_counter() - t0) * 1e3
    sess = BASession(p.K, ptr, cam, uv, p.n_poses, p.n_fixed, args.lam, ctx)
    sess.set_state(p.poses_cw, pts)
    stats = sess.plan_stats()

    def barrier():
        if dist is not None:
            dist.barrier()

    def timed(steps: int, profiled: bool) -> float:
        barrier()
        sess.synchronize()
        _lib.profile_enable(ctx, profiled)
        t0 = time.perf_counter()
        sess.run_async(steps)
        sess.synchronize()
        t1 = time.perf_counter()
        barrier()
        dt_ = t1 - t0
        if dist is not None:
            import torch

            t = torch.tensor([dt_], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt_ = float(t[0])
        return dt_

    sess.run_async(args.warmup)
    sess.synchronize()
    # timed regions 1-3 (the metric): K iterations each, no event markers between the kernels;
    # the value is the median region's rate (a transient of the box cannot set it),
    # every region is reported
    regions = [timed(args.steps, False) for _ in range(3)]
    dt = sorted(regions)[len(regions) // 2]
    # timed region 2: the same K iterations with HIP events around every kernel on the
    # library stream -> per-kernel average durations for the roofline
    dt_prof = timed(args.steps, True)
    prof = _lib.profile_read(ctx)
    _lib.profile_enable(ctx, False)
    # guard: the timed iterations must not have failed (status is checked by a sync run)
    rc, costs = sess.run(1)
    if rc != _lib.VO_OK or not np.all(np.isfinite(costs)):
        print(f"error: BA status {rc}, costs {costs}", file=sys.stderr)
        return 1
    # parity guard (not timed): the same build from the window's start state, 2 iterations,
    # against the C oracle at the north-star tolerance -- a wrong-result build prints no number
    guard = ba_parity_guard(sess, p, pts, p0, p1, args.lam)
    if not guard["ok"]:
        print(f"error: BA parity guard failed: {guard}", file=sys.stderr)
        return 1

    value = args.steps / dt
    n_free = p.n_poses - p.n_fixed
    kern = {}
    best = None
    for k, (ms, cnt) in prof.items():
        avg_us = ms / cnt * 1e3
        kern[k] = {"avg_us": round(avg_us, 3), "launches": cnt, "total_ms": round(ms, 3)}
        if best is None or ms > prof[best][0]:
            best = k
    nbytes = ba_kernel_bytes(best, p.n_poses, p1 - p0, int(ptr[-1]), n_free, stats["profile_blocks"])
    if best == "ba_solve" and "ba_reduce" not in prof:  # K2 fused into K3's launch (one rank)
        nbytes += ba_kernel_bytes("ba_reduce", p.n_poses, p1 - p0, int(ptr[-1]), n_free, stats["profile_blocks"])
    avg_s = prof[best][0] / prof[best][1] / 1e3
    achieved = nbytes / avg_s / 1e9
    tpath = args.traffic_json or str(ROOT / "profiles" / f"traffic_{args.config}.json")
    ba_traffic, traffic_why = traffic_for(tpath, args.config, args.lam, world, "ba", sorted(prof))
    traffic = ba_traffic.get(best)
    lin_bytes = ba_kernel_bytes("ba_lin", p.n_poses, p1 - p0, int(ptr[-1]), n_free, stats["profile_blocks"])
    lin_avg = prof["ba_lin"][0] / prof["ba_lin"][1] / 1e3
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "GN-iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "ms_per_step_with_kernel_events": dt_prof / args.steps * 1e3,
        "timed_regions": {"steps_each": args.steps, "reported": "median",
                          "ms_per_step": [r / args.steps * 1e3 for r in regions],
                          "value": [args.steps / r for r in regions]},
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"{args.config}: synthetic sliding-window BA window, "
                        f"{p.n_poses} poses x {p.n_points} landmarks, {p.n_obs} observations "
                        f"(seed {BA_CONFIGS[args.config][2]}, KITTI K, first {p.n_fixed} poses fixed, "
                        f"lambda={args.lam}); one step = one full GN iteration",
            "poses": p.n_poses, "landmarks": p.n_points, "observations": p.n_obs,
            "parallelism": f"landmark-sharded x{world}" + (" + RCCL all-reduce" if world > 1 else ""),
            "k1_variant": args.k1,
            "plan": stats,
            "reserve_ms": reserve_ms,
        },
        "kernels": kern,
        "roofline": {
            "bound": "hbm", "kernel": best, "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_note": traffic_why, "traffic_file": tpath, "traffic_all_kernels": ba_traffic or None,
            "bytes_per_launch": nbytes,
            "note": "algorithmic bytes per launch / HIP-event average duration on the library stream",
        },
        "roofline_ba_lin": {"achieved": lin_bytes / lin_avg / 1e9, "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": lin_bytes / lin_avg / 1e9 / HBM_PEAK_GBS,
                            "bytes_per_launch": lin_bytes},
        "algorithmic_bytes_per_iter": stats["algorithmic_bytes_per_iter"],
        "parity_guard": guard,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_ba(p, args.lam)
        line["speedup_vs_cpu_baseline"] = value / line["cpu_baseline"]["value"]
    if rank == 0 and world == 1 and not args.no_matcher:
        line["secondary"] = bench_matcher(ctx, traffic_path=tpath)
        line["matcher_float"] = bench_matcher_float(ctx, traffic_path=tpath)
        line["triangulate"] = bench_triangulate(ctx)
        line["pnp"] = bench_pnp(ctx)
        line["sift"] = bench_sift(ctx)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
