"""GPU parity of the matcher (vo_match_*) against the CPU oracle -- bit-exact.

Integer indices and float32 distances must be identical to oracle/match_ref
(OpenCV BFMatcher(NORM_L2).knnMatch(k=2) + ratio test semantics,
reference src/modules/frontend.py:86-111).
"""

import numpy as np
import pytest

from oracle import match_ref
from visualodometry_amd import matcher
from visualodometry_amd.synthetic import sift_like_pair, superpoint_like_pair

pytestmark = pytest.mark.gpu


def _check_knn2(d0, d1, ctx, oracle="int"):
    idx, dist = matcher.match_knn2(d0, d1, ctx=ctx)
    if oracle == "int":
        ri, rd = match_ref.knn2_int(d0, d1)
    else:
        ri, rd = match_ref.knn2_c(d0, d1, nthreads=8)
    np.testing.assert_array_equal(idx, ri)
    np.testing.assert_array_equal(dist.view(np.uint32), rd.view(np.uint32))
    pairs = matcher.match_knn2_ratio(d0, d1, ctx=ctx)
    np.testing.assert_array_equal(pairs, match_ref.ratio_filter(ri, rd))
    assert pairs.dtype == np.int64 and pairs.ndim == 2 and pairs.shape[1] == 2


@pytest.mark.parametrize("n0,n1,seed", [(512, 512, 0), (1000, 1200, 1), (37, 5, 2), (300, 17, 3),
                                        (2048, 2048, 4)])
def test_sift_like_bit_exact(ctx, n0, n1, seed):
    d0, d1 = sift_like_pair(n0, n1, seed)
    _check_knn2(d0, d1, ctx)


def test_sift_kitti_size_4000(ctx):
    """BASELINE config: KITTI SIFT, 4000 x 4000 x 128 (config.py:64)."""
    d0, d1 = sift_like_pair(4000, 4000, 11)
    _check_knn2(d0, d1, ctx)


@pytest.mark.parametrize("dim", [64, 100, 192, 256])
def test_int_dims(ctx, dim):
    d0, d1 = sift_like_pair(333, 444, 5, dim=dim)
    _check_knn2(d0, d1, ctx)


def test_int_valued_dim_over_256_takes_float_path(ctx):
    # integer data with D > 256 runs on the fp32 path; integer sums are exact there too
    d0, d1 = sift_like_pair(200, 300, 6, dim=320)
    _check_knn2(d0, d1, ctx)


def test_superpoint_like_float_bit_exact(ctx):
    d0, d1 = superpoint_like_pair(700, 900, 7)
    _check_knn2(d0, d1, ctx, oracle="c")


def test_superpoint_2048(ctx):
    """BASELINE config 5: SuperPoint-like 2048 x 2048 x 256 (config.py:15)."""
    d0, d1 = superpoint_like_pair(2048, 2048, 8)
    _check_knn2(d0, d1, ctx, oracle="c")


@pytest.mark.parametrize("dim", [32, 100, 192, 256])
def test_float_shortlist_dims(ctx, dim):
    """bf16 MFMA shortlist + exact re-rank (match_bf16.hip) at every K padding."""
    d0, d1 = superpoint_like_pair(333, 517, 30 + dim, dim=dim)
    _check_knn2(d0, d1, ctx, oracle="c")


def test_float_shortlist_unnormalised(ctx):
    """Non-integer descriptors with large norms: the candidate bound scales with them."""
    rng = np.random.default_rng(31)
    d0 = (rng.standard_normal((400, 128)) * 50 + 100).astype(np.float32)
    d1 = np.concatenate([d0[:200] + rng.standard_normal((200, 128)).astype(np.float32),
                         (rng.standard_normal((300, 128)) * 50 + 100).astype(np.float32)])
    _check_knn2(d0, d1, ctx, oracle="c")


def test_float_shortlist_overflow_rescans_exactly(ctx):
    """Hundreds of train rows within the bf16 error of each other: more than 32
    candidates per query, so those rows take the exact full re-scan."""
    rng = np.random.default_rng(32)
    base = rng.standard_normal((1, 256)).astype(np.float32)
    d1 = np.concatenate([base + 1e-4 * rng.standard_normal((300, 256)).astype(np.float32),
                         rng.standard_normal((200, 256)).astype(np.float32)])
    d0 = np.concatenate([base + 1e-4 * rng.standard_normal((20, 256)).astype(np.float32),
                         rng.standard_normal((50, 256)).astype(np.float32)])
    _check_knn2(d0, d1, ctx, oracle="c")


def test_float_shortlist_exact_ties(ctx):
    """Duplicate float train rows: equal exact distances keep the lower train index."""
    d0, d1 = superpoint_like_pair(200, 100, 33)
    d1 = np.concatenate([d1, d1, d1[::-1]])
    _check_knn2(d0, d1, ctx, oracle="c")


def test_ties_keep_lower_train_index(ctx):
    rng = np.random.default_rng(0)
    base = rng.integers(0, 256, (8, 128)).astype(np.float32)
    d1 = np.concatenate([base, base, base])  # every row appears 3 times
    d0 = base.copy()
    idx, dist = matcher.match_knn2(d0, d1, ctx=ctx)
    np.testing.assert_array_equal(idx[:, 0], np.arange(8))
    np.testing.assert_array_equal(idx[:, 1], np.arange(8) + 8)
    assert (dist[:, :2] == 0).all()
    # equal best and second distances: 0 < 0.75 * 0 fails -> no match
    assert matcher.match_knn2_ratio(d0, d1, ctx=ctx).shape == (0, 2)


def test_single_train_row_gives_no_matches(ctx):
    d0, d1 = sift_like_pair(50, 1, 9)
    idx, dist = matcher.match_knn2(d0, d1, ctx=ctx)
    assert (idx[:, 0] == 0).all() and (idx[:, 1] == -1).all()
    assert matcher.match_knn2_ratio(d0, d1, ctx=ctx).shape == (0, 2)


def test_empty_inputs(ctx):
    d = np.zeros((10, 128), np.float32)
    e = np.zeros((0, 128), np.float32)
    assert matcher.match_knn2_ratio(e, d, ctx=ctx).shape == (0, 2)
    assert matcher.match_knn2_ratio(d, e, ctx=ctx).shape == (0, 2)
    idx, _ = matcher.match_knn2(d, e, ctx=ctx)
    assert (idx == -1).all()


def test_many_to_one(ctx):
    """No crossCheck (frontend.py:34): several queries may keep the same train row."""
    rng = np.random.default_rng(3)
    d1 = rng.integers(0, 256, (64, 128)).astype(np.float32)
    d0 = np.repeat(d1[:1], 5, axis=0)
    d0[:, 0] = np.clip(d0[:, 0] + np.arange(5), 0, 255)
    pairs = matcher.match_knn2_ratio(d0, d1, ctx=ctx)
    np.testing.assert_array_equal(pairs, match_ref.match_int(d0, d1))
    assert (pairs[:, 1] == 0).all() and len(pairs) == 5


def test_sqrt_collision_rescan(ctx):
    """d2 = n and n+1 (>= 2^22) that sqrtf maps to the same float: the (dist, j) key
    must then prefer the lower train index even though its d2 is larger."""
    # find n with sqrtf(n) == sqrtf(n + 1), n in the reachable range (< 128 * 255^2)
    n = None
    for cand in range(4_200_000, 8_000_000, 7):
        if np.sqrt(np.float32(cand)) == np.sqrt(np.float32(cand + 1)):
            n = cand
            break
    assert n is not None
    rng = np.random.default_rng(5)

    def vec_with_d2(target):
        # query = zeros; a train row with sum of squares == target, values 0..255
        v = np.zeros(128, np.int64)
        rem = target
        k = 0
        while rem > 0:
            x = int(min(255, np.floor(np.sqrt(rem))))
            v[k] = x
            rem -= x * x
            k += 1
        assert rem == 0 and k <= 128
        return rng.permutation(v).astype(np.float32)

    q = np.zeros((1, 128), np.float32)
    far = vec_with_d2(n + 4000)
    t = np.stack([far, vec_with_d2(n + 1), far, vec_with_d2(n), far])  # j=1 has the larger d2
    idx, dist = matcher.match_knn2(q, t, ctx=ctx)
    ri, rd = match_ref.knn2_int(q, t)
    np.testing.assert_array_equal(idx, ri)
    np.testing.assert_array_equal(dist, rd)
    assert idx[0, 0] == 1 and idx[0, 1] == 3


def test_batch_device_matches_single(ctx):
    from visualodometry_amd._lib import DeviceArray

    B, n0, n1 = 4, 500, 600
    pairs = [sift_like_pair(n0, n1, 100 + b) for b in range(B)]
    a = DeviceArray.from_numpy(ctx, np.stack([p[0] for p in pairs]))
    b = DeviceArray.from_numpy(ctx, np.stack([p[1] for p in pairs]))
    best = matcher.match_batch_device(a, b, ctx=ctx)
    matcher.synchronize(ctx)
    best = best.numpy()
    for k in range(B):
        ref = match_ref.match_int(*pairs[k])
        got = np.nonzero(best[k] >= 0)[0]
        np.testing.assert_array_equal(np.stack([got, best[k][got]], 1), ref)


def test_int_and_float_calls_alternate_on_one_context(ctx):
    """The per-call "not 0..255 integers" flag is a generation tag (no reset between
    calls): an integer call right after a float call must take the int8 path again."""
    s0, s1 = sift_like_pair(300, 400, 21)
    f0, f1 = superpoint_like_pair(300, 400, 22)
    for _ in range(2):
        _check_knn2(s0, s1, ctx)
        _check_knn2(f0, f1, ctx, oracle="c")
    # one non-integer value in the train side alone switches the whole call
    g1 = s1.copy()
    g1[7, 3] += 0.5
    _check_knn2(s0, g1, ctx, oracle="c")
    _check_knn2(s0, s1, ctx)


def test_duplicate_train_rows_across_lanes_tiles_and_splits(ctx):
    """500 distinct rows, each repeated 8 times at shuffled positions among 4000 train rows:
    exact d2 ties inside a 16-lane group, across column tiles and across splits must all
    resolve to the lower train index, as in the oracle."""
    rng = np.random.default_rng(31)
    base = rng.integers(0, 256, (500, 128)).astype(np.float32)
    d1 = base[rng.permutation(np.repeat(np.arange(500), 8))]
    d0 = np.concatenate([base[:300], rng.integers(0, 256, (700, 128)).astype(np.float32)])
    _check_knn2(d0, d1, ctx)


def test_float_hint_skips_int_pack_and_stays_exact(ctx):
    """Under the float hint no int8 pack (and no integer check) runs: the bf16 shortlist + exact
    re-rank must still reproduce the integer oracle on SIFT bytes (the fp32 chains of squared
    byte differences are exact) and the fp32 oracle on floats, and a non-finite value must still
    reach the exact sweep (fpack flags it) -- same outputs as without the hint."""
    d0, d1 = sift_like_pair(2048, 2048, 21)
    f0, f1 = superpoint_like_pair(1024, 1500, 22)
    n0, n1 = f0.copy(), f1.copy()
    n0[5, 7] = np.nan
    n1[9, 3] = np.inf
    auto = [matcher.match_knn2(n0, n1, ctx=ctx)]
    _check_knn2(n0, n1, ctx, oracle="c")  # the exact sweep (inside merge_kernel) vs the C oracle
    matcher.set_descriptor_kind(matcher.DESC_FLOAT, ctx)
    try:
        _check_knn2(d0, d1, ctx)
        _check_knn2(f0, f1, ctx, oracle="c")
        hinted = matcher.match_knn2(n0, n1, ctx=ctx)
        _check_knn2(n0, n1, ctx, oracle="c")  # the re-rank kernel's exact scan vs the C oracle
    finally:
        matcher.set_descriptor_kind(matcher.DESC_AUTO, ctx)
    np.testing.assert_array_equal(hinted[0], auto[0][0])
    np.testing.assert_array_equal(hinted[1].view(np.uint32), auto[0][1].view(np.uint32))


def test_sift_hint_with_float_values_takes_the_exact_sweep(ctx):
    """Under the SIFT hint no shortlist is launched: float (and non-finite) values that reach the
    int8 launch are answered by the exact fp32 sweep inside merge_kernel, bit-exact vs the C
    oracle; SIFT bytes keep the int8 path."""
    f0, f1 = superpoint_like_pair(700, 900, 23)
    n0, n1 = f0.copy(), f1.copy()
    n0[11, 2] = -np.inf
    n1[4, 0] = np.nan
    s0, s1 = sift_like_pair(600, 800, 24)
    matcher.set_descriptor_kind(matcher.DESC_SIFT, ctx)
    try:
        _check_knn2(f0, f1, ctx, oracle="c")
        _check_knn2(n0, n1, ctx, oracle="c")
        _check_knn2(s0, s1, ctx)
    finally:
        matcher.set_descriptor_kind(matcher.DESC_AUTO, ctx)


def test_query_cache_torch_cpu_tensors(ctx):
    """cache_query=True keeps the keyframe side (vo.py:64-65) packed across calls while the same
    unmodified torch tensor comes back; an in-place write (version bump) or another tensor
    repacks it.  Every result equals the oracle's."""
    torch = pytest.importorskip("torch")
    d0, d1 = sift_like_pair(1500, 1600, 21)
    _, d2 = sift_like_pair(1500, 1400, 22)
    t0 = torch.from_numpy(d0.copy())[None]
    for other in (d1, d2, d1):  # hit, hit (a different train side each time)
        got = matcher.match_knn2_ratio(t0, other, ctx=ctx, kind=matcher.DESC_SIFT, cache_query=True)
        np.testing.assert_array_equal(got, match_ref.match_int(d0, other))
    t0[0, 5, :] = t0[0, 9, :]  # in place: the cached rows are stale now
    m0 = t0[0].numpy().copy()
    got = matcher.match_knn2_ratio(t0, d1, ctx=ctx, kind=matcher.DESC_SIFT, cache_query=True)
    np.testing.assert_array_equal(got, match_ref.match_int(m0, d1))
    t1 = torch.from_numpy(d2.copy())[None]  # another keyframe
    got = matcher.match_knn2_ratio(t1, d1, ctx=ctx, kind=matcher.DESC_SIFT, cache_query=True)
    np.testing.assert_array_equal(got, match_ref.match_int(d2, d1))
    # a float query behind the cache takes the exact sweep, as an uncached call does
    f0 = torch.from_numpy((d0 + 0.25).astype(np.float32))[None]
    got = matcher.match_knn2_ratio(f0, d1, ctx=ctx, kind=matcher.DESC_SIFT, cache_query=True)
    np.testing.assert_array_equal(got, matcher.match_knn2_ratio(f0[0].numpy(), d1, ctx=ctx))


def test_query_cache_tag_and_pointer_keyed(ctx):
    """The C-level cache key: (pointer, n0, dim, tag).  The same tag with another pointer or
    size is a miss; numpy arrays are never cached by the Python layer (no version counter)."""
    from visualodometry_amd._lib import C, check, ptr

    d0, d1 = sift_like_pair(700, 900, 31)
    e0, _ = sift_like_pair(700, 900, 32)
    out = np.empty((700, 2), dtype=np.int32)
    cnt = np.zeros(1, dtype=np.int32)
    for a in (d0, e0, d0[:650].copy()):
        check(ctx.lib.vo_match_knn2_ratio_q(ctx.handle, ptr(a, C.c_float), a.shape[0], C.c_uint64(7),
                                            ptr(d1, C.c_float), d1.shape[0], 128, 0.75, ptr(out, C.c_int32),
                                            ptr(cnt, C.c_int32)), "q")
        np.testing.assert_array_equal(out[: cnt[0]], match_ref.match_int(a, d1))
    assert matcher._tags(ctx).tag_for(d0) == 0


def test_dev_entry_refuses_host_pointers(ctx):
    """vo_match_knn2_ratio_dev validates both pointers as this runtime's device memory of the
    context's GPU before any launch: host memory is VO_ERR_ARG, never a kernel fault."""
    from visualodometry_amd import _lib
    from visualodometry_amd._lib import C, ptr

    d0, d1 = sift_like_pair(64, 64, 41)
    out = np.empty((64, 2), dtype=np.int32)
    cnt = np.zeros(1, dtype=np.int32)
    rc = ctx.lib.vo_match_knn2_ratio_dev(ctx.handle, C.c_void_p(d0.ctypes.data), 64, C.c_uint64(0),
                                         C.c_void_p(d1.ctypes.data), 64, 128, 0.75, ptr(out, C.c_int32),
                                         ptr(cnt, C.c_int32))
    assert rc == _lib.VO_ERR_ARG
    # device memory of the library itself is accepted, and a range past its allocation is not
    a = _lib.DeviceArray.from_numpy(ctx, d0)
    b = _lib.DeviceArray.from_numpy(ctx, d1)
    rc = ctx.lib.vo_match_knn2_ratio_dev(ctx.handle, C.c_void_p(a.ptr), 64, C.c_uint64(0), C.c_void_p(b.ptr), 64,
                                         128, 0.75, ptr(out, C.c_int32), ptr(cnt, C.c_int32))
    assert rc == _lib.VO_OK
    np.testing.assert_array_equal(out[: cnt[0]], match_ref.match_int(d0, d1))
    big = np.empty((64 + 4096, 2), dtype=np.int32)  # rows far past the allocation (any rounding of it)
    rc = ctx.lib.vo_match_knn2_ratio_dev(ctx.handle, C.c_void_p(a.ptr), 64 + 4096, C.c_uint64(0), C.c_void_p(b.ptr),
                                         64, 128, 0.75, ptr(big, C.c_int32), ptr(cnt, C.c_int32))
    assert rc == _lib.VO_ERR_ARG
