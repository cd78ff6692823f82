"""ctypes binding of ``libvo_hip.so`` (the C-ABI declared in ``include/vo_hip.h``).

The product path has no CPU fallback: if the library or a gfx950 device is
missing, :func:`context` raises.  ``load()`` alone (no device needed) is used by
the CPU test-suite to check that every declared symbol is exported.
"""

from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

# VO_LIB_PATH selects an alternative build of the same library (tuning experiments)
LIB_PATH = Path(os.environ.get("VO_LIB_PATH") or Path(__file__).resolve().parent / "lib" / "libvo_hip.so")
HEADER = Path(__file__).resolve().parents[1] / "include" / "vo_hip.h"
# test-only entry points (the loopback communicator, the split-reduce switch), outside the product header
TEST_HEADER = HEADER.with_name("vo_hip_testing.h")

VO_OK = 0
VO_ERR_ARG = -1
VO_ERR_HIP = -2
VO_ERR_NOT_SPD = -3
VO_ERR_RCCL = -4
VO_ERR_NOMEM = -5
VO_ERR_STATE = -6
VO_ERR_NODEV = -7
STATUS_NAMES = {
    VO_OK: "ok", VO_ERR_ARG: "bad argument", VO_ERR_HIP: "HIP error",
    VO_ERR_NOT_SPD: "not positive definite", VO_ERR_RCCL: "RCCL error",
    VO_ERR_NOMEM: "out of device memory", VO_ERR_STATE: "bad call order",
    VO_ERR_NODEV: "no gfx950 device",
}


class VoError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


class BAProblemC(C.Structure):
    _fields_ = [
        ("n_poses", C.c_int32), ("n_points", C.c_int32), ("n_obs", C.c_int32),
        ("n_fixed", C.c_int32),
        ("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
        ("lam", C.c_double),
        ("point_ptr", C.POINTER(C.c_int32)), ("obs_cam", C.POINTER(C.c_int32)),
        ("obs_uv", C.POINTER(C.c_float)),
    ]


_P = C.c_void_p
_I = C.c_int
_D = C.c_double
_PI32 = C.POINTER(C.c_int32)
_PF = C.POINTER(C.c_float)
_PD = C.POINTER(C.c_double)
_PI64 = C.POINTER(C.c_int64)

# name -> (restype, argtypes); must cover every function in include/vo_hip.h
SIGNATURES = {
    "vo_abi_version": (_I, []),
    "vo_last_error": (C.c_char_p, []),
    "vo_create": (_P, [_I, _I]),
    "vo_destroy": (None, [_P]),
    "vo_stream": (_P, [_P]),
    "vo_synchronize": (_I, [_P]),
    "vo_device_alloc": (_P, [_P, C.c_uint64]),
    "vo_device_free": (_I, [_P, _P]),
    "vo_memcpy_h2d": (_I, [_P, _P, _P, C.c_uint64]),
    "vo_memcpy_d2h": (_I, [_P, _P, _P, C.c_uint64]),
    "vo_match_knn2_ratio": (_I, [_P, _PF, _I, _PF, _I, _I, _D, _PI32, _PI32]),
    "vo_match_knn2_ratio_q": (_I, [_P, _PF, _I, C.c_uint64, _PF, _I, _I, _D, _PI32, _PI32]),
    "vo_match_knn2_ratio_dev": (_I, [_P, C.c_void_p, _I, C.c_uint64, C.c_void_p, _I, _I, _D, _PI32, _PI32]),
    "vo_match_knn2": (_I, [_P, _PF, _I, _PF, _I, _I, _PI32, _PF]),
    "vo_match_batch_async": (_I, [_P, _P, _P, _I, _I, _I, _I, _D, _P]),
    "vo_match_hint": (_I, [_P, _I]),
    "vo_ba_setup": (_I, [_P, C.POINTER(BAProblemC), C.POINTER(C.c_uint64)]),
    "vo_ba_set_state": (_I, [_P, C.c_uint64, _PD, _PD]),
    "vo_ba_reserve": (_I, [_P, _I, _I, C.c_int64, _I]),
    "vo_ba_get_state": (_I, [_P, C.c_uint64, _PD, _PD]),
    "vo_ba_run": (_I, [_P, C.c_uint64, _I, _PD]),
    "vo_ba_run_async": (_I, [_P, C.c_uint64, _I]),
    "vo_ba_gn_step": (_I, [_P, C.c_uint64, _PD, _PD, _PD, _PD]),
    "vo_ba_solve": (_I, [_P, C.POINTER(BAProblemC), _PD, _PD, _I, _PD]),
    "vo_ba_plan_stats": (_I, [_P, _PI64, _I]),
    "vo_ba_debug_stamps": (_I, [_P, C.POINTER(C.c_uint64), _I]),
    "vo_ba_group_by_point": (_I, [_I, _I, _PI32, _PI32, _PI32]),
    "vo_ba_plan_probe": (_I, [C.POINTER(BAProblemC), _I, _PI64, _I]),
    "vo_ba_plan_digest": (_I, [C.POINTER(BAProblemC), _I, C.POINTER(C.c_uint64)]),
    "vo_profile_enable": (_I, [_P, _I]),
    "vo_profile_read": (_I, [_P, _PD, _PI64]),
    "vo_comm_unique_id": (_I, [C.c_char_p]),
    "vo_triangulate": (_I, [_P, _PD, _PD, _PD, _PD, _PF, _PF, _I, C.c_double, C.c_double, _PF,
                            C.POINTER(C.c_uint8)]),
    "vo_triangulate_async": (_I, [_P, _PD, _PD, _PD, _PD, _P, _P, _I, C.c_double, C.c_double, _P, _P]),
    "vo_pnp_ransac": (_I, [_P, _PF, _PF, _I, _PD, _I, _D, _D, _PD, _PD, C.POINTER(C.c_uint8), _PI32]),
    "vo_pnp_ransac_batch_async": (_I, [_P, _P, _P, _PI32, _I, _PD, _I, _D, _D, _P, _P, _P]),
    "vo_pnp_subsets": (_I, [_I, _I, _PI32]),
    "vo_sift_detect": (_I, [_P, C.POINTER(C.c_uint8), _I, _I, _D, _D, _D, _I, _I, _PF, _PI32, _PI32]),
    "vo_sift_detect_batch_async": (_I, [_P, _P, _I, _I, _I, _D, _D, _D, _I, _I, _P, _P, _P]),
    "vo_sift_pyramid": (_I, [_P, C.POINTER(C.c_uint8), _I, _I, _D, _I, _PF, C.c_int64, _PF, C.c_int64]),
    "vo_sift_layout": (_I, [_I, _I, _I, _PI64, _I]),
    "vo_sift_detect_and_compute": (_I, [_P, C.POINTER(C.c_uint8), _I, _I, _I, _D, _D, _D, _I, _I, _P, _PF, _PI32]),
    "vo_sift_detect_and_compute_dev": (_I, [_P, C.POINTER(C.c_uint8), _I, _I, _I, _D, _D, _D, _I, _I, C.c_void_p, C.c_void_p, C.POINTER(C.c_int32)]),
    "vo_sift_detect_and_compute_batch_async": (_I, [_P, _P, _I, _I, _I, _I, _D, _D, _D, _I, _I, _P, _P, _P]),
    "vo_comm_init": (_I, [_P, _I, _I, C.c_char_p]),
    "vo_comm_init_loopback": (_I, [_P, _I, _I, C.c_char_p]),
    "vo_ba_split_reduce": (_I, [_P, _I]),
    "vo_ba_testing_no_split": (_I, [_P, _I]),
    "vo_ba_testing_drop_reducers": (_I, [_P, _I]),
    "vo_ba_testing_k1": (_I, [_P, _I]),
    "vo_pnp_testing_split": (_I, [_P, _I]),
    "vo_pnp_testing_group": (_I, [_P, _I]),
    "vo_pnp_testing_last_split": (_I, [_P, _PI32, _PI32]),
    "vo_ba_testing_plan_slide": (_I, [C.c_void_p, C.c_void_p, _I, _I, C.POINTER(C.c_uint64), _PI64]),
}

_lib = None
_lock = threading.Lock()


def load() -> C.CDLL:
    """Loads the in-tree library (raises if it was not built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not LIB_PATH.exists():
                raise RuntimeError(
                    f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                    " (hipcc --offload-arch=gfx950)"
                )
            lib = C.CDLL(str(LIB_PATH))
            tuning = bool(os.environ.get("VO_LIB_PATH"))
            for name, (res, args) in SIGNATURES.items():
                try:
                    fn = getattr(lib, name)
                except AttributeError:
                    if tuning:  # an older tuning build (A/B runs): entry points it predates stay unbound
                        continue
                    raise
                fn.restype = res
                fn.argtypes = args
            if lib.vo_abi_version() != 1:
                raise RuntimeError("libvo_hip.so ABI mismatch")
            _lib = lib
    return _lib


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        msg = load().vo_last_error().decode(errors="replace")
        raise VoError(rc, f"{what}: {msg}" if what else msg)
    return rc


class Context:
    """Owns a ``vo_ctx`` (one gfx950 device + stream)."""

    def __init__(self, device: int = 0):
        lib = load()
        h = lib.vo_create(device, 0)
        if not h:
            raise VoError(VO_ERR_NODEV, lib.vo_last_error().decode(errors="replace"))
        self.handle = h
        self.device = device
        self.lib = lib

    def close(self):
        if getattr(self, "handle", None):
            self.lib.vo_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_contexts: dict[int, Context] = {}


def context(device: int | None = None) -> Context:
    """Process-wide default context per device (``VO_DEVICE`` or 0)."""
    if device is None:
        device = int(os.environ.get("VO_DEVICE", "0"))
    with _lock:
        ctx = _contexts.get(device)
    if ctx is None:
        ctx = Context(device)
        with _lock:
            _contexts.setdefault(device, ctx)
            ctx = _contexts[device]
    return ctx


class DeviceArray:
    """A dense array in the context device's HBM (owned; freed on close/GC)."""

    def __init__(self, ctx: "Context", shape, dtype):
        import numpy as np

        self.ctx = ctx
        self.shape = tuple(int(x) for x in shape)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = ctx.lib.vo_device_alloc(ctx.handle, self.nbytes)
        if not p:
            raise VoError(VO_ERR_NOMEM, ctx.lib.vo_last_error().decode(errors="replace"))
        self.ptr = p

    @classmethod
    def from_numpy(cls, ctx: "Context", a) -> "DeviceArray":
        import numpy as np

        a = np.ascontiguousarray(a)
        d = cls(ctx, a.shape, a.dtype)
        check(ctx.lib.vo_memcpy_h2d(ctx.handle, d.ptr, a.ctypes.data, d.nbytes), "vo_memcpy_h2d")
        return d

    def numpy(self):
        import numpy as np

        out = np.empty(self.shape, self.dtype)
        check(self.ctx.lib.vo_memcpy_d2h(self.ctx.handle, out.ctypes.data, self.ptr, self.nbytes),
              "vo_memcpy_d2h")
        return out

    def close(self):
        if getattr(self, "ptr", None):
            self.ctx.lib.vo_device_free(self.ctx.handle, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


KERNEL_NAMES = ["ba_lin", "ba_reduce", "ba_solve", "match_pack", "match_i8", "match_f32",
                "match_merge", "triangulate", "pnp_hyp", "pnp_score", "pnp_final", "sift_pyramid",
                "sift_extrema", "sift_orient", "sift_select", "sift_desc", "match_rerank", "pnp_decide",
                "pnp_hyp_tail", "pnp_score_tail"]


def profile_enable(ctx: "Context", on: bool = True) -> None:
    check(ctx.lib.vo_profile_enable(ctx.handle, int(on)), "vo_profile_enable")


def profile_read(ctx: "Context") -> dict:
    """{kernel: (total_ms, launches)} from HIP events on the library stream."""
    import numpy as np

    ms = np.zeros(len(KERNEL_NAMES))
    cnt = np.zeros(len(KERNEL_NAMES), dtype=np.int64)
    check(ctx.lib.vo_profile_read(ctx.handle, ptr(ms, C.c_double), ptr(cnt, C.c_int64)),
          "vo_profile_read")
    return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(KERNEL_NAMES) if cnt[i]}


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    check(load().vo_comm_unique_id(buf), "vo_comm_unique_id")
    return buf.raw


def comm_init(ctx: "Context", nranks: int, rank: int, uid: bytes) -> None:
    check(ctx.lib.vo_comm_init(ctx.handle, nranks, rank, uid), "vo_comm_init")


def comm_init_loopback(ctx: "Context", nranks: int, rank: int, group: bytes) -> None:
    """Test stand-in for :func:`comm_init`: joins the in-process loopback group ``group``
    (contexts of this process, one host thread each); see vo_comm_init_loopback."""
    gid = C.create_string_buffer(group[:128].ljust(128, b"\0"), 128)
    check(ctx.lib.vo_comm_init_loopback(ctx.handle, nranks, rank, gid), "vo_comm_init_loopback")


def ba_split_reduce(ctx: "Context", on: bool = True) -> None:
    """Test/tool switch: keep the BA's slab reduction a launch of its own on this context (the
    multi-rank layout); see vo_ba_split_reduce."""
    check(ctx.lib.vo_ba_split_reduce(ctx.handle, int(bool(on))), "vo_ba_split_reduce")


def ba_testing_drop_reducers(ctx: "Context", n: int) -> None:
    """Test switch: fused launches of this context leave out ``n`` reducer workgroups, so
    the solver's bounded wait times out; see vo_ba_testing_drop_reducers."""
    check(ctx.lib.vo_ba_testing_drop_reducers(ctx.handle, int(n)), "vo_ba_testing_drop_reducers")


def ba_testing_no_split(ctx: "Context", on: bool = True) -> None:
    """Test switch: the context's later setups never take the banded solver's split layout
    (ring layout instead, where one workgroup's LDS is too small); see vo_ba_testing_no_split."""
    check(ctx.lib.vo_ba_testing_no_split(ctx.handle, int(bool(on))), "vo_ba_testing_no_split")


def ba_reserve(ctx: "Context", n_poses: int, n_points: int, n_obs: int, n_fixed: int = 2) -> None:
    """``vo_ba_reserve``: pre-size the context's BA buffers for windows of about this size
    (once, before the first keyframe); the context has no BA problem afterwards."""
    check(ctx.lib.vo_ba_reserve(ctx.handle, int(n_poses), int(n_points), int(n_obs), int(n_fixed)),
          "vo_ba_reserve")


def ba_testing_k1(ctx: "Context", variant: int = 0) -> None:
    """Test switch: the K1 variant of the context's later setups (0 default, -1 four-wave K1,
    n = 1..6 one-wave K1 with n chunks per segment); see vo_ba_testing_k1."""
    check(ctx.lib.vo_ba_testing_k1(ctx.handle, int(variant)), "vo_ba_testing_k1")


def pnp_testing_group(ctx: "Context", mode: int = 0) -> None:
    """Test switch: the EPnP hypothesis kernel (0 auto, 1 lane groups, -1 one lane per
    hypothesis); see vo_pnp_testing_group."""
    check(ctx.lib.vo_pnp_testing_group(ctx.handle, int(mode)), "vo_pnp_testing_group")


def pnp_testing_split(ctx: "Context", h1: int = 0) -> None:
    """Test/tool switch: PnP calls of the context solve the first ``h1`` hypotheses of every
    frame before replaying the RANSAC loop (0 auto, -1 all at once); see vo_pnp_testing_split."""
    check(ctx.lib.vo_pnp_testing_split(ctx.handle, int(h1)), "vo_pnp_testing_split")


def pnp_testing_last_split(ctx: "Context") -> tuple:
    """(h1, tail_frames) of the context's last PnP call; see vo_pnp_testing_last_split."""
    h1, tail = C.c_int32(0), C.c_int32(0)
    check(ctx.lib.vo_pnp_testing_last_split(ctx.handle, C.byref(h1), C.byref(tail)), "vo_pnp_testing_last_split")
    return h1.value, tail.value


def ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))
