"""The C-ABI library builds, loads and exports every symbol include/*.h declares (no GPU)."""

import re

import numpy as np
import pytest

from visualodometry_amd import _lib


def header_functions(path=None):
    paths = [path] if path else [_lib.HEADER, _lib.TEST_HEADER]
    text = "".join(p.read_text() for p in paths)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vo_[a-z0-9_]+)\s*\(", text)))


def test_library_loads_and_abi_version():
    lib = _lib.load()
    assert lib.vo_abi_version() == 1


def test_every_declared_function_is_exported_and_bound():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} not exported by libvo_hip.so"
        assert n in _lib.SIGNATURES, f"{n} has no ctypes signature in _lib.py"
    assert set(_lib.SIGNATURES) <= set(names)


def test_product_header_has_no_test_entry_points():
    """The loopback communicator and the split-reduce switch are test-only: declared in
    vo_hip_testing.h, not vo_hip.h."""
    assert "vo_comm_init_loopback" not in header_functions(_lib.HEADER)
    assert header_functions(_lib.TEST_HEADER) == ["vo_ba_split_reduce", "vo_ba_testing_drop_reducers",
                                                  "vo_ba_testing_k1", "vo_ba_testing_no_split",
                                                  "vo_ba_testing_plan_slide", "vo_comm_init_loopback", "vo_pnp_testing_group",
                                                  "vo_pnp_testing_last_split", "vo_pnp_testing_split"]


def test_no_device_fails_loudly(monkeypatch):
    from tests.conftest import gpu_available

    if gpu_available():
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.VoError) as e:
        _lib.Context(0)
    assert e.value.code in (_lib.VO_ERR_NODEV, _lib.VO_ERR_HIP)


def test_matcher_has_no_cpu_fallback():
    from tests.conftest import gpu_available

    if gpu_available():
        pytest.skip("a GPU is present")
    from visualodometry_amd import matcher

    d = np.zeros((4, 128), np.float32)
    with pytest.raises(_lib.VoError):
        matcher.match_knn2_ratio(d, d)


def test_pnp_host_entry_points_validate_arguments():
    """vo_pnp_subsets runs on the host; bad arguments come back as VO_ERR_ARG with a message."""
    import ctypes as C

    lib = _lib.load()
    out = np.zeros((4, 5), np.int32)
    assert lib.vo_pnp_subsets(5, 4, out.ctypes.data_as(C.POINTER(C.c_int32))) == _lib.VO_ERR_ARG
    assert b"count > 5" in lib.vo_last_error()
    assert lib.vo_pnp_subsets(6, 4, out.ctypes.data_as(C.POINTER(C.c_int32))) == _lib.VO_OK
    assert all(len(set(r)) == 5 for r in out)
