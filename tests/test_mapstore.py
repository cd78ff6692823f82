"""Map store and trajectory evaluation on CPU: ``MapStore`` behaves as
the reference's ``map_points`` dict (``vo.py:17,35-47,123-130,281,349``) under the
reference's access pattern, and the ATE of a trajectory is invariant to the similarity
that monocular VO leaves unobservable."""

import numpy as np
import pytest

from visualodometry_amd.dropin import hooks
from visualodometry_amd.mapstore import MAX_POINTS, MapStore, ate, trajectory_xz, umeyama


def _keyframe_sequence(store, ref, rng, n_kf=30, max_new=3000, cap=MAX_POINTS):
    nxt = 0
    for _ in range(n_kf):
        k = int(rng.integers(0, max_new))
        X = rng.normal(0, 10, (k, 3)).astype(np.float32)
        for x in X:  # vo.py:279-283
            store[nxt] = x
            ref[nxt] = x
            nxt += 1
        thr = nxt - cap  # _prune_map, vo.py:35-47
        if isinstance(store, MapStore):
            store.prune_below(thr)
        else:
            for pid in [p for p in store if p < thr]:
                del store[pid]
        for pid in [p for p in ref if p < thr]:
            del ref[pid]
        yield nxt


def test_behaves_as_the_dict():
    rng = np.random.default_rng(0)
    store, ref = MapStore(), {}
    for nxt in _keyframe_sequence(store, ref, rng):
        assert len(store) == len(ref) and list(store) == list(ref)
        probe = rng.integers(-5, nxt + 5, 500)
        assert [p in store for p in probe] == [p in ref for p in probe]
        np.testing.assert_array_equal(store.contains(probe), [p in ref for p in probe])
        live = probe[store.contains(probe)]
        got = np.array([store[p] for p in live]).reshape(-1, 3)  # vo.py:130
        want = np.array([ref[p] for p in live]).reshape(-1, 3)
        assert got.dtype == np.float32
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(store.gather(live), want)
    ids, xyz = store.arrays()
    np.testing.assert_array_equal(ids, sorted(ref))
    np.testing.assert_array_equal(xyz, np.array([ref[i] for i in ids]).reshape(-1, 3))
    assert [k for k, _ in store.items()] == list(ref)


def test_dict_style_prune_and_errors():
    store, ref = MapStore(capacity=50), {}
    rng = np.random.default_rng(1)
    for _ in _keyframe_sequence(store, ref, rng, n_kf=10, max_new=30, cap=50):
        pass
    with pytest.raises(KeyError):
        store[-1]
    with pytest.raises(KeyError):
        store.gather([0])
    small = MapStore(capacity=2, slots=4)
    for i in range(4):
        small[i] = np.zeros(3)
    with pytest.raises(OverflowError):  # slot 0 still holds id 0
        small[4] = np.zeros(3)
    small.prune_below(2)
    small[4] = np.ones(3)
    assert 4 in small and 0 not in small and len(small) == 3
    small.scatter([4], [[1, 2, 3]])
    np.testing.assert_array_equal(small[4], [1, 2, 3])


def test_hooks_swap_in_the_store_and_prune_vectorised():
    class V:
        def __init__(self, K, config):
            self.K, self.cfg, self.map_points, self.next_pt_id = K, config, {}, 0

        def _prune_map(self):
            raise AssertionError("the vectorised prune replaces this")

        def _reset_system(self):
            self.map_points = {}

    class Cfg:
        pnp_on_gpu = True
        map_store_arrays = True

    V.__init__ = hooks._wrap_init(V.__init__)
    V._prune_map = hooks._wrap_prune(V._prune_map)
    V._reset_system = hooks._wrap_reset(V._reset_system)
    vo = V(np.eye(3), Cfg())
    assert isinstance(vo.map_points, MapStore)
    for i in range(MAX_POINTS + 10):
        vo.map_points[i] = np.zeros(3, np.float32)
    vo.next_pt_id = MAX_POINTS + 10
    vo._prune_map()
    assert len(vo.map_points) == MAX_POINTS and 9 not in vo.map_points and 10 in vo.map_points
    vo._reset_system()
    assert isinstance(vo.map_points, MapStore) and len(vo.map_points) == 0


def test_cv2_proxy_routes_only_solvepnpransac():
    import types

    real = types.SimpleNamespace(solvePnPRansac=lambda *a, **k: "cpu", Rodrigues=lambda r: "rodrigues")
    on = [False]
    proxy = hooks.Cv2Proxy(real, lambda: on[0])
    assert proxy.Rodrigues(None) == "rodrigues"
    assert proxy.solvePnPRansac(np.zeros((6, 3)), np.zeros((6, 2)), np.eye(3), None) == "cpu"
    from tests.conftest import gpu_available

    if gpu_available():
        pytest.skip("GPU present: covered by the GPU tests")
    on[0] = True
    from visualodometry_amd import _lib

    with pytest.raises(_lib.VoError):  # the MI355X path needs the device: never a CPU path
        proxy.solvePnPRansac(np.zeros((6, 3), np.float32), np.zeros((6, 2), np.float32), np.eye(3), None)


def test_ate_is_similarity_invariant():
    rng = np.random.default_rng(2)
    gt = np.cumsum(rng.normal(0, 1, (300, 2)), axis=0)
    th, s, t = 0.7, 0.05, np.array([3.0, -2.0])
    R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    est = (gt @ R.T) * s + t  # a monocular estimate: unknown rotation, scale, offset
    r = ate(est, gt)
    assert r["rmse"] < 1e-9 and abs(r["scale"] - 1 / s) < 1e-9
    noisy = est + rng.normal(0, 0.01 * s, est.shape)
    r2 = ate(noisy, gt)
    assert 0.005 < r2["rmse"] < 0.03
    rigid = ate(gt + [1.0, 2.0], gt, with_scale=False)
    assert rigid["rmse"] < 1e-9 and rigid["scale"] == 1.0
    s2, R2, t2 = umeyama(est, gt)
    np.testing.assert_allclose(R2, R.T, atol=1e-12)


def test_trajectory_xz_layout():
    tr = [np.array([1.0, 2.0, 3.0]), np.array([4.0, 5.0, 6.0])]  # vo.trajectory entries
    np.testing.assert_array_equal(trajectory_xz(tr), [[1.0, 3.0], [4.0, 6.0]])  # GT cols 3, 11


def test_items_values_keys_vectorised_equal_dict():
    """items()/values()/keys() come from one vectorised pass and equal the
    dict they replace, in id order, with float32 coordinates."""
    import time

    rng = np.random.default_rng(3)
    store, ref = MapStore(), {}
    for pid in range(25000):
        x = rng.normal(size=3).astype(np.float32)
        store[pid] = x
        ref[pid] = x
    store.prune_below(5000)
    for pid in range(5000):
        del ref[pid]
    assert list(store.keys()) == list(ref.keys())
    assert 5000 in store.keys() and 4999 not in store.keys()  # KeysView containment (__contains__)
    for (k, v), (rk, rv) in zip(store.items(), ref.items()):
        assert k == rk and np.array_equal(v, rv) and v.dtype == np.float32
    assert all(np.array_equal(a, b) for a, b in zip(store.values(), ref.values()))
    t0 = time.perf_counter()
    n = sum(1 for _ in store.items())
    assert n == 20000 and time.perf_counter() - t0 < 0.5
