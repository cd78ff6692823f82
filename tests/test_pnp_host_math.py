"""The per-hypothesis math of the PnP kernels (csrc/pnp_math.h: EPnP with OpenCV's Jacobi
SVD, Householder least squares, the Rodrigues round trip), compiled for the host by
``pnp_host_check`` and run on CPU, against the oracle (oracle/pnp_ref.py) hypothesis by
hypothesis.  With the same operation order, no FMA contraction and the host's libm the
two are bitwise identical; on the GPU only the libm-level functions (hypot, acos, sin,
cos) round differently (tests/test_gpu_pnp.py)."""

import os
import subprocess
import tempfile
from pathlib import Path

import numpy as np
import pytest

from oracle import pnp_ref as P
from visualodometry_amd.synthetic import pnp_case

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "visualodometry_amd" / "lib" / "pnp_host_check"


@pytest.fixture(scope="module")
def exe():
    if not EXE.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "visualodometry_amd" / "csrc"), "../lib/pnp_host_check"],
                       check=True)
    return EXE


def host_models(exe, pw, us, K):
    with tempfile.TemporaryDirectory() as d:
        fi, fo = os.path.join(d, "in"), os.path.join(d, "out")
        with open(fi, "wb") as f:
            np.array([pw.shape[0]], np.int32).tofile(f)
            np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2]]).tofile(f)
            np.concatenate([pw.reshape(-1, 15), us.reshape(-1, 10)], 1).astype(np.float64).tofile(f)
        subprocess.run([str(exe), fi, fo], check=True)
        return np.fromfile(fo).reshape(-1, 25)


@pytest.mark.parametrize("seed,noise,frac", [(100, 0.3, 0.25), (7, 0.0, 0.0), (8, 2.0, 0.5)])
def test_hypotheses_bitwise_equal_oracle(exe, seed, noise, frac):
    X, uv, K, T, out = pnp_case(1000, seed, noise_px=noise, outlier_frac=frac)
    sub = P.ransac_subsets(1000, 100)
    pw, us = X[sub].astype(np.float64), uv[sub].astype(np.float64)
    h = host_models(exe, pw, us, K)
    R, t, ok = P.epnp(pw, us, K)
    rv = P.rodrigues_to_vec(np.where(ok[:, None, None], R, np.eye(3)))
    np.testing.assert_array_equal(h[:, 24] == 1, ok)
    np.testing.assert_array_equal(h[ok, :9], R[ok].reshape(-1, 9))
    np.testing.assert_array_equal(h[ok, 9:12], t[ok])
    np.testing.assert_array_equal(h[ok, 12:15], rv[ok])
    np.testing.assert_array_equal(h[ok, 15:24], P.rodrigues_to_mat(rv[ok]).reshape(-1, 9))
