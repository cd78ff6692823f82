"""torch and libvo_hip.so in one process, torch first.

The reference's ``frontend.py:3`` imports torch and moves tensors to the GPU
(``:66-67``) before any hook runs, and torch ships its own ``libamdhip64`` under the
same SONAME as the one libvo_hip.so links.  ``tests/torch_coexist_check.py`` runs in a
fresh process so that torch really is initialised first; it checks match_frames (through
the hook, torch-tensor descriptors), one SlidingWindowBA.optimize and one SIFT
detectAndCompute against the oracle, then uses torch again.
"""

import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
SCRIPT = Path(__file__).resolve().parent / "torch_coexist_check.py"


def test_torch_then_libvo_hip_in_one_process():
    try:
        import torch  # noqa: F401
    except ImportError:
        pytest.skip("torch is not importable on this box")
    r = subprocess.run([sys.executable, str(SCRIPT)], capture_output=True, text=True, timeout=240)
    out = r.stdout + r.stderr
    if "SKIP:" in r.stdout:
        pytest.skip(r.stdout.strip())
    assert r.returncode == 0, out[-4000:]
    assert r.stdout.strip().splitlines()[-1] == "OK", out[-4000:]
