import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running")


_gpu_ok = None


def gpu_available() -> bool:
    """A gfx950 device reachable through libvo_hip.so itself (no torch in the GPU path)."""
    global _gpu_ok
    if _gpu_ok is None:
        from visualodometry_amd import _lib

        try:
            _lib.context(int(os.environ.get("VO_DEVICE", "0")))
            _gpu_ok = True
        except _lib.VoError:
            _gpu_ok = False
    return _gpu_ok


@pytest.fixture(scope="session")
def ctx():
    """The library context on device 0 -- a GPU test never falls back to the CPU."""
    if not gpu_available():
        pytest.skip("no GPU in this container (run with -m gpu on the MI355X box)")
    from visualodometry_amd import _lib

    return _lib.context(int(os.environ.get("VO_DEVICE", "0")))
