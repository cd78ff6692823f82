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
    global _gpu_ok
    if _gpu_ok is None:
        try:
            import torch

            _gpu_ok = bool(torch.cuda.is_available())
        except Exception:
            _gpu_ok = False
    return _gpu_ok


@pytest.fixture(scope="session")
def ctx():
    """The library context on device 0 -- a GPU test never falls back to the CPU."""
    if not gpu_available():
        pytest.skip("no GPU in this container (run with -m gpu on the MI355X box)")
    from visualodometry_amd import _lib

    return _lib.context(int(os.environ.get("VO_DEVICE", "0")))
