import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libptsharp_hip.so)")
    config.addinivalue_line("markers", "slow: long CPU test")


def gpu_available() -> bool:
    try:
        import ctypes as C

        from ptsharp_amd import _abi
        lib = _abi.load_library()
        n = C.c_int32(0)
        return lib.pt_device_count(C.byref(n)) == 0 and n.value > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device / libptsharp_hip.so (no CPU fallback exists)")
    return 0
