"""Shared test setup.

`-m "not gpu"` tests run in the CPU container: oracle vs golden fixtures and
known-answer tests, the libm / introsort pins, host logic, and the C-ABI symbol
check.  `-m gpu` tests call the HIP product through the C-ABI and compare it
with the oracle (test infrastructure only)."""
import importlib.util
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")
    config.addinivalue_line("markers", "slow: long-running")


def _load_ffi():
    spec = importlib.util.spec_from_file_location("legoffi", REPO / "lego-loam_amd" / "legoffi.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules["legoffi"] = mod
    spec.loader.exec_module(mod)
    return mod


_built = False


def ensure_built():
    global _built
    if _built:
        return
    import __graft_entry__  # noqa: F401

    need = [REPO / "oracle/build/liblego_oracle.so", REPO / "lego-loam_amd/build/liblego_synth.so",
            REPO / "lego-loam_amd/build/liblego_hip.so"]
    if not all(p.exists() for p in need):
        __graft_entry__.build()
    _built = True


@pytest.fixture(scope="session")
def L():
    ensure_built()
    # PyTorch ships its own HIP runtime next to /opt/rocm's, which our library
    # links.  Both work in one process only when torch's initialises first (a
    # later torch init reports "No HIP GPUs are available"), so GPU sessions
    # bring torch up before the first context is created, as bench.py does.
    if gpu_available():
        import torch

        torch.cuda.init()
    return _load_ffi()


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False
