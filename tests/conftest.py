"""Shared fixtures.  GPU tests are marked @pytest.mark.gpu; everything else
runs on the CPU (the driver runs `pytest -m "not gpu"` here)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def reload_library_settings():
    """libmchecksum reads its MCHECKSUM_* settings once per process; a test
    that changes them re-reads them (mchecksum_gpu_reload_settings)."""
    from mercury_amd import _lib
    if _lib._lib is not None:
        _lib.reload_settings()


class _SettingsMonkeyPatch(pytest.MonkeyPatch):
    """monkeypatch whose setenv / delenv of an MCHECKSUM_* variable, and whose
    undo, make the library re-read its settings."""

    def setenv(self, name, value, prepend=None):
        super().setenv(name, value, prepend)
        if name.startswith("MCHECKSUM_"):
            reload_library_settings()

    def delenv(self, name, raising=True):
        super().delenv(name, raising)
        if name.startswith("MCHECKSUM_"):
            reload_library_settings()


@pytest.fixture
def monkeypatch():
    mp = _SettingsMonkeyPatch()
    yield mp
    mp.undo()
    reload_library_settings()


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def product_lib():
    """libmchecksum.so (built by `make`; the CPU test run builds the
    host-only objects if hipcc output is absent)."""
    from mercury_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-s", "-C", ROOT, "all"], check=True)
    return _lib.load_library()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    from mercury_amd import gpu as G
    assert G.gpu_available(), "libmchecksum sees no HIP device"
    return G


@pytest.fixture(autouse=True)
def _no_queue_faults(request):
    """Every GPU test also checks that the batch kernels' work queue never gave
    up a wait (crc_gpu_device.h: bounded waits count a fault instead of
    hanging)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch
    if not torch.cuda.is_available():
        return
    from mercury_amd import gpu as G
    assert G.queue_faults() == 0, "work-queue protocol fault counted (mchecksum_gpu_queue_faults)"
