import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-successor-features-for-transfer_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsfx.so on the GPU)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
        return cache[name]

    return load


@pytest.fixture(autouse=True)
def _device_bounds_checks(request):
    """With SFX_CHECK_RUN=1 and SFX_LIB pointing at the bounds-check build (libsfx_check.so,
    `make -C deep-successor-features-for-transfer_amd/csrc check`): every GPU test must end with no
    failed device bounds check (sfx_check_failures; SURVEY §5 debug mode)."""
    yield
    if os.environ.get("SFX_CHECK_RUN") != "1" or request.node.get_closest_marker("gpu") is None or not gpu_available():
        return
    import ctypes

    from sfx import _lib

    n = ctypes.c_longlong()
    rec = (ctypes.c_longlong * 32)()
    assert _lib.lib.sfx_check_failures(ctypes.byref(n), rec, 1) == 0
    assert n.value >= 0, "SFX_CHECK_RUN=1 needs SFX_LIB=.../libsfx_check.so (the product build has no checks)"
    assert n.value == 0, f"{n.value} device bounds checks failed; first (line, a, b, c): " + \
        str([tuple(rec[4 * i:4 * i + 4]) for i in range(min(n.value, 8))])
