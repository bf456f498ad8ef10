import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


def _have_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not _have_gpu():
        pytest.skip("no ROCm GPU in this container")
    import torch
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture
def knobs():
    """Set library knobs for one test and restore them after it.  The library
    reads the environment once, when it is loaded (syncfast_amd/csrc/
    sf_knobs.cpp), so tests set knobs through the test hook
    (include/syncfast_amd_test.h), not with monkeypatch.setenv."""
    from syncfast_amd import _lib
    saved = {}

    class Knobs:
        def set(self, name, value):
            old = _lib.set_knob(name, int(value))
            saved.setdefault(name, old)

        def get(self, name):
            return _lib.get_knob(name)

    yield Knobs()
    for name, value in saved.items():
        _lib.set_knob(name, value)
