import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kat_data():
    """rand.New(rand.NewSource(5)).Read(5,000,000 bytes) — repo/splitter/splitter_test.go:13-18."""
    from oracle import coracle
    return coracle.gorand_read(5, 5_000_000).tobytes()


@pytest.fixture(scope="session")
def gpu():
    """The product library with at least one gfx950 device; skips elsewhere."""
    from kopia_amd import _lib
    if _lib.lib().kcdc_device_count() < 1:
        pytest.skip("no gfx950 device")
    import torch
    assert torch.cuda.is_available()
    return torch.device("cuda:0")
