"""Shared test setup: import paths for the engine package and the oracle.

`-m "not gpu"` tests run anywhere (the oracle vs the reference's KATs, host-side
logic, ABI exports); `-m gpu` tests are the parity tests proper and call the HIP
engine through its C ABI.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "embeddingtables.jl_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def _gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc

    orc.lib()
    return orc


@pytest.fixture(scope="session")
def kat():
    import json

    with open(os.path.join(REPO, "tests", "golden", "kat.json")) as f:
        return json.load(f)
