"""pytest configuration: import paths, the `gpu` marker, shared fixtures.

`-m "not gpu"` (CPU, this container): oracle known-answer tests, reference
golden fixtures, host logic, C-ABI load/exports, host-only filter parity,
gloo multi-process sharding.  `-m gpu` (MI355X box): HIP parity vs the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "processing-chain_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    from pixpath import ops
    ops.context(0)
    return torch.device("cuda", 0)
