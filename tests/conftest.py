import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "knowledge-graph-embedding_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def hiplib():
    """The built libkge_hip.so (GPU tests require it; no fallback)."""
    import __graft_entry__
    __graft_entry__.build()
    from KGE import _hip
    return _hip.lib()
