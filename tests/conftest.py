import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")


@pytest.fixture(scope="session")
def port():
    from oracle.oracle import Port
    return Port()


@pytest.fixture(scope="session")
def ref():
    from oracle.oracle import Ref
    if not Ref.available():
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    return Ref()


@pytest.fixture(scope="session")
def hip():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import lifeapi_amd.hip as h
    return h
