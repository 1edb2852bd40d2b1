import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libicx.so on cuda:0)")


@pytest.fixture(scope="session")
def oracle():
    from tests.oracle_ffi import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    from tests.oracle_ffi import load_golden
    return load_golden()


@pytest.fixture(scope="session")
def codec():
    import icx
    try:
        import torch
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
    except ImportError:
        pass
    c = icx.Codec(0)
    yield c
    c.close()
