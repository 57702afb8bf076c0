import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from tests.oracle_lib import Oracle

    return Oracle()


@pytest.fixture(scope="session")
def refo():
    from tests.oracle_lib import RefOracle, ref_available

    if not ref_available():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    return RefOracle()


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="session", params=["md5", "table"])
def tag_mode(request):
    """Both tag modes of the library (rsk_set_tag_mode): "md5" = one MD5 compression per packet and
    lane (the default, as util/rhash.cpp:20-41), "table" = the key's 256-entry tag table.  Every GPU
    test that takes `codec` (or this fixture) runs in both and must give identical bytes."""
    return request.param


@pytest.fixture(scope="session")
def codec(gpu, tag_mode):
    from rsock_amd.codec import Codec

    c = Codec(b"hello135", 0, tag_mode=tag_mode)
    assert c.tag_mode == tag_mode
    yield c
    c.close()
