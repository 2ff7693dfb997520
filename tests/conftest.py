import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binius-ntt_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running case")


@pytest.fixture(scope="session")
def ntt_md5():
    with open(os.path.join(GOLDEN, "additive_ntt_md5.json")) as f:
        return json.load(f)["hashes"]


@pytest.fixture(scope="session")
def field_kats():
    with open(os.path.join(GOLDEN, "field_kats.json")) as f:
        return json.load(f)["kats"]


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        import binius_ntt_amd as B
        if B.check_gpu_capabilities():
            pytest.fail("the HIP engine sees a gfx950 GPU but torch does not (torch.cuda.is_available() is False)")
        pytest.skip("no GPU")
    return torch.device("cuda:0")
