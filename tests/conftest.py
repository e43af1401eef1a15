import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through libnrk.so)")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU in this container")
    from newsrecommend_amd import _lib

    _lib.load()  # fail loudly if the HIP library is missing on a GPU box
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def oracle_knn():
    from oracle import knn_oracle

    return knn_oracle
