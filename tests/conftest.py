import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = "/root/reference"  # read only as DATA (fixtures), never imported; absent on GPU boxes


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "stepwise_only: a shape only the stepwise path covers")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    return torch.device("cuda:0")
