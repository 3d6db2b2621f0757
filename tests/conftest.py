import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
for p in (REPO, REPO / "convex-mpc-unitree-go2_amd", REPO / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device) and the HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def plan():
    import torch
    from cmpc import Plan, SolverParams
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return Plan(SolverParams(max_batch=65536))
