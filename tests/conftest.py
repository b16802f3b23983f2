import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fem-glass-tempering_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU and the built libtvfem.so")
    # the reference writes its five output series every step, and so does
    # ThermoViscoProblem by default; the test session turns that off (tests that
    # check the writers pass write_output=True, and python main.py keeps it on)
    from tvfem.problem import ThermoViscoProblem
    ThermoViscoProblem.WRITE_OUTPUT_DEFAULT = False


@pytest.fixture(scope="session")
def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
