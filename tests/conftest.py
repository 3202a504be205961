import importlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PKG_NAME = "infrared-colorization-with-resnet-generator-and-patchgan_amd"
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")


def pkg():
    return importlib.import_module(PKG_NAME)


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, f"step_{name}.npz")))


@pytest.fixture(scope="session")
def irgan():
    return pkg()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
