import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pkg(sub=None):
    """The product package (directory name `multimodal-s2ut_amd`, imported by path)."""
    return importlib.import_module("multimodal-s2ut_amd" + (f".{sub}" if sub else ""))


def golden_files(prefix):
    return sorted(os.path.join(GOLDEN, f) for f in os.listdir(GOLDEN) if f.startswith(prefix))


@pytest.fixture(scope="session")
def mm():
    return pkg()
