"""Shared test setup: import paths, the `gpu` marker, GPU detection."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microsoft-mpi_amd"))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def msxlib():
    import msx
    return msx.init(errors_return=True)


@pytest.fixture(scope="session")
def C():
    import msx
    return msx.C
