import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session", autouse=True)
def _oracle_built():
    """The oracle restatement is test infrastructure: build it (and, where /root/reference exists,
    the real reference into oracle/_ref) before any test runs."""
    so = os.path.join(ROOT, "oracle", "_build", "libatz_oracle.so")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], capture_output=True, text=True)
    if r.returncode != 0 and not os.path.exists(so):
        pytest.exit("oracle build failed:\n" + r.stdout + r.stderr)
    yield
