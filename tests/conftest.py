import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "one-class-ffm_amd")
for p in (PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: larger-than-tiny inputs")


def _ensure_built():
    lib = os.path.join(PKG, "libocffm.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", PKG, "-j4"], check=True)
    oracle = os.path.join(REPO, "oracle", "liboracle.so")
    if not os.path.exists(oracle) or not os.path.exists(os.path.join(REPO, "oracle", "oracle_train")):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def tiny():
    import synth
    return synth.tiny()


@pytest.fixture(scope="session")
def kk_small():
    import synth
    return synth.kkbox_small()
