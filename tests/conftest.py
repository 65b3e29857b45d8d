import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs through libcwq.so")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    O.lib()
    return O


@pytest.fixture(scope="session")
def mathcheck():
    import ctypes
    import subprocess
    so = os.path.join(REPO, "tests", "native", "libcwq_mathcheck.so")
    subprocess.check_call(["make", "-C", REPO, "tests/native/libcwq_mathcheck.so"],
                          stdout=subprocess.DEVNULL)
    return ctypes.CDLL(so)


@pytest.fixture(scope="session")
def cwqlib():
    from compression_without_quantization_amd import build as B
    B.build(verbose=False)
    from compression_without_quantization_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))
    return load
