"""Shared fixtures.  `gpu` marks tests that need an MI355X (run with -m gpu)."""
import importlib
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (HIP path)")


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module("ltr-lowrank-sdp_amd")


@pytest.fixture(scope="session")
def oracle_lib():
    """CPU restatement (test infrastructure only), built on demand."""
    import ctypes as C
    so = os.path.join(ROOT, "oracle", "_build", "liblrsdp_oracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    lib = C.CDLL(so)
    lib.oracle_read.restype = C.c_void_p
    lib.oracle_read.argtypes = [C.c_char_p]
    lib.oracle_free.argtypes = [C.c_void_p]
    lib.oracle_kernels.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.oracle_solve.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_double)]
    lib.oracle_alm_rate.restype = C.c_long
    lib.oracle_alm_rate.argtypes = [C.c_char_p, C.c_int, C.c_double, C.POINTER(C.c_double)]
    lib.oracle_rand_seq.argtypes = [C.c_uint, C.c_int, C.POINTER(C.c_int)]
    return lib
