"""The C-ABI library loads and exports every symbol include/lrsdp.h declares
(no compute: runs on CPU-only machines)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ltr-lowrank-sdp_amd", "_build", "liblrsdp.so")
BIN = os.path.join(ROOT, "ltr-lowrank-sdp_amd", "_build", "LoRADS_v_2_0_1-alpha")
HDR = os.path.join(ROOT, "include", "lrsdp.h")


def declared_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(lrs_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "ltr-lowrank-sdp_amd", "csrc"), "-j8"], check=True,
                       capture_output=True)
    return LIB


def test_header_declares_boundary():
    fns = declared_functions()
    for f in ["lrs_ctx_create", "lrs_load_sdpa", "lrs_op_q12", "lrs_op_grad", "lrs_solve", "lrs_write_json"]:
        assert f in fns


def test_library_exports_every_declared_symbol(built):
    out = subprocess.run(["nm", "-D", "--defined-only", built], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (lrs_[a-z0-9_]+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing


def test_library_loads_and_reports(built):
    lib = C.CDLL(built)
    lib.lrs_version.restype = C.c_char_p
    assert b"gfx950" in lib.lrs_version()


def test_params_default_matches_reference_defaults(built, pkg):
    from importlib import import_module
    solver = import_module("ltr-lowrank-sdp_amd.solver")
    p = solver.default_params()
    # main.c:56-86
    assert p.rhoMax == 5000.0 and p.maxALMIter == 200 and p.maxADMMIter == 10000
    assert p.timesLogRank == 2.0 and p.phase1Tol == 1e-3 and p.phase2Tol == 1e-5
    assert p.lbfgsListLength == 2 and p.endTauTol == 1e-16 and p.endALMSubTol == 1e-10
    assert p.reoptLevel == 2 and p.dyrankLevel == 2 and p.ALMRhoFactor == 2.0


def test_cli_binary_built_for_benchmark_py(built):
    # benchmark.py:25 resolves this executable name
    assert os.path.exists(BIN) and os.access(BIN, os.X_OK)


def build_c_caller(tmpdir):
    """gcc (plain C11) against include/lrsdp.h, linked to liblrsdp.so."""
    exe = os.path.join(str(tmpdir), "capi_solve")
    src = os.path.join(ROOT, "tests", "c", "capi_solve.c")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), src, "-o", exe,
                        "-L", os.path.dirname(LIB), "-llrsdp", "-Wl,-rpath," + os.path.dirname(LIB)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_c_caller_compiles_and_links(built, tmp_path):
    exe = build_c_caller(tmp_path)
    assert os.access(exe, os.X_OK)


@pytest.mark.gpu
def test_c_caller_solves_like_reference(built, tmp_path):
    """The C caller solves the golden MaxCut instance through the C-ABI: objective against the
    reference's solve (tests/golden/solves.json) within 1e-6, and the JSON it writes has the
    reference's key set."""
    import json
    exe = build_c_caller(tmp_path)
    inst = os.path.join(ROOT, "tests", "golden", "instances", "mc_rand200.dat-s")
    js = tmp_path / "o.json"
    r = subprocess.run([exe, inst, str(js), "0"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    m = re.search(r"pobj=(\S+)", r.stdout)
    ref = [s for s in json.load(open(os.path.join(ROOT, "tests", "golden", "solves.json")))
           if s["instance"] == "mc_rand200" and s["flags"] == ["--reoptLevel", "0"]][0]
    assert abs(float(m.group(1)) - ref["result"]["admm_pobj"]) <= 1e-6 * abs(ref["result"]["admm_pobj"])
    out = json.load(open(js))
    assert set(out["metrics"]) == set(ref["json"]["metrics"])
