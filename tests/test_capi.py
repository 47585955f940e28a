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


def test_c_caller_null_context_contract(built, tmp_path):
    """include/lrsdp.h's error contract from a plain-C caller: every entry point handed a NULL
    context (or a NULL required output) returns a negative code with a message, no crash.  No
    context is created, so this needs no GPU."""
    exe = build_c_caller(tmp_path)
    r = subprocess.run([exe, "--null"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "CAPI_NULL failures=0" in r.stdout


def test_python_mirror_null_context(built):
    """The same contract through ctypes (the test mirror's binding)."""
    lib = C.CDLL(built)
    lib.lrs_last_error.restype = C.c_char_p
    for name, args in (("lrs_op_admm_half", (None, 0, 0, C.c_double(1.0), C.c_double(1e-8), 10, None, None)),
                       ("lrs_op_dual_update", (None, C.c_double(1.0))), ("lrs_op_admm_constr", (None,)),
                       ("lrs_set_log_path", (None, b"x.log")), ("lrs_load_sdpa", (None, b"x.dat-s", None)),
                       ("lrs_problem_info", (None, None, None, None, None, None))):
        assert getattr(lib, name)(*args) < 0, name
        assert b"null" in lib.lrs_last_error(), name


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["theta25x3", "mc_rand200", "rsparse60", "theta40"])
def test_c_caller_admm_sweep_matches_reference(built, tmp_path, name):
    """The C caller runs the reference's ADMM variable update (LORADSUpdateSDPVar: every cone, U
    then V, each followed by the cone's constraint refresh) through lrs_op_admm_half(cone, side)
    -- cones k > 0 included on theta25x3 -- and LORADSUpdateDualVar through lrs_op_dual_update,
    against the reference's own run on the same inputs (tests/golden/admm_sweep_*.npz,
    scripts/make_golden_admm.py, CG at cg_tol 1e-9).  Bars: factors and multipliers within 1e-6
    relative (the bar of the single half-step test); the CG counts -- hundreds of iterations on
    these random starting factors, where the residual curve is flat near the tolerance and the
    count follows the summation order -- of each cone's V solve within 25 % (50 % where the
    reference's count exceeds the n r unknowns of the solve: past CG's exact-arithmetic
    termination the count is set by rounding alone, e.g. theta25x3's 289 iterations for 125
    unknowns) and the total within 15 %."""
    import numpy as np
    exe = build_c_caller(tmp_path)
    g = np.load(os.path.join(ROOT, "tests", "golden", f"admm_sweep_{name}.npz"))
    k = np.load(os.path.join(ROOT, "tests", "golden", f"kernels_{name}.npz"))
    vec, m = k["inputs"], int(k["m"])
    dims = [int(d) for d in k["dims"]]
    rank = int(k["rank"])
    NR = sum(d * rank for d in dims)
    tail = vec[9 * NR + 2 * m:]
    inp = np.concatenate([vec[7 * NR:9 * NR], vec[9 * NR:9 * NR + m], [tail[3], float(g["cg_tol"])]])
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    inp.astype(np.float64).tofile(fin)
    inst = os.path.join(ROOT, "tests", "golden", "instances", f"{name}.dat-s")
    r = subprocess.run([exe, "--sweep", inst, str(rank), str(fin), str(fout)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = np.fromfile(fout, dtype=np.float64)
    U, V, lam, its = out[:NR], out[NR:2 * NR], out[2 * NR:2 * NR + m], out[2 * NR + m:]

    def rel(a, b):
        return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)
    assert rel(U, g["U"]) < 1e-6, rel(U, g["U"])
    assert rel(V, g["V"]) < 1e-6, rel(V, g["V"])
    assert rel(lam, g["lam"]) < 1e-6, rel(lam, g["lam"])
    for c in range(len(dims)):
        ref = float(g["cg_last"][c])
        bar = 0.5 if ref > dims[c] * rank else 0.25
        assert abs(its[2 * c + 1] - ref) <= max(2, bar * ref), (c, its, g["cg_last"])
    assert abs(its.sum() - float(g["cg_total"])) <= max(4, 0.15 * float(g["cg_total"])), (its, g["cg_total"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mc_rand200", "theta40"])
def test_c_caller_steps_alm_from_operators(built, tmp_path, name):
    """The reference's ALM inner loop (lorads_alm.c:1302-1379) stepped by a plain-C caller from
    the C-ABI operators alone -- lrs_op_lbfgs, lrs_op_q12, lrs_op_line_search,
    lrs_op_alm_update (setAsNegGrad + ALMupdateVar + the constrValSum update + ALMCalGrad +
    setlbfgsHisTwo) and lrs_op_dimacs (updateDimacsALM) -- from the reference's own state
    after its first trip (tests/golden/steps_<name>.npz K1: R, G, the newest L-BFGS pair and
    its beta, lambda, constrValSum; rho = 1/sqrt(sum of block sizes), the reference's initial
    penalty with initRho 0, data/lorads_solver.c:1598-1607), four more trips, against the
    reference's trips 2..5 and its state after trip 5 (the K5 dump).  Bars as the fused
    kernels' per-trip test: tau, ||G||^2 and pinf to 1e-9 relative with the same root count;
    R, G, A(RR^T), the newest pair and its beta to 1e-9 (norm-wise)."""
    import numpy as np
    exe = build_c_caller(tmp_path)
    z = np.load(os.path.join(ROOT, "tests", "golden", f"steps_{name}.npz"))
    dims = [int(d) for d in z["dims"]]
    m, nr = int(z["m"]), int(z["nr"])
    rank = nr // sum(dims)
    assert rank * sum(dims) == nr
    rho = 1.0 / np.sqrt(float(sum(dims)))
    assert int(z["K5_trips"].shape[0]) == 5
    inp = np.concatenate([z["K1_R"], z["K1_G"], z["K1_s"], z["K1_y"], z["K1_lam"], z["K1_cvs"],
                          [float(z["K1_beta"][0]), rho, 1.0]])
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    inp.astype(np.float64).tofile(fin)
    inst = os.path.join(ROOT, "tests", "golden", "instances", f"{name}.dat-s")
    nt = 4
    r = subprocess.run([exe, "--steps", inst, str(rank), str(fin), str(fout), str(nt)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = np.fromfile(fout, dtype=np.float64)
    trips = out[:4 * nt].reshape(nt, 4)
    o = 4 * nt
    R, G = out[o:o + nr], out[o + nr:o + 2 * nr]
    cvs, lam = out[o + 2 * nr:o + 2 * nr + m], out[o + 2 * nr + m:o + 2 * nr + 2 * m]
    s, y = out[o + 2 * nr + 2 * m:o + 3 * nr + 2 * m], out[o + 3 * nr + 2 * m:o + 4 * nr + 2 * m]
    beta = out[o + 4 * nr + 2 * m]
    ref = z["K5_trips"]
    tol = 1e-9
    for t in range(nt):
        tau, rn, lag, pinf = ref[t + 1]
        assert int(trips[t, 1]) == int(rn), (t, trips[t], ref[t + 1])
        for q, v in ((0, tau), (2, lag), (3, pinf)):
            assert abs(trips[t, q] - v) <= tol * abs(v), (t, q, trips[t, q], v)

    def rel(a, b):
        return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)
    for nm, got, want in (("R", R, z["K5_R"]), ("G", G, z["K5_G"]), ("cvs", cvs, z["K5_cvs"]), ("s", s, z["K5_s"]),
                          ("y", y, z["K5_y"])):
        assert rel(got, want) <= tol, (nm, rel(got, want))
    assert np.array_equal(lam, z["K5_lam"])
    assert abs(beta - float(z["K5_beta"][0])) <= tol * abs(float(z["K5_beta"][0])), (beta, z["K5_beta"])
