"""Helpers shared by the parity tests: golden fixtures written by the reference
itself (scripts/make_golden.py) and the oracle call wrappers."""
import ctypes as C
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
KERNEL_CASES = ["mc_rand200", "mc_torus12x10", "mc_rand300w", "theta40", "theta25x3", "rsparse60"]


def instance(name):
    return os.path.join(GOLDEN, "instances", f"{name}.dat-s")


def load_kernels(name):
    z = np.load(os.path.join(GOLDEN, f"kernels_{name}.npz"))
    return {k: z[k] for k in z.files}


def load_solves():
    with open(os.path.join(GOLDEN, "solves.json")) as f:
        return json.load(f)


def split_inputs(g):
    m = int(g["m"])
    dims = [int(d) for d in g["dims"]]
    rank = int(g["rank"])
    NR = sum(n * rank for n in dims)
    v = g["inputs"]
    names = ["R", "D", "G", "s1", "y1", "s2", "y2", "U", "V"]
    out = {nm: v[i * NR:(i + 1) * NR] for i, nm in enumerate(names)}
    out["lam"] = v[9 * NR:9 * NR + m]
    out["cvs"] = v[9 * NR + m:9 * NR + 2 * m]
    tail = v[9 * NR + 2 * m:]
    out.update(rho=tail[0], beta1=tail[1], beta2=tail[2], rho_admm=tail[3], cg_tol=tail[4])
    out.update(m=m, dims=dims, rank=rank, NR=NR)
    return out


def split_outputs(out, m, NR, n0r0):
    o, p = {}, 0

    def take(k):
        nonlocal p
        v = out[p:p + k]
        p += k
        return v
    o["q1"] = take(m); o["p1"] = take(1)[0]; o["q2"] = take(m); o["p2"] = take(1)[0]
    o["cvs_rr"] = take(m); o["pinf_rr"] = take(1)[0]; o["pobj_rr"] = take(1)[0]
    o["grad"] = take(NR); o["lag"] = take(1)[0]
    o["tau"] = take(1)[0]; o["rootnum"] = take(1)[0]
    o["d_lbfgs2"] = take(NR); o["d_lbfgs1"] = take(NR)
    o["u_cg"] = take(NR); o["rhs_cg"] = take(n0r0); o["cg_iters"] = take(1)[0]
    return o


def rel_err(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def oracle_kernels(lib, name):
    g = load_kernels(name)
    s = split_inputs(g)
    p = lib.oracle_read(instance(name).encode())
    assert p, "oracle_read failed"
    inp = np.ascontiguousarray(g["inputs"], dtype=np.float64)
    out = np.zeros(inp.size * 2 + 1024)
    n = lib.oracle_kernels(p, s["rank"], inp.ctypes.data_as(C.POINTER(C.c_double)),
                           out.ctypes.data_as(C.POINTER(C.c_double)))
    lib.oracle_free(p)
    return g, split_outputs(out[:n], s["m"], s["NR"], s["dims"][0] * s["rank"])


def oracle_solve(lib, name, flags):
    return oracle_solve_path(lib, instance(name), flags)


def oracle_solve_path(lib, path, flags):
    arr = (C.c_char_p * len(flags))(*[f.encode() for f in flags])
    res = (C.c_double * 16)()
    rc = lib.oracle_solve(str(path).encode(), len(flags), arr, res)
    assert rc == 0
    keys = ["alm_inner", "alm_outer", "alm_pobj", "alm_dobj", "alm_pinf", "alm_gap", "alm_rho", "admm_iter",
            "admm_pobj", "admm_dobj", "admm_pinf", "admm_gap", "admm_rho", "solve_time", "rank", "alm_time"]
    return dict(zip(keys, list(res)))


def read_sdpa_dense(path):
    """Test-side SDPA reader (the contract of LReadSDPA, io/lorads_file_io.c:59-455: '*' / '"'
    comment lines, '{ ( ' ,' as separators, C = -F0, A_i = F_i, |v| < 1e-12 dropped, entries
    symmetric).  Returns m, block dims, b, dense C per block, A as {(i, blk): [(r, c, v)]}.
    LP blocks (negative dims) are not supported by this test-side reader (the device and oracle
    readers take them; tests/test_gpu_lp.py has its own LP-block reader)."""
    toks = []
    with open(path) as f:
        for line in f:
            s = line.strip()
            if not s or s[0] in '*"':
                continue
            for ch in "{}(),'":
                s = s.replace(ch, " ")
            toks.append(s.split())
    m = int(toks[0][0])
    nb = int(toks[1][0])
    dims = [abs(int(x)) for x in toks[2][:nb]]
    b = np.array([float(x) for x in toks[3][:m]])
    C = [np.zeros((d, d)) for d in dims]
    A = {}
    for t in toks[4:]:
        if len(t) < 5:
            continue
        i, blk, r, c, v = int(t[0]), int(t[1]) - 1, int(t[2]) - 1, int(t[3]) - 1, float(t[4])
        if abs(v) < 1e-12:
            continue
        if i == 0:
            C[blk][r, c] = -v
            C[blk][c, r] = -v
        else:
            A.setdefault((i - 1, blk), []).append((r, c, v))
    return m, dims, b, C, A


def block_traces(path):
    """Per block, tr(X_k) when one constraint is v I over that block alone (theta-type blocks,
    each with its own trace constraint), else None for the file."""
    with open(path) as f:
        toks = [t for ln in f if not ln.lstrip().startswith(("*", '"')) for t in ln.replace(",", " ").replace("{", " ")
                .replace("}", " ").replace("(", " ").replace(")", " ").split()]
    m, nb = int(toks[0]), int(toks[1])
    dims = [abs(int(float(t))) for t in toks[2:2 + nb]]
    b = [float(t) for t in toks[2 + nb:2 + nb + m]]
    ents = {}
    q = 2 + nb + m
    while q + 4 < len(toks):
        c, blk, i, j, v = int(toks[q]), int(toks[q + 1]), int(toks[q + 2]), int(toks[q + 3]), float(toks[q + 4])
        q += 5
        if c >= 1 and v != 0.0:
            ents.setdefault(c, []).append((blk, i, j, v))
    tr = [None] * nb
    for c, e in ents.items():
        blks = {blk for blk, *_ in e}
        if len(blks) != 1:
            continue
        k = next(iter(blks)) - 1
        if len(e) == dims[k] and all(i == j for _, i, j, _ in e) and len({v for *_, v in e}) == 1 and \
                len({i for _, i, _, _ in e}) == dims[k]:
            tr[k] = b[c - 1] / e[0][3]
    return None if any(t is None for t in tr) else tr


def fixed_trace(path):
    """tr(X) when the constraints fix it for every feasible X of the SDPA file at `path`, else
    None: either every diagonal entry of every block is its own single-entry constraint
    v X_kk = b (MaxCut-type diag(X) = b / v), or one constraint is v I over all blocks (theta-type
    tr(X) = b / v).  Used for the weak-duality bound <C, X> >= b^T lambda + lambda_min(S) tr(X)."""
    with open(path) as f:
        toks = [t for ln in f if not ln.lstrip().startswith(("*", '"')) for t in ln.replace(",", " ").replace("{", " ")
                .replace("}", " ").replace("(", " ").replace(")", " ").split()]
    m, nb = int(toks[0]), int(toks[1])
    dims = [abs(int(float(t))) for t in toks[2:2 + nb]]
    b = [float(t) for t in toks[2 + nb:2 + nb + m]]
    ents = {}
    q = 2 + nb + m
    while q + 4 < len(toks):
        c, blk, i, j, v = int(toks[q]), int(toks[q + 1]), int(toks[q + 2]), int(toks[q + 3]), float(toks[q + 4])
        q += 5
        if c >= 1 and v != 0.0:
            ents.setdefault(c, []).append((blk, i, j, v))
    ndiag = sum(dims)
    diag = {}
    for c, e in ents.items():
        if len(e) == 1 and e[0][1] == e[0][2]:
            diag[(e[0][0], e[0][1])] = b[c - 1] / e[0][3]
    if len(diag) == ndiag:
        return sum(diag.values())
    for c, e in ents.items():
        if len(e) == ndiag and all(i == j for _, i, j, _ in e) and len({v for *_, v in e}) == 1 and \
                len({(blk, i) for blk, i, _, _ in e}) == ndiag:
            return b[c - 1] / e[0][3]
    return None
