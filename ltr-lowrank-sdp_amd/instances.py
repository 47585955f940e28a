"""Seeded synthetic SDPA instances for the BASELINE configs.

The real Gset / SDPLIB files named by BASELINE.json (G1, G22, G67, G81, theta3)
are not in the reference checkout (`.MISSING_LARGE_BLOBS`), so every config is
restated as a generator with the same structure:

* MaxCut (lorads/data/gen_MaxCut.jl:213-243): A_i = e_i e_i^T, b_i = 1, and the
  objective written as ``0 1 i j v`` with v = L_ij / 2 for i <= j, so the
  reader's ``C = -F0`` (io/lorads_file_io.c:317-319) gives C = -L/2.
* Lovász theta: C = -J (dense), tr(X) = 1, X_ij = 0 on edges.
* random sparse SDP (C5): C = I (or dense), A_i with k random lower entries,
  b_i = <A_i, I> so X = I is feasible.
* MaxCut with an LP block (the SDPA negative block size, io/lorads_file_io.c:104-194):
  X_ii + s_i = 1 with LP slacks s_i >= 0, plus LP columns that touch many constraints.

Files are written in plain SDPA ``.dat-s`` text, one entry per line.
"""
from __future__ import annotations

import os

import numpy as np

__all__ = [
    "maxcut_random",
    "maxcut_torus",
    "maxcut_torus_problem",
    "coo_arrays",
    "theta",
    "theta_multiblock",
    "random_sparse",
    "random_sparse_problem",
    "write_sdpa",
    "config_instance",
    "maxcut_lp",
]


def write_sdpa(path, m, dims, b, entries):
    """entries: iterable of arrays (con, blk, i, j, v) with 1-based blk/i/j, i <= j."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        f.write(f"{m}\n{len(dims)}\n")
        f.write(" ".join(str(int(d)) for d in dims) + "\n")
        f.write(" ".join(repr(float(x)) for x in b) + "\n")
        for con, blk, ii, jj, vv in entries:
            con = np.asarray(con, dtype=np.int64)
            blk = np.broadcast_to(np.asarray(blk, dtype=np.int64), con.shape)
            ii, jj, vv = np.asarray(ii), np.asarray(jj), np.asarray(vv, dtype=float)
            for a in range(0, con.size, 1 << 20):   # chunks: a dense C has 5e7 entries at n = 1e4
                z = slice(a, a + (1 << 20))
                f.writelines(f"{c} {bk} {i} {j} {v!r}\n"
                             for c, bk, i, j, v in zip(con[z].tolist(), blk[z].tolist(), ii[z].tolist(),
                                                       jj[z].tolist(), vv[z].tolist()))
    return path


def coo_arrays(problem):
    """(m, dims, b, entries) -> dict of flat arrays for Solver(coo=...) / lrs_load_coo."""
    m, dims, b, entries = problem
    con, blk, row, col, val = [], [], [], [], []
    for c, bk, ii, jj, vv in entries:
        c = np.asarray(c, dtype=np.int32)
        con.append(c)
        blk.append(np.broadcast_to(np.asarray(bk, dtype=np.int32), c.shape))
        row.append(np.asarray(ii, dtype=np.int32))
        col.append(np.asarray(jj, dtype=np.int32))
        val.append(np.asarray(vv, dtype=np.float64))
    cat = lambda xs, t: np.ascontiguousarray(np.concatenate(xs).astype(t))
    return dict(m=int(m), dims=np.asarray(dims, dtype=np.int32), b=np.asarray(b, dtype=np.float64),
                con=cat(con, np.int32), blk=cat(blk, np.int32), row=cat(row, np.int32), col=cat(col, np.int32),
                val=cat(val, np.float64))


def _maxcut_problem(n, ei, ej, w):
    """MaxCut SDP (m, dims, b, entries) from an edge list (0-based, i != j)."""
    lo = np.minimum(ei, ej)
    hi = np.maximum(ei, ej)
    deg = np.zeros(n)
    np.add.at(deg, lo, w)
    np.add.at(deg, hi, w)
    # objective: 0.5 * L, L = D - A: off-diagonal -w/2, diagonal deg/2
    obj_i = np.concatenate([lo, np.arange(n)]) + 1
    obj_j = np.concatenate([hi, np.arange(n)]) + 1
    obj_v = np.concatenate([-0.5 * w, 0.5 * deg])
    keep = np.abs(obj_v) >= 1e-12
    con_i = np.arange(1, n + 1)
    entries = [
        (np.zeros(int(keep.sum()), dtype=np.int64), 1, obj_i[keep], obj_j[keep], obj_v[keep]),
        (con_i, 1, con_i, con_i, np.ones(n)),
    ]
    return n, [n], np.ones(n), entries


def _maxcut_from_edges(path, n, ei, ej, w):
    return write_sdpa(path, *_maxcut_problem(n, ei, ej, w))


def maxcut_random(path, n, n_edges, seed, weights="one"):
    """G1/G22-like: uniform random graph with exactly n_edges edges."""
    rng = np.random.default_rng(seed)
    total = n * (n - 1) // 2
    pick = rng.choice(total, size=n_edges, replace=False)
    # unrank pair index -> (i, j), i < j
    i = (n - 2 - np.floor(np.sqrt(-8 * pick + 4 * n * (n - 1) - 7) / 2.0 - 0.5)).astype(np.int64)
    j = (pick + i + 1 - n * (n - 1) // 2 + (n - i) * ((n - i) - 1) // 2).astype(np.int64)
    w = np.ones(n_edges) if weights == "one" else rng.choice([-1.0, 1.0], size=n_edges)
    return _maxcut_from_edges(path, n, i, j, w)


def maxcut_torus(path, rows, cols, seed):
    """G67/G81-like: 2-D toroidal grid rows x cols, weights uniform in {-1, +1}."""
    return write_sdpa(path, *maxcut_torus_problem(rows, cols, seed))


def maxcut_torus_problem(rows, cols, seed):
    """The maxcut_torus instance in memory: (m, dims, b, entries)."""
    rng = np.random.default_rng(seed)
    n = rows * cols
    idx = np.arange(n).reshape(rows, cols)
    right = np.roll(idx, -1, axis=1)
    down = np.roll(idx, -1, axis=0)
    ei = np.concatenate([idx.ravel(), idx.ravel()])
    ej = np.concatenate([right.ravel(), down.ravel()])
    w = rng.choice([-1.0, 1.0], size=ei.size)
    return _maxcut_problem(n, ei, ej, w)


def _theta_entries(n, ei, ej, blk, con0):
    iu, ju = np.triu_indices(n)
    entries = [(np.zeros(iu.size, dtype=np.int64), blk, iu + 1, ju + 1, np.ones(iu.size))]
    d = np.arange(1, n + 1)
    entries.append((np.full(n, con0, dtype=np.int64), blk, d, d, np.ones(n)))
    lo = np.minimum(ei, ej) + 1
    hi = np.maximum(ei, ej) + 1
    entries.append((con0 + 1 + np.arange(ei.size), blk, lo, hi, np.ones(ei.size)))
    return entries


def _random_edges(rng, n, n_edges):
    total = n * (n - 1) // 2
    pick = rng.choice(total, size=n_edges, replace=False)
    i = (n - 2 - np.floor(np.sqrt(-8 * pick + 4 * n * (n - 1) - 7) / 2.0 - 0.5)).astype(np.int64)
    j = (pick + i + 1 - n * (n - 1) // 2 + (n - i) * ((n - i) - 1) // 2).astype(np.int64)
    return i, j


def theta(path, n, n_edges, seed):
    """theta3-like Lovász theta SDP (single block, dense C = -J)."""
    rng = np.random.default_rng(seed)
    ei, ej = _random_edges(rng, n, n_edges)
    m = 1 + n_edges
    b = np.zeros(m)
    b[0] = 1.0
    return write_sdpa(path, m, [n], b, _theta_entries(n, ei, ej, 1, 1))


def theta_multiblock(path, n, n_edges, nblocks, seed):
    """Block-diagonal stack of independent theta instances (multi-cone coverage)."""
    rng = np.random.default_rng(seed)
    entries, b = [], []
    con0 = 1
    for blk in range(1, nblocks + 1):
        ei, ej = _random_edges(rng, n, n_edges)
        entries += _theta_entries(n, ei, ej, blk, con0)
        b += [1.0] + [0.0] * n_edges
        con0 += 1 + n_edges
    return write_sdpa(path, len(b), [n] * nblocks, np.array(b), entries)


def random_sparse_problem(n, m, k, seed, dense_c=False):
    """C5-like in memory: C = I (or dense), each A_i has k random lower-triangle N(0,1)
    entries, b_i = <A_i, I> (X = I feasible).  Returns (m, dims, b, entries)."""
    rng = np.random.default_rng(seed)
    ii = rng.integers(0, n, size=(m, k))
    jj = rng.integers(0, n, size=(m, k))
    lo = np.minimum(ii, jj)
    hi = np.maximum(ii, jj)
    v = rng.standard_normal((m, k))
    b = np.where(lo == hi, v, 0.0).sum(axis=1)
    con = np.repeat(np.arange(1, m + 1), k)
    entries = []
    if dense_c:
        iu, ju = np.triu_indices(n)
        cv = rng.standard_normal(iu.size) / np.sqrt(n)
        cv[iu == ju] += n
        entries.append((np.zeros(iu.size, dtype=np.int64), 1, iu + 1, ju + 1, -cv))
    else:
        d = np.arange(1, n + 1)
        entries.append((np.zeros(n, dtype=np.int64), 1, d, d, -np.ones(n)))
    entries.append((con, 1, lo.ravel() + 1, hi.ravel() + 1, v.ravel()))
    return m, [n], b, entries


def random_sparse(path, n, m, k, seed, dense_c=False):
    """random_sparse_problem written as a .dat-s file."""
    return write_sdpa(path, *random_sparse_problem(n, m, k, seed, dense_c))


# BASELINE.json configs restated; small = parity-test sizes
CONFIGS = {
    "G1": dict(kind="maxcut_random", n=800, n_edges=19176, seed=1),
    "G22": dict(kind="maxcut_random", n=2000, n_edges=19990, seed=22),
    "G67": dict(kind="maxcut_torus", rows=100, cols=100, seed=67),
    "G81": dict(kind="maxcut_torus", rows=100, cols=200, seed=81),
    "theta3": dict(kind="theta", n=150, n_edges=1105, seed=3),
    "theta3x3": dict(kind="theta_multiblock", n=150, n_edges=1105, nblocks=3, seed=3),
    "R2000": dict(kind="maxcut_torus", rows=2000, cols=2000, seed=2000),
    "C5": dict(kind="random_sparse", n=10000, m=1000000, k=6, seed=5),
}


def config_instance(name, directory):
    """Write (once) and return the path of a config instance."""
    spec = dict(CONFIGS[name])
    kind = spec.pop("kind")
    path = os.path.join(directory, f"{name}.dat-s")
    if os.path.exists(path):
        return path
    fn = {"maxcut_random": maxcut_random, "maxcut_torus": maxcut_torus, "theta": theta,
          "theta_multiblock": theta_multiblock, "random_sparse": random_sparse}[kind]
    tmp = path + f".tmp{os.getpid()}"
    fn(tmp, **spec)
    os.replace(tmp, path)
    return path


def maxcut_lp(path, n, p_edge, seed):
    """MaxCut relaxation with inequality constraints through an LP block (LoRADS's LP cone,
    data/lorads_lp_conic.c): SDP block n (C = -L/2 of a G(n, p) graph, unit weights), LP block of
    n + 3 columns.  Constraint i (1..n): X_ii + s_i + [i % 3 == 0] 0.01 d = 1 (slack s_i, column i;
    d = column n + 3 touches every third constraint: a dense LP column, >= 25 % of the rows);
    constraint n + 1: X_12 + t_1 - t_2 = 0 (columns n + 1, n + 2: a free variable split in two).
    LP costs c_s = 0.1, c_t = 0.5, c_d = 1 (written as F0 = -c, the reader's C = -F0)."""
    rng = np.random.default_rng(seed)
    iu, ju = np.triu_indices(n, 1)
    keep = rng.random(iu.size) < p_edge
    ei, ej = iu[keep], ju[keep]
    m = n + 1
    nlp = n + 3
    deg = np.zeros(n)
    np.add.at(deg, ei, 1.0)
    np.add.at(deg, ej, 1.0)
    ents = []
    # SDP objective F0 = L / 2 (C = -L/2)
    ents.append((np.zeros(ei.size, int), 1, ei + 1, ej + 1, -0.5 * np.ones(ei.size)))
    ents.append((np.zeros(n, int), 1, np.arange(n) + 1, np.arange(n) + 1, 0.5 * deg))
    # LP objective F0 = -c
    cs = np.concatenate([np.full(n, 0.1), [0.5, 0.5, 1.0]])
    ents.append((np.zeros(nlp, int), 2, np.arange(nlp) + 1, np.arange(nlp) + 1, -cs))
    # X_ii + s_i (+ 0.01 d) = 1
    ents.append((np.arange(n) + 1, 1, np.arange(n) + 1, np.arange(n) + 1, np.ones(n)))
    ents.append((np.arange(n) + 1, 2, np.arange(n) + 1, np.arange(n) + 1, np.ones(n)))
    rows3 = np.arange(0, n, 3)
    ents.append((rows3 + 1, 2, np.full(rows3.size, n + 3), np.full(rows3.size, n + 3), np.full(rows3.size, 0.01)))
    # X_12 + t_1 - t_2 = 0 (SDP entry (1, 2) is the symmetric pair: coefficient 1/2 each side)
    ents.append((np.array([m]), 1, np.array([1]), np.array([2]), np.array([0.5])))
    ents.append((np.array([m, m]), 2, np.array([n + 1, n + 2]), np.array([n + 1, n + 2]), np.array([1.0, -1.0])))
    b = np.concatenate([np.ones(n), [0.0]])
    return write_sdpa(path, m, [n, -nlp], b, ents)
