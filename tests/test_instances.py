"""Synthetic instance generators and the oracle reader on them."""
import os

import numpy as np


def test_maxcut_torus_structure(tmp_path, pkg, oracle_lib):
    p = pkg.instances.maxcut_torus(str(tmp_path / "t.dat-s"), 6, 7, seed=3)
    lines = open(p).read().split("\n")
    assert lines[0] == "42" and lines[1] == "1" and lines[2] == "42"
    ent = [l.split() for l in lines[4:] if l.strip()]
    cons = [e for e in ent if e[0] != "0"]
    assert len(cons) == 42 and all(e[2] == e[3] == e[0] and float(e[4]) == 1.0 for e in cons)
    # objective = L/2 on the upper triangle: row sums of L vanish
    n = 42
    L = np.zeros((n, n))
    for e in ent:
        if e[0] == "0":
            i, j, v = int(e[2]) - 1, int(e[3]) - 1, float(e[4])
            L[i, j] += 2 * v
            if i != j:
                L[j, i] += 2 * v
    assert np.allclose(L.sum(axis=1), 0.0)
    assert oracle_lib.oracle_read(p.encode())


def test_random_graph_edge_count(tmp_path, pkg):
    p = pkg.instances.maxcut_random(str(tmp_path / "r.dat-s"), 50, 300, seed=1)
    ent = [l.split() for l in open(p).read().split("\n")[4:] if l.strip()]
    off = [e for e in ent if e[0] == "0" and e[2] != e[3]]
    assert len(off) == 300
    assert len({(e[2], e[3]) for e in off}) == 300


def test_generators_deterministic(tmp_path, pkg):
    a = pkg.instances.random_sparse(str(tmp_path / "a.dat-s"), 30, 50, 3, seed=9)
    b = pkg.instances.random_sparse(str(tmp_path / "b.dat-s"), 30, 50, 3, seed=9)
    assert open(a).read() == open(b).read()
