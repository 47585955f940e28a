"""The bandwidth regime's restructured stage-B kernel against the one it replaces, bitwise.

k_bw_b (the fused stage B on plain rows) issues a row's loads in four dependency levels instead
of k_it_b MODE 0's walk per entry, but keeps its arithmetic and its order (entries summed in
adjacency order, the slots finished by lane 0 with the records broadcast from the lanes that
fetched them).  So K trips of the inner loop on the bandwidth-regime path (lrs_set_kernel_path
2) must give bit-identical R, G, D, A(RR^T), lambda and L-BFGS pairs with k_bw_b (LRS_BW_B=1)
and with k_it_b (LRS_BW_B=0): read once per process, hence one subprocess per setting.

Cases: torus rows (every entry prefetched), mc_lp60 (an LP cone beside the SDP one: diagonal
rows whose slots lie in several constraints), random sparse problems of low degree
(instances.random_sparse_problem: rows longer than the window, slots shared by constraints; with
k = 2 global constraints too); mc_rand200 / theta40 / rsparse60 rows are dense enough for teams
(T > 1): they run k_it_b either way and pin that the switch leaves them alone."""
import os
import subprocess
import sys

import numpy as np
import pytest

from golden_util import ROOT, instance

pytestmark = pytest.mark.gpu

RUN = r"""
import importlib, sys
import numpy as np
sys.path.insert(0, {root!r})
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
src = {path!r}
if src.startswith("rsp:"):
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    n, m, k, seed = (int(x) for x in src[4:].split(":"))
    sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(n, m, k, seed)))
else:
    sv = solver.Solver(src)
sv.set_kernel_path(2)
r = sv.alm_steps({K}, reoptLevel=0)
arr = {{k: np.asarray(r[k]) for k in ("R", "G", "cvs", "lam", "s", "y", "tau", "inner")}}
arr["D"] = sv.get_factor(solver.D)
arr["q1"] = sv.get_vec(solver.Q1)
np.savez({out!r}, **arr)
sv.close()
"""


def run(path, K, out, env_over):
    env = dict(os.environ)
    env.update(env_over)
    code = RUN.format(root=ROOT, path=path, K=K, out=out)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(out)


@pytest.mark.parametrize("name,K", [("mc_torus12x10", 12), ("mc_rand200", 12), ("theta40", 8), ("rsparse60", 8),
                                    ("mc_lp60", 8), ("rsp:400:1200:1:11", 10), ("rsp:600:900:2:12", 10)])
def test_bw_kernels_bitwise(tmp_path, name, K):
    src = name if name.startswith("rsp:") else instance(name)
    new = run(src, K, str(tmp_path / "new.npz"), {"LRS_BW_B": "1"})
    old = run(src, K, str(tmp_path / "old.npz"), {"LRS_BW_B": "0"})
    assert int(new["inner"]) == int(old["inner"]) == K
    for key in ("R", "G", "cvs", "lam", "s", "y", "tau", "D"):
        assert np.array_equal(new[key], old[key]), (name, key, float(np.max(np.abs(new[key] - old[key]))))


@pytest.mark.parametrize("name,K", [("mc_torus12x10", 12), ("mc_lp60", 8), ("rsp:400:1200:1:11", 10)])
def test_fused_stage_a_matches_split(tmp_path, name, K):
    """Stage A as one launch in the bandwidth regime (k_it_a MODE 0 at U = 1: the lower neighbours'
    D recomputed from G and the pairs; the default for factors up to 32 MB) against the split
    form (LRS_A_FUSED=0: D written by MODE 1, read back by MODE 2): the same formulas, so K trips
    agree to rounding (the recomputed D may fuse the other of its two-product sums)."""
    src = name if name.startswith("rsp:") else instance(name)
    fused = run(src, K, str(tmp_path / "fused.npz"), {"LRS_A_FUSED": "1"})
    split = run(src, K, str(tmp_path / "split.npz"), {"LRS_A_FUSED": "0"})
    assert int(fused["inner"]) == int(split["inner"]) == K
    for key in ("R", "G", "cvs", "lam", "s", "y", "D"):
        a, b = fused[key], split[key]
        err = float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
        assert err <= 1e-12, (name, key, err)
