"""Two contexts driven from two host threads at once (include/lrsdp.h allows it): the library
keeps no module-level device state -- the finals that the generic L-BFGS loop's line search and
the standalone operators reduce into live in each context (lrs_ctx s_fin / s_tmpfin / s_tickets /
s_rpart, bound to the calling thread).  Thread A runs the --lbfgsListLength 3 inner trips
(run_inner_generic: op_q12_fin + the device line search on every trip) against the reference's
(steps_mc_rand200_l3.npz); thread B repeats the white-box line search (ALMCalq12p12 +
ALMLineSearch) on theta40 against the reference's (kernels_theta40.npz).  ctypes releases the
GIL around every library call, so the two threads' calls interleave on the device.  Both at
1e-9, as their single-thread tests."""
import importlib
import os
import threading

import numpy as np
import pytest

from golden_util import GOLDEN, instance, load_kernels, rel_err, split_inputs

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module")
def solver_mod():
    return importlib.import_module("ltr-lowrank-sdp_amd.solver")


def test_two_contexts_two_threads(solver_mod):
    errors = []
    start = threading.Barrier(2)

    def ring_of_three():
        try:
            z = np.load(os.path.join(GOLDEN, "steps_mc_rand200_l3.npz"))
            sv = solver_mod.Solver(os.path.join(GOLDEN, "instances", "mc_rand200.dat-s"))
            start.wait()
            for _ in range(3):
                for K in [int(k) for k in z["ks"]]:
                    trips = z[f"K{K}_trips"]
                    if trips.shape[0] < K:
                        continue
                    d = sv.alm_steps(K, reoptLevel=0, lbfgsListLength=3)
                    tau, rn, lag, pinf = trips[K - 1]
                    assert d["inner"] == K, (K, d["inner"])
                    assert abs(d["tau"] - tau) <= TOL * abs(tau), (K, d["tau"], tau)
                    assert abs(d["lag"] - lag) <= TOL * abs(lag), (K, d["lag"], lag)
                    assert abs(d["pinf"] - pinf) <= TOL * max(abs(pinf), 1e-300), (K, d["pinf"], pinf)
                    for key in ("R", "G", "s", "y"):
                        assert rel_err(d[key], z[f"K{K}_{key}"]) < TOL, (K, key)
            sv.close()
        except BaseException as e:   # reported by the main thread
            errors.append(("ring_of_three", repr(e)))

    def line_search():
        try:
            g = load_kernels("theta40")
            s = split_inputs(g)
            sv = solver_mod.Solver(instance("theta40"))
            sv.set_rank([s["rank"]] * len(s["dims"]))
            S = solver_mod
            start.wait()
            for _ in range(40):
                sv.set_factor(S.R, s["R"])
                sv.set_factor(S.D, s["D"])
                sv.set_vec(S.LAMBDA, s["lam"])
                sv.set_vec(S.CVS, s["cvs"])
                q1, p1, q2, p2 = sv.q12()
                assert rel_err(q1, g["q1"]) < 1e-10 and rel_err(q2, g["q2"]) < 1e-10
                tau, rn = sv.line_search(s["rho"])
                assert rn == int(g["rootnum"]), (rn, g["rootnum"])
                assert abs(tau - g["tau"]) <= TOL * max(1, abs(g["tau"])), (tau, g["tau"])
            sv.close()
        except BaseException as e:
            errors.append(("line_search", repr(e)))

    ts = [threading.Thread(target=ring_of_three), threading.Thread(target=line_search)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    assert not any(t.is_alive() for t in ts), "a thread did not finish"
    assert not errors, errors
