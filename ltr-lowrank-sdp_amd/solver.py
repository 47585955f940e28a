"""Host-side mirror of the reference's solver interface over the C-ABI
(include/lrsdp.h).

* :func:`run_lorads` mirrors benchmark.py's ``run_lorads`` (benchmark.py:219-285):
  same argv contract, runs the MI355X drop-in binary, returns
  ``(success, solve_time_sec, primal_obj)`` from the JSON metrics.
* :class:`Solver` exposes the per-operator entry points (the reference's
  ``lorads_func`` / cone / coefficient vtable slots, lorads_solver.c:1014-1053)
  for tests and benchmarking.

The product path is the HIP library; there is no CPU fallback: importing this
module on a machine without the built ``liblrsdp.so`` raises.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "_build" / "liblrsdp.so"
BIN_PATH = _HERE / "_build" / "LoRADS_v_2_0_1-alpha"

R, D, G, U, V, S0, Y0, S1, Y1 = range(9)
LAMBDA, CVS, Q1, Q2, B = range(5)


class Params(C.Structure):
    _fields_ = [
        ("initRho", C.c_double), ("rhoMax", C.c_double), ("rhoCellingALM", C.c_double),
        ("rhoCellingADMM", C.c_double), ("maxALMIter", C.c_int), ("maxADMMIter", C.c_int),
        ("timesLogRank", C.c_double), ("fixedRank", C.c_int), ("initRank", C.c_int), ("rhoFreq", C.c_int),
        ("rhoFactor", C.c_double), ("ALMRhoFactor", C.c_double), ("rankUpdateFactor", C.c_double),
        ("phase1Tol", C.c_double), ("phase2Tol", C.c_double), ("timeSecLimit", C.c_double),
        ("heuristicFactor", C.c_double), ("lbfgsListLength", C.c_int), ("endTauTol", C.c_double),
        ("endALMSubTol", C.c_double), ("l2Rescaling", C.c_int), ("reoptLevel", C.c_int),
        ("dyrankLevel", C.c_int), ("highAccMode", C.c_int), ("oracleRankNaive", C.c_int),
        ("disableOracle", C.c_int), ("nearStallFactor", C.c_double), ("rankSchedule", C.POINTER(C.c_int)),
        ("rankScheduleLen", C.c_int), ("verbose", C.c_int), ("almInnerBudget", C.c_long), ("skipADMM", C.c_int),
    ]


class Result(C.Structure):
    _fields_ = [
        ("alm_inner", C.c_long), ("alm_outer", C.c_long), ("admm_iter", C.c_long), ("cg_iter", C.c_long),
        ("alm_pobj", C.c_double), ("alm_dobj", C.c_double), ("alm_pinf", C.c_double), ("alm_gap", C.c_double),
        ("alm_rho", C.c_double), ("pobj", C.c_double), ("dobj", C.c_double), ("pinf", C.c_double),
        ("pinf_inf", C.c_double), ("gap", C.c_double), ("rho", C.c_double), ("solve_time", C.c_double),
        ("alm_time", C.c_double), ("admm_time", C.c_double), ("read_time", C.c_double), ("status", C.c_int),
        ("retcode", C.c_int), ("final_rank", C.c_int), ("oracle_rank", C.c_int), ("traj1_len", C.c_int),
        ("traj2_len", C.c_int), ("rho_max", C.c_double), ("dinf", C.c_double), ("dinf_inf", C.c_double),
        ("dinf_2", C.c_double), ("dinf_converged", C.c_int), ("dinf_iters", C.c_int), ("dinf_steps", C.c_long),
        ("dinf_time", C.c_double), ("obj_scale", C.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None
_HOOK = C.CFUNCTYPE(C.c_long, C.c_void_p, C.c_long)


def load_library(path=None):
    """Load liblrsdp.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise RuntimeError(f"HIP library not built: {p} (run __graft_entry__.build())")
    lib = C.CDLL(str(p))
    dp = C.POINTER(C.c_double)
    ip = C.POINTER(C.c_int)
    vp = C.c_void_p
    sig = {
        "lrs_params_default": (None, [C.POINTER(Params)]),
        "lrs_last_error": (C.c_char_p, []),
        "lrs_version": (C.c_char_p, []),
        "lrs_ctx_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "lrs_ctx_destroy": (None, [vp]),
        "lrs_load_sdpa": (C.c_int, [vp, C.c_char_p, dp]),
        "lrs_problem_info": (C.c_int, [vp, ip, ip, ip, C.POINTER(C.c_long), C.POINTER(C.c_long)]),
        "lrs_determine_rank": (C.c_int, [vp, C.POINTER(Params), ip]),
        "lrs_set_rank": (C.c_int, [vp, ip]),
        "lrs_get_rank": (C.c_int, [vp, ip]),
        "lrs_factor_set": (C.c_int, [vp, C.c_int, dp]),
        "lrs_factor_get": (C.c_int, [vp, C.c_int, dp]),
        "lrs_vec_set": (C.c_int, [vp, C.c_int, dp]),
        "lrs_vec_get": (C.c_int, [vp, C.c_int, dp]),
        "lrs_op_q12": (C.c_int, [vp, dp, dp, dp, dp]),
        "lrs_op_constr_rr": (C.c_int, [vp, dp, dp, dp]),
        "lrs_op_grad": (C.c_int, [vp, C.c_double, dp]),
        "lrs_op_line_search": (C.c_int, [vp, C.c_double, dp, ip]),
        "lrs_op_lbfgs": (C.c_int, [vp, C.c_int, C.c_double, C.c_double]),
        "lrs_op_admm_constr": (C.c_int, [vp]),
        "lrs_op_admm_half": (C.c_int, [vp, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int, ip, dp]),
        "lrs_op_dual_update": (C.c_int, [vp, C.c_double]),
        "lrs_op_gram": (C.c_int, [vp, C.c_int, C.c_int, dp]),
        "lrs_op_alm_update": (C.c_int, [vp, C.c_double, C.c_double, dp, dp]),
        "lrs_op_adjoint": (C.c_int, [vp, dp, C.c_int, dp, C.c_double, C.c_int]),
        "lrs_op_auv": (C.c_int, [vp, C.c_int, C.c_int, dp, dp]),
        "lrs_op_dimacs": (C.c_int, [vp, C.c_int, dp]),
        "lrs_abi_version": (C.c_int, []),
        "lrs_solve": (C.c_int, [vp, C.POINTER(Params), C.POINTER(Result)]),
        "lrs_trajectory": (C.c_int, [vp, C.c_int, ip, ip, C.c_int]),
        "lrs_write_json": (C.c_int, [vp, C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(Result),
                                     C.POINTER(Params)]),
        "lrs_alm_throughput": (C.c_int, [vp, C.POINTER(Params), C.c_long, C.c_long, dp, C.POINTER(C.c_long),
                                         dp, dp]),
        "lrs_set_log_path": (C.c_int, [vp, C.c_char_p]),
        "lrs_set_budget_hook": (C.c_int, [vp, _HOOK, vp]),
        "lrs_sync": (C.c_int, [vp]),
        "lrs_alm_last_step": (C.c_int, [vp, dp, ip]),
        "lrs_time_auut": (C.c_int, [vp, C.c_int, dp]),
        "lrs_profile_stages": (C.c_int, [vp, C.POINTER(Params), C.c_long, dp, C.POINTER(C.c_long)]),
        "lrs_time_stages": (C.c_int, [vp, C.c_int, dp]),
        "lrs_set_kernel_path": (C.c_int, [vp, C.c_int]),
        "lrs_op_dual_infeasibility": (C.c_int, [vp, dp, dp]),
        "lrs_get_kernel_path": (C.c_int, [vp, ip]),
        "lrs_stage_bytes": (C.c_int, [vp, dp]),
        "lrs_tile_info": (C.c_int, [vp, ip, ip]),
        "lrs_tile_used": (C.c_int, [vp, ip]),
        "lrs_auut_bytes": (C.c_int, [vp, dp]),
        "lrs_time_gram": (C.c_int, [vp, C.c_int, C.c_int, dp, dp]),
        "lrs_mfma_f64_peak": (C.c_int, [vp, dp]),
        "lrs_mfma_f64_probe": (C.c_int, [vp, C.c_int, C.c_int, dp, dp, dp]),
        "lrs_time_dense": (C.c_int, [vp, C.c_int, C.c_int, dp]),
        "lrs_load_coo": (C.c_int, [vp, C.c_int, C.c_int, ip, dp, C.c_long, ip, ip, ip, ip, dp]),
        "lrs_debug_phase_times": (C.c_int, [vp, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]),
        "lrs_comm_unique_id": (C.c_int, [C.c_char_p]),
        "lrs_shard_rccl": (C.c_int, [vp, C.c_int, C.c_int, C.c_char_p]),
        "lrs_loopback_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "lrs_loopback_destroy": (None, [vp]),
        "lrs_shard_loopback": (C.c_int, [vp, vp, C.c_int]),
        "lrs_shard_info": (C.c_int, [vp, ip, ip, ip, ip, ip]),
        "lrs_shard_comm_ranks": (C.c_int, [vp, ip]),
        "lrs_shard_comm_record": (C.c_int, [vp, C.c_int]),
        "lrs_xwg_fallbacks": (C.c_int, [vp, ip]),
        "lrs_shard_comm_log": (C.c_int, [vp, C.POINTER(C.c_long), C.c_long, C.POINTER(C.c_long)]),
        "lrs_shard_plan": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_long), ip, ip, ip, ip, ip, ip, ip]),
    }
    for name, (res, args) in sig.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if os.environ.get("LRS_LIB"):   # an older build compared side by side (scripts/*_probe.py)
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def default_params(**kw):
    lib = load_library()
    p = Params()
    lib.lrs_params_default(C.byref(p))
    sched = kw.pop("rankSchedule", None)
    for k, v in kw.items():
        if not hasattr(p, k):
            raise AttributeError(k)
        setattr(p, k, v)
    if sched:
        arr = (C.c_int * len(sched))(*sched)
        p.rankSchedule = arr
        p.rankScheduleLen = len(sched)
        p._sched_keepalive = arr
    return p


def _dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def comm_unique_id():
    """RCCL unique id (128 bytes) for lrs_shard_rccl; made on rank 0 and broadcast."""
    lib = load_library()
    buf = C.create_string_buffer(128)
    if lib.lrs_comm_unique_id(buf) != 0:
        raise RuntimeError(f"comm_unique_id: {lib.lrs_last_error().decode()}")
    return buf.raw


class LoopbackGroup:
    """One-process loopback transport of a sharded solve (tests): `world` Solvers on one
    GPU, each driven by its own thread, call Solver.shard_loopback(group, rank)."""

    def __init__(self, world):
        self.lib = load_library()
        self.h = C.c_void_p()
        if self.lib.lrs_loopback_create(world, C.byref(self.h)) != 0:
            raise RuntimeError(f"loopback_create: {self.lib.lrs_last_error().decode()}")
        self.world = world

    def close(self):
        if self.h:
            self.lib.lrs_loopback_destroy(self.h)
            self.h = C.c_void_p()


class Solver:
    """One device context with a loaded SDPA problem."""

    def __init__(self, path=None, device=0, coo=None):
        """path: SDPA .dat-s file; or coo: dict from instances.coo_arrays (lrs_load_coo)."""
        self.lib = load_library()
        self.ctx = C.c_void_p()
        self._check(self.lib.lrs_ctx_create(device, C.byref(self.ctx)), "ctx_create")
        t = C.c_double()
        if coo is not None:
            import time as _time
            t0 = _time.perf_counter()
            a = {k: coo[k] for k in ("dims", "b", "con", "blk", "row", "col", "val")}
            ip_ = lambda x: x.ctypes.data_as(C.POINTER(C.c_int))
            dp_ = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))
            self._check(self.lib.lrs_load_coo(self.ctx, int(coo["m"]), len(a["dims"]), ip_(a["dims"]), dp_(a["b"]),
                                              len(a["con"]), ip_(a["con"]), ip_(a["blk"]), ip_(a["row"]),
                                              ip_(a["col"]), dp_(a["val"])), "load_coo")
            t.value = _time.perf_counter() - t0
        else:
            self._check(self.lib.lrs_load_sdpa(self.ctx, str(path).encode(), C.byref(t)), "load_sdpa")
        self.read_time = t.value
        m, k = C.c_int(), C.c_int()
        self._check(self.lib.lrs_problem_info(self.ctx, C.byref(m), C.byref(k), None, None, None), "info")
        self.m, self.K = m.value, k.value
        dims = (C.c_int * self.K)()
        ns, nz = C.c_long(), C.c_long()
        self._check(self.lib.lrs_problem_info(self.ctx, None, None, dims, C.byref(ns), C.byref(nz)), "info")
        self.dims = list(dims)
        self.nslots, self.nnz = ns.value, nz.value
        self.ranks = None

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.lib.lrs_last_error().decode()}")

    def close(self):
        if self.ctx:
            self.lib.lrs_ctx_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- sharded solve (include/lrsdp.h lrs_shard_*): call after loading, before solving
    def shard_rccl(self, world, rank, uid):
        self._check(self.lib.lrs_shard_rccl(self.ctx, world, rank, uid), "shard_rccl")
        self._after_shard()

    def shard_loopback(self, group, rank):
        self._check(self.lib.lrs_shard_loopback(self.ctx, group.h, rank), "shard_loopback")
        self._after_shard()

    def _after_shard(self):
        """The shard's local sizes (every cone: owned + halo rows; the local constraints)."""
        m, k = C.c_int(), C.c_int()
        self._check(self.lib.lrs_problem_info(self.ctx, C.byref(m), C.byref(k), None, None, None), "info")
        dims = (C.c_int * max(1, k.value))()
        self._check(self.lib.lrs_problem_info(self.ctx, C.byref(m), C.byref(k), dims, None, None), "info")
        self.m, self.dims = m.value, list(dims)[:k.value]

    def shard_info(self):
        """(world, rank, first global row, owned rows, halo rows)."""
        v = [C.c_int() for _ in range(5)]
        self._check(self.lib.lrs_shard_info(self.ctx, *[C.byref(x) for x in v]), "shard_info")
        return tuple(x.value for x in v)

    def xwg_fallbacks(self):
        """Inner-loop calls rerun on the multi-launch iteration after a one-workgroup-per-cone
        exchange timed out (include/lrsdp.h lrs_xwg_fallbacks)."""
        n = C.c_int()
        self._check(self.lib.lrs_xwg_fallbacks(self.ctx, C.byref(n)), "xwg_fallbacks")
        return n.value

    def comm_record(self, on=True):
        """Start (clearing the log) or stop recording the transport's operations."""
        self._check(self.lib.lrs_shard_comm_record(self.ctx, 1 if on else 0), "comm_record")

    def comm_log(self):
        """The recorded operations: an (n, 5) int64 array {kind, peer, cone, count, offset}
        (include/lrsdp.h lrs_shard_comm_log)."""
        n = C.c_long()
        self._check(self.lib.lrs_shard_comm_log(self.ctx, None, 0, C.byref(n)), "comm_log")
        out = np.zeros(5 * max(1, n.value), dtype=np.int64)
        self._check(self.lib.lrs_shard_comm_log(self.ctx, out.ctypes.data_as(C.POINTER(C.c_long)), n.value,
                                                C.byref(n)), "comm_log")
        return out[:5 * n.value].reshape(-1, 5)

    def comm_ranks(self):
        """Ranks the shard transport counts itself (RCCL ncclCommCount; 1 unsharded)."""
        n = C.c_int()
        self._check(self.lib.lrs_shard_comm_ranks(self.ctx, C.byref(n)), "shard_comm_ranks")
        return n.value

    # ---- ranks / state
    def determine_rank(self, **kw):
        out = (C.c_int * self.K)()
        self._check(self.lib.lrs_determine_rank(self.ctx, C.byref(default_params(**kw)), out), "determine_rank")
        return list(out)

    def set_rank(self, ranks):
        ranks = list(ranks)
        self._check(self.lib.lrs_set_rank(self.ctx, (C.c_int * self.K)(*ranks)), "set_rank")
        self.ranks = ranks

    def nr(self):
        # the context's current ranks (a solve may have grown them since set_rank): every host
        # buffer handed to the library is sized from them
        self.ranks = self.get_rank()
        return sum(n * r for n, r in zip(self.dims, self.ranks))

    def set_factor(self, which, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        assert x.size == self.nr()
        self._check(self.lib.lrs_factor_set(self.ctx, which, _dptr(x)), "factor_set")

    def get_factor(self, which):
        x = np.empty(self.nr())
        self._check(self.lib.lrs_factor_get(self.ctx, which, _dptr(x)), "factor_get")
        return x

    def set_vec(self, which, v):
        v = np.ascontiguousarray(v, dtype=np.float64)
        assert v.size == self.m
        self._check(self.lib.lrs_vec_set(self.ctx, which, _dptr(v)), "vec_set")

    def get_vec(self, which):
        v = np.empty(self.m)
        self._check(self.lib.lrs_vec_get(self.ctx, which, _dptr(v)), "vec_get")
        return v

    # ---- operators
    def q12(self):
        q1, q2 = np.empty(self.m), np.empty(self.m)
        p1, p2 = C.c_double(), C.c_double()
        self._check(self.lib.lrs_op_q12(self.ctx, _dptr(q1), C.byref(p1), _dptr(q2), C.byref(p2)), "q12")
        return q1, p1.value, q2, p2.value

    def constr_rr(self):
        cvs = np.empty(self.m)
        pinf, pobj = C.c_double(), C.c_double()
        self._check(self.lib.lrs_op_constr_rr(self.ctx, _dptr(cvs), C.byref(pinf), C.byref(pobj)), "constr_rr")
        return cvs, pinf.value, pobj.value

    def grad(self, rho):
        lag = C.c_double()
        self._check(self.lib.lrs_op_grad(self.ctx, rho, C.byref(lag)), "grad")
        return self.get_factor(G), lag.value

    def line_search(self, rho):
        tau, rn = C.c_double(), C.c_int()
        self._check(self.lib.lrs_op_line_search(self.ctx, rho, C.byref(tau), C.byref(rn)), "line_search")
        return tau.value, rn.value

    def lbfgs(self, node_num, beta_new, beta_old):
        self._check(self.lib.lrs_op_lbfgs(self.ctx, node_num, beta_new, beta_old), "lbfgs")
        return self.get_factor(D)

    def admm_constr(self):
        """LORADSInitConstrValAll + Sum on (U, V): the state the ADMM half-steps read."""
        self._check(self.lib.lrs_op_admm_constr(self.ctx), "admm_constr")

    def admm_half(self, rho, cg_tol, cg_maxit=800, cone=0, side=0, init=True):
        """One half-step of LORADSUpdateSDPVar for `cone` (side 0: U with V fixed, 1: V with U
        fixed) and the cone's constraint refresh; init=True first recomputes the constraint
        values from (U, V).  Returns (the updated factor, all cones; the cone's RHS; CG its)."""
        if init:
            self.admm_constr()
        it = C.c_int()
        rhs = np.empty(self.dims[cone] * self.get_rank()[cone])
        self._check(self.lib.lrs_op_admm_half(self.ctx, cone, side, rho, cg_tol, cg_maxit, C.byref(it), _dptr(rhs)),
                    "admm_half")
        return self.get_factor(V if side else U), rhs, it.value

    def dual_update(self, rho):
        """LORADSUpdateDualVar: lambda += rho (b - A(X))."""
        self._check(self.lib.lrs_op_dual_update(self.ctx, rho), "dual_update")

    def alm_update(self, rho, tau):
        """setAsNegGrad + ALMupdateVar + constrValSum update + ALMCalGrad + setlbfgsHisTwo
        (lorads_alm.c:1340-1355): returns (||G||^2, beta of the new pair)."""
        lag, beta = C.c_double(), C.c_double()
        self._check(self.lib.lrs_op_alm_update(self.ctx, rho, tau, C.byref(lag), C.byref(beta)), "alm_update")
        return lag.value, beta.value

    def adjoint(self, y, which=R, scale=1.0, with_c=True):
        """scale (with_c C + sum_i y_i A_i) X_which (sdpDataWSum + mul_rk)."""
        y = np.ascontiguousarray(y, dtype=np.float64)
        assert y.size == self.m
        out = np.empty(self.nr())
        self._check(self.lib.lrs_op_adjoint(self.ctx, _dptr(y), which, _dptr(out), scale, 1 if with_c else 0),
                    "adjoint")
        return out

    def auv(self, u=R, v=R):
        """(A(sym(X_u X_v^T)), <C, sym(X_u X_v^T)>) -- coneAUV + objAUV; the state is unchanged."""
        out, cobj = np.empty(self.m), C.c_double()
        self._check(self.lib.lrs_op_auv(self.ctx, u, v, _dptr(out), C.byref(cobj)), "auv")
        return out, cobj.value

    def dimacs(self, admm=False):
        """updateDimacsALM / ADMM with the objectives: {pobj, dobj, pinf, pinf_inf, gap}."""
        o = np.empty(5)
        self._check(self.lib.lrs_op_dimacs(self.ctx, 1 if admm else 0, _dptr(o)), "dimacs")
        return dict(zip(("pobj", "dobj", "pinf", "pinf_inf", "gap"), o.tolist()))

    def gram(self, cone=0, which=R):
        r = self.get_rank()[cone]
        g = np.empty(r * r)
        self._check(self.lib.lrs_op_gram(self.ctx, cone, which, _dptr(g)), "gram")
        return g.reshape(r, r)

    # ---- solves
    def solve(self, **kw):
        p = default_params(**kw)
        res = Result()
        self._check(self.lib.lrs_solve(self.ctx, C.byref(p), C.byref(res)), "solve")
        return res.as_dict()

    def trajectory(self, phase):
        n = self.lib.lrs_trajectory(self.ctx, phase, None, None, 0)
        cur, orc = (C.c_int * max(n, 1))(), (C.c_int * max(n, 1))()
        self.lib.lrs_trajectory(self.ctx, phase, cur, orc, n)
        return list(cur)[:n], list(orc)[:n]

    def alm_throughput(self, warmup, steps, auut=False, **kw):
        p = default_params(**kw)
        sec, kms, ims = C.c_double(), C.c_double(), C.c_double()
        done = C.c_long()
        self._check(self.lib.lrs_alm_throughput(self.ctx, C.byref(p), warmup, steps, C.byref(sec), C.byref(done),
                                                C.byref(kms) if auut else None, C.byref(ims)), "alm_throughput")
        return {"seconds": sec.value, "done": done.value, "auut_ms": kms.value if auut else None,
                "iter_ms": ims.value}

    def alm_timed(self, warmup, steps, on_start=None, on_stop=None, **kw):
        """ONE phase-1 solve: `warmup` inner iterations, then exactly `steps` more of the same
        solve (lrs_set_budget_hook), with no solver setup between them.  on_start() runs when
        the warmup iterations are done and the stream is idle, on_stop() after the timed ones
        (the caller's barrier + clock); returns {"done": timed iterations, "seconds": host
        time between the two callbacks (the callbacks' own work excluded), "inner": total}."""
        import time as _time
        kw = dict(kw)
        p = default_params(**kw)
        p.phase1Tol = 1e-300
        p.maxALMIter = 1000000000
        p.skipADMM = 1
        p.timeSecLimit = 1e30
        p.almInnerBudget = max(1, int(warmup))
        st = {"t0": None, "t1": None, "i0": 0, "i1": 0}

        def hook(_user, inner):
            if st["t0"] is None:
                if on_start:
                    on_start()
                st["i0"] = inner
                st["t0"] = _time.perf_counter()
                return inner + int(steps)
            st["t1"] = _time.perf_counter()
            st["i1"] = inner
            if on_stop:
                on_stop()
            return 0

        cb = _HOOK(hook)
        self._check(self.lib.lrs_set_budget_hook(self.ctx, cb, None), "set_budget_hook")
        try:
            res = Result()
            self._check(self.lib.lrs_solve(self.ctx, C.byref(p), C.byref(res)), "solve")
        finally:
            self.lib.lrs_set_budget_hook(self.ctx, _HOOK(), None)
        if st["t0"] is None or st["t1"] is None:
            raise RuntimeError("alm_timed: the phase-1 budget was not reached")
        return {"done": st["i1"] - st["i0"], "seconds": st["t1"] - st["t0"], "inner": res.alm_inner}

    def alm_steps(self, K, **kw):
        """Exactly K ALM inner iterations of a fresh phase-1 solve (budget stop), then
        (tau, ||G||^2, pinf, beta) of trip K, the newest pair's index and the state."""
        kw = dict(kw)
        p = default_params(**kw)
        p.maxALMIter = 1000000000
        p.skipADMM = 1
        p.timeSecLimit = 1e30
        p.almInnerBudget = int(K)
        res = Result()
        self._check(self.lib.lrs_solve(self.ctx, C.byref(p), C.byref(res)), "solve")
        out = (C.c_double * 4)()
        nw = C.c_int()
        self._check(self.lib.lrs_alm_last_step(self.ctx, out, C.byref(nw)), "alm_last_step")
        self.ranks = self.get_rank()
        pair = (S0, Y0) if nw.value == 0 else (S1, Y1)
        return {"inner": res.alm_inner, "tau": out[0], "lag": out[1], "pinf": out[2], "beta": out[3],
                "R": self.get_factor(R), "G": self.get_factor(G), "cvs": self.get_vec(CVS),
                "lam": self.get_vec(LAMBDA), "s": self.get_factor(pair[0]), "y": self.get_factor(pair[1])}

    def get_rank(self):
        out = (C.c_int * self.K)()
        self._check(self.lib.lrs_get_rank(self.ctx, out), "get_rank")
        return list(out)

    def sync(self):
        self._check(self.lib.lrs_sync(self.ctx), "sync")

    def profile_stages(self, steps, **kw):
        """Average ms per launch of the four split-iteration stages (HIP events)."""
        p = default_params(**kw)
        ms = (C.c_double * 4)()
        done = C.c_long()
        self._check(self.lib.lrs_profile_stages(self.ctx, C.byref(p), steps, ms, C.byref(done)), "profile_stages")
        return list(ms), done.value

    def auut_bytes(self):
        """Algorithmic bytes of one A(UU^T) (constraint-entry kernel) launch."""
        v = C.c_double()
        self._check(self.lib.lrs_auut_bytes(self.ctx, C.byref(v)), "auut_bytes")
        return v.value

    def tile_info(self):
        """(constraint entries in 2-D tiles, lower pattern in 2-D tiles) for some cone."""
        a, b = C.c_int(), C.c_int()
        self._check(self.lib.lrs_tile_info(self.ctx, C.byref(a), C.byref(b)), "tile_info")
        return a.value, b.value

    def tile_used(self):
        """True when the last ALM iteration ran its stages over the 2-D tiles."""
        v = C.c_int()
        self._check(self.lib.lrs_tile_used(self.ctx, C.byref(v)), "tile_used")
        return bool(v.value)

    def stage_bytes(self):
        """Algorithmic bytes per launch of the stages [A, G, B] at the current ranks."""
        v = (C.c_double * 3)()
        self._check(self.lib.lrs_stage_bytes(self.ctx, v), "stage_bytes")
        return list(v)

    def set_kernel_path(self, path):
        """0 = automatic (latency-regime kernels where they apply), 1 = general row kernels."""
        self._check(self.lib.lrs_set_kernel_path(self.ctx, int(path)), "set_kernel_path")

    def dual_infeasibility(self):
        """(l1 dual infeasibility, [lambda_min(S_k)] per cone) of the current multipliers."""
        l1 = C.c_double()
        lm = np.zeros(max(1, len(self.dims)))
        self._check(self.lib.lrs_op_dual_infeasibility(self.ctx, C.byref(l1), _dptr(lm)), "dual_infeasibility")
        return l1.value, lm[:len(self.dims)]

    def kernel_path(self):
        """Path of the last enqueued ALM iteration: 0 latency-regime kernels, 1 general, -1 none."""
        v = C.c_int(-1)
        self._check(self.lib.lrs_get_kernel_path(self.ctx, C.byref(v)), "get_kernel_path")
        return v.value

    def time_stages(self, reps=200):
        """Per-launch ms of the split-iteration stages [A, G, B] (back-to-back relaunches)."""
        ms = (C.c_double * 3)()
        self._check(self.lib.lrs_time_stages(self.ctx, reps, ms), "time_stages")
        return list(ms)

    def debug_phase_times(self):
        """In-kernel timestamps (diagnostics library only): ([4][16] block-0 phase ticks,
        [4][1024][2] per-block entry/exit ticks) or None from the product library."""
        out = (C.c_ulonglong * 64)()
        blk = (C.c_ulonglong * (4 * 1024 * 2))()
        rc = self.lib.lrs_debug_phase_times(self.ctx, out, blk)
        if rc < 0:
            raise RuntimeError(self.lib.lrs_last_error().decode())
        if rc != 64:
            return None
        ph = [list(out[16 * k:16 * k + 16]) for k in range(4)]
        b = [[(blk[(k * 1024 + i) * 2], blk[(k * 1024 + i) * 2 + 1]) for i in range(1024)] for k in range(4)]
        return ph, b

    def time_gram(self, cone=0, reps=20):
        """(ms per Gram incl. reduction, ms of the MFMA kernel alone) on R of `cone`."""
        ms, kms = C.c_double(), C.c_double()
        self._check(self.lib.lrs_time_gram(self.ctx, cone, reps, C.byref(ms), C.byref(kms)), "time_gram")
        return ms.value, kms.value

    def time_dense(self, cone=0, reps=10):
        """ms per dense-objective product C R of `cone` on the matrix cores (lrs_time_dense)."""
        t = C.c_double()
        self._check(self.lib.lrs_time_dense(self.ctx, cone, reps, C.byref(t)), "time_dense")
        return t.value

    def mfma_f64_peak(self):
        """Measured FP64 matrix-core TFLOP/s of this device (lrs_mfma_f64_peak)."""
        t = C.c_double()
        self._check(self.lib.lrs_mfma_f64_peak(self.ctx, C.byref(t)), "mfma_f64_peak")
        return t.value

    def mfma_f64_probe(self, waves_per_simd=4, chains=8):
        """(TFLOP/s, shader MHz under the load, cycles per MFMA per SIMD) of the FP64 matrix-core
        probe at the given occupancy (lrs_mfma_f64_probe)."""
        t, f, cy = C.c_double(), C.c_double(), C.c_double()
        self._check(self.lib.lrs_mfma_f64_probe(self.ctx, int(waves_per_simd), int(chains), C.byref(t), C.byref(f),
                                                C.byref(cy)), "mfma_f64_probe")
        return t.value, f.value, cy.value

    def time_auut(self, reps=100):
        ms = C.c_double()
        self._check(self.lib.lrs_time_auut(self.ctx, reps, C.byref(ms)), "time_auut")
        return ms.value


def shard_plan(path, world, rank):
    """Host-only row partition of a sharded solve (lrs_shard_plan; no device needed)."""
    lib = load_library()
    cnt = (C.c_long * 8)()
    nul = C.POINTER(C.c_int)()
    rc = lib.lrs_shard_plan(str(path).encode(), world, rank, cnt, nul, nul, nul, nul, nul, nul, nul)
    if rc != 0:
        raise RuntimeError(lib.lrs_last_error().decode())
    n, r0, nown, nl, ns, nsh, ml, w = list(cnt)
    arr = {k: np.zeros(max(1, v), dtype=np.int32) for k, v in
           (("bounds", world + 1), ("local_gid", nl), ("send_ptr", world + 1), ("send_gid", ns),
            ("shared_gid", nsh), ("con_gid", ml), ("primary", ml))}
    ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
    rc = lib.lrs_shard_plan(str(path).encode(), world, rank, cnt, ip(arr["bounds"]), ip(arr["local_gid"]),
                            ip(arr["send_ptr"]), ip(arr["send_gid"]), ip(arr["shared_gid"]), ip(arr["con_gid"]),
                            ip(arr["primary"]))
    if rc != 0:
        raise RuntimeError(lib.lrs_last_error().decode())
    out = {k: v[:n_] for (k, v), n_ in zip(arr.items(), (world + 1, nl, world + 1, ns, nsh, ml, ml))}
    out.update(n=n, row0=r0, nown=nown)
    return out


def run_lorads(instance_path, json_output_path, params, fixed_rank=None, rank_schedule_path=None,
               near_stall_factor=0.7, timeout=3600, device=0):
    """Same contract as benchmark.py:219-285, on the MI355X binary."""
    if not BIN_PATH.exists():
        raise RuntimeError(f"binary not built: {BIN_PATH}")
    json_output_path = Path(json_output_path)
    json_output_path.parent.mkdir(parents=True, exist_ok=True)
    cmd = [str(BIN_PATH), str(instance_path)]
    for k, v in params.items():
        cmd += [f"--{k}", str(v)]
    cmd += ["--jsonfile", str(json_output_path), "--disableOracle", "--device", str(device)]
    if fixed_rank is not None and rank_schedule_path is not None:
        raise ValueError("fixed_rank and rank_schedule_path are mutually exclusive")
    if rank_schedule_path is not None:
        cmd += ["--rankSchedule", str(rank_schedule_path), "--nearStallFactor", str(near_stall_factor)]
    elif fixed_rank is not None:
        cmd += ["--fixedRank", str(fixed_rank)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0:
            print(f"  [error] lorads failed: {r.stderr[:200]}")
            return False, None, None
        if not json_output_path.exists():
            return False, None, None
        with open(json_output_path) as f:
            out = json.load(f)
        # same key fallbacks as benchmark.py:270-274
        m = out.get("final_metrics", out.get("metrics", {}))
        return True, m.get("solve_time_sec"), m.get("primal_obj", m.get("primal_objective"))
    except subprocess.TimeoutExpired:
        print("  [error] lorads timed out")
        return False, None, None
    except Exception as e:   # benchmark.py:283-285
        print(f"  [error] unexpected error: {e}")
        return False, None, None
