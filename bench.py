#!/usr/bin/env python3
"""ALM iterations/s of the MI355X low-rank SDP solver on MaxCut G67 (BASELINE.json).

Workload: G67-structured MaxCut (2-D toroidal grid 100 x 100, weights +-1, n = m =
10 000; the real Gset file is not in the reference checkout),
default LoRADS rank r = ceil(2 ln n) = 19 held fixed so every step costs the same.
A "step" is one ALM inner iteration (alm_state.innerIter, lorads_alm.c:1372) of the
real phase-1 control flow (dual/rho updates and oracle-rank records included) on
the device.  Multi-GPU (the north star's constraint sharding): one process
per GPU, ONE G67 instance row-sharded over the N ranks through RCCL (lrs_shard_rccl: halo
exchange of the direction rows + all-reduced stage totals per inner iteration) -- strong
scaling of a single instance; barrier + max-over-ranks timing.  The instance-level replicas
(each rank its own instance, dataset/run_lorads.sh:85-114, weak scaling, no data-path
collective) are reported beside it under `replicas`.

Prints one JSON line (rank 0).  Besides the contract keys:
  roofline          dominant split-iteration stage on the workload (HIP-event timed,
                    algorithmic bytes from lrs_stage_bytes; DESIGN.md "Kernels")
  roofline_at_scale the same stages on a 2000 x 2000 torus (n = 4e6, r = 16: factors
                    far beyond the 256 MB Infinity Cache), where HBM bandwidth binds
  north_star        MaxCut n = 20 000, r = 64 (G81-like): device vs reference CPU it/s
  wall_clock_to_eps full ALM + ADMM solve to eps = 1e-5 with the Gset flags
  configs_wall_clock_to_eps  G1, G22, theta3 (and a 3-block theta3) solved to eps, device vs
                    the reference, with benchmark.py's flags per subtype
  cpu_baseline      the reference LoRADS C (oracle/_ref, built from /root/reference)
                    timed on this host, 1 core, on a bounded sample of the workload
  config_c5         BASELINE config C5 (random sparse SDP n = 1e4, m = 1e6, r = 128): ALM it/s
                    and the r x r Gram on the FP64 matrix cores (TFLOP/s vs the MFMA peak)
  sharded           ONE G81-like instance (n = 20 000, r = 64) row-sharded over all N ranks;
                    at N > 1 also C5 (n = 1e4, m = 1e6, r = 128) and the 2000^2 torus
                    (RCCL: halo exchange of direction rows + all-reduced stage totals per
                    inner iteration): strong-scaling it/s of the single instance
"""
import argparse
import importlib
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "ltr-lowrank-sdp_amd"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_MFMA_PEAK_TFS = 78.6   # MI355X FP64 matrix peak (AMD spec)
FP64_VALU_PEAK_TFS = 78.6   # FP64 vector FMA: 256 CUs x 64 FMA/clk x 2 flop x 2.4 GHz
LDS_PEAK_GBS = 256 * 256 * 2.4   # 256 B/clk/CU for ds_read_b64/b128 (MI355X_MICROARCH.md §LDS), 2.4 GHz
STAGES = ("A: {a} (control, L-BFGS direction, SDDMM sym(RD^T)/DD^T, local q1/q2)",
          "G: k_it_g (phase-1 test, multi-slot constraints' q1/q2)",
          "B: {b} (line search, R+tau D, adjoint S=C+A*(M1), G=2SR, A(RR^T), L-BFGS pair)")
# kernels per path (lrs_get_kernel_path): 0 latency-regime kernels, 1 general row kernels
STAGE_KERNELS = {0: ("k_lat_a", "k_lat_b"), 1: ("k_it_a", "k_it_b")}


def leg_profile(leg):
    """The newest committed rocprofv3 leg summary of `leg` (profiles/<tag>_<leg>_pmc.json, written by
    scripts/leg_profile.sh -> scripts/leg_summary.py): per stage of the split iteration and for
    A(UU^T), the summed kernel time over the FULL launches of lrs_time_stages / lrs_time_auut
    relaunch loops and the HBM-side bytes per launch (separate FETCH_SIZE / WRITE_SIZE passes,
    FETCH doubled per MI355X_MICROARCH.md "HBM").  None if absent."""
    import glob
    # newest round tag last (r05 < r06a < r06b ...): file names, not mtimes, which a checkout resets
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{leg}_pmc.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if "_stages" in d:
            d["_source"] = os.path.relpath(f, ROOT).replace("_pmc.json", "_summary.md")
            return d
    return None


def attach_traffic(res, leg):
    """roofline.traffic (and per-stage / A(UU^T) traffic) from the leg's committed rocprof summary;
    the summary's per-stage rocprof kernel time sits beside the bench's HIP-event time so the two
    can be compared (the probe's relaunch loops are the same lrs_time_stages calls)."""
    prof = leg_profile(leg)
    if prof is None:
        return res
    st = prof["_stages"]
    # the kernels the profile saw per stage (which row kernel family ran: e.g. k_bw_b for the
    # bandwidth regime's fused stage B on plain rows, k_it_b on team rows)
    ran = {}
    for name, v in prof.items():
        if not name.startswith("_") and isinstance(v, dict) and "stage" in v:
            short = name.split("::")[-1].split("<")[0]
            if short not in ran.setdefault(v["stage"], []):
                ran[v["stage"]].append(short)
    for o in res["stages"]:
        s = st.get(o["stage"][0])
        if s:
            o["traffic"] = s["traffic_bytes"]
            o["rocprof_us"] = s["rocprof_us"]
            o["rocprof_frac"] = s["frac_rocprof"]
        ks = ran.get(o["stage"][0])
        if ks:
            label = " + ".join(ks)
            old_stage = o["stage"]
            o["stage"] = old_stage.replace(o["kernel"], label, 1)
            if res["kernel"] == old_stage:
                res["kernel"] = o["stage"]
            o["kernel"] = label
    if "auut" in st:
        res["a_uut"]["traffic"] = st["auut"]["traffic_bytes"]
        res["a_uut"]["rocprof_us"] = st["auut"]["rocprof_us"]
        res["a_uut"]["rocprof_frac"] = st["auut"]["frac_rocprof"]
    dom = st.get(res["kernel"][0])
    if dom:
        res["traffic"] = dom["traffic_bytes"]
        res["rocprof_us"] = dom["rocprof_us"]
        res["rocprof_frac"] = dom["frac_rocprof"]
    res["traffic_source"] = (f"{prof['_source']}: per launch, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE summed over the "
                             "stage's kernels, full relaunches only (scripts/leg_profile.sh)")
    return res


def instance_for(rank_id, rows, cols, cache, seed0=67):
    inst = importlib.import_module(PKG + ".instances")
    path = os.path.join(cache, f"torus{rows}x{cols}_s{seed0 + rank_id}.dat-s")
    if not os.path.exists(path):
        tmp = path + f".tmp{os.getpid()}"
        inst.maxcut_torus(tmp, rows, cols, seed=seed0 + rank_id)
        os.replace(tmp, path)
    return path


def host_cpu():
    """(threads this process may use, CPU model) of the host running the bench."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return n, model


def cpu_reference_rate(path, rank, seconds, threads=1):
    """Reference LoRADS (oracle/_ref, built from /root/reference sources) phase-1
    rate on the host (its BLAS on `threads` threads); falls back to the CPU restatement if
    the reference build is absent."""
    harness = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")
    env = dict(os.environ, OPENBLAS_NUM_THREADS=str(threads), OMP_NUM_THREADS=str(threads))
    if os.path.exists(harness):
        r = subprocess.run([harness, "alm_rate", path, str(rank), "0", str(seconds)], capture_output=True,
                           text=True, env=env, timeout=seconds * 6 + 120)
        m = re.search(r"REF_RATE inner=(\d+) seconds=(\S+)", r.stdout)
        if m:
            return int(m.group(1)), float(m.group(2)), "reference"
    orc = os.path.join(ROOT, "oracle", "_build", "lrsdp_oracle")
    if not os.path.exists(orc):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    r = subprocess.run([orc, "alm_rate", path, str(rank), str(seconds)], capture_output=True, text=True,
                       timeout=seconds * 6 + 120)
    m = re.search(r"ORACLE_RATE inner=(\d+) seconds=(\S+)", r.stdout)
    return int(m.group(1)), float(m.group(2)), "port"


def cpu_reference_solve(path, flags, timeout):
    harness = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")
    if not os.path.exists(harness):
        return None
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1")
    t0 = time.perf_counter()
    r = subprocess.run([harness, "solve", path] + flags, capture_output=True, text=True, env=env, timeout=timeout)
    wall = time.perf_counter() - t0
    m = re.search(r"solve_time=(\S+)", r.stdout)
    p = re.search(r"alm_pobj=(\S+)", r.stdout)
    if not m:
        return None
    return {"solve_time_sec": float(m.group(1)), "process_wall_sec": wall, "alm_pobj": float(p.group(1))}


def mfma_probe(sv):
    """The FP64 matrix-core ceiling actually reachable with v_mfma_f64_16x16x4f64 (8 waves a SIMD,
    8 independent chains: the best of the occupancy sweep, profiles/r03j_mfma_probe.md), with the
    shader clock under that load and the cycles per MFMA per SIMD -- the 78.6 TF spec implies 64
    at 2.4 GHz; the probe measures ~100, so the spec is not reachable by this instruction."""
    tf, mhz, cyc = sv.mfma_f64_probe(8, 8)
    return tf, {"tflops": tf, "shader_mhz_under_load": mhz, "cycles_per_mfma_per_simd": cyc,
                "waves_per_simd": 8, "chains": 8, "spec_cycles_per_mfma": 64}


def tile_bounds(us, lds_bytes, flop):
    """The LDS-read and FP64-FMA side of a tile kernel whose operands are LDS-resident (the
    HBM fraction alone does not say how far off its real bound it is): algorithmic LDS bytes
    and flops per launch against the chip's LDS read rate and FP64 vector peak."""
    s = us * 1e-6
    return {"lds_bytes": lds_bytes, "lds_GBs": lds_bytes / s / 1e9, "lds_peak_GBs": LDS_PEAK_GBS,
            "lds_frac": lds_bytes / s / 1e9 / LDS_PEAK_GBS, "fp64_flop": flop,
            "fp64_TFs": flop / s / 1e12, "fp64_frac": flop / s / 1e12 / FP64_VALU_PEAK_TFS}


def stage_roofline(sv, reps, leg=None, rank=None):
    """Per-launch ms of the split-iteration stages (back-to-back relaunches between two
    HIP events on the solver stream) and their algorithmic bytes -> GB/s.  With `rank` and
    the 2-D tile kernels active, also each tile stage's LDS-read and FP64 fractions
    (tile_bounds): per lower slot stage A reads R_i, D_i, R_j, D_j (4 r doubles, 3 r FMA),
    stage B A(R R^T) on it (2 r doubles, r FMA) and S R over both its adjacency entries
    (r doubles, r FMA each); A(U U^T) per constraint entry 2 r doubles, r FMA."""
    ms = sv.time_stages(reps)
    by = sv.stage_bytes()
    ka, kb = STAGE_KERNELS.get(sv.kernel_path(), STAGE_KERNELS[1])
    n0 = sv.dims[0]
    # long-row cones over 2-D LDS tiles (the upload's rule in lrs_problem.cpp)
    ntl = (n0 + 127) // 128
    per_tile = 768 * ntl * (ntl + 1) / 2
    slot_tiles = len(sv.dims) == 1 and n0 >= 2048 and sv.nslots >= per_tile and sv.kernel_path() == 1
    auv_tiles = len(sv.dims) == 1 and n0 >= 2048 and sv.nnz >= per_tile
    if slot_tiles:
        ka, kb = "k_it_a + k_tile_a", "k_it_b + k_tile_b1 + k_tile_b2 + k_wide_bf"
    out = []
    for k in range(3):
        if ms[k] <= 0:
            continue
        gbs = by[k] / (ms[k] * 1e-3) / 1e9
        out.append({"stage": STAGES[k].format(a=ka, b=kb), "kernel": (ka, "k_it_g", kb)[k],
                    "avg_launch_us": ms[k] * 1e3, "bytes_per_launch": by[k], "achieved_GBs": gbs,
                    "frac": gbs / HBM_PEAK_GBS})
    if rank and slot_tiles:
        P, n = sv.nslots, n0
        adj = 2 * P - n
        for o in out:
            if o["stage"].startswith("A"):
                o["tile_bounds"] = tile_bounds(o["avg_launch_us"], P * 4 * rank * 8, P * 3 * rank * 2)
            elif o["stage"].startswith("B"):
                o["tile_bounds"] = tile_bounds(o["avg_launch_us"], (P * 2 + adj) * rank * 8, (P + adj) * rank * 2)
    dom = max(out, key=lambda s: s["avg_launch_us"])
    # the north-star's named operator: A(UU^T) straight from the constraint entries
    ams = sv.time_auut(reps)
    aby = sv.auut_bytes()
    agbs = aby / (ams * 1e-3) / 1e9
    diag = len(sv.dims) == 1 and sv.m == n0 and sv.nnz == n0   # MaxCut's diag(X) = 1: k_auv_diag
    akern = ("k_auv_tile<1> + k_auv_tsum (A(UU^T) over 2-D LDS tiles of constraint entries)" if auv_tiles
             else "k_auv_diag<XX^T> (A(UU^T) of identity-diagonal constraints: row-wise dots)" if diag
             else "k_auv_con<XX^T> (A(UU^T) over constraint entries)")
    auut = {"kernel": akern, "avg_launch_us": ams * 1e3,
            "bytes_per_launch": aby, "achieved_GBs": agbs, "frac": agbs / HBM_PEAK_GBS}
    if rank and auv_tiles:
        auut["tile_bounds"] = tile_bounds(ams * 1e3, sv.nnz * 2 * rank * 8, sv.nnz * rank * 2)
    res = {"bound": "hbm", "kernel": dom["stage"], "achieved": dom["achieved_GBs"], "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": dom["frac"], "traffic": None, "bytes_per_launch": dom["bytes_per_launch"],
           "avg_launch_us": dom["avg_launch_us"], "stages": out, "a_uut": auut}
    return attach_traffic(res, leg) if leg else res


def config_c5(solver, local, iters=20, cpu_seconds=0.0, cache=None):
    """BASELINE config C5 in memory: ALM it/s at r = 128, stage roofline, MFMA Gram; with
    cpu_seconds > 0 also the reference CPU rate on a C5-structured sample (m = 1e5)."""
    inst = importlib.import_module(PKG + ".instances")
    t0 = time.perf_counter()
    sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(10000, 1000000, 6, 5)), device=local)
    load_s = time.perf_counter() - t0
    kw = dict(fixedRank=128, reoptLevel=0)
    # one solve: warmup trips, then `iters` timed trips of the same solve (no setup inside)
    o = sv.alm_timed(3, iters, **kw)
    rl = stage_roofline(sv, 10, leg="c5", rank=128)
    ms, kms = sv.time_gram(0, 20)
    ceil_tf, probe = mfma_probe(sv)
    n = sv.dims[0]
    fl = n * 128 * 129   # the symmetric product (dsyrk count)
    sv.close()
    return {"workload": "random sparse SDP n=1e4, m=1e6, 6 entries/constraint, C=I, --fixedRank 128 (in memory)",
            "gpu_it_s": o["done"] / o["seconds"], "load_sec": load_s, "roofline": rl,
            "gram_mfma": {"kernel": "k_gram<2,4> (register-blocked v_mfma_f64_16x16x4_f64), R^T R, n=1e4, r=128",
                          "bound": "mfma", "avg_launch_us": kms * 1e3, "with_reduction_us": ms * 1e3,
                          "flop_per_launch": fl, "achieved": fl / (kms * 1e-3) / 1e12, "peak": FP64_MFMA_PEAK_TFS,
                          "unit": "TFLOP/s", "frac": fl / (kms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFS,
                          "frac_with_reduction": fl / (ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFS,
                          "measured_mfma_f64_tflops": ceil_tf, "mfma_probe": probe,
                          "frac_of_measured": fl / (kms * 1e-3) / 1e12 / ceil_tf},
            "cpu_baseline": c5_cpu_sample(solver, local, cpu_seconds, cache) if cpu_seconds > 0 else
            "not run (--no-cpu)"}


def config_c5b(solver, local, iters=30, ref_densec=None):
    """BASELINE config C5b in memory: C5 with C a dense random symmetric matrix (N(0, 1/n) + n I),
    the dense-objective path (C as a full matrix on the FP64 matrix cores):
    ALM it/s at r = 128, per-stage times, and the C R product against the MFMA roofline
    (2 n^2 r flop per launch).  The reference's rate on the same structure at test size
    (tests/golden/solves_densec.json: its own wall clock over its inner iterations) is quoted
    beside it, labelled as such: a full-size reference run (n = 10^4, 5*10^7 objective entries
    through its dense syr2k path) is not a bounded sample."""
    inst = importlib.import_module(PKG + ".instances")
    t0 = time.perf_counter()
    sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(10000, 1000000, 6, 5, dense_c=True)),
                       device=local)
    load_s = time.perf_counter() - t0
    kw = dict(fixedRank=128, reoptLevel=0)
    o = sv.alm_timed(3, iters, **kw)
    st = sv.time_stages(3)
    dm = sv.time_dense(0, 10)
    ceil_tf, probe = mfma_probe(sv)
    sv.close()
    n, r = 10000, 128
    fl = 2.0 * n * n * r
    out = {"workload": "random sparse SDP n=1e4, m=1e6, 6 entries/constraint, dense C (N(0,1/n) + n I), "
                       "--fixedRank 128 (in memory), dense-objective path",
           "gpu_it_s": o["done"] / o["seconds"], "load_sec": load_s,
           "stage_us": [round(x * 1e3, 1) for x in st],
           "dense_cr": {"kernel": "k_cgemm (v_mfma_f64_16x16x4_f64), C R, n=1e4, r=128", "bound": "mfma",
                        "avg_launch_us": dm * 1e3, "flop_per_launch": fl, "achieved": fl / (dm * 1e-3) / 1e12,
                        "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": fl / (dm * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFS,
                        "measured_mfma_f64_tflops": ceil_tf, "mfma_probe": probe,
                        "frac_of_measured": fl / (dm * 1e-3) / 1e12 / ceil_tf}}
    if ref_densec:
        out["reference_test_size"] = ref_densec
    return out


def ref_densec_rates():
    """The reference's inner-iteration rate on the dense-objective fixtures (its own solves,
    tests/golden/solves_densec.json; wall clock includes presolve and ADMM, so a lower bound)."""
    path = os.path.join(ROOT, "tests", "golden", "solves_densec.json")
    if not os.path.exists(path):
        return None
    rows = []
    for g in json.load(open(path)):
        rows.append({"instance": g["instance"], "n": g["n"], "m": g["m"], "flags": g["flags"],
                     "alm_inner": g["result"].get("alm_inner"), "wall_sec": g["wall_sec"],
                     "it_s_lower_bound": g["result"].get("alm_inner", 0) / g["wall_sec"], "cores": 1})
    return rows


def c5_cpu_sample(solver, local, seconds, cache):
    """The reference's rate on the C5 structure with m = 1e5 (a bounded sample: at m = 1e6 its
    hash-chain presolve alone takes ~1600 s; its iteration cost is the dense
    n^2 path it takes at > 10 % pattern fill, independent of m), the device's rate on the same
    file beside it."""
    inst = importlib.import_module(PKG + ".instances")
    path = os.path.join(cache, "c5_m1e5.dat-s")
    if not os.path.exists(path):
        tmp = path + f".tmp{os.getpid()}"
        inst.random_sparse(tmp, 10000, 100000, 6, 5)
        os.replace(tmp, path)
    it, sec, kind = cpu_reference_rate(path, 128, seconds)
    sv = solver.Solver(path, device=local)
    kw = dict(fixedRank=128, reoptLevel=0)
    o = sv.alm_timed(3, 20, **kw)
    sv.close()
    gpu = o["done"] / o["seconds"]
    return {"value": it / sec, "unit": "ALM inner iterations/s", "cores": 1, "kind": kind,
            "sample": f"C5 structure with m = 1e5 (n = 1e4, 6 entries/constraint, --fixedRank 128): {it} inner "
                      f"iterations in {sec:.1f} s wall, presolve excluded (OPENBLAS_NUM_THREADS=1)",
            "gpu_it_s_same_file": gpu, "speedup_same_file": gpu / (it / sec) if it else None}


def sharded_strong(solver, dist, world, rank_id, local, cache, replicas, steps=500, all_legs=False):
    """ONE instance row-sharded over the `world` ranks through RCCL (lrs_shard_rccl): whole-
    instance ALM it/s, strong scaling.  The G81-like torus (n = 20 000, r = 64) always; at
    world > 1 also BASELINE config C5 (n = 10^4, m = 10^6, r = 128, the 2-D tile kernels on each
    shard's owned rows, every row in every halo) and the 2000 x 2000 torus (n = 4*10^6, r = 16),
    whose one-GPU rates are config_c5.gpu_it_s and roofline_at_scale.it_s of the N = 1 line."""
    inst = importlib.import_module(PKG + ".instances")
    legs = [("g81", 50, steps)]
    if world > 1 or all_legs:
        legs += [("c5", 3, 20), ("torus2000", 5, 40)]
    out = {}
    for name, warm, k in legs:
        t0 = time.perf_counter()
        if name == "g81":
            sv = solver.Solver(instance_for(0, 100, 200, cache, seed0=81), device=local)
            kw = dict(fixedRank=64, reoptLevel=0)
            wl = "MaxCut torus 100x200 (G81 structure), n=m=20000, --fixedRank 64"
        elif name == "c5":
            sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(10000, 1000000, 6, 5)), device=local)
            kw = dict(fixedRank=128, reoptLevel=0)
            wl = "random sparse SDP n=1e4, m=1e6, 6 entries/constraint, C=I, --fixedRank 128 (BASELINE C5)"
        else:
            sv = solver.Solver(coo=inst.coo_arrays(inst.maxcut_torus_problem(2000, 2000, 2000)), device=local)
            kw = dict(fixedRank=16, reoptLevel=0)
            wl = "MaxCut torus 2000x2000, n=m=4e6, --fixedRank 16"
        # a fresh RCCL id per communicator (an id's bootstrap root ends with its communicator)
        uid = solver.comm_unique_id() if rank_id == 0 else None
        if dist is not None:
            box = [uid]
            dist.broadcast_object_list(box, src=0)
            uid = box[0]
        sv.shard_rccl(world, rank_id, uid)
        info = sv.shard_info()
        comm_ranks = sv.comm_ranks()
        if world > 1 and comm_ranks != world:
            raise RuntimeError(f"RCCL communicator counts {comm_ranks} ranks, expected {world}")
        tiles = sv.tile_info()
        load_s = time.perf_counter() - t0
        clock = {}

        def on_start():
            sv.sync()
            replicas.barrier_sync(dist)
            clock["t0"] = time.perf_counter()

        def on_stop():
            sv.sync()
            replicas.barrier_sync(dist)
            clock["t1"] = time.perf_counter()

        o = sv.alm_timed(warm, k, on_start, on_stop, **kw)
        used = sv.tile_used()
        sv.close()
        _, t_max = replicas.aggregate(dist, o["done"], clock["t1"] - clock["t0"])
        out[name] = {"workload": f"{wl}, ONE instance row-sharded over {world} GPU(s)", "it_s": o["done"] / t_max,
                     "steps": o["done"], "n_gpus": world, "scaling": "strong", "load_sec": load_s,
                     "comm_ranks": comm_ranks, "rank0_rows": info[3], "rank0_halo_rows": info[4], "slot_tiles_built": bool(tiles[1]),
                     "tile_kernels_ran": used}
    res = dict(out["g81"])
    res["transport"] = "RCCL (ncclSend/Recv halo, ncclAllReduce totals)"
    for name in ("c5", "torus2000"):
        if name in out:
            res[name] = out[name]
    return res


def build_provenance():
    """sha256 (first 16 hex) of the HIP library this run loads and of the sources it is built
    from, and the library's mtime: whether the box ran the build of these sources is checkable
    against the committed tree (`make -C ltr-lowrank-sdp_amd/csrc` rebuilds it)."""
    import hashlib
    csrc = os.path.join(ROOT, PKG, "csrc")
    lib = os.path.join(ROOT, PKG, "_build", "liblrsdp.so")
    h = hashlib.sha256()
    names = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".cpp", ".h")) or f == "Makefile")
    for f in names + ["../../include/lrsdp.h"]:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    out = {"sources_sha256_16": h.hexdigest()[:16], "sources": names + ["include/lrsdp.h"]}
    if os.path.exists(lib):
        with open(lib, "rb") as fh:
            out["liblrsdp_sha256_16"] = hashlib.sha256(fh.read()).hexdigest()[:16]
        out["liblrsdp_mtime"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(os.path.getmtime(lib)))
    return out


def spawn_ranks(n, argv):
    """`bench.py --gpus N` with no external launcher (WORLD_SIZE unset): start N fresh worker
    processes of this script, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in
    their environment -- the same environment torch.distributed.run gives them -- before this
    parent touches the GPU (it never does).  Rank 0's stdout is forwarded line by line and its
    JSON line checked for n_gpus == N; if a rank fails, the others are ended (their PIDs) and
    the exit status is the first failure's."""
    import socket
    import threading
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))
    lines = []

    def pump():
        for ln in procs[0].stdout:
            lines.append(ln)
            sys.stdout.write(ln)
            sys.stdout.flush()
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    rc = 0
    live = set(range(n))
    # an overall deadline: ranks stalled before the sharded leg's own watchdog starts (e.g. in
    # init_process_group) end the launcher with a non-zero status instead of hanging it
    deadline = time.time() + float(os.environ.get("LRS_BENCH_DEADLINE_S", "1500"))
    while live:
        if time.time() > deadline:
            print(f"bench.py launcher: ranks {sorted(live)} still running past the deadline; ending them",
                  file=sys.stderr)
            for q in live:
                procs[q].terminate()
            for q in live:
                try:
                    procs[q].wait(timeout=20)
                except subprocess.TimeoutExpired:
                    procs[q].kill()
            rc = rc or 124
            break
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench.py launcher: rank {r} exited with {c}; ending the other ranks", file=sys.stderr)
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    th.join(timeout=10)
    js = [ln for ln in lines if ln.lstrip().startswith("{")]
    if rc == 0:
        if not js:
            print("bench.py launcher: rank 0 printed no result line", file=sys.stderr)
            return 5
        if json.loads(js[-1]).get("n_gpus") != n:
            print(f"bench.py launcher: result line does not report n_gpus = {n}", file=sys.stderr)
            return 5
    return rc


def sharded_headline_line(args, world, rank_id, dist, replicas, solver, local, cache):
    """N > 1: the headline instance (seed 67, the same file on every rank) row-sharded over the N
    ranks through RCCL; W warmup trips, K timed trips of the same solve between barrier + device
    synchronisation, max over ranks.  Returns (rank, it/s, done, seconds, shard info)."""
    path = instance_for(0, args.rows, args.cols, cache)
    sv = solver.Solver(path, device=local)
    r = args.rank if args.rank > 0 else sv.determine_rank()[0]
    uid = solver.comm_unique_id() if rank_id == 0 else None
    if dist is not None:
        box = [uid]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    sv.shard_rccl(world, rank_id, uid)
    if sv.comm_ranks() != world:
        raise RuntimeError(f"RCCL communicator counts {sv.comm_ranks()} ranks, expected {world}")
    info = sv.shard_info()
    clock = {}

    def on_start():
        sv.sync()
        replicas.barrier_sync(dist)
        clock["t0"] = time.perf_counter()

    def on_stop():
        sv.sync()
        replicas.barrier_sync(dist)
        clock["t1"] = time.perf_counter()

    out = sv.alm_timed(max(1, args.warmup), args.steps, on_start, on_stop, fixedRank=r, reoptLevel=0)
    sv.close()
    _, t_max = replicas.aggregate(dist, 0, clock["t1"] - clock["t0"])
    return r, out["done"] / t_max, out["done"], t_max, info


def dry_run_line(args, world, rank_id, dist, replicas):
    """--dry-run: the launch and timing protocol only (no GPU, no solver): every rank joins the
    process group, meets the barriers around an empty timed region and contributes to the
    (sum, max) aggregate, so the multi-rank plumbing is testable on a CPU host with gloo."""
    replicas.barrier_sync(dist)
    t0 = time.perf_counter()
    replicas.barrier_sync(dist)
    dt = time.perf_counter() - t0
    joined, t_max = replicas.aggregate(dist, 1, dt)   # each rank counts itself once
    return {"metric": "ALM iters/sec, MaxCut G67 (torus 100x100 +-1, n=m=10000), fixed default rank",
            "value": 0.0, "unit": "ALM inner iterations/s", "n_gpus": world, "steps": 0, "warmup": 0,
            "ms_per_step": t_max * 1e3, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64", "data": "dry run: launch and timing protocol only, no GPU work",
            "config": {"workload": "none (dry run)", "parallelism": headline_parallelism(world)},
            "headline": headline_kind(world), "replicas": {"scaling": "weak", "value": None},
            "dry_run": True, "backend": dist.get_backend() if dist is not None else None,
            "ranks_aggregated": int(joined)}


def headline_kind(world):
    return "single instance" if world == 1 else "sharded (one instance row-sharded over RCCL, lrs_shard_rccl)"


def headline_parallelism(world):
    return "none (1 GPU)" if world == 1 else f"row-sharded x{world} (one instance; RCCL halo + all-reduce)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node, one process each (default: WORLD_SIZE, else 1); without an "
                         "external launcher the script starts the N rank processes itself")
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--rows", type=int, default=100)
    ap.add_argument("--cols", type=int, default=100)
    ap.add_argument("--rank", type=int, default=0, help="fixed rank (0 = LoRADS default)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-eps", action="store_true")
    ap.add_argument("--no-scale", action="store_true")
    ap.add_argument("--no-north-star", action="store_true")
    ap.add_argument("--no-configs", action="store_true")
    ap.add_argument("--no-c5", action="store_true")
    ap.add_argument("--no-c5b", action="store_true")
    ap.add_argument("--no-sharded", action="store_true")
    ap.add_argument("--sharded-timeout", type=float, default=300.0)
    ap.add_argument("--sharded-all", action="store_true",
                    help="the C5 and 2000^2-torus sharded legs at N = 1 too (with LRS_FORCE_SHARD=1: "
                         "the sharded iteration over a one-rank RCCL communicator)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch + barrier/aggregate protocol only over gloo, no GPU (CPU tests)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world) if env_world is not None else 1
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE = {world}", file=sys.stderr)
        sys.exit(2)
    rank_id = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if args.dry_run:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl")
    replicas = importlib.import_module(PKG + ".replicas")
    if args.dry_run:
        line = dry_run_line(args, world, rank_id, dist, replicas)
        if rank_id == 0:
            print(json.dumps(line), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    solver = importlib.import_module(PKG + ".solver")
    cache = os.path.join(ROOT, ".bench_instances")
    os.makedirs(cache, exist_ok=True)
    failed = 0
    sharded_head = None
    if world > 1:
        # the headline at N > 1: ONE instance row-sharded over the ranks (a watchdog keeps a stuck
        # collective from swallowing the run: the replicas line below is then labelled as such)
        import threading

        def fire_head():
            print(f"bench.py rank {rank_id}: sharded headline hung for {args.sharded_timeout:.0f} s", file=sys.stderr,
                  flush=True)
            os._exit(3)
        wd0 = threading.Timer(args.sharded_timeout, fire_head)
        wd0.daemon = True
        wd0.start()
        try:
            sharded_head = sharded_headline_line(args, world, rank_id, dist, replicas, solver, local, cache)
        except Exception as e:
            sharded_head = {"error": repr(e)[:300]}
            print(f"bench.py rank {rank_id}: sharded headline failed: {e!r}", file=sys.stderr, flush=True)
            failed = 4
        wd0.cancel()
    path = instance_for(rank_id, args.rows, args.cols, cache)
    sv = solver.Solver(path, device=local)
    r = args.rank if args.rank > 0 else sv.determine_rank()[0]
    n = sv.dims[0]
    kw = dict(fixedRank=r, reoptLevel=0)

    # ONE phase-1 solve: W untimed warmup inner iterations (solver setup, initial point and
    # first gradient included), then exactly K inner iterations of the same solve timed
    # between barrier + device synchronisation on both sides (lrs_set_budget_hook)
    clock = {}

    def on_start():
        sv.sync()
        replicas.barrier_sync(dist)
        clock["t0"] = time.perf_counter()

    def on_stop():
        sv.sync()
        replicas.barrier_sync(dist)
        clock["t1"] = time.perf_counter()

    out = sv.alm_timed(max(1, args.warmup), args.steps, on_start, on_stop, **kw)
    dt = clock["t1"] - clock["t0"]
    done = out["done"]
    done_tot, t_max = replicas.aggregate(dist, done, dt)

    line = {
        "metric": "ALM iters/sec, MaxCut G67 (torus 100x100 +-1, n=m=10000), fixed default rank",
        "value": done_tot / t_max,
        "unit": "ALM inner iterations/s",
        "n_gpus": world,
        "steps": int(done),
        "warmup": args.warmup,
        "ms_per_step": t_max * 1e3 / max(1, done),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: seeded G67-structured toroidal grid (real Gset file absent)",
        "config": {"workload": f"MaxCut torus {args.rows}x{args.cols} (G67 structure)", "n": n, "m": sv.m,
                   "rank": r, "pattern_slots": sv.nslots, "constraint_nnz": sv.nnz,
                   "flags": "--fixedRank %d --reoptLevel 0, phase-1 exit disabled, budget = steps" % r,
                   "parallelism": headline_parallelism(world)},
        "headline": headline_kind(world),
        "alm_phase_rate": done / out["seconds"],
        "build": build_provenance(),
        "roofline": stage_roofline(sv, 300, leg="g67"),
    }
    if world > 1:
        # value = the single row-sharded instance; the per-rank instances (this run's unsharded
        # solves above) are the weak-scaling replicas
        line["replicas"] = {"value": done_tot / t_max, "unit": "ALM inner iterations/s (sum over ranks)",
                            "scaling": "weak", "steps_per_rank": int(done), "seconds_max": t_max,
                            "workload": "one G67-structured instance per rank (seeds 67 + rank), no data-path collective"}
        if isinstance(sharded_head, tuple):
            rs, rate, sdone, ssec, info = sharded_head
            line["value"] = rate
            line["steps"] = int(sdone)
            line["ms_per_step"] = ssec * 1e3 / max(1, sdone)
            line["config"]["rank"] = rs
            line["sharded_headline"] = {"transport": "RCCL (ncclSend/Recv halo, ncclAllReduce totals)",
                                        "rank0_rows": info[3], "rank0_halo_rows": info[4], "seconds_max": ssec}
        else:
            # labelled fallback: the replicas' rate (weak scaling), and a non-zero exit status
            line["scaling"] = "weak"
            line["config"]["parallelism"] = f"replicas x{world} (instance-level, weak) -- sharded headline FAILED"
            line["headline"] = "replicas (the sharded headline FAILED: see sharded_headline.error)"
            line["sharded_headline"] = sharded_head
    if rank_id == 0 and world == 1 and not args.no_eps:
        eps_flags = dict(reoptLevel=0, heuristicFactor=10.0, phase1Tol=1e-2, phase2Tol=1e-5)
        t1 = time.perf_counter()
        sol = sv.solve(**eps_flags)
        wall = time.perf_counter() - t1
        line["wall_clock_to_eps"] = {"eps": 1e-5, "flags": "--reoptLevel 0 --heuristicFactor 10 --phase1Tol 1e-2",
                                     "solve_time_sec": sol["solve_time"], "call_wall_sec": wall,
                                     "alm_inner": sol["alm_inner"], "admm_iter": sol["admm_iter"],
                                     "primal_obj": sol["pobj"], "alm_primal_obj": sol["alm_pobj"],
                                     "pinf": sol["pinf"], "gap": sol["gap"], "rank": sol["final_rank"]}
    sv.close()
    if rank_id == 0 and world == 1 and not args.no_cpu:
        it, sec, kind = cpu_reference_rate(path, r, args.cpu_seconds)
        nthr, model = host_cpu()
        line["cpu_baseline"] = {"value": it / sec, "unit": "ALM inner iterations/s", "cores": 1, "kind": kind,
                                "sample": f"phase-1 ALM on the same instance at rank {r}, {it} inner iterations "
                                          f"in {sec:.1f} s wall (OPENBLAS_NUM_THREADS=1)",
                                "host": {"cpu_model": model, "threads_available": nthr}}
        # the reference's BLAS on every thread this process may use (its loop is single-threaded C;
        # only BLAS calls can spread), at most 16: the GPU box's CPU share for one GPU
        # (OMP_NUM_THREADS / MAX_JOBS are 16 there; nproc shows the whole host)
        ta = min(nthr, 16)
        it2, sec2, _ = cpu_reference_rate(path, r, min(args.cpu_seconds, 10.0), threads=ta)
        line["cpu_baseline"]["all_cores"] = {"value": it2 / sec2, "threads": ta,
                                             "sample": f"{it2} inner iterations in {sec2:.1f} s wall "
                                                       f"(OPENBLAS_NUM_THREADS={ta}: the box's CPU share "
                                                       f"for one GPU is 16 threads)"}
        if not args.no_eps:
            ref = cpu_reference_solve(path, ["--reoptLevel", "0", "--heuristicFactor", "10", "--phase1Tol", "1e-2"],
                                      timeout=600)
            if ref:
                line["cpu_baseline"]["wall_clock_to_eps"] = ref
    if rank_id == 0 and world == 1 and not args.no_north_star:
        # BASELINE.json target: >= 10x CPU LoRADS it/s on MaxCut n = 20 000, rank 64, 1 GPU
        p81 = instance_for(0, 100, 200, cache, seed0=81)
        s81 = solver.Solver(p81, device=local)
        kw81 = dict(fixedRank=64, reoptLevel=0)
        s81.alm_throughput(0, 100, **kw81)
        o81 = s81.alm_throughput(0, 1000, **kw81)
        ns = {"workload": "MaxCut torus 100x200 (G81 structure), n=m=20000, --fixedRank 64",
              "gpu_it_s": o81["done"] / o81["seconds"], "roofline": stage_roofline(s81, 100, leg="g81")}
        s81.close()
        if not args.no_cpu:
            it, sec, kind = cpu_reference_rate(p81, 64, min(args.cpu_seconds, 10.0))
            ns["cpu_it_s"] = it / sec
            ns["cpu_kind"] = kind
            ns["speedup"] = ns["gpu_it_s"] / ns["cpu_it_s"]
        line["north_star"] = ns
    if rank_id == 0 and world == 1 and not args.no_configs:
        # the other BASELINE.json configs as whole solves to eps = 1e-5 with benchmark.py's
        # flags for their subtype (get_lorads_params, benchmark.py:136-200), device vs reference
        inst = importlib.import_module(PKG + ".instances")
        gset = {"reoptLevel": 0, "heuristicFactor": 10.0, "phase1Tol": 1e-2, "rhoMax": 5000.0}
        sdplib = {"reoptLevel": 0, "heuristicFactor": 1.0, "phase1Tol": 1e-3, "rhoMax": 5000.0}
        rows = []
        for name, flags in (("G1", gset), ("G22", gset), ("theta3", sdplib), ("theta3x3", sdplib)):
            pth = inst.config_instance(name, cache)
            s1 = solver.Solver(pth, device=local)
            res = s1.solve(**flags)
            s1.close()
            row = {"config": name, "gpu_solve_s": res["solve_time"], "alm_inner": res["alm_inner"],
                   "admm_iter": res["admm_iter"], "primal_obj": res["pobj"], "gap": res["gap"], "pinf": res["pinf"]}
            if not args.no_cpu:
                cli = []
                for k, v in flags.items():
                    cli += [f"--{k}", str(v)]
                ref = cpu_reference_solve(pth, cli, timeout=300)
                if ref:
                    row["cpu_solve_s"] = ref["solve_time_sec"]
                    row["speedup"] = ref["solve_time_sec"] / res["solve_time"]
            rows.append(row)
        line["configs_wall_clock_to_eps"] = rows
    if rank_id == 0 and world == 1 and not args.no_scale:
        # roofline at scale: 2000 x 2000 torus built in memory (lrs_load_coo), rank 16
        inst = importlib.import_module(PKG + ".instances")
        t1 = time.perf_counter()
        big = solver.Solver(coo=inst.coo_arrays(inst.maxcut_torus_problem(2000, 2000, 2000)), device=local)
        load_s = time.perf_counter() - t1
        kwb = dict(fixedRank=16, reoptLevel=0)
        ob = big.alm_timed(5, 60, **kwb)
        rl = stage_roofline(big, 20, leg="torus2000")
        rl["workload"] = "MaxCut torus 2000x2000 (n=m=4e6), --fixedRank 16, in-memory load"
        rl["it_s"] = ob["done"] / ob["seconds"]
        rl["load_sec"] = load_s
        big.close()
        line["roofline_at_scale"] = rl
    if rank_id == 0 and world == 1 and not args.no_c5:
        line["config_c5"] = config_c5(solver, local, cpu_seconds=0.0 if args.no_cpu else 20.0, cache=cache)
    if rank_id == 0 and world == 1 and not args.no_c5b:
        line["config_c5b"] = config_c5b(solver, local, ref_densec=ref_densec_rates())
    if not args.no_sharded:
        # a watchdog keeps a stuck collective from swallowing the result line
        import threading

        def fire():
            # a stuck collective: the headline above is measured and printed, the sharded section
            # is reported as failed in the line and on stderr, and every rank leaves without
            # waiting on the communicator -- with a non-zero status, so the hang reads as a failure
            if rank_id == 0:
                line["sharded"] = {"error": f"no result within {args.sharded_timeout:.0f} s"}
                print(json.dumps(line), flush=True)
            print(f"bench.py rank {rank_id}: sharded section hung for {args.sharded_timeout:.0f} s", file=sys.stderr,
                  flush=True)
            os._exit(3)
        wd = threading.Timer(args.sharded_timeout, fire)
        wd.daemon = True
        wd.start()
        try:
            line["sharded"] = sharded_strong(solver, dist, world, rank_id, local, cache, replicas,
                                             all_legs=args.sharded_all)
        except Exception as e:   # reported in the line (the headline stands) and in the exit status
            line["sharded"] = {"error": repr(e)[:300]}
            print(f"bench.py rank {rank_id}: sharded section failed: {e!r}", file=sys.stderr, flush=True)
            failed = 4
        wd.cancel()
    if rank_id == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if failed:
        sys.exit(failed)


if __name__ == "__main__":
    main()
