/*
 * lrsdp.h -- C-ABI of the MI355X-native low-rank SDP inner solver (liblrsdp.so).
 *
 * This is the in-process boundary that replaces the reference's operator
 * vtables on the hot path:
 *   - algorithm slots  lorads_func        (lorads/src/src_semi/data/def_lorads_solver.h:169-187,
 *                                          bound in data/lorads_solver.c:1014-1053)
 *   - cone slots       lorads_sdp_cone    (data/def_lorads_sdp_conic.h:100-124,
 *                                          bound in data/lorads_sdp_conic.c:974-1029)
 *   - coefficient slots sdp_coeff         (data/def_lorads_sdp_data.h:66-85)
 *   - CG callback      Mvec               (linalg/def_lorads_cgs.h:71-72, linalg/lorads_cgs.c:107)
 * The process boundary (the LoRADS CLI that benchmark.py calls,
 * benchmark.py:240-262 / src_semi/main.c:256) is the `LoRADS_v_2_0_1-alpha`
 * binary built on top of this library.
 *
 * Conventions: every function returns 0 on success and a negative code on
 * failure (message via lrs_last_error()); no function calls exit().  A NULL
 * context, a context with no problem loaded (or, for the operators, no ranks
 * set) and a NULL required pointer are failures of that kind, never a crash.  All
 * arrays crossing the boundary are host memory, column-major n x r per cone
 * (the reference layout, lorads_alg_common.c:62-68), cones concatenated in
 * cone order.  Device memory is owned by the context.
 */
#ifndef LRSDP_H
#define LRSDP_H
/* ABI revision, also in lrs_version()'s string.  2: lrs_op_admm_half takes (cone, side) and
 * refreshes the cone's constraint values itself (was: the whole sweep's first half-step);
 * lrs_op_alm_update, lrs_op_adjoint, lrs_op_auv and lrs_op_dimacs added. */
#define LRSDP_ABI_VERSION 2
#ifdef __cplusplus
extern "C" {
#endif

typedef struct lrs_ctx lrs_ctx;
typedef struct lrs_loopback lrs_loopback;

/* LoRADS flags (main.c:56-86 defaults, main.c:125-154 names) + the three flags
 * benchmark.py passes that the reference never implemented. */
typedef struct {
    double initRho, rhoMax, rhoCellingALM, rhoCellingADMM;
    int maxALMIter, maxADMMIter;
    double timesLogRank;
    int fixedRank, initRank, rhoFreq;
    double rhoFactor, ALMRhoFactor, rankUpdateFactor, phase1Tol, phase2Tol, timeSecLimit, heuristicFactor;
    int lbfgsListLength;
    double endTauTol, endALMSubTol;
    int l2Rescaling, reoptLevel, dyrankLevel, highAccMode, oracleRankNaive;
    /* additions (INTEGRATION.md "rank-schedule hook") */
    int disableOracle;
    double nearStallFactor;
    const int *rankSchedule;
    int rankScheduleLen;
    int verbose;          /* print the LoRADS-format iteration log to stdout */
    long almInnerBudget;  /* >0: stop phase 1 after this many inner iterations (benchmarking) */
    int skipADMM;         /* 1: phase 1 only */
} lrs_params;

typedef struct {
    long alm_inner, alm_outer, admm_iter, cg_iter;
    double alm_pobj, alm_dobj, alm_pinf, alm_gap, alm_rho;
    double pobj, dobj, pinf, pinf_inf, gap, rho;   /* admm_state after main.c:519-525 */
    double solve_time, alm_time, admm_time, read_time;
    int status;          /* lorads_status: 0 unknown, 1 primal-dual optimal, 2 primal optimal, 3 maxiter, 4 time limit */
    int retcode;         /* RET_CODE_* of phase 1 */
    int final_rank, oracle_rank;
    int traj1_len, traj2_len;
    double rho_max;      /* params.rhoMax after LORADS_ALMtoADMM (written to the JSON) */
    double dinf, dinf_inf, dinf_2;   /* dual infeasibility l_1 / l_inf / l_2 (main.c:515-521); -1 if not evaluated */
    int dinf_converged;  /* 1: every cone's eigen-solve met its test (ARPACK's tol 1e-2 relative Ritz estimate,
                            or an absolute one that pins the l_1 value to 1e-3 phase2Tol); 0: the 600 update
                            iterations ran out (dinf is then a lower bound and status 1 is withheld); -1: not
                            evaluated */
    int dinf_iters;      /* thick-restart update iterations (dsaupd's iparam(3) count) over cones and calls */
    long dinf_steps;     /* Lanczos steps (matrix-vector products) over cones and calls */
    double dinf_time;    /* seconds in the dual-infeasibility eigen-solves (inside solve_time, as main.c:515-521) */
    double obj_scale;    /* scaleObjHis at the end (the reopt rounds' objScale_dualvar factors; 1 without reopt) */
} lrs_result;

/* factor / vector selectors */
enum { LRS_R = 0, LRS_D = 1, LRS_G = 2, LRS_U = 3, LRS_V = 4, LRS_S0 = 5, LRS_Y0 = 6, LRS_S1 = 7, LRS_Y1 = 8 };
enum { LRS_LAMBDA = 0, LRS_CVS = 1, LRS_Q1 = 2, LRS_Q2 = 3, LRS_B = 4 };

void lrs_params_default(lrs_params *p);
const char *lrs_last_error(void);
const char *lrs_version(void);
int lrs_abi_version(void);   /* LRSDP_ABI_VERSION of the library */

int lrs_ctx_create(int device, lrs_ctx **out);
void lrs_ctx_destroy(lrs_ctx *ctx);

/* SDPA .dat-s reader + presolve + upload (replaces LReadSDPA io/lorads_file_io.c:59,
 * LORADSPreprocess data/lorads_solver.c:278, AConePresolveData data/lorads_sdp_conic.c:1185).
 * read_seconds may be NULL. */
int lrs_load_sdpa(lrs_ctx *ctx, const char *path, double *read_seconds);
int lrs_problem_info(lrs_ctx *ctx, int *m, int *ncones, int *dims, long *nslots, long *nnz_constraints);

/* ranks: LORADSDetermineRank (data/lorads_solver.c:406) given flags; or explicit. */
int lrs_determine_rank(lrs_ctx *ctx, const lrs_params *p, int *ranks_out);
int lrs_set_rank(lrs_ctx *ctx, const int *ranks);
int lrs_get_rank(lrs_ctx *ctx, int *ranks);

int lrs_factor_set(lrs_ctx *ctx, int which, const double *colmajor);
int lrs_factor_get(lrs_ctx *ctx, int which, double *colmajor);
int lrs_vec_set(lrs_ctx *ctx, int which, const double *v);
int lrs_vec_get(lrs_ctx *ctx, int which, double *v);

/* ---- operators (one device pass each; scalars returned through pointers) ---- */
/* ALMCalq12p12 (lorads_alm.c:714): q1 = 2A(sym RD^T), p1 = 2<C,sym RD^T>, q2 = A(DD^T), p2 = <C,DD^T> */
int lrs_op_q12(lrs_ctx *ctx, double *q1, double *p1, double *q2, double *p2);
/* primalInfeasibility (lorads_alg_common.c:386) on R: CVS <- A(RR^T); pinf; and <C,RR^T> */
int lrs_op_constr_rr(lrs_ctx *ctx, double *cvs, double *pinf, double *pobj);
/* ALMCalGrad (lorads_alm.c:74) from LAMBDA, CVS at rho: G <- 2(C + A^*(M1))R */
int lrs_op_grad(lrs_ctx *ctx, double rho, double *lag_norm_sq);
/* ALMLineSearch (lorads_alm.c:266) on the state left by lrs_op_q12 with q0 = b - CVS */
int lrs_op_line_search(lrs_ctx *ctx, double rho, double *tau, int *root_num);
/* LBFGSDirection + LBFGSDirectionUseGrad (lorads_alm.c:468-505, :607-627) from G and
 * the ring (S0,Y0 = newest pair with beta_new; S1,Y1 = older pair with beta_old),
 * node_num in {0,1,2}; result in D. */
int lrs_op_lbfgs(lrs_ctx *ctx, int node_num, double beta_new, double beta_old);
/* LORADSInitConstrValAll + LORADSInitConstrValSum (lorads_alg_common.c:104-229) on (U, V):
 * the per-cone A_k(sym UV^T) and their sum CVS that the ADMM half-steps read and update. */
int lrs_op_admm_constr(lrs_ctx *ctx);
/* One ADMM half-step of LORADSUpdateSDPVar (lorads_alg_common.c:298-326) for cone `cone`:
 * LORADSUpdateSDPVarOne (lorads_admm.c:564-616) solving side 0 = U with V fixed or side 1 =
 * V with U fixed (RHS -(S Y - rho Y)/rho with S = C + A*(rho (CVS - A_k(UV^T) - b) - LAMBDA),
 * CG at cg_tol / cg_maxit, warm-started from the current factor), then the cone's
 * constraint-value refresh (CVS -= A_k, A_k <- A_k(sym UV^T), CVS += A_k).  Calling it for
 * (0, 0), (0, 1), (1, 0), (1, 1), ... after lrs_op_admm_constr is the reference's sweep.
 * cg_iters (may be NULL): this solve's CG iterations; rhs (may be NULL): the cone's
 * right-hand side, column-major n_k x r_k. */
int lrs_op_admm_half(lrs_ctx *ctx, int cone, int side, double rho, double cg_tol, int cg_maxit, int *cg_iters,
                     double *rhs);
/* LP blocks (LORADSSetLpCone, data/lorads_lp_conic.c:347; the *LP slots of lorads_func bound in
 * LORADSInitFuncSet, data/lorads_solver.c:1014-1053): a problem whose last SDPA block has negative
 * size -k carries its k LP columns (x_j = r_j^2) as one more cone, the LAST one, of k rows at rank 1
 * (lrs_get_rank reports 1 for it; lrs_set_rank refuses another rank).  Factors therefore hold the
 * LP values after the SDP cones' (the reference's rLp / uLp / vLp), and every operator above acts on
 * it as on an SDP cone with a diagonal pattern -- which is the LP algebra.  Two exceptions follow
 * the reference: lrs_op_admm_half(ctx, lp_cone, 0, ...) runs the LP block's whole ADMM update, the
 * closed-form column sweep of LORADSUpdateSDPLPVar (u_j then v_j per column, lorads_admm.c:759-792;
 * side 1 is refused, cg_iters = 0, rhs untouched), and lrs_op_dual_infeasibility's LP term is
 * sum_j |min(c_j - sum_i lambda_i a_ij, 0)| (lam_min[lp_cone] = the smallest such value).  The
 * oracle rank, AUG_RANK and the reported ranks cover the SDP cones only.  Sharded contexts refuse
 * LP blocks. */
/* LORADSUpdateDualVar (lorads_alg_common.c:511-524): LAMBDA += rho (b - CVS). */
int lrs_op_dual_update(lrs_ctx *ctx, double rho);
/* The second half of one ALM inner trip after the line search (lorads_alm.c:1340-1355):
 * setAsNegGrad (:780-801), ALMupdateVar R += tau D (:804-833), CVS += tau q1 + tau^2 q2 with the
 * q1, q2 of the last lrs_op_q12 (:1349-1352), ALMCalGrad at rho (:74-87: G <- 2(C + A^*(M1))R,
 * lag_norm_sq = ||G||^2) and setlbfgsHisTwo (:842-863: s = tau D, y = G_new - G_old, beta =
 * 1/<y,s>).  The new pair lands in (LRS_S0, LRS_Y0) and the previous newest moves to (LRS_S1,
 * LRS_Y1), the roles lrs_op_lbfgs reads, so a caller steps the reference's loop with
 * lrs_op_lbfgs -> lrs_op_q12 -> lrs_op_line_search -> lrs_op_alm_update -> lrs_op_dimacs
 * (updateDimacsALM).  lag_norm_sq, beta may be NULL.  Unsharded contexts. */
int lrs_op_alm_update(lrs_ctx *ctx, double rho, double tau, double *lag_norm_sq, double *beta);
/* sdpDataWSum + mul_rk (data/def_lorads_sdp_data.h:66-85) over every cone: out = scale (with_C C +
 * sum_i y[i] A_i) X, X the factor `which` (LRS_R, LRS_U, ...), y[m] host, out column-major like
 * lrs_factor_get.  Unsharded contexts. */
int lrs_op_adjoint(lrs_ctx *ctx, const double *y, int which, double *out, double scale, int with_C);
/*   lrs_op_adjoint works in the solver's scratch: the constraint weights (the M1 buffer), the slot
 *   values S, and the X / CG-Q work factors are overwritten.  No operator reads those across
 *   calls -- lrs_op_grad, lrs_op_admm_half and the fused loops form M1 and S afresh -- so the
 *   iterate (R, U, V, D, G, the L-BFGS pairs), LAMBDA and CVS are unchanged by it. */
/* coneAUV + objAUV (data/def_lorads_sdp_conic.h:106-111) summed over the cones: out_m[i] =
 * <A_i, sym(X_u X_v^T)> (u == v: X_u X_u^T), cobj = <C, sym(X_u X_v^T)> before the division by
 * the reopt objective scale.  Leaves the solver state (CVS) unchanged.  out_m, cobj may be NULL.
 * Unsharded contexts. */
int lrs_op_auv(lrs_ctx *ctx, int u, int v, double *out_m, double *cobj);
/* LORADSUpdateDimacsErrorALM (admm = 0, on R) / LORADSUpdateDimacsErrorADMM (admm = 1: R = (U +
 * V)/2 first) (lorads_alg/lorads_alg_common.c:424-428, :454-462) with the objectives they read
 * (LORADSCalObjRR_ALM lorads_alm.c:1488, LORADSCalObjUV_ADMM, LORADSCalDualObj
 * lorads_alg_common.c:531): CVS <- A(R R^T); out5 = {pObj, dObj, l_1 primal infeasibility, l_inf
 * primal infeasibility, |pObj - dObj| / (1 + |pObj| + |dObj|)}. */
int lrs_op_dimacs(lrs_ctx *ctx, int admm, double *out5);
/* Gram R^T R of cone k (r x r, row-major) */
int lrs_op_gram(lrs_ctx *ctx, int cone, int which, double *gram);
/* Dual infeasibility of the current multipliers (calculate_dual_infeasibility_solver,
 * data/lorads_solver.c:1396-1426): l1 = sum_k |min(lambda_min(S_k), 0)| / scaleObjHis /
 * (||C||_1 + 1) with S = C - sum_i lambda_i A_i; lam_min[k] per cone (may be NULL).  The
 * reference's ARPACK dsaupd "SA" (ncv 40, tol 1e-2, data/lorads_sdp_conic.c:1636-1699) is
 * replaced by a device thick-restart Lanczos with dsaupd's semantics: a basis of 40 vectors,
 * 20 Ritz vectors kept per restart, two-pass classical Gram-Schmidt, convergence when the
 * Ritz residual is <= tol * max(eps^(2/3), |theta|), at most 600 restarts. */
int lrs_op_dual_infeasibility(lrs_ctx *ctx, double *l1, double *lam_min);

/* ---- whole solves ---- */
/* main.c:380-610 flow: ALM phase, ADMM phase, reoptLevel 1/2 rounds (all on the device), dual
 * infeasibility (skipped after a time-limit exit, as main.c:505-510 jumps to END_SOLVING). */
int lrs_solve(lrs_ctx *ctx, const lrs_params *p, lrs_result *res);
/* trajectory (phase 1 then phase 2) after lrs_solve: curr and oracle ranks */
int lrs_trajectory(lrs_ctx *ctx, int phase, int *curr_rank, int *oracle_rank, int cap);
/* JSON like lorads_logging.c:618-712 */
int lrs_write_json(lrs_ctx *ctx, const char *path, const char *problem_id, const char *file_path,
                   const lrs_result *res, const lrs_params *p);

/* Phase-1 throughput: runs `warmup` then `steps` ALM inner iterations at the
 * current rank (phase1Tol effectively off), timing the steps with device events.
 * kernel_ms (optional) receives per-kernel average durations of the A(UU^T)
 * SDDMM kernel measured with HIP events on the solver stream. */
int lrs_alm_throughput(lrs_ctx *ctx, const lrs_params *p, long warmup, long steps, double *seconds,
                       long *done, double *sddmm_avg_ms, double *iter_avg_ms);

/* Benchmark hook on the phase-1 budget (lrs_params.almInnerBudget): when the ALM inner
 * loop reaches the budget, the solve synchronises its stream and calls
 * hook(user, inner_iterations_done).  A return value larger than the count continues the
 * SAME solve (same iterate, L-BFGS ring and control block) up to that new absolute budget;
 * anything else ends phase 1 as without a hook.  This lets a caller time exactly K inner
 * iterations after W warmup iterations with no solver setup inside the timed region.
 * NULL removes the hook.  (No reference counterpart: benchmarking only.) */
typedef long (*lrs_budget_hook)(void *user, long inner_done);
int lrs_set_budget_hook(lrs_ctx *ctx, lrs_budget_hook hook, void *user);
/* The last completed ALM inner iteration of the last solve (after a budget stop: trip
 * almInnerBudget): out4 = {tau, ||G||^2, l_1 primal infeasibility, beta of the newest
 * L-BFGS pair}; newest_pair = 0 if that pair is (LRS_S0, LRS_Y0), 1 if (LRS_S1, LRS_Y1).
 * (Test hook for the per-iteration parity against the reference's inner loop,
 * lorads_alm.c:1302-1379.) */
int lrs_alm_last_step(lrs_ctx *ctx, double *out4, int *newest_pair);
/* Wait for every operation enqueued on the context's stream. */
int lrs_sync(lrs_ctx *ctx);

/* Mirror the iteration log into a file (the reference's --logfile). */
int lrs_set_log_path(lrs_ctx *ctx, const char *path);

/* Kernel selection of the ALM inner iteration (same arithmetic either way):
 * 0 = automatic (the latency-regime kernels k_lat_a/k_lat_b when every row's lane group is
 * resident at once, else the general row kernels), 1 = general row kernels only,
 * 2 = general row kernels in their bandwidth-regime form (stages split in two launches),
 * 3 = as 2 with the long-row neighbour kernels k_wide_a/k_wide_b wherever the layout allows.
 * The environment variable LRS_NO_LAT=1 forces 1 for every context. */
int lrs_set_kernel_path(lrs_ctx *ctx, int path);
/* The path the last enqueued ALM inner iteration of this context took (0 latency-regime
 * kernels, 1 general row kernels; -1 none enqueued yet). */
int lrs_get_kernel_path(lrs_ctx *ctx, int *used);

/* Standalone A(UU^T) on R (the constraint-entry kernel k_auv_con, all cones): reps
 * launches back to back between two HIP events, average ms per launch; and its
 * algorithmic bytes (factor rows touched once + entry data + outputs). */
int lrs_time_auut(lrs_ctx *ctx, int reps, double *avg_ms);
int lrs_auut_bytes(lrs_ctx *ctx, double *bytes);

/* Standalone r x r Gram R^T R of one cone (build_gram_from_factor, lorads_logging.c:216-240;
 * k_gram on the FP64 matrix cores, then the fixed-order partial reduction): avg_ms = ms per
 * Gram (kernel + reduction), gram_ms = ms of the MFMA kernel alone (may be NULL). */
int lrs_time_gram(lrs_ctx *ctx, int cone, int reps, double *avg_ms, double *gram_ms);

/* The FP64 matrix-core ceiling on this device, measured: TFLOP/s of back-to-back
 * v_mfma_f64_16x16x4f64 on every CU (8 independent accumulators a wave, 2 waves a SIMD).
 * Diagnostics for the Gram's roofline; no reference counterpart. */
int lrs_mfma_f64_peak(lrs_ctx *ctx, double *tflops);
/* The same probe at `waves_per_simd` (1..8) waves a SIMD with `chains` (4 or 8) independent
 * accumulators a wave, plus the shader clock under that load (s_memtime against the 100 MHz
 * wall clock, MHz) and the cycles a SIMD spends per v_mfma_f64_16x16x4f64: the matrix-core
 * rate separated from the clock (bench.py "mfma_probe").  No reference counterpart. */
int lrs_mfma_f64_probe(lrs_ctx *ctx, int waves_per_simd, int chains, double *tflops, double *mhz,
                       double *cycles_per_mfma);

/* Dense objective (a cone whose C is kept as a full n x n matrix: LRS_DENSE_C=1, or n >= 1024
 * with C filling >= 1/4 of the lower triangle): ms per C R product on the FP64 matrix cores
 * (k_cgemm, 2 n^2 r flop), averaged over `reps`.  Fails when the cone has no dense objective. */
int lrs_time_dense(lrs_ctx *ctx, int cone, int reps, double *avg_ms);

/* Per-stage timing of the split ALM inner iteration: runs `steps` inner iterations at
 * the current rank like lrs_alm_throughput, with HIP events on the solver stream
 * around each of the four launches (S1 direction+SDDMM, S2 q-gather, S3 update+
 * adjoint, S4 gradient).  stage_ms[4] = average ms per launch; *done = iterations. */
int lrs_profile_stages(lrs_ctx *ctx, const lrs_params *p, long steps, double *stage_ms, long *done);

/* In-memory problem in SDPA entry semantics (replaces LReadSDPA for callers that
 * already hold the data, io/lorads_file_io.c:59-455): nblk blocks of sizes dims
 * (the last may be negative: an LP block of -dims[nblk-1] columns, entry row = column, col
 * unused), b[m], and nnz entries (con, blk, row, col, val) with 1-based blk/row/col and con 0 =
 * F0 (C = -F0). */
int lrs_load_coo(lrs_ctx *ctx, int m, int nblk, const int *dims, const double *b, long nnz, const int *con,
                 const int *blk, const int *row, const int *col, const double *val);

/* Which kernels the upload chose for the long-row cones: *auv = 1 when
 * some cone's constraint entries are in 2-D LDS tiles (A(XY^T) by k_auv_tile), *slot = 1
 * when some cone's lower pattern is (stage A / B and S X by k_tile_a / k_tile_b1/b2).  No
 * reference counterpart (the reference's 10 % dense rule picks a BLAS-3 branch instead,
 * data/lorads_sdp_data.c:1187-1193). */
int lrs_tile_info(lrs_ctx *ctx, int *auv, int *slot);
/* *used = 1 when the last enqueued ALM iteration ran its stages over those tiles (k_tile_a,
 * k_tile_b1/b2: the stage plan picked the long-row kernels for a tiled cone), else 0. */
int lrs_tile_used(lrs_ctx *ctx, int *used);

/* Algorithmic HBM bytes per launch of the split-iteration stages A, G, B at the
 * current ranks (the roofline numerators, DESIGN.md "Kernels"). */
int lrs_stage_bytes(lrs_ctx *ctx, double *bytes);

/* Per-launch duration (ms) of the split-iteration stages A, G, B on the current solver
 * state (call after lrs_alm_throughput): each stage is relaunched `reps` times back to
 * back between two HIP events on the solver stream (the stages are idempotent for a
 * fixed control block).  stage_ms[1] = 0 when there are no multi-slot constraints. */
int lrs_time_stages(lrs_ctx *ctx, int reps, double *stage_ms);

/* Diagnostics: in-kernel phase timestamps of the last split iteration (block 0,
 * 100 MHz wall clock), out[4][16], and (blk, optional) per-block entry/exit stamps
 * blk[4][1024][2].  Returns 64 from the diagnostics build (liblrsdp_timing.so), 0
 * from the product build. */
int lrs_debug_phase_times(lrs_ctx *ctx, unsigned long long *out, unsigned long long *blk);

/* ---- Sharded solve of one instance over several GPUs.
 * Replaces the reference's single-process operator slots for one cone split by rows:
 * every process loads the whole problem (lrs_load_sdpa / lrs_load_coo), then calls one
 * lrs_shard_* with its rank; the context then owns a contiguous block of rows (+ the
 * halo of neighbour rows) and the constraints inside it, and lrs_solve /
 * lrs_alm_throughput run whole solves (ALM + ADMM + reopt rounds + the dual
 * infeasibility) with, per inner iteration, one halo exchange of direction rows and
 * all-reduces of the stage totals (line search; L-BFGS dots + residual; shared
 * constraints' sums).  Any number of SDP cones, each split alike; constraints may span row
 * blocks (shared: every holder sums its owned entries, the sums meet in an all-reduce);
 * a dense objective is held as each shard's owned row block of C with every row in the
 * halo; long-row cones keep their 2-D tile stage kernels over the owned rows.  The ADMM CG
 * runs on owned rows with its dot products all-reduced; the Lanczos of the dual
 * infeasibility on owned rows with a vector halo.  DESIGN.md §6.  Every shard
 * must make the same calls in the same order (the collectives are matched by order). */
/* RCCL: rank 0 creates the id (128 bytes) and broadcasts it; every rank then calls
 * lrs_shard_rccl on its own GPU (ncclCommInitRank is collective). */
int lrs_comm_unique_id(char *id_out);
int lrs_shard_rccl(lrs_ctx *ctx, int world, int rank, const char *id);
/* One-process loopback transport (tests): `world` contexts on one GPU, one host thread
 * each; lrs_shard_loopback is collective over the group's threads. */
int lrs_loopback_create(int world, lrs_loopback **out);
void lrs_loopback_destroy(lrs_loopback *g);
int lrs_shard_loopback(lrs_ctx *ctx, lrs_loopback *g, int rank);
/* world, rank, first global row, owned rows, halo rows of this context (1, 0, 0, n, 0 unsharded) */
int lrs_shard_info(lrs_ctx *ctx, int *world, int *rank, int *row0, int *nown, int *nhalo);
/* ranks the context's transport counts itself (RCCL: ncclCommCount; loopback: its group's
 * world; 1 unsharded), so a launcher can check that every GPU joined the communicator */
int lrs_shard_comm_ranks(lrs_ctx *ctx, int *count);
/* Recording of the transport's operations (sharded contexts): on != 0 clears the log and records
 * every later operation, 0 stops.  lrs_shard_comm_log: *n = entries recorded; out (may be NULL)
 * receives min(cap, *n) records of 5 longs {kind, peer, cone, count, offset}: kind 0 = the start
 * of one halo-exchange group (cone = the vector's cone or -1 for factor rows, count = its ops),
 * 1 = send to peer, 2 = receive from peer (count doubles; offset: send-buffer position, or the
 * landing rows' local offset x ld), 3 / 4 = device / host all-reduce of count doubles.  Both
 * transports issue their groups from one op list, so the loopback transport's log is the
 * sequence of ncclSend / ncclRecv / ncclAllReduce calls the RCCL transport makes. */
int lrs_shard_comm_record(lrs_ctx *ctx, int on);
/* Inner-loop calls whose one-workgroup-per-cone launch timed out in its
 * workgroups' exchange and was rerun from the kept state on the multi-launch iteration (the
 * context then stays on it).  LRS_XWG_SPIN=k sets the exchange's spin limit to 2^k polls
 * (default 26; -1: no wait) -- k = -1 forces the fallback (tests). */
int lrs_xwg_fallbacks(lrs_ctx *ctx, int *count);
int lrs_shard_comm_log(lrs_ctx *ctx, long *out, long cap, long *n);
/* Host-only (no device, no context) view of the row partition of a sharded solve of the
   instance at `path`: counts[8] = {n_global, first owned global row, owned rows, local rows
   (owned + halo), send rows (all peers), shared constraints, local constraints, world}, then
   (arrays may be null) bounds[world+1], local_gid[local rows], send_ptr[world+1],
   send_gid[send rows] (global ids, grouped by peer), shared_gid[shared], con_gid[local
   constraints], primary[local constraints] (1: this shard counts it in sums).  Replaces the
   reference's nothing: LoRADS has no multi-process path. */
int lrs_shard_plan(const char *path, int world, int rank, long *counts, int *bounds, int *local_gid,
                   int *send_ptr, int *send_gid, int *shared_gid, int *con_gid, int *primary);

#ifdef __cplusplus
}
#endif
#endif
