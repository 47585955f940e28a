/*
 * oracle/lrsdp_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the LoRADS low-rank SDP path (reference:
 * /root/reference/lorads/src/src_semi, cited file:line in lrsdp_oracle.c).
 * Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
 * always as the checker, never as the thing measured or shipped.
 *
 * Parity pin: every kernel and the phase-1/phase-2 trajectories are checked
 * against golden fixtures produced by the reference itself (oracle/_ref,
 * scripts/make_golden.py) -- see tests/test_oracle_golden.py.
 */
#ifndef LRSDP_ORACLE_H
#define LRSDP_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

typedef struct oproblem oproblem;

/* Read an SDPA .dat-s file and presolve it (pattern, slot maps).  NULL on error. */
oproblem *oracle_read(const char *path);
void oracle_free(oproblem *p);
int oracle_dims(const oproblem *p, int *m, int *ncones, int *dims);

/* One call of each hot-path operator on caller-provided iterates.
 * `in`/`out` use exactly the binary layout of oracle/ref_harness.c mode_kernels. */
int oracle_kernels(oproblem *p, int rank, const double *in, double *out);
/* LORADSUpdateSDPVar over every cone + LORADSUpdateDualVar on the same input layout; out = U,
 * V, A(UV^T), lambda, total CG iterations, per cone its last CG count (returns the length) */
int oracle_admm_sweep(oproblem *p, int rank, const double *in, double *out);
/* The same with the LP block (the last cone, rank 1): the SDP cones' CG half-steps, then the LP
 * column sweep; out = U, V, A(UV^T), lambda, total CG iterations (oracle/ref_harness.c
 * admm_sweep_lp's layout; returns the length) */
int oracle_admm_sweep_lp(oproblem *p, int rank, const double *in, double *out);

/* Full solve with LoRADS flags (argv-style, e.g. {"--reoptLevel","0"}).
 * res[0..15] = alm_inner, alm_outer, alm_pobj, alm_dobj, alm_pinf, alm_gap, alm_rho,
 *              admm_iter, admm_pobj, admm_dobj, admm_pinf, admm_gap, admm_rho,
 *              solve_time, rank, alm_time */
int oracle_solve(const char *path, int nflags, char **flags, double *res);

/* Bounded phase-1 rate at fixed rank: returns inner iterations done within
 * `seconds` of wall time; *elapsed receives the phase-1 time. */
long oracle_alm_rate(const char *path, int rank, double seconds, double *elapsed);

/* Exactly K phase-1 inner iterations from the reference's initial point (rank <= 0: the
 * default rank); out = R, G, A(RR^T), lambda (R, G col-major per cone).  Returns the
 * doubles per factor, or -1 (read error, fewer than K iterations, or cap too small). */
long oracle_alm_steps(const char *path, int rank, long K, double *out, long cap);

/* First n outputs of the restated glibc rand() after srand(seed). */
int oracle_rand_seq(unsigned seed, int n, int *out);

#ifdef __cplusplus
}
#endif
#endif
