/* A plain-C caller of the boundary (include/lrsdp.h), as the reference's own host code (C)
 * would bind it.  Built by tests/test_capi.py with gcc (no C++ and no HIP headers needed on
 * the caller's side).
 *
 * usage: capi_solve <file.dat-s> <out.json> [reoptLevel]
 *          load an SDPA file, solve with the LoRADS defaults, print the result, write the
 *          reference-format JSON
 *        capi_solve --null
 *          the error contract: every entry point called with a NULL context (and the
 *          context-free ones with NULL outputs) returns a negative code, no crash; no GPU
 *        capi_solve --sweep <file.dat-s> <rank> <in.bin> <out.bin>
 *          the reference's ADMM variable update over every cone through the per-cone
 *          operators (LORADSUpdateSDPVar, lorads_alg_common.c:298-326) and the dual update
 *          (:511-524): in.bin = U, V (column-major per cone, cones concatenated), lambda[m],
 *          rho, cg_tol; out.bin = U, V, lambda, CG iterations per (cone, side)
 *        capi_solve --steps <file.dat-s> <rank> <in.bin> <out.bin> <ntrips>
 *          the reference's ALM inner loop (lorads_alm.c:1302-1379) stepped from the operators
 *          alone: per trip lrs_op_lbfgs (LBFGSDirection + UseGrad), lrs_op_q12 (ALMCalq12p12),
 *          lrs_op_line_search (ALMLineSearch), lrs_op_alm_update (setAsNegGrad, ALMupdateVar,
 *          the constrValSum update, ALMCalGrad, setlbfgsHisTwo) and lrs_op_dimacs
 *          (updateDimacsALM).  in.bin = R, G, s, y (the newest pair), lambda[m], CVS[m], beta,
 *          rho, trips done so far (the clearLBFGS count); out.bin = per trip {tau, rootNum,
 *          ||G||^2, pinf}, then R, G, CVS, lambda, s, y, beta after the last trip */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lrsdp.h"

static int null_contract(void) {
    int bad = 0, iv = 0;
    double dv = 0.0;
    long lv = 0;
    lrs_params p;
    lrs_result r;
    lrs_params_default(&p);
#define EXPECT_FAIL(call)                                                     \
    do {                                                                      \
        if ((call) >= 0) {                                                    \
            fprintf(stderr, "NULL contract broken: %s returned >= 0\n", #call); \
            bad++;                                                            \
        }                                                                     \
    } while (0)
    EXPECT_FAIL(lrs_load_sdpa(NULL, "x.dat-s", NULL));
    EXPECT_FAIL(lrs_problem_info(NULL, &iv, &iv, NULL, NULL, NULL));
    EXPECT_FAIL(lrs_determine_rank(NULL, &p, &iv));
    EXPECT_FAIL(lrs_set_rank(NULL, &iv));
    EXPECT_FAIL(lrs_get_rank(NULL, &iv));
    EXPECT_FAIL(lrs_factor_set(NULL, LRS_R, &dv));
    EXPECT_FAIL(lrs_factor_get(NULL, LRS_R, &dv));
    EXPECT_FAIL(lrs_vec_set(NULL, LRS_LAMBDA, &dv));
    EXPECT_FAIL(lrs_vec_get(NULL, LRS_LAMBDA, &dv));
    EXPECT_FAIL(lrs_op_q12(NULL, NULL, NULL, NULL, NULL));
    EXPECT_FAIL(lrs_op_constr_rr(NULL, NULL, NULL, NULL));
    EXPECT_FAIL(lrs_op_grad(NULL, 1.0, NULL));
    EXPECT_FAIL(lrs_op_line_search(NULL, 1.0, NULL, NULL));
    EXPECT_FAIL(lrs_op_lbfgs(NULL, 2, 1.0, 1.0));
    EXPECT_FAIL(lrs_op_admm_constr(NULL));
    EXPECT_FAIL(lrs_op_admm_half(NULL, 0, 0, 1.0, 1e-8, 10, NULL, NULL));
    EXPECT_FAIL(lrs_op_dual_update(NULL, 1.0));
    EXPECT_FAIL(lrs_op_alm_update(NULL, 1.0, 0.5, &dv, &dv));
    EXPECT_FAIL(lrs_op_adjoint(NULL, &dv, LRS_R, &dv, 1.0, 1));
    EXPECT_FAIL(lrs_op_auv(NULL, LRS_R, LRS_R, &dv, &dv));
    EXPECT_FAIL(lrs_op_dimacs(NULL, 0, &dv));
    EXPECT_FAIL(lrs_op_gram(NULL, 0, LRS_R, &dv));
    EXPECT_FAIL(lrs_op_dual_infeasibility(NULL, &dv, NULL));
    EXPECT_FAIL(lrs_solve(NULL, &p, &r));
    EXPECT_FAIL(lrs_trajectory(NULL, 1, NULL, NULL, 0));
    EXPECT_FAIL(lrs_write_json(NULL, "x.json", "id", "x.dat-s", &r, &p));
    EXPECT_FAIL(lrs_alm_throughput(NULL, &p, 0, 1, &dv, &lv, NULL, NULL));
    EXPECT_FAIL(lrs_set_budget_hook(NULL, NULL, NULL));
    EXPECT_FAIL(lrs_alm_last_step(NULL, &dv, &iv));
    EXPECT_FAIL(lrs_sync(NULL));
    EXPECT_FAIL(lrs_set_log_path(NULL, "x.log"));
    EXPECT_FAIL(lrs_set_kernel_path(NULL, 0));
    EXPECT_FAIL(lrs_get_kernel_path(NULL, &iv));
    EXPECT_FAIL(lrs_time_auut(NULL, 1, &dv));
    EXPECT_FAIL(lrs_auut_bytes(NULL, &dv));
    EXPECT_FAIL(lrs_time_gram(NULL, 0, 1, &dv, NULL));
    EXPECT_FAIL(lrs_mfma_f64_peak(NULL, &dv));
    EXPECT_FAIL(lrs_mfma_f64_probe(NULL, 2, 8, &dv, NULL, NULL));
    EXPECT_FAIL(lrs_time_dense(NULL, 0, 1, &dv));
    EXPECT_FAIL(lrs_profile_stages(NULL, &p, 1, &dv, &lv));
    EXPECT_FAIL(lrs_load_coo(NULL, 0, 0, NULL, NULL, 0, NULL, NULL, NULL, NULL, NULL));
    EXPECT_FAIL(lrs_tile_info(NULL, &iv, &iv));
    EXPECT_FAIL(lrs_tile_used(NULL, &iv));
    EXPECT_FAIL(lrs_stage_bytes(NULL, &dv));
    EXPECT_FAIL(lrs_time_stages(NULL, 1, &dv));
    EXPECT_FAIL(lrs_debug_phase_times(NULL, NULL, NULL));
    EXPECT_FAIL(lrs_shard_rccl(NULL, 1, 0, "id"));
    EXPECT_FAIL(lrs_shard_loopback(NULL, NULL, 0));
    EXPECT_FAIL(lrs_shard_info(NULL, &iv, &iv, &iv, &iv, &iv));
    EXPECT_FAIL(lrs_shard_comm_ranks(NULL, &iv));
    EXPECT_FAIL(lrs_ctx_create(0, NULL));
    EXPECT_FAIL(lrs_loopback_create(2, NULL));
    EXPECT_FAIL(lrs_comm_unique_id(NULL));
    EXPECT_FAIL(lrs_shard_plan(NULL, 2, 0, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL));
    lrs_ctx_destroy(NULL);
    lrs_loopback_destroy(NULL);
    lrs_params_default(NULL);
    if (strlen(lrs_last_error()) == 0) {
        fprintf(stderr, "no error message after a failed call\n");
        bad++;
    }
    printf("CAPI_NULL failures=%d last_error=\"%s\"\n", bad, lrs_last_error());
    return bad ? 1 : 0;
}

static int sweep(const char *path, int rank, const char *in_path, const char *out_path) {
    lrs_ctx *ctx = NULL;
    if (lrs_ctx_create(0, &ctx) != 0) { fprintf(stderr, "ctx: %s\n", lrs_last_error()); return 1; }
    int rc = 1, m = 0, K = 0;
    int *dims = NULL, *ranks = NULL, *its = NULL;
    double *buf = NULL, *rhs = NULL;
    FILE *f = NULL;
    if (lrs_load_sdpa(ctx, path, NULL) != 0) { fprintf(stderr, "load: %s\n", lrs_last_error()); goto done; }
    lrs_problem_info(ctx, &m, &K, NULL, NULL, NULL);
    dims = malloc(sizeof(int) * K);
    ranks = malloc(sizeof(int) * K);
    its = malloc(sizeof(int) * 2 * K);
    lrs_problem_info(ctx, &m, &K, dims, NULL, NULL);
    long NR = 0, nmax = 0;
    for (int k = 0; k < K; ++k) {
        ranks[k] = rank;
        NR += (long)dims[k] * rank;
        if ((long)dims[k] * rank > nmax) nmax = (long)dims[k] * rank;
    }
    if (lrs_set_rank(ctx, ranks) != 0) { fprintf(stderr, "rank: %s\n", lrs_last_error()); goto done; }
    const long nin = 2 * NR + m + 2;
    buf = malloc(sizeof(double) * nin);
    rhs = malloc(sizeof(double) * nmax);
    f = fopen(in_path, "rb");
    if (!f || fread(buf, sizeof(double), nin, f) != (size_t)nin) { fprintf(stderr, "read %s\n", in_path); goto done; }
    fclose(f);
    f = NULL;
    const double rho = buf[2 * NR + m], tol = buf[2 * NR + m + 1];
    if (lrs_factor_set(ctx, LRS_U, buf) || lrs_factor_set(ctx, LRS_V, buf + NR) ||
        lrs_vec_set(ctx, LRS_LAMBDA, buf + 2 * NR) || lrs_op_admm_constr(ctx)) {
        fprintf(stderr, "state: %s\n", lrs_last_error());
        goto done;
    }
    for (int k = 0; k < K; ++k)
        for (int side = 0; side < 2; ++side)
            if (lrs_op_admm_half(ctx, k, side, rho, tol, 800, &its[2 * k + side], rhs) != 0) {
                fprintf(stderr, "admm_half(%d, %d): %s\n", k, side, lrs_last_error());
                goto done;
            }
    if (lrs_op_admm_half(ctx, K, 0, rho, tol, 800, NULL, NULL) >= 0) { fprintf(stderr, "cone K accepted\n"); goto done; }
    if (lrs_op_admm_half(ctx, 0, 2, rho, tol, 800, NULL, NULL) >= 0) { fprintf(stderr, "side 2 accepted\n"); goto done; }
    if (lrs_op_dual_update(ctx, rho) != 0) { fprintf(stderr, "dual: %s\n", lrs_last_error()); goto done; }
    if (lrs_factor_get(ctx, LRS_U, buf) || lrs_factor_get(ctx, LRS_V, buf + NR) ||
        lrs_vec_get(ctx, LRS_LAMBDA, buf + 2 * NR)) {
        fprintf(stderr, "fetch: %s\n", lrs_last_error());
        goto done;
    }
    f = fopen(out_path, "wb");
    if (!f) goto done;
    fwrite(buf, sizeof(double), 2 * NR + m, f);
    for (int q = 0; q < 2 * K; ++q) {
        const double d = its[q];
        fwrite(&d, sizeof(double), 1, f);
    }
    printf("CAPI_SWEEP cones=%d m=%d cg", K, m);
    for (int q = 0; q < 2 * K; ++q) printf(" %d", its[q]);
    printf("\n");
    rc = 0;
done:
    if (f) fclose(f);
    free(dims); free(ranks); free(its); free(buf); free(rhs);
    lrs_ctx_destroy(ctx);
    return rc;
}

static int steps(const char *path, int rank, const char *in_path, const char *out_path, int ntrips) {
    lrs_ctx *ctx = NULL;
    if (lrs_ctx_create(0, &ctx) != 0) { fprintf(stderr, "ctx: %s\n", lrs_last_error()); return 1; }
    int rc = 1, m = 0, K = 0;
    int *dims = NULL, *ranks = NULL;
    double *buf = NULL, *trips = NULL;
    FILE *f = NULL;
    if (lrs_load_sdpa(ctx, path, NULL) != 0) { fprintf(stderr, "load: %s\n", lrs_last_error()); goto done; }
    lrs_problem_info(ctx, &m, &K, NULL, NULL, NULL);
    dims = malloc(sizeof(int) * K);
    ranks = malloc(sizeof(int) * K);
    lrs_problem_info(ctx, &m, &K, dims, NULL, NULL);
    long NR = 0;
    for (int k = 0; k < K; ++k) {
        ranks[k] = rank;
        NR += (long)dims[k] * rank;
    }
    if (lrs_set_rank(ctx, ranks) != 0) { fprintf(stderr, "rank: %s\n", lrs_last_error()); goto done; }
    const long nin = 4 * NR + 2 * m + 3;
    buf = malloc(sizeof(double) * (4 * NR + 2 * m + 1));
    trips = malloc(sizeof(double) * 4 * (ntrips > 0 ? ntrips : 1));
    double *in = malloc(sizeof(double) * nin);
    f = fopen(in_path, "rb");
    if (!in || !f || fread(in, sizeof(double), nin, f) != (size_t)nin) { fprintf(stderr, "read %s\n", in_path); free(in); goto done; }
    fclose(f);
    f = NULL;
    double beta_new = in[4 * NR + 2 * m], beta_old = 0.0;
    const double rho = in[4 * NR + 2 * m + 1];
    long clear = (long)in[4 * NR + 2 * m + 2];
    if (lrs_factor_set(ctx, LRS_R, in) || lrs_factor_set(ctx, LRS_G, in + NR) || lrs_factor_set(ctx, LRS_S0, in + 2 * NR) ||
        lrs_factor_set(ctx, LRS_Y0, in + 3 * NR) || lrs_vec_set(ctx, LRS_LAMBDA, in + 4 * NR) ||
        lrs_vec_set(ctx, LRS_CVS, in + 4 * NR + m)) {
        fprintf(stderr, "state: %s\n", lrs_last_error());
        free(in);
        goto done;
    }
    free(in);
    for (int t = 0; t < ntrips; ++t) {
        /* lorads_alm.c:1304-1309: the ring holds min(clearLBFGS, L = 2) pairs */
        const int nodes = clear < 2 ? (int)clear : 2;
        double tau = 0.0, lag = 0.0, beta = 0.0, dm[5];
        int rn = 0;
        if (lrs_op_lbfgs(ctx, nodes, beta_new, beta_old) || lrs_op_q12(ctx, NULL, NULL, NULL, NULL) ||
            lrs_op_line_search(ctx, rho, &tau, &rn)) {
            fprintf(stderr, "trip %d: %s\n", t, lrs_last_error());
            goto done;
        }
        trips[4 * t] = tau;
        trips[4 * t + 1] = rn;
        if (rn == 0) { fprintf(stderr, "trip %d: no root\n", t); goto done; }
        if (lrs_op_alm_update(ctx, rho, tau, &lag, &beta) || lrs_op_dimacs(ctx, 0, dm)) {
            fprintf(stderr, "trip %d: %s\n", t, lrs_last_error());
            goto done;
        }
        trips[4 * t + 2] = lag;
        trips[4 * t + 3] = dm[2];
        beta_old = beta_new;
        beta_new = beta;
        clear++;
        printf("CAPI_TRIP %d tau=%.17g root=%d lag=%.17g pinf=%.17g pobj=%.17g\n", t, tau, rn, lag, dm[2], dm[0]);
    }
    if (lrs_factor_get(ctx, LRS_R, buf) || lrs_factor_get(ctx, LRS_G, buf + NR) ||
        lrs_vec_get(ctx, LRS_CVS, buf + 2 * NR) || lrs_vec_get(ctx, LRS_LAMBDA, buf + 2 * NR + m) ||
        lrs_factor_get(ctx, LRS_S0, buf + 2 * NR + 2 * m) || lrs_factor_get(ctx, LRS_Y0, buf + 3 * NR + 2 * m)) {
        fprintf(stderr, "fetch: %s\n", lrs_last_error());
        goto done;
    }
    buf[4 * NR + 2 * m] = beta_new;
    f = fopen(out_path, "wb");
    if (!f) goto done;
    fwrite(trips, sizeof(double), 4 * ntrips, f);
    fwrite(buf, sizeof(double), 4 * NR + 2 * m + 1, f);
    rc = 0;
done:
    if (f) fclose(f);
    free(dims); free(ranks); free(buf); free(trips);
    lrs_ctx_destroy(ctx);
    return rc;
}

int main(int argc, char **argv) {
    if (argc >= 2 && !strcmp(argv[1], "--null")) return null_contract();
    if (argc >= 6 && !strcmp(argv[1], "--sweep")) return sweep(argv[2], atoi(argv[3]), argv[4], argv[5]);
    if (argc >= 7 && !strcmp(argv[1], "--steps")) return steps(argv[2], atoi(argv[3]), argv[4], argv[5], atoi(argv[6]));
    if (argc < 3) {
        fprintf(stderr, "usage: %s <file.dat-s> <out.json> [reoptLevel] | --null | --sweep ...\n", argv[0]);
        return 2;
    }
    lrs_params p;
    lrs_params_default(&p);
    if (argc > 3) p.reoptLevel = atoi(argv[3]);
    lrs_ctx *ctx = NULL;
    if (lrs_ctx_create(0, &ctx) != 0) {
        fprintf(stderr, "ctx: %s\n", lrs_last_error());
        return 1;
    }
    double tread = 0.0;
    if (lrs_load_sdpa(ctx, argv[1], &tread) != 0) {
        fprintf(stderr, "load: %s\n", lrs_last_error());
        lrs_ctx_destroy(ctx);
        return 1;
    }
    int m = 0, ncones = 0;
    lrs_problem_info(ctx, &m, &ncones, NULL, NULL, NULL);
    lrs_result r;
    if (lrs_solve(ctx, &p, &r) != 0) {
        fprintf(stderr, "solve: %s\n", lrs_last_error());
        lrs_ctx_destroy(ctx);
        return 1;
    }
    if (lrs_write_json(ctx, argv[2], "capi", argv[1], &r, &p) != 0) {
        fprintf(stderr, "json: %s\n", lrs_last_error());
        lrs_ctx_destroy(ctx);
        return 1;
    }
    printf("CAPI m=%d cones=%d alm_inner=%ld admm_iter=%ld pobj=%.17g dobj=%.17g pinf=%.6e gap=%.6e status=%d rank=%d\n",
           m, ncones, r.alm_inner, r.admm_iter, r.pobj, r.dobj, r.pinf, r.gap, r.status, r.final_rank);
    lrs_ctx_destroy(ctx);
    return 0;
}
