/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY (never shipped, never linked
 * into the product).  Our own driver, linked against the reference LoRADS
 * objects built by oracle/Makefile.ref, used to produce golden fixtures that pin
 * the CPU restatement (oracle/lrsdp_oracle.c) and, on the GPU box, to time the
 * real reference CPU path for bench.py's cpu_baseline.
 *
 * Modes
 *   solve   <file.dat-s> [--flag value ...]
 *       The init sequence of main.c:380-418, then LORADS_ALMOptimize
 *       (main.c:450), LORADS_ALMtoADMM + LORADSADMMOptimize (main.c:456-457)
 *       and the reoptLevel>=1 loop (main.c:491-513).  The ARPACK dual
 *       infeasibility (main.c:515) is skipped (ARPACK is not in the image).
 *       Prints "REF_RESULT ..." lines and writes --jsonfile like
 *       lorads_logging.c:618.
 *   alm_rate <file.dat-s> <rank> <iters>
 *       Runs phase 1 at --fixedRank <rank> for a bounded number of ALM inner
 *       iterations (maxALMIter large, phase1Tol tiny) and prints the rate.
 *   kernels <file.dat-s> <rank> <in.bin> <out.bin>
 *       One call of each hot-path operator on caller-provided iterates (see
 *       scripts/make_golden.py for the exact binary layout).
 *   alm_steps <file.dat-s> <rank> <K[,K2,...]> <out.bin> [--flag value ...]
 *       From the reference's own initial point (srand(925), data/lorads_solver.c:625)
 *       the preamble of LORADS_ALMOptimize (lorads_alm.c:1233-1243) and exactly K
 *       trips of its inner L-BFGS loop (lorads_alm.c:1302-1379), through the same
 *       lorads_func slots in the same order; dumps per trip (tau, rootNum,
 *       ||G||^2, pinf) and after the last one R, G, A(RR^T), lambda and the newest
 *       L-BFGS pair (s, y, beta).  Layout in scripts/make_golden_steps.py.
 *       With a comma list of K (ascending) one run dumps the state at each K into
 *       <out.bin>.K<k>, at the point a stand-alone run with that K stops (so a
 *       C5-sized presolve is paid once).
 *   admm_sweep <file.dat-s> <rank> <in.bin> <out.bin>
 *       One ADMM variable update over every cone (LORADSUpdateSDPVar) and the dual
 *       update after it (LORADSUpdateDualVar) on the `kernels` inputs' U, V, lambda
 *       (scripts/make_golden_admm.py).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <getopt.h>
#include <sys/time.h>

#include "lorads_file_io.h"
#include "def_lorads_user_data.h"
#include "lorads_user_data.h"
#include "lorads_utils.h"
#include "def_lorads_solver.h"
#include "lorads_solver.h"
#include "lorads_alm.h"
#include "lorads_admm.h"
#include "lorads_alg_common.h"
#include "lorads_logging.h"
#include "lorads_cgs.h"

extern int MAX_ALM_SUB_ITER;

static double now_s(void) {
    struct timeval tv; gettimeofday(&tv, NULL);
    return tv.tv_sec + 1e-6 * tv.tv_usec;
}

static void default_params(lorads_params *p) {
    memset(p, 0, sizeof(*p));
    p->fname = "NULL"; p->logFile = NULL; p->jsonFile = NULL;
    p->initRho = 0.0; p->rhoMax = 5000.0; p->rhoCellingALM = 1e8;
    p->rhoCellingADMM = 5000.0 * 200; p->maxALMIter = 200; p->maxADMMIter = 10000;
    p->timesLogRank = 2.0; p->fixedRank = -1; p->initRank = -1; p->rhoFreq = 5;
    p->rhoFactor = 1.2; p->ALMRhoFactor = 2.0; p->rankUpdateFactor = 1.5;
    p->phase1Tol = 1e-3; p->phase2Tol = 1e-5; p->timeSecLimit = 3600.0;
    p->heuristicFactor = 1.0; p->lbfgsListLength = 2; p->endTauTol = 1e-16;
    p->endALMSubTol = 1e-10; p->l2Rescaling = false; p->reoptLevel = 2;
    p->dyrankLevel = 2; p->highAccMode = false;
    p->oracleRankMethod = LORADS_ORACLE_RANK_GRAM;
}

static struct option long_opts[] = {
    {"logfile", required_argument, 0, 1025}, {"jsonfile", required_argument, 0, 1026},
    {"initRho", required_argument, 0, 1000}, {"rhoMax", required_argument, 0, 1001},
    {"rhoCellingALM", required_argument, 0, 1002}, {"rhoCellingADMM", required_argument, 0, 1003},
    {"maxALMIter", required_argument, 0, 1004}, {"maxADMMIter", required_argument, 0, 1005},
    {"timesLogRank", required_argument, 0, 1006}, {"fixedRank", required_argument, 0, 1022},
    {"initRank", required_argument, 0, 1023}, {"rhoFreq", required_argument, 0, 1007},
    {"rhoFactor", required_argument, 0, 1008}, {"ALMRhoFactor", required_argument, 0, 1009},
    {"rankUpdateFactor", required_argument, 0, 1024}, {"phase1Tol", required_argument, 0, 1010},
    {"phase2Tol", required_argument, 0, 1011}, {"timeSecLimit", required_argument, 0, 1012},
    {"heuristicFactor", required_argument, 0, 1013}, {"lbfgsListLength", required_argument, 0, 1014},
    {"endTauTol", required_argument, 0, 1015}, {"endALMSubTol", required_argument, 0, 1016},
    {"l2Rescaling", required_argument, 0, 1017}, {"reoptLevel", required_argument, 0, 1018},
    {"dyrankLevel", required_argument, 0, 1019}, {"highAccMode", required_argument, 0, 1020},
    {"oracleRankNaive", no_argument, 0, 1021}, {0, 0, 0, 0}};

static void parse_flags(lorads_params *p, int argc, char **argv) {
    int opt, li = 0;
    optind = 1;
    while ((opt = getopt_long(argc, argv, "r:", long_opts, &li)) != -1) {
        switch (opt) {
        case 1025: p->logFile = optarg; break;          case 1026: p->jsonFile = optarg; break;
        case 1000: p->initRho = atof(optarg); break;    case 1001: p->rhoMax = atof(optarg); break;
        case 1002: p->rhoCellingALM = atof(optarg); break;
        case 1003: p->rhoCellingADMM = atof(optarg); break;
        case 1004: p->maxALMIter = atoi(optarg); break; case 1005: p->maxADMMIter = atoi(optarg); break;
        case 1006: p->timesLogRank = atof(optarg); break;
        case 1022: p->fixedRank = atoi(optarg); break;  case 1023: p->initRank = atoi(optarg); break;
        case 1007: p->rhoFreq = atoi(optarg); break;    case 1008: p->rhoFactor = atof(optarg); break;
        case 1009: p->ALMRhoFactor = atof(optarg); break;
        case 1024: p->rankUpdateFactor = atof(optarg); break;
        case 1010: p->phase1Tol = atof(optarg); break;  case 1011: p->phase2Tol = atof(optarg); break;
        case 1012: p->timeSecLimit = atof(optarg); break;
        case 1013: p->heuristicFactor = atof(optarg); break;
        case 1014: p->lbfgsListLength = atoi(optarg); break;
        case 1015: p->endTauTol = atof(optarg); break;  case 1016: p->endALMSubTol = atof(optarg); break;
        case 1017: p->l2Rescaling = atoi(optarg); break; case 1018: p->reoptLevel = atoi(optarg); break;
        case 1019: p->dyrankLevel = atoi(optarg); break; case 1020: p->highAccMode = atoi(optarg); break;
        case 1021: p->oracleRankMethod = LORADS_ORACLE_RANK_NAIVE; break;
        default: break;
        }
    }
    p->rhoCellingADMM = p->rhoMax * 200;   /* main.c:350 */
}

typedef struct {
    lorads_solver *S;
    lorads_int nConstrs, nBlks, *BlkDims, nLpCols;
    lorads_int **coneMatBeg, **coneMatIdx; double **coneMatElem, *rowRHS;
    lorads_int *LpMatBeg, *LpMatIdx; double *LpMatElem;
    user_data **SDPDatas;
    lorads_alm_state alm; lorads_admm_state admm; SDPConst sc;
} ref_ctx;

/* main.c:380-419 */
static int ref_setup(ref_ctx *c, lorads_params *p, double *t_read, double *t_solve_start) {
    lorads_int nCols = 0, nElem = 0;
    double t0 = now_s();
    if (LReadSDPA(p->fname, &c->nConstrs, &c->nBlks, &c->BlkDims, &c->rowRHS, &c->coneMatBeg,
                  &c->coneMatIdx, &c->coneMatElem, &nCols, &c->nLpCols, &c->LpMatBeg,
                  &c->LpMatIdx, &c->LpMatElem, &nElem) != LORADS_RETCODE_OK)
        return -1;
    *t_read = now_s() - t0;
    *t_solve_start = now_s();
    LORADS_INIT(c->S, lorads_solver, 1);
    LORADS_INIT(c->S->var, lorads_variable, 1);
    LORADSInitSolver(c->S, c->nConstrs, c->nBlks, c->BlkDims, c->nLpCols);
    LORADS_INIT(c->SDPDatas, user_data *, c->nBlks);
    LORADSSetDualObjective(c->S, c->rowRHS);
    LORADSInitConeData(c->S, c->SDPDatas, c->coneMatElem, c->coneMatBeg, c->coneMatIdx, c->BlkDims,
                       c->nConstrs, c->nBlks, c->nLpCols, c->LpMatBeg, c->LpMatIdx, c->LpMatElem);
    LORADSPreprocess(c->S, c->BlkDims);
    LORADSDetermineRank(c->S, c->BlkDims, p->timesLogRank, p->fixedRank, p->initRank);
    LORADSInitALMVars(c->S, c->S->var->rankElem, c->BlkDims, c->nBlks, c->nLpCols, p->lbfgsListLength);
    c->S->hisRecT = p->lbfgsListLength;
    LORADSInitADMMVars(c->S, c->S->var->rankElem, c->BlkDims, c->nBlks, c->nLpCols);
    initial_solver_state(p, c->S, &c->alm, &c->admm, &c->sc);
    lorads_logging_init(c->S, p, *t_solve_start);
    return 0;
}

static int mode_solve(int argc, char **argv) {
    lorads_params p; default_params(&p);
    p.fname = argv[2];
    parse_flags(&p, argc - 2, argv + 2);
    ref_ctx c; memset(&c, 0, sizeof(c));
    double t_read, tss;
    if (ref_setup(&c, &p, &t_read, &tss)) { printf("REF_RESULT read_failed\n"); return 0; }
    lorads_solver *S = c.S;
    double all_time = 0.0;
    int bad = 0;
    double ts = now_s();
    double t_alm0 = now_s();
    LORADS_ALMOptimize(&p, S, &c.alm, p.maxALMIter, tss);
    double t_alm = now_s() - t_alm0;
    long alm_inner = (long)c.alm.innerIter;
    if (now_s() - tss > p.timeSecLimit) goto END;
    LORADS_ALMtoADMM(S, &p, &c.alm, &c.admm);
    if (LORADSADMMOptimize(&p, S, &c.admm, p.maxADMMIter, tss) == RET_CODE_BAD_ITER) bad = 1;
    all_time += now_s() - ts;
    if (p.reoptLevel >= 1) {
        double rp = 5; lorads_int ai = 3, di = 50;
        int cnt = 0;
        while ((c.alm.primal_dual_gap > p.phase2Tol || c.alm.l_1_primal_infeasibility > p.phase2Tol) &&
               (c.admm.primal_dual_gap > p.phase2Tol || c.admm.l_1_primal_infeasibility > p.phase2Tol)) {
            if (cnt >= 1) break;
            double t1 = now_s();
            reopt(&p, S, &c.alm, &c.admm, &rp, &ai, &di, tss, &bad, 1);
            all_time += now_s() - t1;
            cnt++;
            if (now_s() - tss > p.timeSecLimit) break;
        }
    }
END:;
    /* main.c:519-525 (the dual-infeasibility value itself needs ARPACK and is not computed) */
    c.admm.primal_dual_gap = S->dimacError[LORADS_DIMAC_ERROR_PDGAP];
    c.admm.l_1_primal_infeasibility = S->dimacError[LORADS_DIMAC_ERROR_CONSTRVIO_L1];
    c.admm.l_inf_primal_infeasibility = S->dimacError[LORADS_DIMAC_ERROR_CONSTRVIO_L1] * (1 + S->bRHSNrm1) / (1 + S->bRHSNrmInf);
    lorads_int orank = lorads_compute_oracle_rank(S, 2);
    if (orank < 0) orank = 0;
    lorads_write_json_output(S, orank, c.admm.primal_objective_value, c.admm.dual_objective_value,
                             c.admm.l_1_primal_infeasibility, c.admm.l_inf_primal_infeasibility,
                             c.admm.primal_dual_gap, all_time, p.rhoMax, p.heuristicFactor);
    lorads_logging_close(S);
    /* REF_DUMP=<file>: the final iterate for a device-side check (tests/test_tight_objectives.py):
       doubles {K, rank_0..rank_{K-1}, R_0..R_{K-1} (column-major n_k x rank_k), m, lambda[m]} */
    const char *dump = getenv("REF_DUMP");
    if (dump) {
        FILE *fd = fopen(dump, "wb");
        if (fd) {
            /* an LP block: one more "cone" of rank 1 holding r (the device's layout) */
            const int lp = S->nLpCols > 0;
            double v = (double)(S->nCones + lp);
            fwrite(&v, 8, 1, fd);
            for (lorads_int k = 0; k < S->nCones; ++k) { v = (double)S->var->R[k]->rank; fwrite(&v, 8, 1, fd); }
            if (lp) { v = 1.0; fwrite(&v, 8, 1, fd); }
            for (lorads_int k = 0; k < S->nCones; ++k)
                fwrite(S->var->R[k]->matElem, 8, (size_t)S->var->R[k]->nRows * S->var->R[k]->rank, fd);
            if (lp) fwrite(S->var->rLp->matElem, 8, (size_t)S->nLpCols, fd);
            v = (double)S->nRows;
            fwrite(&v, 8, 1, fd);
            fwrite(S->var->dualVar, 8, (size_t)S->nRows, fd);
            fclose(fd);
        }
    }
    printf("REF_RESULT alm_inner=%ld alm_outer=%ld alm_time=%.9e alm_pobj=%.17e alm_dobj=%.17e "
           "alm_pinf=%.17e alm_gap=%.17e alm_rho=%.17e\n",
           alm_inner, (long)c.alm.outerIter, t_alm, c.alm.primal_objective_value,
           c.alm.dual_objective_value, c.alm.l_1_primal_infeasibility, c.alm.primal_dual_gap, c.alm.rho);
    printf("REF_RESULT admm_iter=%ld admm_pobj=%.17e admm_dobj=%.17e admm_pinf=%.17e admm_gap=%.17e "
           "admm_rho=%.17e solve_time=%.9e read_time=%.9e rank=%ld\n",
           (long)c.admm.iter, c.admm.primal_objective_value, c.admm.dual_objective_value,
           c.admm.l_1_primal_infeasibility, c.admm.primal_dual_gap, c.admm.rho, all_time, t_read,
           (long)S->var->R[0]->rank);
    fflush(stdout);
    return 0;
}

/* Bounded phase-1 timing: ALM inner iterations / phase-1 wall time at fixed rank. */
static int mode_alm_rate(int argc, char **argv) {
    lorads_params p; default_params(&p);
    p.fname = argv[2];
    p.fixedRank = atoi(argv[3]);
    long iters = atol(argv[4]);
    p.phase1Tol = 1e-300;           /* never satisfied: keep iterating */
    p.maxALMIter = 100000;
    p.timeSecLimit = argc > 5 ? atof(argv[5]) : 30.0;  /* wall budget (the sample bound) */
    p.reoptLevel = 0;
    ref_ctx c; memset(&c, 0, sizeof(c));
    double t_read, tss;
    if (ref_setup(&c, &p, &t_read, &tss)) { printf("REF_RATE read_failed\n"); return 0; }
    (void)iters;
    double t0 = now_s();
    LORADS_ALMOptimize(&p, c.S, &c.alm, p.maxALMIter, t0);
    double dt = now_s() - t0;
    printf("REF_RATE inner=%ld seconds=%.9e rate=%.9e rank=%ld\n", (long)c.alm.innerIter, dt,
           c.alm.innerIter / dt, (long)c.S->var->R[0]->rank);
    return 0;
}

/* ---------------- kernels mode: one call of each hot-path operator ---------------- */
static void col_copy(double *dst, const double **src, lorads_int len) {
    memcpy(dst, *src, sizeof(double) * len); *src += len;
}

static int mode_kernels(int argc, char **argv) {
    lorads_params p; default_params(&p);
    p.fname = argv[2];
    p.fixedRank = atoi(argv[3]);
    ref_ctx c; memset(&c, 0, sizeof(c));
    double t_read, tss;
    if (ref_setup(&c, &p, &t_read, &tss)) { fprintf(stderr, "read failed\n"); return 1; }
    lorads_solver *S = c.S;
    lorads_int m = S->nRows, K = S->nCones, NR = 0;
    for (lorads_int k = 0; k < K; ++k) NR += S->var->R[k]->nRows * S->var->R[k]->rank;
    FILE *fi = fopen(argv[4], "rb");
    if (!fi) return 1;
    fseek(fi, 0, SEEK_END); long sz = ftell(fi); fseek(fi, 0, SEEK_SET);
    double *in = malloc(sz); if (fread(in, 1, sz, fi) != (size_t)sz) return 1; fclose(fi);
    const double *ip = in;
    /* layout: R, D, G, s1, y1, s2, y2, U, V (each NR, col-major per cone, cones concatenated),
               lambda[m], cvs[m], rho, beta1, beta2, rho_admm, cg_tol */
    double *R = malloc(8 * NR), *D = malloc(8 * NR), *G = malloc(8 * NR), *s1 = malloc(8 * NR),
           *y1 = malloc(8 * NR), *s2 = malloc(8 * NR), *y2 = malloc(8 * NR), *U = malloc(8 * NR),
           *V = malloc(8 * NR);
    col_copy(R, &ip, NR); col_copy(D, &ip, NR); col_copy(G, &ip, NR); col_copy(s1, &ip, NR);
    col_copy(y1, &ip, NR); col_copy(s2, &ip, NR); col_copy(y2, &ip, NR); col_copy(U, &ip, NR);
    col_copy(V, &ip, NR);
    double *lam = malloc(8 * m), *cvs = malloc(8 * m);
    col_copy(lam, &ip, m); col_copy(cvs, &ip, m);
    double rho = *ip++, beta1 = *ip++, beta2 = *ip++, rho_admm = *ip++, cg_tol = *ip++;

    FILE *fo = fopen(argv[5], "wb");
    lorads_int off;
#define LOAD(dstArr, src) do { off = 0; for (lorads_int k = 0; k < K; ++k) { \
        lorads_int len = dstArr[k]->nRows * dstArr[k]->rank; \
        memcpy(dstArr[k]->matElem, (src) + off, 8 * len); off += len; } } while (0)
#define DUMPF(arr) do { off = 0; for (lorads_int k = 0; k < K; ++k) { \
        lorads_int len = arr[k]->nRows * arr[k]->rank; \
        fwrite(arr[k]->matElem, 8, len, fo); off += len; } } while (0)

    /* (1) q1 = 2 A(sym(R D^T)), p1 = 2 <C, sym(R D^T)>, q2 = A(D D^T), p2 = <C, D D^T>
           via ALMCalq12p12 (lorads_alm.c:714) */
    LOAD(S->var->R, R);
    LOAD(S->var->U, D);
    double p12[2];
    ALMCalq12p12(S, S->var->rLp, S->var->uLp, S->var->R, S->var->U, S->var->ARDSum, S->var->ADDSum, p12);
    fwrite(S->var->ARDSum, 8, m, fo); fwrite(&p12[0], 8, 1, fo);
    fwrite(S->var->ADDSum, 8, m, fo); fwrite(&p12[1], 8, 1, fo);
    /* (2) A(R R^T) from scratch + pinf (primalInfeasibility, alg_common.c:386) and <C, R R^T> */
    S->pObjVal = 0.0; S->dObjVal = 0.0;
    primalInfeasibility(S, S->var->R, S->var->R, S->var->rLp, S->var->rLp);
    fwrite(S->var->constrValSum, 8, m, fo);
    fwrite(&S->dimacError[LORADS_DIMAC_ERROR_CONSTRVIO_L1], 8, 1, fo);
    LORADSCalObjRR_ALM(S);
    fwrite(&S->pObjVal, 8, 1, fo);
    /* (3) gradient G = 2 (C + A^*(rho (cvs - b) - lambda)) R  (ALMCalGrad, lorads_alm.c:74) */
    memcpy(S->var->dualVar, lam, 8 * m);
    memcpy(S->var->constrValSum, cvs, 8 * m);
    double lag = 0.0;
    ALMCalGrad(S, S->var->rLp, S->var->gradLp, S->var->R, S->var->Grad, &lag, rho);
    DUMPF(S->var->Grad); fwrite(&lag, 8, 1, fo);
    /* (4) line search on (q0 = b - cvs, q1, q2, p1, p2)  (ALMLineSearch, lorads_alm.c:266) */
    {
        /* recompute q1,q2 for (R,D) since (2) overwrote constrVal */
        LOAD(S->var->R, R); LOAD(S->var->U, D);
        ALMCalq12p12(S, S->var->rLp, S->var->uLp, S->var->R, S->var->U, S->var->ARDSum, S->var->ADDSum, p12);
        double *q0 = malloc(8 * m);
        for (lorads_int i = 0; i < m; ++i) q0[i] = S->rowRHS[i] - cvs[i];
        double tau = 0.0;
        lorads_int rn = ALMLineSearch(rho, m, lam, p12[0], p12[1], q0, S->var->ARDSum, S->var->ADDSum, &tau);
        double rnd = (double)rn;
        fwrite(&tau, 8, 1, fo); fwrite(&rnd, 8, 1, fo);
        free(q0);
    }
    /* (5) L-BFGS two-loop with 2 pairs (LBFGSDirection, lorads_alm.c:468-505):
           newest pair = (s1, y1, beta1), older = (s2, y2, beta2) */
    {
        LOAD(S->var->Grad, G);
        lbfgs_node *head = S->lbfgsHis;          /* next slot to write  */
        lbfgs_node *newest = head->prev, *older = newest->prev;
        memcpy(newest->s, s1, 8 * NR); memcpy(newest->y, y1, 8 * NR); newest->beta = beta1;
        memcpy(older->s, s2, 8 * NR); memcpy(older->y, y2, 8 * NR); older->beta = beta2;
        LBFGSDirection(&p, S, head, S->var->gradLp, S->var->uLp, S->var->Grad, S->var->U, 5);
        LBFGSDirectionUseGrad(S, S->var->uLp, S->var->gradLp, S->var->U, S->var->Grad);
        DUMPF(S->var->U);
        LBFGSDirection(&p, S, head, S->var->gradLp, S->var->uLp, S->var->Grad, S->var->U, 1);
        LBFGSDirectionUseGrad(S, S->var->uLp, S->var->gradLp, S->var->U, S->var->Grad);
        DUMPF(S->var->U);
    }
    /* (6) one ADMM half-step: solve for U with V fixed (LORADSUpdateSDPVarOne,
           lorads_admm.c:564), state A(UV^T) from (U, V), dual = lambda */
    {
        LOAD(S->var->U, U); LOAD(S->var->V, V);
        memcpy(S->var->dualVar, lam, 8 * m);
        LORADSInitConstrValAll(S, S->var->uLp, S->var->vLp, S->var->U, S->var->V);
        LORADSInitConstrValSum(S);
        S->cgIter = 0;
        LORADSUpdateSDPVarOne(S, S->var->U[0], S->var->V[0], 0, rho_admm, cg_tol, 800);
        DUMPF(S->var->U);
        fwrite(S->var->bLinSys[0], 8, S->var->U[0]->nRows * S->var->U[0]->rank, fo);
        double it = (double)S->CGLinsys[0]->iter;
        fwrite(&it, 8, 1, fo);
    }
    fclose(fo);
    return 0;
}

/* ---------------- admm_sweep mode: one ADMM variable update over every cone ----------------
 * Same input file as `kernels`.  State: U, V, lambda; constraint values from (U, V)
 * (LORADSInitConstrValAll + Sum); then LORADSUpdateSDPVar (lorads_alg_common.c:298-326: per
 * cone U with V fixed, refresh, V with U fixed, refresh) at rho_admm, cg_tol, 800 iterations,
 * then LORADSUpdateDualVar (:511-524) at rho_admm.  Dump: U, V (all cones), constrValSum[m],
 * dualVar[m], total CG iterations, per cone the last (V-side) CG iteration count. */
static int mode_admm_sweep(int argc, char **argv) {
    if (argc < 6) return 2;
    lorads_params p; default_params(&p);
    p.fname = argv[2];
    p.fixedRank = atoi(argv[3]);
    ref_ctx c; memset(&c, 0, sizeof(c));
    double t_read, tss;
    if (ref_setup(&c, &p, &t_read, &tss)) { fprintf(stderr, "read failed\n"); return 1; }
    lorads_solver *S = c.S;
    lorads_int m = S->nRows, K = S->nCones, NR = 0;
    for (lorads_int k = 0; k < K; ++k) NR += S->var->R[k]->nRows * S->var->R[k]->rank;
    FILE *fi = fopen(argv[4], "rb");
    if (!fi) return 1;
    fseek(fi, 0, SEEK_END); long sz = ftell(fi); fseek(fi, 0, SEEK_SET);
    double *in = malloc(sz); if (fread(in, 1, sz, fi) != (size_t)sz) return 1; fclose(fi);
    const double *U = in + 7 * NR, *V = in + 8 * NR, *lam = in + 9 * NR;
    const double *tail = in + 9 * NR + 2 * m;
    const double rho_admm = tail[3], cg_tol = tail[4];
    lorads_int off;
    LOAD(S->var->U, U); LOAD(S->var->V, V);
    memcpy(S->var->dualVar, lam, 8 * m);
    LORADSInitConstrValAll(S, S->var->uLp, S->var->vLp, S->var->U, S->var->V);
    LORADSInitConstrValSum(S);
    S->cgIter = 0;
    LORADSUpdateSDPVar(S, rho_admm, cg_tol, 800);
    LORADSUpdateDualVar(S, rho_admm);
    FILE *fo = fopen(argv[5], "wb");
    if (!fo) return 1;
    DUMPF(S->var->U);
    DUMPF(S->var->V);
    fwrite(S->var->constrValSum, 8, m, fo);
    fwrite(S->var->dualVar, 8, m, fo);
    double it = (double)S->cgIter;
    fwrite(&it, 8, 1, fo);
    for (lorads_int k = 0; k < K; ++k) { it = (double)S->CGLinsys[k]->iter; fwrite(&it, 8, 1, fo); }
    fclose(fo);
    free(in);
    printf("REF_ADMM_SWEEP cg=%ld\n", (long)S->cgIter);
    return 0;
}

/* ---------------- alm_steps mode: K inner iterations, per-iteration dump ---------------- */
static int steps_dump(lorads_solver *S, const double *trips, long done, const char *out, long K) {
    char path[4096];
    if (K >= 0) snprintf(path, sizeof(path), "%s.K%ld", out, K);
    else snprintf(path, sizeof(path), "%s", out);
    FILE *fo = fopen(path, "wb");
    if (!fo) return 1;
    lorads_int m = S->nRows;
    double dd = (double)done;
    fwrite(&dd, 8, 1, fo);
    fwrite(trips, 8, 4 * done, fo);
    /* an LP block's r and gradient follow the SDP cones' (the device appends the LP block as the
       last cone at rank 1; the L-BFGS pairs hold the LP part last too, setlbfgsHisTwoLP) */
    for (lorads_int k = 0; k < S->nCones; ++k)
        fwrite(S->var->R[k]->matElem, 8, S->var->R[k]->nRows * S->var->R[k]->rank, fo);
    if (S->nLpCols > 0) fwrite(S->var->rLp->matElem, 8, S->nLpCols, fo);
    for (lorads_int k = 0; k < S->nCones; ++k)
        fwrite(S->var->Grad[k]->matElem, 8, S->var->Grad[k]->nRows * S->var->Grad[k]->rank, fo);
    if (S->nLpCols > 0) fwrite(S->var->gradLp->matElem, 8, S->nLpCols, fo);
    fwrite(S->var->constrValSum, 8, m, fo);
    fwrite(S->var->dualVar, 8, m, fo);
    lbfgs_node *newest = S->lbfgsHis->prev;
    fwrite(newest->s, 8, newest->allElem, fo);
    fwrite(newest->y, 8, newest->allElem, fo);
    fwrite(&newest->beta, 8, 1, fo);
    fclose(fo);
    printf("REF_STEPS_DUMP K=%ld done=%ld\n", K, done);
    fflush(stdout);
    return 0;
}

/* admm_sweep_lp <file> <rank> <in> <out>: the ADMM sweep of a problem with an LP block
 * (LORADSUpdateSDPLPVar, lorads_alg_common.c:352-372: every SDP cone's U / V half-steps, then per
 * LP column LORADSUpdateLPVarOne for u_j and v_j, lorads_admm.c:759-792) and the dual update, on
 * given U, V, lambda.  Input doubles: U, V (SDP cones column-major, then the LP block's nLpCols
 * values: the device's LP cone at rank 1), lambda[m], rho_admm, cg_tol.  Dump: U, V (same
 * layout), constrValSum[m], dualVar[m], total CG iterations. */
static int mode_admm_sweep_lp(int argc, char **argv) {
    if (argc < 6) return 2;
    lorads_params p; default_params(&p);
    p.fname = argv[2];
    p.fixedRank = atoi(argv[3]);
    ref_ctx c; memset(&c, 0, sizeof(c));
    double t_read, tss;
    if (ref_setup(&c, &p, &t_read, &tss)) { fprintf(stderr, "read failed\n"); return 1; }
    lorads_solver *S = c.S;
    lorads_int m = S->nRows, K = S->nCones, NR = 0, nlp = S->nLpCols;
    for (lorads_int k = 0; k < K; ++k) NR += S->var->R[k]->nRows * S->var->R[k]->rank;
    const lorads_int NA = NR + nlp;
    FILE *fi = fopen(argv[4], "rb");
    if (!fi) return 1;
    fseek(fi, 0, SEEK_END); long sz = ftell(fi); fseek(fi, 0, SEEK_SET);
    double *in = malloc(sz); if (fread(in, 1, sz, fi) != (size_t)sz) return 1; fclose(fi);
    if (sz != (long)(8 * (2 * NA + m + 2))) { fprintf(stderr, "input size %ld, expected %ld\n", sz, (long)(8 * (2 * NA + m + 2))); return 1; }
    const double *U = in, *V = in + NA, *lam = in + 2 * NA;
    const double rho_admm = in[2 * NA + m], cg_tol = in[2 * NA + m + 1];
    lorads_int off;
    LOAD(S->var->U, U); LOAD(S->var->V, V);
    if (nlp > 0) { memcpy(S->var->uLp->matElem, U + NR, 8 * nlp); memcpy(S->var->vLp->matElem, V + NR, 8 * nlp); }
    memcpy(S->var->dualVar, lam, 8 * m);
    if (nlp > 0) {
        LORADSInitConstrValAllLP(S, S->var->uLp, S->var->vLp, S->var->U, S->var->V);
        LORADSInitConstrValSumLP(S);
    } else {
        LORADSInitConstrValAll(S, S->var->uLp, S->var->vLp, S->var->U, S->var->V);
        LORADSInitConstrValSum(S);
    }
    S->cgIter = 0;
    if (nlp > 0) LORADSUpdateSDPLPVar(S, rho_admm, cg_tol, 800);
    else LORADSUpdateSDPVar(S, rho_admm, cg_tol, 800);
    LORADSUpdateDualVar(S, rho_admm);
    FILE *fo = fopen(argv[5], "wb");
    if (!fo) return 1;
    DUMPF(S->var->U);
    if (nlp > 0) fwrite(S->var->uLp->matElem, 8, nlp, fo);
    DUMPF(S->var->V);
    if (nlp > 0) fwrite(S->var->vLp->matElem, 8, nlp, fo);
    fwrite(S->var->constrValSum, 8, m, fo);
    fwrite(S->var->dualVar, 8, m, fo);
    double it = (double)S->cgIter;
    fwrite(&it, 8, 1, fo);
    fclose(fo);
    free(in);
    printf("REF_ADMM_SWEEP_LP cg=%ld\n", (long)S->cgIter);
    return 0;
}

static int mode_alm_steps(int argc, char **argv) {
    if (argc < 6) return 2;
    lorads_params p; default_params(&p);
    p.fname = argv[2];
    if (argc > 6) parse_flags(&p, argc - 5, argv + 5);   /* trailing --flag value pairs */
    p.fixedRank = atoi(argv[3]);
    long Ks[64]; int nK = 0;
    for (char *tok = strtok(argv[4], ","); tok && nK < 64; tok = strtok(NULL, ",")) Ks[nK++] = atol(tok);
    const long K = nK ? Ks[nK - 1] : 0;
    const int multi = nK > 1;
    int nextK = 0;
    ref_ctx c; memset(&c, 0, sizeof(c));
    double t_read, tss;
    if (ref_setup(&c, &p, &t_read, &tss)) { fprintf(stderr, "read failed\n"); return 1; }
    lorads_solver *S = c.S;
    lorads_alm_state *st = &c.alm;
    lorads_func *aFunc;
    LORADSInitFuncSet(&aFunc, S->nLpCols);
    lorads_int incx = 1, m = S->nRows;
    double minusOne = -1.0, tau = 0.0, lagNormSquare = 0.0;
    /* lorads_alm.c:1233-1243 */
    double rc_tol = 0.1 / st->rho;
    aFunc->InitConstrValAll(S, S->var->rLp, S->var->rLp, S->var->R, S->var->R);
    aFunc->InitConstrValSum(S);
    aFunc->ALMCalGrad(S, S->var->rLp, S->var->gradLp, S->var->R, S->var->Grad, &lagNormSquare, st->rho);
    double rc_val = sqrt(lagNormSquare) / (1 + S->cObjNrmInf);
    lorads_int localIter = 0, clearLBFGS = 0;
    double *trips = calloc(4 * (K + 1), sizeof(double));
    long done = 0;
    int stop = K <= 0;
    /* the inner loops of the first outer iterations (lorads_alm.c:1285-1409), trip by trip */
    /* the state is dumped where trip K + 1 would start (after the dual / rho updates that
       follow an inner loop ending at trip K), as a phase-1 budget of K stops there */
    while (!stop) {
        /* UpdateRho (lorads_alm.c:1403-1409) whenever the certificate is already met
           (:1297-1300), then a fresh inner loop (localIter = 0, :1285) */
        while (rc_val <= rc_tol) {
            do {
                st->rho *= p.ALMRhoFactor;
                aFunc->ALMCalGrad(S, S->var->rLp, S->var->gradLp, S->var->R, S->var->Grad, &lagNormSquare, st->rho);
                rc_val = sqrt(lagNormSquare) / (1 + S->cObjNrmInf);
                rc_tol = 0.1 / st->rho;
            } while (rc_tol >= rc_val);
            if (st->l_inf_primal_infeasibility <= p.phase1Tol) { stop = 1; break; }   /* :1423-1426 */
        }
        if (stop) break;
        localIter = 0;
        while (rc_val - rc_tol > p.endALMSubTol) {   /* lorads_alm.c:1302-1379 */
            while (multi && nextK < nK - 1 && done >= Ks[nextK]) {
                steps_dump(S, trips, done, argv[5], Ks[nextK]); nextK++;
            }
            if (done >= K) { stop = 1; break; }
            if (localIter % 300 == 0) clearLBFGS = 0;
            aFunc->LBFGSDirection(&p, S, S->lbfgsHis, S->var->gradLp, S->var->uLp, S->var->Grad, S->var->U, clearLBFGS);
            aFunc->LBFGSDirUseGrad(S, S->var->uLp, S->var->gradLp, S->var->U, S->var->Grad);
            double *q0 = S->var->M1temp;
            memcpy(q0, S->rowRHS, sizeof(double) * m);
            axpy(&m, &minusOne, S->var->constrValSum, &incx, q0, &incx);
            double p12[2];
            aFunc->ALMCalq12p12(S, S->var->rLp, S->var->uLp, S->var->R, S->var->U, S->var->ARDSum, S->var->ADDSum, p12);
            lorads_int rn = ALMLineSearch(st->rho, m, S->var->dualVar, p12[0], p12[1], q0, S->var->ARDSum,
                                          S->var->ADDSum, &tau);
            trips[4 * done] = tau; trips[4 * done + 1] = (double)rn;
            if (rn == 0 || fabs(tau) < p.endTauTol) { done++; stop = 1; break; }
            aFunc->setAsNegGrad(S, S->var->gradLp, S->var->Grad);
            aFunc->ALMupdateVar(S, S->var->rLp, S->var->uLp, S->var->R, S->var->U, tau);
            double tau2 = tau * tau;
            axpy(&m, &tau, S->var->ARDSum, &incx, S->var->constrValSum, &incx);
            axpy(&m, &tau2, S->var->ADDSum, &incx, S->var->constrValSum, &incx);
            lagNormSquare = 0.0;
            aFunc->ALMCalGrad(S, S->var->rLp, S->var->gradLp, S->var->R, S->var->Grad, &lagNormSquare, st->rho);
            aFunc->setlbfgsHisTwo(S, S->var->gradLp, S->var->uLp, S->var->Grad, S->var->U, tau);
            aFunc->updateDimacsALM(S, S->var->R, S->var->R, S->var->rLp, S->var->rLp);
            st->l_1_primal_infeasibility = S->dimacError[LORADS_DIMAC_ERROR_CONSTRVIO_L1];
            st->l_inf_primal_infeasibility = st->l_1_primal_infeasibility * (1 + S->bRHSNrm1) / (1 + S->bRHSNrmInf);
            trips[4 * done + 2] = lagNormSquare;
            trips[4 * done + 3] = S->dimacError[LORADS_DIMAC_ERROR_CONSTRVIO_L1];
            localIter++; clearLBFGS++; done++;
            if (st->l_inf_primal_infeasibility <= p.phase1Tol &&
                (st->primal_dual_gap <= p.phase1Tol || !p.highAccMode)) { stop = 1; break; }
            rc_val = sqrt(lagNormSquare) / (1 + S->cObjNrmInf);
            if (localIter > 800) break;
        }
        if (stop) break;
        /* lorads_alm.c:1380-1383: dual update, gradient, certificate; the difficulty only
           decides between another inner loop and UpdateRho, both of which start from here */
        LORADSUpdateDualVar(S, st->rho);
        aFunc->ALMCalGrad(S, S->var->rLp, S->var->gradLp, S->var->R, S->var->Grad, &lagNormSquare, st->rho);
        rc_val = sqrt(lagNormSquare) / (1 + S->cObjNrmInf);
        if (localIter <= 20) {   /* EASY: leave the outer iteration through UpdateRho */
            do {
                st->rho *= p.ALMRhoFactor;
                aFunc->ALMCalGrad(S, S->var->rLp, S->var->gradLp, S->var->R, S->var->Grad, &lagNormSquare, st->rho);
                rc_val = sqrt(lagNormSquare) / (1 + S->cObjNrmInf);
                rc_tol = 0.1 / st->rho;
            } while (rc_tol >= rc_val);
            if (st->l_inf_primal_infeasibility <= p.phase1Tol) break;
        }
    }
    /* Ks not reached (the loop stopped first): the final state, as stand-alone runs would dump */
    for (; multi && nextK < nK; ++nextK) steps_dump(S, trips, done, argv[5], Ks[nextK]);
    if (!multi && steps_dump(S, trips, done, argv[5], -1)) return 1;
    free(trips);
    printf("REF_STEPS done=%ld\n", done);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s solve|alm_rate|kernels file ...\n", argv[0]); return 2; }
    if (!strcmp(argv[1], "solve")) return mode_solve(argc, argv);
    if (!strcmp(argv[1], "alm_rate")) return mode_alm_rate(argc, argv);
    if (!strcmp(argv[1], "admm_sweep_lp")) return mode_admm_sweep_lp(argc, argv);
    if (!strcmp(argv[1], "kernels")) return mode_kernels(argc, argv);
    if (!strcmp(argv[1], "alm_steps")) return mode_alm_steps(argc, argv);
    if (!strcmp(argv[1], "admm_sweep")) return mode_admm_sweep(argc, argv);
    return 2;
}
