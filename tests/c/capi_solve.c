/* A plain-C caller of the boundary (include/lrsdp.h), as the reference's own host code (C)
 * would bind it: load an SDPA file, solve with the LoRADS defaults given on the command
 * line, print the result, write the reference-format JSON.  Built by tests/test_capi.py with
 * gcc (no C++ and no HIP headers needed on the caller's side).
 * usage: capi_solve <file.dat-s> <out.json> [reoptLevel] */
#include <stdio.h>
#include <stdlib.h>

#include "lrsdp.h"

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <file.dat-s> <out.json> [reoptLevel]\n", argv[0]);
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
