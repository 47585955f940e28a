/* oracle/oracle_main.c -- TEST INFRASTRUCTURE ONLY: CLI over the CPU restatement.
 *   lrsdp_oracle solve <file.dat-s> [--flag value ...]
 *   lrsdp_oracle alm_rate <file.dat-s> <rank> <seconds>
 *   lrsdp_oracle kernels <file.dat-s> <rank> <in.bin> <out.bin>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "lrsdp_oracle.h"

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s solve|alm_rate|kernels file ...\n", argv[0]); return 2; }
    if (!strcmp(argv[1], "solve")) {
        double r[16];
        if (oracle_solve(argv[2], argc - 3, argv + 3, r)) { printf("ORACLE_RESULT read_failed\n"); return 0; }
        printf("ORACLE_RESULT alm_inner=%ld alm_outer=%ld alm_pobj=%.17e alm_dobj=%.17e alm_pinf=%.17e "
               "alm_gap=%.17e alm_rho=%.17e admm_iter=%ld admm_pobj=%.17e admm_dobj=%.17e admm_pinf=%.17e "
               "admm_gap=%.17e admm_rho=%.17e solve_time=%.9e rank=%ld alm_time=%.9e\n",
               (long)r[0], (long)r[1], r[2], r[3], r[4], r[5], r[6], (long)r[7], r[8], r[9], r[10], r[11],
               r[12], r[13], (long)r[14], r[15]);
        return 0;
    }
    if (!strcmp(argv[1], "alm_rate")) {
        double el = 0;
        long it = oracle_alm_rate(argv[2], atoi(argv[3]), atof(argv[4]), &el);
        printf("ORACLE_RATE inner=%ld seconds=%.9e rate=%.9e\n", it, el, it / el);
        return 0;
    }
    if (!strcmp(argv[1], "kernels")) {
        oproblem *p = oracle_read(argv[2]);
        if (!p) return 1;
        FILE *f = fopen(argv[4], "rb");
        fseek(f, 0, SEEK_END); long sz = ftell(f); fseek(f, 0, SEEK_SET);
        double *in = malloc(sz);
        if (fread(in, 1, sz, f) != (size_t)sz) return 1;
        fclose(f);
        double *out = malloc(sz * 2 + 1024);
        int n = oracle_kernels(p, atoi(argv[3]), in, out);
        f = fopen(argv[5], "wb");
        fwrite(out, 8, n, f);
        fclose(f);
        oracle_free(p);
        return 0;
    }
    return 2;
}
