/*
 * oracle/lrsdp_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the
 * LoRADS low-rank SDP solve path.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * Every function cites the reference function it restates
 * (paths relative to /root/reference/lorads/src/src_semi/).  Storage follows the
 * reference: factors column-major n x r per cone (lorads_alg_common.c:62-68),
 * cones concatenated for the L-BFGS vectors (lorads_alm.c:468-475).  Every
 * coefficient is kept as a lower-triangle COO with a slot index into the cone's
 * union pattern (data/lorads_sdp_data.c:313-329); a "dense path" cone
 * (data/lorads_sdp_conic.c:1201-1280) simply has the full packed lower triangle
 * as its pattern, which is the same arithmetic as the reference's
 * dsyr2k/dsymm/packed-dot formulation (lorads_alg_common.c:72-89,
 * data/lorads_sdp_data.c:948-1034) up to summation order.  An LP block (the SDPA
 * block of negative size, data/lorads_lp_conic.c) is the last cone, diagonal, at
 * rank 1 (x_j = r_j^2) -- the product's layout -- and its ADMM update is the
 * reference's column sweep (lp_update_var).
 *
 * Parity pin: tests/test_oracle_golden.py checks this file against fixtures
 * written by the reference itself (oracle/_ref, scripts/make_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "lrsdp_oracle.h"

#define OMAX(a, b) ((a) > (b) ? (a) : (b))
#define OMIN(a, b) ((a) < (b) ? (a) : (b))

static double o_now(void) {
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return tv.tv_sec + 1e-6 * tv.tv_usec;
}

/* ------------------------------------------------------------------------ */
/* glibc rand()/srand() (TYPE_3 additive feedback), restated so the initial  */
/* point of data/lorads_solver.c:529-539 (srand(925) at :625) is reproduced   */
/* bit-for-bit without touching libc's global generator.                      */
/* ------------------------------------------------------------------------ */
typedef struct { int32_t r[34]; int32_t tbl[31]; int f, b; } grand_t;

static void grand_seed(grand_t *g, unsigned seed) {
    int32_t r[344];
    if (seed == 0) seed = 1;
    r[0] = (int32_t)seed;
    for (int i = 1; i < 31; i++) {
        int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int64_t word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = (int32_t)word;
    }
    for (int i = 31; i < 34; i++) r[i] = r[i - 31];
    for (int i = 34; i < 344; i++) r[i] = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
    /* state = the 31 words preceding the first output r[344] */
    for (int i = 0; i < 31; i++) g->tbl[i] = r[313 + i];
    g->f = 0;  /* slot holding r[k-31] for the next k */
}

static int grand_next(grand_t *g) {
    /* r[k] = r[k-31] + r[k-3]; output r[k] >> 1 (glibc random_r TYPE_3) */
    int32_t *t = g->tbl;
    int i = g->f;
    int j = (g->f + 28) % 31;
    int32_t v = (int32_t)((uint32_t)t[i] + (uint32_t)t[j]);
    t[i] = v;
    g->f = (g->f + 1) % 31;
    return (int)((uint32_t)v >> 1);
}
#define O_RAND_MAX 2147483647

/* ------------------------------------------------------------------------ */
/* Problem model                                                              */
/* ------------------------------------------------------------------------ */
typedef struct {
    int nnz;
    int *row, *col, *slot;   /* lower triangle: row >= col, sorted by (col,row) */
    double *val;
    int dense;               /* >10 % fill (data/lorads_sdp_data.c:1189) */
} ocoeff;

typedef struct {
    int n;
    int densePath;           /* data/lorads_sdp_conic.c:1201, :1287, :1389 */
    int P;                   /* pattern slots */
    int *prow, *pcol;        /* pattern, sorted by (col,row) (sdp_conic.c:1075) */
    ocoeff C;
    int ncoef;               /* constraints with a nonzero coefficient in this cone */
    int *con;                /* constraint id of each coefficient */
    ocoeff *A;
    double *uvt;             /* pattern scratch: sdp_obj_sum / sdp_coeff_w_sum */
    int rank, rank_max;
    /* the LP block (lorads_lp_conic.c) restated as the diagonal cone at rank 1, as the product
       does (lrs_problem.cpp build_problem): its columns the rows, x_j = r_j^2; per column its
       (constraint, a) list in constraint order (lp_cone_presolve, :90-125), c_j and ||a_j||^2 */
    int lp;
    int *lp_ptr, *lp_con;
    double *lp_a, *lp_c, *lp_nrm2;
} ocone;

struct oproblem {
    int m, K;
    double *b;
    ocone *cones;
};

static void coeff_free(ocoeff *c) {
    free(c->row); free(c->col); free(c->slot); free(c->val);
    memset(c, 0, sizeof(*c));
}

void oracle_free(oproblem *p) {
    if (!p) return;
    for (int k = 0; k < p->K; ++k) {
        ocone *c = &p->cones[k];
        coeff_free(&c->C);
        for (int i = 0; i < c->ncoef; ++i) coeff_free(&c->A[i]);
        free(c->A); free(c->con); free(c->prow); free(c->pcol); free(c->uvt);
        free(c->lp_ptr); free(c->lp_con); free(c->lp_a); free(c->lp_c); free(c->lp_nrm2);
    }
    free(p->cones); free(p->b); free(p);
}

int oracle_dims(const oproblem *p, int *m, int *ncones, int *dims) {
    if (m) *m = p->m;
    if (ncones) *ncones = p->K;
    if (dims) for (int k = 0; k < p->K; ++k) dims[k] = p->cones[k].n;
    return 0;
}

/* ---------------- SDPA reader: io/lorads_file_io.c:59-455 ---------------- */
typedef struct { char *s; size_t pos, len; } otext;

static int skip_to_number(otext *t) {
    while (t->pos < t->len) {
        char ch = t->s[t->pos];
        if (ch == '{' || ch == '}' || ch == '(' || ch == ')' || ch == ',' || ch == '\'' ||
            ch == ' ' || ch == '\t' || ch == '\r' || ch == '\n')
            t->pos++;
        else
            return 1;
    }
    return 0;
}

static int next_line(otext *t, char **line) {
    if (t->pos >= t->len) return 0;
    *line = t->s + t->pos;
    while (t->pos < t->len && t->s[t->pos] != '\n') t->pos++;
    if (t->pos < t->len) { t->s[t->pos] = '\0'; t->pos++; }
    return 1;
}

typedef struct { int idx, con; double v; int seq; } oentry;

static int cmp_entry(const void *a, const void *b) {
    const oentry *x = a, *y = b;
    if (x->con != y->con) return x->con < y->con ? -1 : 1;     /* CSC column */
    if (x->idx != y->idx) return x->idx < y->idx ? -1 : 1;     /* ascending sort :154-156 */
    return x->seq < y->seq ? -1 : (x->seq > y->seq);
}

static int cmp_pair(const void *a, const void *b) {   /* cmpfunc, sdp_conic.c:1075 */
    const int *x = a, *y = b;
    if (x[1] != y[1]) return x[1] < y[1] ? -1 : 1;
    return (x[0] > y[0]) - (x[0] < y[0]);
}

/* packed lower column-major index -> (row, col), tsp_decompress (linalg/lorads_sparse_opts.c:82) */
static void unpack_idx(int n, long idx, int *row, int *col) {
    long j = 0, thresh = n;
    while (idx >= thresh) { j++; thresh += n - j; }
    *row = (int)(idx - thresh + n);
    *col = (int)j;
}

static long pack_idx(int n, int row, int col) { return (long)(2L * n - col - 1) * col / 2 + row; }

static void build_coeff(ocoeff *c, int n, oentry *e, int cnt) {
    c->nnz = cnt;
    c->row = malloc(sizeof(int) * (cnt ? cnt : 1));
    c->col = malloc(sizeof(int) * (cnt ? cnt : 1));
    c->slot = malloc(sizeof(int) * (cnt ? cnt : 1));
    c->val = malloc(sizeof(double) * (cnt ? cnt : 1));
    for (int k = 0; k < cnt; ++k) {
        unpack_idx(n, e[k].idx, &c->row[k], &c->col[k]);
        c->val[k] = e[k].v;
        c->slot[k] = -1;
    }
    c->dense = (double)cnt > 0.1 * (double)((long)n * (n + 1) / 2);
}

static int slot_lookup(const ocone *c, int row, int col) {
    if (c->densePath) return (int)pack_idx(c->n, row, col);
    /* binary search in pattern sorted by (col,row) */
    int lo = 0, hi = c->P - 1;
    while (lo <= hi) {
        int mid = (lo + hi) >> 1;
        int mc = c->pcol[mid], mr = c->prow[mid];
        if (mc == col && mr == row) return mid;
        if (mc < col || (mc == col && mr < row)) lo = mid + 1; else hi = mid - 1;
    }
    return -1;
}

/* AConePresolveData, data/lorads_sdp_conic.c:1185-1393 */
static void presolve_cone(ocone *c) {
    int n = c->n;
    int dense = (n < 20) || c->C.dense;
    if (c->lp) dense = 0;   /* the LP block: per-column operations, never the packed dense path */
    for (int i = 0; i < c->ncoef && !dense && !c->lp; ++i) dense |= c->A[i].dense;
    if (!dense) {
        long tot = c->C.nnz;
        for (int i = 0; i < c->ncoef; ++i) tot += c->A[i].nnz;
        int *pairs = malloc(sizeof(int) * 2 * (tot ? tot : 1));
        long q = 0;
        for (int k = 0; k < c->C.nnz; ++k) { pairs[2 * q] = c->C.row[k]; pairs[2 * q + 1] = c->C.col[k]; q++; }
        for (int i = 0; i < c->ncoef; ++i)
            for (int k = 0; k < c->A[i].nnz; ++k) {
                pairs[2 * q] = c->A[i].row[k]; pairs[2 * q + 1] = c->A[i].col[k]; q++;
            }
        qsort(pairs, tot, 2 * sizeof(int), cmp_pair);
        int P = 0;
        for (long k = 0; k < tot; ++k)
            if (k == 0 || pairs[2 * k] != pairs[2 * k - 2] || pairs[2 * k + 1] != pairs[2 * k - 1]) {
                pairs[2 * P] = pairs[2 * k]; pairs[2 * P + 1] = pairs[2 * k + 1]; P++;
            }
        double spRatio = (double)P / (double)((long)n * (n + 1) / 2);
        if (spRatio < 0.1) {
            c->P = P;
            c->prow = malloc(sizeof(int) * P);
            c->pcol = malloc(sizeof(int) * P);
            for (int k = 0; k < P; ++k) { c->prow[k] = pairs[2 * k]; c->pcol[k] = pairs[2 * k + 1]; }
        } else {
            dense = 1;
        }
        free(pairs);
    }
    if (dense) {
        c->densePath = 1;
        c->P = (int)((long)n * (n + 1) / 2);
        c->prow = malloc(sizeof(int) * c->P);
        c->pcol = malloc(sizeof(int) * c->P);
        long q = 0;
        for (int col = 0; col < n; ++col)
            for (int row = col; row < n; ++row) { c->prow[q] = row; c->pcol[q] = col; q++; }
    }
    for (int k = 0; k < c->C.nnz; ++k) c->C.slot[k] = slot_lookup(c, c->C.row[k], c->C.col[k]);
    for (int i = 0; i < c->ncoef; ++i)
        for (int k = 0; k < c->A[i].nnz; ++k) c->A[i].slot[k] = slot_lookup(c, c->A[i].row[k], c->A[i].col[k]);
    c->uvt = calloc(c->P, sizeof(double));
}

oproblem *oracle_read(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    otext t;
    t.s = malloc(sz + 1);
    t.len = fread(t.s, 1, sz, f);
    t.s[t.len] = '\0';
    t.pos = 0;
    fclose(f);
    char *line = NULL;
    /* comments */
    do {
        if (!next_line(&t, &line)) { free(t.s); return NULL; }
    } while (line[0] == '*' || line[0] == '"');
    int m = 0, nb = 0;
    if (sscanf(line, "%d", &m) != 1) { free(t.s); return NULL; }
    if (!next_line(&t, &line) || sscanf(line, "%d", &nb) != 1) { free(t.s); return NULL; }
    int *dims = calloc(nb, sizeof(int));
    int nlp = 0, K = nb;
    for (int k = 0; k < nb; ++k) {
        if (!skip_to_number(&t)) { free(t.s); free(dims); return NULL; }
        char *endp;
        long d = strtol(t.s + t.pos, &endp, 10);
        t.pos = endp - t.s;
        if (k < nb - 1 && d <= 0) { free(t.s); free(dims); return NULL; }  /* :159-166 */
        if (k == nb - 1 && d < 0) { nlp = (int)-d; K = nb - 1; }            /* :187-190 */
        dims[k] = (int)d;
    }
    if (nlp > 0) { dims[nb - 1] = nlp; K = nb; }   /* the LP block: cone nb - 1, diagonal */
    double *b = calloc(m, sizeof(double));
    for (int i = 0; i < m; ++i) {
        if (!skip_to_number(&t)) { free(t.s); free(dims); free(b); return NULL; }
        char *endp;
        b[i] = strtod(t.s + t.pos, &endp);
        if (endp == t.s + t.pos) { t.pos++; --i; continue; }
        t.pos = endp - t.s;
    }
    /* rest of the b line */
    while (t.pos < t.len && t.s[t.pos] != '\n') t.pos++;
    if (t.pos < t.len) t.pos++;
    /* entries, :260-331 */
    size_t cap = 1024, cnt = 0;
    oentry *ent = malloc(sizeof(oentry) * cap);
    int *blk = malloc(sizeof(int) * cap);
    while (next_line(&t, &line)) {
        int ic, ib, ii, ij;
        double v;
        if (sscanf(line, "%d %d %d %d %lg", &ic, &ib, &ii, &ij, &v) != 5) {
            int blank = 1;
            for (char *q = line; *q; ++q) if (*q != ' ' && *q != '\t' && *q != '\r') blank = 0;
            if (blank) continue;
            /* :264-279: stop at the 'BEGIN.COMMENT' trailer or at end of file (a last line
               without a newline: next_line leaves it unterminated), else reject */
            if (strncmp(line, "BEGIN.COMMENT", 13) == 0 || (t.pos >= t.len && t.s[t.len - 1] != '\0')) break;
            free(t.s); free(dims); free(b); free(ent); free(blk);
            return NULL;
        }
        ib -= 1; ii -= 1; ij -= 1;
        if (fabs(v) < 1e-12) continue;                        /* :288-294 */
        if (ib < 0 || ib >= K) continue;
        if (nlp > 0 && ib == K - 1) ij = ii;                  /* LP: column iRow, :297-309 */
        if (ii > ij) { int tmp = ii; ii = ij; ij = tmp; }    /* :311-315 */
        if (ic == 0) v = -v;                                 /* :317-319, C = -F0 */
        if (cnt == cap) { cap *= 2; ent = realloc(ent, sizeof(oentry) * cap); blk = realloc(blk, sizeof(int) * cap); }
        ent[cnt].idx = (int)pack_idx(dims[ib], ij, ii);       /* PACK_IDX(n, iCol, iRow) :321 */
        ent[cnt].con = ic;
        ent[cnt].v = v;
        ent[cnt].seq = (int)cnt;
        blk[cnt] = ib;
        cnt++;
    }
    free(t.s);
    oproblem *p = calloc(1, sizeof(oproblem));
    p->m = m; p->K = K; p->b = b;
    p->cones = calloc(K, sizeof(ocone));
    for (int k = 0; k < K; ++k) {
        ocone *c = &p->cones[k];
        c->n = dims[k];
        c->lp = nlp > 0 && k == K - 1;
        size_t nk = 0;
        for (size_t e = 0; e < cnt; ++e) if (blk[e] == k) nk++;
        oentry *ek = malloc(sizeof(oentry) * (nk ? nk : 1));
        nk = 0;
        for (size_t e = 0; e < cnt; ++e) if (blk[e] == k) ek[nk++] = ent[e];
        qsort(ek, nk, sizeof(oentry), cmp_entry);
        /* per-constraint coefficients */
        size_t s = 0;
        int ncoef = 0;
        c->A = calloc(m > 0 ? m : 1, sizeof(ocoeff));
        c->con = calloc(m > 0 ? m : 1, sizeof(int));
        while (s < nk && ek[s].con == 0) s++;
        build_coeff(&c->C, c->n, ek, (int)s);
        while (s < nk) {
            size_t e = s;
            while (e < nk && ek[e].con == ek[s].con) e++;
            build_coeff(&c->A[ncoef], c->n, ek + s, (int)(e - s));
            c->con[ncoef] = ek[s].con - 1;
            ncoef++;
            s = e;
        }
        c->ncoef = ncoef;
        free(ek);
        if (c->lp) {
            /* lp_cone_presolve (lorads_lp_conic.c:85-147): per column its constraints in order, the
               column's ||a||^2 from its raw entries; a column in >= 1/4 of the constraints is
               LP_COEFF_DENSE, whose create routine leaves its row count 0 (lorads_lp_data.c:178-193:
               calloc), so its coefficients reach neither A(x) nor A^*(y) -- dropped here, norm kept */
            int n = c->n;
            int *cnt = calloc(n, sizeof(int));
            c->lp_nrm2 = calloc(n, sizeof(double));
            c->lp_c = calloc(n, sizeof(double));
            for (int q = 0; q < c->C.nnz; ++q) c->lp_c[c->C.row[q]] += c->C.val[q];
            for (int i = 0; i < ncoef; ++i)
                for (int q = 0; q < c->A[i].nnz; ++q) {
                    cnt[c->A[i].row[q]]++;
                    c->lp_nrm2[c->A[i].row[q]] += c->A[i].val[q] * c->A[i].val[q];
                }
            for (int j = 0; j < n; ++j) { double tq = sqrt(c->lp_nrm2[j]); c->lp_nrm2[j] = tq * tq; }
            for (int i = 0; i < ncoef; ++i) {
                int w = 0;
                for (int q = 0; q < c->A[i].nnz; ++q) {
                    int j = c->A[i].row[q];
                    if (cnt[j] != 0 && (double)cnt[j] / (double)m >= 0.25) continue;
                    c->A[i].row[w] = c->A[i].row[q]; c->A[i].col[w] = c->A[i].col[q]; c->A[i].val[w] = c->A[i].val[q];
                    w++;
                }
                c->A[i].nnz = w;
                c->A[i].dense = 0;
            }
            c->lp_ptr = calloc(n + 1, sizeof(int));
            long tot = 0;
            for (int i = 0; i < ncoef; ++i)
                for (int q = 0; q < c->A[i].nnz; ++q) { c->lp_ptr[c->A[i].row[q] + 1]++; tot++; }
            for (int j = 0; j < n; ++j) c->lp_ptr[j + 1] += c->lp_ptr[j];
            c->lp_con = malloc(sizeof(int) * (tot ? tot : 1));
            c->lp_a = malloc(sizeof(double) * (tot ? tot : 1));
            int *fill = calloc(n, sizeof(int));
            for (int i = 0; i < ncoef; ++i)   /* constraints ascending: each column's list in order */
                for (int q = 0; q < c->A[i].nnz; ++q) {
                    int j = c->A[i].row[q];
                    c->lp_con[c->lp_ptr[j] + fill[j]] = c->con[i];
                    c->lp_a[c->lp_ptr[j] + fill[j]] = c->A[i].val[q];
                    fill[j]++;
                }
            free(cnt); free(fill);
        }
        presolve_cone(c);
    }
    free(ent); free(blk); free(dims);
    return p;
}

/* ------------------------------------------------------------------------ */
/* Hot-path operators                                                          */
/* ------------------------------------------------------------------------ */

/* LORADSUVt sparse branch, lorads_alg/lorads_alg_common.c:51-71:
   uvt[slot(i,j)] = 0.5(U_i.V_j + U_j.V_i) (i != j), U_i.V_i (i == j) */
static void o_uvt(ocone *c, const double *U, const double *V, int r) {
    int n = c->n;
    for (int s = 0; s < c->P; ++s) {
        int i = c->prow[s], j = c->pcol[s];
        if (i != j) {
            double a = 0.0, bb = 0.0;
            for (int q = 0; q < r; ++q) a += U[i + (long)q * n] * V[j + (long)q * n];
            for (int q = 0; q < r; ++q) bb += U[j + (long)q * n] * V[i + (long)q * n];
            c->uvt[s] = 0.5 * a + 0.5 * bb;
        } else {
            double a = 0.0;
            for (int q = 0; q < r; ++q) a += U[i + (long)q * n] * V[i + (long)q * n];
            c->uvt[s] = a;
        }
    }
}

/* <A, sym UV^T> through the slot map: sparseAUV / denseAUV,
   data/lorads_sdp_data.c:803-856 (2a*uvt, minus half of it on the diagonal) */
static double o_coeff_dot(const ocoeff *a, const double *uvt) {
    double res = 0.0;
    for (int k = 0; k < a->nnz; ++k) {
        double tmp = 2 * a->val[k] * uvt[a->slot[k]];
        res += tmp;
        if (a->row[k] == a->col[k]) res -= 0.5 * tmp;
    }
    return res;
}

/* coneAUV, data/lorads_sdp_conic.c:378-385 / :681-688: out[con] = <A_con, uvt> */
static void o_cone_auv(const ocone *c, double *out_m) {
    for (int i = 0; i < c->ncoef; ++i) out_m[c->con[i]] = o_coeff_dot(&c->A[i], c->uvt);
}

/* sdpDataWSum (+ addObjCoeff), data/lorads_sdp_conic.c:448-460, :608-616, :894-902 */
static void o_wsum(ocone *c, const double *w, int withC, double *S) {
    memset(S, 0, sizeof(double) * c->P);
    if (withC)
        for (int k = 0; k < c->C.nnz; ++k) S[c->C.slot[k]] += c->C.val[k];
    for (int i = 0; i < c->ncoef; ++i) {
        double wi = w[c->con[i]];
        const ocoeff *a = &c->A[i];
        for (int k = 0; k < a->nnz; ++k) S[a->slot[k]] += wi * a->val[k];
    }
}

/* mul_rk, data/lorads_sdp_data.c:750-763: AX = S X (symmetric, lower-stored) */
static void o_spmm(const ocone *c, const double *S, const double *X, int r, double *AX) {
    int n = c->n;
    memset(AX, 0, sizeof(double) * (long)n * r);
    for (int s = 0; s < c->P; ++s) {
        double v = S[s];
        if (v == 0.0) continue;
        int i = c->prow[s], j = c->pcol[s];
        for (int q = 0; q < r; ++q) AX[i + (long)q * n] += v * X[j + (long)q * n];
        if (i != j)
            for (int q = 0; q < r; ++q) AX[j + (long)q * n] += v * X[i + (long)q * n];
    }
}

/* ------------------------------------------------------------------------ */
/* Solver state                                                                */
/* ------------------------------------------------------------------------ */
typedef struct {
    double initRho, rhoMax, rhoCellingALM, rhoCellingADMM;
    int maxALMIter, maxADMMIter;
    double timesLogRank;
    int fixedRank, initRank, rhoFreq;
    double rhoFactor, ALMRhoFactor, rankUpdateFactor, phase1Tol, phase2Tol, timeSecLimit,
        heuristicFactor;
    int lbfgsListLength;
    double endTauTol, endALMSubTol;
    int reoptLevel, dyrankLevel, highAccMode, disableOracle;
} oparams;

typedef struct {
    long outerIter, innerIter, iter, cg_iter;
    double rho, pobj, dobj, pinf1, pinfinf, gap;
} ostate;

typedef struct {
    oproblem *p;
    oparams prm;
    int m, K;
    int *rank;
    long *off;          /* factor offsets (col-major per cone), off[K] = NR */
    long NR;
    double *R, *U, *V, *G, *Dtmp;
    /* L-BFGS ring (lorads_solver.c:680-707) */
    int L;
    double **ls, **ly, *lbeta, *lalpha;
    int head;
    double *lam, *cvs, *cvc; /* dual, constrValSum, per-cone constrVal (K*m) */
    double *q1, *q2, *M1, *S, *M2, *bls, *vio;
    double cObjNrm1, cObjNrm2, cObjNrmInf, bNrm1, bNrmInf, bNrm2, scaleObjHis;
    double pObjVal, dObjVal, dimPinf, dimGap;
    long *cgIterCone;   /* CG "iter" persists per cone (linalg/lorads_cgs.c:220) */
    long cgIter;
    int *traj1_cur, *traj1_orc, *traj2_cur, *traj2_orc;
    int n1, n2, cap1, cap2;
} osolver;

static void nrm_consts(osolver *s) {   /* cal_sdp_const, data/lorads_solver.c:1462 */
    oproblem *p = s->p;
    s->cObjNrm1 = 0; s->cObjNrm2 = 0; s->cObjNrmInf = 0;
    for (int k = 0; k < p->K; ++k) {
        ocoeff *C = &p->cones[k].C;
        double n1 = 0, n2 = 0, ni = 0;
        for (int q = 0; q < C->nnz; ++q) {
            double a = C->val[q];
            n1 += 2 * fabs(a); n2 += 2 * a * a; ni = OMAX(ni, fabs(a));
            if (C->row[q] == C->col[q]) { n1 -= fabs(a); n2 -= a * a; }
        }
        if (p->cones[k].lp) n2 = n1 * n1;   /* lp_cone_obj_nrm2Square, lorads_lp_conic.c:171-176 */
        s->cObjNrm1 += n1; s->cObjNrm2 += n2; s->cObjNrmInf = OMAX(s->cObjNrmInf, ni);
    }
    s->cObjNrm2 = pow(s->cObjNrm2, 0.5);
    s->bNrm1 = 0; s->bNrm2 = 0; s->bNrmInf = 0;
    int imax = 0;
    double bmax = -1.0;
    for (int i = 0; i < s->m; ++i) {
        s->bNrm1 += fabs(p->b[i]); s->bNrm2 += p->b[i] * p->b[i];
        if (fabs(p->b[i]) > bmax) { bmax = fabs(p->b[i]); imax = i; }
    }
    /* data/lorads_solver.c:1469 (UNDER_BLAS): b[idamax_(b)] with Fortran's 1-based idamax_
       as a C index -- the entry after the first largest |b_i| (the largest itself if last) */
    if (s->m > 0) s->bNrmInf = fabs(p->b[imax + 1 < s->m ? imax + 1 : imax]);
    s->bNrm2 = sqrt(s->bNrm2);
}

/* LORADSDetermineRank, data/lorads_solver.c:406-459 */
static int n_sdp(const osolver *s) { return s->K - (s->K > 0 && s->p->cones[s->K - 1].lp ? 1 : 0); }
static void determine_rank(osolver *s) {
    for (int k = 0; k < s->K; ++k) {
        ocone *c = &s->p->cones[k];
        if (c->lp) { s->rank[k] = 1; c->rank_max = 1; continue; }   /* x_j = r_j^2 */
        int nnzRows = c->ncoef;
        int calc_max = OMIN((int)sqrt(2.0 * nnzRows) + 1, c->n);
        if (s->prm.fixedRank > 0) {
            s->rank[k] = OMAX(1, OMIN(s->prm.fixedRank, c->n));
            c->rank_max = s->rank[k];
            continue;
        }
        c->rank_max = calc_max;
        if (s->prm.initRank > 0) {
            s->rank[k] = OMAX(1, OMIN(s->prm.initRank, c->n));
        } else {
            int rk;
            if (s->prm.timesLogRank <= 1e-6) rk = calc_max;
            else if (nnzRows / c->n >= 20 && c->n <= 400 && n_sdp(s) <= 3) rk = calc_max;   /* nCones */
            else rk = (int)OMIN(ceil(s->prm.timesLogRank * log((double)c->n)), (double)calc_max);
            s->rank[k] = OMAX(1, rk);
        }
    }
}

static void alloc_factors(osolver *s) {
    s->off = realloc(s->off, sizeof(long) * (s->K + 1));
    s->NR = 0;
    for (int k = 0; k < s->K; ++k) { s->off[k] = s->NR; s->NR += (long)s->p->cones[k].n * s->rank[k]; }
    s->off[s->K] = s->NR;
}

static osolver *osolver_new(oproblem *p, const oparams *prm) {
    osolver *s = calloc(1, sizeof(osolver));
    s->p = p; s->prm = *prm; s->m = p->m; s->K = p->K;
    s->rank = calloc(s->K, sizeof(int));
    determine_rank(s);
    alloc_factors(s);
    s->R = calloc(s->NR, 8); s->U = calloc(s->NR, 8); s->V = calloc(s->NR, 8);
    s->G = calloc(s->NR, 8); s->Dtmp = calloc(s->NR, 8);
    /* initial point: srand(925), R then U then V per cone (lorads_solver.c:625, :654, :923-924) */
    grand_t g;
    grand_seed(&g, 925);
    for (long i = 0; i < s->NR; ++i) {
        s->R[i] = (double)grand_next(&g) / O_RAND_MAX;
        s->R[i] -= (double)grand_next(&g) / O_RAND_MAX;
    }
    for (int k = 0; k < s->K; ++k) {
        for (long i = s->off[k]; i < s->off[k + 1]; ++i) {
            s->U[i] = (double)grand_next(&g) / O_RAND_MAX; s->U[i] -= (double)grand_next(&g) / O_RAND_MAX;
        }
        for (long i = s->off[k]; i < s->off[k + 1]; ++i) {
            s->V[i] = (double)grand_next(&g) / O_RAND_MAX; s->V[i] -= (double)grand_next(&g) / O_RAND_MAX;
        }
    }
    s->L = prm->lbfgsListLength;
    s->ls = calloc(s->L, sizeof(double *)); s->ly = calloc(s->L, sizeof(double *));
    for (int q = 0; q < s->L; ++q) { s->ls[q] = calloc(s->NR, 8); s->ly[q] = calloc(s->NR, 8); }
    s->lbeta = calloc(s->L, 8); s->lalpha = calloc(s->L, 8);
    s->head = 0;
    int m = s->m;
    s->lam = calloc(m, 8); s->cvs = calloc(m, 8); s->cvc = calloc((long)s->K * m, 8);
    s->q1 = calloc(m, 8); s->q2 = calloc(m, 8); s->M1 = calloc(m, 8); s->vio = calloc(m, 8);
    int Pmax = 1;
    for (int k = 0; k < s->K; ++k) Pmax = OMAX(Pmax, p->cones[k].P);
    s->S = calloc(Pmax, 8);
    s->M2 = calloc(s->NR, 8); s->bls = calloc(s->NR, 8);
    s->cgIterCone = calloc(s->K, sizeof(long));
    s->scaleObjHis = 1;
    nrm_consts(s);
    s->cap1 = s->cap2 = 128;
    s->traj1_cur = calloc(128, sizeof(int)); s->traj1_orc = calloc(128, sizeof(int));
    s->traj2_cur = calloc(128, sizeof(int)); s->traj2_orc = calloc(128, sizeof(int));
    return s;
}

static void osolver_free(osolver *s) {
    if (!s) return;
    for (int q = 0; q < s->L; ++q) { free(s->ls[q]); free(s->ly[q]); }
    free(s->ls); free(s->ly); free(s->lbeta); free(s->lalpha);
    free(s->R); free(s->U); free(s->V); free(s->G); free(s->Dtmp);
    free(s->lam); free(s->cvs); free(s->cvc); free(s->q1); free(s->q2); free(s->M1); free(s->vio);
    free(s->S); free(s->M2); free(s->bls); free(s->rank); free(s->off); free(s->cgIterCone);
    free(s->traj1_cur); free(s->traj1_orc); free(s->traj2_cur); free(s->traj2_orc);
    free(s);
}

static double o_dot(long n, const double *a, const double *b) {
    double acc = 0.0;
    for (long i = 0; i < n; ++i) acc += a[i] * b[i];
    return acc;
}

/* LORADSInitConstrValAll + LORADSInitConstrValSum, lorads_alg_common.c:116-122, :221-229 */
static void constr_val_all(osolver *s, const double *U, const double *V) {
    memset(s->cvs, 0, sizeof(double) * s->m);
    for (int k = 0; k < s->K; ++k) {
        ocone *c = &s->p->cones[k];
        double *cv = s->cvc + (long)k * s->m;
        memset(cv, 0, sizeof(double) * s->m);
        o_uvt(c, U + s->off[k], V + s->off[k], s->rank[k]);
        o_cone_auv(c, cv);
        for (int i = 0; i < s->m; ++i) s->cvs[i] += cv[i];
    }
}

/* LORADSObjConstrValAll, lorads_alg_common.c:169-176: per-cone constrVal <- A(sym UV^T),
   obj += <C, sym UV^T>; LORADSConstrValSumALMtemp sums into q */
static double obj_constr_val_all(osolver *s, const double *U, const double *V, double *q) {
    double obj = 0.0;
    memset(q, 0, sizeof(double) * s->m);
    for (int k = 0; k < s->K; ++k) {
        ocone *c = &s->p->cones[k];
        double *cv = s->cvc + (long)k * s->m;
        memset(cv, 0, sizeof(double) * s->m);
        o_uvt(c, U + s->off[k], V + s->off[k], s->rank[k]);
        obj += o_coeff_dot(&c->C, c->uvt);
        o_cone_auv(c, cv);
        for (int i = 0; i < s->m; ++i) q[i] += cv[i];
    }
    return obj;
}

/* ALMSetGrad / ALMCalGrad, lorads_alm.c:32-87 */
static double alm_cal_grad(osolver *s, double rho) {
    for (int i = 0; i < s->m; ++i) s->M1[i] = -s->lam[i] - rho * s->p->b[i] + rho * s->cvs[i];
    double lag = 0.0;
    for (int k = 0; k < s->K; ++k) {
        ocone *c = &s->p->cones[k];
        o_wsum(c, s->M1, 1, s->S);
        o_spmm(c, s->S, s->R + s->off[k], s->rank[k], s->G + s->off[k]);
        long len = s->off[k + 1] - s->off[k];
        for (long i = 0; i < len; ++i) s->G[s->off[k] + i] *= 2.0;
        double nrm = sqrt(o_dot(len, s->G + s->off[k], s->G + s->off[k]));
        lag += nrm * nrm;
    }
    return lag;
}

/* LORADScubic_equation, lorads_alm.c:191-231 */
static int o_cubic(double a, double b, double c, double d, double *res) {
    double A = b * b - 3 * a * c, B = b * c - 9 * a * d, C = c * c - 3 * b * d;
    double delta = B * B - 4 * A * C;
    res[0] = res[1] = res[2] = 0.0;
    if (A == 0 && B == 0) { res[0] = OMAX(res[0], -c / b); return 1; }
    else if (delta > 0) {
        double Y1 = A * b + 1.5 * a * (-B + sqrt(delta));
        double Y2 = A * b + 1.5 * a * (-B - sqrt(delta));
        double Y1_3 = Y1 > 0 ? pow(Y1, 1.0 / 3) : -pow(-Y1, 1.0 / 3);
        double Y2_3 = Y2 > 0 ? pow(Y2, 1.0 / 3) : -pow(-Y2, 1.0 / 3);
        res[0] = OMAX(res[0], (-b - Y1_3 - Y2_3) / 3 / a);
        return 1;
    } else if (delta == 0 && A != 0 && B != 0) {
        double Kk = B / A;
        res[0] = -b / a + Kk; res[1] = -Kk / 2;
        return 2;
    } else if (delta < 0) {
        double sqA = sqrt(A);
        double T = (A * b - 1.5 * a * B) / (A * sqA);
        double theta = acos(T);
        double csth = cos(theta / 3), sn3th = sqrt(3) * sin(theta / 3);
        res[0] = (-b - 2 * sqA * csth) / 3 / a;
        res[1] = (-b + sqA * (csth + sn3th)) / 3 / a;
        res[2] = (-b + sqA * (csth - sn3th)) / 3 / a;
        return 3;
    }
    return 0;
}

static double o_fval(double a, double b, double c, double d, double x) {
    return a * pow(x, 4) + b * pow(x, 3) + c * pow(x, 2) + d * x;
}

/* ALMLineSearch, lorads_alm.c:266-333 (q0 is modified in place like the reference) */
static int alm_line_search(double rho, int m, const double *lam, double p1, double p2, double *q0,
                           const double *q1, const double *q2, double *tau) {
    double q2n = sqrt(o_dot(m, q2, q2));
    double a = rho * q2n * q2n / 2;
    double b = rho * o_dot(m, q1, q2);
    double rhoInv = 1 / rho;
    for (int i = 0; i < m; ++i) q0[i] += rhoInv * lam[i];
    double q1n = sqrt(o_dot(m, q1, q1));
    double c = p2 - rho * o_dot(m, q0, q2) + rho * q1n * q1n / 2;
    double d = p1 - rho * o_dot(m, q0, q1);
    double roots[3];
    int rn = o_cubic(4 * a, 3 * b, 2 * c, d, roots);
    double f0 = 0.0, f1 = o_fval(a, b, c, d, 1.0), fr1 = 1e30, fr2 = 1e30, fr3 = 1e30;
    if (rn >= 1 && roots[0] > 1e-20 && roots[0] <= 1.0) fr1 = o_fval(a, b, c, d, roots[0]);
    if (rn >= 2 && roots[1] > 1e-20 && roots[1] <= 1.0) fr2 = o_fval(a, b, c, d, roots[1]);
    if (rn == 3 && roots[2] > 1e-20 && roots[2] <= 1.0) fr3 = o_fval(a, b, c, d, roots[2]);
    double mn = OMIN(OMIN(OMIN(OMIN(f0, f1), fr1), fr2), fr3);
    if (fabs(mn - f0) < 1e-10) *tau = 0.0;
    if (fabs(mn - f1) < 1e-10) *tau = 1.0;
    if (fabs(mn - fr1) < 1e-10) *tau = roots[0];
    if (fabs(mn - fr2) < 1e-10) *tau = roots[1];
    if (fabs(mn - fr3) < 1e-10) *tau = roots[2];
    return rn;
}

/* LBFGSDirection (non-FIX_INI_POINT branch), lorads_alm.c:468-505; result in U */
static void lbfgs_direction(osolver *s, int innerIter) {
    long NR = s->NR;
    if (innerIter == 0) {
        for (long i = 0; i < NR; ++i) s->U[i] = -s->G[i];
        return;
    }
    double *Dt = s->Dtmp;
    memcpy(Dt, s->G, sizeof(double) * NR);
    int nodeNum = (innerIter <= s->L - 1) ? innerIter : s->L;
    int node = (s->head - 1 + s->L) % s->L;                 /* newest */
    for (int k = 0; k < nodeNum; ++k) {
        double tmp = o_dot(NR, s->ls[node], Dt);
        s->lalpha[node] = s->lbeta[node] * tmp;
        double an = -s->lalpha[node];
        for (long i = 0; i < NR; ++i) Dt[i] += an * s->ly[node][i];
        node = (node - 1 + s->L) % s->L;
    }
    node = (node + 1) % s->L;
    for (int k = 0; k < nodeNum; ++k) {
        double w = s->lalpha[node] - s->lbeta[node] * o_dot(NR, s->ly[node], Dt);
        for (long i = 0; i < NR; ++i) Dt[i] += w * s->ls[node][i];
        node = (node + 1) % s->L;
    }
    for (long i = 0; i < NR; ++i) s->U[i] = -Dt[i];
}

/* LBFGSDirectionUseGrad, lorads_alm.c:607-627 */
static void lbfgs_use_grad(osolver *s) {
    double ip = 0.0;
    for (int k = 0; k < s->K; ++k) {
        long len = s->off[k + 1] - s->off[k];
        ip += o_dot(len, s->U + s->off[k], s->G + s->off[k]);
    }
    if (ip >= 0)
        for (long i = 0; i < s->NR; ++i) s->U[i] = -s->G[i];
}

/* primalInfeasibility + gap, lorads_alg_common.c:386-394, :424-428 */
static void update_dimacs_alm(osolver *s, const double *X) {
    constr_val_all(s, X, X);
    for (int i = 0; i < s->m; ++i) s->vio[i] = s->p->b[i] - s->cvs[i];
    s->dimPinf = sqrt(o_dot(s->m, s->vio, s->vio)) / (1 + s->bNrm1);
    double gap = s->pObjVal - s->dObjVal;
    s->dimGap = fabs(gap) / (1 + fabs(s->pObjVal) + fabs(s->dObjVal));
}

/* LORADSCalObjRR_ALM, lorads_alm.c:1488-1497 */
static void cal_obj_rr(osolver *s, const double *X) {
    s->pObjVal = 0.0;
    for (int k = 0; k < s->K; ++k) {
        ocone *c = &s->p->cones[k];
        o_uvt(c, X + s->off[k], X + s->off[k], s->rank[k]);
        s->pObjVal += o_coeff_dot(&c->C, c->uvt);
    }
    s->pObjVal /= s->scaleObjHis;
}

static void cal_dual_obj(osolver *s) {   /* LORADSCalDualObj, lorads_alg_common.c:531-537 */
    s->dObjVal = o_dot(s->m, s->p->b, s->lam) / s->scaleObjHis;
}

/* ---- oracle rank: Gram + symmetric eigenvalues (lorads_logging.c:216-366) ---- */
static void jacobi_eigs(int n, double *A, double *w) {
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0.0;
        for (int i = 0; i < n; ++i) for (int j = i + 1; j < n; ++j) off += A[i * n + j] * A[i * n + j];
        if (off < 1e-30) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                double apq = A[p * n + q];
                if (fabs(apq) < 1e-300) continue;
                double app = A[p * n + p], aqq = A[q * n + q];
                double th = 0.5 * (aqq - app) / apq;
                double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
                double cs = 1.0 / sqrt(t * t + 1.0), sn = t * cs;
                for (int k = 0; k < n; ++k) {
                    double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = cs * akp - sn * akq; A[k * n + q] = sn * akp + cs * akq;
                }
                for (int k = 0; k < n; ++k) {
                    double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = cs * apk - sn * aqk; A[q * n + k] = sn * apk + cs * aqk;
                }
            }
    }
    for (int i = 0; i < n; ++i) w[i] = A[i * n + i];
}

static int count_significant(int r, double *gram, double eps) {
    double *w = malloc(sizeof(double) * r);
    jacobi_eigs(r, gram, w);
    double mx = -1e300;
    for (int i = 0; i < r; ++i) mx = OMAX(mx, w[i]);
    int cnt = 0;
    if (mx > 0) for (int i = 0; i < r; ++i) if (w[i] > eps * mx) cnt++;
    free(w);
    return cnt;
}

static int oracle_rank(osolver *s, int phase) {
    int tot = 0;
    for (int k = 0; k < s->K; ++k) {
        if (s->p->cones[k].lp) continue;   /* lorads_compute_oracle_rank: the SDP cones */
        int n = s->p->cones[k].n, r = s->rank[k];
        double *gram = calloc((long)r * r, 8);
        const double *X = s->R + s->off[k], *U = s->U + s->off[k], *V = s->V + s->off[k];
        for (int c1 = 0; c1 < r; ++c1)
            for (int c2 = c1; c2 < r; ++c2) {
                double sum = 0.0;
                for (int i = 0; i < n; ++i) {
                    if (phase == 1) sum += X[i + (long)c1 * n] * X[i + (long)c2 * n];
                    else sum += 0.5 * (U[i + (long)c1 * n] + V[i + (long)c1 * n]) *
                                0.5 * (U[i + (long)c2 * n] + V[i + (long)c2 * n]);
                }
                gram[c1 * r + c2] = gram[c2 * r + c1] = sum;
            }
        tot += count_significant(r, gram, 1e-6);
        free(gram);
    }
    return tot;
}

static int sum_rank(osolver *s) {
    int t = 0;
    for (int k = 0; k < s->K; ++k) t += s->p->cones[k].lp ? 0 : s->rank[k];
    return t;
}

static void append_traj(osolver *s, int phase, int cur, int orc) {
    int **cv = phase == 1 ? &s->traj1_cur : &s->traj2_cur, **ov = phase == 1 ? &s->traj1_orc : &s->traj2_orc;
    int *n = phase == 1 ? &s->n1 : &s->n2, *cap = phase == 1 ? &s->cap1 : &s->cap2;
    if (*n >= *cap) { *cap *= 2; *cv = realloc(*cv, sizeof(int) * *cap); *ov = realloc(*ov, sizeof(int) * *cap); }
    (*cv)[*n] = cur; (*ov)[*n] = orc; (*n)++;
}

static void record_state(osolver *s, int phase) {   /* ALMRecordState / ADMMRecordState */
    int cur = sum_rank(s);
    int orc = s->prm.disableOracle ? cur : oracle_rank(s, phase);
    append_traj(s, phase, cur, orc);
}

/* CheckAllRankMax, data/lorads_solver.c:1066-1082 */
static int check_all_rank_max(osolver *s, double f) {
    int cnt = 0;
    for (int k = 0; k < s->K; ++k) {
        if (s->p->cones[k].lp) continue;
        int nr = (int)OMIN(ceil(s->rank[k] * f), (double)s->p->cones[k].rank_max);
        if (nr >= s->p->cones[k].rank_max) cnt++;
    }
    return cnt == n_sdp(s);
}

static double *grow_cols(const double *old, long off_old_k, int n, int r_old, int r_new, long NR_new,
                         long off_new_k, double *dst, int diag) {
    memcpy(dst + off_new_k, old + off_old_k, sizeof(double) * (long)n * r_old);
    if (diag) {   /* lpRandomDiag, data/lorads_solver.c:1096-1106 */
        int aug = r_new - r_old, r = OMIN(n, aug);
        for (int i = 0; i < r; ++i) dst[off_new_k + (long)n * r_old + (long)i * n + i] = 1 / sqrt((double)r);
    }
    (void)NR_new;
    return dst;
}

/* AUG_RANK, data/lorads_solver.c:1154-1254 */
static int aug_rank(osolver *s, double f) {
    if (check_all_rank_max(s, 1.0)) return 1;
    int *nr = calloc(s->K, sizeof(int));
    long NRn = 0;
    long *offn = calloc(s->K + 1, sizeof(long));
    for (int k = 0; k < s->K; ++k) {
        nr[k] = (int)OMIN(ceil(s->rank[k] * f), (double)s->p->cones[k].rank_max);
        offn[k] = NRn; NRn += (long)s->p->cones[k].n * nr[k];
    }
    offn[s->K] = NRn;
    double *Rn = calloc(NRn, 8), *Un = calloc(NRn, 8), *Vn = calloc(NRn, 8), *Gn = calloc(NRn, 8), *M2n = calloc(NRn, 8);
    for (int k = 0; k < s->K; ++k) {
        int n = s->p->cones[k].n;
        grow_cols(s->U, s->off[k], n, s->rank[k], nr[k], NRn, offn[k], Un, 1);
        grow_cols(s->V, s->off[k], n, s->rank[k], nr[k], NRn, offn[k], Vn, 1);
        grow_cols(s->R, s->off[k], n, s->rank[k], nr[k], NRn, offn[k], Rn, 1);
        grow_cols(s->G, s->off[k], n, s->rank[k], nr[k], NRn, offn[k], Gn, 1);
        grow_cols(s->M2, s->off[k], n, s->rank[k], nr[k], NRn, offn[k], M2n, 0);
    }
    free(s->R); free(s->U); free(s->V); free(s->G); free(s->M2); free(s->Dtmp); free(s->bls);
    s->R = Rn; s->U = Un; s->V = Vn; s->G = Gn; s->M2 = M2n;
    s->Dtmp = calloc(NRn, 8); s->bls = calloc(NRn, 8);
    for (int q = 0; q < s->L; ++q) { free(s->ls[q]); free(s->ly[q]); s->ls[q] = calloc(NRn, 8); s->ly[q] = calloc(NRn, 8); }
    memcpy(s->rank, nr, sizeof(int) * s->K);
    memcpy(s->off, offn, sizeof(long) * (s->K + 1));
    s->NR = NRn;
    free(nr); free(offn);
    return check_all_rank_max(s, f);
}

/* LUtilUpdateCheckEma, lorads_utils.c:564-594 */
static int update_check_ema(double *cur, double *old, double v, double alpha, double thr, int interval, int *counter) {
    int result = 1;
    *cur = alpha * v + (1 - alpha) * (*cur);
    if (*counter >= interval) {
        if (*old != 0) {
            double ch = (*cur - *old) / *old;
            result = (ch >= -thr) && (ch <= thr);
        }
        *old = *cur;
        *counter = 1;
    } else {
        (*counter)++;
    }
    return result;
}

enum { EASY = 'e', MEDIUM = 'm', HARD = 'h', SUPER = 's' };

/* LORADS_ALMOptimize, lorads_alm.c:1220-1484 */
static int alm_optimize(osolver *s, ostate *st, double timeSolveStart, long inner_budget) {
    oparams *prm = &s->prm;
    int MAX_SUB = 5000;
    int is_rank_max = check_all_rank_max(s, 1.0);
    int retcode = 0;
    int last_outer_start = 1;
    double tau = 0.0;
    double rc, rc_tol, rc_val, lag;
    char difficulty;
    int localIter, clearL, rank_flag, rho_factor_flag;
    double rank_update_factor, rho_update_factor, rank_flag_thres = 15;
    int max_inc = 10000, max_ceil = 25000, upd_cnt = 0;
    int m = s->m;
ALG_START:
    upd_cnt = 0;   /* declared after the label in the reference (lorads_alm.c:1266) */
    rc = 0.1;
    rc_tol = rc / st->rho;
    lag = 0.0;
    constr_val_all(s, s->R, s->R);
    lag = alm_cal_grad(s, st->rho);
    rc_val = sqrt(lag) / (1 + s->cObjNrmInf);
    difficulty = HARD;
    localIter = 0; clearL = 0; rank_flag = 0;
    rank_update_factor = prm->rankUpdateFactor;
    rho_update_factor = prm->ALMRhoFactor;
    rho_factor_flag = 0;
    if (prm->dyrankLevel == 0) rank_flag_thres = 1e8;
    else if (prm->dyrankLevel == 1) rank_flag_thres = 150;
    else if (prm->dyrankLevel == 2) rank_flag_thres = 15;
    else if (prm->dyrankLevel == 3) rank_flag_thres = 5;
    for (long k = st->outerIter; k <= prm->maxALMIter; k++) {
        double ema_alpha = 0.1, ema_thr = 0.005, ema_cur = 0.0, ema_old = 0.0;
        int ema_int = 5, ema_cnt = 1;
        int cur_iter_counter = 1;
        if (upd_cnt >= 2) { upd_cnt = 0; MAX_SUB += max_inc; MAX_SUB = OMIN(MAX_SUB, max_ceil); }
        while (difficulty != EASY) {
            localIter = 0;
            int if_break = update_check_ema(&ema_cur, &ema_old, rc_val, ema_alpha, ema_thr, ema_int, &ema_cnt);
            if (!if_break && !prm->highAccMode) break;
            if (cur_iter_counter >= MAX_SUB) { upd_cnt += 1; break; }
            if (rank_flag >= rank_flag_thres && !is_rank_max && (k - last_outer_start >= 3)) break;
            if (rc_val <= rc_tol) break;
            while (rc_val - rc_tol > prm->endALMSubTol) {
                if (inner_budget > 0 && st->innerIter >= inner_budget) goto PRINT_AND_EXIT;
                if (localIter % 300 == 0) clearL = 0;
                lbfgs_direction(s, clearL);
                lbfgs_use_grad(s);
                double *q0 = s->M1;
                for (int i = 0; i < m; ++i) q0[i] = s->p->b[i] - s->cvs[i];
                /* ALMCalq12p12, lorads_alm.c:714-734 */
                double p1 = 2 * obj_constr_val_all(s, s->R, s->U, s->q1);
                for (int i = 0; i < m; ++i) s->q1[i] *= 2;
                double p2 = obj_constr_val_all(s, s->U, s->U, s->q2);
                int rn = alm_line_search(st->rho, m, s->lam, p1, p2, q0, s->q1, s->q2, &tau);
                if (rn == 0) { retcode = 4; goto END_ALM; }
                if (fabs(tau) < prm->endTauTol) {
                    st->innerIter++; localIter++; cur_iter_counter++; clearL++;
                    goto UpdateRho;
                }
                /* SetyAsNegGrad :768-783 */
                double *yh = s->ly[s->head];
                for (long i = 0; i < s->NR; ++i) yh[i] = -s->G[i];
                /* ALMupdateVar :826-830 */
                for (long i = 0; i < s->NR; ++i) s->R[i] += tau * s->U[i];
                double tau2 = tau * tau;
                for (int i = 0; i < m; ++i) s->cvs[i] += tau * s->q1[i];
                for (int i = 0; i < m; ++i) s->cvs[i] += tau2 * s->q2[i];
                lag = alm_cal_grad(s, st->rho);
                /* setlbfgsHisTwo :842-863 */
                double *sh = s->ls[s->head];
                for (long i = 0; i < s->NR; ++i) { sh[i] = tau * s->U[i]; yh[i] += s->G[i]; }
                s->lbeta[s->head] = 1.0 / o_dot(s->NR, yh, sh);
                s->head = (s->head + 1) % s->L;
                update_dimacs_alm(s, s->R);
                st->pinf1 = s->dimPinf;
                st->pinfinf = st->pinf1 * (1 + s->bNrm1) / (1 + s->bNrmInf);
                if ((st->pinfinf <= prm->phase1Tol) && ((st->gap <= prm->phase1Tol) || (!prm->highAccMode))) {
                    st->outerIter = k; st->innerIter += 1; localIter += 1; cur_iter_counter += 1; clearL += 1;
                    goto END_ALM;
                }
                rc_val = sqrt(lag) / (1 + s->cObjNrmInf);
                st->innerIter += 1; localIter++; cur_iter_counter++; clearL++;
                if (localIter > 800) break;
            }
            /* LORADSUpdateDualVar, lorads_alg_common.c:511-524 */
            for (int i = 0; i < m; ++i) s->lam[i] += st->rho * s->p->b[i];
            for (int i = 0; i < m; ++i) s->lam[i] += -st->rho * s->cvs[i];
            lag = alm_cal_grad(s, st->rho);
            rc_val = sqrt(lag) / (1 + s->cObjNrmInf);
            if (localIter <= 20) difficulty = EASY;
            else if (localIter <= 100) { difficulty = MEDIUM; rank_flag += 2; }
            else if (localIter < 400) { difficulty = HARD; rank_flag += 3; }
            else { difficulty = SUPER; rank_flag += 4; }
            if (difficulty == EASY) rank_flag = 0;
        }
    UpdateRho:
        do {
            st->rho *= rho_update_factor;
            lag = alm_cal_grad(s, st->rho);
            rc_val = sqrt(lag) / (1 + s->cObjNrmInf);
            rc_tol = rc / st->rho;
        } while (rc_tol >= rc_val);
        if (st->rho >= 5e4 && rho_factor_flag < 4) { rho_update_factor = sqrt(sqrt(rho_update_factor)); rho_factor_flag = 4; }
        else if (st->rho >= 5e6 && rho_factor_flag < 6) { rho_update_factor = sqrt(sqrt(rho_update_factor)); rho_factor_flag = 6; }
        else if (st->rho >= 5e8 && rho_factor_flag < 8) { rho_update_factor = sqrt(sqrt(rho_update_factor)); rho_factor_flag = 8; }
        difficulty = HARD;
        clearL = 0;
        st->outerIter = k;
        {
            if ((st->pinfinf <= prm->phase1Tol) && ((st->gap <= prm->phase1Tol) || (!prm->highAccMode))) goto END_ALM;
            cal_obj_rr(s, s->R);
            cal_dual_obj(s);
            update_dimacs_alm(s, s->R);
            st->gap = s->dimGap; st->pobj = s->pObjVal; st->dobj = s->dObjVal;
            st->pinf1 = s->dimPinf;
            st->pinfinf = st->pinf1 * (1 + s->bNrm1) / (1 + s->bNrmInf);
            if (st->gap <= prm->phase1Tol * 1e-3 && st->pinf1 <= prm->phase1Tol * 1e-3) goto PRINT_AND_EXIT;
            record_state(s, 1);
            if (getenv("ORACLE_VERBOSE"))
                printf("ALM OuterIter:%ld InnerIter:%ld pObj:%.10e dObj:%.10e pInfea(1):%.6e rho:%g rank:%d\n",
                       st->outerIter, st->innerIter, st->pobj, st->dobj, st->pinf1, st->rho, s->rank[0]);
            if (o_now() - timeSolveStart >= prm->timeSecLimit) goto PRINT_AND_EXIT;
        }
        if (rank_flag >= rank_flag_thres && !is_rank_max) {
            rank_flag = 0;
            if (k - last_outer_start >= 2) {
                is_rank_max = aug_rank(s, rank_update_factor);
                st->outerIter = k;
                last_outer_start = (int)st->outerIter;
                goto ALG_START;
            }
        }
    }
END_ALM:
    cal_obj_rr(s, s->R);
    cal_dual_obj(s);
    update_dimacs_alm(s, s->R);
    st->pobj = s->pObjVal; st->dobj = s->dObjVal; st->gap = s->dimGap;
    st->pinf1 = s->dimPinf;
    st->pinfinf = st->pinf1 * (1 + s->bNrm1) / (1 + s->bNrmInf);
PRINT_AND_EXIT:
    record_state(s, 1);
    return retcode;
}

/* ----------------------------- ADMM phase ----------------------------- */
/* LORADSUpdateConstrValCG + linSysProduct, lorads_admm.c:442-486: res = A^*(A(sym(xV^T)))V + x */
static void lin_sys_product(osolver *s, int k, const double *V, const double *x, double *res) {
    ocone *c = &s->p->cones[k];
    int r = s->rank[k];
    long len = (long)c->n * r;
    o_uvt(c, x, V, r);
    double *w = s->M1;
    for (int i = 0; i < c->ncoef; ++i) w[c->con[i]] = o_coeff_dot(&c->A[i], c->uvt);
    o_wsum(c, w, 0, s->S);
    o_spmm(c, s->S, V, r, res);
    for (long i = 0; i < len; ++i) res[i] += x[i];
}

static double o_nrm1(long n, const double *x) { double a = 0; for (long i = 0; i < n; ++i) a += fabs(x[i]); return a; }

/* CGSolve, linalg/lorads_cgs.c:128-287 */
static void cg_solve(osolver *s, int k, const double *V, double *x, const double *b, double tol, int maxit) {
    long nr = (long)s->p->cones[k].n * s->rank[k];
    double *r = calloc(nr, 8), *p = calloc(nr, 8), *q = calloc(nr, 8), *qn = calloc(nr, 8), *Q = calloc(nr, 8);
    int nRestart = 20;
    double bNorm = o_nrm1(nr, b);
    lin_sys_product(s, k, V, x, r);
    for (long i = 0; i < nr; ++i) r[i] = -(r[i] - b[i]);
    double resi = sqrt(o_dot(nr, r, r));
    if (resi / bNorm < tol) goto done;
    memcpy(p, r, 8 * nr); memcpy(q, r, 8 * nr);
    double qTr = o_dot(nr, q, r);
    s->cgIterCone[k] = 0;
    for (int it = 0; it < maxit; ++it) {
        s->cgIterCone[k] += 1;
        lin_sys_product(s, k, V, p, Q);
        qTr = o_dot(nr, q, r);
        double pTQ = o_dot(nr, p, Q);
        double alpha = qTr / pTQ;
        for (long i = 0; i < nr; ++i) x[i] += alpha * p[i];
        for (long i = 0; i < nr; ++i) r[i] += -alpha * Q[i];
        resi = sqrt(o_dot(nr, r, r));
        if (resi / bNorm < tol) goto done;
        if (it % nRestart == 0) {
            lin_sys_product(s, k, V, x, r);
            for (long i = 0; i < nr; ++i) r[i] = -(r[i] - b[i]);
            memcpy(p, r, 8 * nr); memcpy(q, r, 8 * nr);
            qTr = o_dot(nr, q, r);
        }
        memcpy(qn, r, 8 * nr);
        double qTrNew = o_dot(nr, qn, r);
        double beta = qTrNew / qTr;
        for (long i = 0; i < nr; ++i) p[i] = beta * p[i] + r[i];
        qTr = qTrNew;
        memcpy(q, qn, 8 * nr);
    }
done:
    free(r); free(p); free(q); free(qn); free(Q);
}

/* LORADSUpdateSDPVarOne, lorads_admm.c:564-616: solve for X (=U or V) with Y fixed */
static void update_var_one(osolver *s, int k, double *X, const double *Y, double rho, double tol, int maxit) {
    ocone *c = &s->p->cones[k];
    int m = s->m;
    long len = (long)c->n * s->rank[k];
    const double *cv = s->cvc + (long)k * m;
    for (int i = 0; i < m; ++i) s->M1[i] = -s->p->b[i];
    for (int i = 0; i < m; ++i) s->M1[i] += s->cvs[i];
    for (int i = 0; i < m; ++i) s->M1[i] += -cv[i];
    for (int i = 0; i < m; ++i) s->M1[i] *= rho;
    for (int i = 0; i < m; ++i) s->M1[i] += -s->lam[i];
    o_wsum(c, s->M1, 1, s->S);
    double *M2 = s->M2 + s->off[k];
    o_spmm(c, s->S, Y, s->rank[k], M2);
    for (long i = 0; i < len; ++i) M2[i] += -rho * Y[i];
    double *bl = s->bls + s->off[k];
    for (long i = 0; i < len; ++i) bl[i] = (-1.0 / rho) * M2[i];
    cg_solve(s, k, Y, X, bl, tol, maxit);
    s->cgIter += s->cgIterCone[k];
}

/* LORADSUpdateConstrVal for one cone + running sum, lorads_alg_common.c:308-324 */
static void refresh_cone_constr(osolver *s, int k) {
    ocone *c = &s->p->cones[k];
    double *cv = s->cvc + (long)k * s->m;
    for (int i = 0; i < s->m; ++i) s->cvs[i] -= cv[i];
    o_uvt(c, s->U + s->off[k], s->V + s->off[k], s->rank[k]);
    o_cone_auv(c, cv);
    for (int i = 0; i < s->m; ++i) s->cvs[i] += cv[i];
}

/* the LP block's loop of LORADSUpdateSDPLPVar (lorads_alg_common.c:352-372): per column j in
   order, LORADSUpdateLPVarOne (lorads_admm.c:759-792) for u_j with v_j fixed, the constraint
   sums refreshed (constrValLP add / recompute / add), then v_j with u_j fixed */
static void lp_update_var(osolver *s, int k, double rho) {
    ocone *c = &s->p->cones[k];
    double *u = s->U + s->off[k], *v = s->V + s->off[k], *cv = s->cvc + (long)k * s->m;
    const double *b = s->p->b;
    for (int j = 0; j < c->n; ++j) {
        for (int side = 0; side < 2; ++side) {
            double uv = u[j] * v[j];
            double w = 0.0;
            w += c->lp_c[j];
            for (int e = c->lp_ptr[j]; e < c->lp_ptr[j + 1]; ++e) {
                int i = c->lp_con[e];
                double a = c->lp_a[e];
                double m1 = -b[i];
                m1 = m1 + s->cvs[i];
                m1 = m1 + (-1.0) * (uv * a);
                m1 = m1 * rho;
                m1 = m1 + (-1.0) * s->lam[i];
                w += a * m1;
            }
            double y = side == 0 ? v[j] : u[j];
            double M2 = w * y;
            M2 = M2 - rho * y;
            double x = (-1.0 * M2 / rho) / (1 + c->lp_nrm2[j] * y * y);
            if (side == 0) u[j] = x; else v[j] = x;
            double uvn = u[j] * v[j];
            for (int e = c->lp_ptr[j]; e < c->lp_ptr[j + 1]; ++e) {
                int i = c->lp_con[e];
                s->cvs[i] += (-1.0) * (uv * c->lp_a[e]);
                cv[i] += (-1.0) * (uv * c->lp_a[e]);
            }
            for (int e = c->lp_ptr[j]; e < c->lp_ptr[j + 1]; ++e) {
                int i = c->lp_con[e];
                s->cvs[i] += 1.0 * (uvn * c->lp_a[e]);
                cv[i] += 1.0 * (uvn * c->lp_a[e]);
            }
        }
    }
}

/* LORADSUpdateSDPVar, lorads_alg_common.c:298-326 (+ the LP block's loop after the cones) */
static void admm_update_var(osolver *s, double rho, double tol, int maxit) {
    for (int k = 0; k < s->K; ++k) {
        if (s->p->cones[k].lp) continue;
        update_var_one(s, k, s->U + s->off[k], s->V + s->off[k], rho, tol, maxit);
        refresh_cone_constr(s, k);
        update_var_one(s, k, s->V + s->off[k], s->U + s->off[k], rho, tol, maxit);
        refresh_cone_constr(s, k);
    }
    for (int k = 0; k < s->K; ++k)
        if (s->p->cones[k].lp) lp_update_var(s, k, rho);
}

static void average_uv(osolver *s) {   /* averageUV, lorads_admm.c:372-377 */
    for (long i = 0; i < s->NR; ++i) s->R[i] = (s->U[i] + s->V[i]) / 2;
}

static void cal_obj_admm(osolver *s) { average_uv(s); cal_obj_rr(s, s->R); }   /* :398-410 */

static void update_dimacs_admm(osolver *s) {   /* lorads_alg_common.c:454-462 */
    average_uv(s);
    update_dimacs_alm(s, s->R);
}

/* LORADSADMMOptimize, lorads_admm.c:84-209 */
static int admm_optimize(osolver *s, ostate *st, long iter_ceiling, double timeSolveStart) {
    oparams *prm = &s->prm;
    if (st->gap <= prm->phase2Tol && st->pinf1 <= prm->phase2Tol) return 0;
    int maxCG = 800;
    st->rho = OMIN(st->rho, prm->rhoMax);
    s->cgIter = 0;
    constr_val_all(s, s->U, s->V);
    cal_obj_admm(s);
    cal_dual_obj(s);
    update_dimacs_admm(s);
    st->pobj = s->pObjVal; st->dobj = s->dObjVal; st->gap = s->dimGap; st->pinf1 = s->dimPinf;
    st->pinfinf = st->pinf1 * (1 + s->bNrm1) / (1 + s->bNrmInf);
    double cur_rho_max = prm->rhoMax, old_mean = 1e30, buf[10] = {0};
    int bad_pd = 0, count = 0;
    while (st->iter <= prm->maxADMMIter || st->gap >= prm->phase2Tol || st->pinf1 >= prm->phase2Tol) {
        if (st->iter >= iter_ceiling) break;
        double cgtol = OMIN(st->pinf1 * 1e-2, 1e-8);
        admm_update_var(s, st->rho, cgtol, maxCG);
        st->cg_iter = s->cgIter;
        cal_obj_admm(s);
        cal_dual_obj(s);
        update_dimacs_admm(s);
        st->pobj = s->pObjVal; st->dobj = s->dObjVal; st->pinf1 = s->dimPinf;
        st->pinfinf = st->pinf1 * (1 + s->bNrm1) / (1 + s->bNrmInf);
        st->gap = s->dimGap;
        record_state(s, 2);
        if (st->pinfinf >= 1e10 || st->gap >= 1 - 1e-8) return 4;
        if (st->gap <= prm->phase2Tol * 5) { bad_pd -= 5; bad_pd = OMAX(0, bad_pd); }
        else if (st->gap <= prm->phase2Tol) { bad_pd -= 10; bad_pd = OMAX(0, bad_pd); }
        if (st->gap >= prm->phase1Tol * 1e2) bad_pd += 2;
        if (bad_pd >= 800) return 0;
        buf[count % 10] = st->pinfinf;
        if (st->pinfinf <= prm->phase2Tol) {
            update_dimacs_admm(s);
            st->pobj = s->pObjVal; st->dobj = s->dObjVal; st->gap = s->dimGap; st->pinf1 = s->dimPinf;
            return 0;
        }
        for (int i = 0; i < s->m; ++i) s->lam[i] += st->rho * s->p->b[i];
        for (int i = 0; i < s->m; ++i) s->lam[i] += -st->rho * s->cvs[i];
        if ((st->iter + 1) % prm->rhoFreq == 0) {
            st->rho *= prm->rhoFactor;
            if (st->rho >= cur_rho_max) {
                st->rho = cur_rho_max;
                if ((st->iter + 1) % (prm->rhoFreq * 100) == 0) {
                    double mean = o_nrm1(10, buf) / 10.0;
                    if (mean / old_mean >= 0.65) {
                        st->rho *= pow(prm->rhoFactor, round(log(prm->rhoFreq * 100) / log(prm->rhoFreq)));
                        cur_rho_max = st->rho;
                    }
                    old_mean = mean;
                }
            }
            if (st->rho >= prm->rhoCellingADMM) st->rho = prm->rhoCellingADMM;
        }
        if (st->iter % 50 == 0) {
            update_dimacs_admm(s);
            st->pobj = s->pObjVal; st->dobj = s->dObjVal; st->gap = s->dimGap; st->pinf1 = s->dimPinf;
            if (o_now() - timeSolveStart >= prm->timeSecLimit) return 1;
        }
        if (st->gap <= prm->phase2Tol * 1e-3 && st->pinf1 <= prm->phase2Tol * 1e-3) return 0;
        st->iter++;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
static void default_oparams(oparams *p) {   /* initCommandLineArgs, main.c:56-86 */
    memset(p, 0, sizeof(*p));
    p->initRho = 0.0; p->rhoMax = 5000.0; p->rhoCellingALM = 1e8; p->rhoCellingADMM = 5000.0 * 200;
    p->maxALMIter = 200; p->maxADMMIter = 10000; p->timesLogRank = 2.0; p->fixedRank = -1;
    p->initRank = -1; p->rhoFreq = 5; p->rhoFactor = 1.2; p->ALMRhoFactor = 2.0;
    p->rankUpdateFactor = 1.5; p->phase1Tol = 1e-3; p->phase2Tol = 1e-5; p->timeSecLimit = 3600.0;
    p->heuristicFactor = 1.0; p->lbfgsListLength = 2; p->endTauTol = 1e-16; p->endALMSubTol = 1e-10;
    p->reoptLevel = 2; p->dyrankLevel = 2; p->highAccMode = 0;
}

static void parse_oflags(oparams *p, int n, char **f) {
    for (int i = 0; i < n; ++i) {
        const char *k = f[i];
        if (!strncmp(k, "--", 2)) k += 2;
        if (!strcmp(k, "disableOracle")) { p->disableOracle = 1; continue; }
        if (i + 1 >= n) break;
        const char *v = f[++i];
        double d = atof(v);
        if (!strcmp(k, "initRho")) p->initRho = d;
        else if (!strcmp(k, "rhoMax")) p->rhoMax = d;
        else if (!strcmp(k, "maxALMIter")) p->maxALMIter = atoi(v);
        else if (!strcmp(k, "maxADMMIter")) p->maxADMMIter = atoi(v);
        else if (!strcmp(k, "timesLogRank")) p->timesLogRank = d;
        else if (!strcmp(k, "fixedRank")) p->fixedRank = atoi(v);
        else if (!strcmp(k, "initRank")) p->initRank = atoi(v);
        else if (!strcmp(k, "rhoFreq")) p->rhoFreq = atoi(v);
        else if (!strcmp(k, "rhoFactor")) p->rhoFactor = d;
        else if (!strcmp(k, "ALMRhoFactor")) p->ALMRhoFactor = d;
        else if (!strcmp(k, "rankUpdateFactor")) p->rankUpdateFactor = d;
        else if (!strcmp(k, "phase1Tol")) p->phase1Tol = d;
        else if (!strcmp(k, "phase2Tol")) p->phase2Tol = d;
        else if (!strcmp(k, "timeSecLimit")) p->timeSecLimit = d;
        else if (!strcmp(k, "heuristicFactor")) p->heuristicFactor = d;
        else if (!strcmp(k, "lbfgsListLength")) p->lbfgsListLength = atoi(v);
        else if (!strcmp(k, "endTauTol")) p->endTauTol = d;
        else if (!strcmp(k, "endALMSubTol")) p->endALMSubTol = d;
        else if (!strcmp(k, "reoptLevel")) p->reoptLevel = atoi(v);
        else if (!strcmp(k, "dyrankLevel")) p->dyrankLevel = atoi(v);
        else if (!strcmp(k, "highAccMode")) p->highAccMode = atoi(v);
    }
    p->rhoCellingADMM = p->rhoMax * 200;   /* main.c:350 */
}

/* main.c:380-610 with reoptLevel 0 semantics (the ARPACK dual-infeasibility
   step, main.c:515, is not restated: it is off the hot path). */
int oracle_solve(const char *path, int nflags, char **flags, double *res) {
    oparams prm;
    default_oparams(&prm);
    parse_oflags(&prm, nflags, flags);
    oproblem *p = oracle_read(path);
    if (!p) return -1;
    double tss = o_now();
    osolver *s = osolver_new(p, &prm);
    ostate alm = {0}, admm = {0};
    double rho = prm.initRho;
    if (rho == 0) {   /* initial_solver_state, data/lorads_solver.c:1599-1606: the SDP blocks */
        long sd = 0;
        for (int k = 0; k < s->K; ++k) sd += p->cones[k].lp ? 0 : p->cones[k].n;
        rho = 1 / sqrt((double)sd);
    }
    alm.rho = rho; admm.rho = rho;
    alm.pobj = alm.dobj = alm.pinf1 = alm.pinfinf = 1e30; alm.gap = 0.0;
    admm.pobj = admm.dobj = admm.pinf1 = admm.pinfinf = admm.gap = 1e30;
    double t0 = o_now();
    alm_optimize(s, &alm, tss, 0);
    double t_alm = o_now() - t0;
    long alm_inner = alm.innerIter;
    if (o_now() - tss > prm.timeSecLimit) goto END;   /* main.c:451-455 */
    /* LORADS_ALMtoADMM, data/lorads_solver.c:1351-1387 */
    memcpy(s->V, s->R, 8 * s->NR);
    memcpy(s->U, s->V, 8 * s->NR);
    admm.pinf1 = alm.pinf1; admm.pinfinf = alm.pinfinf; admm.gap = alm.gap;
    admm.rho = alm.rho * prm.heuristicFactor;
    if (alm.rho > prm.rhoMax) {
        admm.rho = OMIN(sqrt(OMAX(prm.rhoMax, alm.rho) / prm.rhoMax) * prm.rhoMax, alm.rho);
        s->prm.rhoMax = admm.rho;
    }
    admm_optimize(s, &admm, s->prm.maxADMMIter, tss);
END:;
    double all_time = o_now() - t0;
    /* main.c:519-525 */
    admm.gap = s->dimGap;
    admm.pinf1 = s->dimPinf;
    admm.pinfinf = s->dimPinf * (1 + s->bNrm1) / (1 + s->bNrmInf);
    if (res) {
        double v[16] = {(double)alm_inner, (double)alm.outerIter, alm.pobj, alm.dobj, alm.pinf1, alm.gap, alm.rho,
                        (double)admm.iter, admm.pobj, admm.dobj, admm.pinf1, admm.gap, admm.rho,
                        all_time, (double)s->rank[0], t_alm};
        memcpy(res, v, sizeof(v));
    }
    osolver_free(s);
    oracle_free(p);
    return 0;
}

long oracle_alm_rate(const char *path, int rank, double seconds, double *elapsed) {
    oparams prm;
    default_oparams(&prm);
    prm.fixedRank = rank;
    prm.phase1Tol = 1e-300;
    prm.maxALMIter = 100000;
    prm.timeSecLimit = seconds;
    prm.disableOracle = 1;
    oproblem *p = oracle_read(path);
    if (!p) return -1;
    osolver *s = osolver_new(p, &prm);
    ostate alm = {0};
    long sd = 0;
    for (int k = 0; k < s->K; ++k) sd += p->cones[k].lp ? 0 : p->cones[k].n;
    alm.rho = 1 / sqrt((double)sd);
    alm.pobj = alm.dobj = alm.pinf1 = alm.pinfinf = 1e30;
    double t0 = o_now();
    alm_optimize(s, &alm, t0, 0);
    if (elapsed) *elapsed = o_now() - t0;
    long it = alm.innerIter;
    osolver_free(s);
    oracle_free(p);
    return it;
}

/* Exactly K ALM inner iterations from the reference's initial point (phase 1 with an inner
 * budget, lorads_alm.c:1302-1379 between the budget checks); out = R, G (col-major per cone,
 * cones concatenated), A(RR^T), lambda.  Returns NR (doubles per factor) or -1. */
long oracle_alm_steps(const char *path, int rank, long K, double *out, long cap) {
    oparams prm;
    default_oparams(&prm);
    prm.fixedRank = rank;
    prm.reoptLevel = 0;
    prm.disableOracle = 1;
    oproblem *p = oracle_read(path);
    if (!p) return -1;
    osolver *s = osolver_new(p, &prm);
    ostate alm = {0};
    long sd = 0;
    for (int k = 0; k < s->K; ++k) sd += p->cones[k].lp ? 0 : p->cones[k].n;
    alm.rho = 1 / sqrt((double)sd);
    alm.pobj = alm.dobj = alm.pinf1 = alm.pinfinf = 1e30;
    alm_optimize(s, &alm, o_now(), K);
    long NR = s->NR, need = 2 * NR + 2 * s->m;
    if (need <= cap) {
        memcpy(out, s->R, 8 * NR);
        memcpy(out + NR, s->G, 8 * NR);
        memcpy(out + 2 * NR, s->cvs, 8 * s->m);
        memcpy(out + 2 * NR + s->m, s->lam, 8 * s->m);
    }
    long inner = alm.innerIter;
    osolver_free(s);
    oracle_free(p);
    return inner == K && need <= cap ? NR : -1;
}

/* Same layout as oracle/ref_harness.c mode_kernels. */
int oracle_kernels(oproblem *p, int rank, const double *in, double *out) {
    oparams prm;
    default_oparams(&prm);
    prm.fixedRank = rank;
    osolver *s = osolver_new(p, &prm);
    long NR = s->NR;
    int m = s->m;
    const double *ip = in;
    const double *R = ip; ip += NR;
    const double *D = ip; ip += NR;
    const double *G = ip; ip += NR;
    const double *s1 = ip; ip += NR;
    const double *y1 = ip; ip += NR;
    const double *s2 = ip; ip += NR;
    const double *y2 = ip; ip += NR;
    const double *U = ip; ip += NR;
    const double *V = ip; ip += NR;
    const double *lam = ip; ip += m;
    const double *cvs = ip; ip += m;
    double rho = *ip++, beta1 = *ip++, beta2 = *ip++, rho_admm = *ip++, cg_tol = *ip++;
    double *op = out;
    /* (1) */
    memcpy(s->R, R, 8 * NR); memcpy(s->U, D, 8 * NR);
    double p1 = 2 * obj_constr_val_all(s, s->R, s->U, s->q1);
    for (int i = 0; i < m; ++i) s->q1[i] *= 2;
    double p2 = obj_constr_val_all(s, s->U, s->U, s->q2);
    memcpy(op, s->q1, 8 * m); op += m; *op++ = p1;
    memcpy(op, s->q2, 8 * m); op += m; *op++ = p2;
    /* (2) */
    s->pObjVal = 0; s->dObjVal = 0;
    update_dimacs_alm(s, s->R);
    memcpy(op, s->cvs, 8 * m); op += m; *op++ = s->dimPinf;
    cal_obj_rr(s, s->R);
    *op++ = s->pObjVal;
    /* (3) */
    memcpy(s->lam, lam, 8 * m); memcpy(s->cvs, cvs, 8 * m);
    double lag = alm_cal_grad(s, rho);
    memcpy(op, s->G, 8 * NR); op += NR; *op++ = lag;
    /* (4) */
    {
        double *q0 = malloc(8 * m);
        for (int i = 0; i < m; ++i) q0[i] = p->b[i] - cvs[i];
        double tau = 0.0;
        int rn = alm_line_search(rho, m, lam, p1, p2, q0, s->q1, s->q2, &tau);
        *op++ = tau; *op++ = (double)rn;
        free(q0);
    }
    /* (5) */
    memcpy(s->G, G, 8 * NR);
    s->head = 0;
    int newest = (s->head - 1 + s->L) % s->L, older = (newest - 1 + s->L) % s->L;
    memcpy(s->ls[newest], s1, 8 * NR); memcpy(s->ly[newest], y1, 8 * NR); s->lbeta[newest] = beta1;
    memcpy(s->ls[older], s2, 8 * NR); memcpy(s->ly[older], y2, 8 * NR); s->lbeta[older] = beta2;
    lbfgs_direction(s, 5);
    lbfgs_use_grad(s);
    memcpy(op, s->U, 8 * NR); op += NR;
    lbfgs_direction(s, 1);
    lbfgs_use_grad(s);
    memcpy(op, s->U, 8 * NR); op += NR;
    /* (6) */
    memcpy(s->U, U, 8 * NR); memcpy(s->V, V, 8 * NR);
    memcpy(s->lam, lam, 8 * m);
    constr_val_all(s, s->U, s->V);
    s->cgIter = 0;
    update_var_one(s, 0, s->U + s->off[0], s->V + s->off[0], rho_admm, cg_tol, 800);
    memcpy(op, s->U, 8 * NR); op += NR;
    long len0 = s->off[1] - s->off[0];
    memcpy(op, s->bls, 8 * len0); op += len0;
    *op++ = (double)s->cgIterCone[0];
    osolver_free(s);
    return (int)(op - out);
}

/* One ADMM variable update over every cone (LORADSUpdateSDPVar, lorads_alg_common.c:298-326)
 * and the dual update after it (LORADSUpdateDualVar, :511-524) on the `kernels` input layout's
 * U, V, lambda, rho_admm, cg_tol: out = U, V, A(UV^T) summed, lambda, total CG iterations,
 * per cone its last (V-side) CG count -- what oracle/ref_harness.c `admm_sweep` dumps. */
int oracle_admm_sweep(oproblem *p, int rank, const double *in, double *out) {
    oparams prm;
    default_oparams(&prm);
    prm.fixedRank = rank;
    osolver *s = osolver_new(p, &prm);
    long NR = s->NR;
    int m = s->m;
    const double *U = in + 7 * NR, *V = in + 8 * NR, *lam = in + 9 * NR;
    const double *tail = in + 9 * NR + 2 * m;
    const double rho = tail[3], cg_tol = tail[4];
    memcpy(s->U, U, 8 * NR); memcpy(s->V, V, 8 * NR);
    memcpy(s->lam, lam, 8 * m);
    constr_val_all(s, s->U, s->V);
    s->cgIter = 0;
    admm_update_var(s, rho, cg_tol, 800);
    for (int i = 0; i < m; ++i) s->lam[i] += rho * s->p->b[i];
    for (int i = 0; i < m; ++i) s->lam[i] += -rho * s->cvs[i];
    double *op = out;
    memcpy(op, s->U, 8 * NR); op += NR;
    memcpy(op, s->V, 8 * NR); op += NR;
    memcpy(op, s->cvs, 8 * m); op += m;
    memcpy(op, s->lam, 8 * m); op += m;
    *op++ = (double)s->cgIter;
    for (int k = 0; k < s->K; ++k) *op++ = (double)s->cgIterCone[k];
    osolver_free(s);
    return (int)(op - out);
}

/* oracle/ref_harness.c admm_sweep_lp's layout: in = U, V (the LP block after the SDP cones),
 * lambda[m], rho_admm, cg_tol; out = U, V, constrValSum, lambda (after the dual update), total
 * CG iterations.  LORADSUpdateSDPLPVar + LORADSUpdateDualVar. */
int oracle_admm_sweep_lp(oproblem *p, int rank, const double *in, double *out) {
    oparams prm;
    default_oparams(&prm);
    prm.fixedRank = rank;
    osolver *s = osolver_new(p, &prm);
    long NR = s->NR;
    int m = s->m;
    memcpy(s->U, in, 8 * NR); memcpy(s->V, in + NR, 8 * NR);
    memcpy(s->lam, in + 2 * NR, 8 * m);
    const double rho = in[2 * NR + m], cg_tol = in[2 * NR + m + 1];
    constr_val_all(s, s->U, s->V);
    s->cgIter = 0;
    admm_update_var(s, rho, cg_tol, 800);
    for (int i = 0; i < m; ++i) s->lam[i] += rho * s->p->b[i];
    for (int i = 0; i < m; ++i) s->lam[i] += -rho * s->cvs[i];
    double *op = out;
    memcpy(op, s->U, 8 * NR); op += NR;
    memcpy(op, s->V, 8 * NR); op += NR;
    memcpy(op, s->cvs, 8 * m); op += m;
    memcpy(op, s->lam, 8 * m); op += m;
    *op++ = (double)s->cgIter;
    osolver_free(s);
    return (int)(op - out);
}

/* Test hook: first n outputs of the restated glibc generator. */
int oracle_rand_seq(unsigned seed, int n, int *out) {
    grand_t g;
    grand_seed(&g, seed);
    for (int i = 0; i < n; ++i) out[i] = grand_next(&g);
    return n;
}
