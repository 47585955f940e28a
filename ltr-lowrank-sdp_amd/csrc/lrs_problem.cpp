// lrs_problem.cpp -- SDPA reader and presolve (host), producing the device
// formats described in lrs_device.h.  Reference semantics:
//   reader    io/lorads_file_io.c:59-455
//   presolve  data/lorads_sdp_conic.c:1185-1393 (union pattern + slot maps)
//             data/lorads_sdp_data.c:313-329     (nnzIdx2ResIdx)
// The presolve is sort-based (O(Z log Z)) instead of the reference's chained
// hash (data/lorads_sdp_data.c:48-69), which dominates its wall time at large m.
#include "lrs_problem.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace lrs {

namespace {

struct RawEntry {
    int cone, con, row, col;   // row >= col
    double v;
};

bool is_sep(char c) {
    return c == '{' || c == '}' || c == '(' || c == ')' || c == ',' || c == '\'' || c == ' ' || c == '\t' ||
           c == '\r' || c == '\n';
}

}  // namespace

static bool build_problem(int m, int K, const std::vector<int> &dims, int nLp, bool lpEntries,
                          std::vector<RawEntry> &raw, HostProblem &hp, std::string &err, bool allow_dense = true);

bool read_sdpa(const std::string &path, HostProblem &hp, std::string &err) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) { err = "cannot open " + path; return false; }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::string s;
    s.resize(sz);
    if (sz > 0 && fread(&s[0], 1, sz, f) != (size_t)sz) { fclose(f); err = "short read"; return false; }
    fclose(f);
    size_t pos = 0;
    auto next_line = [&](std::string &line) -> bool {
        if (pos >= s.size()) return false;
        size_t e = s.find('\n', pos);
        if (e == std::string::npos) e = s.size();
        line.assign(s, pos, e - pos);
        pos = e + 1;
        return true;
    };
    std::string line;
    do {
        if (!next_line(line)) { err = "empty file"; return false; }
    } while (!line.empty() && (line[0] == '*' || line[0] == '"'));
    int m = 0, nb = 0;
    if (sscanf(line.c_str(), "%d", &m) != 1) { err = "bad constraint count"; return false; }
    if (!next_line(line) || sscanf(line.c_str(), "%d", &nb) != 1) { err = "bad block count"; return false; }
    std::vector<int> dims(nb);
    auto skip = [&]() { while (pos < s.size() && is_sep(s[pos])) pos++; return pos < s.size(); };
    for (int k = 0; k < nb; ++k) {
        if (!skip()) { err = "bad block sizes"; return false; }
        char *endp;
        long d = strtol(s.c_str() + pos, &endp, 10);
        if (endp == s.c_str() + pos) { err = "bad block size token"; return false; }
        pos = endp - s.c_str();
        if (k < nb - 1 && d <= 0) { err = "only the last block may be an LP block"; return false; }
        dims[k] = (int)d;
    }
    int K = nb, nLp = 0;
    if (nb > 0 && dims[nb - 1] < 0) { nLp = -dims[nb - 1]; K = nb - 1; }
    hp.b.assign(m, 0.0);
    for (int i = 0; i < m; ++i) {
        if (!skip()) { err = "bad rhs"; return false; }
        char *endp;
        double v = strtod(s.c_str() + pos, &endp);
        if (endp == s.c_str() + pos) { pos++; --i; continue; }
        pos = endp - s.c_str();
        hp.b[i] = v;
    }
    while (pos < s.size() && s[pos] != '\n') pos++;
    if (pos < s.size()) pos++;
    std::vector<RawEntry> raw;
    raw.reserve(1 << 16);
    bool lpEntries = false;
    while (next_line(line)) {
        int ic, ib, ii, ij;
        double v;
        if (sscanf(line.c_str(), "%d %d %d %d %lg", &ic, &ib, &ii, &ij, &v) != 5) {
            bool blank = true;
            for (char c : line) if (c != ' ' && c != '\t' && c != '\r') blank = false;
            if (blank) continue;
            // the reference stops at the 'BEGIN.COMMENT' trailer or at end of file (a last line
            // without a newline), and rejects any other line that is not an entry
            // (io/lorads_file_io.c:264-279)
            if (line.compare(0, 13, "BEGIN.COMMENT") == 0 || pos > s.size()) break;
            err = "bad entry line: " + line.substr(0, 80);
            return false;
        }
        ib -= 1; ii -= 1; ij -= 1;
        if (std::fabs(v) < 1e-12) continue;                 // :288-294
        if (ib == K && nLp > 0) {
            // LP block (io/lorads_file_io.c:297-309): column i of the diagonal block, j unused,
            // C = -F0 as for the SDP blocks
            if (ic < 0 || ic > m || ii < 0 || ii >= nLp) { err = "LP entry out of range"; return false; }
            if (ic == 0) v = -v;
            raw.push_back({K, ic, ii, ii, v});
            lpEntries = true;
            continue;
        }
        if (ib < 0 || ib >= K || ic < 0 || ic > m) { err = "entry out of range"; return false; }
        if (ii > ij) std::swap(ii, ij);                     // :311-315
        if (ii < 0 || ij >= dims[ib]) { err = "entry index out of block"; return false; }
        if (ic == 0) v = -v;                                // :317-319 (C = -F0)
        raw.push_back({ib, ic, ij, ii, v});
    }
    return build_problem(m, K, dims, nLp, lpEntries, raw, hp, err);
}

// allow_dense = false (a shard's local problem): every objective entry stays in the slot
// pattern; shard_problem installs a dense cone's owned row block itself.
static bool build_problem(int m, int K, const std::vector<int> &dims, int nLp, bool lpEntries,
                          std::vector<RawEntry> &raw, HostProblem &hp, std::string &err, bool allow_dense) {
    (void)lpEntries;
    // An LP block of nLp columns (x_j = r_j^2, data/lorads_lp_conic.c) is the diagonal SDP cone
    // of nLp rows at rank 1: X = r r^T has X_jj = r_j^2, and the LP data (objective c_j,
    // constraint coefficients a_ij) touch only the diagonal, so A(X), <C, X>, the gradient
    // 2 (c_j + sum_i M1_i a_ij) r_j (ALMSetGradLP, lorads_alm.c:99-121), q1 / q2 / p1 / p2
    // (ALMCalq12p12LP, :748-765) and the L-BFGS streams are the SDP cone's formulas on that
    // cone.  It is appended after the SDP cones (cone K), where the reference draws its random
    // start (lpRandom after the SDP cones' R, data/lorads_solver.c:668-676).  What differs is
    // host policy (rank fixed at 1, no AUG_RANK, no oracle rank, rho0 and curr_rank over the SDP
    // cones only, ||C||_2^2 taken as ||c||_1^2 like lp_cone_obj_nrm2Square) and the ADMM update,
    // which is the reference's closed-form column sweep (LORADSUpdateLPVarOne, lorads_admm.c:759-
    // 792) instead of a CG (lrs_kernels.hip k_lp_admm).
    std::vector<int> dimsx(dims.begin(), dims.begin() + K);
    if (nLp > 0) { dimsx.push_back(nLp); K += 1; }
    const std::vector<int> &dims_all = dimsx;
    hp.m = m; hp.K = K; hp.nLp = nLp;
    hp.nEntries = (long)raw.size();
    hp.cones.assign(K, HostCone());
    // sort: cone, con, row, col -> merge duplicates (the reference sums them in AUV / WSum)
    std::sort(raw.begin(), raw.end(), [](const RawEntry &a, const RawEntry &b) {
        if (a.cone != b.cone) return a.cone < b.cone;
        if (a.con != b.con) return a.con < b.con;
        if (a.row != b.row) return a.row < b.row;
        return a.col < b.col;
    });
    // auto constant objective (lrs_problem.h policy): every cone's C constant or absent, and
    // the lean single-workgroup layout (R, D at the widest reachable layout + the pattern)
    // within kSmallLdsBudget
    bool auto_const = false;
    {
        const char *ek = getenv("LRS_CONST_C");
        const char *ev = getenv("LRS_DENSE_C");
        const char *es = getenv("LRS_SMALL");
        if (allow_dense && nLp == 0 && !ek && !(ev && ev[0] == '0') && !(es && atoi(es) == 0)) {
            bool ok = true, any = false;
            long N = 0, Ptot = 0;
            int ldmax = 0, ldmin = 1 << 30, nconst = 0;
            // the single-workgroup loop's own gates (lrs_solver.cpp use_small, lrs_kernels.hip
            // small_alm_args) that the data decides: at most kSmallAutoMaxGlobal multi-slot
            // constraints (LRS_SMALL=1 lifts it, as there), at most kSmallAutoMaxConst constant
            // cones, one row layout for every cone at its largest reachable rank
            if (!(es && atoi(es) == 1)) {
                std::vector<int> cnt(m + 1, 0);
                for (size_t e = 0; e < raw.size(); ++e) {
                    if (raw[e].con == 0) continue;
                    if (e > 0 && raw[e - 1].cone == raw[e].cone && raw[e - 1].con == raw[e].con &&
                        raw[e - 1].row == raw[e].row && raw[e - 1].col == raw[e].col)
                        continue;   // a duplicate of the previous entry (merged below)
                    cnt[raw[e].con]++;
                }
                long mg = 0;
                for (int i = 1; i <= m; ++i) mg += cnt[i] > 1 ? 1 : 0;
                if (mg > kSmallAutoMaxGlobal) ok = false;
            }
            size_t e0 = 0;
            std::vector<long> cone_lds(K, 0);   // per cone: 2 n + (slots) ... in doubles, ld added below
            std::vector<int> cone_n(K, 0);
            for (int k = 0; k < K && ok; ++k) {
                size_t e1 = e0;
                while (e1 < raw.size() && raw[e1].cone == k) e1++;
                const int n = dims_all[k];
                cone_n[k] = n;
                N += n;
                if (N > 4096) { ok = false; break; }
                std::vector<std::pair<int, int>> pr, cc;
                std::vector<int> cons;
                for (size_t e = e0; e < e1; ++e) {
                    if (raw[e].con == 0) cc.push_back({raw[e].row, raw[e].col});
                    else { pr.push_back({raw[e].row, raw[e].col}); cons.push_back(raw[e].con); }
                }
                std::sort(pr.begin(), pr.end());
                cone_lds[k] = (long)(std::unique(pr.begin(), pr.end()) - pr.begin());
                Ptot += cone_lds[k];
                std::sort(cons.begin(), cons.end());
                const long nnzRows = (long)(std::unique(cons.begin(), cons.end()) - cons.begin());
                std::sort(cc.begin(), cc.end());
                const long ncobj = (long)(std::unique(cc.begin(), cc.end()) - cc.begin());
                if (ncobj > 0) {
                    // every entry of the block equal (duplicates summed like the merge below)
                    if (ncobj != (long)n * (n + 1) / 2 || n < kConstCMinN) { ok = false; break; }
                    std::vector<std::pair<std::pair<int, int>, double>> vv;
                    for (size_t e = e0; e < e1; ++e)
                        if (raw[e].con == 0) vv.push_back({{raw[e].row, raw[e].col}, raw[e].v});
                    std::sort(vv.begin(), vv.end());
                    double v0 = 0.0;
                    bool first = true;
                    for (size_t a = 0; a < vv.size() && ok;) {
                        double s = 0.0;
                        size_t b2 = a;
                        while (b2 < vv.size() && vv[b2].first == vv[a].first) s += vv[b2++].second;
                        if (first) { v0 = s; first = false; }
                        else if (s != v0) ok = false;
                        a = b2;
                    }
                    if (!ok || v0 == 0.0) { ok = false; break; }
                    any = true;
                    if (++nconst > kSmallAutoMaxConst) { ok = false; break; }
                }
                const int rmax = std::min((int)std::sqrt(2.0 * nnzRows) + 1, n);
                const int ldk = choose_layout(std::max(1, rmax)).ld;
                ldmax = std::max(ldmax, ldk);
                ldmin = std::min(ldmin, ldk);
                e0 = e1;
            }
            bool fits = (2L * N * (ldmax + 2) + Ptot) * (long)sizeof(double) <= kSmallLdsBudget;
            if (ok && !fits && K >= 2 && K <= kSmallAutoMaxCones) {
                // one workgroup per cone (lrs_kernels.hip small_alm_args): every constraint within
                // one cone and each cone's R, D and slots within the budget
                std::vector<int> owner(m + 1, -1);
                bool sep = true;
                for (size_t e = 0; e < raw.size() && sep; ++e) {
                    if (raw[e].con == 0) continue;
                    int &o = owner[raw[e].con];
                    if (o < 0) o = raw[e].cone;
                    else if (o != raw[e].cone) sep = false;
                }
                fits = sep;
                for (int k = 0; k < K && fits; ++k)
                    fits = (2L * cone_n[k] * (ldmax + 2) + cone_lds[k]) * (long)sizeof(double) <= kSmallLdsBudget;
            }
            auto_const = ok && any && ldmax <= 64 && ldmin == ldmax && fits;
        }
    }
    size_t q = 0;
    for (int k = 0; k < K; ++k) {
        HostCone &c = hp.cones[k];
        c.n = dims_all[k];
        c.lp = nLp > 0 && k == K - 1;
        size_t b0 = q;
        while (q < raw.size() && raw[q].cone == k) q++;
        // merged entries of this cone
        std::vector<RawEntry> me;
        me.reserve(q - b0);
        for (size_t e = b0; e < q; ++e) {
            if (!me.empty() && me.back().con == raw[e].con && me.back().row == raw[e].row && me.back().col == raw[e].col)
                me.back().v += raw[e].v;
            else
                me.push_back(raw[e]);
        }
        if (c.lp) {
            // the LP block's columns as lp_cone_presolve types them (lorads_lp_conic.c:110-125):
            // a column in >= 1/4 of the constraints is LP_COEFF_DENSE, whose create routine never
            // sets its row count (LPdataMatCreateDenseImpl, lorads_lp_data.c:178-193: calloc'ed
            // nRows = 0), so the reference's A(x), A^*(y) and constraint values see none of its
            // coefficients; only ||a_j||^2 (taken from the raw entries, :132-133) reaches the ADMM
            // update's denominator.  Reproduced: those entries leave the cone, their norm stays.
            std::vector<int> cnt(c.n, 0);
            c.lp_nrm2.assign(c.n, 0.0);
            for (auto &e : me)
                if (e.con != 0) { cnt[e.row]++; c.lp_nrm2[e.row] += e.v * e.v; }
            for (auto &v : c.lp_nrm2) { const double t = std::sqrt(v); v = t * t; }   // nrm2, then squared
            std::vector<RawEntry> keep;
            keep.reserve(me.size());
            for (auto &e : me)
                if (e.con == 0 || !(cnt[e.row] != 0 && (double)cnt[e.row] / (double)m >= 0.25)) keep.push_back(e);
                else c.lp_dense_dropped++;
            me.swap(keep);
        }
        // dense objective: C out of the pattern, into a full matrix (lrs_problem.h policy)
        long ncobj = 0;
        for (auto &e : me) ncobj += e.con == 0 ? 1 : 0;
        {
            const char *ev = getenv("LRS_DENSE_C");
            const long tri = (long)c.n * (c.n + 1) / 2;
            if (ev && ev[0] == '0') c.dense_c = false;
            else if (ev && ev[0] == '1') c.dense_c = ncobj > 0;
            else c.dense_c = c.n >= kDenseCMinN && 4 * ncobj >= tri;
            if (!allow_dense || c.lp) c.dense_c = false;
            // constant C (all entries one value): the rank-one products, no n x n matrix
            const char *ek = getenv("LRS_CONST_C");
            if (allow_dense && !c.lp && ((ek && ek[0] == '1') || auto_const) && !(ev && ev[0] == '0') && c.n >= kConstCMinN &&
                ncobj == tri) {
                double v0 = 0.0;
                bool same = true, first = true;
                for (auto &e : me) {
                    if (e.con != 0) continue;
                    if (first) { v0 = e.v; first = false; }
                    else if (e.v != v0) { same = false; break; }
                }
                if (same && v0 != 0.0) { c.const_c = true; c.c_alpha = v0; c.dense_c = true; }
            }
        }
        if (c.dense_c && !c.const_c) c.Cfull.assign((size_t)c.n * c.n, 0.0);
        // pattern = unique (row,col), row-major
        std::vector<std::pair<int, int>> pr;
        pr.reserve(me.size());
        for (auto &e : me)
            if (!(c.dense_c && e.con == 0)) pr.push_back({e.row, e.col});
        std::sort(pr.begin(), pr.end());
        pr.erase(std::unique(pr.begin(), pr.end()), pr.end());
        const int P = (int)pr.size();
        c.prow.resize(P); c.pcol.resize(P);
        for (int t = 0; t < P; ++t) { c.prow[t] = pr[t].first; c.pcol[t] = pr[t].second; }
        auto slot_of = [&](int row, int col) {
            auto it = std::lower_bound(pr.begin(), pr.end(), std::make_pair(row, col));
            return (int)(it - pr.begin());
        };
        c.Craw.assign(P, 0.0);
        c.Chas.assign(P, 0);
        long cn = 0;
        int lastCon = -1, cnt = 0;
        const double fill = 0.1 * (double)((long)c.n * (c.n + 1) / 2);
        for (size_t e = 0; e < me.size(); ++e) {
            const RawEntry &r = me[e];
            if (r.con == 0) {
                // objective norms (sdpSparseConeObjNrm*, data/lorads_sdp_data.c:217-262)
                const double a = r.v;
                const bool dg = r.row == r.col;
                c.cNrm1 += dg ? std::fabs(a) : 2 * std::fabs(a);
                c.cNrm2sq += dg ? a * a : 2 * a * a;
                c.cNrmInf = std::max(c.cNrmInf, std::fabs(a));
                cn++;
                if (c.dense_c) {
                    if (!c.const_c) {
                        c.Cfull[(size_t)r.row * c.n + r.col] += r.v;
                        if (!dg) c.Cfull[(size_t)r.col * c.n + r.row] += r.v;
                    }
                    continue;
                }
                const int sl = slot_of(r.row, r.col);
                c.Craw[sl] += r.v;
                c.Chas[sl] = 1;
            } else {
                const int sl = slot_of(r.row, r.col);
                c.ent.push_back({r.con - 1, sl, r.v, r.row == r.col});
                if (r.con != lastCon) {
                    if (lastCon > 0 && cnt > fill) c.denseCoeff = true;
                    c.nnzRows++;
                    lastCon = r.con;
                    cnt = 0;
                }
                cnt++;
            }
        }
        if (lastCon > 0 && cnt > fill) c.denseCoeff = true;
        if ((double)cn > fill) c.denseCoeff = true;
        if (c.lp) {
            c.denseCoeff = false;
            c.cNrm2sq = c.cNrm1 * c.cNrm1;   // lp_cone_obj_nrm2Square (lorads_lp_conic.c:171-176): nrm1^2
        }
        // symmetric adjacency, columns ascending per row; lower prefix = col <= row
        std::vector<int> deg(c.n, 0);
        for (int t = 0; t < P; ++t) {
            deg[c.prow[t]]++;
            if (c.prow[t] != c.pcol[t]) deg[c.pcol[t]]++;
        }
        c.adj_ptr.assign(c.n + 1, 0);
        for (int i = 0; i < c.n; ++i) c.adj_ptr[i + 1] = c.adj_ptr[i] + deg[i];
        const long nadj = c.adj_ptr[c.n];
        c.adj_col.assign(nadj, 0);
        c.adj_slot.assign(nadj, 0);
        std::vector<int> fillp(c.adj_ptr.begin(), c.adj_ptr.end() - 1);
        // pass 1: lower entries in row-major order already sorted by col within a row
        for (int t = 0; t < P; ++t) {
            int i = c.prow[t];
            c.adj_col[fillp[i]] = c.pcol[t];
            c.adj_slot[fillp[i]] = t;
            fillp[i]++;
        }
        c.adj_low.assign(c.n, 0);
        for (int i = 0; i < c.n; ++i) c.adj_low[i] = fillp[i];
        // pass 2: upper entries (j > i): slot (j, i) -> row i, col j; rows j ascending
        for (int t = 0; t < P; ++t) {
            int i = c.prow[t], j = c.pcol[t];
            if (i == j) continue;
            c.adj_col[fillp[j]] = i;
            c.adj_slot[fillp[j]] = t;
            fillp[j]++;
        }
    }
    double bn1 = 0, bn2 = 0, bmax = -1.0;
    size_t imax = 0;
    for (size_t i = 0; i < hp.b.size(); ++i) {
        const double v = hp.b[i];
        bn1 += std::fabs(v);
        bn2 += v * v;
        if (std::fabs(v) > bmax) { bmax = std::fabs(v); imax = i; }
    }
    // ||b||_inf as the reference forms it (cal_sdp_const, data/lorads_solver.c:1469, the Linux
    // build's UNDER_BLAS branch): Fortran idamax_ returns the 1-based position of the first
    // largest |b_i|, used there as a 0-based index -- so the entry AFTER the largest.  (It
    // scales l_inf_primal_infeasibility and thereby the ALM exit test.)  Largest entry last:
    // the reference reads past b; here the largest itself.
    const size_t inext = imax + 1 < hp.b.size() ? imax + 1 : imax;
    hp.bNrm1 = bn1; hp.bNrm2 = std::sqrt(bn2); hp.bNrmInf = hp.b.empty() ? 0.0 : std::fabs(hp.b[inext]);
    double c1 = 0, c2 = 0, ci = 0;
    for (auto &c : hp.cones) { c1 += c.cNrm1; c2 += c.cNrm2sq; ci = std::max(ci, c.cNrmInf); }
    hp.cNrm1 = c1; hp.cNrm2 = std::pow(c2, 0.5); hp.cNrmInf = ci;
    return true;
}


bool build_problem_coo(int m, int nblk, const int *dims_in, const double *b, long nnz, const int *con,
                       const int *blk, const int *row, const int *col, const double *val, HostProblem &hp,
                       std::string &err) {
    // same entry semantics as the file reader (1-based blocks/rows/cols, con 0 = F0)
    std::vector<int> dims(dims_in, dims_in + nblk);
    for (int k = 0; k < nblk - 1; ++k)
        if (dims[k] <= 0) { err = "only the last block may be an LP block"; return false; }
    int K = nblk, nLp = 0;
    if (nblk > 0 && dims[nblk - 1] < 0) { nLp = -dims[nblk - 1]; K = nblk - 1; }
    hp.b.assign(b, b + m);
    std::vector<RawEntry> raw;
    raw.reserve(nnz);
    bool lpEntries = false;
    for (long t = 0; t < nnz; ++t) {
        int ic = con[t], ib = blk[t] - 1, ii = row[t] - 1, ij = col[t] - 1;
        double v = val[t];
        if (std::fabs(v) < 1e-12) continue;
        if (ib == K && nLp > 0) {   // LP block: column i (read_sdpa)
            if (ic < 0 || ic > m || ii < 0 || ii >= nLp) { err = "LP entry out of range"; return false; }
            if (ic == 0) v = -v;
            raw.push_back({K, ic, ii, ii, v});
            lpEntries = true;
            continue;
        }
        if (ib < 0 || ib >= K || ic < 0 || ic > m) { err = "entry out of range"; return false; }
        if (ii > ij) std::swap(ii, ij);
        if (ii < 0 || ij >= dims[ib]) { err = "entry index out of block"; return false; }
        if (ic == 0) v = -v;
        raw.push_back({ib, ic, ij, ii, v});
    }
    return build_problem(m, K, dims, nLp, lpEntries, raw, hp, err);
}

bool shard_problem(const HostProblem &g, int world, int rank, HostProblem &out, ShardPlan &plan, std::string &err) {
    const int K = g.K;
    if (world < 1 || world > kMaxShards || rank < 0 || rank >= world) {
        err = "sharded solve: bad world/rank";
        return false;
    }
    if (g.nLp > 0) {
        // the LP block's ADMM update is the reference's sequential column sweep (each column
        // sees the constraint sums its predecessors left): one workgroup walks it, unsharded
        err = "sharded solve: an LP block is not supported (its ADMM update is a sequential column sweep)";
        return false;
    }
    for (int k = 0; k < K; ++k)
        if (g.cones[k].n < world) { err = "sharded solve: a cone has fewer rows than shards"; return false; }
    // a constant objective (C = c_alpha J) is sharded as the slot path: every pair with an owned
    // endpoint carries C in the local pattern, every row is in the halo.  A dense objective
    // (C a full matrix): each shard holds the row block C_own (owned rows x all n columns) and
    // every row in its halo, so C_own X reads a complete X after the halo exchange.
    auto dense_mat = [&](int k) { return g.cones[k].dense_c && !g.cones[k].const_c; };
    plan = ShardPlan();
    plan.world = world; plan.rank = rank;
    plan.cones.assign(K, ShardConePlan());
    // per cone: contiguous blocks balanced by (adjacency entries + 1) per row
    std::vector<std::vector<int>> lid(K);
    for (int k = 0; k < K; ++k) {
        const HostCone &gc = g.cones[k];
        ShardConePlan &cp = plan.cones[k];
        const int n = gc.n;
        cp.n_global = n;
        std::vector<long> cum(n + 1, 0);
        for (int i = 0; i < n; ++i) cum[i + 1] = cum[i] + (gc.adj_ptr[i + 1] - gc.adj_ptr[i]) + 1;
        cp.bounds.assign(world + 1, 0);
        for (int q = 1; q < world; ++q) {
            const long target = cum[n] * q / world;
            int b = (int)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
            b = std::max(b, cp.bounds[q - 1] + 1);
            b = std::min(b, n - (world - q));
            cp.bounds[q] = b;
        }
        cp.bounds[world] = n;
    }
    auto owner = [&](int k, int i) {
        const std::vector<int> &b = plan.cones[k].bounds;
        return (int)(std::upper_bound(b.begin(), b.end(), i) - b.begin()) - 1;
    };
    // the shards holding each constraint: those owning an endpoint of one of its entries' slots
    // (constraints without entries: shard 0, for the residual b_i)
    std::vector<unsigned long long> holders(g.m, 0ull);
    for (int k = 0; k < K; ++k) {
        const HostCone &gc = g.cones[k];
        for (const HostEntry &e : gc.ent)
            holders[e.con] |= (1ull << owner(k, gc.prow[e.slot])) | (1ull << owner(k, gc.pcol[e.slot]));
    }
    for (int i = 0; i < g.m; ++i)
        if (holders[i] == 0) holders[i] = 1ull;
    auto holds = [&](int i) { return ((holders[i] >> rank) & 1ull) != 0; };
    for (int i = 0; i < g.m; ++i)
        if (__builtin_popcountll(holders[i]) > 1) plan.shared_gid.push_back(i);
    // local rows per cone: owned + halo, in global order
    std::vector<int> dims(K);
    for (int k = 0; k < K; ++k) {
        const HostCone &gc = g.cones[k];
        ShardConePlan &cp = plan.cones[k];
        const int n = gc.n, r0 = cp.bounds[rank], r1 = cp.bounds[rank + 1];
        std::vector<char> need(n, (gc.const_c || dense_mat(k)) ? 1 : 0);
        for (int i = r0; i < r1; ++i) {
            need[i] = 1;
            for (int q = gc.adj_ptr[i]; q < gc.adj_ptr[i + 1]; ++q) need[gc.adj_col[q]] = 1;
        }
        lid[k].assign(n, -1);
        for (int i = 0; i < n; ++i)
            if (need[i]) { lid[k][i] = (int)cp.gid.size(); cp.gid.push_back(i); }
        cp.row0 = lid[k][r0];
        cp.nown = r1 - r0;
        dims[k] = (int)cp.gid.size();
    }
    // local constraints in global order
    std::vector<int> clid(g.m, -1);
    for (int i = 0; i < g.m; ++i)
        if (holds(i)) {
            clid[i] = (int)plan.con_gid.size();
            plan.con_gid.push_back(i);
            plan.primary.push_back(__builtin_ctzll(holders[i]) == rank ? 1 : 0);
        }
    for (int gi : plan.shared_gid) plan.shared_lid.push_back(clid[gi]);
    const int ml = (int)plan.con_gid.size();
    // entries of the local problem (already merged and sign-converted: build_problem input):
    // the slots with an owned endpoint
    std::vector<RawEntry> raw;
    for (int k = 0; k < K; ++k) {
        const HostCone &gc = g.cones[k];
        for (size_t t = 0; t < gc.prow.size(); ++t) {
            const int i = gc.prow[t], j = gc.pcol[t];
            if (!gc.Chas[t] || (owner(k, i) != rank && owner(k, j) != rank)) continue;
            raw.push_back({k, 0, lid[k][i], lid[k][j], gc.Craw[t]});
        }
        if (gc.const_c)   // every lower pair with an owned endpoint (local ids keep the global order)
            for (int i = 0; i < gc.n; ++i)
                for (int j = 0; j <= i; ++j)
                    if (owner(k, i) == rank || owner(k, j) == rank)
                        raw.push_back({k, 0, lid[k][i], lid[k][j], gc.c_alpha});
        for (const HostEntry &e : gc.ent) {
            const int i = gc.prow[e.slot], j = gc.pcol[e.slot];
            if (owner(k, i) != rank && owner(k, j) != rank) continue;   // slot not present here
            raw.push_back({k, clid[e.con] + 1, lid[k][i], lid[k][j], e.a});
        }
    }
    out = HostProblem();
    out.b.resize(ml);
    for (int q = 0; q < ml; ++q) out.b[q] = g.b[plan.con_gid[q]];
    if (!build_problem(ml, K, dims, 0, false, raw, out, err, false)) return false;
    // the solve's norms and rank statistics are the whole problem's
    out.bNrm1 = g.bNrm1; out.bNrm2 = g.bNrm2; out.bNrmInf = g.bNrmInf;
    out.cNrm1 = g.cNrm1; out.cNrm2 = g.cNrm2; out.cNrmInf = g.cNrmInf;
    for (int k = 0; k < K; ++k) {
        const HostCone &gc = g.cones[k];
        HostCone &oc = out.cones[k];
        const ShardConePlan &cp = plan.cones[k];
        oc.nnzRows = gc.nnzRows; oc.denseCoeff = gc.denseCoeff;
        oc.cNrm1 = gc.cNrm1; oc.cNrm2sq = gc.cNrm2sq; oc.cNrmInf = gc.cNrmInf;
        // entries count in A(.) on the shard owning their slot's lower row
        const int o0 = cp.row0, o1 = cp.row0 + cp.nown;
        for (HostEntry &e : oc.ent) e.owned = oc.prow[e.slot] >= o0 && oc.prow[e.slot] < o1;
        oc.own0 = o0;
        oc.own1 = o1;
        if (dense_mat(k)) {   // every row local, local ids = global ids: C's owned row block
            const int n = gc.n, r0 = cp.bounds[rank];
            oc.dense_c = true;
            oc.Cfull.assign(gc.Cfull.begin() + (size_t)r0 * n, gc.Cfull.begin() + (size_t)(r0 + cp.nown) * n);
        }
    }
    // shared constraints stay on the multi-slot path on every holder
    out.force_glob.assign(ml, 0);
    for (int l : plan.shared_lid)
        if (l >= 0) out.force_glob[l] = 1;
    // halo exchange plan per cone: rows of ours adjacent to each peer's rows (both sides derive
    // the same global-order lists), and the peers' rows in our halo (contiguous locally)
    for (int k = 0; k < K; ++k) {
        const HostCone &gc = g.cones[k];
        ShardConePlan &cp = plan.cones[k];
        const int r0 = cp.bounds[rank], r1 = cp.bounds[rank + 1], nl = (int)cp.gid.size();
        cp.send_ptr.assign(world + 1, 0);
        cp.recv_start.assign(world, 0);
        cp.recv_cnt.assign(world, 0);
        for (int q = 0; q < world; ++q) {
            cp.send_ptr[q] = (int)cp.send_rows.size();
            if (q == rank) continue;
            const int q0 = cp.bounds[q], q1 = cp.bounds[q + 1];
            for (int i = r0; i < r1; ++i) {
                bool adj = gc.const_c || dense_mat(k);   // C couples every pair of rows
                for (int t = gc.adj_ptr[i]; t < gc.adj_ptr[i + 1] && !adj; ++t)
                    adj = gc.adj_col[t] >= q0 && gc.adj_col[t] < q1;
                if (adj) cp.send_rows.push_back(lid[k][i]);
            }
            int first = -1, cnt = 0;
            for (int l = 0; l < nl; ++l)
                if (cp.gid[l] >= q0 && cp.gid[l] < q1) { if (first < 0) first = l; cnt++; }
            cp.recv_start[q] = first < 0 ? 0 : first;
            cp.recv_cnt[q] = cnt;
        }
        cp.send_ptr[world] = (int)cp.send_rows.size();
    }
    return true;
}

// Entry order inside one 2-D tile item for conflict-free LDS reads (lrs_kernels.hip
// auv_chunk): position t of an item is lane t % 64 of a wave-round, and a ds_read_b128
// services a wave in four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32;
// MI355X_MICROARCH.md §LDS) whose 16-B slots must differ.  A staged row of local index x sits
// at slot x mod 16 (rows 17 slots apart), so a group reads without conflicts when its 16
// entries have distinct p mod 16 and distinct q mod 16 (or share p: a broadcast).  The sorted
// (p, q) order keeps p shared but leaves the 16 random q's colliding (~3-4 way).  Here each
// group takes one entry from each cell (p mod 16, q mod 16) along a diagonal q = p + s of the
// 16 x 16 cell grid while one is complete, then greedily distinct q's; only leftovers collide.
// Results are unchanged: an entry's dot product is the same wherever it runs (k_auv_tsum sums
// each constraint in entry order through `pos`; the slot epilogue's partial sums change order).
static int swz_group_of(int lane) {
    static const signed char g[64] = {0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 1, 1, 1, 1, 0, 0,
                                      0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3,
                                      2, 2, 2, 2, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3};
    return g[lane & 63];
}
// perm[i] = the sorted-order index of the entry placed at item position i (0 <= i < cnt).
// Groups of 16 are formed from a window of consecutive rows with distinct p mod 16 (so the
// p side is conflict-free or a broadcast), taking entries of unused q mod 16 in row order;
// a group the window cannot complete is filled with the next entries in order.
static void swizzle_item(const unsigned *pq, long cnt, std::vector<long> &perm) {
    std::vector<std::vector<long>> rows;   // entries of each row, in (p, q) order
    for (long t = 0; t < cnt; ++t) {
        if (t == 0 || (pq[t] >> 16) != (pq[t - 1] >> 16)) rows.emplace_back();
        rows.back().push_back(t);
    }
    std::vector<long> order;
    order.reserve(cnt);
    size_t first = 0;
    long left = cnt;
    std::vector<long> keep;
    while (left > 0) {
        while (first < rows.size() && rows[first].empty()) ++first;
        long grp[16];
        int ng = 0;
        bool pu[16] = {false}, qu[16] = {false};
        for (size_t r = first; r < rows.size() && ng < 16; ++r) {
            if (rows[r].empty()) continue;
            const int pc = (int)((pq[rows[r][0]] >> 16) & 15);
            if (pu[pc]) break;
            pu[pc] = true;
            keep.clear();
            for (long t : rows[r]) {
                const int qc = (int)(pq[t] & 15);
                if (ng < 16 && !qu[qc]) { grp[ng++] = t; qu[qc] = true; }
                else keep.push_back(t);
            }
            rows[r].swap(keep);
        }
        for (size_t r = first; r < rows.size() && ng < 16; ++r)
            while (ng < 16 && !rows[r].empty()) {
                grp[ng++] = rows[r].front();
                rows[r].erase(rows[r].begin());
            }
        for (int k = 0; k < ng; ++k) order.push_back(grp[k]);
        left -= ng;
    }
    // groups onto lane positions: wave-round w (64 consecutive positions) holds groups
    // 4w..4w+3, group g's k-th member at the k-th lane of hardware group g; the last partial
    // round keeps the remaining entries in order
    perm.assign(cnt, -1);
    std::vector<int> lanes[4];
    for (int l = 0; l < 64; ++l) lanes[swz_group_of(l)].push_back(l);
    const long ngt = (long)order.size() / 16;
    long gi = 0;
    for (long base = 0; gi < ngt && base + 64 <= cnt; base += 64)
        for (int g = 0; g < 4 && gi < ngt; ++g, ++gi)
            for (int k = 0; k < 16; ++k) perm[base + lanes[g][k]] = order[gi * 16 + k];
    long o = gi * 16;
    for (long i = 0; i < cnt; ++i)
        if (perm[i] < 0) perm[i] = order[o++];
}
static bool tile_swizzle_on() {
    const char *e = getenv("LRS_TILE_SWZ");
    return !(e && e[0] == '0');
}


template <typename T>
static bool dput(T **dst, const std::vector<T> &v, std::string &err) {
    size_t bytes = std::max<size_t>(1, v.size()) * sizeof(T);
    if (hipMalloc((void **)dst, bytes) != hipSuccess) { err = "hipMalloc failed"; return false; }
    if (!v.empty() && hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) {
        err = "hipMemcpy failed";
        return false;
    }
    return true;
}

// The single-workgroup ADMM half-step's lists of one small cone (lrs_device.h DevCone::cg_*,
// lrs_kernels.hip k_small_cg): built when the objective is constant (rank-one form, or every
// slot of the block holding one value), absent, or at most 16 entries a row; else cg_ok stays 0
// and the cone's half-steps take the multi-launch CG.
constexpr int kScLong = 16;   // constraints with more entries in the cone: a wave each (= lrs_kernels.hip)
static bool upload_small_cg(const HostCone &c, int m, DevCone &d, std::string &err) {
    const int P = (int)c.prow.size();
    std::vector<int> s2cs(P, -1), csl;
    for (const HostEntry &e : c.ent) s2cs[e.slot] = 0;
    for (int t = 0; t < P; ++t)
        if (s2cs[t] == 0) { s2cs[t] = (int)csl.size(); csl.push_back(t); }
    const int ncs = (int)csl.size();
    int cconst = 0, cslot = 0;
    long nC = 0;
    if (c.const_c) {
        cconst = 2;
    } else {
        bool same = true;
        for (int t = 0; t < P; ++t) {
            if (!c.Chas[t]) continue;
            if (nC == 0) cslot = t;
            else if (c.Craw[t] != c.Craw[cslot]) same = false;
            nC++;
        }
        if (nC > 0 && nC == (long)c.n * (c.n + 1) / 2 && same) cconst = 1;
    }
    if (ncs == 0 || ncs >= 65536 || (cconst == 0 && nC > 16L * c.n)) return true;
    // constraint-slot adjacency, in the adjacency's (column) order
    std::vector<int> cap(c.n + 1, 0), cadj;
    for (int i = 0; i < c.n; ++i) {
        for (int q = c.adj_ptr[i]; q < c.adj_ptr[i + 1]; ++q)
            if (s2cs[c.adj_slot[q]] >= 0) cadj.push_back((c.adj_col[q] << 16) | s2cs[c.adj_slot[q]]);
        cap[i + 1] = (int)cadj.size();
    }
    // the cone's constraints (entries sorted by (con, slot)): the short ones, then the long ones
    std::vector<int> cons, cbeg;
    for (size_t e = 0; e < c.ent.size();) {
        size_t f = e;
        while (f < c.ent.size() && c.ent[f].con == c.ent[e].con) ++f;
        cons.push_back(c.ent[e].con);
        cbeg.push_back((int)e);
        e = f;
    }
    cbeg.push_back((int)c.ent.size());
    const int ncl = (int)cons.size();
    std::vector<int> order;
    for (int pass = 0; pass < 2; ++pass)
        for (int j = 0; j < ncl; ++j)
            if ((cbeg[j + 1] - cbeg[j] > kScLong) == (pass == 1)) order.push_back(j);
    int ns = 0;
    for (int j = 0; j < ncl; ++j) ns += cbeg[j + 1] - cbeg[j] <= kScLong ? 1 : 0;
    std::vector<int> compact(std::max(1, m), -1), clcon, clp(1, 0), ce;
    std::vector<double> cew;
    for (int o = 0; o < ncl; ++o) {
        const int j = order[o];
        compact[cons[j]] = o;
        clcon.push_back(cons[j]);
        for (int e = cbeg[j]; e < cbeg[j + 1]; ++e) {
            const HostEntry &he = c.ent[e];
            ce.push_back((s2cs[he.slot] << 1) | (he.diag ? 1 : 0));
            cew.push_back((he.diag ? 1.0 : 2.0) * he.a);
        }
        clp.push_back((int)ce.size());
    }
    // per constraint slot its (compact constraint, a), constraints ascending (as slot_con)
    std::vector<int> sp(ncs + 1, 0), sj(c.ent.size());
    std::vector<double> sa(c.ent.size());
    for (const HostEntry &he : c.ent) sp[s2cs[he.slot] + 1]++;
    for (int t = 0; t < ncs; ++t) sp[t + 1] += sp[t];
    std::vector<int> fp(sp.begin(), sp.end() - 1);
    for (const HostEntry &he : c.ent) {
        const int t = s2cs[he.slot];
        sj[fp[t]] = compact[he.con];
        sa[fp[t]] = he.a;
        fp[t]++;
    }
    // objective entries of each row (column, global slot) when C is neither constant nor absent
    std::vector<int> ccp(c.n + 1, 0), cc;
    if (cconst == 0)
        for (int i = 0; i < c.n; ++i) {
            for (int q = c.adj_ptr[i]; q < c.adj_ptr[i + 1]; ++q)
                if (c.Chas[c.adj_slot[q]]) { cc.push_back(c.adj_col[q]); cc.push_back(d.slot_off + c.adj_slot[q]); }
            ccp[i + 1] = (int)(cc.size() / 2);
        }
    if (!dput(&d.cg_cadj_ptr, cap, err) || !dput(&d.cg_cadj, cadj, err) || !dput(&d.cg_cl_con, clcon, err) ||
        !dput(&d.cg_cl_ptr, clp, err) || !dput(&d.cg_ce, ce, err) || !dput(&d.cg_ce_w, cew, err) ||
        !dput(&d.cg_sp, sp, err) || !dput(&d.cg_sj, sj, err) || !dput(&d.cg_sa, sa, err) ||
        !dput(&d.cg_cc_ptr, ccp, err) || !dput(&d.cg_cc, cc, err))
        return false;
    d.cg_ncs = ncs; d.cg_ncl = ncl; d.cg_ns = ns; d.cg_nce = (int)ce.size(); d.cg_nsc = (int)sj.size();
    d.cg_nadj = (int)cadj.size(); d.cg_cconst = cconst; d.cg_cslot = d.slot_off + cslot;
    d.cg_ok = 1;
    return true;
}

bool upload_problem(const HostProblem &hp, DevProblem &dp, std::string &err) {
    // per-cone scalars live in the fixed tmpfin slots (TF_SD + 2k < TF_GATHER)
    if (hp.K > kMaxCones) { err = "at most " + std::to_string(kMaxCones) + " SDP cones are supported"; return false; }
    dp.m = hp.m;
    dp.K = hp.K;
    dp.lp_cone = -1;
    dp.cones.assign(hp.K, DevCone());
    dp.ndense = 0;
    dp.dense_scale = 1.0;
    int Ptot = 0;
    for (int k = 0; k < hp.K; ++k) { dp.cones[k].slot_off = Ptot; dp.cones[k].P = (int)hp.cones[k].prow.size(); Ptot += dp.cones[k].P; }
    dp.Ptot = Ptot;
    std::vector<double> Cw(Ptot), Craw(Ptot);
    for (int k = 0; k < hp.K; ++k) {
        const HostCone &c = hp.cones[k];
        for (int t = 0; t < (int)c.prow.size(); ++t) {
            const int g = dp.cones[k].slot_off + t;
            Craw[g] = c.Craw[t];
            Cw[g] = (c.prow[t] == c.pcol[t] ? 1.0 : 2.0) * c.Craw[t];
        }
    }
    // constraint CSR, cone-major rows: row = k*m + i
    const int m = hp.m;
    std::vector<int> con_ptr((long)hp.K * m + 1, 0), con_slot;
    std::vector<double> con_w;
    long Z = 0;
    for (int k = 0; k < hp.K; ++k) Z += (long)hp.cones[k].ent.size();
    con_slot.reserve(Z);
    con_w.reserve(Z);
    for (int k = 0; k < hp.K; ++k) {
        const HostCone &c = hp.cones[k];
        size_t e = 0;
        for (int i = 0; i < m; ++i) {
            while (e < c.ent.size() && c.ent[e].con == i) {
                con_slot.push_back(dp.cones[k].slot_off + c.ent[e].slot);
                con_w.push_back(c.ent[e].owned ? (c.ent[e].diag ? 1.0 : 2.0) * c.ent[e].a : 0.0);
                e++;
            }
            con_ptr[(long)k * m + i + 1] = (int)con_slot.size();
        }
    }
    dp.cone_sep = true;   // (the one-workgroup-per-cone inner loop needs no cross-cone sums per constraint)
    for (int i = 0; i < m && dp.cone_sep; ++i) {
        int nk = 0;
        for (int k = 0; k < hp.K; ++k) nk += con_ptr[(long)k * m + i + 1] > con_ptr[(long)k * m + i] ? 1 : 0;
        dp.cone_sep = nk <= 1;
    }
    // slot -> (con, a) CSR, constraints ascending per slot
    std::vector<int> slot_ptr(Ptot + 1, 0), slot_con(Z);
    std::vector<double> slot_a(Z);
    for (int k = 0; k < hp.K; ++k)
        for (auto &e : hp.cones[k].ent) slot_ptr[dp.cones[k].slot_off + e.slot + 1]++;
    for (int s = 0; s < Ptot; ++s) slot_ptr[s + 1] += slot_ptr[s];
    std::vector<int> fp(slot_ptr.begin(), slot_ptr.end() - 1);
    for (int k = 0; k < hp.K; ++k)
        for (auto &e : hp.cones[k].ent) {   // entries sorted by (con, slot) -> per-slot con ascending
            const int g = dp.cones[k].slot_off + e.slot;
            slot_con[fp[g]] = e.con;
            slot_a[fp[g]] = e.a;
            fp[g]++;
        }
    dp.Z = Z;
    // slot coordinates (row, col) inside their cone, for the constraint-entry A(UV^T)
    std::vector<int> slot_rc(2L * std::max(1, Ptot), 0);
    for (int k = 0; k < hp.K; ++k) {
        const HostCone &c = hp.cones[k];
        for (int t = 0; t < (int)c.prow.size(); ++t) {
            slot_rc[2L * (dp.cones[k].slot_off + t)] = c.prow[t];
            slot_rc[2L * (dp.cones[k].slot_off + t) + 1] = c.pcol[t];
        }
    }
    if (!dput(&dp.slot_rc, slot_rc, err)) return false;
    {   // the same in the all-cones row space (the single-workgroup inner loop)
        std::vector<int> sg(2L * std::max(1, Ptot), 0);
        long r0 = 0;
        for (int k = 0; k < hp.K; ++k) {
            const HostCone &c = hp.cones[k];
            for (int t = 0; t < (int)c.prow.size(); ++t) {
                sg[2L * (dp.cones[k].slot_off + t)] = (int)(r0 + c.prow[t]);
                sg[2L * (dp.cones[k].slot_off + t) + 1] = (int)(r0 + c.pcol[t]);
            }
            r0 += c.n;
        }
        if (!dput(&dp.slot_g, sg, err)) return false;
    }
    // per (cone, constraint) row with exactly one entry: its (p, q) and weight, so the
    // constraint-entry kernels read them in one coalesced load; p = -1 otherwise
    {
        const long rows = (long)hp.K * m;
        std::vector<int> c1pq(2 * std::max(1L, rows), -1);
        std::vector<double> c1w(std::max(1L, rows), 0.0);
        // long rows (> kLongRow entries) go to the wave-per-constraint kernel: p = -2
        std::vector<int> long_ptr(hp.K + 1, 0), long_rows;
        for (int k = 0; k < hp.K; ++k) {
            for (int i = 0; i < m; ++i) {
                const long r = (long)k * m + i;
                if (con_ptr[r + 1] - con_ptr[r] > kLongRow) {
                    long_rows.push_back(i);
                    c1pq[2 * r] = -2;
                }
            }
            long_ptr[k + 1] = (int)long_rows.size();
        }
        dp.long_ptr_h = long_ptr;
        if (long_rows.empty()) long_rows.push_back(0);
        if (!dput(&dp.long_rows, long_rows, err)) return false;
        for (long r = 0; r < rows; ++r) {
            if (con_ptr[r + 1] - con_ptr[r] != 1) continue;
            const int e = con_ptr[r];
            c1pq[2 * r] = slot_rc[2L * con_slot[e]];
            c1pq[2 * r + 1] = slot_rc[2L * con_slot[e] + 1];
            c1w[r] = con_w[e];
        }
        if (!dput(&dp.con1_pq, c1pq, err) || !dput(&dp.con1_w, c1w, err)) return false;
        // cones whose constraint i is the single entry (i, i) for every i (m = n: MaxCut's
        // diag(X) = 1): A(X Y^T) is a row-wise dot product (k_auv_diag, no index loads)
        for (int k = 0; k < hp.K; ++k) {
            bool id = m == hp.cones[k].n && m > 0;
            for (int i = 0; id && i < m; ++i) {
                const long r = (long)k * m + i;
                id = c1pq[2 * r] == i && c1pq[2 * r + 1] == i;
            }
            dp.cones[k].auv_diag = id;
        }
        // 2-D tiles for the constraint-entry A(X Y^T) (lrs_device.h kAuvT): cones with many
        // entries per row and no long constraint rows
        const char *ev = getenv("LRS_AUV_TILES");
        for (int k = 0; k < hp.K; ++k) {
            const int n = hp.cones[k].n;
            const long eb = con_ptr[(long)k * m], ee = con_ptr[(long)k * m + m];
            const long Zk = ee - eb;
            const double ntl = (double)((n + kAuvT - 1) / kAuvT);
            bool on = n >= kAuvMinN && (double)Zk >= kAuvMinPerTile * ntl * (ntl + 1) / 2;
            if (ev && ev[0] == '0') on = false;
            if (ev && ev[0] == '1') on = Zk > 0;
            if (long_ptr[k + 1] > long_ptr[k]) on = false;
            if (hp.cones[k].own1 >= 0) on = false;   // sharded: the A(.) operators keep the gather path
            if (!on) continue;
            const long nt = (n + kAuvT - 1) / kAuvT;
            std::vector<std::pair<unsigned long long, int>> key(Zk);
            for (long e = eb; e < ee; ++e) {
                const int s = con_slot[e];
                int p = slot_rc[2L * s], q = slot_rc[2L * s + 1];
                if (p < q) std::swap(p, q);
                const unsigned long long tile = (unsigned long long)(p / kAuvT) * nt + (q / kAuvT);
                key[e - eb] = {(tile << 32) | ((unsigned)(p % kAuvT) << 16) | (unsigned)(q % kAuvT), (int)(e - eb)};
            }
            std::sort(key.begin(), key.end());
            std::vector<int> item, pos(Zk);
            std::vector<unsigned> pq(Zk);
            long t0 = 0;
            const bool swz = tile_swizzle_on();
            std::vector<long> perm;
            for (long t = 0; t < Zk; ++t) {
                pq[t] = (unsigned)(key[t].first & 0xffffffffu);
                pos[t] = key[t].second;
                const bool last = t + 1 == Zk || (key[t + 1].first >> 32) != (key[t].first >> 32) ||
                                  t + 1 - t0 == kAuvItem;
                if (!last) continue;
                const unsigned long long tile = key[t].first >> 32;
                item.push_back((int)(tile / nt) * kAuvT);
                item.push_back((int)(tile % nt) * kAuvT);
                item.push_back((int)t0);
                item.push_back((int)(t + 1));
                if (swz) {   // conflict-free LDS reads (swizzle_item)
                    swizzle_item(pq.data() + t0, t + 1 - t0, perm);
                    std::vector<unsigned> pq2(perm.size());
                    std::vector<int> pos2(perm.size());
                    for (size_t i = 0; i < perm.size(); ++i) { pq2[i] = pq[t0 + perm[i]]; pos2[i] = pos[t0 + perm[i]]; }
                    std::copy(pq2.begin(), pq2.end(), pq.begin() + t0);
                    std::copy(pos2.begin(), pos2.end(), pos.begin() + t0);
                }
                t0 = t + 1;
            }
            DevCone &d = dp.cones[k];
            d.auv_items = (int)(item.size() / 4);
            d.auv_ebase = eb;
            if (!dput(&d.auv_item, item, err) || !dput(&d.auv_pq, pq, err) || !dput(&d.auv_pos, pos, err))
                return false;
            if (hipMalloc((void **)&d.auv_val, (size_t)Zk * sizeof(double)) != hipSuccess) {
                err = "hipMalloc failed";
                return false;
            }
            // the objective's slots (op_constr_xx of a tiled cone: A(.) from the constraint-entry
            // tiles, <C, X Y^T> from C's own entries instead of a pattern-wide SDDMM + gather)
            if (hp.cones[k].own1 < 0) {
                const HostCone &hc = hp.cones[k];
                std::vector<int> co;
                for (size_t t = 0; t < hc.prow.size(); ++t)
                    if (hc.Chas[t]) co.push_back(d.slot_off + (int)t);
                d.cobj_n = (int)co.size();
                if (!dput(&d.cobj_slot, co, err)) return false;
            }
        }
    }
    // Single-slot ("local") constraints: exactly one merged entry over all cones.  Their
    // A(.) value is one pattern slot, so the row that owns the slot evaluates them inside
    // the row kernels; every other constraint is "global" (lrs_kernels.hip, split iteration).
    std::vector<int> nent(m, 0), only_slot(m, -1);
    std::vector<double> only_w(m, 0.0);
    for (int k = 0; k < hp.K; ++k)
        for (int i = 0; i < m; ++i)
            for (int e = con_ptr[(long)k * m + i]; e < con_ptr[(long)k * m + i + 1]; ++e) {
                nent[i]++;
                only_slot[i] = con_slot[e];
                only_w[i] = con_w[e];
            }
    std::vector<int> glob, loc_ptr(Ptot + 1, 0), loc_con;
    std::vector<double> loc_w;
    auto is_loc = [&](int i) { return nent[i] == 1 && (hp.force_glob.empty() || !hp.force_glob[i]); };
    for (int i = 0; i < m; ++i) {
        if (is_loc(i)) loc_ptr[only_slot[i] + 1]++;
        else glob.push_back(i);
    }
    for (int t = 0; t < Ptot; ++t) loc_ptr[t + 1] += loc_ptr[t];
    loc_con.assign(loc_ptr[Ptot], 0);
    loc_w.assign(loc_ptr[Ptot], 0.0);
    {
        std::vector<int> fpl(loc_ptr.begin(), loc_ptr.end() - 1);
        for (int i = 0; i < m; ++i)
            if (is_loc(i)) {
                const int t = fpl[only_slot[i]]++;
                loc_con[t] = i;
                loc_w[t] = only_w[i];
            }
    }
    // per slot, its single constraint entry / single local constraint as one 16-byte record
    // {a or w, con} (con = -1: none, -2: several -> the lists): one dependent load less per
    // neighbour in the row kernels (slot -> record -> rec[con] instead of slot -> ptr -> con -> rec)
    {
        std::vector<double> s1(2L * std::max(1, Ptot), 0.0), l1(2L * std::max(1, Ptot), 0.0);
        for (int t = 0; t < Ptot; ++t) {
            const int ns = slot_ptr[t + 1] - slot_ptr[t];
            s1[2L * t] = ns == 1 ? slot_a[slot_ptr[t]] : 0.0;
            s1[2L * t + 1] = ns == 0 ? -1.0 : (ns == 1 ? (double)slot_con[slot_ptr[t]] : -2.0);
            const int nl = loc_ptr[t + 1] - loc_ptr[t];
            l1[2L * t] = nl == 1 ? loc_w[loc_ptr[t]] : 0.0;
            l1[2L * t + 1] = nl == 0 ? -1.0 : (nl == 1 ? (double)loc_con[loc_ptr[t]] : -2.0);
        }
        if (!dput(&dp.slot1, s1, err) || !dput(&dp.loc1, l1, err)) return false;
    }
    dp.mg = (int)glob.size();
    dp.glob_maxlen = 0;
    for (int i : glob) dp.glob_maxlen = std::max(dp.glob_maxlen, nent[i]);
    if (glob.empty()) glob.push_back(0);
    if (loc_con.empty()) { loc_con.push_back(0); loc_w.push_back(0.0); }
    if (!dput(&dp.glob, glob, err) || !dput(&dp.loc_ptr, loc_ptr, err) || !dput(&dp.loc_con, loc_con, err) ||
        !dput(&dp.loc_w, loc_w, err))
        return false;
    if (!dput(&dp.b, hp.b, err) || !dput(&dp.Cw, Cw, err) || !dput(&dp.Craw, Craw, err) ||
        !dput(&dp.con_ptr, con_ptr, err) || !dput(&dp.con_slot, con_slot, err) || !dput(&dp.con_w, con_w, err) ||
        !dput(&dp.slot_ptr, slot_ptr, err) || !dput(&dp.slot_con, slot_con, err) || !dput(&dp.slot_a, slot_a, err))
        return false;
    // all cones as one block-diagonal row space (global rows, global columns): the split
    // iteration launches once over it when every cone has the same row layout
    if (hp.K > 1) {
        DevCone &mc = dp.merged;
        long ntot = 0, nadj = 0, Ptot_l = 0;
        for (auto &c : hp.cones) { ntot += c.n; nadj += (long)c.adj_col.size(); Ptot_l += (long)c.prow.size(); }
        std::vector<int> ap(ntot + 1, 0), al(ntot, 0), ac(nadj, 0), as(nadj, 0);
        long r0 = 0, e0 = 0;
        for (int k = 0; k < hp.K; ++k) {
            const HostCone &c = hp.cones[k];
            for (int i = 0; i < c.n; ++i) {
                ap[r0 + i] = (int)(e0 + c.adj_ptr[i]);
                al[r0 + i] = (int)(e0 + c.adj_low[i]);
            }
            for (size_t t = 0; t < c.adj_col.size(); ++t) {
                ac[e0 + t] = (int)(r0 + c.adj_col[t]);
                as[e0 + t] = dp.cones[k].slot_off + c.adj_slot[t];
            }
            r0 += c.n;
            e0 += (long)c.adj_col.size();
        }
        ap[ntot] = (int)e0;
        mc.n = (int)ntot;
        mc.nown = (int)ntot;
        mc.P = (int)Ptot_l;
        mc.adj_nnz = nadj;
        for (long q = 0; q < ntot; ++q) {
            mc.maxdeg = std::max(mc.maxdeg, ap[q + 1] - ap[q]);
            mc.maxlow = std::max(mc.maxlow, al[q] - ap[q]);
            if (al[q] - ap[q] > kDenseRow) { mc.dra_h.push_back((int)q); mc.dra_n.push_back(al[q] - ap[q]); }
            if (ap[q + 1] - ap[q] > kDenseRow) {
                mc.drb_h.push_back((int)q);
                mc.drb_n.push_back(ap[q + 1] - ap[q]);
                mc.gl_need += (long)((ap[q + 1] - ap[q] + kSliceMinB - 1) / kSliceMinB) * 256;
            }
        }
        if (!dput(&mc.dra, mc.dra_h, err) || !dput(&mc.drb, mc.drb_h, err)) return false;
        if (!dput(&mc.adj_ptr, ap, err) || !dput(&mc.adj_low, al, err) || !dput(&mc.adj_col, ac, err) ||
            !dput(&mc.adj_slot, as, err))
            return false;
        dp.has_merged = true;
    }
    for (int k = 0; k < hp.K; ++k) {
        const HostCone &c = hp.cones[k];
        DevCone &d = dp.cones[k];
        d.n = c.n;
        d.nown = c.n;
        std::vector<int> adj_slot_g(c.adj_slot.size());
        for (size_t t = 0; t < c.adj_slot.size(); ++t) adj_slot_g[t] = d.slot_off + c.adj_slot[t];
        d.adj_nnz = (long)c.adj_col.size();
        for (int q = 0; q < c.n; ++q) {
            d.maxdeg = std::max(d.maxdeg, c.adj_ptr[q + 1] - c.adj_ptr[q]);
            d.maxlow = std::max(d.maxlow, c.adj_low[q] - c.adj_ptr[q]);
            if (c.adj_low[q] - c.adj_ptr[q] > kDenseRow) {
                d.dra_h.push_back(q);
                d.dra_n.push_back(c.adj_low[q] - c.adj_ptr[q]);
            }
            if (c.adj_ptr[q + 1] - c.adj_ptr[q] > kDenseRow) {
                d.drb_h.push_back(q);
                d.drb_n.push_back(c.adj_ptr[q + 1] - c.adj_ptr[q]);
                d.gl_need += (long)((c.adj_ptr[q + 1] - c.adj_ptr[q] + kSliceMinB - 1) / kSliceMinB) * 256;
            }
        }
        if (!dput(&d.dra, d.dra_h, err) || !dput(&d.drb, d.drb_h, err)) return false;
        if (!dput(&d.adj_ptr, c.adj_ptr, err) || !dput(&d.adj_low, c.adj_low, err) ||
            !dput(&d.adj_col, c.adj_col, err) || !dput(&d.adj_slot, adj_slot_g, err))
            return false;
        // (a constant objective, const_c, is dense_c too: its rank-one form is the kernel's cconst 2)
        if (c.own1 < 0 && c.n <= kScMaxN && (!c.dense_c || c.const_c) && !upload_small_cg(c, hp.m, d, err))
            return false;
        if (c.n >= kNX && (long)c.adj_col.size() >= (long)kTileMinDeg * c.n) {
            std::vector<int> cs((size_t)c.n * (kNX + 1));
            for (int i = 0; i < c.n; ++i) {
                int e = c.adj_ptr[i];
                for (int x = 0; x <= kNX; ++x) {
                    const int cb = (int)((long)x * c.n / kNX);
                    while (e < c.adj_ptr[i + 1] && c.adj_col[e] < cb) ++e;
                    cs[(size_t)i * (kNX + 1) + x] = x == kNX ? c.adj_ptr[i + 1] : e;
                }
            }
            if (!dput(&d.colseg, cs, err)) return false;
        }
        {
            // the lower pattern in 2-D tiles for k_tile_a (lrs_device.h kAuvT), slots sorted by
            // (row tile, column tile, row, column), items of at most kAuvItem slots.  A shard
            // (own1 >= 0) tiles its owned rows only: the lower slots of owned rows, the row tiles
            // holding them, and lists the slots of halo lower rows (S only, k_slot_sv).
            const long P = (long)c.prow.size();
            const int o0 = c.own1 >= 0 ? c.own0 : 0, o1 = c.own1 >= 0 ? c.own1 : c.n;
            const long nt = (c.n + kAuvT - 1) / kAuvT;
            const long tI0 = o0 / kAuvT, tI1 = o1 > o0 ? (o1 - 1) / kAuvT + 1 : tI0;
            std::vector<long> own_t;
            own_t.reserve(P);
            for (long t = 0; t < P; ++t)
                if (c.prow[t] >= o0 && c.prow[t] < o1) own_t.push_back(t);
            const long Po = (long)own_t.size();
            double pairs = 0;   // lower tile pairs of the owned row tiles: nt (nt + 1) / 2 unsharded
            for (long I = tI0; I < tI1; ++I) pairs += (double)(I + 1);
            const char *ev = getenv("LRS_SLOT_TILES");
            bool on = c.n >= kAuvMinN && (double)Po >= kAuvMinPerTile * pairs;
            if (ev && ev[0] == '0') on = false;
            if (ev && ev[0] == '1') on = Po > 0;
            if (on) {
                std::vector<std::pair<unsigned long long, int>> key(Po);
                for (long u = 0; u < Po; ++u) {
                    const long t = own_t[u];
                    const int p = c.prow[t], q = c.pcol[t];   // lower: p >= q
                    const unsigned long long tile = (unsigned long long)(p / kAuvT) * nt + (q / kAuvT);
                    key[u] = {(tile << 32) | ((unsigned)(p % kAuvT) << 16) | (unsigned)(q % kAuvT), (int)t};
                }
                std::sort(key.begin(), key.end());
                std::vector<int> item, sl(Po);
                std::vector<unsigned> pq(Po);
                long t0 = 0;
                const bool swz = tile_swizzle_on();
                std::vector<long> perm;
                for (long t = 0; t < Po; ++t) {
                    pq[t] = (unsigned)(key[t].first & 0xffffffffu);
                    sl[t] = d.slot_off + key[t].second;
                    const bool last = t + 1 == Po || (key[t + 1].first >> 32) != (key[t].first >> 32) ||
                                      t + 1 - t0 == kAuvItem;
                    if (!last) continue;
                    const unsigned long long tile = key[t].first >> 32;
                    item.push_back((int)(tile / nt) * kAuvT);
                    item.push_back((int)(tile % nt) * kAuvT);
                    item.push_back((int)t0);
                    item.push_back((int)(t + 1));
                    if (swz) {   // conflict-free LDS reads (swizzle_item)
                        swizzle_item(pq.data() + t0, t + 1 - t0, perm);
                        std::vector<unsigned> pq2(perm.size());
                        std::vector<int> sl2(perm.size());
                        for (size_t i = 0; i < perm.size(); ++i) { pq2[i] = pq[t0 + perm[i]]; sl2[i] = sl[t0 + perm[i]]; }
                        std::copy(pq2.begin(), pq2.end(), pq.begin() + t0);
                        std::copy(sl2.begin(), sl2.end(), sl.begin() + t0);
                    }
                    t0 = t + 1;
                }
                d.sa_items = (int)(item.size() / 4);
                d.sa_n = (int)Po;
                // sub-items of at most kTileSub slots (cut at multiples of 16: the swizzled groups stay whole)
                std::vector<int> sub;
                for (size_t q = 0; q < item.size(); q += 4)
                    for (int e = item[q + 2]; e < item[q + 3]; e += kTileSub)
                        sub.insert(sub.end(), {item[q], item[q + 1], e, std::min(e + kTileSub, item[q + 3])});
                d.sa_nsub = (int)(sub.size() / 4);
                // k_tile_a's groups: runs of at most kTileGrp sub-items of one row tile
                std::vector<int> grp;
                for (int q = 0; q < d.sa_nsub; ++q)
                    if (grp.empty() || q - grp.back() == kTileGrp || sub[4 * q] != sub[4 * grp.back()]) grp.push_back(q);
                d.sa_ngrp = (int)grp.size();
                grp.push_back(d.sa_nsub);
                if (!dput(&d.sa_item, item, err) || !dput(&d.sa_pq, pq, err) || !dput(&d.sa_slot, sl, err) ||
                    !dput(&d.sa_sub, sub, err) || !dput(&d.sa_grp, grp, err))
                    return false;
                // symmetric adjacency of the owned rows by (row tile I, column tile J): counting
                // sort over the row-ordered, column-sorted adjacency keeps (row, column) order
                // inside a tile pair
                long nnz = 0;
                for (int i = o0; i < o1; ++i) nnz += c.adj_ptr[i + 1] - c.adj_ptr[i];
                std::vector<long> cnt((size_t)nt * nt + 1, 0);
                for (int i = o0; i < o1; ++i)
                    for (int e = c.adj_ptr[i]; e < c.adj_ptr[i + 1]; ++e)
                        cnt[(size_t)(i / kAuvT) * nt + c.adj_col[e] / kAuvT + 1]++;
                for (size_t q = 0; q + 1 < cnt.size(); ++q) cnt[q + 1] += cnt[q];
                std::vector<int> ent(2 * std::max(1L, nnz)), epl(std::max(1L, nnz));
                std::vector<long> fill(cnt.begin(), cnt.end() - 1);
                for (int i = o0; i < o1; ++i)
                    for (int e = c.adj_ptr[i]; e < c.adj_ptr[i + 1]; ++e) {
                        const long at = fill[(size_t)(i / kAuvT) * nt + c.adj_col[e] / kAuvT]++;
                        ent[2 * at] = c.adj_col[e] % kAuvT;
                        ent[2 * at + 1] = d.slot_off + c.adj_slot[e];
                        epl[at] = i % kAuvT;
                    }
                std::vector<int> blk(2L * std::max(1L, tI1 - tI0) * kNX), tp, rp;
                for (long I = tI0; I < tI1; ++I)
                    for (int x = 0; x < kNX; ++x) {
                        blk[2 * ((I - tI0) * kNX + x)] = (int)(tp.size() / 2);
                        for (long J = x * nt / kNX; J < (x + 1) * nt / kNX; ++J) {
                            const long e0 = cnt[I * nt + J], e1 = cnt[I * nt + J + 1];
                            if (e0 == e1) continue;
                            tp.push_back((int)(J * kAuvT));
                            tp.push_back((int)rp.size());
                            long e = e0;
                            for (int r0 = 0; r0 <= kAuvT; ++r0) {
                                while (e < e1 && epl[e] < r0) ++e;
                                rp.push_back((int)e);
                            }
                        }
                        blk[2 * ((I - tI0) * kNX + x) + 1] = (int)(tp.size() / 2);
                    }
                if (tp.empty()) { tp.assign(2, 0); rp.assign(kAuvT + 1, 0); }
                d.sb_blocks = (int)((tI1 - tI0) * kNX);
                d.sb_I0 = (int)tI0;
                if (!dput(&d.sb_blk, blk, err) || !dput(&d.sb_tp, tp, err) || !dput(&d.sb_rp, rp, err) ||
                    !dput(&d.sb_ent, ent, err))
                    return false;
                // a shard: the slots whose lower row is a halo row (S for k_tile_b2's upper entries)
                if (c.own1 >= 0) {
                    std::vector<int> sx;
                    for (long t = 0; t < P; ++t)
                        if (c.prow[t] < o0 || c.prow[t] >= o1) sx.push_back(d.slot_off + (int)t);
                    d.sx_n = (int)sx.size();
                    if (sx.empty()) sx.push_back(0);
                    if (!dput(&d.sx_slot, sx, err)) return false;
                }
                if (hipMalloc((void **)&d.sa_S, (size_t)std::max(1L, P) * sizeof(double)) != hipSuccess) {
                    err = "hipMalloc failed";
                    return false;
                }
            }
        }
        d.lp = c.lp;
        if (c.lp) {
            dp.lp_cone = k;
            std::vector<int> ls(std::max(1, c.n), -1);
            for (int t = 0; t < (int)c.prow.size(); ++t) ls[c.prow[t]] = t;
            std::vector<double> nr(c.lp_nrm2);
            if (nr.empty()) nr.push_back(0.0);
            if (!dput(&d.lp_slot, ls, err) || !dput(&d.lp_nrm2, nr, err)) return false;
        }
        if (c.dense_c) {
            if (c.const_c) {
                d.dense_c = 2;
                d.c_alpha = c.c_alpha;
            } else {
                if (!dput(&d.Cd, c.Cfull, err)) return false;
                d.dense_c = 1;
            }
            dp.ndense++;
        }
    }
    return true;
}

void free_problem(DevProblem &dp) {
    auto f = [](void *p) { if (p) (void)hipFree(p); };
    f(dp.b); f(dp.Cw); f(dp.Craw); f(dp.con_ptr); f(dp.con_slot); f(dp.con_w);
    f(dp.slot_ptr); f(dp.slot_con); f(dp.slot_a); f(dp.slot_g);
    f(dp.glob); f(dp.loc_ptr); f(dp.loc_con); f(dp.loc_w); f(dp.slot1); f(dp.loc1); f(dp.slot_rc); f(dp.con1_pq); f(dp.con1_w); f(dp.long_rows);
    f(dp.sh_idx); f(dp.cmask); f(dp.bprim); f(dp.g3); f(dp.gpack); f(dp.spack);
    for (auto &c : dp.cones) { f(c.adj_ptr); f(c.adj_low); f(c.adj_col); f(c.adj_slot); f(c.dra); f(c.drb); f(c.Cd); f(c.colseg); f(c.auv_item); f(c.auv_pq); f(c.auv_pos); f(c.auv_val); f(c.sa_item); f(c.sa_sub); f(c.sa_grp); f(c.sa_pq); f(c.sa_slot);
        f(c.sb_blk); f(c.sb_tp); f(c.sb_rp); f(c.sb_ent); f(c.sa_S); f(c.sx_slot);
        f(c.cg_cadj_ptr); f(c.cg_cadj); f(c.cg_cl_con); f(c.cg_cl_ptr); f(c.cg_ce); f(c.cg_sp); f(c.cg_sj);
        f(c.cg_cc_ptr); f(c.cg_cc); f(c.cg_ce_w); f(c.cg_sa); f(c.cobj_slot); f(c.lp_slot); f(c.lp_nrm2); }
    if (dp.has_merged) {
        f(dp.merged.adj_ptr); f(dp.merged.adj_low); f(dp.merged.adj_col); f(dp.merged.adj_slot);
        f(dp.merged.dra); f(dp.merged.drb);
    }
    dp = DevProblem();
}

}  // namespace lrs
