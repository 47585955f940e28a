// lrs_device.h -- device-side data model and kernel launchers for the MI355X
// (gfx950) low-rank SDP inner solver.  Host code (lrs_solver.cpp) owns all
// scalar control; the hot path runs as the kernels declared here.
//
// Data layout in HBM (DESIGN.md "Data layout"):
//  * factors R, D, G, L-BFGS s/y, U, V: ROW-major n x ld per cone (ld = G*E >= r,
//    zero padded), all cones concatenated in one buffer ("factor buffer").  A row
//    is read by one lane group of G lanes, E consecutive doubles per lane.
//  * pattern ("slots"): the union of the lower-triangle nonzeros of C and every
//    A_i of a cone, ordered row-major (row i, col <= i); all cones' slots
//    concatenated in one global slot space.
//  * symmetric adjacency per cone (row i -> (j, slot)) for the row-owned SpMM;
//    its prefix with j <= i is the lower part used by the row-owned SDDMM.
//  * constraints: CSR over global slots with the symmetric weight folded in
//    ((2 - delta_ij) * a, data/lorads_sdp_data.c:803-856) for A(.) ; the inverse
//    slot -> (constraint, a) CSR for A^*(y) (data/lorads_sdp_data.c:878-922).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace lrs {

constexpr int kBlock = 256;          // threads per block (4 waves)
constexpr int kMaxPartialBlocks = 4096;
constexpr int kMaxPartialVals = 16;

// ---- ALM inner-loop control block (double array, double-buffered by iteration parity)
enum CtrlIdx {
    C_ACTIVE = 0,   // 1 while the inner L-BFGS loop runs
    C_EXIT,         // exit reason (ExitReason)
    C_INNER,        // alm_state.innerIter
    C_LOCAL,        // localIter
    C_CLEAR,        // clearLBFGS
    C_HEAD,         // L-BFGS ring head (next slot to write)
    C_GCUR,         // which G buffer holds the current gradient
    C_PENDING,      // previous iteration left partials to fold
    C_RCVAL,        // rho_certificate_val
    C_LAG,          // ||G||^2
    C_PINF1,        // l_1 primal infeasibility
    C_PINFINF,      // l_inf primal infeasibility
    C_BETA0, C_BETA1,   // 1/<y,s> per ring slot
    C_YY0, C_YY1,       // <y,y> per ring slot
    C_NODENUM,
    C_CG, C_CS0, C_CY0, C_CS1, C_CY1,  // D = -(cG G + cs0 s0 + cy0 y0 + cs1 s1 + cy1 y1)
    C_DG,           // <D, G> after LBFGSDirectionUseGrad
    C_LASTTAU,
    // dots of the current gradient with the ring (stash, valid when PENDING == 2)
    C_DSG, C_DYG, C_DSOG, C_DYOG, C_DSOY, C_DYOY,
    // written by the gather stage of the split iteration (authoritative after it ran)
    C_ACT2,         // ACTIVE after the phase-1 (l_inf pinf) test of the completed iteration
    C_EXIT2,        // exit reason after that test
    C_RRDONE,       // 1 if this iteration's first stage refreshed A(RR^T) and the residual
    C_RCUR,         // which factor buffer (R, R2) holds the current iterate
    C_NCTRL = 40
};
enum ExitReason {
    EXIT_NONE = 0,
    EXIT_CONVERGED = 1,   // rho_certificate_val - tol <= endALMSubTol (while condition)
    EXIT_PHASE1 = 2,      // l_inf pinf <= phase1Tol  -> END_ALM
    EXIT_LOCAL800 = 3,    // localIter > 800          -> break
    EXIT_TINYTAU = 4,     // |tau| < endTauTol        -> UpdateRho
    EXIT_NUMERR = 5,      // no root                  -> RET_CODE_NUM_ERR
    EXIT_BUDGET = 6,      // bench budget of inner iterations reached
    EXIT_XWG = 7          // one-workgroup-per-cone loop: the workgroups' exchange timed out (an error)
};
// ---- parameters read by the device loop
enum ParIdx {
    P_RHO = 0, P_RCTOL, P_ENDSUB, P_ENDTAU, P_PH1TOL, P_BN1, P_BNINF, P_CNINF,
    P_HIGHACC, P_BUDGET, P_L, P_GAP, P_NPAR = 16
};
// ---- line-search result, double-buffered by parity: tau, rootNum, flag
enum LsIdx { LS_TAU = 0, LS_ROOTNUM, LS_FLAG, LS_N = 4 };
// ---- finals of the standalone launchers (offsets into the per-context tmpfin scratch)
constexpr int kMaxCones = 256;
constexpr int kFinN = 416;           // per-context finals of the line search / direction kernels (FinIdx)
// TF_DOTC + k: cone k's <X, C Y> of a dense objective (op_constr_xx), read with the gather's sums
enum TmpFinIdx {
    TF_SD = 0, TF_GATHER = 2 * kMaxCones, TF_RESID, TF_DOT, TF_DOTC, TF_SPMM = TF_DOTC + kMaxCones,
    TF_N = TF_SPMM + kMaxCones
};
constexpr int kMaxShards = 64;       // processes of one sharded solve
constexpr int kLongRow = 32;         // constraint rows longer than this get a wave each

struct Layout {
    int G = 1, E = 1, ld = 1;
};
Layout choose_layout(int r);

struct DevCone {
    int n = 0, r = 0, ld = 0, G = 0, E = 0;
    bool lp = false;    // the LP block as the diagonal cone at rank 1 (lrs_problem.cpp build_problem)
    // LP cone: per row (LP column) its local slot or -1 (a column without data), and per row
    // the column's squared 2-norm (lp_cone_presolve nrm2Square, lorads_lp_conic.c:132-133)
    int *lp_slot = nullptr;
    double *lp_nrm2 = nullptr;
    // rows the kernels compute: [row0, row0 + nown) -- the whole cone, or in a sharded
    // solve this process's rows (the others, the halo, are read as neighbours only)
    int row0 = 0, nown = 0;
    long foff = 0;      // offset (doubles) of this cone in the factor buffer
    int slot_off = 0, P = 0;
    int *adj_ptr = nullptr, *adj_low = nullptr, *adj_col = nullptr, *adj_slot = nullptr;
    long adj_nnz = 0;
    // constraint i of this cone is the single entry (i, i), every i (m = n): k_auv_diag
    bool auv_diag = false;
    // most adjacency entries of one row (all, and lower incl. the diagonal); 0 = unknown
    int maxdeg = 0, maxlow = 0;
    // dense rows (far more entries than the rest, e.g. a hub vertex): the latency kernels
    // spread their entries over extra slice blocks.  A: rows whose lower part has more than
    // kDenseRow entries; B: rows whose adjacency has.  Host ids (for the grids) and device copies.
    std::vector<int> dra_h, drb_h;
    std::vector<int> dra_n, drb_n;       // their entry counts (A: lower incl. diagonal, B: all)
    int *dra = nullptr, *drb = nullptr;
    long gl_need = 0;                    // doubles of slice gradients the B slices can need (any layout)
    // dense objective (lrs_problem.h), not in the slots: 1 = C as a full n x n row-major
    // matrix, 2 = the constant C = c_alpha J (rank-one products, no matrix)
    int dense_c = 0;
    double *Cd = nullptr;
    double c_alpha = 0.0;
    // long rows (>= kTileMinDeg adjacency entries per row on average): per row, the first entry
    // at or past column x n / kNX, x = 0..kNX ([n][kNX + 1]); the column-tiled k_wide_* kernels
    int *colseg = nullptr;
    // A(X Y^T) over 2-D tiles (many constraint entries per row, e.g. C5): the cone's constraint
    // entries bucketed by (row tile, column tile) of kAuvT rows each, items of at most kAuvItem
    // entries {row0, col0, begin, end}, per tiled entry its local (row, col) packed 16:16 and its
    // constraint entry (cone order), and the per-entry values in cone entry order (scratch)
    int auv_items = 0;
    long auv_ebase = 0;                  // first constraint entry of this cone (con_ptr[k m])
    int *auv_item = nullptr;             // [items][4]
    unsigned *auv_pq = nullptr;          // [Zk]
    int *auv_pos = nullptr;              // [Zk]
    double *auv_val = nullptr;           // [Zk]
    // the lower pattern in the same 2-D tiles (k_tile_a, stage A of the long-row path): items
    // {row0, col0, begin, end}, per tiled slot its local (row, col) 16:16 and its global slot
    int sa_items = 0;
    int sa_n = 0;                        // tiled slots (sa_slot's length)
    int *sa_item = nullptr;
    int sa_nsub = 0;                     // the items cut at kTileSub slots (k_tile_a's sub-items)
    int *sa_sub = nullptr;
    int sa_ngrp = 0;                     // runs of <= kTileGrp sub-items of one row tile: [ngrp + 1] starts
    int *sa_grp = nullptr;
    unsigned *sa_pq = nullptr;
    int *sa_slot = nullptr;
    // stage B's gradient S R_new over the symmetric pattern in the same tiles (k_tile_b2): one
    // block per (row tile I, column group x of kNX), its tile pairs {col0, row-pointer offset}
    // ([nt * kNX][2] ranges into sb_tp), per tile pair kAuvT + 1 row pointers into the entries
    // {local column, slot}; sa_S holds the slot values of S = C + A^*(M1) between the two kernels
    int sb_blocks = 0;
    int *sb_blk = nullptr, *sb_tp = nullptr, *sb_rp = nullptr, *sb_ent = nullptr;
    double *sa_S = nullptr;
    // sharded solve: the tiles cover the owned rows only -- sa_* the owned rows' lower slots,
    // sb_* the row tiles from sb_I0 on; sx_slot the slots whose lower row is a halo row (the
    // upper entries of owned rows), whose S k_slot_sv forms for k_tile_b2
    int sb_I0 = 0;
    int sx_n = 0;
    int *sx_slot = nullptr;
    // single-workgroup ADMM half-step (launch_small_cg; small unsharded cones, lrs_problem.cpp):
    // the constraint slots (slots with a constraint entry, cg_ncs) and their symmetric adjacency
    // per row packed (col << 16 | constraint slot); the cone's constraints in compact order (the
    // cg_ns short ones, then the long ones; cg_cl_con their ids) with their entries packed
    // (constraint slot << 1 | diagonal) and weights (2 - delta) a; per constraint slot its
    // (compact constraint, a) pairs; the objective as constant (cg_cconst 1: slot form, alpha =
    // Craw[cg_cslot]; 2: the rank-one form) or its entries per row (col, global slot)
    int cg_ok = 0, cg_ncs = 0, cg_ncl = 0, cg_ns = 0, cg_nce = 0, cg_nsc = 0, cg_nadj = 0, cg_cconst = 0, cg_cslot = 0;
    int *cg_cadj_ptr = nullptr, *cg_cadj = nullptr, *cg_cl_con = nullptr, *cg_cl_ptr = nullptr, *cg_ce = nullptr;
    int *cg_sp = nullptr, *cg_sj = nullptr, *cg_cc_ptr = nullptr, *cg_cc = nullptr;
    double *cg_ce_w = nullptr, *cg_sa = nullptr;
    // a cone with constraint-entry tiles (auv_items): the global slots holding C entries, for
    // <C, X Y^T> straight from the factor rows (launch_cobj)
    int cobj_n = 0;
    int *cobj_slot = nullptr;
};
constexpr int kScMaxN = 256;         // rows of a cone the single-workgroup ADMM half-step takes
constexpr int kMaxRankLd = 512;      // widest factor row (choose_layout: 64 lanes x 8 doubles)
constexpr int kAuvT = 128;           // rows of one side of an A(X Y^T) tile
constexpr int kAuvC = 32;            // factor columns staged in LDS at a time
constexpr int kAuvThreads = 512;
constexpr int kAuvNpt = 8;           // entries per thread of one item
constexpr int kAuvItem = kAuvThreads * kAuvNpt;
constexpr int kTileSub = 1024;       // slots of one k_tile_a sub-item (one a thread)
constexpr int kTileGrp = 2;          // most sub-items of one k_tile_a group (one row tile)
constexpr int kAuvMinN = 2048;       // tiled when n >= this and the lower triangle's tiles hold on average
constexpr int kAuvMinPerTile = 768;  //   >= this many entries (constraint entries for A(X Y^T), pattern slots
                                     //   for the stage kernels: 3x reuse of each staged row); C5 ~1850, a
                                     //   C5-structured m = 1e5 ~98 (slower tiled); LRS_AUV_TILES /
                                     //   LRS_SLOT_TILES = 0/1 override
constexpr int kCgSplitSlabs = 8;      // k_cgemm2's most K-slices (DevWork::CGK slabs)
constexpr int kNX = 8;              // column blocks of the tiled long-row kernels (one per XCD)
constexpr int kTileMinDeg = 32;
constexpr int kDenseRow = 64;        // entries of a row past which the latency kernels slice it
constexpr int kSliceMinB = 28;       // fewest entries of one B slice block (G = 64: 7 groups x 4)
constexpr int kMaxDenseRows = 32;    // more dense rows than this: the general row kernels

// Sharded solve (one process per GPU, rows of the cone split into contiguous blocks):
// the collectives the split iteration calls between its stages, provided by the host
// (lrs_solver.cpp: RCCL, or the one-process loopback transport of the tests).
struct ShardHooks {
    void *self = nullptr;
    // direction rows D of this shard's halo from their owners (and its rows to theirs)
    int (*halo)(void *self, double *D, hipStream_t st) = nullptr;
    // in-place sum over the shards of n contiguous doubles in device memory
    int (*allreduce)(void *self, double *buf, int n, hipStream_t st) = nullptr;
};

struct DevProblem {
    const ShardHooks *shard = nullptr;   // non-null in a sharded solve
    int no_lat = 0;                      // kernel path (lrs_set_kernel_path): 1 never the latency kernels, 2 + bandwidth regime, 3 + long-row kernels, 4 the single-workgroup inner loop
    int *slot_g = nullptr;               // [Ptot][2] every slot's (row, col) in the all-cones row space
    mutable int last_path = -1;          // path of the last enqueued iteration (0 lat, 1 general)
    mutable int last_tiles = 0;          // the last enqueued iteration ran stage A / B over the 2-D tiles
    int m = 0, K = 0;
    int lp_cone = -1;   // the LP block's cone (the last), -1 without one
    long NRpad = 0;     // factor buffer length (doubles)
    int Ptot = 0;
    long Z = 0;
    double *b = nullptr;
    double *Cw = nullptr, *Craw = nullptr;                   // [Ptot]
    int *con_ptr = nullptr, *con_slot = nullptr;             // [m+1], [Z]
    double *con_w = nullptr;                                 // [Z]
    int *slot_ptr = nullptr, *slot_con = nullptr;            // [Ptot+1], [Z]
    double *slot_a = nullptr;                                // [Z]
    // single-slot ("local") constraints per slot, and the list of the others
    int mg = 0;                                              // number of global constraints
    int glob_maxlen = 0;                                     // most entries of one global constraint
    int *glob = nullptr;                                     // [mg]
    int *loc_ptr = nullptr, *loc_con = nullptr;              // [Ptot+1], [m - mg]
    double *loc_w = nullptr;                                 // (2 - delta) a of that one entry
    int *slot_rc = nullptr;                                  // [Ptot][2] (row, col) in the cone
    double *slot1 = nullptr;                                 // [Ptot][2] {a, con} of a slot's single
                                                             //   constraint entry (con -1 none, -2 several)
    double *loc1 = nullptr;                                  // [Ptot][2] {w, con} of its single local constraint
    int *con1_pq = nullptr;                                  // [K*m][2] single-entry rows: (p, q); -1 other; -2 long
    int *long_rows = nullptr;                                // constraints with > kLongRow entries in a cone,
    std::vector<int> long_ptr_h;                             //   grouped by cone: long_ptr_h[k]..[k+1]
    double *con1_w = nullptr;                                // [K*m] their weight
    // sharded solve: constraints held by several shards ("shared", lrs_problem.h ShardPlan)
    int nsh = 0;                                             // shared constraints (same on every shard)
    int *sh_idx = nullptr;                                   // [m] local constraint -> shared index, -1
    double *cmask = nullptr;                                 // [m] 1 where this shard counts the constraint
    double *bprim = nullptr;                                 // [m] b * cmask (b^T lambda counted once)
    double *g3 = nullptr;                                    // [3][m] owned-slot sums RR, RD, DD (global cons)
    double *gpack = nullptr;                                 // [nsh][3] the shared ones, all-reduced
    double *spack = nullptr;                                 // [nsh] one m-vector's shared entries
    std::vector<DevCone> cones;
    int ndense = 0;                                          // cones with a dense objective (DevCone::Cd)
    bool tiles = false;                                      // column-tiled long-row kernels (LRS_TILES=1 at alloc)
    double *gp = nullptr;                                    // DevWork::GP (kNX partial factors), the tiled S X's scratch
    double *cgk = nullptr;                                   // DevWork::CGK: k_cgemm2's split-K slabs (kCgSplitSlabs x NRpad)
    double dense_scale = 1.0;                                // objScale_dualvar's factor on those C
    // K > 1: all cones as one block-diagonal row space (global rows and columns); used by
    // the split iteration when every cone has the same (G, E) row layout
    DevCone merged;
    bool has_merged = false;
    bool cone_sep = false;                                   // every constraint's entries lie in one cone
};

// Scratch shared by the kernels of one solve.
struct DevWork {
    double *R = nullptr, *D = nullptr, *G[2] = {nullptr, nullptr};
    double *R2 = nullptr;      // second factor buffer of the split iteration (R double-buffered)
    // dense-objective cones (DevCone::Cd): C R of the current iterate (carried C R + tau C D
    // through the inner loop, recomputed by op_grad) and C D of the iteration; zero elsewhere
    double *CR = nullptr, *CD = nullptr;
    double *CGK = nullptr;   // k_cgemm2's split-K slabs (dense cones of >= 2048 rows): kCgSplitSlabs x NR
    // column-tiled long-row kernels: kNX partial S R_new factors (kNX * NRpad), null when no cone
    // has long rows
    double *GP = nullptr;
    double *ls[2] = {nullptr, nullptr}, *ly[2] = {nullptr, nullptr};
    double *U = nullptr, *V = nullptr, *X = nullptr;         // ADMM / scratch factors
    double *cg_r = nullptr, *cg_p = nullptr, *cg_Q = nullptr, *cg_b = nullptr, *M2 = nullptr;
    double *uvt0 = nullptr, *uvt1 = nullptr, *uvt2 = nullptr, *S = nullptr;   // [Ptot]
    double *uvp = nullptr;   // [Ptot][2] the tiled stage A's (sym(RD^T), DD^T) per slot, for k_it_g
    double *lam = nullptr, *cvs = nullptr, *q1 = nullptr, *q2 = nullptr, *M1 = nullptr, *wtmp = nullptr;
    double *cvc = nullptr;                                   // per-cone A(UV^T), K*m
    double *lpw = nullptr;                                   // the LP sweep's scratch (lp_sweep_scratch)
    double *part = nullptr;    // [kMaxPartialVals][kMaxPartialBlocks] partial sums (scratch A)
    double *partB = nullptr;   // second partial buffer (scratch B)
    double *partC = nullptr;   // third partial buffer (scratch C)
    double *ctrl = nullptr;    // [2][C_NCTRL]
    double *lsres = nullptr;   // [2][LS_N]
    double *par = nullptr;     // [P_NPAR]
    double *gram = nullptr;    // gram partials
    double *rec = nullptr;     // [m][4] per-constraint {A(RR^T), q1, q2, -lam - rho b}
    double *cgc = nullptr;     // [8] device CG control (CgIdx)
    double *tot = nullptr;     // [32] sharded solve: summed stage totals (A: 0..7, B: 16..25)
    double *gl = nullptr;      // latency kernels: partial gradients of the dense rows' slices [slices][ld]
    long gl_len = 0;
};

// ---------------------------- launchers -----------------------------------
// All launchers enqueue on `st` and return hipSuccess / an error code.

// uvt_out0[slot] (and uvt_out1) over the cone's pattern; objective partials
// sum_slot Cw*uvt -> part[0 or 1][pblk_off + b].  mode: 0 = sym(X Y^T),
// 1 = X X^T (Y ignored), 2 = sym(X Y^T) into out0 and Y Y^T into out1.
int launch_sddmm(const DevProblem &P, int cone, int mode, const double *X, const double *Y,
                 double *out0, double *out1, double *part, int pblk_off, int *nblk_used,
                 hipStream_t st);
// out[i] = scale * sum_e w_e uvt[slot_e] for every constraint (A(.)), plus
// partial sum of (b - out)^2 if vio_part != nullptr (primal residual).
int launch_gather(const DevProblem &P, const double *uvt, double scale, double *out,
                  const double *b_for_vio, double *vio_part, hipStream_t st, int *nblk_used);
// Constraint-entry A(.) of one cone without the pattern pass: every constraint's
// entries of cone `cone` read their two factor rows directly (mode 0: sym(X Y^T),
// mode 1: X X^T).  out[i] = (accumulate ? out[i] : 0) + scale * value_of_this_cone; optional
// residual sum (b - out)^2 -> tmpfin TF_GATHER.  Bitwise equal to sddmm + gather_cone.
int launch_auv_con(const DevProblem &P, int cone, int mode, const double *X, const double *Y, double scale,
                   int accumulate, double *out, const double *b_for_vio, double *vio_part, hipStream_t st,
                   const double *guard = nullptr, double *sum_upd = nullptr);   // sum_upd[i] += new - old out[i]
// <C, sym(X Y^T)> (mode 0) or <C, X X^T> (mode 1) of a cone with constraint-entry tiles over
// its C entries only (DevCone::cobj_slot), into tmpfin TF_SD + 2 cone (as launch_sddmm's sums)
int launch_cobj(const DevProblem &P, int cone, int mode, const double *X, const double *Y, double *part,
                hipStream_t st);
// S[slot] = (withC ? Craw[slot] : 0) + sum_(con,a) w[con] * a
int launch_wsum(const DevProblem &P, const double *w, int withC, double *S, hipStream_t st);
// out = scale * S X (+ addX * X) per cone, partial ||out||^2 -> part[0][pblk_off+b]
int launch_spmm(const DevProblem &P, int cone, const double *S, const double *X, double scale,
                const double *addX, double addScale, double *out, double *part, int pblk_off,
                int *nblk_used, hipStream_t st);
// generic BLAS-1 over the factor buffer / m-vectors with partial dots
int launch_axpby(long n, double a, const double *x, double b, double *y, hipStream_t st);
int launch_dot(long n, const double *x, const double *y, double *part, hipStream_t st, int *nblk_used,
               int fin = TF_DOT);
int launch_fill(long n, double v, double *x, hipStream_t st);
// lam += rho (b - cvs)
int launch_dual_update(const DevProblem &P, double rho, double *lam, const double *cvs, hipStream_t st);
// M1 = -lam - rho b + rho cvs   (ALMSetGrad, lorads_alm.c:38-50)
int launch_alm_m1(const DevProblem &P, double rho, const double *lam, const double *cvs, double *M1,
                  hipStream_t st);
// r x r Gram X^T X (avg=0) or ((U+V)/2)^T((U+V)/2) (avg=1) of one cone, one launch:
// gram[0, r*r) <- the Gram, gram[r*r, ...) chunk partials (gram_buf_len(rmax) doubles)
constexpr int kGramMaxChunks = 64;
size_t gram_buf_len(int rmax);
int launch_gram(const DevProblem &P, int cone, const double *X, const double *Y, int avg,
                double *gram, int *nblk_used, hipStream_t st, bool reduce = true);
// sustained v_mfma_f64_16x16x4f64 rate: every CU, 2 waves a SIMD, 8 accumulators a wave
int mfma_f64_peak(hipStream_t st, double *tflops);
int mfma_f64_probe(hipStream_t st, int wps, int chains, double *tflops, double *mhz, double *cyc_per_mfma);
// dense objective of cone `cone` (DevCone::Cd): Y = scale C X + beta Y on the cone's rows
// (X, Y full factor buffers; columns r..ld of Y written 0)
int launch_dense_cx(const DevProblem &P, int cone, const double *X, double *Y, double beta, hipStream_t st);
// ALM iteration, between stage A and B: CD = scale C D of every dense cone, and the partials
// <R, CD>, <D, CD> (slots 0, 1 of 8) of stage A's objective terms at partial offset `off`
// (R: the current iterate by the control block); returns the partial blocks written
int dense_cd_blocks(const DevProblem &P);
int launch_dense_cd(const DevProblem &P, const DevWork &W, const double *ctrl, int off, hipStream_t st);

// ---- fused ALM inner iteration (device-side control; see lrs_kernels.hip) ----
struct AlmIterArgs {
    const DevProblem *P;
    DevWork *W;
    hipEvent_t *ev;    // optional: 5 events recorded before S1..S4 and after S4
    double *hmirror = nullptr;   // optional: device pointer of a pinned host slot; stage B
    double seq = 0;              // mirrors the control block there, then writes seq after it
};
// Four launches per inner iteration (lrs_kernels.hip "split iteration").
int enqueue_alm_iteration(const AlmIterArgs &a, int parity, hipStream_t st);
// whether stage A is split into direction + SDDMM launches (bandwidth regime)
bool alm_stage_a_split(const DevProblem &P);
bool alm_stage_b_split(const DevProblem &P);   // stage B likewise (line search + update, gradient)
// a subset of the stages (mask bit 0 = A, 1 = G, 2 = B), for per-stage timing
int enqueue_alm_stages(const AlmIterArgs &a, int parity, int mask, hipStream_t st);

// ---- single-workgroup persistent inner loop (lrs_kernels.hip "Single-workgroup"): small
// problems (R and D of every cone in one CU's LDS, ld <= 64, no full dense C) ----
bool small_alm_fits(const DevProblem &P, DevWork &W);
// workgroups of the single-workgroup inner loop for this problem (> 1: one per cone, the
// exchanges between them), 0 when it does not fit
int small_alm_workgroups(const DevProblem &P, DevWork &W);
int launch_small_alm(const DevProblem &P, DevWork &W, const double *ctrl_in, double *ctrl_out, double *ls_out,
                     hipStream_t st);

// ---- device-resident CG (lrs_kernels.hip "Device-resident CG") ----
enum CgIdx { CG_ACTIVE = 0, CG_ITERS, CG_BNORM, CG_RR, CG_QTR0, CG_QTR1, CG_TOTAL, CG_N = 8 };
int launch_cg_mv(const DevProblem &P, int cone, const double *w, const double *V, const double *Xin, double *Q,
                 double *part, const double *cgc, int guarded, hipStream_t st, int *nblk);
int launch_cg_nrm1(long nr, const double *b, double *part, hipStream_t st, int *nblk);
int launch_cg_upd(long nr, double *X, double *r, const double *p, const double *Q, const double *partB, int nblkB,
                  double *partC, double *cgc, int par, int it, hipStream_t st, int *nblk);
int launch_cg_conv(long nr, const double *r, double *p, const double *partC, int nblkC, double *cgc, double tol,
                   int par, int restart, hipStream_t st);
int launch_cg_resid(long nr, const double *b, const double *Q, double *r, double *p, double *partC, double *cgc,
                    const double *partA, int nblkA, int init, hipStream_t st, int *nblk);
int launch_cg_resid2(long nr, const double *r, double *p, const double *partC, int nblkC, double *cgc, double tol,
                     int par, int init, hipStream_t st);
// single-workgroup ADMM half-step of cone `cone` (LORADSUpdateSDPVarOne + CGSolve + the cone's
// constraint refresh, one launch): side 0 solves U with V fixed, 1 V with U fixed; the RHS into
// W.cg_b, this solve's CG iterations into W.cgc[CG_ITERS], added to W.cgc[CG_TOTAL]
bool small_cg_fits(const DevProblem &P, int cone);
int launch_small_cg(const DevProblem &P, DevWork &W, int cone, int side, double rho, double tol, int maxit,
                    hipStream_t st);
// every cone's half-step of one side in one launch (a block a cone; cones whose constraints
// each lie in one cone, all fitting k_small_cg with the same variant)
bool small_cg_batch_fits(const DevProblem &P);
// the ADMM iteration's evaluation (R = (U + V) / 2, A(R R^T) into cvs / cvc, and per cone
// {sum (b - A(X))^2, <C, R R^T>, b^T lambda} into out[4k..]) in one launch, a block a cone
bool small_eval_fits(const DevProblem &P);
int launch_small_eval(const DevProblem &P, DevWork &W, const double *U, const double *V, double *out, hipStream_t st);
// the LP block's ADMM update: the reference's closed-form column sweep (k_lp_admm), both sides
int launch_lp_admm(const DevProblem &P, DevWork &W, double rho, hipStream_t st);
long lp_sweep_scratch(const DevProblem &P);
int launch_small_cg_batch(const DevProblem &P, DevWork &W, int side, double rho, double tol, int maxit,
                          hipStream_t st);

// ---- dual infeasibility (Lanczos for lambda_min of S per cone) ----
// y = S x over one cone's adjacency (S on the global slots, x / y cone-local vectors)
int launch_symv(const DevProblem &P, int cone, const double *S, const double *x, double *y, hipStream_t st);
// w -= Q (Q^T w): Q column-major n x k (leading dimension ldq); part >= 64 k doubles, h >= k
int launch_reorth(int n, int k, const double *Q, long ldq, double *w, double *part, double *h, hipStream_t st);
// thick-restart Lanczos (ARPACK dsaupd semantics, lrs_solver.cpp trl_min): one step's launches.
// Vectors are cone-local rows; norm / dots / sub / restart take pointers pre-offset to the first
// owned row and n = owned rows; symv runs the cone's owned rows [row0, row0 + nown) itself.
constexpr int kTrlMaxV = 64;   // basis vectors at most (ncv = 40 in the reference)
int trl_nblk(int n);           // partial blocks per column of launch_trl_dots
int launch_trl_norm(int n, const double *w, const double *b2, double *vj, hipStream_t st);
// y = S (x / sqrt(*b2)) (+ scale C v on a dense cone); vj (optional) = x / sqrt(*b2); b2 = null: 1
int launch_trl_symv(const DevProblem &P, int cone, const double *S, const double *x, const double *b2, double *vj,
                    double *y, hipStream_t st);
int launch_trl_dots(int n, const double *V, long ldv, int k, const double *y, double *part, hipStream_t st);
int launch_trl_fold(int k, int nb, const double *part, double *tot, hipStream_t st);
int launch_trl_sub(int n, const double *V, long ldv, int k, const double *part, int nb, double *y, double *Hc,
                   int pass, double *npart, double *bw2, hipStream_t st);
int launch_trl_restart(int n, const double *V, long ldv, int m, const double *Y, int kk, double *Vt, hipStream_t st);

// per-context scratch of the standalone reductions for the calling thread (no module-level fallback)
void bind_scratch(unsigned *tickets, double *tmpfin, double *rpart, double *fin);
// sharded solve helpers
int launch_pack_rows(int nrows, int ld, const int *rows, const double *src, double *dst, hipStream_t st);
// sharded: sum an m-vector's shared-constraint entries over the shards (no-op otherwise)
int sync_shared(const DevProblem &P, double *v, hipStream_t st);
// fold one scalar's per-block partials into out[0] (sharded CG, before its all-reduce)
int launch_fold1(const double *part, int nblk, double *out, hipStream_t st);
// par[P_NPAR] and ctl[C_NCTRL] (host arrays) into dpar / dctl, stream-ordered, as one launch
int launch_put_ctrl(const double *par, const double *ctl, double *dpar, double *dctl, hipStream_t st);
int launch_sum_shards(int n, int world, const double *const *src, double *out, hipStream_t st);

const char *last_device_error();
// diagnostics build only: copies g_phase[4][16] (returns 64), else returns 0
int read_phase_times(unsigned long long *out, unsigned long long *blk);

}  // namespace lrs
