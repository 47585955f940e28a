// lrs_solver.cpp -- host control of the solve (ALM phase 1, ADMM phase 2) on
// top of the device operators, and the C-ABI of include/lrsdp.h.
//
// The control flow restates the reference (paths relative to
// /root/reference/lorads/src/src_semi): LORADS_ALMOptimize lorads_alm.c:1220-1484,
// LORADSADMMOptimize lorads_alg/lorads_admm.c:84-209, LORADS_ALMtoADMM
// data/lorads_solver.c:1351-1387, main.c:380-610.  The ALM inner L-BFGS loop
// runs as batches of fused device iterations (enqueue_alm_iteration) with
// device-side control; the host only intervenes between inner loops.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <limits>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/lrsdp.h"
#include "lrs_device.h"
#include "lrs_problem.h"

namespace lrs {
double *device_tmpfin();
int launch_gather_cone(const DevProblem &P, int cone, const double *uvt, double *out, hipStream_t st);
int launch_resid(int m, const double *b, const double *x, hipStream_t st, const double *mask = nullptr);
int launch_avg(long n, const double *U, const double *V, double *R, hipStream_t st);
int launch_admm_m1(int m, double rho, const double *b, const double *cvs, const double *cv, const double *lam,
                   double *M1, hipStream_t st);
int launch_ls_only(const DevProblem &P, DevWork &W, hipStream_t st);
int launch_alm_dir_only(const DevProblem &P, DevWork &W, hipStream_t st);
}  // namespace lrs

using namespace lrs;

static thread_local std::string g_lrs_err;
static void set_err(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_lrs_err = buf;
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define HIPC(x)                                                                               \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            set_err("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_));          \
            return -1;                                                                        \
        }                                                                                     \
    } while (0)
#define OPC(x)                                                                                \
    do {                                                                                      \
        int r_ = (x);                                                                         \
        if (r_ != 0) {                                                                        \
            set_err("%s:%d %s failed: %s", __FILE__, __LINE__, #x, last_device_error());     \
            return -1;                                                                        \
        }                                                                                     \
    } while (0)

// glibc random_r TYPE_3 restated (srand(925) initial point, data/lorads_solver.c:625, :529-539)
struct GlibcRand {
    int32_t t[31];
    int f = 0;
    explicit GlibcRand(unsigned seed) {
        int32_t r[344];
        if (seed == 0) seed = 1;
        r[0] = (int32_t)seed;
        for (int i = 1; i < 31; i++) {
            int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
            int64_t w = 16807 * lo - 2836 * hi;
            if (w < 0) w += 2147483647;
            r[i] = (int32_t)w;
        }
        for (int i = 31; i < 34; i++) r[i] = r[i - 31];
        for (int i = 34; i < 344; i++) r[i] = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
        for (int i = 0; i < 31; i++) t[i] = r[313 + i];
    }
    int next() {
        int i = f, j = (f + 28) % 31;
        int32_t v = (int32_t)((uint32_t)t[i] + (uint32_t)t[j]);
        t[i] = v;
        f = (f + 1) % 31;
        return (int)((uint32_t)v >> 1);
    }
};

struct AlmState {
    long outerIter = 0, innerIter = 0;
    double rho = 0, pobj = 1e30, dobj = 1e30, pinf1 = 1e30, pinfinf = 1e30, gap = 0;
};
struct AdmmState {
    long iter = 0, cg_iter = 0;
    double rho = 0, pobj = 1e30, dobj = 1e30, pinf1 = 1e30, pinfinf = 1e30, gap = 1e30;
};

// Pinned host scratch (lrs_ctx::hpin), one region per user, so that reads staged behind one
// sync never overlap: standalone reads (read_tmpfin, lrs_time_stages), the two ALM control
// mirrors, the device CG's control-block poll, the CG total read behind admm_eval's sync, the
// line search of the generic L-BFGS loop, and read_tmpfin2's several ranges.
enum HpinSlot {
    kHpRead = 0, kHpReadN = 128,
    kHpCtrl = 128,          // 2 x 64: [128, 256)
    kHpCg = 256,            // CG_N (8)
    kHpCgTotal = 300,       // 1
    kHpLs = 512,            // LS_N (4)
    kHpRead2 = 1024, kHpRead2N = 1024,
    kHpinN = 4096
};
static_assert(CG_N <= kHpCgTotal - kHpCg && 2 * 64 <= kHpCg - kHpCtrl && LS_N <= kHpRead2 - kHpLs, "pinned layout");

struct lrs_ctx {
    int device = 0;
    hipStream_t st = nullptr;
    HostProblem hp;
    DevProblem dp;
    bool loaded = false;
    std::vector<int> rank, rank_max;
    std::vector<Layout> lay;
    DevWork W;
    bool walloc = false;
    double *hpin = nullptr;     // pinned scalars (layout: HpinSlot)
    double *hgram = nullptr;    // pinned: every cone's r x r Gram of one oracle-rank evaluation
    size_t hgram_n = 0;
    bool naive_warned = false;   // --oracleRankNaive: the fallback line printed this solve
    // one-workgroup-per-cone inner loop: the pre-launch state (xwg_snapshot), whether an exchange
    // timed out in this context (the multi-launch iteration from then on) and how often
    double *xwg_snap = nullptr;
    long xwg_snap_len = 0;
    bool small_off = false;
    int xwg_fallbacks = 0;
    // L-BFGS mirror
    int head = 0, gcur = 0;
    double beta[2] = {0, 0}, yy[2] = {0, 0};
    double scaleObjHis = 1.0;
    double pObjVal = 0, dObjVal = 0, dimPinf = 0, dimGap = 0;
    std::vector<int> t1c, t1o, t2c, t2o;
    long cgIterTotal = 0;
    std::vector<long> cgIterCone;
    bool cg_dev_total = false;   // some half-step of this ADMM iteration counted its CG on the device
    std::string path;
    FILE *logfp = nullptr;
    // hipGraph cache of inner-iteration batches (keyed by batch size; the kernels'
    // arguments are the workspace pointers, so a new workspace drops the cache)
    std::map<int, hipGraphExec_t> graphs;
    // per-cone thick-restart Lanczos workspace (dual infeasibility), kept across calls and
    // re-allocated only when the cone's local row count changes; no captured graphs
    struct LzWork {
        int n = 0;                 // local rows the buffers are sized for
        double *V = nullptr;       // basis: kTrlMaxV + 1 vectors of n doubles
        double *Vt = nullptr;      // restart product (kTrlMaxV vectors)
        double *y[2] = {nullptr, nullptr};
        double *part = nullptr;    // dot partials [kTrlMaxV][64] + norm partials [kMaxPartialBlocks]
        double *H = nullptr;       // coefficient columns [kTrlMaxV][kTrlMaxV + 1] + bw2 [kTrlMaxV] + tot
        double *Y = nullptr;       // restart coefficients (ncv x kk)
    };
    std::vector<LzWork> lz;
    double *d_sendvec = nullptr;   // sharded: packed send rows of one Lanczos vector
    long sendvec_len = 0;
    // initial point cache (device layout, host copy) for the ranks it was drawn at
    std::vector<int> init_ranks;
    std::vector<double> init_cache;
    // running estimate of inner iterations per run_inner call (first batch size)
    double inner_est = 8.0;
    bool use_graphs = false;   // eager launches measured faster than graph replay (LRS_GRAPHS=1)
    // per-stage event profiling (lrs_profile_stages)
    bool prof = false;
    // host-loop statistics (LRS_STATS=1): run_inner calls, batches, iterations, seconds
    bool stats = false;
    long st_calls = 0, st_batches = 0, st_iters = 0, st_nop = 0;
    double st_inner_s = 0;
    hipEvent_t pev[2][5] = {};
    hipEvent_t bev[2] = {nullptr, nullptr};   // completion of the two batches in flight (run_inner)
    int pipe_batch = 8;                         // iterations per pipelined batch (LRS_PIPE_BATCH)
    int cg_slack = 1;                           // CG first batch = previous count + slack (LRS_CG_SLACK)
    double *hmir = nullptr, *dmir = nullptr;    // pinned control mirror [2][64] (host / device view)
    double mseq = 0;                            // last sequence number handed to a batch
    double pacc[4] = {0, 0, 0, 0};
    long pn = 0;
    // MAX_ALM_SUB_ITER (lorads_alm.c:20): reset by the ALM phase, carried into reopt
    int max_sub = 5000;
    // objective scaling of reopt (objScale_dualvar): the unscaled C, restored per solve
    double *Cw0 = nullptr, *Craw0 = nullptr;
    bool c_scaled = false;
    // per-context scratch of the standalone reductions (bound to the calling thread)
    unsigned *s_tickets = nullptr;
    double *s_tmpfin = nullptr, *s_rpart = nullptr, *s_fin = nullptr;
    // sharded solve (lrs_shard_*): this process's rows, the transport, the stage hooks
    struct ShardComm *comm = nullptr;
    ShardPlan plan;
    ShardHooks hooks;
    std::vector<int *> d_send_rows;   // per cone: its send rows (local ids, grouped by peer)
    double *d_sendbuf = nullptr;
    long sendbuf_len = 0;
    // phase-1 budget hook (lrs_set_budget_hook): called when almInnerBudget is reached;
    // a larger absolute budget continues the same solve from the saved control block
    lrs_budget_hook bhook = nullptr;
    void *buser = nullptr;
    double last_ctl[C_NCTRL] = {0};
    double last_trip[3] = {0, 0, 0};   // tau, ||G||^2, pinf of the last completed inner trip
    double dinf_tol = 1e-5;            // phase2Tol of the running solve (dual-infeasibility accuracy)
    long dinf_steps = 0, dinf_iters = 0;   // eigen-solve work of the running solve
    bool rank_warned = false;              // the rank clamp's stderr line, once per solve
    int lbfgsL = 2;                        // lbfgsListLength of the running solve
    // lbfgsListLength >= 3: the ring of L pairs (run_inner_generic)
    std::vector<double *> ring_s, ring_y;
    std::vector<double> ring_beta;
    long ring_len = 0;
    double dinf_time = 0.0;
};

// ------------------------------------------------------------------------
// sharded solve: transports.  Every collective is called by all shards in the same
// order (the host control flow is identical on every shard: it only sees summed values).
// ------------------------------------------------------------------------
// One point-to-point or collective operation of a shard, as the transport issues it: the halo
// exchanges' per-(peer, cone) send / receive in the order of halo_ops (the RCCL transport's group
// body), the all-reduces with their lengths.  Recorded when the context's record flag is on
// (lrs_shard_comm_record), so a test can check on the loopback transport that every send pairs
// with the peer's receive of the same length in the same order, and that every shard issues the
// same collectives -- the sequence the RCCL transport drives from the same op list.
enum CommOpKind { COP_GROUP = 0, COP_SEND = 1, COP_RECV = 2, COP_ALLREDUCE_DEV = 3, COP_ALLREDUCE_HOST = 4 };
struct CommOp {
    int kind, peer, cone;
    long count;      // doubles
    long offset;     // send: offset in the packed send buffer; recv: local row of the landing rows x ld
};
struct ShardComm {
    bool recording = false;
    std::vector<CommOp> log;
    void rec(int kind, int peer, int cone, long count, long offset = 0) {
        if (recording) log.push_back(CommOp{kind, peer, cone, count, offset});
    }
    virtual ~ShardComm() {}
    // in-place sum over shards of n device doubles, ordered on stream st
    virtual int allreduce_dev(lrs_ctx *c, double *buf, int n, hipStream_t st) = 0;
    // blocking sum over shards of n host doubles
    virtual int allreduce_host(lrs_ctx *c, double *v, int n) = 0;
    // direction rows: this shard's send rows to each peer, the halo rows from them
    virtual int halo(lrs_ctx *c, double *D, hipStream_t st) = 0;
    // the same for one vector x of cone k's local rows (a Lanczos vector)
    virtual int halo_vec(lrs_ctx *c, int k, double *x, hipStream_t st) = 0;
    // ranks the transport itself counts (RCCL: ncclCommCount; loopback: its world)
    virtual int ranks(int *n) = 0;
};
static bool sharded(const lrs_ctx *c) { return c->comm != nullptr; }
// the LP block's cone (lrs_problem.cpp build_problem: the diagonal cone at rank 1, appended last)
static bool is_lp(const lrs_ctx *c, int k) { return k == c->dp.lp_cone; }
static int n_sdp(const lrs_ctx *c) { return c->dp.K - (c->dp.lp_cone >= 0 ? 1 : 0); }
static int cone_n_global(const lrs_ctx *c, int k) {
    return sharded(c) ? c->plan.cones[k].n_global : c->hp.cones[k].n;
}

// send-buffer offset (doubles) of cone k's segment: cone-major, each cone's rows grouped by peer
static long send_base(const ShardPlan &pl, const DevProblem &dp, int k) {
    long b = 0;
    for (int q = 0; q < k; ++q) b += (long)pl.cones[q].send_rows.size() * dp.cones[q].ld;
    return b;
}

// pack this shard's send rows (every cone, all peers) of the factor buffer X into the send buffer
static int pack_send_rows(lrs_ctx *c, const double *X, hipStream_t st) {
    const int K = c->dp.K;
    const long need = std::max(1L, send_base(c->plan, c->dp, K));
    if (need > c->sendbuf_len) {
        if (c->d_sendbuf) HIPC(hipFree(c->d_sendbuf));
        HIPC(hipMalloc((void **)&c->d_sendbuf, sizeof(double) * need));
        c->sendbuf_len = need;
    }
    for (int k = 0; k < K; ++k) {
        const DevCone &dc = c->dp.cones[k];
        OPC(launch_pack_rows((int)c->plan.cones[k].send_rows.size(), dc.ld, c->d_send_rows[k], X + dc.foff,
                             c->d_sendbuf + send_base(c->plan, c->dp, k), st));
    }
    return 0;
}

// pack cone k's send rows of the vector x (cone-local rows) into c->d_sendvec
static int pack_send_vec(lrs_ctx *c, int k, const double *x, hipStream_t st) {
    const long need = std::max<long>(1, (long)c->plan.cones[k].send_rows.size());
    if (need > c->sendvec_len) {
        if (c->d_sendvec) HIPC(hipFree(c->d_sendvec));
        HIPC(hipMalloc((void **)&c->d_sendvec, sizeof(double) * need));
        c->sendvec_len = need;
    }
    OPC(launch_pack_rows((int)c->plan.cones[k].send_rows.size(), 1, c->d_send_rows[k], x, c->d_sendvec, st));
    return 0;
}

// The halo exchange's operations in issue order, shared by both transports: per peer, per cone
// (cone order on both sides), this shard's send rows to the peer, then the peer's rows into the
// halo.  `vec_cone` >= 0: one vector of that cone's rows (ld 1) instead of every cone's factor rows.
static void halo_ops(const lrs_ctx *c, int vec_cone, std::vector<CommOp> &ops) {
    const ShardPlan &pl = c->plan;
    ops.clear();
    for (int q = 0; q < pl.world; ++q)
        for (int k = 0; k < c->dp.K; ++k) {
            if (vec_cone >= 0 && k != vec_cone) continue;
            const ShardConePlan &cp = pl.cones[k];
            const int ld = vec_cone >= 0 ? 1 : c->dp.cones[k].ld;
            const long base = vec_cone >= 0 ? 0 : send_base(pl, c->dp, k);
            const int ns = cp.send_ptr[q + 1] - cp.send_ptr[q];
            if (ns > 0) ops.push_back(CommOp{COP_SEND, q, k, (long)ns * ld, base + (long)cp.send_ptr[q] * ld});
            if (cp.recv_cnt[q] > 0)
                ops.push_back(CommOp{COP_RECV, q, k, (long)cp.recv_cnt[q] * ld, (long)cp.recv_start[q] * ld});
        }
}

#define LRS_STR_(x) #x
#define LRS_STR(x) LRS_STR_(x)
#define NCCLC(x)                                                                            \
    do {                                                                                    \
        ncclResult_t r_ = (x);                                                              \
        if (r_ != ncclSuccess) {                                                            \
            set_err("%s:%d %s: %s", __FILE__, __LINE__, #x, ncclGetErrorString(r_));        \
            return -1;                                                                      \
        }                                                                                   \
    } while (0)

// inside ncclGroupStart / ncclGroupEnd: an error closes the group before returning, so the
// communicator is left usable (no dangling group on this thread)
#define NCCLG(x)                                                                            \
    do {                                                                                    \
        ncclResult_t r_ = (x);                                                              \
        if (r_ != ncclSuccess) {                                                            \
            set_err("%s:%d %s: %s", __FILE__, __LINE__, #x, ncclGetErrorString(r_));        \
            (void)ncclGroupEnd();                                                           \
            return -1;                                                                      \
        }                                                                                   \
    } while (0)

// RCCL over xGMI: one process per GPU
struct RcclComm : ShardComm {
    ncclComm_t comm = nullptr;
    double *dscr = nullptr;   // host all-reduce staging
    int dscr_len = 0;
    ~RcclComm() override {
        if (comm) (void)ncclCommDestroy(comm);
        if (dscr) (void)hipFree(dscr);
    }
    int allreduce_dev(lrs_ctx *, double *buf, int n, hipStream_t st) override {
        rec(COP_ALLREDUCE_DEV, -1, -1, n);
        NCCLC(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, comm, st));
        return 0;
    }
    int allreduce_host(lrs_ctx *c, double *v, int n) override {
        if (n > dscr_len) {
            if (dscr) HIPC(hipFree(dscr));
            HIPC(hipMalloc((void **)&dscr, sizeof(double) * n));
            dscr_len = n;
        }
        HIPC(hipMemcpyAsync(dscr, v, sizeof(double) * n, hipMemcpyHostToDevice, c->st));
        rec(COP_ALLREDUCE_HOST, -1, -1, n);
        NCCLC(ncclAllReduce(dscr, dscr, n, ncclDouble, ncclSum, comm, c->st));
        HIPC(hipMemcpyAsync(v, dscr, sizeof(double) * n, hipMemcpyDeviceToHost, c->st));
        HIPC(hipStreamSynchronize(c->st));
        return 0;
    }
    // one group per exchange, its body the shared op list (halo_ops): each send from the packed
    // send buffer, each receive in place into the peer's halo rows (contiguous locally)
    int group(lrs_ctx *c, int vec_cone, const double *sendbuf, double *base, hipStream_t st) {
        halo_ops(c, vec_cone, ops);
        rec(COP_GROUP, -1, vec_cone, (long)ops.size());
        NCCLC(ncclGroupStart());
        for (const CommOp &o : ops) {
            rec(o.kind, o.peer, o.cone, o.count, o.offset);
            if (o.kind == COP_SEND)
                NCCLG(ncclSend(sendbuf + o.offset, (size_t)o.count, ncclDouble, o.peer, comm, st));
            else
                NCCLG(ncclRecv(base + (vec_cone >= 0 ? 0 : c->dp.cones[o.cone].foff) + o.offset, (size_t)o.count,
                               ncclDouble, o.peer, comm, st));
        }
        NCCLC(ncclGroupEnd());
        return 0;
    }
    std::vector<CommOp> ops;
    int halo(lrs_ctx *c, double *D, hipStream_t st) override {
        if (pack_send_rows(c, D, st)) return -1;
        return group(c, -1, c->d_sendbuf, D, st);
    }
    int halo_vec(lrs_ctx *c, int k, double *x, hipStream_t st) override {
        if (pack_send_vec(c, k, x, st)) return -1;
        return group(c, k, c->d_sendvec, x, st);
    }
    int ranks(int *n) override {
        NCCLC(ncclCommCount(comm, n));
        return 0;
    }
};

// One-process loopback transport for tests: the shards are contexts on one GPU driven by
// one host thread each; collectives meet at host barriers and order the shards' streams
// with events (every shard waits for all shards' work before reading their buffers, and
// again before anyone reuses them).
struct lrs_loopback {
    int world = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long gen = 0;
    std::vector<hipEvent_t> ev_pre, ev_post;
    std::vector<const double *> bufs;
    std::vector<const double *> sendbufs;
    std::vector<const ShardPlan *> plans;
    std::vector<std::vector<double>> hv;
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const long g = gen;
        if (++arrived == world) { arrived = 0; gen++; cv.notify_all(); }
        else cv.wait(lk, [&] { return gen != g; });
    }
};
struct LoopComm : ShardComm {
    lrs_loopback *g = nullptr;
    int rank = 0;
    double *dsum = nullptr;
    int dsum_len = 0;
    ~LoopComm() override { if (dsum) (void)hipFree(dsum); }
    int ranks(int *n) override { *n = g->world; return 0; }
    int pre(hipStream_t st) {
        HIPC(hipEventRecord(g->ev_pre[rank], st));
        g->barrier();
        for (int q = 0; q < g->world; ++q) HIPC(hipStreamWaitEvent(st, g->ev_pre[q], 0));
        return 0;
    }
    int post(hipStream_t st) {
        HIPC(hipEventRecord(g->ev_post[rank], st));
        g->barrier();
        for (int q = 0; q < g->world; ++q) HIPC(hipStreamWaitEvent(st, g->ev_post[q], 0));
        return 0;
    }
    int allreduce_dev(lrs_ctx *, double *buf, int n, hipStream_t st) override {
        if (n > dsum_len) {
            if (dsum) HIPC(hipFree(dsum));
            HIPC(hipMalloc((void **)&dsum, sizeof(double) * n));
            dsum_len = n;
        }
        g->bufs[rank] = buf;
        rec(COP_ALLREDUCE_DEV, -1, -1, n);
        if (pre(st)) return -1;
        OPC(launch_sum_shards(n, g->world, g->bufs.data(), dsum, st));
        if (post(st)) return -1;
        HIPC(hipMemcpyAsync(buf, dsum, sizeof(double) * n, hipMemcpyDeviceToDevice, st));
        return 0;
    }
    int allreduce_host(lrs_ctx *, double *v, int n) override {
        rec(COP_ALLREDUCE_HOST, -1, -1, n);
        g->hv[rank].assign(v, v + n);
        g->barrier();
        for (int i = 0; i < n; ++i) {
            double t = 0.0;
            for (int q = 0; q < g->world; ++q) t += g->hv[q][i];
            v[i] = t;
        }
        g->barrier();
        return 0;
    }
    std::vector<CommOp> ops;
    void record_ops(lrs_ctx *c, int vec_cone) {   // what the RCCL transport's group would issue
        if (!recording) return;
        halo_ops(c, vec_cone, ops);
        rec(COP_GROUP, -1, vec_cone, (long)ops.size());
        for (const CommOp &o : ops) rec(o.kind, o.peer, o.cone, o.count, o.offset);
    }
    int halo(lrs_ctx *c, double *D, hipStream_t st) override {
        if (pack_send_rows(c, D, st)) return -1;
        record_ops(c, -1);
        g->sendbufs[rank] = c->d_sendbuf;
        if (pre(st)) return -1;
        for (int q = 0; q < g->world; ++q)
            for (int k = 0; k < c->dp.K; ++k) {
                const ShardConePlan &cp = c->plan.cones[k];
                const int cnt = cp.recv_cnt[q], ld = c->dp.cones[k].ld;
                if (q == rank || cnt == 0) continue;
                const ShardPlan &pq = *g->plans[q];
                const ShardConePlan &qc = pq.cones[k];
                if (qc.send_ptr[rank + 1] - qc.send_ptr[rank] != cnt) { set_err("loopback halo: plan mismatch"); return -1; }
                // the peer's segment offset (same ranks, so the same layouts on every shard)
                HIPC(hipMemcpyAsync(D + c->dp.cones[k].foff + (long)cp.recv_start[q] * ld,
                                    g->sendbufs[q] + send_base(pq, c->dp, k) + (long)qc.send_ptr[rank] * ld,
                                    sizeof(double) * cnt * ld, hipMemcpyDeviceToDevice, st));
            }
        return post(st);
    }
    int halo_vec(lrs_ctx *c, int k, double *x, hipStream_t st) override {
        if (pack_send_vec(c, k, x, st)) return -1;
        record_ops(c, k);
        g->sendbufs[rank] = c->d_sendvec;
        if (pre(st)) return -1;
        const ShardConePlan &cp = c->plan.cones[k];
        for (int q = 0; q < g->world; ++q) {
            const int cnt = cp.recv_cnt[q];
            if (q == rank || cnt == 0) continue;
            const ShardConePlan &qc = g->plans[q]->cones[k];
            if (qc.send_ptr[rank + 1] - qc.send_ptr[rank] != cnt) { set_err("loopback halo: plan mismatch"); return -1; }
            HIPC(hipMemcpyAsync(x + cp.recv_start[q], g->sendbufs[q] + qc.send_ptr[rank], sizeof(double) * cnt,
                                hipMemcpyDeviceToDevice, st));
        }
        return post(st);
    }
};

static int hook_halo(void *self, double *D, hipStream_t st) {
    lrs_ctx *c = static_cast<lrs_ctx *>(self);
    return c->comm->halo(c, D, st);
}
static int hook_allreduce(void *self, double *buf, int n, hipStream_t st) {
    lrs_ctx *c = static_cast<lrs_ctx *>(self);
    return c->comm->allreduce_dev(c, buf, n, st);
}
// this context's device, stream-free scratch bound to the calling thread
static void bind(lrs_ctx *c) {
    (void)hipSetDevice(c->device);
    bind_scratch(c->s_tickets, c->s_tmpfin, c->s_rpart, c->s_fin);
}

static void free_lz(lrs_ctx::LzWork &w) {
    double *ptrs[] = {w.V, w.Vt, w.y[0], w.y[1], w.part, w.H, w.Y};
    for (double *p : ptrs)
        if (p) (void)hipFree(p);
    w = lrs_ctx::LzWork();
}
static void drop_lanczos(lrs_ctx *c) {
    if (c->lz.empty()) return;
    (void)hipStreamSynchronize(c->st);   // nothing is still in flight on the buffers
    for (auto &w : c->lz) free_lz(w);
    c->lz.clear();
}
static void drop_graphs(lrs_ctx *c) {
    for (auto &kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
    c->graphs.clear();
    drop_lanczos(c);
}

static void logf_(lrs_ctx *c, const lrs_params *p, const char *fmt, ...) {
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (p->verbose) fputs(buf, stdout);
    if (c->logfp) { fputs(buf, c->logfp); fflush(c->logfp); }
}

// ------------------------------------------------------------------------
// workspace
// ------------------------------------------------------------------------
static void free_work(lrs_ctx *c) {
    drop_graphs(c);
    if (!c->walloc) return;
    DevWork &W = c->W;
    double *ptrs[] = {W.R, W.D, W.G[0], W.G[1], W.ls[0], W.ly[0], W.ls[1], W.ly[1], W.U, W.V, W.X, W.cg_r,
                      W.cg_p, W.cg_Q, W.cg_b, W.M2, W.uvt0, W.uvt1, W.uvt2, W.S, W.lam, W.cvs, W.q1, W.q2,
                      W.M1, W.wtmp, W.cvc, W.part, W.partB, W.partC, W.ctrl, W.lsres, W.par, W.gram, W.rec, W.R2,
                      W.cgc, W.tot, W.gl, W.CR, W.CD, W.GP, W.CGK, W.uvp, W.lpw};
    for (double *p : ptrs)
        if (p) (void)hipFree(p);
    for (double *q : c->ring_s) if (q) (void)hipFree(q);
    for (double *q : c->ring_y) if (q) (void)hipFree(q);
    c->ring_s.clear(); c->ring_y.clear(); c->ring_beta.clear(); c->ring_len = 0;
    c->W = DevWork();
    c->dp.gp = nullptr;
    c->dp.cgk = nullptr;
    c->walloc = false;
}

static int zero_work(lrs_ctx *c) {
    DevWork &W = c->W;
    const DevProblem &P = c->dp;
    const long NR = std::max(2L, P.NRpad);
    const int m = std::max(1, P.m), Pt = std::max(1, P.Ptot);
    struct Z { double *p; long n; } zs[] = {
        {W.R, NR}, {W.D, NR}, {W.G[0], NR}, {W.G[1], NR}, {W.ls[0], NR}, {W.ly[0], NR}, {W.ls[1], NR}, {W.ly[1], NR},
        {W.U, NR}, {W.V, NR}, {W.X, NR}, {W.cg_r, NR}, {W.cg_p, NR}, {W.cg_Q, NR}, {W.cg_b, NR}, {W.M2, NR},
        {W.R2, NR}, {W.uvt0, Pt}, {W.uvt1, Pt}, {W.uvt2, Pt}, {W.S, Pt}, {W.lam, m}, {W.cvs, m}, {W.q1, m},
        {W.q2, m}, {W.M1, m}, {W.wtmp, m}, {W.cvc, (long)m * std::max(1, P.K)}, {W.ctrl, 2 * C_NCTRL},
        {W.lsres, 2 * LS_N}, {W.rec, 4L * m}, {W.tot, 32}, {W.CR, W.CR ? NR : 0}, {W.CD, W.CD ? NR : 0}};
    for (auto &z : zs)
        if (z.p) HIPC(hipMemsetAsync(z.p, 0, sizeof(double) * z.n, c->st));
    c->head = 0; c->gcur = 0;
    c->beta[0] = c->beta[1] = c->yy[0] = c->yy[1] = 0;
    for (size_t q = 0; q < c->ring_s.size(); ++q) {   // lbfgsListLength >= 3
        HIPC(hipMemsetAsync(c->ring_s[q], 0, sizeof(double) * std::max(2L, c->ring_len), c->st));
        HIPC(hipMemsetAsync(c->ring_y[q], 0, sizeof(double) * std::max(2L, c->ring_len), c->st));
        c->ring_beta[q] = 0.0;
    }
    return 0;
}

static int alloc_work(lrs_ctx *c, const std::vector<int> &ranks) {
    // same ranks as the live workspace: keep the buffers (and the captured graphs), zero them
    if (c->walloc && ranks == c->rank) return zero_work(c);
    free_work(c);
    DevProblem &P = c->dp;
    c->rank = ranks;
    c->lay.assign(P.K, Layout());
    long off = 0;
    int rmax = 1;
    for (int k = 0; k < P.K; ++k) {
        Layout L = choose_layout(ranks[k]);
        if (ranks[k] > L.ld) { set_err("rank %d unsupported (max 512)", ranks[k]); return -1; }
        c->lay[k] = L;
        DevCone &dc = P.cones[k];
        dc.r = ranks[k]; dc.ld = L.ld; dc.G = L.G; dc.E = L.E; dc.foff = off;
        off += (long)dc.n * L.ld;
        rmax = std::max(rmax, ranks[k]);
    }
    P.NRpad = off;
    DevWork &W = c->W;
    const long NR = std::max(2L, off);
    const int m = std::max(1, P.m);
    const int Pt = std::max(1, P.Ptot);
    auto A = [&](double **p, long n) -> int {
        HIPC(hipMalloc((void **)p, sizeof(double) * n));
        HIPC(hipMemsetAsync(*p, 0, sizeof(double) * n, c->st));
        return 0;
    };
    if (A(&W.R, NR) || A(&W.D, NR) || A(&W.G[0], NR) || A(&W.G[1], NR) || A(&W.ls[0], NR) || A(&W.ly[0], NR) ||
        A(&W.ls[1], NR) || A(&W.ly[1], NR) || A(&W.U, NR) || A(&W.V, NR) || A(&W.X, NR) || A(&W.cg_r, NR) ||
        A(&W.cg_p, NR) || A(&W.cg_Q, NR) || A(&W.cg_b, NR) || A(&W.M2, NR) || A(&W.uvt0, Pt) || A(&W.uvt1, Pt) ||
        A(&W.uvt2, Pt) || A(&W.S, Pt) || A(&W.lam, m) || A(&W.cvs, m) || A(&W.q1, m) || A(&W.q2, m) ||
        A(&W.M1, m) || A(&W.wtmp, m) || A(&W.cvc, (long)m * std::max(1, P.K)) ||
        A(&W.part, (long)kMaxPartialVals * kMaxPartialBlocks) || A(&W.partB, (long)kMaxPartialVals * kMaxPartialBlocks) ||
        A(&W.partC, (long)kMaxPartialVals * kMaxPartialBlocks) || A(&W.ctrl, 2 * C_NCTRL) ||
        A(&W.lsres, 2 * LS_N) || A(&W.par, P_NPAR) || A(&W.gram, (long)gram_buf_len(rmax)) || A(&W.rec, 4L * m) || A(&W.R2, NR) || A(&W.cgc, 8) ||
        A(&W.tot, 32))
        return -1;
    {   // slice gradients of the latency kernels' dense rows
        long gl = 1, sum = 0;
        for (const auto &dc : P.cones) sum += dc.gl_need;   // per-cone launches: disjoint ranges
        gl = std::max(gl, sum);
        if (P.has_merged) gl = std::max(gl, P.merged.gl_need);
        if (A(&W.gl, gl)) return -1;
        W.gl_len = gl;
    }
    if (P.ndense && (A(&W.CR, NR) || A(&W.CD, NR))) return -1;
    if (P.lp_cone >= 0 && A(&W.lpw, std::max(2L, lp_sweep_scratch(P)))) return -1;   // k_lp_admm, unstaged
    {   // k_cgemm2's split-K slabs for the large dense cones
        bool big = false;
        for (const DevCone &dc : P.cones) big = big || (dc.dense_c == 1 && dc.n >= 2048);
        if (big && A(&W.CGK, (long)kCgSplitSlabs * NR)) return -1;
        P.cgk = W.CGK;
    }
    {   // column-tiled long-row kernels: the partial S R_new factors
        bool tiles = false;
        const char *ev = getenv("LRS_TILES");
        for (const auto &dc : P.cones) tiles = tiles || (dc.colseg != nullptr && ev && ev[0] == '1');
        bool btiles = false;   // long-row B over 2-D tiles (DevCone::sb_blocks): k_wide_bf's partial rows
        for (const auto &dc : P.cones) btiles = btiles || dc.sb_blocks > 0;
        if ((tiles || btiles) && A(&W.GP, (long)kNX * NR)) return -1;
        bool stiles = false;   // the tiled stage A's slot-value records (DevWork::uvp)
        for (const auto &dc : P.cones) stiles = stiles || dc.sa_items > 0;
        if (stiles && A(&W.uvp, 2L * std::max(1, P.Ptot))) return -1;
        P.gp = W.GP;
        P.tiles = tiles;
    }
    HIPC(hipStreamSynchronize(c->st));
    c->walloc = true;
    c->head = 0; c->gcur = 0;
    c->beta[0] = c->beta[1] = c->yy[0] = c->yy[1] = 0;
    return 0;
}

// column-major (reference) <-> row-major ld-padded device layout
// Synchronous host -> device copy ordered after the solver stream's pending work (the stream
// is non-blocking, so a plain hipMemcpy on the null stream could overtake kernels still
// reading the destination).
static hipError_t h2d_sync(lrs_ctx *c, void *dst, const void *src, size_t bytes) {
    hipError_t e = hipStreamSynchronize(c->st);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->st);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(c->st);
}

static int factor_put(lrs_ctx *c, double *dst, const double *colmajor) {
    std::vector<double> h(c->dp.NRpad, 0.0);
    long src = 0;
    for (int k = 0; k < c->dp.K; ++k) {
        const DevCone &d = c->dp.cones[k];
        for (int q = 0; q < d.r; ++q)
            for (int i = 0; i < d.n; ++i) h[d.foff + (long)i * d.ld + q] = colmajor[src + i + (long)q * d.n];
        src += (long)d.n * d.r;
    }
    HIPC(h2d_sync(c, dst, h.data(), sizeof(double) * c->dp.NRpad));
    return 0;
}
static int factor_fetch(lrs_ctx *c, const double *srcd, double *colmajor) {
    std::vector<double> h(c->dp.NRpad);
    HIPC(hipStreamSynchronize(c->st));
    HIPC(hipMemcpy(h.data(), srcd, sizeof(double) * c->dp.NRpad, hipMemcpyDeviceToHost));
    long dst = 0;
    for (int k = 0; k < c->dp.K; ++k) {
        const DevCone &d = c->dp.cones[k];
        for (int q = 0; q < d.r; ++q)
            for (int i = 0; i < d.n; ++i) colmajor[dst + i + (long)q * d.n] = h[d.foff + (long)i * d.ld + q];
        dst += (long)d.n * d.r;
    }
    return 0;
}

static double *factor_ptr(lrs_ctx *c, int which) {
    DevWork &W = c->W;
    switch (which) {
    case LRS_R: return W.R;
    case LRS_D: return W.D;
    case LRS_G: return W.G[c->gcur];
    case LRS_U: return W.U;
    case LRS_V: return W.V;
    case LRS_S0: return W.ls[0];
    case LRS_Y0: return W.ly[0];
    case LRS_S1: return W.ls[1];
    case LRS_Y1: return W.ly[1];
    }
    return nullptr;
}
static double *vec_ptr(lrs_ctx *c, int which) {
    switch (which) {
    case LRS_LAMBDA: return c->W.lam;
    case LRS_CVS: return c->W.cvs;
    case LRS_Q1: return c->W.q1;
    case LRS_Q2: return c->W.q2;
    case LRS_B: return c->dp.b;
    }
    return nullptr;
}

static int read_tmpfin2(lrs_ctx *c, int idx1, int n1, int idx2, int n2, double *out);
static int read_tmpfin(lrs_ctx *c, int idx, int n, double *out) {
    if (n > kHpReadN) return read_tmpfin2(c, idx, n, 0, 0, out);
    double *h = c->hpin + kHpRead;
    HIPC(hipMemcpyAsync(h, device_tmpfin() + idx, sizeof(double) * n, hipMemcpyDeviceToHost, c->st));
    HIPC(hipStreamSynchronize(c->st));
    for (int i = 0; i < n; ++i) out[i] = h[i];
    // sharded: every standalone reduction is a sum over the shard's rows / constraints
    if (sharded(c)) return c->comm->allreduce_host(c, out, n);
    return 0;
}

// several tmpfin ranges behind one stream sync (staged at hpin + kHpRead2, clear of the
// ALM mirror slots and the CG poll): out = [idx1, idx1 + n1) ++ [idx2, idx2 + n2)
static int read_tmpfin2(lrs_ctx *c, int idx1, int n1, int idx2, int n2, double *out) {
    if (n1 + n2 > kHpRead2N) { set_err("read_tmpfin2: %d values past the %d staged", n1 + n2, kHpRead2N); return -1; }
    double *h = c->hpin + kHpRead2;
    HIPC(hipMemcpyAsync(h, device_tmpfin() + idx1, sizeof(double) * n1, hipMemcpyDeviceToHost, c->st));
    if (n2 > 0)
        HIPC(hipMemcpyAsync(h + n1, device_tmpfin() + idx2, sizeof(double) * n2, hipMemcpyDeviceToHost, c->st));
    HIPC(hipStreamSynchronize(c->st));
    for (int i = 0; i < n1 + n2; ++i) out[i] = h[i];
    if (sharded(c)) return c->comm->allreduce_host(c, out, n1 + n2);
    return 0;
}

// ------------------------------------------------------------------------
// host-driven operators
// ------------------------------------------------------------------------
static int op_dot(lrs_ctx *c, long n, const double *x, const double *y, double *out);
// A(X X^T) for every cone -> cvc[k], cvs = sum_k, returns pinf (primalInfeasibility)
// and the objective <C, X X^T> (unscaled), with X given per-cone rows in factor buffer.
// blam != nullptr: also b^T lambda (tmpfin TF_DOT), read behind the same sync
static int op_constr_xx(lrs_ctx *c, const double *X, const double *Y, double *pinf, double *obj,
                        double *blam = nullptr) {
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    int fin;
    const char *ct = getenv("LRS_CONSTR_TILES");
    if (P.K == 1 && !sharded(c) && P.cones[0].auv_items > 0 && P.cones[0].cobj_slot && !(ct && ct[0] == '0')) {
        // a cone with constraint-entry tiles (C5): A(.) and the residual straight from the tiles
        // (k_auv_tile + k_auv_tsum), <C, .> over C's own entries -- not a pattern-wide SDDMM
        // then a gather of 10^6 constraints' slot values (C5: 203 + 95 + 282 -> ~240 us)
        OPC(launch_auv_con(P, 0, Y ? 0 : 1, X, Y, 1.0, 0, W.cvs, P.b, W.part, c->st));
        OPC(launch_cobj(P, 0, Y ? 0 : 1, X, Y, W.partB, c->st));
        HIPC(hipMemcpyAsync(W.cvc, W.cvs, sizeof(double) * P.m, hipMemcpyDeviceToDevice, c->st));
        fin = TF_GATHER;
        goto READ;
    }
    // every cone's <C, X Y^T> (tmpfin TF_SD + 2k) and the residual norm in one read
    for (int k = 0; k < P.K; ++k)
        OPC(launch_sddmm(P, k, Y ? 0 : 1, X, Y, W.uvt2, nullptr, W.part, 0, nullptr, c->st));
    if (P.K == 1 && P.nsh > 0) {
        // sharded, shared constraints: the holders' owned-entry sums summed over the shards,
        // then the residual with each constraint counted once (its primary holder)
        OPC(launch_gather(P, W.uvt2, 1.0, W.cvs, nullptr, nullptr, c->st, nullptr));
        OPC(sync_shared(P, W.cvs, c->st));
        HIPC(hipMemcpyAsync(W.cvc, W.cvs, sizeof(double) * P.m, hipMemcpyDeviceToDevice, c->st));
        OPC(launch_resid(P.m, P.b, W.cvs, c->st, P.cmask));
        fin = TF_RESID;
    } else if (P.K == 1) {
        OPC(launch_gather(P, W.uvt2, 1.0, W.cvs, P.b, W.part, c->st, nullptr));
        HIPC(hipMemcpyAsync(W.cvc, W.cvs, sizeof(double) * P.m, hipMemcpyDeviceToDevice, c->st));
        fin = TF_GATHER;
    } else {
        OPC(launch_fill(P.m, 0.0, W.cvs, c->st));
        for (int k = 0; k < P.K; ++k) {
            OPC(launch_gather_cone(P, k, W.uvt2, W.cvc + (long)k * P.m, c->st));
            OPC(sync_shared(P, W.cvc + (long)k * P.m, c->st));   // sharded: the holders' sums
            OPC(launch_axpby(P.m, 1.0, W.cvc + (long)k * P.m, 1.0, W.cvs, c->st));
        }
        OPC(launch_resid(P.m, P.b, W.cvs, c->st, P.cmask));   // sharded: each constraint once
        fin = TF_RESID;
    }
READ:
    if (blam) OPC(launch_dot(P.m, P.bprim ? P.bprim : P.b, W.lam, W.part, c->st, nullptr));
    // dense objective: <C, sym X Y^T> = <X, C Y> over the rows C X covers (sharded: the owned
    // rows, summed over the shards), into TF_DOTC + k, read behind the same sync
    for (int k = 0; k < P.K && obj; ++k) {
        const DevCone &dc = P.cones[k];
        if (!dc.dense_c) continue;
        OPC(launch_dense_cx(P, k, Y ? Y : X, W.CD, 0.0, c->st));
        const long ro = dc.foff + (long)dc.row0 * dc.ld;
        OPC(launch_dot((long)dc.nown * dc.ld, X + ro, W.CD + ro, W.part, c->st, nullptr, TF_DOTC + k));
    }
    double t[3 * kMaxCones + 3];
    if (read_tmpfin2(c, TF_SD, 2 * P.K, TF_GATHER, 3 + P.K, t)) return -1;   // GATHER, RESID, DOT, DOTC
    double o = 0.0;
    for (int k = 0; k < P.K; ++k) o += t[2 * k];
    for (int k = 0; k < P.K && obj; ++k)
        if (P.cones[k].dense_c) o += t[2 * P.K + (TF_DOTC - TF_GATHER) + k];
    if (pinf) *pinf = std::sqrt(t[2 * P.K + (fin - TF_GATHER)]) / (1 + c->hp.bNrm1);
    if (blam) *blam = t[2 * P.K + (TF_DOT - TF_GATHER)];
    if (obj) *obj = o;
    return 0;
}

// ALMCalGrad (lorads_alm.c:74-87): G[gcur] = 2 (C + A^*(M1)) R, returns ||G||^2
static int op_grad(lrs_ctx *c, double rho, double *lag) {
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    OPC(launch_alm_m1(P, rho, W.lam, W.cvs, W.M1, c->st));
    OPC(launch_wsum(P, W.M1, 1, W.S, c->st));
    for (int k = 0; k < P.K; ++k)
        OPC(launch_spmm(P, k, W.S, W.R, 2.0, nullptr, 0.0, W.G[c->gcur], W.part, 0, nullptr, c->st));
    double v[TF_N - TF_SPMM];
    if (read_tmpfin2(c, TF_SPMM, P.K, 0, 0, v)) return -1;
    // dense objective: C R (the inner loop carries it), G += 2 C R, ||G||^2 anew
    for (int k = 0; k < P.K; ++k) {
        const DevCone &dc = P.cones[k];
        if (!dc.dense_c) continue;
        const long ro = dc.foff + (long)dc.row0 * dc.ld;   // the rows C R covers (sharded: owned)
        double *Gk = W.G[c->gcur] + ro;
        OPC(launch_dense_cx(P, k, W.R, W.CR, 0.0, c->st));
        OPC(launch_axpby((long)dc.nown * dc.ld, 2.0, W.CR + ro, 1.0, Gk, c->st));
        if (op_dot(c, (long)dc.nown * dc.ld, Gk, Gk, &v[k])) return -1;
    }
    double tot = 0.0;
    for (int k = 0; k < P.K; ++k) {
        double nrm = std::sqrt(v[k]);
        tot += nrm * nrm;
    }
    *lag = tot;
    return 0;
}

static int op_dot(lrs_ctx *c, long n, const double *x, const double *y, double *out) {
    OPC(launch_dot(n, x, y, c->W.part, c->st, nullptr));
    return read_tmpfin(c, TF_DOT, 1, out);
}

// ------------------------------------------------------------------------
// Dual infeasibility (calculate_dual_infeasibility_solver, data/lorads_solver.c:1396-1426):
// S = C + A^*(-lambda) on the pattern, lambda_min(S) per cone, and
// err = sum_k |min(lambda_min,k, 0)| / scaleObjHis / (||C||_1 + 1).  The reference's
// eigensolver is ARPACK dsaupd "SA" (ncv 40, tol 1e-2, data/lorads_sdp_conic.c:1636-1699);
// here a Lanczos process with full reorthogonalisation (device kernels launch_symv /
// launch_reorth), run to a 1e-10 relative Ritz residual or its step cap.
// ------------------------------------------------------------------------
// Symmetric eigen-decomposition of the m x m matrix A (row-major) by cyclic Jacobi rotations:
// eigenvalues ascending in w, unit eigenvectors in the columns of Z (row-major).  m <= 64.
static void jacobi_eig(int m, std::vector<double> A, std::vector<double> &w, std::vector<double> &Z) {
    std::vector<double> V((size_t)m * m, 0.0);
    for (int i = 0; i < m; ++i) V[(size_t)i * m + i] = 1.0;
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0.0, dia = 0.0;
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < m; ++j) (i == j ? dia : off) += A[(size_t)i * m + j] * A[(size_t)i * m + j];
        if (off <= 1e-32 * (dia + off) || off == 0.0) break;
        for (int p = 0; p < m; ++p)
            for (int q = p + 1; q < m; ++q) {
                const double apq = A[(size_t)p * m + q];
                if (apq == 0.0) continue;
                const double th = (A[(size_t)q * m + q] - A[(size_t)p * m + p]) / (2.0 * apq);
                const double t = std::fabs(th) > 1e150 ? 0.5 / th
                                                       : (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
                const double cs = 1.0 / std::sqrt(t * t + 1.0), sn = t * cs;
                for (int r = 0; r < m; ++r) {   // columns p, q
                    const double ap = A[(size_t)r * m + p], aq = A[(size_t)r * m + q];
                    A[(size_t)r * m + p] = cs * ap - sn * aq;
                    A[(size_t)r * m + q] = sn * ap + cs * aq;
                }
                for (int r = 0; r < m; ++r) {   // rows p, q
                    const double ap = A[(size_t)p * m + r], aq = A[(size_t)q * m + r];
                    A[(size_t)p * m + r] = cs * ap - sn * aq;
                    A[(size_t)q * m + r] = sn * ap + cs * aq;
                }
                A[(size_t)p * m + q] = A[(size_t)q * m + p] = 0.0;
                for (int r = 0; r < m; ++r) {
                    const double vp = V[(size_t)r * m + p], vq = V[(size_t)r * m + q];
                    V[(size_t)r * m + p] = cs * vp - sn * vq;
                    V[(size_t)r * m + q] = sn * vp + cs * vq;
                }
            }
    }
    std::vector<int> ord(m);
    for (int i = 0; i < m; ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(),
                     [&](int a, int b) { return A[(size_t)a * m + a] < A[(size_t)b * m + b]; });
    w.assign(m, 0.0);
    Z.assign((size_t)m * m, 0.0);
    for (int e = 0; e < m; ++e) {
        w[e] = A[(size_t)ord[e] * m + ord[e]];
        for (int r = 0; r < m; ++r) Z[(size_t)r * m + e] = V[(size_t)r * m + ord[e]];
    }
}

static int op_dot(lrs_ctx *c, long n, const double *x, const double *y, double *out);

// lambda_min of S on cone k (S: device slot values) with ARPACK dsaupd's semantics, the call
// of dual_infeasible (data/lorads_sdp_conic.c:1636-1699): which = "SA", nev = 1, ncv = 40
// (2 when n < 40), exact shifts, tol = 1e-2, at most 600 update iterations.  Restated as a
// thick-restart Lanczos (Wu & Simon: with exact shifts, implicitly restarted Lanczos keeps the
// span of the wanted Ritz vectors, which a thick restart keeps explicitly): a cycle extends the
// basis to ncv vectors (device: S v_j, two Gram-Schmidt passes against the whole basis, the
// coefficients = the entries of V^T S V), the host takes the Ritz pairs of that ncv x ncv
// matrix (Jacobi) and the Ritz estimates beta |e_m^T y|, and either stops or restarts from the
// kk smallest Ritz vectors plus the residual direction.  kk is dsaup2's adjusted nev (nev = 1,
// no converged value yet: kplusp / 2 = 20, or 2 / 1 for tiny kplusp).  Stop: dsconv's test
// bound <= tol max(eps^(2/3), |theta|) on the smallest Ritz value, or an absolute bound below
// 1e-3 of the amount of lambda_min that moves the l_1 dual infeasibility by phase2Tol (the value
// is then pinned far past every threshold it feeds), or an invariant subspace (breakdown).
// Sharded: the vectors are the owned rows (the matvec reads the halo rows, exchanged per step),
// and the coefficient sums and norms are all-reduced in the stream, so every shard sees the
// same matrix and takes the same decisions.
static int trl_min(lrs_ctx *c, int k, const double *S, double *lam_min, int *steps_out, int *iters_out,
                   bool *converged) {
    const DevCone &dc = c->dp.cones[k];
    const bool sh = sharded(c);
    const int nl = dc.n, r0 = dc.row0, nown = dc.nown;
    const int N = cone_n_global(c, k);
    int ncv = 40;
    if (ncv > N) ncv = 2;
    if (const char *e = getenv("LRS_TRL_NCV")) ncv = std::max(2, std::min(atoi(e), kTrlMaxV));   // tests
    ncv = std::max(1, std::min(ncv, N));
    int maxiter = 600;
    if (const char *e = getenv("LRS_TRL_MAXITER")) maxiter = std::max(0, atoi(e));   // tests
    const int kk = ncv >= 6 ? ncv / 2 : (ncv > 2 ? 2 : 1);
    const double tol = 1e-2, eps23 = std::pow(std::numeric_limits<double>::epsilon(), 2.0 / 3.0);
    const double abs_tol = 1e-3 * c->dinf_tol * (1 + c->hp.cNrm1) * c->scaleObjHis;
    const long ldv = ((long)nl + 7) & ~7L;
    constexpr int ldh = kTrlMaxV + 1;
    if ((int)c->lz.size() < c->dp.K) c->lz.resize(c->dp.K);
    lrs_ctx::LzWork &Z = c->lz[k];
    if (Z.n != nl) {   // this cone's buffers only
        HIPC(hipStreamSynchronize(c->st));
        free_lz(Z);
        HIPC(hipMalloc((void **)&Z.V, sizeof(double) * ldv * (kTrlMaxV + 1)));
        HIPC(hipMalloc((void **)&Z.Vt, sizeof(double) * ldv * kTrlMaxV));
        HIPC(hipMalloc((void **)&Z.y[0], sizeof(double) * ldv));
        HIPC(hipMalloc((void **)&Z.y[1], sizeof(double) * ldv));
        HIPC(hipMalloc((void **)&Z.part, sizeof(double) * (64L * kTrlMaxV + kMaxPartialBlocks)));
        HIPC(hipMalloc((void **)&Z.H, sizeof(double) * ((long)ldh * kTrlMaxV + 2L * kTrlMaxV + 8)));
        HIPC(hipMalloc((void **)&Z.Y, sizeof(double) * kTrlMaxV * kTrlMaxV));
        HIPC(hipMemsetAsync(Z.y[0], 0, sizeof(double) * ldv, c->st));
        HIPC(hipMemsetAsync(Z.y[1], 0, sizeof(double) * ldv, c->st));
        Z.n = nl;
    }
    double *V = Z.V, *Hd = Z.H, *bw2 = Z.H + (long)ldh * kTrlMaxV, *tot = bw2 + kTrlMaxV;
    double *npart = Z.part + 64L * kTrlMaxV;
    HIPC(hipMemsetAsync(V, 0, sizeof(double) * ldv * (kTrlMaxV + 1), c->st));
    {   // start vector (the reference's ARPACK draws a random residual): a pseudo-random
        // combination of the factor's columns plus 1 % pseudo-random noise keyed by the global
        // row.  Near optimality S R ~ 0 (complementarity), so lambda_min sits in the near-null
        // cluster spanned by R, which this start reaches in far fewer steps than a plain random
        // vector; the noise keeps every eigendirection in the Krylov space.  LRS_TRL_START=random:
        // the noise alone.
        const bool rnd_only = getenv("LRS_TRL_START") && !strcmp(getenv("LRS_TRL_START"), "random");
        std::vector<double> Rh((size_t)nown * dc.ld, 0.0), q0(nown), z(nown), g(dc.ld, 0.0);
        HIPC(hipMemcpyAsync(Rh.data(), c->W.R + dc.foff + (long)r0 * dc.ld, sizeof(double) * Rh.size(),
                            hipMemcpyDeviceToHost, c->st));
        HIPC(hipStreamSynchronize(c->st));
        unsigned long long st = 0x9E3779B97F4A7C15ULL;
        for (int q = 0; q < dc.r; ++q) {
            st = st * 6364136223846793005ULL + 1442695040888963407ULL;
            g[q] = ((double)(st >> 11) / 9007199254740992.0) - 0.5;
        }
        double sums[3] = {0.0, 0.0, 0.0};
        for (int i = 0; i < nown; ++i) {
            double t = 0.0;
            if (!rnd_only)
                for (int q = 0; q < dc.r; ++q) t += Rh[(size_t)i * dc.ld + q] * g[q];
            q0[i] = t;
            unsigned long long h = (unsigned long long)(sh ? c->plan.cones[k].gid[r0 + i] : i) + 0x632BE59BD9B4E019ULL;
            h = (h ^ (h >> 30)) * 0xBF58476D1CE4E5B9ULL;
            h = (h ^ (h >> 27)) * 0x94D049BB133111EBULL;
            h ^= h >> 31;
            z[i] = ((double)(h >> 11) / 9007199254740992.0) - 0.5;
            sums[0] += t * t;
            sums[1] += z[i] * z[i];
        }
        if (sh && c->comm->allreduce_host(c, sums, 2)) return -1;
        const double zs = (sums[0] > 0 ? 1e-2 * std::sqrt(sums[0]) : 1.0) / std::sqrt(std::max(sums[1], 1e-300));
        for (int i = 0; i < nown; ++i) {
            q0[i] += zs * z[i];
            sums[2] += q0[i] * q0[i];
        }
        double nrm2 = sums[2];
        if (sh && c->comm->allreduce_host(c, &nrm2, 1)) return -1;
        const double inv = 1.0 / std::sqrt(std::max(nrm2, 1e-300));
        for (double &v : q0) v *= inv;
        HIPC(hipMemcpyAsync(V + r0, q0.data(), sizeof(double) * nown, hipMemcpyHostToDevice, c->st));
        HIPC(hipStreamSynchronize(c->st));   // q0 is a host temporary
    }
    std::vector<double> Hh((size_t)ldh * ncv), b2h(ncv), T, w, Zm, Yh, keep;
    const double *win = V;       // v_j's unnormalized source (the start vector is normalized)
    const double *b2in = nullptr;
    int cur = 0, j0 = 0, iter = 0, steps = 0, msz = ncv;
    double theta = 0.0, bound = 0.0;
    bool conv = false;
    int rc = 0;
    for (;;) {
        for (int j = j0; j < ncv && rc == 0; ++j) {
            double *vj = V + (long)j * ldv, *y = Z.y[cur];
            if (sh) {
                if (b2in) OPC(launch_trl_norm(nown, win + r0, b2in, vj + r0, c->st));
                if (c->comm->halo_vec(c, k, vj, c->st)) return -1;
                OPC(launch_trl_symv(c->dp, k, S, vj, nullptr, nullptr, y, c->st));
            } else {
                OPC(launch_trl_symv(c->dp, k, S, win, b2in, b2in ? vj : nullptr, y, c->st));
            }
            for (int pass = 0; pass < 2; ++pass) {
                OPC(launch_trl_dots(nown, V + r0, ldv, j + 1, y + r0, Z.part, c->st));
                int nb = trl_nblk(nown);
                const double *pp = Z.part;
                if (sh) {
                    OPC(launch_trl_fold(j + 1, nb, Z.part, tot, c->st));
                    if (c->comm->allreduce_dev(c, tot, j + 1, c->st)) return -1;
                    pp = tot;
                    nb = 1;
                }
                OPC(launch_trl_sub(nown, V + r0, ldv, j + 1, pp, nb, y + r0, Hd + (long)j * ldh, pass, npart, bw2 + j,
                                   c->st));
            }
            if (sh && c->comm->allreduce_dev(c, bw2 + j, 1, c->st)) return -1;
            win = y;
            b2in = bw2 + j;
            cur ^= 1;
            steps++;
        }
        HIPC(hipMemcpyAsync(Hh.data(), Hd, sizeof(double) * ldh * ncv, hipMemcpyDeviceToHost, c->st));
        HIPC(hipMemcpyAsync(b2h.data(), bw2, sizeof(double) * ncv, hipMemcpyDeviceToHost, c->st));
        HIPC(hipStreamSynchronize(c->st));
        // the Rayleigh matrix V^T S V: kept Ritz values on the diagonal, the new columns from the
        // coefficients (the coupling to the previous vector averaged with its beta)
        T.assign((size_t)ncv * ncv, 0.0);
        for (int q = 0; q < j0; ++q) T[(size_t)q * ncv + q] = keep[q];
        for (int j = j0; j < ncv; ++j)
            for (int q = 0; q <= j; ++q) {
                double v = Hh[(size_t)j * ldh + q];
                if (q == j - 1 && j > j0) v = 0.5 * (v + std::sqrt(std::max(b2h[j - 1], 0.0)));
                T[(size_t)q * ncv + j] = T[(size_t)j * ncv + q] = v;
            }
        double tnorm = 0.0;
        for (int q = 0; q < ncv; ++q) {
            double a = 0.0;
            for (int j = 0; j < ncv; ++j) a += std::fabs(T[(size_t)q * ncv + j]);
            tnorm = std::max(tnorm, a);
        }
        // an invariant subspace inside this cycle: the leading block is exact
        msz = ncv;
        double betam = std::sqrt(std::max(b2h[ncv - 1], 0.0));
        for (int j = j0; j < ncv - 1; ++j)
            if (std::sqrt(std::max(b2h[j], 0.0)) <= 1e-14 * std::max(1.0, tnorm)) { msz = j + 1; betam = 0.0; break; }
        std::vector<double> Tm((size_t)msz * msz);
        for (int q = 0; q < msz; ++q)
            for (int j = 0; j < msz; ++j) Tm[(size_t)q * msz + j] = T[(size_t)q * ncv + j];
        jacobi_eig(msz, Tm, w, Zm);
        theta = w[0];
        bound = betam * std::fabs(Zm[(size_t)(msz - 1) * msz + 0]);
        iter++;
        const bool brk = betam <= 1e-14 * std::max(1.0, tnorm);
        conv = brk || bound <= tol * std::max(eps23, std::fabs(theta)) || bound <= abs_tol;
        if (getenv("LRS_LANCZOS_TRACE") && (iter <= 3 || iter % 20 == 0 || conv))
            fprintf(stderr, "  trl cone %d iter %d steps %d theta %.12e bound %.3e (tol %.3e abs %.3e)\n", k, iter, steps,
                    theta, bound, tol * std::max(eps23, std::fabs(theta)), abs_tol);
        if (conv || iter > maxiter || msz < ncv) break;
        // restart from the kk smallest Ritz vectors (ascending) and the residual direction
        Yh.assign((size_t)ncv * kk, 0.0);
        for (int q = 0; q < ncv; ++q)
            for (int e = 0; e < kk; ++e) Yh[(size_t)q * kk + e] = Zm[(size_t)q * ncv + e];
        HIPC(hipMemcpyAsync(Z.Y, Yh.data(), sizeof(double) * Yh.size(), hipMemcpyHostToDevice, c->st));
        OPC(launch_trl_restart(nown, V + r0, ldv, ncv, Z.Y, kk, Z.Vt + r0, c->st));
        HIPC(hipMemcpy2DAsync(V + r0, sizeof(double) * ldv, Z.Vt + r0, sizeof(double) * ldv, sizeof(double) * nown, kk,
                              hipMemcpyDeviceToDevice, c->st));
        HIPC(hipStreamSynchronize(c->st));   // Yh is a host temporary
        keep.assign(w.begin(), w.begin() + kk);
        j0 = kk;
        b2in = bw2 + (ncv - 1);   // v_kk = residual / beta_m (the residual is `win`)
    }
    if (!conv)
        fprintf(stderr, "[lrsdp] dual infeasibility: the eigen-solve on cone %d stopped after %d update iterations "
                "(%d steps; Ritz value %.6e, Ritz estimate %.3e): lambda_min may be lower, the l_1 value a lower bound\n",
                k, iter, steps, theta, bound);
    *lam_min = theta;
    if (steps_out) *steps_out = steps;
    if (iters_out) *iters_out = iter;
    if (converged) *converged = conv;
    if (getenv("LRS_LANCZOS_TRACE"))
        fprintf(stderr, "trl cone %d: n %d, ncv %d, %d update iterations, %d steps, lambda_min %.12e\n", k, N, ncv, iter,
                steps, theta);
    return rc;
}

// l_1 dual infeasibility of the current lambda (data/lorads_solver.c:1396-1426); lam_min per
// cone into lmin (may be null)
static int dual_infeasibility(lrs_ctx *c, double *l1, double *lmin, int *all_conv = nullptr) {
    DevWork &W = c->W;
    const int m = c->dp.m;
    HIPC(hipMemsetAsync(W.wtmp, 0, sizeof(double) * m, c->st));
    OPC(launch_axpby(m, -1.0, W.lam, 1.0, W.wtmp, c->st));          // negLambd = -dualVar
    OPC(launch_wsum(c->dp, W.wtmp, 1, W.S, c->st));                 // S = C + A^*(negLambd)
    double err = 0.0;
    const double t0 = now_s();
    for (int k = 0; k < c->dp.K; ++k) {
        double lk = 0.0;
        bool conv = true;
        int steps = 0, iters = 0;
        if (is_lp(c, k)) {
            // the LP block (calculate_dual_infeasibility_solver, data/lorads_solver.c:1405-1412):
            // per column |min(c_j - sum_i lambda_i a_ij, 0)|, i.e. the negative part of every
            // diagonal slot of S; a column without data contributes 0
            const DevCone &d = c->dp.cones[k];
            std::vector<double> s(std::max(1, d.P));
            HIPC(hipMemcpyAsync(s.data(), W.S + d.slot_off, sizeof(double) * d.P, hipMemcpyDeviceToHost, c->st));
            HIPC(hipStreamSynchronize(c->st));
            double lpe = 0.0;
            lk = d.P < d.n ? 0.0 : 1e300;
            for (int t = 0; t < d.P; ++t) {
                lpe += std::fabs(std::min(s[t], 0.0));
                lk = std::min(lk, s[t]);
            }
            if (lmin) lmin[k] = lk;
            err += lpe;
            continue;
        }
        if (trl_min(c, k, W.S, &lk, &steps, &iters, &conv)) return -1;
        c->dinf_steps += steps;
        c->dinf_iters += iters;
        if (lmin) lmin[k] = lk;
        if (all_conv && !conv) *all_conv = 0;
        err += std::fabs(std::min(lk, 0.0));
    }
    err /= c->scaleObjHis;
    err /= (c->hp.cNrm1 + 1);
    *l1 = err;
    c->dinf_time += now_s() - t0;
    return 0;
}

static void cal_dual_obj(lrs_ctx *c) {   // LORADSCalDualObj lorads_alg_common.c:531
    double v = 0;
    op_dot(c, c->dp.m, c->dp.bprim ? c->dp.bprim : c->dp.b, c->W.lam, &v);   // sharded: once per constraint
    c->dObjVal = v / c->scaleObjHis;
}

// updateDimacsALM on R (lorads_alg_common.c:424-428) + objective
static int update_dimacs(lrs_ctx *c, const double *X, const double *Y, bool with_obj) {
    double pinf, obj;
    if (op_constr_xx(c, X, Y, &pinf, &obj)) return -1;
    if (with_obj) c->pObjVal = obj / c->scaleObjHis;
    c->dimPinf = pinf;
    double gap = c->pObjVal - c->dObjVal;
    c->dimGap = std::fabs(gap) / (1 + std::fabs(c->pObjVal) + std::fabs(c->dObjVal));
    return 0;
}

// ---- oracle rank: device Gram + host Jacobi eigenvalues (lorads_logging.c:216-366)
// Number of eigenvalues of the symmetric r x r matrix A above eps * lambda_max
// (count_significant_from_matrix, lorads_logging.c:272-366, which takes all eigenvalues from
// dsyevr): Householder reduction to tridiagonal form, lambda_max by Sturm bisection, then one
// Sturm count at eps * lambda_max -- O(r^3) once instead of a Jacobi sweep loop (the oracle
// rank runs every ADMM iteration, lorads_admm.c:60).
static int sym_count(int r, std::vector<double> A, double eps) {
    if (r <= 0) return 0;
    std::vector<double> d(r), e(r, 0.0), v(r), w(r);
    for (int k = 0; k < r - 2; ++k) {
        // Householder vector for column k below the diagonal
        double alpha = 0.0;
        for (int i = k + 1; i < r; ++i) alpha += A[i * r + k] * A[i * r + k];
        alpha = std::sqrt(alpha);
        if (alpha == 0.0) { e[k] = 0.0; continue; }
        const double x0 = A[(k + 1) * r + k];
        if (x0 > 0) alpha = -alpha;
        e[k] = alpha;
        double vn = 0.0;
        for (int i = k + 1; i < r; ++i) v[i] = A[i * r + k];
        v[k + 1] -= alpha;
        for (int i = k + 1; i < r; ++i) vn += v[i] * v[i];
        if (vn == 0.0) continue;
        // A <- H A H on the trailing block, H = I - 2 v v^T / (v^T v)
        const double beta = 2.0 / vn;
        double vw = 0.0;
        for (int i = k + 1; i < r; ++i) {
            double t = 0.0;
            for (int j = k + 1; j < r; ++j) t += A[i * r + j] * v[j];
            w[i] = beta * t;
            vw += v[i] * w[i];
        }
        const double hk = 0.5 * beta * vw;
        for (int i = k + 1; i < r; ++i) w[i] -= hk * v[i];
        for (int i = k + 1; i < r; ++i)
            for (int j = k + 1; j < r; ++j) A[i * r + j] -= v[i] * w[j] + w[i] * v[j];
    }
    for (int i = 0; i < r; ++i) d[i] = A[i * r + i];
    if (r >= 2) e[r - 2] = A[(r - 1) * r + (r - 2)];
    // Sturm count of eigenvalues below x for tridiag(e, d, e)
    auto below = [&](double x) {
        int cnt = 0;
        double q = 1.0;
        for (int i = 0; i < r; ++i) {
            q = (d[i] - x) - (i > 0 ? e[i - 1] * e[i - 1] / q : 0.0);
            if (q == 0.0) q = -1e-300;
            if (q < 0) ++cnt;
        }
        return cnt;
    };
    double lo = 1e300, hi = -1e300;
    for (int i = 0; i < r; ++i) {
        const double rad = (i > 0 ? std::fabs(e[i - 1]) : 0.0) + (i < r - 1 ? std::fabs(e[i]) : 0.0);
        lo = std::min(lo, d[i] - rad);
        hi = std::max(hi, d[i] + rad);
    }
    for (int it = 0; it < 200 && hi - lo > 1e-14 * std::max(std::fabs(lo), std::fabs(hi)) + 1e-300; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (mid <= lo || mid >= hi) break;
        if (below(mid) >= r) hi = mid;   // every eigenvalue below mid: lambda_max < mid
        else lo = mid;
    }
    const double mx = 0.5 * (lo + hi);
    if (!(mx > 0)) return 0;
    return r - below(eps * mx);
}

static int gram_of(lrs_ctx *c, int k, const double *X, const double *Y, int avg, std::vector<double> &g) {
    int nblk = 0;
    OPC(launch_gram(c->dp, k, X, Y, avg, c->W.gram, &nblk, c->st));
    const int rr = c->rank[k] * c->rank[k];
    g.resize(rr);
    HIPC(hipMemcpyAsync(g.data(), c->W.gram, sizeof(double) * rr, hipMemcpyDeviceToHost, c->st));
    HIPC(hipStreamSynchronize(c->st));
    if (sharded(c)) return c->comm->allreduce_host(c, g.data(), rr);
    return 0;
}

static int oracle_rank(lrs_ctx *c, int phase) {
    const int K = c->dp.K;
    // every cone's Gram copied behind its launch into one pinned buffer, one synchronisation
    size_t need = 0;
    for (int k = 0; k < K; ++k) need += (size_t)c->rank[k] * c->rank[k];
    if (need > c->hgram_n) {
        if (c->hgram) HIPC(hipHostFree(c->hgram));
        c->hgram = nullptr;
        HIPC(hipHostMalloc((void **)&c->hgram, sizeof(double) * need));
        c->hgram_n = need;
    }
    size_t off = 0;
    for (int k = 0; k < K; ++k) {
        if (is_lp(c, k)) continue;   // lorads_compute_oracle_rank runs over the SDP cones
        int nblk = 0;
        if (phase == 1) OPC(launch_gram(c->dp, k, c->W.R, nullptr, 0, c->W.gram, &nblk, c->st));
        else OPC(launch_gram(c->dp, k, c->W.U, c->W.V, 1, c->W.gram, &nblk, c->st));
        const size_t rr = (size_t)c->rank[k] * c->rank[k];
        HIPC(hipMemcpyAsync(c->hgram + off, c->W.gram, sizeof(double) * rr, hipMemcpyDeviceToHost, c->st));
        off += rr;
    }
    HIPC(hipStreamSynchronize(c->st));
    int tot = 0;
    off = 0;
    for (int k = 0; k < K; ++k) {
        if (is_lp(c, k)) continue;
        const size_t rr = (size_t)c->rank[k] * c->rank[k];
        std::vector<double> g(c->hgram + off, c->hgram + off + rr);
        if (sharded(c) && c->comm->allreduce_host(c, g.data(), (int)rr)) return -1;
        tot += sym_count(c->rank[k], g, 1e-6);
        off += rr;
    }
    return tot;
}
// --oracleRankNaive (LORADS_ORACLE_RANK_NAIVE, lorads_logging.c:406-451 selected at :516-533):
// per cone of at most kNaiveMaxN rows the n x n matrix X = R R^T (phase 1) or
// ((U+V)/2)((U+V)/2)^T (phase 2) formed in full on the host from the device factor and its
// eigenvalues above 1e-6 lambda_max counted (sym_count: the same Householder + Sturm count the
// Gram path uses, i.e. count_significant_from_matrix's rule on the n x n matrix); larger cones
// take the Gram path after one log line, as the reference prints once per solve.  A sharded
// context holds only its rows, so it keeps the Gram path (the all-reduced Gram is exact).
constexpr int kNaiveMaxN = 2000;
static int oracle_rank_naive(lrs_ctx *c, const lrs_params *p, int phase) {
    if (sharded(c)) return oracle_rank(c, phase);
    int tot = 0;
    for (int k = 0; k < c->dp.K; ++k) {
        if (is_lp(c, k)) continue;
        const DevCone &d = c->dp.cones[k];
        const int n = d.n, r = c->rank[k];
        if (n > kNaiveMaxN) {
            if (!c->naive_warned) {
                logf_(c, p, "skip naive oracle rank for n=%ld, falling back to gram approach.\n", (long)n);
                c->naive_warned = true;
            }
            std::vector<double> g;
            if (phase == 1) OPC(gram_of(c, k, c->W.R, nullptr, 0, g));
            else OPC(gram_of(c, k, c->W.U, c->W.V, 1, g));
            tot += sym_count(r, g, 1e-6);
            continue;
        }
        std::vector<double> F((size_t)n * d.ld), F2;
        HIPC(hipStreamSynchronize(c->st));
        HIPC(hipMemcpy(F.data(), (phase == 1 ? c->W.R : c->W.U) + d.foff, sizeof(double) * F.size(),
                       hipMemcpyDeviceToHost));
        if (phase != 1) {
            F2.resize(F.size());
            HIPC(hipMemcpy(F2.data(), c->W.V + d.foff, sizeof(double) * F2.size(), hipMemcpyDeviceToHost));
            for (size_t q = 0; q < F.size(); ++q) F[q] = 0.5 * (F[q] + F2[q]);
        }
        std::vector<double> X((size_t)n * n);
        for (int i = 0; i < n; ++i)
            for (int j = i; j < n; ++j) {
                double s = 0.0;
                for (int q = 0; q < r; ++q) s += F[(size_t)i * d.ld + q] * F[(size_t)j * d.ld + q];
                X[(size_t)i * n + j] = s;
                X[(size_t)j * n + i] = s;
            }
        tot += sym_count(n, std::move(X), 1e-6);
    }
    return tot;
}

static int sum_rank(lrs_ctx *c) {   // curr_rank: the SDP cones' (the reference's rankElem)
    int t = 0;
    for (int k = 0; k < (int)c->rank.size(); ++k) t += is_lp(c, k) ? 0 : c->rank[k];
    return t;
}

static void record_state(lrs_ctx *c, const lrs_params *p, int phase) {
    int cur = sum_rank(c);
    int orc = p->disableOracle ? cur : p->oracleRankNaive ? oracle_rank_naive(c, p, phase) : oracle_rank(c, phase);
    if (orc < 0) orc = 0;
    if (phase == 1) { c->t1c.push_back(cur); c->t1o.push_back(orc); }
    else { c->t2c.push_back(cur); c->t2o.push_back(orc); }
}

// ---- rank determination (data/lorads_solver.c:406-459) + schedule hook
// Ranks past the widest factor layout (choose_layout: 512 columns) are clamped there, with one
// stderr line per solve: --fixedRank, rank-schedule entries and AUG_RANK's rank_max =
// sqrt(2 nnzRows) + 1 (C5's m = 10^6 gives 1 415) would otherwise end the solve.
constexpr int kMaxRank = 512;
static int clamp_rank(int r, bool *warned) {
    if (r <= kMaxRank) return r;
    if (warned && !*warned) {
        fprintf(stderr, "[lrsdp] rank %d above the device maximum %d: clamped to %d\n", r, kMaxRank, kMaxRank);
        *warned = true;
    }
    return kMaxRank;
}

static void determine_rank(lrs_ctx *c, const lrs_params *p, std::vector<int> &rank, std::vector<int> &rmax) {
    const int K = c->hp.K;
    rank.assign(K, 1);
    rmax.assign(K, 1);
    int tot_default = 0;
    std::vector<int> dflt(K);
    for (int k = 0; k < K; ++k) {
        const HostCone &hc = c->hp.cones[k];
        if (hc.lp) { rank[k] = rmax[k] = dflt[k] = 1; continue; }   // x_j = r_j^2: rank 1, no growth
        const int hn = cone_n_global(c, k);
        int nnzRows = hc.nnzRows;
        int calc = std::min((int)std::sqrt(2.0 * nnzRows) + 1, hn);
        if (p->fixedRank > 0) {
            rank[k] = std::max(1, std::min(p->fixedRank, hn));
            rmax[k] = rank[k];
            dflt[k] = rank[k];
            tot_default += rank[k];
            continue;
        }
        rmax[k] = calc;
        int rk;
        if (p->initRank > 0) rk = std::min(p->initRank, hn);
        else if (p->timesLogRank <= 1e-6) rk = calc;
        else if (nnzRows / hn >= 20 && hn <= 400 && K - (c->hp.nLp > 0 ? 1 : 0) <= 3) rk = calc;   // nCones: SDP blocks
        else rk = (int)std::min(std::ceil(p->timesLogRank * std::log((double)hn)), (double)calc);
        rank[k] = std::max(1, rk);
        dflt[k] = rank[k];
        tot_default += rank[k];
    }
    if (p->rankSchedule && p->rankScheduleLen > 0 && p->fixedRank <= 0) {
        // entry 0 is the initial TOTAL rank, split across cones in proportion to the default ranks
        int tot = std::max(1, p->rankSchedule[0]);
        for (int k = 0; k < K; ++k) {
            if (c->hp.cones[k].lp) continue;
            int rk = (int)std::lround((double)tot * dflt[k] / std::max(1, tot_default));
            rank[k] = std::max(1, std::min(rk, cone_n_global(c, k)));
            rmax[k] = std::max(rmax[k], rank[k]);
        }
    }
    bool warned = false;
    for (int k = 0; k < K; ++k) {
        rank[k] = clamp_rank(rank[k], &warned);
        rmax[k] = std::min(rmax[k], kMaxRank);   // growth stops at the cap silently (AUG_RANK's max)
    }
}

// random initial point R (LORADS_RANDOM_rk_MAT), cones in order, column-major draw order
static int init_point(lrs_ctx *c) {
    if (c->init_ranks == c->rank && !c->init_cache.empty()) {
        HIPC(hipMemcpyAsync(c->W.R, c->init_cache.data(), sizeof(double) * c->init_cache.size(),
                            hipMemcpyHostToDevice, c->st));
        return 0;
    }
    GlibcRand g(925);
    long NRc = 0;
    for (int k = 0; k < c->dp.K; ++k) NRc += (long)cone_n_global(c, k) * c->rank[k];
    std::vector<double> R(NRc);
    for (long i = 0; i < NRc; ++i) {
        double v = (double)g.next() / 2147483647.0;
        v -= (double)g.next() / 2147483647.0;
        R[i] = v;
    }
    if (sharded(c)) {
        // the whole problem's draw (cones in order, each column-major), then this shard's rows
        // (owned + halo) of every cone
        long NRl = 0, og = 0, ol = 0;
        for (int k = 0; k < c->dp.K; ++k) NRl += (long)c->dp.cones[k].n * c->rank[k];
        std::vector<double> Rl(NRl);
        for (int k = 0; k < c->dp.K; ++k) {
            const ShardConePlan &cp = c->plan.cones[k];
            const int ng = cp.n_global, nl = c->dp.cones[k].n, r = c->rank[k];
            for (int q = 0; q < r; ++q)
                for (int l = 0; l < nl; ++l) Rl[ol + l + (long)q * nl] = R[og + cp.gid[l] + (long)q * ng];
            og += (long)ng * r;
            ol += (long)nl * r;
        }
        R.swap(Rl);
    }
    if (factor_put(c, c->W.R, R.data())) return -1;
    // keep the device-layout copy: every solve at these ranks starts from the same point
    c->init_cache.assign(c->dp.NRpad, 0.0);
    HIPC(hipMemcpy(c->init_cache.data(), c->W.R, sizeof(double) * c->dp.NRpad, hipMemcpyDeviceToHost));
    c->init_ranks = c->rank;
    return 0;
}

// ---- AUG_RANK (data/lorads_solver.c:1154-1254)
static int check_all_rank_max(lrs_ctx *c, double f) {
    int cnt = 0;
    for (int k = 0; k < c->dp.K; ++k) {
        if (is_lp(c, k)) continue;   // CheckAllRankMax runs over the SDP cones
        int nr = (int)std::min(std::ceil(c->rank[k] * f), (double)c->rank_max[k]);
        if (nr >= c->rank_max[k]) cnt++;
    }
    return cnt == n_sdp(c);
}

static int regrow(lrs_ctx *c, const std::vector<int> &nr) {
    // fetch R, U, V, G in reference layout, extend columns, reallocate, upload
    long NRo = 0;
    for (int k = 0; k < c->dp.K; ++k) NRo += (long)c->dp.cones[k].n * c->rank[k];
    std::vector<double> R(NRo), U(NRo), V(NRo), G(NRo);
    if (factor_fetch(c, c->W.R, R.data()) || factor_fetch(c, c->W.U, U.data()) ||
        factor_fetch(c, c->W.V, V.data()) || factor_fetch(c, c->W.G[c->gcur], G.data()))
        return -1;
    std::vector<double> lam(c->dp.m), cvs(c->dp.m);
    HIPC(hipMemcpy(lam.data(), c->W.lam, sizeof(double) * c->dp.m, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(cvs.data(), c->W.cvs, sizeof(double) * c->dp.m, hipMemcpyDeviceToHost));
    long NRn = 0;
    for (int k = 0; k < c->dp.K; ++k) NRn += (long)c->dp.cones[k].n * nr[k];
    std::vector<double> Rn(NRn, 0.0), Un(NRn, 0.0), Vn(NRn, 0.0), Gn(NRn, 0.0);
    long so = 0, dn = 0;
    for (int k = 0; k < c->dp.K; ++k) {
        const int n = c->dp.cones[k].n, ro = c->rank[k], rn = nr[k];
        auto grow = [&](const std::vector<double> &src, std::vector<double> &dst) {
            std::copy(src.begin() + so, src.begin() + so + (long)n * ro, dst.begin() + dn);
            const int aug = rn - ro, r = std::min(cone_n_global(c, k), aug);   // lpRandomDiag :1096-1106
            if (sharded(c)) {   // global row i of new column i, on the shard's local rows
                for (int l = 0; l < n; ++l) {
                    const int gi = c->plan.cones[k].gid[l];
                    if (gi < r) dst[dn + (long)n * ro + (long)gi * n + l] = 1 / std::sqrt((double)r);
                }
            } else {
                for (int i = 0; i < r; ++i) dst[dn + (long)n * ro + (long)i * n + i] = 1 / std::sqrt((double)r);
            }
        };
        grow(R, Rn); grow(U, Un); grow(V, Vn); grow(G, Gn);
        so += (long)n * ro;
        dn += (long)n * rn;
    }
    int gc = c->gcur;
    if (alloc_work(c, nr)) return -1;
    c->gcur = gc;
    if (factor_put(c, c->W.R, Rn.data()) || factor_put(c, c->W.U, Un.data()) || factor_put(c, c->W.V, Vn.data()) ||
        factor_put(c, c->W.G[c->gcur], Gn.data()))
        return -1;
    HIPC(h2d_sync(c, c->W.lam, lam.data(), sizeof(double) * c->dp.m));
    HIPC(h2d_sync(c, c->W.cvs, cvs.data(), sizeof(double) * c->dp.m));
    return 0;
}

static int aug_rank(lrs_ctx *c, double f, const lrs_params *p, int *sched_pos, int *is_max) {
    if (check_all_rank_max(c, 1.0)) { *is_max = 1; return 0; }
    std::vector<int> nr(c->dp.K);
    bool sched = p->rankSchedule && p->rankScheduleLen > 0 && p->fixedRank <= 0;
    if (sched) {
        int pos = *sched_pos + 1;
        if (pos >= p->rankScheduleLen) { *is_max = 1; return 0; }
        *sched_pos = pos;
        int tot = std::max(1, p->rankSchedule[pos]), cur = sum_rank(c);
        for (int k = 0; k < c->dp.K; ++k) {
            if (is_lp(c, k)) { nr[k] = 1; continue; }
            int rk = (int)std::lround((double)tot * c->rank[k] / std::max(1, cur));
            nr[k] = clamp_rank(std::max(c->rank[k], std::min(rk, cone_n_global(c, k))), &c->rank_warned);
            c->rank_max[k] = std::max(c->rank_max[k], nr[k]);
        }
    } else {
        for (int k = 0; k < c->dp.K; ++k)
            nr[k] = is_lp(c, k) ? 1 : (int)std::min(std::ceil(c->rank[k] * f), (double)c->rank_max[k]);
    }
    if (regrow(c, nr)) return -1;
    if (sched) *is_max = (*sched_pos + 1 >= p->rankScheduleLen) ? 1 : 0;
    else *is_max = check_all_rank_max(c, f);
    return 0;
}

// LUtilUpdateCheckEma (lorads_utils.c:564-594)
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

// ---- device inner loop
// Batch of B inner iterations (B even, so the batch ends on parity 1) captured once
// into a hipGraph and replayed: one host launch per batch instead of 4B.
static int get_batch_graph(lrs_ctx *c, int B, hipGraphExec_t *out) {
    auto it = c->graphs.find(B);
    if (it != c->graphs.end()) { *out = it->second; return 0; }
    AlmIterArgs a{&c->dp, &c->W, nullptr};
    hipGraph_t g = nullptr;
    HIPC(hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal));
    int rc = 0;
    for (int j = 0; j < B && rc == 0; ++j) rc = enqueue_alm_iteration(a, j & 1, c->st);
    hipError_t e = hipStreamEndCapture(c->st, &g);
    if (rc != 0) { if (g) (void)hipGraphDestroy(g); set_err("capture: %s", last_device_error()); return -1; }
    if (e != hipSuccess) { set_err("hipStreamEndCapture: %s", hipGetErrorString(e)); return -1; }
    hipGraphExec_t ge = nullptr;
    e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) { set_err("hipGraphInstantiate: %s", hipGetErrorString(e)); return -1; }
    c->graphs[B] = ge;
    *out = ge;
    return 0;
}

struct InnerIo {
    long inner, local, clear;
    double rcval, lag, pinf1, pinfinf;
    int exitReason;
    bool resume = false;   // continue from the control block the last call stopped on (budget exit)
};

// The single-workgroup inner loop (lrs_kernels.hip k_small_alm) where the problem fits it (not
// sharded, two L-BFGS pairs, one factor layout, no full dense C, R and D of every cone in one
// CU's LDS): kernel path 4 always; the automatic path 0 unless LRS_SMALL=0, with at most
// kSmallMaxGlobal multi-slot constraints (LRS_SMALL=1 lifts that bound) -- each takes a wave
// of the workgroup per phase, and on rsparse60 (every constraint multi-slot) the multi-launch
// iteration is faster (scripts/small_compare.py).
constexpr int kSmallMaxGlobal = 16;
static bool use_small(lrs_ctx *c) {
    const char *e = getenv("LRS_SMALL");
    const int env = e ? atoi(e) : -1;
    if (sharded(c) || c->lbfgsL != 2 || c->small_off) return false;
    if (c->dp.no_lat != 4) {
        if (c->dp.no_lat != 0 || env == 0) return false;
        if (env != 1 && c->dp.mg > kSmallMaxGlobal) return false;
    }
    return small_alm_fits(c->dp, c->W);
}

// what k_small_alm writes (the iterate, both gradients, the L-BFGS pairs, A(RR^T), the
// constraint records, the control blocks, the line search): kept before a one-workgroup-per-cone
// launch (save = true) and put back after its exchange timed out (save = false)
static int xwg_snapshot(lrs_ctx *c, bool save) {
    DevWork &W = c->W;
    const long NR = std::max(2L, c->dp.NRpad), m = std::max(1, c->dp.m);
    struct B { double *p; long n; } bs[] = {{W.R, NR}, {W.G[0], NR}, {W.G[1], NR}, {W.ls[0], NR}, {W.ly[0], NR},
                                            {W.ls[1], NR}, {W.ly[1], NR}, {W.cvs, m}, {W.rec, 4 * m},
                                            {W.ctrl, 2 * C_NCTRL}, {W.lsres, 2 * LS_N}};
    long need = 0;
    for (auto &b : bs) need += b.n;
    if (need > c->xwg_snap_len) {
        if (c->xwg_snap) HIPC(hipFree(c->xwg_snap));
        c->xwg_snap = nullptr;
        HIPC(hipMalloc((void **)&c->xwg_snap, sizeof(double) * need));
        c->xwg_snap_len = need;
    }
    long off = 0;
    for (auto &b : bs) {
        if (save) HIPC(hipMemcpyAsync(c->xwg_snap + off, b.p, sizeof(double) * b.n, hipMemcpyDeviceToDevice, c->st));
        else HIPC(hipMemcpyAsync(b.p, c->xwg_snap + off, sizeof(double) * b.n, hipMemcpyDeviceToDevice, c->st));
        off += b.n;
    }
    return 0;
}

static int run_inner(lrs_ctx *c, const lrs_params *p, double rho, double rctol, double gap, long budget, InnerIo &io,
                     bool ph1_exit = true) {
    double par[P_NPAR] = {0};
    par[P_RHO] = rho; par[P_RCTOL] = rctol; par[P_ENDSUB] = p->endALMSubTol; par[P_ENDTAU] = p->endTauTol;
    par[P_PH1TOL] = ph1_exit ? p->phase1Tol : -1.0; par[P_BN1] = c->hp.bNrm1; par[P_BNINF] = c->hp.bNrmInf; par[P_CNINF] = c->hp.cNrmInf;
    par[P_HIGHACC] = p->highAccMode; par[P_BUDGET] = (double)budget; par[P_L] = p->lbfgsListLength; par[P_GAP] = gap;
    double ctl[C_NCTRL] = {0};
    ctl[C_ACTIVE] = 1; ctl[C_EXIT] = EXIT_NONE; ctl[C_INNER] = (double)io.inner; ctl[C_LOCAL] = (double)io.local;
    ctl[C_ACT2] = 1; ctl[C_EXIT2] = EXIT_NONE; ctl[C_RRDONE] = 0; ctl[C_RCUR] = 0;
    ctl[C_CLEAR] = (double)io.clear; ctl[C_HEAD] = c->head; ctl[C_GCUR] = c->gcur; ctl[C_PENDING] = 0;
    ctl[C_RCVAL] = io.rcval; ctl[C_LAG] = io.lag; ctl[C_PINF1] = io.pinf1; ctl[C_PINFINF] = io.pinfinf;
    ctl[C_BETA0] = c->beta[0]; ctl[C_BETA1] = c->beta[1]; ctl[C_YY0] = c->yy[0]; ctl[C_YY1] = c->yy[1];
    if (io.resume) {
        // a budget exit stops an iteration after its fold (PENDING = 2, the L-BFGS dots of
        // the new gradient kept) and before its direction: restart exactly there.  R was
        // moved back into W.R by the previous call, so RCUR restarts at 0.
        memcpy(ctl, c->last_ctl, sizeof(ctl));
        ctl[C_ACTIVE] = 1; ctl[C_EXIT] = EXIT_NONE; ctl[C_ACT2] = 1; ctl[C_EXIT2] = EXIT_NONE; ctl[C_RCUR] = 0;
    }
    OPC(launch_put_ctrl(par, ctl, c->W.par, c->W.ctrl + C_NCTRL, c->st));
    AlmIterArgs a{&c->dp, &c->W, nullptr};
    // Batch sizes: start near the running estimate of this call's length, double after
    // each batch, never beyond the iterations to a certain exit (budget, localIter 800)
    // + 1 (the iteration whose first stage detects it).  B stays even (parity).
    long certain = 801 - io.local;
    if (budget > 0) certain = std::min(certain, budget - io.inner);
    certain = std::max(0L, certain) + 1;
    auto even_clamp = [](long v) { v = std::max(4L, std::min(64L, v)); return (int)(v + (v & 1)); };
    int B = even_clamp((long)(c->inner_est * 0.5));
    double *res = c->hpin + kHpCtrl;
    const double t_in = c->stats ? now_s() : 0.0;
    long enq = 0;
    // the single-workgroup inner loop (small problems): the whole call is one launch
    bool small = !c->prof && use_small(c);
    bool fell_back = false;
    if (small) {
        // one workgroup per cone: the workgroups hand sums to each other through device memory,
        // which assumes they are co-resident; another stream or context holding the CUs can delay
        // one past the exchange's spin limit (EXIT_XWG).  The state the loop writes is kept
        // first, so such a call is rerun from it on the multi-launch iteration.
        const bool mc = small_alm_workgroups(c->dp, c->W) > 1;
        if (mc && xwg_snapshot(c, true)) return -1;
        OPC(launch_small_alm(c->dp, c->W, c->W.ctrl + C_NCTRL, c->W.ctrl + C_NCTRL, c->W.lsres, c->st));
        HIPC(hipMemcpyAsync(c->hpin + kHpCtrl, c->W.ctrl + C_NCTRL, sizeof(double) * C_NCTRL, hipMemcpyDeviceToHost,
                            c->st));
        HIPC(hipStreamSynchronize(c->st));
        res = c->hpin + kHpCtrl;
        if ((int)res[C_EXIT] == EXIT_XWG) {
            if (!mc) {
                set_err("single-workgroup inner loop: exchange timed out");
                return -1;
            }
            if (xwg_snapshot(c, false)) return -1;
            if (!c->small_off)
                fprintf(stderr, "[lrsdp] one-workgroup-per-cone inner loop: the workgroups' exchange timed out; "
                                "this solve continues on the multi-launch iteration\n");
            c->small_off = true;
            c->xwg_fallbacks++;
            small = false;
            fell_back = true;
            res = c->hpin + kHpCtrl;
        } else {
            enq = std::max(0L, (long)res[C_INNER] - io.inner);
            c->dp.last_path = 4;
            if (c->stats) c->st_batches++;
        }
    }
    (void)fell_back;
    if (!c->prof && !small) {
        // Two batches in flight: batch k+1 is enqueued before the host waits for batch k, so
        // the GPU never idles on the host's submission or on the wait's wake-up.  Each batch
        // ends with a copy of the control block into its own pinned slot.  At the loop's exit
        // the batch still in flight runs as no-op iterations (the kernels' fast exits) and
        // leaves the state unchanged; later work on the stream is ordered after it.
        // Eager launches: the batch's last stage B writes the control block and a sequence
        // number into a pinned slot and the host spins on the number (no copy kernel, no
        // stream synchronisation).  Graph replay: a copy into the slot and an event.
        for (auto &e : c->bev)
            if (!e) HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        if (!c->hmir) {
            HIPC(hipHostMalloc((void **)&c->hmir, 128 * sizeof(double), hipHostMallocCoherent));
            HIPC(hipHostGetDevicePointer((void **)&c->dmir, c->hmir, 0));
            for (int q = 0; q < 128; ++q) c->hmir[q] = -1.0;
        }
        const bool mirror = !c->use_graphs;
        long k = 0, kw = 0;
        double bseq[2] = {0, 0};
        auto enqueue = [&](int Bk) -> int {
            if (c->use_graphs) {
                hipGraphExec_t ge;
                if (get_batch_graph(c, Bk, &ge)) return -1;
                HIPC(hipGraphLaunch(ge, c->st));
                HIPC(hipMemcpyAsync(c->hpin + kHpCtrl + 64 * (k & 1), c->W.ctrl + C_NCTRL, sizeof(double) * C_NCTRL,
                                    hipMemcpyDeviceToHost, c->st));
                HIPC(hipEventRecord(c->bev[k & 1], c->st));
            } else {
                bseq[k & 1] = (c->mseq += 1.0);
                for (int j = 0; j < Bk; ++j) {
                    a.hmirror = (j == Bk - 1) ? c->dmir + 64 * (k & 1) : nullptr;
                    a.seq = bseq[k & 1];
                    OPC(enqueue_alm_iteration(a, (int)((enq + j) & 1), c->st));   // parity runs across batches
                }
                a.hmirror = nullptr;
            }
            ++k;
            enq += Bk;
            if (c->stats) c->st_batches++;
            return 0;
        };
        // small fixed batches: the batch in flight at the exit bounds the no-op iterations,
        // and one batch of GPU work outlasts the host's submission of the next.  Eager batches
        // end exactly at the certain exit (the iteration parity runs on across batches);
        // captured graphs start at parity 0, so their lengths stay even.
        const int Bp = c->pipe_batch;
        auto next_b = [&]() -> int {
            const long left = std::max(1L, certain - enq);
            return c->use_graphs ? std::min(Bp, even_clamp(left)) : (int)std::min<long>(Bp, left);
        };
        if (enqueue(next_b())) return -1;
        for (;;) {
            if (enq < certain) {
                if (enqueue(next_b())) return -1;
            }
            if (mirror) {
                volatile double *slot = c->hmir + 64 * (kw & 1);
                const double t_w = now_s();
                long spins = 0;
                while (slot[C_NCTRL] != bseq[kw & 1]) {
                    if ((++spins & 0xFFFF) == 0) {
                        if (hipStreamQuery(c->st) == hipSuccess && slot[C_NCTRL] != bseq[kw & 1]) {
                            set_err("control mirror not written by the batch");
                            return -1;
                        }
                        if (now_s() - t_w > 600.0) { set_err("inner-loop batch timed out"); return -1; }
                    }
                }
                std::atomic_thread_fence(std::memory_order_acquire);
                for (int q = 0; q < C_NCTRL; ++q) c->hpin[kHpCtrl + 64 * (kw & 1) + q] = slot[q];
            } else {
                HIPC(hipEventSynchronize(c->bev[kw & 1]));
            }
            res = c->hpin + kHpCtrl + 64 * (kw & 1);
            ++kw;
            if (res[C_ACT2] == 0.0) break;
            if (kw == k) {   // still active past the certain exits (cannot happen): keep going
                if (enqueue(even_clamp(8))) return -1;
            }
        }
    }
    for (; c->prof;) {
        B = std::min(B, even_clamp(certain - enq));
        enq += B;
        if (c->prof) {
            // two iterations with events around each launch, then read the control
            B = 2;
            for (int j = 0; j < B; ++j) {
                a.ev = c->pev[j];
                OPC(enqueue_alm_iteration(a, j & 1, c->st));
            }
            a.ev = nullptr;
        } else if (c->use_graphs) {
            hipGraphExec_t ge;
            if (get_batch_graph(c, B, &ge)) return -1;
            HIPC(hipGraphLaunch(ge, c->st));
        } else {
            for (int j = 0; j < B; ++j) OPC(enqueue_alm_iteration(a, j & 1, c->st));
        }
        HIPC(hipMemcpyAsync(res, c->W.ctrl + C_NCTRL, sizeof(double) * C_NCTRL, hipMemcpyDeviceToHost, c->st));
        HIPC(hipStreamSynchronize(c->st));
        if (c->prof && res[C_ACT2] != 0.0) {
            for (int j = 0; j < 2; ++j)
                for (int q = 0; q < 4; ++q) {
                    float ms = 0;
                    HIPC(hipEventElapsedTime(&ms, c->pev[j][q], c->pev[j][q + 1]));
                    c->pacc[q] += ms;
                }
            c->pn += 2;
        }
        if (c->stats) c->st_batches++;
        if (res[C_ACT2] == 0.0) break;
        B = std::min(B * 2, 64);
    }
    c->inner_est = 0.7 * c->inner_est + 0.3 * (double)std::max(1L, (long)res[C_INNER] - io.inner);
    if (c->stats) {
        c->st_calls++;
        c->st_iters += (long)res[C_INNER] - io.inner;
        c->st_nop += enq - ((long)res[C_INNER] - io.inner);
        c->st_inner_s += now_s() - t_in;
    }
    if ((long)res[C_INNER] > io.inner) {
        // a later inner loop that stops before its first trip (budget) keeps this record
        c->last_trip[0] = res[C_LASTTAU]; c->last_trip[1] = res[C_LAG]; c->last_trip[2] = res[C_PINF1];
    }
    io.inner = (long)res[C_INNER]; io.local = (long)res[C_LOCAL]; io.clear = (long)res[C_CLEAR];
    io.rcval = res[C_RCVAL]; io.lag = res[C_LAG]; io.pinf1 = res[C_PINF1]; io.pinfinf = res[C_PINFINF];
    io.exitReason = (int)res[C_EXIT2];
    memcpy(c->last_ctl, res, sizeof(double) * C_NCTRL);
    // the iterate lives in R2 after an odd number of completed iterations
    if (res[C_RCUR] != 0.0)
        HIPC(hipMemcpyAsync(c->W.R, c->W.R2, sizeof(double) * c->dp.NRpad, hipMemcpyDeviceToDevice, c->st));
    c->head = (int)res[C_HEAD]; c->gcur = (int)res[C_GCUR];
    c->beta[0] = res[C_BETA0]; c->beta[1] = res[C_BETA1]; c->yy[0] = res[C_YY0]; c->yy[1] = res[C_YY1];
    return 0;
}

// ---- inner loop for lbfgsListLength != 2 (the fused kernels keep two pairs in coefficient
// space).  The reference's own step sequence (lorads_alm.c:1302-1379) with the host in control
// and device operators per step: LBFGSDirection's two-loop over the ring of L pairs
// (lorads_alm.c:468-505, device dot / axpy), LBFGSDirectionUseGrad (:607-627), ALMCalq12p12
// (:714-734), ALMLineSearch (:266-333, the device line search), SetyAsNegGrad (:768-783),
// ALMupdateVar (:826-830), the A(X) update (:1351-1353), ALMCalGrad (:74-87), setlbfgsHisTwo
// (:842-863), updateDimacsALM (lorads_alg_common.c:424-428) and the exits of :1359-1379.  The
// ring is L device vectors pairs (lrs_ctx::ring_s / ring_y); about a dozen host reads per trip,
// so this path is for the option's semantics, not for speed.
static int ring_alloc(lrs_ctx *c, int L) {
    if ((int)c->ring_s.size() == L && c->ring_len == c->dp.NRpad) return 0;
    HIPC(hipStreamSynchronize(c->st));
    for (double *q : c->ring_s) if (q) (void)hipFree(q);
    for (double *q : c->ring_y) if (q) (void)hipFree(q);
    c->ring_s.assign(L, nullptr);
    c->ring_y.assign(L, nullptr);
    for (int q = 0; q < L; ++q) {
        HIPC(hipMalloc((void **)&c->ring_s[q], sizeof(double) * std::max(2L, c->dp.NRpad)));
        HIPC(hipMalloc((void **)&c->ring_y[q], sizeof(double) * std::max(2L, c->dp.NRpad)));
        HIPC(hipMemsetAsync(c->ring_s[q], 0, sizeof(double) * std::max(2L, c->dp.NRpad), c->st));
        HIPC(hipMemsetAsync(c->ring_y[q], 0, sizeof(double) * std::max(2L, c->dp.NRpad), c->st));
    }
    c->ring_beta.assign(L, 0.0);
    c->ring_len = c->dp.NRpad;
    c->head = 0;
    return 0;
}

// q1 = 2 A(sym R D^T), q2 = A(D D^T) into W.q1 / W.q2 and the device line search's finals;
// p1 (before its factor 2) and p2 returned
static int op_q12_fin(lrs_ctx *c, double *p1h, double *p2h) {
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    double a = 0, b = 0;
    for (int k = 0; k < P.K; ++k) {
        OPC(launch_sddmm(P, k, 2, W.R, W.D, W.uvt0, W.uvt1, W.part, 0, nullptr, c->st));
        double t[2];
        if (read_tmpfin(c, TF_SD + 2 * k, 2, t)) return -1;
        a += t[0]; b += t[1];
        const DevCone &dc = P.cones[k];
        if (dc.dense_c) {   // <C, sym R D^T> = <R, C D>, <C, D D^T> = <D, C D>
            OPC(launch_dense_cx(P, k, W.D, W.CD, 0.0, c->st));
            double u, v;
            const long ro = dc.foff + (long)dc.row0 * dc.ld;   // sharded: the owned rows
            if (op_dot(c, (long)dc.nown * dc.ld, W.R + ro, W.CD + ro, &u)) return -1;
            if (op_dot(c, (long)dc.nown * dc.ld, W.D + ro, W.CD + ro, &v)) return -1;
            a += u; b += v;
        }
    }
    OPC(launch_gather(P, W.uvt0, 2.0, W.q1, nullptr, nullptr, c->st, nullptr));
    OPC(launch_gather(P, W.uvt1, 1.0, W.q2, nullptr, nullptr, c->st, nullptr));
    double *fin = c->s_fin;   // this context's finals (the line search reads them)
    double h[64] = {0};
    h[0] = a; h[1] = b;
    HIPC(h2d_sync(c, fin, h, sizeof(double) * 2 * std::max(1, std::min(P.K, 32))));
    *p1h = a; *p2h = b;
    return 0;
}

static int run_inner_generic(lrs_ctx *c, const lrs_params *p, double rho, double rctol, double gap, long budget,
                             InnerIo &io, bool ph1_exit = true) {
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    const int L = p->lbfgsListLength;
    if (sharded(c)) { set_err("lbfgsListLength %d: not supported in a sharded solve", L); return -1; }   // (solve_impl refuses first)
    if (ring_alloc(c, L)) return -1;
    const long NR = P.NRpad;
    double par[P_NPAR] = {0};
    par[P_RHO] = rho; par[P_ENDTAU] = p->endTauTol;
    HIPC(h2d_sync(c, W.par, par, sizeof(par)));
    const double phase1 = ph1_exit ? p->phase1Tol : -1.0;
    int exitr = EXIT_NONE;
    for (;;) {
        // loop head (lorads_alm.c:1302) and the budget (benchmarking)
        if (!(io.rcval - rctol > p->endALMSubTol)) { exitr = EXIT_CONVERGED; break; }
        if (budget > 0 && io.inner >= budget) { exitr = EXIT_BUDGET; break; }
        if (io.local % 300 == 0) io.clear = 0;
        const int nodeNum = io.clear <= L - 1 ? (int)io.clear : L;
        double *G = W.G[c->gcur];
        // LBFGSDirection: Dtemp = G; newest -> oldest alpha_i = beta_i <s_i, Dtemp>, Dtemp -= alpha_i y_i;
        // oldest -> newest Dtemp += (alpha_i - beta_i <y_i, Dtemp>) s_i; D = -Dtemp
        HIPC(hipMemcpyAsync(W.D, G, sizeof(double) * NR, hipMemcpyDeviceToDevice, c->st));
        std::vector<double> alpha(L, 0.0);
        int node = (c->head - 1 + L) % L;
        for (int t = 0; t < nodeNum; ++t) {
            double v;
            if (op_dot(c, NR, c->ring_s[node], W.D, &v)) return -1;
            alpha[node] = c->ring_beta[node] * v;
            OPC(launch_axpby(NR, -alpha[node], c->ring_y[node], 1.0, W.D, c->st));
            node = (node - 1 + L) % L;
        }
        node = (node + 1) % L;
        for (int t = 0; t < nodeNum; ++t) {
            double v;
            if (op_dot(c, NR, c->ring_y[node], W.D, &v)) return -1;
            OPC(launch_axpby(NR, alpha[node] - c->ring_beta[node] * v, c->ring_s[node], 1.0, W.D, c->st));
            node = (node + 1) % L;
        }
        OPC(launch_axpby(NR, 0.0, W.D, -1.0, W.D, c->st));
        double dg;
        if (op_dot(c, NR, W.D, G, &dg)) return -1;
        if (dg >= 0) OPC(launch_axpby(NR, -1.0, G, 0.0, W.D, c->st));   // LBFGSDirectionUseGrad
        // q1, q2, p1, p2 and the line search
        double p1, p2;
        if (op_q12_fin(c, &p1, &p2)) return -1;
        OPC(launch_ls_only(P, W, c->st));
        double ls[LS_N];
        HIPC(hipMemcpyAsync(c->hpin + kHpLs, W.lsres, sizeof(ls), hipMemcpyDeviceToHost, c->st));
        HIPC(hipStreamSynchronize(c->st));
        memcpy(ls, c->hpin + kHpLs, sizeof(ls));
        const double tau = ls[LS_TAU];
        if (ls[LS_ROOTNUM] == 0) { exitr = EXIT_NUMERR; break; }
        if (std::fabs(tau) < p->endTauTol) {
            io.inner++; io.local++; io.clear++;
            exitr = EXIT_TINYTAU;
            break;
        }
        // SetyAsNegGrad, ALMupdateVar, A(X) += tau q1 + tau^2 q2
        double *ys = c->ring_y[c->head], *ss = c->ring_s[c->head];
        OPC(launch_axpby(NR, -1.0, G, 0.0, ys, c->st));
        OPC(launch_axpby(NR, tau, W.D, 1.0, W.R, c->st));
        OPC(launch_axpby(P.m, tau, W.q1, 1.0, W.cvs, c->st));
        OPC(launch_axpby(P.m, tau * tau, W.q2, 1.0, W.cvs, c->st));
        // ALMCalGrad into the other gradient buffer
        c->gcur ^= 1;
        double lag;
        if (op_grad(c, rho, &lag)) return -1;
        // setlbfgsHisTwo: s = tau D, y += G_new, beta = 1 / <y, s>, head advances
        OPC(launch_axpby(NR, tau, W.D, 0.0, ss, c->st));
        OPC(launch_axpby(NR, 1.0, W.G[c->gcur], 1.0, ys, c->st));
        double ysd;
        if (op_dot(c, NR, ys, ss, &ysd)) return -1;
        c->ring_beta[c->head] = 1.0 / ysd;
        c->head = (c->head + 1) % L;
        // updateDimacsALM (A(RR^T) afresh, the residual) and the exits of lorads_alm.c:1359-1379
        double pinf;
        if (op_constr_xx(c, W.R, nullptr, &pinf, nullptr)) return -1;
        io.inner++; io.local++; io.clear++;
        io.lag = lag;
        io.pinf1 = pinf;
        io.pinfinf = pinf * (1 + c->hp.bNrm1) / (1 + c->hp.bNrmInf);
        c->last_trip[0] = tau; c->last_trip[1] = lag; c->last_trip[2] = pinf;
        if (io.pinfinf <= phase1 && (gap <= phase1 || !p->highAccMode)) { exitr = EXIT_PHASE1; break; }
        io.rcval = std::sqrt(lag) / (1 + c->hp.cNrmInf);
        if (io.local > 800) { exitr = EXIT_LOCAL800; break; }
    }
    io.exitReason = exitr;
    // the newest pair also in (S0, Y0) for the C-ABI readers (lrs_alm_last_step)
    const int hn = (c->head - 1 + L) % L;
    HIPC(hipMemcpyAsync(W.ls[0], c->ring_s[hn], sizeof(double) * NR, hipMemcpyDeviceToDevice, c->st));
    HIPC(hipMemcpyAsync(W.ly[0], c->ring_y[hn], sizeof(double) * NR, hipMemcpyDeviceToDevice, c->st));
    return 0;
}

static void alm_log(lrs_ctx *c, const lrs_params *p, const AlmState &st, double t) {
    int cur = c->t1c.empty() ? sum_rank(c) : c->t1c.back();
    int orc = c->t1o.empty() ? cur : c->t1o.back();
    logf_(c, p, "ALM OuterIter:%ld InnerIter:%ld pObj:%5.5e dObj:%5.5e pInfea(1):%5.5e pInfea(Inf):%5.5e pdGap:%5.5e "
           "rho:%3.2f CurrRank:%d OracleRank:%d Time:%3.2f\n",
           st.outerIter, st.innerIter, st.pobj, st.dobj, st.pinf1, st.pinfinf, st.gap, st.rho, cur, orc, t);
}

// LORADS_ALMOptimize, lorads_alm.c:1220-1484
static int alm_optimize_body(lrs_ctx *c, const lrs_params *p, AlmState &st, double tss);
static int alm_optimize(lrs_ctx *c, const lrs_params *p, AlmState &st, double tss) {
    c->st_calls = c->st_batches = c->st_iters = c->st_nop = 0;
    c->st_inner_s = 0;
    const double t0 = now_s();
    const int rc = alm_optimize_body(c, p, st, tss);
    if (c->stats)
        fprintf(stderr, "[lrs stats] alm %.3f ms: run_inner calls %ld, batches %ld, iterations %ld, "
                "no-op iterations %ld, in batches %.3f ms, host outside %.3f ms, outer %ld\n",
                (now_s() - t0) * 1e3, c->st_calls, c->st_batches, c->st_iters, c->st_nop, c->st_inner_s * 1e3,
                (now_s() - t0 - c->st_inner_s) * 1e3, st.outerIter);
    return rc;
}
static int alm_optimize_body(lrs_ctx *c, const lrs_params *p, AlmState &st, double tss) {
    const double ori = now_s();
    c->max_sub = 5000;   // lorads_alm.c:1222
    int is_rank_max = check_all_rank_max(c, 1.0);
    int retcode = 0, last_outer_start = 1, sched_pos = 0;
    double rc, rc_tol, rc_val = 0, lag = 0;
    char difficulty;
    long localIter = 0, clearL = 0;
    int rank_flag = 0, rho_factor_flag = 0, upd_cnt = 0;
    double rank_update_factor, rho_update_factor, thres = 15;
    const int max_inc = 10000, max_ceil = 25000;
    const bool sched = p->rankSchedule && p->rankScheduleLen > 0 && p->fixedRank <= 0;
    if (sched && p->rankScheduleLen <= 1) is_rank_max = 1;
    long budget = p->almInnerBudget;
ALG_START:
    upd_cnt = 0;
    rc = 0.1;
    rc_tol = rc / st.rho;
    if (op_constr_xx(c, c->W.R, nullptr, nullptr, nullptr)) return -1;
    if (op_grad(c, st.rho, &lag)) return -1;
    rc_val = std::sqrt(lag) / (1 + c->hp.cNrmInf);
    difficulty = 'h';
    localIter = 0; clearL = 0; rank_flag = 0;
    rank_update_factor = p->rankUpdateFactor;
    rho_update_factor = p->ALMRhoFactor;
    rho_factor_flag = 0;
    if (p->dyrankLevel == 0) thres = 1e8;
    else if (p->dyrankLevel == 1) thres = 150;
    else if (p->dyrankLevel == 2) thres = 15;
    else if (p->dyrankLevel == 3) thres = 5;
    if (sched && p->nearStallFactor > 0) thres = std::max(1.0, thres * p->nearStallFactor);
    for (long k = st.outerIter; k <= p->maxALMIter; k++) {
        double ema_cur = 0, ema_old = 0;
        int ema_cnt = 1;
        long cur_iter_counter = 1;
        if (upd_cnt >= 2) { upd_cnt = 0; c->max_sub = std::min(c->max_sub + max_inc, max_ceil); }
        while (difficulty != 'e') {
            localIter = 0;
            int if_break = update_check_ema(&ema_cur, &ema_old, rc_val, 0.1, 0.005, 5, &ema_cnt);
            if (!if_break && !p->highAccMode) break;
            if (cur_iter_counter >= c->max_sub) { upd_cnt += 1; break; }
            if (rank_flag >= thres && !is_rank_max && (k - last_outer_start >= 3)) break;
            if (rc_val <= rc_tol) break;
            // ---- inner L-BFGS loop on the device (lorads_alm.c:1302-1379)
            InnerIo io;
            io.inner = st.innerIter; io.local = localIter; io.clear = clearL; io.rcval = rc_val; io.lag = lag;
            io.pinf1 = st.pinf1; io.pinfinf = st.pinfinf;
            for (;;) {
                const long before = st.innerIter;
                if (p->lbfgsListLength != 2 ? run_inner_generic(c, p, st.rho, rc_tol, st.gap, budget, io)
                                           : run_inner(c, p, st.rho, rc_tol, st.gap, budget, io))
                    return -1;
                st.innerIter = io.inner; localIter = io.local; clearL = io.clear;
                cur_iter_counter += io.inner - before;
                rc_val = io.rcval; lag = io.lag; st.pinf1 = io.pinf1; st.pinfinf = io.pinfinf;
                if (io.exitReason != EXIT_BUDGET || !c->bhook) break;
                // benchmark hook: a larger budget continues this inner loop where it stopped
                HIPC(hipStreamSynchronize(c->st));
                const long nb = c->bhook(c->buser, st.innerIter);
                if (nb <= st.innerIter) break;
                budget = nb;
                io.resume = true;
            }
            if (io.exitReason == EXIT_PHASE1) { st.outerIter = k; goto END_ALM; }
            if (io.exitReason == EXIT_NUMERR) { retcode = 4; goto END_ALM; }
            if (io.exitReason == EXIT_BUDGET) goto PRINT_AND_EXIT;
            if (io.exitReason == EXIT_TINYTAU) {
                if (p->verbose) printf("update rho since tau is too small.\n");
                goto UpdateRho;
            }
            // LORADSUpdateDualVar (lorads_alg_common.c:511) + gradient
            OPC(launch_dual_update(c->dp, st.rho, c->W.lam, c->W.cvs, c->st));
            if (op_grad(c, st.rho, &lag)) return -1;
            rc_val = std::sqrt(lag) / (1 + c->hp.cNrmInf);
            if (localIter <= 20) difficulty = 'e';
            else if (localIter <= 100) { difficulty = 'm'; rank_flag += 2; }
            else if (localIter < 400) { difficulty = 'h'; rank_flag += 3; }
            else { difficulty = 's'; rank_flag += 4; }
            if (difficulty == 'e') rank_flag = 0;
        }
    UpdateRho:
        do {
            st.rho *= rho_update_factor;
            if (op_grad(c, st.rho, &lag)) return -1;
            rc_val = std::sqrt(lag) / (1 + c->hp.cNrmInf);
            rc_tol = rc / st.rho;
        } while (rc_tol >= rc_val);
        if (st.rho >= 5e4 && rho_factor_flag < 4) { rho_update_factor = std::sqrt(std::sqrt(rho_update_factor)); rho_factor_flag = 4; }
        else if (st.rho >= 5e6 && rho_factor_flag < 6) { rho_update_factor = std::sqrt(std::sqrt(rho_update_factor)); rho_factor_flag = 6; }
        else if (st.rho >= 5e8 && rho_factor_flag < 8) { rho_update_factor = std::sqrt(std::sqrt(rho_update_factor)); rho_factor_flag = 8; }
        difficulty = 'h';
        clearL = 0;
        st.outerIter = k;
        {
            if ((st.pinfinf <= p->phase1Tol) && ((st.gap <= p->phase1Tol) || !p->highAccMode)) goto END_ALM;
            double pinf, obj;
            if (op_constr_xx(c, c->W.R, nullptr, &pinf, &obj)) return -1;
            c->pObjVal = obj / c->scaleObjHis;
            cal_dual_obj(c);
            c->dimPinf = pinf;
            c->dimGap = std::fabs(c->pObjVal - c->dObjVal) / (1 + std::fabs(c->pObjVal) + std::fabs(c->dObjVal));
            st.gap = c->dimGap; st.pobj = c->pObjVal; st.dobj = c->dObjVal;
            st.pinf1 = c->dimPinf;
            st.pinfinf = st.pinf1 * (1 + c->hp.bNrm1) / (1 + c->hp.bNrmInf);
            if (st.gap <= p->phase1Tol * 1e-3 && st.pinf1 <= p->phase1Tol * 1e-3) goto PRINT_AND_EXIT;
            record_state(c, p, 1);
            alm_log(c, p, st, now_s() - ori);
            double tout = now_s() - tss >= p->timeSecLimit ? 1.0 : 0.0;
            if (sharded(c) && c->comm->allreduce_host(c, &tout, 1)) return -1;   // every shard stops together
            if (tout > 0) goto PRINT_AND_EXIT;
        }
        if (rank_flag >= thres && !is_rank_max) {
            rank_flag = 0;
            if (k - last_outer_start >= 2) {
                if (p->verbose) printf("increase the rank, factor:%f.\n", rank_update_factor);
                if (aug_rank(c, rank_update_factor, p, &sched_pos, &is_rank_max)) return -1;
                st.outerIter = k;
                last_outer_start = (int)st.outerIter;
                goto ALG_START;
            }
        }
    }
END_ALM: {
        double pinf, obj;
        if (op_constr_xx(c, c->W.R, nullptr, &pinf, &obj)) return -1;
        c->pObjVal = obj / c->scaleObjHis;
        cal_dual_obj(c);
        c->dimPinf = pinf;
        c->dimGap = std::fabs(c->pObjVal - c->dObjVal) / (1 + std::fabs(c->pObjVal) + std::fabs(c->dObjVal));
        st.pobj = c->pObjVal; st.dobj = c->dObjVal; st.gap = c->dimGap;
        st.pinf1 = c->dimPinf;
        st.pinfinf = st.pinf1 * (1 + c->hp.bNrm1) / (1 + c->hp.bNrmInf);
    }
PRINT_AND_EXIT:
    logf_(c, p, "-----------------------------------------------------------------------\nExit ALM:\n");
    record_state(c, p, 1);
    alm_log(c, p, st, now_s() - ori);
    return retcode;
}

// ------------------------------------------------------------------------
// ADMM phase (lorads_admm.c), host-driven CG on device operators
// ------------------------------------------------------------------------
// x -> x + A^*(A(sym(x Y^T))) Y for cone k (linSysProduct, lorads_admm.c:471-486)
static int lin_sys_product(lrs_ctx *c, int k, const double *Y, const double *x, double *res) {
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    // A(sym(x Y^T)) over cone k's constraint entries only (LORADSUpdateConstrValCG)
    OPC(launch_auv_con(P, k, 0, x, Y, 1.0, 0, W.wtmp, nullptr, nullptr, c->st));
    OPC(launch_wsum(P, W.wtmp, 0, W.S, c->st));
    OPC(launch_spmm(P, k, W.S, Y, 1.0, x, 1.0, res, nullptr, 0, nullptr, c->st));
    return 0;
}

// CGSolve (linalg/lorads_cgs.c:128-287) on the device: initial residual, then batches of
// iterations (4 launches each; the restart every 20 iterations adds 4) with all scalars
// in W.cgc; one poll per batch.  Sharded: the vectors are the owned rows, and each
// reduction (||b||_1, <p, Q>, <r, r>) is folded and summed over the shards in the stream
// (ncclAllReduce of one double) before the kernel that consumes it, which then reads the
// total as its only partial -- the "CG dot-products" all-reduce of SURVEY.md §8(e).  The
// matvec needs no halo: an owned constraint's entries lie in owned rows.
static int cg_solve(lrs_ctx *c, int k, const double *Y, double *X, const double *b, double tol, int maxit) {
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    const DevCone &d = P.cones[k];
    const long o = d.foff + (long)d.row0 * d.ld;
    const long nr = (long)d.nown * d.ld;
    double *r = W.cg_r + o, *p = W.cg_p + o, *Q = W.cg_Q + o;
    double *xk = X + o;
    const double *bk = b + o;
    double *cgc = W.cgc;
    const bool sh = sharded(c);
    double *tot = W.tot + 26;   // sharded: the summed scalar the next kernel reads
    // a reduction's partials -> what its consumer reads (sharded: folded, summed over shards)
    auto sum = [&](double *part, int &nblk) -> int {
        if (!sh) return 0;
        OPC(launch_fold1(part, nblk, tot, c->st));
        if (c->comm->allreduce_dev(c, tot, 1, c->st)) return -1;
        nblk = 1;
        return 0;
    };
    double *pA = sh ? tot : W.part, *pB = sh ? tot : W.partB, *pC = sh ? tot : W.partC;
    int nA = 0, nB = 0, nC = 0, nR = 0;
    // shared constraints: entries on owned slots with a halo endpoint read the halo rows of
    // the CG direction (exchanged before every matvec), and A(.)'s holders' partial sums meet
    // in the shared all-reduce
    const bool shx = sh && P.nsh > 0;
    auto auv = [&](const double *x, const double *guard) -> int {
        if (shx && c->comm->halo(c, const_cast<double *>(x), c->st)) return -1;
        OPC(launch_auv_con(P, k, 0, x, Y, 1.0, 0, W.wtmp, nullptr, nullptr, c->st, guard));
        OPC(sync_shared(P, W.wtmp, c->st));
        return 0;
    };
    OPC(launch_cg_nrm1(nr, bk, W.part, c->st, &nA));
    if (sum(W.part, nA)) return -1;
    if (auv(X, nullptr)) return -1;
    OPC(launch_cg_mv(P, k, W.wtmp, Y, X, W.cg_Q, nullptr, cgc, 0, c->st, &nB));
    OPC(launch_cg_resid(nr, bk, Q, r, p, W.partC, cgc, pA, nA, 1, c->st, &nC));
    if (sum(W.partC, nC)) return -1;
    OPC(launch_cg_resid2(nr, r, p, pC, nC, cgc, tol, 0, 1, c->st));
    double *h = c->hpin + kHpCg;
    // first batch sized from this cone's previous solve (ADMM's CG solves take a handful of
    // iterations each; the batch past convergence runs guarded no-op launches), then doubling
    const long prev = c->cgIterCone[k];
    int it = 0, B = prev > 0 ? (int)std::max(2L, std::min(8L, prev + c->cg_slack)) : 8;
    while (it < maxit) {
        for (int j = 0; j < B && it < maxit; ++j, ++it) {
            const int par = it & 1;
            if (auv(W.cg_p, cgc)) return -1;
            OPC(launch_cg_mv(P, k, W.wtmp, Y, W.cg_p, W.cg_Q, W.partB, cgc, 1, c->st, &nB));
            if (sum(W.partB, nB)) return -1;
            OPC(launch_cg_upd(nr, xk, r, p, Q, pB, nB, W.partC, cgc, par, it, c->st, &nC));
            if (sum(W.partC, nC)) return -1;
            const int restart = (it % 20 == 0);
            OPC(launch_cg_conv(nr, r, p, pC, nC, cgc, tol, par, restart, c->st));
            if (restart) {
                if (auv(X, cgc)) return -1;
                OPC(launch_cg_mv(P, k, W.wtmp, Y, X, W.cg_Q, nullptr, cgc, 1, c->st, &nB));
                OPC(launch_cg_resid(nr, bk, Q, r, p, W.partC, cgc, nullptr, 0, 0, c->st, &nR));
                if (sum(W.partC, nR)) return -1;
                OPC(launch_cg_resid2(nr, r, p, pC, nR, cgc, tol, par, 0, c->st));
            }
        }
        HIPC(hipMemcpyAsync(h, cgc, sizeof(double) * CG_N, hipMemcpyDeviceToHost, c->st));
        HIPC(hipStreamSynchronize(c->st));
        if (h[CG_ACTIVE] == 0.0) break;
        B = std::min(2 * B, 64);
    }
    c->cgIterCone[k] = (long)h[CG_ITERS];
    // sharded: the solved factor's halo rows from their owners (the next half-step's RHS and
    // the objective read them)
    if (sh && c->comm->halo(c, X, c->st)) return -1;
    return 0;
}

// LORADSUpdateSDPVarOne (lorads_admm.c:564-616): solve for X with Y fixed
static int update_var_one(lrs_ctx *c, int k, double *X, const double *Y, double rho, double tol, int maxit) {
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    const DevCone &d = P.cones[k];
    OPC(launch_admm_m1(P.m, rho, P.b, W.cvs, W.cvc + (long)k * P.m, W.lam, W.M1, c->st));
    OPC(launch_wsum(P, W.M1, 1, W.S, c->st));
    OPC(launch_spmm(P, k, W.S, Y, 1.0, Y, -rho, W.M2, nullptr, 0, nullptr, c->st));   // M2 = S Y - rho Y
    OPC(launch_dense_cx(P, k, Y, W.M2, 1.0, c->st));                                     // + C Y (dense objective)
    OPC(launch_axpby((long)d.n * d.ld, -1.0 / rho, W.M2 + d.foff, 0.0, W.cg_b + d.foff, c->st));
    if (cg_solve(c, k, Y, X, W.cg_b, tol, maxit)) return -1;
    c->cgIterTotal += c->cgIterCone[k];
    return 0;
}

static int refresh_cone(lrs_ctx *c, int k) {   // lorads_alg_common.c:310-314
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    double *cv = W.cvc + (long)k * P.m;
    // cvs = (cvs - cvc[k]) + A_k(U V^T) in the pass that rewrites cvc[k] (the same two
    // roundings as the reference's two axpys)
    if (P.nsh > 0) {
        // sharded, shared constraints: the holders' sums of A_k(U V^T) meet first, then the two
        // axpys of the reference (cvs - cvc_old, + cvc_new)
        OPC(launch_axpby(P.m, -1.0, cv, 1.0, W.cvs, c->st));
        OPC(launch_auv_con(P, k, 0, W.U, W.V, 1.0, 0, cv, nullptr, nullptr, c->st, nullptr));
        OPC(sync_shared(P, cv, c->st));
        OPC(launch_axpby(P.m, 1.0, cv, 1.0, W.cvs, c->st));
        return 0;
    }
    OPC(launch_auv_con(P, k, 0, W.U, W.V, 1.0, 0, cv, nullptr, nullptr, c->st, nullptr, W.cvs));
    return 0;
}

// LORADSInitConstrValAll + LORADSInitConstrValSum (lorads_alg_common.c:104-229) on (U, V):
// per-cone A_k(sym UV^T) into cvc[k] and their sum into cvs
static int admm_init_constr(lrs_ctx *c) {
    DevProblem &P = c->dp;
    OPC(launch_fill(P.m, 0.0, c->W.cvs, c->st));
    for (int k = 0; k < P.K; ++k) {
        OPC(launch_auv_con(P, k, 0, c->W.U, c->W.V, 1.0, 0, c->W.cvc + (long)k * P.m, nullptr, nullptr, c->st));
        OPC(sync_shared(P, c->W.cvc + (long)k * P.m, c->st));
        OPC(launch_axpby(P.m, 1.0, c->W.cvc + (long)k * P.m, 1.0, c->W.cvs, c->st));
    }
    return 0;
}

// One half-step of LORADSUpdateSDPVar (lorads_alg_common.c:298-326) for cone k: side 0 solves U
// with V fixed, 1 V with U fixed, then the cone's constraint refresh.  Small unsharded cones take
// the single-workgroup kernel (lrs_kernels.hip k_small_cg: RHS, CG and refresh in one launch, its
// iterations counted on the device in W.cgc[CG_TOTAL]); LRS_SMALL_CG=0 keeps the multi-launch CG.
static bool use_small_cg(lrs_ctx *c, int k) {
    const char *e = getenv("LRS_SMALL_CG");
    const int env = e ? atoi(e) : -1;
    return env != 0 && !is_lp(c, k) && c->dp.lp_cone < 0 && small_cg_fits(c->dp, k);
}
static int admm_half_step(lrs_ctx *c, int k, int side, double rho, double tol, int maxit, bool *on_device) {
    if (use_small_cg(c, k)) {
        OPC(launch_small_cg(c->dp, c->W, k, side, rho, tol, maxit, c->st));
        *on_device = true;
        return 0;
    }
    *on_device = false;
    if (update_var_one(c, k, side ? c->W.V : c->W.U, side ? c->W.U : c->W.V, rho, tol, maxit)) return -1;
    return refresh_cone(c, k);
}

static int admm_update_var(lrs_ctx *c, double rho, double tol, int maxit) {
    bool dev = false;
    // cones with no constraint in common: the sweep's half-steps of one side side by side
    // (LRS_SMALL_CG_BATCH=0: one launch a cone)
    const char *eb = getenv("LRS_SMALL_CG_BATCH");
    const bool batch = !(eb && eb[0] == '0') && use_small_cg(c, 0) && small_cg_batch_fits(c->dp);
    for (int side = 0; side < 2 && batch; ++side) OPC(launch_small_cg_batch(c->dp, c->W, side, rho, tol, maxit, c->st));
    dev = batch;
    for (int k = 0; k < c->dp.K && !batch; ++k)
        for (int side = 0; side < 2 && !is_lp(c, k); ++side) {
            bool d = false;
            if (admm_half_step(c, k, side, rho, tol, maxit, &d)) return -1;
            dev |= d;
        }
    // the LP block after every SDP cone (LORADSUpdateSDPLPVar, lorads_alg_common.c:352-372)
    if (c->dp.lp_cone >= 0) OPC(launch_lp_admm(c->dp, c->W, rho, c->st));
    // the device-counted CG iterations, read behind the next stream sync (admm_eval's)
    if (dev)
        HIPC(hipMemcpyAsync(c->hpin + kHpCgTotal, c->W.cgc + CG_TOTAL, sizeof(double), hipMemcpyDeviceToHost, c->st));
    c->cg_dev_total = dev;
    return 0;
}

static int update_dimacs_admm(lrs_ctx *c) {   // lorads_alg_common.c:454-462
    OPC(launch_avg(c->dp.NRpad, c->W.U, c->W.V, c->W.R, c->st));
    return update_dimacs(c, c->W.R, nullptr, false);
}
// LORADSCalObjUV_ADMM (lorads_admm.c:398-410) + cal_dual_obj + update_dimacs_admm (lorads_admm.c:155-157) in one pass: the
// objective <C, R R^T> of R = (U + V) / 2 comes out of the same SDDMM as A(R R^T), so the
// three evaluations share one set of launches and one host read
static int admm_eval(lrs_ctx *c) {
    double pinf, obj, blam;
    // small cones (the single-workgroup half-steps' lists): R, A(R R^T), the residual, the
    // objective and b^T lambda in one launch, the cones' partials added here in cone order
    // (LRS_SMALL_EVAL=0: the operator launches below)
    const char *ev = getenv("LRS_SMALL_EVAL");
    if (!(ev && ev[0] == '0') && use_small_cg(c, 0) && small_eval_fits(c->dp)) {
        const int K = c->dp.K;
        OPC(launch_small_eval(c->dp, c->W, c->W.U, c->W.V, c->W.tot, c->st));
        HIPC(hipMemcpyAsync(c->hpin + kHpRead, c->W.tot, sizeof(double) * 4 * K, hipMemcpyDeviceToHost, c->st));
        HIPC(hipStreamSynchronize(c->st));
        double r2 = 0.0;
        obj = 0.0;
        blam = 0.0;
        for (int k = 0; k < K; ++k) {
            r2 += c->hpin[kHpRead + 4 * k];
            obj += c->hpin[kHpRead + 4 * k + 1];
            blam += c->hpin[kHpRead + 4 * k + 2];
        }
        pinf = std::sqrt(r2) / (1 + c->hp.bNrm1);
    } else {
        OPC(launch_avg(c->dp.NRpad, c->W.U, c->W.V, c->W.R, c->st));
        if (op_constr_xx(c, c->W.R, nullptr, &pinf, &obj, &blam)) return -1;
    }
    c->pObjVal = obj / c->scaleObjHis;
    c->dObjVal = blam / c->scaleObjHis;
    c->dimPinf = pinf;
    const double gap = c->pObjVal - c->dObjVal;
    c->dimGap = std::fabs(gap) / (1 + std::fabs(c->pObjVal) + std::fabs(c->dObjVal));
    return 0;
}

static void admm_log(lrs_ctx *c, const lrs_params *p, const AdmmState &st, double t) {
    logf_(c, p, "ADMM Iter:%ld pObj:%5.5e dObj:%5.5e pInfea(1):%5.5e pInfea(Inf):%5.5e pdGap:%5.5e rho:%3.2f cgIter:%d "
           "CurrRank:%d OracleRank:%d Time:%3.2f\n",
           st.iter, st.pobj, st.dobj, st.pinf1, st.pinfinf, st.gap, st.rho,
           (int)((double)st.cg_iter / (double)std::max(1, n_sdp(c))), c->t2c.empty() ? 0 : c->t2c.back(),
           c->t2o.empty() ? 0 : c->t2o.back(), t);
}

// LORADSADMMOptimize (lorads_admm.c:84-209); reopt = LORADSADMMOptimize_reopt (:222-363):
// CG tolerance 1e-4 pinf, bad-gap budget 200, exit on l_1 pinf only with the gap met,
// rho schedule on iter instead of iter + 1.
static int admm_optimize(lrs_ctx *c, lrs_params *p, AdmmState &st, long ceiling, double tss, bool reopt = false) {
    if (st.gap <= p->phase2Tol && st.pinf1 <= p->phase2Tol) return 0;
    const int maxCG = 800;
    const double orig = now_s();
    st.rho = std::min(st.rho, p->rhoMax);
    c->cgIterTotal = 0;
    HIPC(hipMemsetAsync(c->W.cgc + CG_TOTAL, 0, sizeof(double), c->st));
    if (admm_init_constr(c)) return -1;
    if (admm_eval(c)) return -1;
    st.pobj = c->pObjVal; st.dobj = c->dObjVal; st.gap = c->dimGap; st.pinf1 = c->dimPinf;
    st.pinfinf = st.pinf1 * (1 + c->hp.bNrm1) / (1 + c->hp.bNrmInf);
    double cur_rho_max = p->rhoMax, old_mean = 1e30, buf[10] = {0};
    int bad_pd = 0, count = 0;
    while (st.iter <= p->maxADMMIter || st.gap >= p->phase2Tol || st.pinf1 >= p->phase2Tol) {
        if (st.iter >= ceiling) {
            if (reopt) record_state(c, p, 2);
            break;
        }
        const double cgtol = std::min(st.pinf1 * (reopt ? 1e-4 : 1e-2), 1e-8);
        if (admm_update_var(c, st.rho, cgtol, maxCG)) return -1;
        if (admm_eval(c)) return -1;
        st.cg_iter = c->cgIterTotal + (c->cg_dev_total ? (long)c->hpin[kHpCgTotal] : 0);
        st.pobj = c->pObjVal; st.dobj = c->dObjVal; st.pinf1 = c->dimPinf;
        st.pinfinf = st.pinf1 * (1 + c->hp.bNrm1) / (1 + c->hp.bNrmInf);
        st.gap = c->dimGap;
        record_state(c, p, 2);
        admm_log(c, p, st, now_s() - orig);
        if (st.pinfinf >= 1e10 || st.gap >= 1 - 1e-8) return 4;
        if (st.gap <= p->phase2Tol * 5) { bad_pd -= 5; bad_pd = std::max(0, bad_pd); }
        else if (st.gap <= p->phase2Tol) { bad_pd -= 10; bad_pd = std::max(0, bad_pd); }
        if (st.gap >= p->phase1Tol * 1e2) bad_pd += 2;
        if (bad_pd >= (reopt ? 200 : 800)) return 0;
        buf[count % 10] = st.pinfinf;
        if ((reopt ? st.pinf1 : st.pinfinf) <= p->phase2Tol) {
            if (update_dimacs_admm(c)) return -1;
            st.pobj = c->pObjVal; st.dobj = c->dObjVal; st.gap = c->dimGap; st.pinf1 = c->dimPinf;
            if (!reopt || st.gap <= p->phase2Tol) return 0;
        }
        OPC(launch_dual_update(c->dp, st.rho, c->W.lam, c->W.cvs, c->st));
        const long rit = reopt ? st.iter : st.iter + 1;
        if (rit % p->rhoFreq == 0) {
            st.rho *= p->rhoFactor;
            if (st.rho >= cur_rho_max) {
                st.rho = cur_rho_max;
                if (rit % (p->rhoFreq * 100) == 0) {
                    double mean = 0;
                    for (double v : buf) mean += std::fabs(v);
                    mean /= 10.0;
                    if (mean / old_mean >= 0.65) {
                        st.rho *= std::pow(p->rhoFactor, std::round(std::log(p->rhoFreq * 100) / std::log(p->rhoFreq)));
                        cur_rho_max = st.rho;
                    }
                    old_mean = mean;
                }
            }
            if (st.rho >= p->rhoCellingADMM) st.rho = p->rhoCellingADMM;
        }
        if (st.iter % 50 == 0) {
            if (update_dimacs_admm(c)) return -1;
            st.pobj = c->pObjVal; st.dobj = c->dObjVal; st.gap = c->dimGap; st.pinf1 = c->dimPinf;
            if (now_s() - tss >= p->timeSecLimit) return 1;
        }
        if (st.gap <= p->phase2Tol * 1e-3 && st.pinf1 <= p->phase2Tol * 1e-3) return 0;
        st.iter++;
    }
    return 0;
}

// ------------------------------------------------------------------------
// reopt (reoptLevel >= 1): main.c:491-513 / :527-580, reopt() data/lorads_solver.c:1497-1539
// ------------------------------------------------------------------------
// LORADS_ALMOptimize_reopt (lorads_alm.c:959-1218) with early_stop = true, as reopt() calls it:
// no phase-1 exit inside the inner loop, outer loop until maxALMIter (shifted by reopt) and
// the phase-1 tolerances, difficulty without the "super" class, rank growth only with <= 10 cones.
static int alm_optimize_reopt(lrs_ctx *c, lrs_params *p, AlmState &st, double rho_update_factor, double tss) {
    const double ori = now_s();
    int is_rank_max = check_all_rank_max(c, 1.0);
    int retcode = 0, sched_pos = 0;
    long last_outer_start = 1, k = 0, k0 = 0, localIter = 0, clearL = 0;
    double rc = 0.1, rc_tol = 0, rc_val = 0, lag = 0;
    char difficulty = 'h';
    int rank_flag = 0, rho_factor_flag = 0, upd_cnt = 0;
    const double rank_update_factor = p->rankUpdateFactor;
    double thres = 15;
    const int max_inc = 10000, max_ceil = 25000;
ALG_START:
    rc = 0.1;
    rc_tol = rc / st.rho;
    if (op_constr_xx(c, c->W.R, nullptr, nullptr, nullptr)) return -1;
    if (op_grad(c, st.rho, &lag)) return -1;
    rc_val = std::sqrt(lag) / (1 + c->hp.cNrmInf);
    difficulty = 'h';
    localIter = 0; clearL = 0; rank_flag = 0;
    k = st.outerIter; k0 = st.outerIter;
    rho_factor_flag = 0;
    if (p->dyrankLevel == 0) thres = 1e8;
    else if (p->dyrankLevel == 1) thres = 150;
    else if (p->dyrankLevel == 2) thres = 15;
    else if (p->dyrankLevel == 3) thres = 5;
    upd_cnt = 0;
    for (;;) {
        if (k > p->maxALMIter && st.pinfinf <= p->phase1Tol &&
            (st.gap <= std::max(p->phase1Tol, p->phase2Tol * 5) || !p->highAccMode))
            break;
        double ema_cur = 0, ema_old = 0;
        int ema_cnt = 1;
        long cur_iter_counter = 1;
        if (upd_cnt >= 2) { upd_cnt = 0; c->max_sub = std::min(c->max_sub + max_inc, max_ceil); }
        while (difficulty != 'e') {
            localIter = 0;
            int if_break = update_check_ema(&ema_cur, &ema_old, rc_val, 0.1, 0.005, 5, &ema_cnt);
            if (!if_break && !p->highAccMode) break;
            if (cur_iter_counter >= c->max_sub) { upd_cnt += 1; break; }
            if (rank_flag >= thres && !is_rank_max && (k - last_outer_start >= 3)) break;
            if (rc_val <= rc_tol) break;
            InnerIo io;
            io.inner = st.innerIter; io.local = localIter; io.clear = clearL; io.rcval = rc_val; io.lag = lag;
            io.pinf1 = st.pinf1; io.pinfinf = st.pinfinf;
            const long before = st.innerIter;
            if (run_inner(c, p, st.rho, rc_tol, st.gap, p->almInnerBudget, io, false)) return -1;
            st.innerIter = io.inner; localIter = io.local; clearL = io.clear;
            cur_iter_counter += io.inner - before;
            rc_val = io.rcval; lag = io.lag; st.pinf1 = io.pinf1; st.pinfinf = io.pinfinf;
            if (io.exitReason == EXIT_NUMERR) { retcode = 4; goto END_ALM; }
            if (io.exitReason == EXIT_BUDGET) goto PRINT_AND_EXIT;
            if (io.exitReason == EXIT_TINYTAU) goto UpdateRho;
            OPC(launch_dual_update(c->dp, st.rho, c->W.lam, c->W.cvs, c->st));
            if (op_grad(c, st.rho, &lag)) return -1;
            rc_val = std::sqrt(lag) / (1 + c->hp.cNrmInf);
            if (localIter <= 20) difficulty = 'e';
            else if (localIter <= 100) { difficulty = 'm'; rank_flag += 2; }
            else { difficulty = 'h'; rank_flag += 3; }
            if (difficulty == 'e') rank_flag = 0;
        }
    UpdateRho:
        do {
            st.rho *= rho_update_factor;
            if (op_grad(c, st.rho, &lag)) return -1;
            rc_val = std::sqrt(lag) / (1 + c->hp.cNrmInf);
            rc_tol = rc / st.rho;
        } while (rc_tol >= rc_val);
        if (st.rho >= 5e4 && rho_factor_flag < 4) { rho_update_factor = std::sqrt(std::sqrt(rho_update_factor)); rho_factor_flag = 4; }
        else if (st.rho >= 5e6 && rho_factor_flag < 6) { rho_update_factor = std::sqrt(std::sqrt(rho_update_factor)); rho_factor_flag = 6; }
        else if (st.rho >= 5e8 && rho_factor_flag < 8) { rho_update_factor = std::sqrt(std::sqrt(rho_update_factor)); rho_factor_flag = 8; }
        difficulty = 'h';
        clearL = 0;
        k += 1;
        st.outerIter = k;
        {
            double pinf, obj;
            if (op_constr_xx(c, c->W.R, nullptr, &pinf, &obj)) return -1;
            c->pObjVal = obj / c->scaleObjHis;
            cal_dual_obj(c);
            c->dimPinf = pinf;
            c->dimGap = std::fabs(c->pObjVal - c->dObjVal) / (1 + std::fabs(c->pObjVal) + std::fabs(c->dObjVal));
            st.gap = c->dimGap; st.pobj = c->pObjVal; st.dobj = c->dObjVal;
            st.pinf1 = c->dimPinf;
            st.pinfinf = st.pinf1 * (1 + c->hp.bNrm1) / (1 + c->hp.bNrmInf);
            if (st.pinf1 <= p->phase1Tol && st.gap <= std::max(p->phase1Tol, p->phase2Tol * 5) && (k - k0) > 1)
                goto PRINT_AND_EXIT;
            record_state(c, p, 1);
            alm_log(c, p, st, now_s() - ori);
            if (now_s() - tss >= p->timeSecLimit) goto PRINT_AND_EXIT;
        }
        if (rank_flag >= thres && !is_rank_max && c->dp.K <= 10) {
            rank_flag = 0;
            if (k - last_outer_start >= 2) {
                if (aug_rank(c, rank_update_factor, p, &sched_pos, &is_rank_max)) return -1;
                st.outerIter = k;
                last_outer_start = st.outerIter;
                goto ALG_START;
            }
        }
    }
END_ALM: {
        double pinf, obj;
        if (op_constr_xx(c, c->W.R, nullptr, &pinf, &obj)) return -1;
        c->pObjVal = obj / c->scaleObjHis;
        cal_dual_obj(c);
        c->dimPinf = pinf;
        c->dimGap = std::fabs(c->pObjVal - c->dObjVal) / (1 + std::fabs(c->pObjVal) + std::fabs(c->dObjVal));
        st.gap = c->dimGap;
        // lorads_alm.c:1208 derives l_1 back from the last l_inf
        st.pinf1 = st.pinfinf * (1 + c->hp.bNrmInf) / (1 + c->hp.bNrm1);
    }
PRINT_AND_EXIT:
    logf_(c, p, "-----------------------------------------------------------------------\nExit ALM:\n");
    record_state(c, p, 1);
    alm_log(c, p, st, now_s() - ori);
    return retcode;
}

// objScale_dualvar (data/lorads_solver.c:1438-1450): C *= f, lambda *= f, scaleObjHis *= f
static int obj_scale(lrs_ctx *c, double f) {
    DevProblem &P = c->dp;
    const long Pt = std::max(1, P.Ptot);
    if (!c->c_scaled) {
        if (!c->Cw0) {
            HIPC(hipMalloc((void **)&c->Cw0, sizeof(double) * Pt));
            HIPC(hipMalloc((void **)&c->Craw0, sizeof(double) * Pt));
        }
        HIPC(hipMemcpyAsync(c->Cw0, P.Cw, sizeof(double) * Pt, hipMemcpyDeviceToDevice, c->st));
        HIPC(hipMemcpyAsync(c->Craw0, P.Craw, sizeof(double) * Pt, hipMemcpyDeviceToDevice, c->st));
        c->c_scaled = true;
    }
    c->scaleObjHis *= f;
    P.dense_scale *= f;   // dense-objective cones: the factor rides on every product with C
    // captured inner-iteration batches (LRS_GRAPHS=1) hold dense_scale as a kernel argument
    if (P.ndense > 0 && f != 1.0) drop_graphs(c);
    OPC(launch_axpby(Pt, 0.0, P.Cw, f, P.Cw, c->st));
    OPC(launch_axpby(Pt, 0.0, P.Craw, f, P.Craw, c->st));
    OPC(launch_axpby(P.m, 0.0, c->W.lam, f, c->W.lam, c->st));
    return 0;
}
static int obj_unscale(lrs_ctx *c) {
    if (!c->c_scaled) return 0;
    DevProblem &P = c->dp;
    const long Pt = std::max(1, P.Ptot);
    HIPC(hipMemcpyAsync(P.Cw, c->Cw0, sizeof(double) * Pt, hipMemcpyDeviceToDevice, c->st));
    HIPC(hipMemcpyAsync(P.Craw, c->Craw0, sizeof(double) * Pt, hipMemcpyDeviceToDevice, c->st));
    HIPC(hipStreamSynchronize(c->st));
    if (P.ndense > 0 && P.dense_scale != 1.0) drop_graphs(c);
    P.dense_scale = 1.0;
    c->c_scaled = false;
    return 0;
}

// LORADS_ALMtoADMM (data/lorads_solver.c:1351-1387)
static int alm_to_admm(lrs_ctx *c, lrs_params *p, const AlmState &alm, AdmmState &admm) {
    HIPC(hipMemcpyAsync(c->W.V, c->W.R, sizeof(double) * c->dp.NRpad, hipMemcpyDeviceToDevice, c->st));
    HIPC(hipMemcpyAsync(c->W.U, c->W.V, sizeof(double) * c->dp.NRpad, hipMemcpyDeviceToDevice, c->st));
    admm.pinf1 = alm.pinf1; admm.pinfinf = alm.pinfinf; admm.gap = alm.gap;
    admm.rho = alm.rho * p->heuristicFactor;
    if (alm.rho > p->rhoMax) {
        admm.rho = std::min(std::sqrt(std::max(p->rhoMax, alm.rho) / p->rhoMax) * p->rhoMax, alm.rho);
        p->rhoMax = admm.rho;
    }
    return 0;
}

// reopt() (data/lorads_solver.c:1497-1539)
static int reopt(lrs_ctx *c, lrs_params *p, AlmState &alm, AdmmState &admm, double reopt_param, long alm_iter,
                 long admm_iter, double tss, int *bad, int level) {
    const long old_maxALM = p->maxALMIter, old_maxADMM = p->maxADMMIter;
    const double old_rhoMax = p->rhoMax;
    p->maxALMIter = alm_iter - 1 + alm.outerIter;
    p->maxADMMIter = admm_iter;
    if (obj_scale(c, reopt_param)) return -1;
    if (admm.rho <= p->rhoMax) alm.rho = std::max(admm.rho, alm.rho);
    if (alm_optimize_reopt(c, p, alm, std::sqrt(p->ALMRhoFactor), tss) < 0) return -1;
    p->rhoMax = std::max(std::sqrt(std::max(admm.rho, alm.rho) / admm.rho) * admm.rho, p->rhoMax);
    if (alm_to_admm(c, p, alm, admm)) return -1;
    if (*bad == 0 || level < 2) {
        const int rc = admm_optimize(c, p, admm, std::min(admm.iter * 4, admm.iter + old_maxADMM), tss, true);
        if (rc < 0) return -1;
        *bad = 0;   // LORADSADMMOptimize_reopt never returns RET_CODE_BAD_ITER
    }
    p->maxALMIter = old_maxALM;
    p->maxADMMIter = old_maxADMM;
    p->rhoMax = old_rhoMax;
    return 0;
}

// ------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------
extern "C" {

// The error contract of include/lrsdp.h: a NULL context, a context without a problem, without
// solver state (ranks set), or a NULL required pointer returns -1 with lrs_last_error() set
#define LRS_NEED_CTX(c)                                                   \
    do {                                                                  \
        if (!(c)) { set_err("%s: null context", __func__); return -1; }   \
        bind(c);                                                          \
    } while (0)
#define LRS_NEED_LOADED(c)                                                                \
    do {                                                                                  \
        LRS_NEED_CTX(c);                                                                  \
        if (!(c)->loaded) { set_err("%s: no problem loaded", __func__); return -1; }      \
    } while (0)
#define LRS_NEED_STATE(c)                                                                         \
    do {                                                                                          \
        LRS_NEED_LOADED(c);                                                                       \
        if (!(c)->walloc) { set_err("%s: no solver state (ranks not set)", __func__); return -1; } \
    } while (0)
#define LRS_NEED_ARG(x)                                                          \
    do {                                                                         \
        if (!(x)) { set_err("%s: null argument %s", __func__, #x); return -1; }  \
    } while (0)

void lrs_params_default(lrs_params *p) {   // main.c:56-86
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->initRho = 0.0; p->rhoMax = 5000.0; p->rhoCellingALM = 1e8; p->rhoCellingADMM = 5000.0 * 200;
    p->maxALMIter = 200; p->maxADMMIter = 10000; p->timesLogRank = 2.0; p->fixedRank = -1; p->initRank = -1;
    p->rhoFreq = 5; p->rhoFactor = 1.2; p->ALMRhoFactor = 2.0; p->rankUpdateFactor = 1.5; p->phase1Tol = 1e-3;
    p->phase2Tol = 1e-5; p->timeSecLimit = 3600.0; p->heuristicFactor = 1.0; p->lbfgsListLength = 2;
    p->endTauTol = 1e-16; p->endALMSubTol = 1e-10; p->l2Rescaling = 0; p->reoptLevel = 2; p->dyrankLevel = 2;
    p->highAccMode = 0; p->oracleRankNaive = 0; p->disableOracle = 0; p->nearStallFactor = 0.0;
    p->rankSchedule = nullptr; p->rankScheduleLen = 0; p->verbose = 0; p->almInnerBudget = 0; p->skipADMM = 0;
}

const char *lrs_last_error(void) { return g_lrs_err.c_str(); }
const char *lrs_version(void) { return "lrsdp-mi355x 0.5 (abi " LRS_STR(LRSDP_ABI_VERSION) ", gfx950)"; }
int lrs_abi_version(void) { return LRSDP_ABI_VERSION; }

int lrs_ctx_create(int device, lrs_ctx **out) {
    LRS_NEED_ARG(out);
    *out = nullptr;
    lrs_ctx *c = new lrs_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) { set_err("hipSetDevice(%d) failed", device); delete c; return -1; }
    if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) { set_err("stream create failed"); delete c; return -1; }
    if (const char *ug = getenv("LRS_GRAPHS")) c->use_graphs = (atoi(ug) != 0);
    if (const char *sv = getenv("LRS_STATS")) c->stats = (atoi(sv) != 0);
    if (const char *cs = getenv("LRS_CG_SLACK")) c->cg_slack = std::max(0, std::min(8, atoi(cs)));
    if (const char *pb = getenv("LRS_PIPE_BATCH")) c->pipe_batch = std::max(2, std::min(64, (atoi(pb) + 1) & ~1));
    if (hipHostMalloc((void **)&c->hpin, kHpinN * sizeof(double), 0) != hipSuccess) { set_err("pinned alloc failed"); delete c; return -1; }
    if (hipMalloc((void **)&c->s_tickets, 64 * sizeof(unsigned)) != hipSuccess ||
        hipMemset(c->s_tickets, 0, 64 * sizeof(unsigned)) != hipSuccess ||
        hipMalloc((void **)&c->s_tmpfin, TF_N * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&c->s_rpart, kMaxPartialBlocks * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&c->s_fin, kFinN * sizeof(double)) != hipSuccess ||
        hipMemset(c->s_fin, 0, kFinN * sizeof(double)) != hipSuccess) {
        set_err("scratch alloc failed");
        lrs_ctx_destroy(c);
        return -1;
    }
    bind(c);
    *out = c;
    return 0;
}

int lrs_set_kernel_path(lrs_ctx *c, int path) {
    LRS_NEED_LOADED(c);
    if (path < 0 || path > 4) {
        set_err("kernel path %d: expected 0 (auto), 1 (general), 2 (general, bandwidth regime), 3 (+ long-row kernels) "
                "or 4 (the single-workgroup inner loop where it fits)", path);
        return -1;
    }
    if (c->dp.no_lat != path) {
        drop_graphs(c);   // captured batches hold the previous kernels
        c->dp.no_lat = path;
    }
    return 0;
}

int lrs_op_dual_infeasibility(lrs_ctx *c, double *l1, double *lam_min) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(l1);
    return dual_infeasibility(c, l1, lam_min);
}

int lrs_get_kernel_path(lrs_ctx *c, int *used) {
    LRS_NEED_CTX(c);
    LRS_NEED_ARG(used);
    *used = c->loaded ? c->dp.last_path : -1;
    return 0;
}

int lrs_set_log_path(lrs_ctx *c, const char *path) {
    LRS_NEED_CTX(c);
    LRS_NEED_ARG(path);
    if (c->logfp) fclose(c->logfp);
    c->logfp = fopen(path, "w");
    if (!c->logfp) { set_err("cannot open log %s", path); return -1; }
    return 0;
}

void lrs_ctx_destroy(lrs_ctx *c) {
    if (!c) return;
    if (c->logfp) fclose(c->logfp);
    free_work(c);
    if (c->loaded) free_problem(c->dp);
    if (c->hpin) (void)hipHostFree(c->hpin);
    if (c->hgram) (void)hipHostFree(c->hgram);
    if (c->hmir) (void)hipHostFree(c->hmir);
    for (auto &e : c->bev)
        if (e) (void)hipEventDestroy(e);
    delete c->comm;
    for (void *q : {(void *)c->s_tickets, (void *)c->s_tmpfin, (void *)c->s_rpart, (void *)c->s_fin, (void *)c->d_sendbuf,
                    (void *)c->d_sendvec, (void *)c->Cw0, (void *)c->Craw0, (void *)c->xwg_snap})
        if (q) (void)hipFree(q);
    for (int *q : c->d_send_rows)
        if (q) (void)hipFree(q);
    bind_scratch(nullptr, nullptr, nullptr, nullptr);
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
}

int lrs_load_sdpa(lrs_ctx *c, const char *path, double *read_seconds) {
    LRS_NEED_CTX(c);
    LRS_NEED_ARG(path);
    const double t0 = now_s();
    std::string err;
    HostProblem hp;
    if (!read_sdpa(path, hp, err)) { set_err("read_sdpa: %s", err.c_str()); return -1; }
    if (read_seconds) *read_seconds = now_s() - t0;
    free_work(c);
    if (c->loaded) free_problem(c->dp);
    c->hp = std::move(hp);
    if (!upload_problem(c->hp, c->dp, err)) { set_err("upload: %s", err.c_str()); return -1; }
    c->loaded = true;
    c->path = path;
    c->cgIterCone.assign(c->hp.K, 0);
    return 0;
}

int lrs_load_coo(lrs_ctx *c, int m, int nblk, const int *dims, const double *b, long nnz, const int *con,
                 const int *blk, const int *row, const int *col, const double *val) {
    LRS_NEED_CTX(c);
    LRS_NEED_ARG(dims);
    if (m > 0) LRS_NEED_ARG(b);
    if (nnz > 0 && (!con || !blk || !row || !col || !val)) { set_err("lrs_load_coo: null entry array"); return -1; }
    std::string err;
    HostProblem hp;
    if (!build_problem_coo(m, nblk, dims, b, nnz, con, blk, row, col, val, hp, err)) {
        set_err("load_coo: %s", err.c_str());
        return -1;
    }
    free_work(c);
    if (c->loaded) free_problem(c->dp);
    c->hp = std::move(hp);
    if (!upload_problem(c->hp, c->dp, err)) { set_err("upload: %s", err.c_str()); return -1; }
    c->loaded = true;
    c->path = "<memory>";
    c->cgIterCone.assign(c->hp.K, 0);
    return 0;
}

int lrs_auut_bytes(lrs_ctx *c, double *bytes) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(bytes);
    // A(U U^T) over constraint entries (SURVEY.md §8(d) B_A with delta = 1): the factor
    // rows touched (each row once when distinct), per entry con_slot + con_w + slot
    // coordinates (16 B), con_ptr, and the m outputs.
    double by = 0;
    for (int k = 0; k < c->dp.K; ++k) {
        const HostCone &hc = c->hp.cones[k];
        std::vector<char> touched(hc.n, 0);
        long rows = 0;
        for (const HostEntry &e : hc.ent) {
            const int p = hc.prow[e.slot], q = hc.pcol[e.slot];
            if (!touched[p]) { touched[p] = 1; rows++; }
            if (!touched[q]) { touched[q] = 1; rows++; }
        }
        by += 8.0 * rows * c->rank[k] + 16.0 * (double)hc.ent.size() + 4.0 * (c->dp.m + 1);
    }
    by += 8.0 * c->dp.m;
    *bytes = by;
    return 0;
}

int lrs_stage_bytes(lrs_ctx *c, double *bytes) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(bytes);
    // Algorithmic HBM bytes per launch of the split-iteration stages:
    // every array the stage must touch, once, at its unpadded size; L-BFGS with two
    // pairs; int32 indices, FP64 values.  n, r per cone; P lower slots; adjacency
    // entries A = 2P - n_diag; Z constraint entries; m constraints (m_l local).
    double a = 0, g = 0, bb = 0;
    const DevProblem &P = c->dp;
    // the latency kernels (the last enqueued iteration's path 0) run each stage as one launch
    // (alm_stage_*_split describe the general kernels' plan)
    const bool lat = P.last_path == 0;
    const bool split_a = !lat && alm_stage_a_split(c->dp), split_b = !lat && alm_stage_b_split(c->dp);
    for (int k = 0; k < P.K; ++k) {
        const HostCone &hc = c->hp.cones[k];
        const double n = hc.n, r = c->rank[k], Pk = (double)hc.prow.size(), A = (double)hc.adj_col.size();
        const double nr8 = 8.0 * n * r;
        // split stage A (bandwidth regime): D is written by the first launch and read back
        a += (split_a ? 8 : 7) * nr8 + 8 * (n + 1) + 8 * Pk /*lower adj col+slot*/ + 8 * Pk /*Cw*/ +
             16 * Pk /*uRD,uDD*/ + 4 * (Pk + 1);
        // split stage B: R_new is written by the first launch and read back by the second
        bb += (split_b ? 11 : 9) * nr8 + 8 * (n + 1) + 8 * A /*adj col+slot*/ + 8 * Pk /*Craw*/ + 4 * (Pk + 1) /*slot_ptr*/ +
              8 * Pk /*uRR*/ + 4 * (Pk + 1) /*loc_ptr*/;
    }
    const double m = P.m, ml = P.m - P.mg, Z = (double)P.Z;
    a += 12 * ml /*loc con,w*/ + 24 * ml /*b,cvs,lam*/ + 32 * ml /*rec*/;
    g = P.mg > 0 ? (12.0 * Z + 4.0 * (P.K * m + 1) + 16.0 * 2 * Z /*uRD,uDD gathers*/ + 24.0 * P.mg + 32.0 * P.mg +
                    4.0 * P.mg) : 0.0;
    bb += 12 * Z /*slot_con,a*/ + 32 * m /*rec*/ + 12 * ml /*loc con,w*/ + 16 * ml /*b read, cvs write*/;
    bytes[0] = a; bytes[1] = g; bytes[2] = bb;
    return 0;
}

int lrs_problem_info(lrs_ctx *c, int *m, int *ncones, int *dims, long *nslots, long *nnzc) {
    LRS_NEED_LOADED(c);
    if (m) *m = c->hp.m;
    if (ncones) *ncones = c->hp.K;
    if (dims) for (int k = 0; k < c->hp.K; ++k) dims[k] = c->hp.cones[k].n;
    if (nslots) *nslots = c->dp.Ptot;
    if (nnzc) *nnzc = c->dp.Z;
    return 0;
}

int lrs_tile_info(lrs_ctx *c, int *auv, int *slot) {
    LRS_NEED_LOADED(c);
    int a = 0, sl = 0;
    for (int k = 0; k < c->dp.K; ++k) {
        a |= c->dp.cones[k].auv_items > 0;
        sl |= c->dp.cones[k].sa_items > 0;
    }
    if (auv) *auv = a;
    if (slot) *slot = sl;
    return 0;
}

int lrs_tile_used(lrs_ctx *c, int *used) {
    LRS_NEED_LOADED(c);
    if (used) *used = c->dp.last_tiles;
    return 0;
}

int lrs_determine_rank(lrs_ctx *c, const lrs_params *p, int *ranks_out) {
    LRS_NEED_LOADED(c);
    LRS_NEED_ARG(p);
    LRS_NEED_ARG(ranks_out);
    std::vector<int> r, rm;
    determine_rank(c, p, r, rm);
    for (int k = 0; k < c->hp.K; ++k) ranks_out[k] = r[k];
    return 0;
}

int lrs_set_rank(lrs_ctx *c, const int *ranks) {
    LRS_NEED_LOADED(c);
    LRS_NEED_ARG(ranks);
    std::vector<int> r(ranks, ranks + c->hp.K);
    if (c->dp.lp_cone >= 0 && r[c->dp.lp_cone] != 1) {
        set_err("lrs_set_rank: the LP cone (cone %d) has rank 1 (x_j = r_j^2), got %d", c->dp.lp_cone, r[c->dp.lp_cone]);
        return -1;
    }
    c->rank_max = r;
    return alloc_work(c, r);
}
int lrs_get_rank(lrs_ctx *c, int *ranks) {
    LRS_NEED_LOADED(c);
    LRS_NEED_ARG(ranks);
    for (size_t k = 0; k < c->rank.size(); ++k) ranks[k] = c->rank[k];
    return 0;
}

int lrs_factor_set(lrs_ctx *c, int which, const double *colmajor) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(colmajor);
    double *d = factor_ptr(c, which);
    if (!d) { set_err("bad factor id"); return -1; }
    return factor_put(c, d, colmajor);
}
int lrs_factor_get(lrs_ctx *c, int which, double *colmajor) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(colmajor);
    double *d = factor_ptr(c, which);
    if (!d) { set_err("bad factor id"); return -1; }
    return factor_fetch(c, d, colmajor);
}
int lrs_vec_set(lrs_ctx *c, int which, const double *v) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(v);
    double *d = vec_ptr(c, which);
    if (!d) { set_err("bad vector id"); return -1; }
    HIPC(h2d_sync(c, d, v, sizeof(double) * c->dp.m));
    return 0;
}
int lrs_vec_get(lrs_ctx *c, int which, double *v) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(v);
    double *d = vec_ptr(c, which);
    if (!d) { set_err("bad vector id"); return -1; }
    HIPC(hipStreamSynchronize(c->st));
    HIPC(hipMemcpy(v, d, sizeof(double) * c->dp.m, hipMemcpyDeviceToHost));
    return 0;
}

int lrs_op_q12(lrs_ctx *c, double *q1, double *p1, double *q2, double *p2) {
    LRS_NEED_STATE(c);
    DevWork &W = c->W;
    DevProblem &P = c->dp;
    // q1, q2 and p1, p2 (a dense objective's <R, C D>, <D, C D> included) with the finals the
    // device line search consumes
    double a = 0, b = 0;
    if (op_q12_fin(c, &a, &b)) return -1;
    if (p1) *p1 = 2 * a;
    if (p2) *p2 = b;
    HIPC(hipStreamSynchronize(c->st));
    if (q1) HIPC(hipMemcpy(q1, W.q1, sizeof(double) * P.m, hipMemcpyDeviceToHost));
    if (q2) HIPC(hipMemcpy(q2, W.q2, sizeof(double) * P.m, hipMemcpyDeviceToHost));
    return 0;
}

int lrs_op_constr_rr(lrs_ctx *c, double *cvs, double *pinf, double *pobj) {
    LRS_NEED_STATE(c);
    double pi, ob;
    if (op_constr_xx(c, c->W.R, nullptr, &pi, &ob)) return -1;
    if (pinf) *pinf = pi;
    if (pobj) *pobj = ob / c->scaleObjHis;
    if (cvs) {
        HIPC(hipStreamSynchronize(c->st));
        HIPC(hipMemcpy(cvs, c->W.cvs, sizeof(double) * c->dp.m, hipMemcpyDeviceToHost));
    }
    return 0;
}

int lrs_op_grad(lrs_ctx *c, double rho, double *lag) {
    LRS_NEED_STATE(c);
    double l;
    if (op_grad(c, rho, &l)) return -1;
    if (lag) *lag = l;
    return 0;
}

int lrs_op_line_search(lrs_ctx *c, double rho, double *tau, int *root_num) {
    LRS_NEED_STATE(c);
    double par[P_NPAR] = {0};
    par[P_RHO] = rho;
    par[P_ENDTAU] = 1e-16;
    HIPC(h2d_sync(c, c->W.par, par, sizeof(par)));
    OPC(launch_ls_only(c->dp, c->W, c->st));
    double ls[LS_N];
    HIPC(hipStreamSynchronize(c->st));
    HIPC(hipMemcpy(ls, c->W.lsres, sizeof(ls), hipMemcpyDeviceToHost));
    if (tau) *tau = ls[LS_TAU];
    if (root_num) *root_num = (int)ls[LS_ROOTNUM];
    return 0;
}

int lrs_op_lbfgs(lrs_ctx *c, int node_num, double beta_new, double beta_old) {
    LRS_NEED_STATE(c);
    // White-box test of the fused direction kernel: ring slot 0 = newest pair
    // (S0, Y0, beta_new), slot 1 = older pair (S1, Y1, beta_old), gradient G[gcur].
    if (node_num < 0 || node_num > 2) { set_err("node_num must be 0..2"); return -1; }
    DevWork &W = c->W;
    const long NR = c->dp.NRpad;
    const double *G = W.G[c->gcur];
    double d[9];
    const double *pairs[9][2] = {{G, G}, {W.ls[0], G}, {W.ly[0], G}, {W.ls[1], G}, {W.ly[1], G},
                                 {W.ls[1], W.ly[0]}, {W.ly[1], W.ly[0]}, {W.ly[0], W.ly[0]}, {W.ly[1], W.ly[1]}};
    for (int q = 0; q < 9; ++q)
        if (op_dot(c, NR, pairs[q][0], pairs[q][1], &d[q])) return -1;
    double par[P_NPAR] = {0};
    par[P_L] = 2; par[P_RCTOL] = -1e300; par[P_ENDSUB] = 0;
    HIPC(h2d_sync(c, W.par, par, sizeof(par)));
    double ctl[C_NCTRL] = {0};
    ctl[C_ACTIVE] = 1; ctl[C_PENDING] = 2; ctl[C_RCVAL] = 1.0;
    ctl[C_LOCAL] = node_num == 0 ? 0 : 1; ctl[C_CLEAR] = node_num;
    ctl[C_HEAD] = 1;                 // newest = slot 0, older = slot 1
    ctl[C_GCUR] = c->gcur; ctl[C_LAG] = d[0];
    ctl[C_BETA0] = beta_new; ctl[C_BETA1] = beta_old; ctl[C_YY0] = d[7]; ctl[C_YY1] = d[8];
    ctl[C_DSG] = d[1]; ctl[C_DYG] = d[2]; ctl[C_DSOG] = d[3]; ctl[C_DYOG] = d[4]; ctl[C_DSOY] = d[5];
    ctl[C_DYOY] = d[6];
    HIPC(h2d_sync(c, W.ctrl + C_NCTRL, ctl, sizeof(ctl)));
    OPC(launch_alm_dir_only(c->dp, W, c->st));
    HIPC(hipStreamSynchronize(c->st));
    return 0;
}

int lrs_op_admm_constr(lrs_ctx *c) {
    LRS_NEED_STATE(c);
    if (admm_init_constr(c)) return -1;
    HIPC(hipStreamSynchronize(c->st));
    return 0;
}

int lrs_op_admm_half(lrs_ctx *c, int cone, int side, double rho, double cg_tol, int cg_maxit, int *cg_iters,
                     double *rhs) {
    LRS_NEED_STATE(c);
    DevProblem &P = c->dp;
    if (cone < 0 || cone >= P.K) { set_err("lrs_op_admm_half: cone %d of %d", cone, P.K); return -1; }
    if (side != 0 && side != 1) { set_err("lrs_op_admm_half: side %d (0 = U, 1 = V)", side); return -1; }
    if (!(rho > 0.0) || cg_maxit < 1) { set_err("lrs_op_admm_half: rho %g, cg_maxit %d", rho, cg_maxit); return -1; }
    // LORADSUpdateSDPVar's half-step for one cone (lorads_alg_common.c:303-314 for U, :316-324
    // for V): solve the side with the other fixed, then the cone's constraint-value refresh
    c->cgIterCone[cone] = 0;
    bool dev = false;
    if (is_lp(c, cone)) {
        // the LP block: its update interleaves u_j and v_j column by column
        // (LORADSUpdateSDPLPVar's LP loop), so side 0 runs the whole sweep and side 1 is refused
        if (side != 0) { set_err("lrs_op_admm_half: the LP cone's sweep updates U and V together (side 0)"); return -1; }
        OPC(launch_lp_admm(P, c->W, rho, c->st));
        HIPC(hipStreamSynchronize(c->st));
        if (cg_iters) *cg_iters = 0;
        return 0;
    }
    if (admm_half_step(c, cone, side, rho, cg_tol, cg_maxit, &dev)) return -1;
    HIPC(hipStreamSynchronize(c->st));
    if (cg_iters) {
        double it = (double)c->cgIterCone[cone];
        if (dev) HIPC(hipMemcpy(&it, c->W.cgc + CG_ITERS, sizeof(double), hipMemcpyDeviceToHost));
        *cg_iters = (int)it;
    }
    if (rhs) {
        const DevCone &d = P.cones[cone];
        std::vector<double> h((size_t)d.n * d.ld);
        HIPC(hipMemcpy(h.data(), c->W.cg_b + d.foff, sizeof(double) * h.size(), hipMemcpyDeviceToHost));
        for (int q = 0; q < d.r; ++q)
            for (int i = 0; i < d.n; ++i) rhs[i + (long)q * d.n] = h[(long)i * d.ld + q];
    }
    return 0;
}

int lrs_op_dual_update(lrs_ctx *c, double rho) {
    LRS_NEED_STATE(c);
    // LORADSUpdateDualVar (lorads_alg_common.c:511-524): lambda += rho (b - CVS)
    OPC(launch_dual_update(c->dp, rho, c->W.lam, c->W.cvs, c->st));
    HIPC(hipStreamSynchronize(c->st));
    return 0;
}

// The host-stepped ALM trip's second half (lorads_alm.c:1340-1355): setAsNegGrad (:780-801),
// ALMupdateVar (:804-833), constrValSum += tau ARDSum + tau^2 ADDSum (:1349-1352), ALMCalGrad
// (:74-87) into the other gradient buffer and setlbfgsHisTwo (:842-863).  The ring keeps
// lrs_op_lbfgs's convention: the new pair goes to (S0, Y0), the previous newest to (S1, Y1).
int lrs_op_alm_update(lrs_ctx *c, double rho, double tau, double *lag_norm_sq, double *beta) {
    LRS_NEED_STATE(c);
    if (sharded(c)) { set_err("lrs_op_alm_update: unsharded contexts only (the ring's dots span whole buffers)"); return -1; }
    if (!(rho > 0.0)) { set_err("lrs_op_alm_update: rho %g", rho); return -1; }
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    const long NR = P.NRpad;
    HIPC(hipMemcpyAsync(W.ls[1], W.ls[0], sizeof(double) * NR, hipMemcpyDeviceToDevice, c->st));
    HIPC(hipMemcpyAsync(W.ly[1], W.ly[0], sizeof(double) * NR, hipMemcpyDeviceToDevice, c->st));
    OPC(launch_axpby(NR, -1.0, W.G[c->gcur], 0.0, W.ly[0], c->st));   // y = -G
    OPC(launch_axpby(NR, tau, W.D, 1.0, W.R, c->st));                 // R += tau D
    OPC(launch_axpby(P.m, tau, W.q1, 1.0, W.cvs, c->st));
    OPC(launch_axpby(P.m, tau * tau, W.q2, 1.0, W.cvs, c->st));
    c->gcur ^= 1;
    double lag;
    if (op_grad(c, rho, &lag)) return -1;
    OPC(launch_axpby(NR, tau, W.D, 0.0, W.ls[0], c->st));             // s = tau D
    OPC(launch_axpby(NR, 1.0, W.G[c->gcur], 1.0, W.ly[0], c->st));    // y += G_new
    double ys;
    if (op_dot(c, NR, W.ly[0], W.ls[0], &ys)) return -1;
    if (lag_norm_sq) *lag_norm_sq = lag;
    if (beta) *beta = 1.0 / ys;
    return 0;
}

// sdpDataWSum + mul_rk (data/def_lorads_sdp_data.h:66-85) over every cone: out = scale (with_C C
// + sum_i y_i A_i) X with X the factor `which` (the ADMM right-hand side's S Y, ALMCalGrad's S R)
int lrs_op_adjoint(lrs_ctx *c, const double *y, int which, double *out, double scale, int with_C) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(y);
    LRS_NEED_ARG(out);
    if (sharded(c)) { set_err("lrs_op_adjoint: unsharded contexts only"); return -1; }
    const double *X = factor_ptr(c, which);
    if (!X) { set_err("lrs_op_adjoint: bad factor id %d", which); return -1; }
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    HIPC(h2d_sync(c, W.M1, y, sizeof(double) * P.m));
    OPC(launch_wsum(P, W.M1, with_C ? 1 : 0, W.S, c->st));
    for (int k = 0; k < P.K; ++k)
        OPC(launch_spmm(P, k, W.S, X, scale, nullptr, 0.0, W.X, W.part, 0, nullptr, c->st));
    for (int k = 0; k < P.K && with_C; ++k) {
        const DevCone &dc = P.cones[k];
        if (!dc.dense_c) continue;   // a dense objective is not on the slots: + scale C X
        OPC(launch_dense_cx(P, k, X, W.cg_Q, 0.0, c->st));
        OPC(launch_axpby((long)dc.n * dc.ld, scale, W.cg_Q + dc.foff, 1.0, W.X + dc.foff, c->st));
    }
    return factor_fetch(c, W.X, out);
}

// coneAUV + objAUV (data/def_lorads_sdp_conic.h:106-111): out_m[i] = A_i(sym(X_u X_v^T)) summed
// over the cones, cobj = <C, sym(X_u X_v^T)> (before the division by scaleObjHis); u == v: X X^T.
// The solver state (CVS and the per-cone values) is left as it was.
int lrs_op_auv(lrs_ctx *c, int u, int v, double *out_m, double *cobj) {
    LRS_NEED_STATE(c);
    if (sharded(c)) { set_err("lrs_op_auv: unsharded contexts only"); return -1; }
    const double *X = factor_ptr(c, u), *Y = factor_ptr(c, v);
    if (!X || !Y) { set_err("lrs_op_auv: bad factor ids %d, %d", u, v); return -1; }
    DevProblem &P = c->dp;
    DevWork &W = c->W;
    const long nsave = (long)P.m * (std::max(1, P.K) + 1);
    double *save = nullptr;
    HIPC(hipMalloc((void **)&save, sizeof(double) * nsave));
    int rc = -1;
    double obj = 0.0;
    if (hipMemcpyAsync(save, W.cvs, sizeof(double) * P.m, hipMemcpyDeviceToDevice, c->st) != hipSuccess ||
        hipMemcpyAsync(save + P.m, W.cvc, sizeof(double) * (nsave - P.m), hipMemcpyDeviceToDevice, c->st) != hipSuccess) {
        set_err("lrs_op_auv: copy failed");
    } else if (op_constr_xx(c, X, u == v ? nullptr : Y, nullptr, &obj) == 0) {
        rc = 0;
        if (out_m && (hipStreamSynchronize(c->st) != hipSuccess ||
                      hipMemcpy(out_m, W.cvs, sizeof(double) * P.m, hipMemcpyDeviceToHost) != hipSuccess)) {
            set_err("lrs_op_auv: fetch failed");
            rc = -1;
        }
    }
    if (hipMemcpyAsync(W.cvs, save, sizeof(double) * P.m, hipMemcpyDeviceToDevice, c->st) != hipSuccess ||
        hipMemcpyAsync(W.cvc, save + P.m, sizeof(double) * (nsave - P.m), hipMemcpyDeviceToDevice, c->st) != hipSuccess ||
        hipStreamSynchronize(c->st) != hipSuccess) {
        set_err("lrs_op_auv: restore failed");
        rc = -1;
    }
    (void)hipFree(save);
    if (rc == 0 && cobj) *cobj = obj;
    return rc;
}

// LORADSUpdateDimacsErrorALM / ADMM (lorads_alg/lorads_alg_common.c:424-428, :454-462) with the
// objectives they read, LORADSCalObjRR_ALM / LORADSCalObjUV_ADMM (lorads_alm.c:1488-1497,
// lorads_admm.c:398-410) and LORADSCalDualObj (lorads_alg_common.c:531): admm = 1 first sets
// R = (U + V) / 2.  CVS <- A(R R^T); out5 = {pObj, dObj, l_1 primal infeasibility, l_inf primal
// infeasibility, relative gap}.
int lrs_op_dimacs(lrs_ctx *c, int admm, double *out5) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(out5);
    double pinf;
    if (admm) {   // the ADMM loop's own evaluation (admm_eval: R = (U + V) / 2 first)
        if (admm_eval(c)) return -1;
        pinf = c->dimPinf;
    } else {
        double obj, blam;
        if (op_constr_xx(c, c->W.R, nullptr, &pinf, &obj, &blam)) return -1;
        c->pObjVal = obj / c->scaleObjHis;
        c->dObjVal = blam / c->scaleObjHis;
        c->dimPinf = pinf;
        c->dimGap = std::fabs(c->pObjVal - c->dObjVal) / (1 + std::fabs(c->pObjVal) + std::fabs(c->dObjVal));
    }
    out5[0] = c->pObjVal;
    out5[1] = c->dObjVal;
    out5[2] = pinf;
    out5[3] = pinf * (1 + c->hp.bNrm1) / (1 + c->hp.bNrmInf);
    out5[4] = c->dimGap;
    return 0;
}

int lrs_op_gram(lrs_ctx *c, int cone, int which, double *gram) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(gram);
    if (cone < 0 || cone >= c->dp.K) { set_err("lrs_op_gram: cone %d of %d", cone, c->dp.K); return -1; }
    std::vector<double> g;
    if (which == LRS_R) { if (gram_of(c, cone, c->W.R, nullptr, 0, g)) return -1; }
    else { if (gram_of(c, cone, c->W.U, c->W.V, 1, g)) return -1; }
    memcpy(gram, g.data(), sizeof(double) * g.size());
    return 0;
}

static int solve_impl(lrs_ctx *c, const lrs_params *pin, lrs_result *res) {
    lrs_params prm = *pin;
    lrs_params *p = &prm;
    p->rhoCellingADMM = p->rhoMax * 200;   // main.c:350
    memset(res, 0, sizeof(*res));
    const double tss = now_s();
    c->dinf_tol = p->phase2Tol;
    c->dinf_steps = c->dinf_iters = 0;
    c->rank_warned = false;
    if (p->lbfgsListLength < 1) { set_err("lbfgsListLength %d < 1", p->lbfgsListLength); return -1; }
    // a sharded solve runs the fused two-pair L-BFGS only: the ring of L != 2 pairs
    // (run_inner_generic) takes its dots over whole local buffers, halo rows included.  Refused
    // here, before any device work, rather than part-way into the ALM phase.
    if (sharded(c) && p->lbfgsListLength != 2) {
        set_err("lbfgsListLength %d: a sharded solve (lrs_shard_rccl / lrs_shard_loopback) supports "
                "lbfgsListLength 2 only (the reference's default, main.c:80)", p->lbfgsListLength);
        return -1;
    }
    c->lbfgsL = p->lbfgsListLength;
    c->dinf_time = 0.0;
    if (obj_unscale(c)) return -1;   // a previous solve's reopt scaled C on the device
    std::vector<int> r, rm;
    determine_rank(c, p, r, rm);
    if (alloc_work(c, r)) return -1;
    c->rank_max = rm;
    if (init_point(c)) return -1;
    c->t1c.clear(); c->t1o.clear(); c->t2c.clear(); c->t2o.clear();
    c->naive_warned = false;
    c->scaleObjHis = 1.0;
    c->pObjVal = c->dObjVal = 0;
    AlmState alm;
    AdmmState admm;
    double rho = p->initRho;
    if (rho == 0) {   // initial_solver_state, data/lorads_solver.c:1599-1606
        long sd = 0;
        for (int k = 0; k < c->hp.K; ++k) sd += is_lp(c, k) ? 0 : cone_n_global(c, k);   // SDP blocks only
        rho = 1 / std::sqrt((double)sd);
    }
    alm.rho = rho; admm.rho = rho;
    const double t0 = now_s();
    int rc = alm_optimize(c, p, alm, tss);
    if (rc < 0) return -1;
    res->retcode = rc;
    const double t_alm = now_s() - t0;
    res->alm_inner = alm.innerIter; res->alm_outer = alm.outerIter;
    res->alm_pobj = alm.pobj; res->alm_dobj = alm.dobj; res->alm_pinf = alm.pinf1; res->alm_gap = alm.gap;
    res->alm_rho = alm.rho;
    res->alm_time = t_alm;
    bool timeout = now_s() - tss > p->timeSecLimit;
    double t_admm = 0;
    double dinf = -1.0;   // not evaluated (phase 2 skipped)
    int dinf_conv = -1;
    if (!timeout && !p->skipADMM) {
        if (alm_to_admm(c, p, alm, admm)) return -1;
        const double ta = now_s();
        int arc = admm_optimize(c, p, admm, p->maxADMMIter, tss);
        if (arc < 0) return -1;
        t_admm = now_s() - ta;
        // reoptLevel >= 1 (main.c:491-513): one reopt round while neither phase met phase2Tol
        const double reopt_param = 5;
        const long alm_min = 3, admm_min = p->highAccMode ? 1000 : 50;   // main.c:436-443
        int bad = 0, cnt = 0;
        if (p->reoptLevel >= 1) {
            while ((alm.gap > p->phase2Tol || alm.pinf1 > p->phase2Tol) &&
                   (admm.gap > p->phase2Tol || admm.pinf1 > p->phase2Tol)) {
                if (cnt >= 1) break;
                if (reopt(c, p, alm, admm, reopt_param, alm_min, admm_min, tss, &bad, 1)) return -1;
                cnt++;
                if (now_s() - tss > p->timeSecLimit) { timeout = true; break; }
            }
        }
        // dual infeasibility of the phase-2 multipliers (main.c:515-527); a time-limit exit of
        // the reopt round jumps past it to END_SOLVING like main.c:505-510
        if (!timeout) {
            dinf_conv = 1;
            if (dual_infeasibility(c, &dinf, nullptr, &dinf_conv)) return -1;
            admm.gap = c->dimGap;
            admm.pinf1 = c->dimPinf;
            logf_(c, p, "-----------------------------------------------------------------------\n"
                        "Dual infeasibility: l_1 = %f, l_inf = %f, l_2 = %f\n"
                        "-----------------------------------------------------------------------\n",
                  dinf, dinf * (1 + c->hp.cNrm1) / (1 + c->hp.cNrmInf), dinf * (1 + c->hp.cNrm1) / (1 + c->hp.cNrm2));
            // reoptLevel >= 2 (main.c:527-580): up to two more rounds, each followed by the
            // U/V average and a new dual infeasibility
            if (p->reoptLevel >= 2 && !timeout) {
                int dual_cnt = 0;
                while (dinf > p->phase2Tol || admm.gap > p->phase2Tol || admm.pinf1 > p->phase2Tol) {
                    if (dual_cnt >= 2) break;
                    if (!p->highAccMode && dinf <= 5 * p->phase2Tol && admm.gap <= 5 * p->phase2Tol &&
                        admm.pinf1 <= p->phase2Tol)
                        break;
                    if (reopt(c, p, alm, admm, reopt_param, 3, 50, tss, &bad, 2)) return -1;
                    OPC(launch_avg(c->dp.NRpad, c->W.U, c->W.V, c->W.R, c->st));
                    HIPC(hipMemcpyAsync(c->W.V, c->W.R, sizeof(double) * c->dp.NRpad, hipMemcpyDeviceToDevice, c->st));
                    dinf_conv = 1;
                    if (dual_infeasibility(c, &dinf, nullptr, &dinf_conv)) return -1;
                    admm.gap = c->dimGap;
                    admm.pinf1 = c->dimPinf;
                    admm.pinfinf = c->dimPinf * (1 + c->hp.bNrm1) / (1 + c->hp.bNrmInf);
                    logf_(c, p, "reopt %d:Dual infeasibility: l_1 = %f, l_inf = %f, l_2 = %f\n", dual_cnt, dinf,
                          dinf * (1 + c->hp.cNrm1) / (1 + c->hp.cNrmInf), dinf * (1 + c->hp.cNrm1) / (1 + c->hp.cNrm2));
                    dual_cnt++;
                    if (now_s() - tss > p->timeSecLimit) { timeout = true; break; }
                }
            }
        }
        t_admm = now_s() - ta;
        // the ALM state after the reopt rounds (alm_inner / alm_time stay the first phase's)
        res->alm_outer = alm.outerIter;
        res->alm_pobj = alm.pobj; res->alm_dobj = alm.dobj; res->alm_pinf = alm.pinf1; res->alm_gap = alm.gap;
        res->alm_rho = alm.rho;
    }
    HIPC(hipStreamSynchronize(c->st));
    const double all_time = now_s() - t0;
    // main.c:519-525 (END_SOLVING after a time limit keeps the ADMM state as it was)
    if (!timeout) {
        admm.gap = c->dimGap;
        admm.pinf1 = c->dimPinf;
        admm.pinfinf = c->dimPinf * (1 + c->hp.bNrm1) / (1 + c->hp.bNrmInf);
    }
    res->admm_iter = admm.iter; res->cg_iter = admm.cg_iter;
    res->pobj = admm.pobj; res->dobj = admm.dobj; res->pinf = admm.pinf1; res->pinf_inf = admm.pinfinf;
    res->gap = admm.gap; res->rho = admm.rho;
    res->solve_time = all_time; res->admm_time = t_admm;
    res->rho_max = p->rhoMax;
    // main.c:592-604
    res->dinf = dinf;
    res->dinf_inf = dinf < 0 ? dinf : dinf * (1 + c->hp.cNrm1) / (1 + c->hp.cNrmInf);
    res->dinf_2 = dinf < 0 ? dinf : dinf * (1 + c->hp.cNrm1) / (1 + c->hp.cNrm2);
    res->dinf_converged = dinf_conv;
    res->dinf_iters = (int)c->dinf_iters;
    res->dinf_steps = c->dinf_steps;
    res->dinf_time = c->dinf_time;
    res->obj_scale = c->scaleObjHis;
    // PRIMAL_DUAL_OPTIMAL only on a dual infeasibility whose eigen-solve converged (a Ritz value
    // after the last update iteration only bounds lambda_min from above)
    if (timeout) res->status = 4;
    else if (dinf >= 0 && dinf_conv == 1 && dinf <= 5 * p->phase2Tol && admm.gap <= 5 * p->phase2Tol && admm.pinf1 <= p->phase2Tol)
        res->status = 1;
    else if (admm.gap <= 5 * p->phase2Tol && admm.pinf1 <= p->phase2Tol) res->status = 2;
    else res->status = 3;
    res->final_rank = sum_rank(c);
    int orc = (p->disableOracle || p->skipADMM) ? res->final_rank : p->oracleRankNaive ? oracle_rank_naive(c, p, 2) : oracle_rank(c, 2);
    res->oracle_rank = orc < 0 ? 0 : orc;
    res->traj1_len = (int)c->t1c.size();
    res->traj2_len = (int)c->t2c.size();
    return 0;
}

int lrs_solve(lrs_ctx *c, const lrs_params *p, lrs_result *res) {
    LRS_NEED_LOADED(c);
    LRS_NEED_ARG(p);
    LRS_NEED_ARG(res);
    return solve_impl(c, p, res);
}

int lrs_trajectory(lrs_ctx *c, int phase, int *curr, int *orc, int cap) {
    LRS_NEED_CTX(c);
    if (phase != 1 && phase != 2) { set_err("lrs_trajectory: phase %d (1 or 2)", phase); return -1; }
    const std::vector<int> &a = phase == 1 ? c->t1c : c->t2c, &b = phase == 1 ? c->t1o : c->t2o;
    int n = std::min(cap, (int)a.size());
    for (int i = 0; i < n; ++i) { if (curr) curr[i] = a[i]; if (orc) orc[i] = b[i]; }
    return (int)a.size();
}

int lrs_write_json(lrs_ctx *c, const char *path, const char *pid, const char *fpath, const lrs_result *r,
                   const lrs_params *p) {
    LRS_NEED_LOADED(c);
    LRS_NEED_ARG(path);
    LRS_NEED_ARG(r);
    LRS_NEED_ARG(p);
    if (!pid) pid = "";
    if (!fpath) fpath = "";
    FILE *f = fopen(path, "w");
    if (!f) { set_err("cannot open %s", path); return -1; }
    fprintf(f, "{\n");
    fprintf(f, "  \"problem_id\": \"%s\",\n", pid);
    fprintf(f, "  \"file_path\": \"%s\",\n", fpath);
    fprintf(f, "  \"metrics\": {\n");
    fprintf(f, "    \"oracle_rank\": %lld,\n", (long long)r->oracle_rank);
    fprintf(f, "    \"primal_obj\": %.16e,\n", r->pobj);
    fprintf(f, "    \"dual_obj\": %.16e,\n", r->dobj);
    fprintf(f, "    \"constr_violation_l1\": %.16e,\n", r->pinf);
    fprintf(f, "    \"constr_violation_inf\": %.16e,\n", r->pinf_inf);
    fprintf(f, "    \"primal_dual_gap\": %.16e,\n", r->gap);
    fprintf(f, "    \"solve_time_sec\": %.16e,\n", r->solve_time);
    fprintf(f, "    \"rho_max\": %.16e,\n", r->rho_max != 0 ? r->rho_max : p->rhoMax);
    fprintf(f, "    \"heuristic_factor\": %.16e\n", p->heuristicFactor);
    fprintf(f, "  },\n");
    fprintf(f, "  \"trajectory\": {\n");
    for (int ph = 1; ph <= 2; ++ph) {
        const std::vector<int> &a = ph == 1 ? c->t1c : c->t2c, &b = ph == 1 ? c->t1o : c->t2o;
        fprintf(f, "    \"phase_%d\": {\n      \"curr_rank\": [", ph);
        for (size_t i = 0; i < a.size(); ++i) fprintf(f, "%s%lld", i ? ", " : "", (long long)a[i]);
        fprintf(f, "],\n      \"oracle_rank\": [");
        for (size_t i = 0; i < b.size(); ++i) fprintf(f, "%s%lld", i ? ", " : "", (long long)b[i]);
        fprintf(f, "]\n    }%s\n", ph == 1 ? "," : "");
    }
    fprintf(f, "  }\n}\n");
    fclose(f);
    return 0;
}

int lrs_alm_throughput(lrs_ctx *c, const lrs_params *pin, long warmup, long steps, double *seconds, long *done,
                       double *sddmm_avg_ms, double *iter_avg_ms) {
    LRS_NEED_LOADED(c);
    LRS_NEED_ARG(pin);
    // ALM iters/s: the real phase-1 control flow (lorads_alm.c:1220)
    // at fixed rank with the phase-1 exit disabled, stopped after a budget of inner
    // iterations.  Warmup = an untimed run of `warmup` iterations from the same start;
    // the timed run does exactly `steps` inner iterations.
    lrs_params prm = *pin;
    prm.phase1Tol = 1e-300;
    prm.maxALMIter = 1000000000;
    prm.skipADMM = 1;
    prm.timeSecLimit = 1e30;
    lrs_result r;
    if (warmup > 0) {
        prm.almInnerBudget = warmup;
        if (solve_impl(c, &prm, &r)) return -1;
    }
    prm.almInnerBudget = steps;
    hipEvent_t e0, e1;
    HIPC(hipEventCreate(&e0));
    HIPC(hipEventCreate(&e1));
    HIPC(hipStreamSynchronize(c->st));
    const double h0 = now_s();
    HIPC(hipEventRecord(e0, c->st));
    if (solve_impl(c, &prm, &r)) return -1;
    HIPC(hipEventRecord(e1, c->st));
    HIPC(hipEventSynchronize(e1));
    const double h1 = now_s();
    if (seconds) *seconds = h1 - h0;
    if (done) *done = r.alm_inner;
    if (iter_avg_ms) *iter_avg_ms = (h1 - h0) * 1e3 / std::max(1L, r.alm_inner);
    if (sddmm_avg_ms) {
        // A(U U^T) operator on the final iterate, same stream: SDDMM(R,R) over the pattern
        // + per-constraint gather, timed with HIP events (lrs_time_auut)
        double ms = 0;
        if (lrs_time_auut(c, 200, &ms)) return -1;
        *sddmm_avg_ms = ms;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}

int lrs_set_budget_hook(lrs_ctx *c, lrs_budget_hook hook, void *user) {
    if (!c) { set_err("null ctx"); return -1; }
    c->bhook = hook;
    c->buser = user;
    return 0;
}

int lrs_alm_last_step(lrs_ctx *c, double *out4, int *newest_pair) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(out4);
    // the control block the last inner loop stopped on: its fold is the last completed trip
    const int L = c->lbfgsL;
    const int hn = c->head == 0 ? L - 1 : c->head - 1;
    out4[0] = c->last_trip[0];
    out4[1] = c->last_trip[1];
    out4[2] = c->last_trip[2];
    if (L != 2) {   // run_inner_generic: the newest pair was copied to (S0, Y0)
        out4[3] = c->ring_beta.empty() ? 0.0 : c->ring_beta[hn];
        if (newest_pair) *newest_pair = 0;
        return 0;
    }
    out4[3] = c->beta[hn];
    if (newest_pair) *newest_pair = hn;
    return 0;
}

int lrs_sync(lrs_ctx *c) {
    if (!c) { set_err("null ctx"); return -1; }
    bind(c);
    HIPC(hipStreamSynchronize(c->st));
    return 0;
}

int lrs_profile_stages(lrs_ctx *c, const lrs_params *pin, long steps, double *stage_ms, long *done) {
    LRS_NEED_LOADED(c);
    LRS_NEED_ARG(pin);
    LRS_NEED_ARG(stage_ms);
    lrs_params prm = *pin;
    prm.phase1Tol = 1e-300;
    prm.maxALMIter = 1000000000;
    prm.skipADMM = 1;
    prm.timeSecLimit = 1e30;
    prm.almInnerBudget = steps;
    for (auto &row : c->pev)
        for (auto &e : row) HIPC(hipEventCreate(&e));
    c->prof = true;
    c->pn = 0;
    for (double &v : c->pacc) v = 0;
    lrs_result r;
    const int rc = solve_impl(c, &prm, &r);
    c->prof = false;
    for (auto &row : c->pev)
        for (auto &e : row) { (void)hipEventDestroy(e); e = nullptr; }
    if (rc) return -1;
    for (int q = 0; q < 4; ++q) stage_ms[q] = c->pn ? c->pacc[q] / c->pn : 0.0;
    if (done) *done = r.alm_inner;
    return 0;
}

int lrs_time_stages(lrs_ctx *c, int reps, double *stage_ms) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(stage_ms);
    // Per-launch durations of the split-iteration stages on the current state: each
    // stage is launched `reps` times back to back between two HIP events on the solver
    // stream.  The stages are idempotent for a fixed control block (A reads ctrl[1] and
    // writes ctrl[0]; G and B read ctrl[0]), so the repeats redo identical work.  The
    // control is set active with every exit test disabled.
    double *h = c->hpin + kHpRead;
    static_assert(2 * C_NCTRL + P_NPAR <= kHpReadN, "lrs_time_stages staging");
    HIPC(hipMemcpyAsync(h, c->W.ctrl, sizeof(double) * 2 * C_NCTRL, hipMemcpyDeviceToHost, c->st));
    HIPC(hipMemcpyAsync(h + 2 * C_NCTRL, c->W.par, sizeof(double) * P_NPAR, hipMemcpyDeviceToHost, c->st));
    HIPC(hipStreamSynchronize(c->st));
    double *ctl = h + C_NCTRL, *par = h + 2 * C_NCTRL;
    // previous control = the last one written; A folds it and continues
    for (int q = 0; q < C_NCTRL; ++q) ctl[q] = h[q];
    ctl[C_ACT2] = 1; ctl[C_EXIT2] = EXIT_NONE; ctl[C_ACTIVE] = 1; ctl[C_EXIT] = EXIT_NONE;
    if (ctl[C_PENDING] == 0) ctl[C_PENDING] = 1;
    par[P_BUDGET] = 0; par[P_RCTOL] = -1e300; par[P_PH1TOL] = -1; par[P_ENDTAU] = 0;
    HIPC(hipMemcpyAsync(c->W.ctrl + C_NCTRL, ctl, sizeof(double) * C_NCTRL, hipMemcpyHostToDevice, c->st));
    HIPC(hipMemcpyAsync(c->W.par, par, sizeof(double) * P_NPAR, hipMemcpyHostToDevice, c->st));
    double zero[LS_N] = {0, 0, 0, 0};
    HIPC(hipMemcpyAsync(c->W.lsres + LS_N, zero, sizeof(zero), hipMemcpyHostToDevice, c->st));
    AlmIterArgs a{&c->dp, &c->W, nullptr};
    // one full iteration first so that every buffer the stages read is populated
    OPC(enqueue_alm_stages(a, 0, 7, c->st));
    // profiling aid (scripts/leg_profile.sh): an idle host gap after the priming iteration and
    // after each stage's loop, so a kernel trace splits into the stages by time alone
    const char *gap_env = getenv("LRS_TIME_STAGES_GAP_US");
    const long gap_us = gap_env ? atol(gap_env) : 0;
    hipEvent_t e[4];
    for (auto &x : e) HIPC(hipEventCreate(&x));
    const int masks[3] = {1, 2, 4};
    for (int q = 0; q < 3; ++q) {
        if (gap_us > 0) {
            HIPC(hipStreamSynchronize(c->st));
            std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
        }
        HIPC(hipEventRecord(e[0], c->st));
        for (int t = 0; t < reps; ++t) OPC(enqueue_alm_stages(a, 0, masks[q], c->st));
        HIPC(hipEventRecord(e[1], c->st));
        HIPC(hipEventSynchronize(e[1]));
        float ms = 0;
        HIPC(hipEventElapsedTime(&ms, e[0], e[1]));
        stage_ms[q] = (q == 1 && c->dp.mg == 0) ? 0.0 : ms / reps;
    }
    for (auto &x : e) (void)hipEventDestroy(x);
    return 0;
}

int lrs_debug_phase_times(lrs_ctx *c, unsigned long long *out, unsigned long long *blk) {
    LRS_NEED_CTX(c);
    HIPC(hipStreamSynchronize(c->st));
    return read_phase_times(out, blk);
}

int lrs_time_auut(lrs_ctx *c, int reps, double *avg_ms) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(avg_ms);
    hipEvent_t e0, e1;
    HIPC(hipEventCreate(&e0));
    HIPC(hipEventCreate(&e1));
    HIPC(hipEventRecord(e0, c->st));
    // A(R R^T): the constraint-entry kernel, cones accumulated in cone order
    for (int q = 0; q < reps; ++q)
        for (int k = 0; k < c->dp.K; ++k)
            OPC(launch_auv_con(c->dp, k, 1, c->W.R, nullptr, 1.0, k > 0, c->W.q1, nullptr, nullptr, c->st));
    HIPC(hipEventRecord(e1, c->st));
    HIPC(hipEventSynchronize(e1));
    float ms = 0;
    HIPC(hipEventElapsedTime(&ms, e0, e1));
    *avg_ms = ms / reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}

// Standalone r x r Gram of cone `cone` on R (one k_gram launch: MFMA tiles + the
// last-arriving chunk's fixed-order reduction): reps back to back between two HIP events.
// Both outputs are that launch's average (the reduction is no longer a second kernel).
int lrs_time_dense(lrs_ctx *c, int cone, int reps, double *avg_ms) {
    if (!c || !avg_ms) { set_err("time_dense: null argument"); return -1; }
    bind(c);
    if (!c->walloc || cone < 0 || cone >= c->dp.K || !c->dp.cones[cone].dense_c) {
        set_err("time_dense: cone %d has no dense objective (or no ranks set)", cone);
        return -1;
    }
    hipEvent_t e0, e1;
    HIPC(hipEventCreate(&e0));
    HIPC(hipEventCreate(&e1));
    OPC(launch_dense_cx(c->dp, cone, c->W.R, c->W.CD, 0.0, c->st));
    HIPC(hipEventRecord(e0, c->st));
    for (int q = 0; q < reps; ++q) OPC(launch_dense_cx(c->dp, cone, c->W.R, c->W.CD, 0.0, c->st));
    HIPC(hipEventRecord(e1, c->st));
    HIPC(hipEventSynchronize(e1));
    float ms = 0;
    HIPC(hipEventElapsedTime(&ms, e0, e1));
    *avg_ms = ms / std::max(1, reps);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}

int lrs_mfma_f64_peak(lrs_ctx *c, double *tflops) {
    if (!c || !tflops) { set_err("mfma_f64_peak: null argument"); return -1; }
    bind(c);
    OPC(mfma_f64_peak(c->st, tflops));
    return 0;
}

int lrs_mfma_f64_probe(lrs_ctx *c, int waves_per_simd, int chains, double *tflops, double *mhz,
                       double *cycles_per_mfma) {
    if (!c || !tflops) { set_err("mfma_f64_probe: null argument"); return -1; }
    bind(c);
    OPC(mfma_f64_probe(c->st, waves_per_simd, chains, tflops, mhz, cycles_per_mfma));
    return 0;
}

int lrs_time_gram(lrs_ctx *c, int cone, int reps, double *avg_ms, double *gram_ms) {
    LRS_NEED_STATE(c);
    LRS_NEED_ARG(avg_ms);
    if (cone < 0 || cone >= c->dp.K) {
        set_err("time_gram: bad cone %d", cone);
        return -1;
    }
    hipEvent_t e0, e1;
    HIPC(hipEventCreate(&e0));
    HIPC(hipEventCreate(&e1));
    int nblk = 0;
    float ms = 0;
    for (int pass = 0; pass < 2; ++pass) {   // 0: MFMA kernel and reduction, 1: the MFMA kernel alone
        const bool reduce = pass == 0;
        OPC(launch_gram(c->dp, cone, c->W.R, nullptr, 0, c->W.gram, &nblk, c->st, reduce));
        HIPC(hipEventRecord(e0, c->st));
        for (int q = 0; q < reps; ++q)
            OPC(launch_gram(c->dp, cone, c->W.R, nullptr, 0, c->W.gram, &nblk, c->st, reduce));
        HIPC(hipEventRecord(e1, c->st));
        HIPC(hipEventSynchronize(e1));
        HIPC(hipEventElapsedTime(&ms, e0, e1));
        if (pass == 0) *avg_ms = ms / reps;
        else if (gram_ms) *gram_ms = ms / reps;
        if (!gram_ms) break;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}

// ---- sharded solve
int lrs_comm_unique_id(char *id_out) {
    LRS_NEED_ARG(id_out);
    ncclUniqueId id;
    NCCLC(ncclGetUniqueId(&id));
    memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

static int shard_setup(lrs_ctx *c, int world, int rank) {
    if (!c->loaded) { set_err("shard: no problem loaded"); return -1; }
    if (sharded(c)) { set_err("shard: context is already sharded"); return -1; }
    HostProblem sh;
    ShardPlan pl;
    std::string err;
    if (!shard_problem(c->hp, world, rank, sh, pl, err)) { set_err("shard: %s", err.c_str()); return -1; }
    free_work(c);
    free_problem(c->dp);
    c->loaded = false;
    c->hp = std::move(sh);
    c->plan = std::move(pl);
    if (!upload_problem(c->hp, c->dp, err)) { set_err("shard upload: %s", err.c_str()); return -1; }
    {   // shared constraints (lrs_problem.h ShardPlan): index map, primary mask, b counted once
        DevProblem &P = c->dp;
        const int m = P.m;
        std::vector<int> idx(std::max(1, m), -1);
        for (size_t q = 0; q < c->plan.shared_lid.size(); ++q)
            if (c->plan.shared_lid[q] >= 0) idx[c->plan.shared_lid[q]] = (int)q;
        std::vector<double> mk(std::max(1, m), 0.0), bp(std::max(1, m), 0.0);
        for (int i = 0; i < m; ++i) { mk[i] = c->plan.primary[i] ? 1.0 : 0.0; bp[i] = mk[i] * c->hp.b[i]; }
        P.nsh = (int)c->plan.shared_gid.size();
        const size_t ns = std::max<size_t>(1, P.nsh);
        HIPC(hipMalloc((void **)&P.sh_idx, sizeof(int) * idx.size()));
        HIPC(hipMalloc((void **)&P.cmask, sizeof(double) * mk.size()));
        HIPC(hipMalloc((void **)&P.bprim, sizeof(double) * bp.size()));
        HIPC(hipMalloc((void **)&P.g3, sizeof(double) * 3 * mk.size()));
        HIPC(hipMalloc((void **)&P.gpack, sizeof(double) * 3 * ns));
        HIPC(hipMalloc((void **)&P.spack, sizeof(double) * ns));
        HIPC(hipMemcpy(P.sh_idx, idx.data(), sizeof(int) * idx.size(), hipMemcpyHostToDevice));
        HIPC(hipMemcpy(P.cmask, mk.data(), sizeof(double) * mk.size(), hipMemcpyHostToDevice));
        HIPC(hipMemcpy(P.bprim, bp.data(), sizeof(double) * bp.size(), hipMemcpyHostToDevice));
        HIPC(hipMemset(P.g3, 0, sizeof(double) * 3 * mk.size()));
    }
    for (int k = 0; k < c->dp.K; ++k) {
        c->dp.cones[k].row0 = c->plan.cones[k].row0;
        c->dp.cones[k].nown = c->plan.cones[k].nown;
    }
    c->hooks.self = c;
    c->hooks.halo = hook_halo;
    c->hooks.allreduce = hook_allreduce;
    c->dp.shard = &c->hooks;
    c->d_send_rows.assign(c->dp.K, nullptr);
    for (int k = 0; k < c->dp.K; ++k) {
        const std::vector<int> &sr = c->plan.cones[k].send_rows;
        HIPC(hipMalloc((void **)&c->d_send_rows[k], sizeof(int) * std::max<size_t>(1, sr.size())));
        if (!sr.empty()) HIPC(hipMemcpy(c->d_send_rows[k], sr.data(), sizeof(int) * sr.size(), hipMemcpyHostToDevice));
    }
    c->init_cache.clear();
    c->init_ranks.clear();
    c->cgIterCone.assign(c->hp.K, 0);
    c->loaded = true;
    return 0;
}

int lrs_shard_rccl(lrs_ctx *c, int world, int rank, const char *id) {
    LRS_NEED_LOADED(c);
    LRS_NEED_ARG(id);
    if (world < 1 || rank < 0 || rank >= world) { set_err("lrs_shard_rccl: rank %d of world %d", rank, world); return -1; }
    // one shard is the unsharded solve: no fold / all-reduce launches per stage (they cost
    // 19 % of the G81 rate at world 1); LRS_FORCE_SHARD=1 keeps the RCCL plumbing (tests)
    const char *force = getenv("LRS_FORCE_SHARD");
    if (world == 1 && rank == 0 && !(force && atoi(force) != 0)) return 0;
    if (shard_setup(c, world, rank)) return -1;
    RcclComm *rc = new RcclComm();
    ncclUniqueId uid;
    memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    const ncclResult_t r = ncclCommInitRank(&rc->comm, world, uid, rank);
    if (r != ncclSuccess) {
        rc->comm = nullptr;
        delete rc;
        set_err("ncclCommInitRank: %s", ncclGetErrorString(r));
        return -1;
    }
    c->comm = rc;
    return 0;
}

int lrs_loopback_create(int world, lrs_loopback **out) {
    LRS_NEED_ARG(out);
    if (world < 1 || world > kMaxShards) { set_err("loopback: world %d", world); return -1; }
    lrs_loopback *g = new lrs_loopback();
    g->world = world;
    g->ev_pre.assign(world, nullptr);
    g->ev_post.assign(world, nullptr);
    g->bufs.assign(world, nullptr);
    g->sendbufs.assign(world, nullptr);
    g->plans.assign(world, nullptr);
    g->hv.assign(world, {});
    *out = g;
    return 0;
}

void lrs_loopback_destroy(lrs_loopback *g) {
    if (!g) return;
    for (auto e : g->ev_pre) if (e) (void)hipEventDestroy(e);
    for (auto e : g->ev_post) if (e) (void)hipEventDestroy(e);
    delete g;
}

int lrs_shard_loopback(lrs_ctx *c, lrs_loopback *g, int rank) {
    LRS_NEED_LOADED(c);
    if (!g || rank < 0 || rank >= g->world) { set_err("loopback: bad arguments"); return -1; }
    int rc = shard_setup(c, g->world, rank);
    if (rc == 0 && (hipEventCreateWithFlags(&g->ev_pre[rank], hipEventDisableTiming) != hipSuccess ||
                    hipEventCreateWithFlags(&g->ev_post[rank], hipEventDisableTiming) != hipSuccess)) {
        set_err("loopback: event create failed");
        rc = -1;
    }
    if (rc == 0) {
        g->plans[rank] = &c->plan;
        LoopComm *lc = new LoopComm();
        lc->g = g;
        lc->rank = rank;
        c->comm = lc;
    }
    g->barrier();   // every shard's plan is registered before the first exchange
    return rc;
}

int lrs_shard_info(lrs_ctx *c, int *world, int *rank, int *row0, int *nown, int *nhalo) {
    if (!c) { set_err("null ctx"); return -1; }
    const bool s = sharded(c);
    if (world) *world = s ? c->plan.world : 1;
    if (rank) *rank = s ? c->plan.rank : 0;
    if (row0) *row0 = s ? c->plan.cones[0].bounds[c->plan.rank] : 0;
    if (nown) *nown = s ? c->plan.cones[0].nown : (c->loaded ? c->hp.cones[0].n : 0);
    if (nhalo) *nhalo = s ? c->dp.cones[0].n - c->plan.cones[0].nown : 0;
    return 0;
}

int lrs_xwg_fallbacks(lrs_ctx *c, int *count) {
    LRS_NEED_CTX(c);
    LRS_NEED_ARG(count);
    *count = c->xwg_fallbacks;
    return 0;
}
int lrs_shard_comm_record(lrs_ctx *c, int on) {
    LRS_NEED_CTX(c);
    if (!c->comm) { set_err("lrs_shard_comm_record: the context is not sharded"); return -1; }
    c->comm->recording = on != 0;
    c->comm->log.clear();
    return 0;
}
int lrs_shard_comm_log(lrs_ctx *c, long *out, long cap, long *n) {
    LRS_NEED_CTX(c);
    LRS_NEED_ARG(n);
    if (!c->comm) { set_err("lrs_shard_comm_log: the context is not sharded"); return -1; }
    const std::vector<CommOp> &L = c->comm->log;
    *n = (long)L.size();
    if (out)
        for (long i = 0; i < std::min(cap, (long)L.size()); ++i) {
            out[5 * i] = L[i].kind; out[5 * i + 1] = L[i].peer; out[5 * i + 2] = L[i].cone;
            out[5 * i + 3] = L[i].count; out[5 * i + 4] = L[i].offset;
        }
    return 0;
}
int lrs_shard_comm_ranks(lrs_ctx *c, int *count) {
    if (!c || !count) { set_err("null argument"); return -1; }
    if (!sharded(c)) { *count = 1; return 0; }
    return c->comm->ranks(count);
}

// Host-only view of shard_problem's partition (no device, no context): the row blocks, this
// shard's local rows, its send lists per peer, the shared constraints and its local ones.
// counts[8] = {n_global, first owned global row, owned rows, local rows, send rows, shared
// constraints, local constraints, world}; any array may be null (counts first, then arrays).
int lrs_shard_plan(const char *path, int world, int rank, long *counts, int *bounds, int *local_gid,
                   int *send_ptr, int *send_gid, int *shared_gid, int *con_gid, int *primary) {
    if (!path || !counts) { set_err("null argument"); return -1; }
    HostProblem g, out;
    ShardPlan pl;
    std::string err;
    if (!read_sdpa(path, g, err)) { set_err("read_sdpa: %s", err.c_str()); return -1; }
    if (!shard_problem(g, world, rank, out, pl, err)) { set_err("shard: %s", err.c_str()); return -1; }
    const ShardConePlan &c0 = pl.cones[0];   // the row partition of cone 0 (every cone is split alike)
    counts[0] = c0.n_global; counts[1] = c0.bounds[rank]; counts[2] = c0.nown; counts[3] = (long)c0.gid.size();
    counts[4] = (long)c0.send_rows.size(); counts[5] = (long)pl.shared_gid.size(); counts[6] = (long)pl.con_gid.size();
    counts[7] = world;
    if (bounds) std::copy(c0.bounds.begin(), c0.bounds.end(), bounds);
    if (local_gid) std::copy(c0.gid.begin(), c0.gid.end(), local_gid);
    if (send_ptr) std::copy(c0.send_ptr.begin(), c0.send_ptr.end(), send_ptr);
    if (send_gid)
        for (size_t q = 0; q < c0.send_rows.size(); ++q) send_gid[q] = c0.gid[c0.send_rows[q]];
    if (shared_gid) std::copy(pl.shared_gid.begin(), pl.shared_gid.end(), shared_gid);
    if (con_gid) std::copy(pl.con_gid.begin(), pl.con_gid.end(), con_gid);
    if (primary)
        for (size_t q = 0; q < pl.primary.size(); ++q) primary[q] = pl.primary[q];
    return 0;
}

}  // extern "C"
