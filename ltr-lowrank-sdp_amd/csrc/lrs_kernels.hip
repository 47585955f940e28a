// lrs_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the low-rank SDP
// hot path.  FP64 everywhere (the reference computes in double).
//
// Row-owned kernels give each factor row to a group of G lanes (E doubles per
// lane, ld = G*E); cross-lane dot products are shuffle butterflies inside the
// group.  Scalar reductions are written as per-block partials and finalised by
// the last-arriving block (agent-scope release/acquire ticket, cdna_hip_programming
// Guideline 16), so every sum is taken in a fixed order: results are bitwise
// reproducible run to run.
//
// Operator map (reference file:line in /root/reference/lorads/src/src_semi):
//   k_sddmm      LORADSUVt sparse branch      lorads_alg/lorads_alg_common.c:51-71
//                + objAUV (<C, .>)            data/lorads_sdp_conic.c:395-402
//   k_gather     coneAUV / sparseAUV          data/lorads_sdp_conic.c:378-385, data/lorads_sdp_data.c:803-856
//   k_wsum       addObjCoeff + sdpDataWSum    data/lorads_sdp_conic.c:448-460, :608-616
//   k_spmm       mul_rk                        data/lorads_sdp_data.c:750-763
//   ALM fused iteration (device control)     lorads_alg/lorads_alm.c:1302-1379
#include <hip/hip_runtime.h>
#include <utility>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <algorithm>

#include "lrs_device.h"

namespace lrs {

static thread_local char g_err[512] = "";

// Optional in-kernel phase timestamps (block 0, thread 0; s_memrealtime, 100 MHz):
// built only into the diagnostics library (make timing -> liblrsdp_timing.so).
#ifdef LRS_PHASE_TIMING
__device__ unsigned long long g_phase[4][16];
__device__ unsigned long long g_phase_tmp[4][16];
#define LRS_TS(k, p)                                                                  \
    do {                                                                              \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_phase_tmp[k][p] = wall_clock64();  \
    } while (0)
// last phase of a kernel that ran its full path: publish the staged stamps
#define LRS_TS_END(k, p)                                                              \
    do {                                                                              \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                                    \
            g_phase_tmp[k][p] = wall_clock64();                                       \
            for (int q_ = 0; q_ <= (p); ++q_) g_phase[k][q_] = g_phase_tmp[k][q_];    \
        }                                                                             \
    } while (0)
// per-block [entry, exit] of the last full run of each split-iteration kernel
__device__ unsigned long long g_blk[4][1024][2];
#define LRS_BLK_BEGIN() const unsigned long long t_begin_ = wall_clock64()
#define LRS_BLK_END(k)                                                                 \
    do {                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < 1024) {                                   \
            g_blk[k][blockIdx.x][0] = t_begin_;                                        \
            g_blk[k][blockIdx.x][1] = wall_clock64();                                  \
        }                                                                              \
    } while (0)
#else
#define LRS_TS(k, p) do { } while (0)
#define LRS_TS_END(k, p) do { } while (0)
#define LRS_BLK_BEGIN() do { } while (0)
#define LRS_BLK_END(k) do { } while (0)
#endif
int read_phase_times(unsigned long long *out, unsigned long long *blk) {
#ifdef LRS_PHASE_TIMING
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(g_phase)) != hipSuccess) return -1;
    if (blk && hipMemcpyFromSymbol(blk, HIP_SYMBOL(g_blk), sizeof(g_blk)) != hipSuccess) return -1;
    return 64;
#else
    (void)out;
    (void)blk;
    return 0;
#endif
}
const char *last_device_error() { return g_err; }

#define LRS_CHECK_LAUNCH()                                                               \
    do {                                                                                 \
        hipError_t e_ = hipGetLastError();                                               \
        if (e_ != hipSuccess) {                                                          \
            snprintf(g_err, sizeof(g_err), "%s:%d %s", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return (int)e_;                                                              \
        }                                                                                \
    } while (0)

Layout choose_layout(int r) {
    // LRS_LAYOUT=GxE (diagnostics): that layout wherever it holds r columns
    if (const char *e = getenv("LRS_LAYOUT")) {
        int g = 0, el = 0;
        if (sscanf(e, "%dx%d", &g, &el) == 2 && (g == 8 || g == 16 || g == 32 || g == 64) && el >= 1 && el <= 4 &&
            g * el >= r) {
            Layout f;
            f.G = g; f.E = el; f.ld = g * el;
            return f;
        }
    }
    static const int Gs[4] = {8, 16, 32, 64};
    static const int Es[4] = {2, 1, 4, 3};   // preference order at equal ld
    Layout best;
    best.ld = 1 << 30;
    for (int ei = 0; ei < 4; ++ei)
        for (int gi = 0; gi < 4; ++gi) {
            int ld = Gs[gi] * Es[ei];
            if (ld >= r && ld < best.ld) { best.G = Gs[gi]; best.E = Es[ei]; best.ld = ld; }
        }
    // ranks 257..512 (AUG_RANK's rank_max = sqrt(2 nnzRows) + 1 exceeds 256 on e.g. theta102,
    // MC_500): full waves per row, 8 doubles per lane
    if (best.ld > 512 && r <= 512) { best.G = 64; best.E = 8; best.ld = 512; }
    return best;
}

// ------------------------------------------------------------------------
// small device helpers
// ------------------------------------------------------------------------
// DPP lane moves on the two 32-bit halves of a double (no LDS round trip, unlike
// __shfl_xor's ds_bpermute).  CTRL: 0xB1 quad_perm[1,0,3,2] (xor 1), 0x4E
// quad_perm[2,3,0,1] (xor 2), 0x141 row_half_mirror (i <-> 7-i in 8 lanes),
// 0x140 row_mirror (i <-> 15-i in 16 lanes).
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// A copy of x the compiler cannot prove equal to x.  k_bw_b meets the diagonal entry with the
// row's own registers where k_it_b loads the row again; a dot of a row with itself is then known
// non-negative, which lets the compiler fold the "0 +" of the sum and fuse the other product (one
// ulp off on a diagonal slot's value, seen on a restructured stage-A kernel; profiles/r06j).
// Opaque, the operand compiles as k_it_b's does: bitwise the same results.
__device__ __forceinline__ double opaque(double x) {
    asm volatile("" : "+v"(x));
    return x;
}

// Sum over an aligned group of G lanes; every lane of the group gets the same value.
template <int G>
__device__ __forceinline__ double group_sum(double v) {
    v += dpp_mov<0xB1>(v);
    v += dpp_mov<0x4E>(v);
    if constexpr (G >= 8) v += dpp_mov<0x141>(v);
    if constexpr (G >= 16) v += dpp_mov<0x140>(v);
    if constexpr (G >= 32) v += __shfl_xor(v, 16, 64);
    if constexpr (G >= 64) v += __shfl_xor(v, 32, 64);
    return v;
}

// Four dot products reduced over an aligned group of G = 4 or 16 lanes by a transposed
// butterfly: each exchange step halves the values a lane holds (G = 4: xor 2, xor 1; G = 16:
// row_mirror, row_half_mirror, then the quad sums), so four sums cost 3 (G = 4) or 5 (G = 16)
// double moves instead of 8 / 16.  Returns entry q's total in the lanes whose group offset
// o satisfies q = o / (G / 4) (G = 4: lane o holds entry o).
template <int G>
__device__ __forceinline__ double group_sum4(const double (&d)[4], int o) {
    static_assert(G == 4 || G == 16, "group of 4 or 16 lanes");
    if constexpr (G == 4) {
        const bool h1 = (o & 2) != 0, h0 = (o & 1) != 0;
        double a0 = h1 ? d[2] : d[0], a1 = h1 ? d[3] : d[1];
        a0 += dpp_mov<0x4E>(h1 ? d[0] : d[2]);
        a1 += dpp_mov<0x4E>(h1 ? d[1] : d[3]);
        return (h0 ? a1 : a0) + dpp_mov<0xB1>(h0 ? a0 : a1);
    } else {
        const bool h3 = (o & 8) != 0, h2 = (o & 4) != 0;
        double a0 = h3 ? d[2] : d[0], a1 = h3 ? d[3] : d[1];
        a0 += dpp_mov<0x140>(h3 ? d[0] : d[2]);
        a1 += dpp_mov<0x140>(h3 ? d[1] : d[3]);
        double v = (h2 ? a1 : a0) + dpp_mov<0x141>(h2 ? a0 : a1);
        v += dpp_mov<0x4E>(v);
        v += dpp_mov<0xB1>(v);
        return v;
    }
}

__device__ __forceinline__ double read_lane(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Value of lane u of this lane's aligned group of G lanes (u group-uniform)
template <int G>
__device__ __forceinline__ int bcast_i(int v, int u) {
    if constexpr (G == 64) return __builtin_amdgcn_readlane(v, u);
    else return __shfl(v, (int)(threadIdx.x & 63 & ~(G - 1)) + u, 64);
}
template <int G>
__device__ __forceinline__ double bcast_d(double v, int u) {
    if constexpr (G == 64) return read_lane(v, u);
    else return __shfl(v, (int)(threadIdx.x & 63 & ~(G - 1)) + u, 64);
}

// Wave (64-lane) sum, wave-uniform result: DPP within rows of 16, then the four
// row sums through readlane.
__device__ __forceinline__ double wave_sum(double v) {
    v = group_sum<16>(v);
    return (read_lane(v, 0) + read_lane(v, 16)) + (read_lane(v, 32) + read_lane(v, 48));
}

template <int E>
__device__ __forceinline__ void ld_row(const double *__restrict__ p, double (&v)[E]) {
    if constexpr (E == 2) {
        double2 t = *reinterpret_cast<const double2 *>(p);
        v[0] = t.x; v[1] = t.y;
    } else if constexpr (E == 4) {
        double2 t0 = reinterpret_cast<const double2 *>(p)[0];
        double2 t1 = reinterpret_cast<const double2 *>(p)[1];
        v[0] = t0.x; v[1] = t0.y; v[2] = t1.x; v[3] = t1.y;
    } else {
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = p[e];
    }
}

template <int E>
__device__ __forceinline__ void st_row(double *__restrict__ p, const double (&v)[E]) {
    if constexpr (E == 2) {
        *reinterpret_cast<double2 *>(p) = make_double2(v[0], v[1]);
    } else if constexpr (E == 4) {
        reinterpret_cast<double2 *>(p)[0] = make_double2(v[0], v[1]);
        reinterpret_cast<double2 *>(p)[1] = make_double2(v[2], v[3]);
    } else {
#pragma unroll
        for (int e = 0; e < E; ++e) p[e] = v[e];
    }
}

// Block-reduce NV per-thread accumulators; thread 0 gets the block sums in s[].
template <int NV, int NT = kBlock>
__device__ __forceinline__ void block_reduce(double (&acc)[NV], double (&s)[NV]) {
    __shared__ double sh[NV][NT / 64];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        double t = wave_sum(acc[v]);
        if (lane == 0) sh[v][wid] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            double t = 0.0;
#pragma unroll
            for (int w = 0; w < NT / 64; ++w) t += sh[v][w];
            s[v] = t;
        }
    }
    __syncthreads();
}

// Write this block's partials; the last-arriving block sums all partials in
// block order and stores fin[0..NV).  Release/acquire per Guideline 16.
template <int NV>
__device__ void partials_finalize(double (&acc)[NV], double *__restrict__ part, unsigned *ticket,
                                  double *__restrict__ fin, int *inc = nullptr) {
    double s[NV];
    block_reduce<NV>(acc, s);
    __shared__ unsigned is_last;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v) part[v * kMaxPartialBlocks + blockIdx.x] = s[v];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = (t == gridDim.x - 1) ? 1u : 0u;
    }
    __syncthreads();
    if (!is_last) return;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    double a2[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        double t = 0.0;
        for (int b = threadIdx.x; b < (int)gridDim.x; b += kBlock) t += part[v * kMaxPartialBlocks + b];
        a2[v] = t;
    }
    double s2[NV];
    block_reduce<NV>(a2, s2);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v) fin[v] = s2[v];
        if (inc) *inc = *inc + 1;   // a step counter the next launch reads (every block has read it)
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

static inline int grid_rows(long rows, int G) {
    long threads = rows * G;
    long b = (threads + kBlock - 1) / kBlock;
    if (b < 1) b = 1;
    if (b > kMaxPartialBlocks) b = kMaxPartialBlocks;
    return (int)b;
}
static inline int grid_elems(long n, int per_thread) {
    long b = (n / per_thread + kBlock - 1) / kBlock;
    if (b < 1) b = 1;
    if (b > kMaxPartialBlocks) b = kMaxPartialBlocks;
    return (int)b;
}

// ------------------------------------------------------------------------
// Tickets / finals of the standalone reductions: per-context device scratch (lrs_ctx
// s_tickets / s_tmpfin / s_fin / s_rpart), bound to the calling thread by bind_scratch --
// no module-level device state, so contexts on several host threads never share it
// ------------------------------------------------------------------------
enum TicketId { T_SDDMM = 0, T_GATHER, T_SPMM, T_DOT, T_GRAD, T_RR, T_Q, T_NT = 16 };

// ------------------------------------------------------------------------
// SDDMM over the lower pattern (row-owned).  MODE 0: sym(X Y^T); MODE 1: X X^T;
// MODE 2: sym(X Y^T) -> out0 and Y Y^T -> out1.  Objective partials with Cw.
// ------------------------------------------------------------------------
template <int G, int E, int MODE>
__global__ void __launch_bounds__(kBlock) k_sddmm(int n, int ld, const int *__restrict__ adj_ptr,
                                                  const int *__restrict__ adj_low, const int *__restrict__ adj_col,
                                                  const int *__restrict__ adj_slot, const double *__restrict__ X,
                                                  const double *__restrict__ Y, double *__restrict__ out0,
                                                  double *__restrict__ out1, const double *__restrict__ Cw,
                                                  double *part, unsigned *ticket, double *fin,
                                                  const double *__restrict__ guard, int row0, int T) {
    if (guard && guard[C_ACTIVE] == 0.0) return;
    // teams of T lane groups per row (dense rows): member `mem` takes entries mem, mem + T, ...
    const int lane = threadIdx.x & (G - 1);
    const int grp = (blockIdx.x * kBlock + threadIdx.x) / G;
    const int ngrp = gridDim.x * kBlock / G;
    const int mem = grp % T;
    double acc[2] = {0.0, 0.0};
    for (int i = row0 + grp / T; i < row0 + n; i += ngrp / T) {
        double xi[E], yi[E];
        ld_row<E>(X + (long)i * ld + lane * E, xi);
        if constexpr (MODE != 1) ld_row<E>(Y + (long)i * ld + lane * E, yi);
        const int kb = adj_ptr[i], ke = adj_low[i];
        for (int k = kb + mem; k < ke; k += T) {
            const int j = adj_col[k];
            const int s = adj_slot[k];
            double xj[E];
            ld_row<E>(X + (long)j * ld + lane * E, xj);
            if constexpr (MODE == 1) {
                double d = 0.0;
#pragma unroll
                for (int e = 0; e < E; ++e) d += xi[e] * xj[e];
                d = group_sum<G>(d);
                if (lane == 0) { out0[s] = d; acc[0] += Cw[s] * d; }
            } else {
                double yj[E];
                ld_row<E>(Y + (long)j * ld + lane * E, yj);
                double d0 = 0.0, d1 = 0.0;
                if (j != i) {
#pragma unroll
                    for (int e = 0; e < E; ++e) d0 += xi[e] * yj[e] + xj[e] * yi[e];
                    d0 *= 0.5;
                } else {
#pragma unroll
                    for (int e = 0; e < E; ++e) d0 += xi[e] * yi[e];
                }
                d0 = group_sum<G>(d0);
                if constexpr (MODE == 2) {
#pragma unroll
                    for (int e = 0; e < E; ++e) d1 += yi[e] * yj[e];
                    d1 = group_sum<G>(d1);
                }
                if (lane == 0) {
                    out0[s] = d0;
                    acc[0] += Cw[s] * d0;
                    if constexpr (MODE == 2) { out1[s] = d1; acc[1] += Cw[s] * d1; }
                }
            }
        }
    }
    partials_finalize<2>(acc, part, ticket, fin);
}

// ------------------------------------------------------------------------
// Gather A(uvt): one thread per constraint (cone < 0: all cones, summed in
// cone order like LORADSInitConstrValSum).  out = scale * value.
// Optional residual partial sum((b - out)^2).
// ------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_gather(int m, int K, int cone, const int *__restrict__ con_ptr,
                                                   const int *__restrict__ con_slot, const double *__restrict__ con_w,
                                                   const double *__restrict__ uvt, double scale,
                                                   double *__restrict__ out, const double *__restrict__ b,
                                                   double *part, unsigned *ticket, double *fin) {
    double acc[1] = {0.0};
    const int k0 = cone < 0 ? 0 : cone, k1 = cone < 0 ? K : cone + 1;
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < m; i += gridDim.x * kBlock) {
        double tot = 0.0;
        for (int k = k0; k < k1; ++k) {
            const long row = (long)k * m + i;
            double v = 0.0;
            int e = con_ptr[row];
            const int e1 = con_ptr[row + 1];
            // long rows (a trace constraint): eight entries' loads in flight, the sum in entry order
            for (; e + 8 <= e1; e += 8) {
                int sl[8];
                double w[8], u[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) { sl[t] = con_slot[e + t]; w[t] = con_w[e + t]; }
#pragma unroll
                for (int t = 0; t < 8; ++t) u[t] = uvt[sl[t]];
#pragma unroll
                for (int t = 0; t < 8; ++t) v += w[t] * u[t];
            }
            for (; e < e1; ++e) v += con_w[e] * uvt[con_slot[e]];
            tot += v;
        }
        tot *= scale;
        out[i] = tot;
        if (b) { double d = b[i] - tot; acc[0] += d * d; }
    }
    if (part) partials_finalize<1>(acc, part, ticket, fin);
}

// Constraint-entry A(X Y^T) (LORADSUpdateConstrValCG lorads_admm.c:442-459 /
// coneAUV data/lorads_sdp_conic.c:378-385 without materialising the pattern): one
// lane group per constraint, each entry (p, q) of cone k read as two factor rows.
template <int E, int MODE>
__device__ __forceinline__ double auv_entry(const double *__restrict__ X, const double *__restrict__ Y, int ld,
                                            int lane, int p, int q) {
    double xp[E];
    ld_row<E>(X + (long)p * ld + lane * E, xp);
    double d = 0.0;
    if (p == q) {
        if constexpr (MODE == 1) {
#pragma unroll
            for (int t = 0; t < E; ++t) d += xp[t] * xp[t];
        } else {
            double yp[E];
            ld_row<E>(Y + (long)p * ld + lane * E, yp);
#pragma unroll
            for (int t = 0; t < E; ++t) d += xp[t] * yp[t];
        }
    } else {
        double xq[E];
        ld_row<E>(X + (long)q * ld + lane * E, xq);
        if constexpr (MODE == 1) {
#pragma unroll
            for (int t = 0; t < E; ++t) d += xp[t] * xq[t];
        } else {
            double yp[E], yq[E];
            ld_row<E>(Y + (long)p * ld + lane * E, yp);
            ld_row<E>(Y + (long)q * ld + lane * E, yq);
#pragma unroll
            for (int t = 0; t < E; ++t) d += xp[t] * yq[t] + xq[t] * yp[t];
            d *= 0.5;
        }
    }
    return d;
}

// Long constraint rows (> kLongRow entries in this cone, e.g. a trace constraint): a
// block per constraint, its kBlock/G lane groups striding over the entries (two entries'
// loads in flight per group; the sum keeps the entry order).
template <int G, int E, int MODE>
__device__ __forceinline__ void auv_long_rows(int blk, int nblk, int nlong, const int *__restrict__ long_rows,
                                              int m, int cone, int ld, const int *__restrict__ con_ptr,
                                              const int *__restrict__ con_slot, const double *__restrict__ con_w,
                                              const int *__restrict__ slot_rc, const double *__restrict__ X,
                                              const double *__restrict__ Y, double scale, int accumulate,
                                              double *__restrict__ out, double *__restrict__ sum_upd) {
    __shared__ double wsum4[kBlock / 64];
    constexpr int NG = kBlock / G;   // lane groups of the block, striding over the entries
    const int lane = threadIdx.x & (G - 1);
    const int gq = threadIdx.x / G;
    for (int t = blk; t < nlong; t += nblk) {   // block-uniform
        const int i = long_rows[t];
        const long row = (long)cone * m + i;
        const int e0 = con_ptr[row], e1 = con_ptr[row + 1];
        double v = 0.0;
        for (int e = e0 + gq; e < e1; e += 2 * NG) {
            // two entries' loads in flight, summed in entry order (group-uniform has1)
            const bool has1 = e + NG < e1;
            const int s0 = con_slot[e], s1 = has1 ? con_slot[e + NG] : s0;
            double d0 = auv_entry<E, MODE>(X, Y, ld, lane, slot_rc[2 * s0], slot_rc[2 * s0 + 1]);
            double d1 = auv_entry<E, MODE>(X, Y, ld, lane, slot_rc[2 * s1], slot_rc[2 * s1 + 1]);
            d0 = group_sum<G>(d0);
            d1 = group_sum<G>(d1);
            v += con_w[e] * d0;
            if (has1) v += con_w[e + NG] * d1;
        }
        v = wave_sum(lane == 0 ? v : 0.0);
        if ((threadIdx.x & 63) == 0) wsum4[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            double w = 0.0;
            for (int q = 0; q < kBlock / 64; ++q) w += wsum4[q];
            double tot = w * scale;
            if (accumulate) tot = out[i] + tot;
            if (sum_upd) sum_upd[i] = (sum_upd[i] - out[i]) + tot;
            out[i] = tot;
        }
        __syncthreads();
    }
}

template <int G, int E, int MODE>
__global__ void __launch_bounds__(kBlock) k_auv_con(int m, int K, int cone, int ld, const int *__restrict__ con_ptr,
                                                    const int *__restrict__ con_slot,
                                                    const double *__restrict__ con_w, const int *__restrict__ slot_rc,
                                                    const int *__restrict__ con1_pq, const double *__restrict__ con1_w,
                                                    const double *__restrict__ X, const double *__restrict__ Y,
                                                    double scale, int accumulate, double *__restrict__ out,
                                                    const double *__restrict__ b, double *part, unsigned *ticket,
                                                    double *fin, const double *__restrict__ guard, int nrowblk,
                                                    int nlong, const int *__restrict__ long_rows,
                                                    double *__restrict__ sum_upd) {
    if (guard && guard[0] == 0.0) return;
    double acc[1] = {0.0};
    if ((int)blockIdx.x >= nrowblk) {
        // the blocks past the row blocks take the long rows (one launch for both)
        auv_long_rows<G, E, MODE>(blockIdx.x - nrowblk, gridDim.x - nrowblk, nlong, long_rows, m, cone, ld, con_ptr,
                                  con_slot, con_w, slot_rc, X, Y, scale, accumulate, out, sum_upd);
        if (part) partials_finalize<1>(acc, part, ticket, fin);
        return;
    }
    const int lane = threadIdx.x & (G - 1);
    const int grp = (blockIdx.x * kBlock + threadIdx.x) / G;
    const int ngrp = nrowblk * kBlock / G;
    for (int i = grp; i < m; i += ngrp) {
        const long row = (long)cone * m + i;
        const int2 pq = reinterpret_cast<const int2 *>(con1_pq)[row];
        if (pq.x == -2) continue;   // long row: the blocks past nrowblk
        double v = 0.0;
        if (pq.x >= 0) {
            // single-entry row: (p, q, w) in one coalesced load, then the factor rows
            const double w = con1_w[row];
            double d = auv_entry<E, MODE>(X, Y, ld, lane, pq.x, pq.y);
            d = group_sum<G>(d);
            v += w * d;
        } else {
            const int e0 = con_ptr[row], e1 = con_ptr[row + 1];
            for (int e = e0; e < e1; ++e) {
                const int s = con_slot[e];
                const int p = slot_rc[2 * s], q = slot_rc[2 * s + 1];
                double d = auv_entry<E, MODE>(X, Y, ld, lane, p, q);
                d = group_sum<G>(d);
                v += con_w[e] * d;
            }
        }
        if (lane == 0) {
            double tot = v * scale;
            if (accumulate) tot = out[i] + tot;
            if (sum_upd) sum_upd[i] = (sum_upd[i] - out[i]) + tot;   // sum += new - old
            out[i] = tot;
            if (b) { const double dd = b[i] - tot; acc[0] += dd * dd; }
        }
    }
    if (part) partials_finalize<1>(acc, part, ticket, fin);
}

// A(X Y^T) of a cone whose constraint i is the single entry (i, i) (DevCone::auv_diag,
// MaxCut's diag(X) = 1): out[i] = w_i d(i, i), the row-wise dot product of X and Y -- no
// (p, q) index load in front of the factor rows, and kDiagU rows per lane group with their
// loads issued together, so one memory trip covers them.  Same lane-group layout and
// group_sum as k_auv_con (values equal up to the FMA contraction of the lane sums).  G81-like
// (n = m = 2e4, r = 64, 10.8 MB), back-to-back launches between HIP events: U = 2 rows per
// group at 256 threads 2.85-3.04 us, U = 1 3.5-3.8, U = 4 3.3-3.4, U = 8 4.2-4.3; 512 / 1024
// threads no better (scripts/auut_probe.py; LRS_DIAG_U / LRS_DIAG_BS select them).
constexpr int kDiagU = 2;
template <int G, int E, int MODE, int kDiagU, int BS>
__global__ void __launch_bounds__(BS) k_auv_diag(int m, long wbase, int ld, const double *__restrict__ con1_w,
                                                     const double *__restrict__ X, const double *__restrict__ Y,
                                                     double scale, int accumulate, double *__restrict__ out,
                                                     const double *__restrict__ b, double *part, unsigned *ticket,
                                                     double *fin, const double *__restrict__ guard,
                                                     double *__restrict__ sum_upd) {
    if (guard && guard[0] == 0.0) return;
    double acc[1] = {0.0};
    const int lane = threadIdx.x & (G - 1);
    const int grp = (blockIdx.x * BS + threadIdx.x) / G;
    const int ngrp = gridDim.x * BS / G;
    for (int i0 = grp; i0 < m; i0 += kDiagU * ngrp) {
        double xv[kDiagU][E], yv[kDiagU][E], w[kDiagU];
#pragma unroll
        for (int u = 0; u < kDiagU; ++u) {
            const int i = min(i0 + u * ngrp, m - 1);
            const long o = (long)i * ld + lane * E;
            ld_row<E>(X + o, xv[u]);
            if (MODE == 0) ld_row<E>(Y + o, yv[u]);
            w[u] = con1_w[wbase + i];
        }
#pragma unroll
        for (int u = 0; u < kDiagU; ++u) {
            const int i = i0 + u * ngrp;
            double d = 0.0;
#pragma unroll
            for (int e = 0; e < E; ++e) d += MODE == 1 ? xv[u][e] * xv[u][e] : xv[u][e] * yv[u][e];
            d = group_sum<G>(d);
            if (lane == 0 && i < m) {
                double tot = (w[u] * d) * scale;
                if (accumulate) tot = out[i] + tot;
                if (sum_upd) sum_upd[i] = (sum_upd[i] - out[i]) + tot;
                out[i] = tot;
                if (b) { const double dd = b[i] - tot; acc[0] += dd * dd; }
            }
        }
    }
    if (part) partials_finalize<1>(acc, part, ticket, fin);
}

// A(X Y^T) over 2-D tiles (cones with many constraint entries per row, e.g. C5's 600):
// the per-entry gather above reads two (MODE 1) or four (MODE 0) 8r-byte factor rows per
// entry from L2 / Infinity Cache, ~12 GB per C5 launch for 118 MB of operands.  Here a
// work item is one (row tile I, column tile J) of kAuvT rows each and up to kAuvItem of the
// entries that fall in it; the block stages the tiles' factor rows kAuvC columns at a time in
// LDS (rows padded to kAuvC + 2 doubles against bank conflicts, read 16 B at a time) and
// every thread accumulates its entries' dot products from there, so each factor row crosses
// L2 once per tile instead of once per entry.  The entry value d(p, q) is what auv_entry computes (MODE 1 X_p.X_q,
// MODE 0 (X_p.Y_q + X_q.Y_p) / 2), stored at the entry's place in the cone's constraint entry
// order; k_auv_tsum then sums each constraint's entries in entry order like k_auv_con.
// Staged tiles in LDS: tl[0] = X_I, tl[1] = X_J, tl[2] = Y_I, tl[3] = Y_J, rows I0.., J0..
// (kAuvT each) of X (and Y), columns [c0, c0 + kAuvC), zero past n rows and r columns.
constexpr int kAuvS = kAuvC + 2;   // LDS row stride (doubles; 16-B aligned rows, 4 banks apart)

// Staging split in two so that the next chunk's loads are in flight while the current one
// is computed: auv_fetch into registers, auv_put into LDS (after a barrier).
constexpr int kAuvPer = kAuvT * kAuvC / 2 / kAuvThreads;   // double2 per thread per operand
static_assert(kAuvPer * kAuvThreads * 2 == kAuvT * kAuvC, "tile staging divides evenly");
template <int NT>
constexpr int auv_per() { return kAuvT * kAuvC / 2 / NT; }   // double2 per thread per operand, NT threads
template <int NA, int NT = kAuvThreads>
__device__ __forceinline__ void auv_fetch(double2 (&v)[NA][auv_per<NT>()], int I0, int J0, int c0, int n, int r,
                                          int ld, const double *__restrict__ X, const double *__restrict__ Y) {
#pragma unroll
    for (int k = 0; k < auv_per<NT>(); ++k) {
        const int x = threadIdx.x + k * NT;
        const int row = x / (kAuvC / 2), col = c0 + 2 * (x % (kAuvC / 2));
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            const int grow = ((a & 1) ? J0 : I0) + row;
            const double *src = (a < 2) ? X : Y;
            double2 t = make_double2(0.0, 0.0);
            if (grow < n && col < r) {
                t = *reinterpret_cast<const double2 *>(src + (long)grow * ld + col);
                if (col + 1 >= r) t.y = 0.0;
            }
            v[a][k] = t;
        }
    }
}
template <int NA, int NT = kAuvThreads>
__device__ __forceinline__ void auv_put(double (*tl)[kAuvT * kAuvS], const double2 (&v)[NA][auv_per<NT>()]) {
#pragma unroll
    for (int k = 0; k < auv_per<NT>(); ++k) {
        const int x = threadIdx.x + k * NT;
        const int o = (x / (kAuvC / 2)) * kAuvS + 2 * (x % (kAuvC / 2));
#pragma unroll
        for (int a = 0; a < NA; ++a) *reinterpret_cast<double2 *>(&tl[a][o]) = v[a][k];
    }
}

// One staged column chunk of an entry (p, q): MODE 1 X_p.X_q, MODE 0 X_p.Y_q + X_q.Y_p,
// MODE 2 both of MODE 0 (into s) and Y_p.Y_q (into s2).
template <int MODE>
__device__ __forceinline__ void auv_chunk(const double (*tl)[kAuvT * kAuvS], int pl, int ql, double &s, double &s2) {
    const double2 *xa = reinterpret_cast<const double2 *>(&tl[0][pl]);
    const double2 *xb = reinterpret_cast<const double2 *>(&tl[1][ql]);
    if constexpr (MODE == 1) {
#pragma unroll 8
        for (int c = 0; c < kAuvC / 2; ++c) {
            const double2 a = xa[c], b = xb[c];
            s += a.x * b.x;
            s += a.y * b.y;
        }
    } else {
        const double2 *ya = reinterpret_cast<const double2 *>(&tl[2][pl]);
        const double2 *yb = reinterpret_cast<const double2 *>(&tl[3][ql]);
#pragma unroll 8
        for (int c = 0; c < kAuvC / 2; ++c) {
            const double2 a = xa[c], b = xb[c], ay = ya[c], by = yb[c];
            s += a.x * by.x + b.x * ay.x;
            s += a.y * by.y + b.y * ay.y;
            if constexpr (MODE == 2) {
                s2 += ay.x * by.x;
                s2 += ay.y * by.y;
            }
        }
    }
}

template <int MODE>
__global__ void __launch_bounds__(kAuvThreads) k_auv_tile(int n, int r, int ld, const int4 *__restrict__ items,
                                                          const unsigned *__restrict__ pq,
                                                          const int *__restrict__ ent,
                                                          const double *__restrict__ X,
                                                          const double *__restrict__ Y, double *__restrict__ val,
                                                          const double *__restrict__ guard) {
    if (guard && guard[0] == 0.0) return;
    constexpr int NA = MODE == 0 ? 4 : 2;           // staged operands: Xa, Xb (+ Ya, Yb)
    __shared__ double tl[NA][kAuvT * kAuvS];
    const int4 it = items[blockIdx.x];
    const int I0 = it.x, J0 = it.y, eb = it.z, ee = it.w;
    int pl[kAuvNpt], ql[kAuvNpt];
    double acc[kAuvNpt];
#pragma unroll
    for (int j = 0; j < kAuvNpt; ++j) {
        const int t = eb + (int)threadIdx.x + j * kAuvThreads;
        const unsigned w = t < ee ? pq[t] : 0u;
        pl[j] = (int)(w >> 16) * kAuvS;
        ql[j] = (int)(w & 0xffffu) * kAuvS;
        acc[j] = 0.0;
    }
    double2 pre[NA][kAuvPer];
    auv_fetch<NA>(pre, I0, J0, 0, n, r, ld, X, Y);
    for (int c0 = 0; c0 < r; c0 += kAuvC) {
        __syncthreads();
        auv_put<NA>(tl, pre);
        __syncthreads();
        if (c0 + kAuvC < r) auv_fetch<NA>(pre, I0, J0, c0 + kAuvC, n, r, ld, X, Y);   // in flight meanwhile
#pragma unroll
        for (int j = 0; j < kAuvNpt; ++j) {
            if (eb + (int)threadIdx.x + j * kAuvThreads >= ee) break;
            double unused = 0.0;
            auv_chunk<MODE>(tl, pl[j], ql[j], acc[j], unused);
        }
    }
#pragma unroll
    for (int j = 0; j < kAuvNpt; ++j) {
        const int t = eb + (int)threadIdx.x + j * kAuvThreads;
        if (t < ee) val[ent[t]] = MODE == 0 ? 0.5 * acc[j] : acc[j];
    }
}

// Per constraint of the cone: sum of w_e d_e over its entries in entry order, then k_auv_con's row epilogue (scale, accumulate, sum_upd, the
// residual partial against b).
__global__ void __launch_bounds__(kBlock) k_auv_tsum(int m, int cone, const int *__restrict__ con_ptr,
                                                     const double *__restrict__ con_w, long ebase,
                                                     const double *__restrict__ val,
                                                     double scale, int accumulate, double *__restrict__ out,
                                                     const double *__restrict__ b, double *part, unsigned *ticket,
                                                     double *fin, const double *__restrict__ guard,
                                                     double *__restrict__ sum_upd) {
    if (guard && guard[0] == 0.0) return;
    double acc[1] = {0.0};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < m; i += gridDim.x * kBlock) {
        const long row = (long)cone * m + i;
        const int e0 = con_ptr[row], e1 = con_ptr[row + 1];
        double v = 0.0;
        const double *vr = val - ebase;
        for (int e = e0; e < e1; ++e) v += con_w[e] * vr[e];
        double tot = v * scale;
        if (accumulate) tot = out[i] + tot;
        if (sum_upd) sum_upd[i] = (sum_upd[i] - out[i]) + tot;
        out[i] = tot;
        if (b) { const double dd = b[i] - tot; acc[0] += dd * dd; }
    }
    if (part) partials_finalize<1>(acc, part, ticket, fin);
}

// S[slot] = (withC ? Craw : 0) + sum w[con] a
__global__ void __launch_bounds__(kBlock) k_wsum(int Ptot, const int *__restrict__ slot_ptr,
                                                 const int *__restrict__ slot_con, const double *__restrict__ slot_a,
                                                 const double *__restrict__ Craw, int withC,
                                                 const double *__restrict__ w, double *__restrict__ S,
                                                 const double *__restrict__ guard, const double *__restrict__ lsguard) {
    if (guard && guard[C_ACTIVE] == 0.0) return;
    if (lsguard && lsguard[LS_FLAG] != 0.0) return;
    for (int s = blockIdx.x * kBlock + threadIdx.x; s < Ptot; s += gridDim.x * kBlock) {
        double v = withC ? Craw[s] : 0.0;
        for (int e = slot_ptr[s]; e < slot_ptr[s + 1]; ++e) v += w[slot_con[e]] * slot_a[e];
        S[s] = v;
    }
}

// out = scale * S X + addScale * addX (row-owned symmetric SpMM), partial ||out||^2
template <int G, int E>
__global__ void __launch_bounds__(kBlock) k_spmm(int n, int ld, const int *__restrict__ adj_ptr,
                                                 const int *__restrict__ adj_col, const int *__restrict__ adj_slot,
                                                 const double *__restrict__ S, const double *__restrict__ X,
                                                 double scale, const double *__restrict__ addX, double addScale,
                                                 double *__restrict__ out, double *part, unsigned *ticket,
                                                 double *fin, int row0, int T) {
    // teams of T lane groups per row (dense rows): members take interleaved entries, their
    // partial rows meet in LDS and member 0 sums them in member order (T = 1: no LDS step)
    __shared__ double gsh[kBlock * E];
    const int lane = threadIdx.x & (G - 1);
    const int gib = threadIdx.x / G;
    const int tpb = (kBlock / G) / T;
    const int tl = gib / T, mem = gib % T;
    double nrm[1] = {0.0};
    for (int ib = row0 + blockIdx.x * tpb; ib < row0 + n; ib += gridDim.x * tpb) {   // block-uniform
        const int i = ib + tl;
        const bool valid = i < row0 + n;
        double acc[E];
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = 0.0;
        if (valid)
            for (int k = adj_ptr[i] + mem; k < adj_ptr[i + 1]; k += T) {
                const double sv = S[adj_slot[k]];
                double xj[E];
                ld_row<E>(X + (long)adj_col[k] * ld + lane * E, xj);
#pragma unroll
                for (int e = 0; e < E; ++e) acc[e] += sv * xj[e];
            }
        if (T > 1) {
#pragma unroll
            for (int e = 0; e < E; ++e) gsh[threadIdx.x * E + e] = acc[e];
            __syncthreads();
            if (mem == 0) {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    double t = 0.0;
                    for (int q = 0; q < T; ++q) t += gsh[((tl * T + q) * G + lane) * E + e];
                    acc[e] = t;
                }
            }
            __syncthreads();
        }
        if (!valid || mem != 0) continue;
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] *= scale;
        if (addX) {
            double a[E];
            ld_row<E>(addX + (long)i * ld + lane * E, a);
#pragma unroll
            for (int e = 0; e < E; ++e) acc[e] += addScale * a[e];
        }
        st_row<E>(out + (long)i * ld + lane * E, acc);
#pragma unroll
        for (int e = 0; e < E; ++e) nrm[0] += acc[e] * acc[e];
    }
    if (part) partials_finalize<1>(nrm, part, ticket, fin);
}

// ---------------------------- BLAS-1 -------------------------------------
__global__ void __launch_bounds__(kBlock) k_axpby(long n, double a, const double *__restrict__ x, double b,
                                                  double *__restrict__ y) {
    for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long)gridDim.x * kBlock)
        y[i] = a * x[i] + b * y[i];
}
__global__ void __launch_bounds__(kBlock) k_fill(long n, double v, double *__restrict__ x) {
    for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long)gridDim.x * kBlock) x[i] = v;
}
__global__ void __launch_bounds__(kBlock) k_dot(long n, const double *__restrict__ x, const double *__restrict__ y,
                                                double *part, unsigned *ticket, double *fin) {
    double acc[1] = {0.0};
    for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long)gridDim.x * kBlock) acc[0] += x[i] * y[i];
    partials_finalize<1>(acc, part, ticket, fin);
}
__global__ void __launch_bounds__(kBlock) k_dual_update(int m, double rho, const double *__restrict__ b,
                                                        double *__restrict__ lam, const double *__restrict__ cvs) {
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < m; i += gridDim.x * kBlock) {
        double l = lam[i] + rho * b[i];      // lorads_alg_common.c:521
        lam[i] = l + (-rho) * cvs[i];        // :523
    }
}
__global__ void __launch_bounds__(kBlock) k_alm_m1(int m, double rho, const double *__restrict__ b,
                                                   const double *__restrict__ lam, const double *__restrict__ cvs,
                                                   double *__restrict__ M1) {
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < m; i += gridDim.x * kBlock)
        M1[i] = ((-lam[i]) + (-rho) * b[i]) + rho * cvs[i];   // lorads_alm.c:45-49
}

// r x r Gram X^T X (or of the average (X+Y)/2), build_gram_from_factor /
// build_gram_from_average (lorads_logging.c:216-270), on the FP64 matrix cores
// (v_mfma_f64_16x16x4f64).  Register-blocked: a wave owns an NB x NB block of 16 x 16
// tiles -- column block A (16 NB columns) against column block B >= A -- and its lane l
// reads, per k-step of 4 rows, NB consecutive doubles of row 4s + (l >> 4) at column
// 16 NB A + NB (l & 15) (one vector load), so sub-tile t of a block holds the columns
// 16 NB A + NB m + t, m = 0..15: NB^2 MFMAs per 2 NB doubles loaded per lane (a diagonal
// block loads once).  Grid (C row chunks) x (block pairs A <= B); C is a multiple of 8,
// so the linear block id y*C + x puts every pair of chunk x on the same XCD (id mod 8)
// and the chunk's rows are fetched into that XCD's L2 once.  The four waves of a
// workgroup take interleaved k-steps of the chunk (unmasked batches, one masked tail),
// their accumulators meet in LDS (wave order, four sub-tiles a round) and the workgroup
// stores the chunk's partial sub-tiles.  k_gram_fin (one workgroup per sub-tile) sums the
// C partials (four interleaved quarters, every load in one trip) and scatters the
// sub-tile and its transpose.  Deterministic.  Columns in [r, 16 NB nbc) are never
// stored: they only reach output entries of their own column, so they are read as they
// lie (padding below the row pitch ld) or from the row's last NB columns (past ld).
// D fragment: col = l & 15, row = (l >> 4) + 4q (cdna_hip_programming.md §3, f64 map).
typedef double gram_acc_t __attribute__((ext_vector_type(4)));
template <int NB>
struct GramVec;
template <>
struct GramVec<1> { typedef double T; };
template <>
struct GramVec<2> { typedef double T __attribute__((ext_vector_type(2))); };
template <>
struct GramVec<4> { typedef double T __attribute__((ext_vector_type(4))); };

template <int NB>
__device__ __forceinline__ void gram_ld(const double *__restrict__ p, double *o) {
    typedef typename GramVec<NB>::T V;
    const V v = *reinterpret_cast<const V *>(p);
    if constexpr (NB == 1) o[0] = v;
    else {
#pragma unroll
        for (int t = 0; t < NB; ++t) o[t] = v[t];
    }
}

// one wave's k-steps of an (A, B) block pair; branch-free so that a batch's U loads are all
// in flight before its MFMAs (the row test is a select; a lane whose NB columns start at or
// past ld reads the row's last NB columns instead -- they lie at or past r, never stored)
template <int NB, int U, bool AVG, bool DIAG>
__device__ __forceinline__ void gram_loop(int nk, int i0, int i1, int w, int lane, long base, long step,
                                          long clamp0, const double *__restrict__ X, const double *__restrict__ Y,
                                          int colA, int colB, gram_acc_t (&acc)[NB][NB]) {
    for (int j0 = 0; j0 < nk; j0 += U) {
        double xa[U][NB], xb[U][NB];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = i0 + 16 * (j0 + u) + 4 * w + (lane >> 4);
            const bool ok = row < i1;
            const long o = ok ? base + (j0 + u) * step : clamp0;
            gram_ld<NB>(X + o + colA, xa[u]);
            if constexpr (!DIAG) gram_ld<NB>(X + o + colB, xb[u]);
            if constexpr (AVG) {
                double ya[NB], yb[NB];
                gram_ld<NB>(Y + o + colA, ya);
                if constexpr (!DIAG) gram_ld<NB>(Y + o + colB, yb);
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    xa[u][t] = 0.5 * (xa[u][t] + ya[t]);
                    if constexpr (!DIAG) xb[u][t] = 0.5 * (xb[u][t] + yb[t]);
                }
            }
#pragma unroll
            for (int t = 0; t < NB; ++t) {
                xa[u][t] = ok ? xa[u][t] : 0.0;
                if constexpr (DIAG) xb[u][t] = xa[u][t];
                else xb[u][t] = ok ? xb[u][t] : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int p = 0; p < NB; ++p)
#pragma unroll
                for (int q = 0; q < NB; ++q)
                    acc[p][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[u][p], xb[u][q], acc[p][q], 0, 0, 0);
    }
}

template <int NB, int U, bool AVG>
__global__ void __launch_bounds__(kBlock) k_gram(int n, int r, int ld, int nbc, const double *__restrict__ X,
                                                 const double *__restrict__ Y, double *__restrict__ part) {
    constexpr int W = 16 * NB;
    __shared__ double red[kBlock / 64][4][256];
    int id = blockIdx.y, A = 0;
    while (id >= nbc - A) { id -= nbc - A; ++A; }
    const int B = A + id, pair = blockIdx.y;
    const int C = gridDim.x, ch = blockIdx.x;
    const int per = ((n + C - 1) / C + 15) / 16 * 16;
    const int i0 = ch * per, i1 = min(n, i0 + per);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int colA = min(W * A + NB * (lane & 15), ld - NB), colB = min(W * B + NB * (lane & 15), ld - NB);
    gram_acc_t acc[NB][NB];
#pragma unroll
    for (int p = 0; p < NB; ++p)
#pragma unroll
        for (int q = 0; q < NB; ++q) acc[p][q] = gram_acc_t{0.0, 0.0, 0.0, 0.0};
    // this wave's k-steps: rows i0 + 16 j + 4 w + (lane >> 4), j = 0, 1, ...
    const int nk = i1 > i0 + 4 * w ? (i1 - i0 - 4 * w + 15) / 16 : 0;
    const long step = 16L * ld, base = (long)(i0 + 4 * w + (lane >> 4)) * ld, clamp0 = (long)i0 * ld;
    if (A == B) gram_loop<NB, U, AVG, true>(nk, i0, i1, w, lane, base, step, clamp0, X, Y, colA, colB, acc);
    else gram_loop<NB, U, AVG, false>(nk, i0, i1, w, lane, base, step, clamp0, X, Y, colA, colB, acc);
    // wave partials -> LDS, four sub-tiles a round, summed in wave order
    const int t = threadIdx.x;   // t = q * 64 + l
#pragma unroll
    for (int g = 0; g < (NB * NB + 3) / 4; ++g) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int st = 4 * g + k;
            if (st < NB * NB)
#pragma unroll
                for (int q = 0; q < 4; ++q) red[w][k][q * 64 + lane] = acc[st / NB][st % NB][q];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int st = 4 * g + k;
            if (st < NB * NB) {
                double v = red[0][k][t];
#pragma unroll
                for (int ww = 1; ww < kBlock / 64; ++ww) v += red[ww][k][t];
                part[(((long)pair * NB * NB + st) * C + ch) * 256 + t] = v;
            }
        }
        __syncthreads();
    }
}
// k_gram_fin: four workgroups per sub-tile, 64 of its elements each; thread (p, e) of a
// workgroup sums the chunks c = p (mod 16) of element e (every load in one memory trip:
// C <= 64), the sixteen partial sums meet in LDS in order
constexpr int kGramFinThreads = 1024;
__global__ void __launch_bounds__(kGramFinThreads) k_gram_fin(int r, int NB, int nbc, int C,
                                                              const double *__restrict__ part,
                                                              double *__restrict__ out) {
    static_assert(kGramMaxChunks <= 64, "4 chunks per thread");
    __shared__ double q16[16][64];
    const int sub = blockIdx.x >> 2, st = sub % (NB * NB);
    int id = sub / (NB * NB), A = 0;
    while (id >= nbc - A) { id -= nbc - A; ++A; }
    const int B = A + id, e = threadIdx.x & 63, pq = threadIdx.x >> 6;
    const int t = (blockIdx.x & 3) * 64 + e;   // element of the sub-tile, t = q * 64 + l
    double pv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int ch = pq + 16 * u;
        pv[u] = ch < C ? part[((long)sub * C + ch) * 256 + t] : 0.0;
    }
    q16[pq][e] = (pv[0] + pv[1]) + (pv[2] + pv[3]);
    __syncthreads();
    if (pq != 0) return;
    double s = q16[0][e];
#pragma unroll
    for (int k = 1; k < 16; ++k) s += q16[k][e];
    const int q = t >> 6, l = t & 63;
    const int W = 16 * NB;
    const int row = W * A + NB * ((l >> 4) + 4 * q) + st / NB, col = W * B + NB * (l & 15) + st % NB;
    if (row < r && col < r && (A != B || row <= col)) {
        out[(long)row * r + col] = s;
        out[(long)col * r + row] = s;
    }
}

// ------------------------------------------------------------------------
// Fused ALM inner iteration, lorads_alm.c:1302-1379.  Control state is
// double-buffered by iteration parity: iteration t reads ctrl[(t-1)&1] and
// block 0 of k_alm_dir writes ctrl[t&1]; every block computes the same state.
// ------------------------------------------------------------------------
struct AlmFinal {            // finals produced inside one iteration (device memory)
    double sd[2];            // p1-part, p2-part  (sum over cones is done by the consumer)
};

// finals layout in `fin` (double array):
//   FIN_SD  + 2*k : sddmm objective partials of cone k (RD, DD)
//   FIN_Q   .. +5 : gather_q dots
//   FIN_GR  + 9*k : grad dots of cone k
//   FIN_RR        : residual
// (FIN_N: lrs_device.h kFinN, the per-context buffer's size)
enum FinIdx { FIN_SD = 0, FIN_Q = 64, FIN_GR = 80, FIN_RR = 400, FIN_N = 416 };
static_assert(FIN_N == kFinN, "finals layout");

__device__ int ctrl_compute(double *c, const double *__restrict__ prev, const double *__restrict__ par,
                            const double *__restrict__ lsprev, int K, const double *__restrict__ fin) {
    // executed by thread 0 only; c is shared memory.
    // PENDING: 0 = nothing to fold (host start: clear == 0), 1 = fold the previous
    // iteration's finals, 2 = dots already stashed in C_DSG..C_DYOY.
    for (int q = 0; q < C_NCTRL; ++q) c[q] = prev[q];
    const int L = (int)par[P_L];
    if (c[C_ACTIVE] != 0.0 && c[C_PENDING] == 1.0) {
        const double flag = lsprev[LS_FLAG];
        if (flag == 1.0) {                      // rootNum == 0: RET_CODE_NUM_ERR (lorads_alm.c:1327)
            c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_NUMERR;
            c[C_PENDING] = 0.0;
        } else if (flag == 2.0) {               // |tau| < endTauTol (lorads_alm.c:1331-1339)
            c[C_INNER] += 1; c[C_LOCAL] += 1; c[C_CLEAR] += 1;
            c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_TINYTAU;
            c[C_PENDING] = 0.0;
        } else {
            double d[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for (int k = 0; k < K; ++k)
                for (int q = 0; q < 9; ++q) d[q] += fin[FIN_GR + 9 * k + q];
            const int h = (int)c[C_HEAD];
            // setlbfgsHisTwo (lorads_alm.c:861): beta = 1/<y,s>; ring head advances (:862)
            c[C_BETA0 + h] = 1.0 / d[1];
            c[C_YY0 + h] = d[2];
            c[C_HEAD] = (double)((h + 1) % L);
            c[C_GCUR] = 1.0 - c[C_GCUR];
            c[C_LAG] = d[0];
            c[C_LASTTAU] = lsprev[LS_TAU];
            // primalInfeasibility (lorads_alg_common.c:393) and l_inf (lorads_alm.c:1359)
            const double pinf1 = sqrt(fin[FIN_RR]) / (1.0 + par[P_BN1]);
            c[C_PINF1] = pinf1;
            c[C_PINFINF] = pinf1 * (1.0 + par[P_BN1]) / (1.0 + par[P_BNINF]);
            c[C_DSG] = d[3]; c[C_DYG] = d[4]; c[C_DSOG] = d[5]; c[C_DYOG] = d[6];
            c[C_DSOY] = d[7]; c[C_DYOY] = d[8];
            c[C_PENDING] = 2.0;
            if ((c[C_PINFINF] <= par[P_PH1TOL]) && ((par[P_GAP] <= par[P_PH1TOL]) || (par[P_HIGHACC] == 0.0))) {
                c[C_INNER] += 1; c[C_LOCAL] += 1; c[C_CLEAR] += 1;
                c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_PHASE1;
            } else {
                c[C_RCVAL] = sqrt(c[C_LAG]) / (1.0 + par[P_CNINF]);
                c[C_INNER] += 1; c[C_LOCAL] += 1; c[C_CLEAR] += 1;
                if (c[C_LOCAL] > 800) { c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_LOCAL800; }
            }
        }
    } else if (c[C_PENDING] == 0.0) {
        c[C_DSG] = c[C_DYG] = c[C_DSOG] = c[C_DYOG] = c[C_DSOY] = c[C_DYOY] = 0.0;
    }
    if (c[C_ACTIVE] != 0.0) {
        if (!(c[C_RCVAL] - par[P_RCTOL] > par[P_ENDSUB])) { c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_CONVERGED; }
        else if (par[P_BUDGET] > 0 && c[C_INNER] >= par[P_BUDGET]) { c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_BUDGET; }
    }
    if (c[C_ACTIVE] == 0.0) return 0;
    // LBFGSDirection (lorads_alm.c:468-505) in coefficient space
    if (((long)c[C_LOCAL]) % 300 == 0) c[C_CLEAR] = 0;
    const int clear = (int)c[C_CLEAR];
    const int nodeNum = clear == 0 ? 0 : (clear <= L - 1 ? clear : L);
    c[C_NODENUM] = nodeNum;
    const double GG = c[C_LAG];
    const double sG = c[C_DSG], yG = c[C_DYG], soG = c[C_DSOG], yoG = c[C_DYOG], soy = c[C_DSOY], yoy = c[C_DYOY];
    const int hn = ((int)c[C_HEAD] - 1 + L) % L;     // newest slot
    const int ho = (hn - 1 + L) % L;                  // older slot
    double cs[2] = {0, 0}, cy[2] = {0, 0};
    double dg;
    if (nodeNum == 0) {
        dg = -GG;
    } else if (nodeNum == 1) {
        const double bn = c[C_BETA0 + hn], yyn = c[C_YY0 + hn];
        const double a1 = bn * sG;
        const double w1 = a1 - bn * (yG - a1 * yyn);
        cy[hn] += -a1; cs[hn] += w1;
        dg = -(GG - a1 * yG + w1 * sG);
    } else {
        const double bn = c[C_BETA0 + hn], yyn = c[C_YY0 + hn];
        const double bo = c[C_BETA0 + ho], yyo = c[C_YY0 + ho];
        const double a1 = bn * sG;
        const double a2 = bo * (soG - a1 * soy);
        const double w2 = a2 - bo * (yoG - a1 * yoy - a2 * yyo);
        const double w1 = a1 - bn * (yG - a1 * yyn - a2 * yoy + w2 * soy);
        cy[hn] += -a1; cy[ho] += -a2; cs[ho] += w2; cs[hn] += w1;
        dg = -(GG - a1 * yG - a2 * yoG + w2 * soG + w1 * sG);
    }
    c[C_CG] = 1.0;
    c[C_CS0] = cs[0]; c[C_CY0] = cy[0]; c[C_CS1] = cs[1]; c[C_CY1] = cy[1];
    // LBFGSDirectionUseGrad (lorads_alm.c:618-626)
    if (dg >= 0) { c[C_CS0] = c[C_CY0] = c[C_CS1] = c[C_CY1] = 0.0; dg = -GG; }
    c[C_DG] = dg;
    c[C_PENDING] = 1.0;
    return 1;
}

__global__ void __launch_bounds__(kBlock) k_alm_dir(long NR, const double *__restrict__ par,
                                                    const double *__restrict__ ctrl_prev, double *__restrict__ ctrl_cur,
                                                    const double *__restrict__ lsprev, int K,
                                                    double *__restrict__ D, const double *__restrict__ G0,
                                                    const double *__restrict__ G1, const double *__restrict__ s0,
                                                    const double *__restrict__ y0, const double *__restrict__ s1,
                                                    const double *__restrict__ y1, const double *__restrict__ fin) {
    __shared__ double c[C_NCTRL];
    if (threadIdx.x == 0) ctrl_compute(c, ctrl_prev, par, lsprev, K, fin);
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x < C_NCTRL) ctrl_cur[threadIdx.x] = c[threadIdx.x];
    if (c[C_ACTIVE] == 0.0) return;
    const double cg = c[C_CG], cs0 = c[C_CS0], cy0 = c[C_CY0], cs1 = c[C_CS1], cy1 = c[C_CY1];
    const double *__restrict__ Gc = c[C_GCUR] == 0.0 ? G0 : G1;
    const bool u0 = (cs0 != 0.0 || cy0 != 0.0), u1 = (cs1 != 0.0 || cy1 != 0.0);
    for (long i = ((long)blockIdx.x * kBlock + threadIdx.x) * 2; i < NR; i += (long)gridDim.x * kBlock * 2) {
        double2 g = *reinterpret_cast<const double2 *>(Gc + i);
        double dx = cg * g.x, dy = cg * g.y;
        if (u0) {
            double2 a = *reinterpret_cast<const double2 *>(s0 + i), b = *reinterpret_cast<const double2 *>(y0 + i);
            dx += cs0 * a.x + cy0 * b.x; dy += cs0 * a.y + cy0 * b.y;
        }
        if (u1) {
            double2 a = *reinterpret_cast<const double2 *>(s1 + i), b = *reinterpret_cast<const double2 *>(y1 + i);
            dx += cs1 * a.x + cy1 * b.x; dy += cs1 * a.y + cy1 * b.y;
        }
        *reinterpret_cast<double2 *>(D + i) = make_double2(-dx, -dy);
    }
}

// q1 = 2 A(sym RD^T), q2 = A(DD^T) and the five line-search reductions
// (ALMCalq12p12 lorads_alm.c:714-734 + ALMLineSearch :269-277)
__global__ void __launch_bounds__(kBlock) k_alm_gather_q(int m, int K, const int *__restrict__ con_ptr,
                                                         const int *__restrict__ con_slot,
                                                         const double *__restrict__ con_w,
                                                         const double *__restrict__ uRD, const double *__restrict__ uDD,
                                                         const double *__restrict__ b, const double *__restrict__ cvs,
                                                         const double *__restrict__ lam, const double *__restrict__ par,
                                                         double *__restrict__ q1o, double *__restrict__ q2o,
                                                         double *part, unsigned *ticket, double *fin,
                                                         const double *__restrict__ guard) {
    if (guard[C_ACTIVE] == 0.0) return;
    const double rhoInv = 1.0 / par[P_RHO];
    double acc[5] = {0, 0, 0, 0, 0};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < m; i += gridDim.x * kBlock) {
        double v1 = 0.0, v2 = 0.0;
        for (int k = 0; k < K; ++k) {
            const long row = (long)k * m + i;
            double a1 = 0.0, a2 = 0.0;
            for (int e = con_ptr[row]; e < con_ptr[row + 1]; ++e) {
                const double w = con_w[e];
                const int s = con_slot[e];
                a1 += w * uRD[s];
                a2 += w * uDD[s];
            }
            v1 += a1; v2 += a2;
        }
        v1 *= 2.0;
        q1o[i] = v1; q2o[i] = v2;
        const double q0 = (b[i] - cvs[i]) + rhoInv * lam[i];
        acc[0] += v2 * v2; acc[1] += v1 * v2; acc[2] += q0 * v2; acc[3] += v1 * v1; acc[4] += q0 * v1;
    }
    partials_finalize<5>(acc, part, ticket, fin);
}

// LORADScubic_equation (lorads_alm.c:191-231)
__device__ int dev_cubic(double a, double b, double c, double d, double *res) {
    const double A = b * b - 3 * a * c, B = b * c - 9 * a * d, C = c * c - 3 * b * d;
    const double delta = B * B - 4 * A * C;
    res[0] = res[1] = res[2] = 0.0;
    if (A == 0 && B == 0) { res[0] = fmax(res[0], -c / b); return 1; }
    if (delta > 0) {
        const double Y1 = A * b + 1.5 * a * (-B + sqrt(delta));
        const double Y2 = A * b + 1.5 * a * (-B - sqrt(delta));
        const double Y13 = Y1 > 0 ? pow(Y1, 1.0 / 3) : -pow(-Y1, 1.0 / 3);
        const double Y23 = Y2 > 0 ? pow(Y2, 1.0 / 3) : -pow(-Y2, 1.0 / 3);
        res[0] = fmax(res[0], (-b - Y13 - Y23) / 3 / a);
        return 1;
    }
    if (delta == 0 && A != 0 && B != 0) {
        const double Kk = B / A;
        res[0] = -b / a + Kk; res[1] = -Kk / 2;
        return 2;
    }
    if (delta < 0) {
        const double sqA = sqrt(A);
        const double T = (A * b - 1.5 * a * B) / (A * sqA);
        const double th = acos(T);
        const double cs = cos(th / 3), sn = sqrt(3.0) * sin(th / 3);
        res[0] = (-b - 2 * sqA * cs) / 3 / a;
        res[1] = (-b + sqA * (cs + sn)) / 3 / a;
        res[2] = (-b + sqA * (cs - sn)) / 3 / a;
        return 3;
    }
    return 0;
}

// Same as dev_cubic, executed by a whole wave (uniform result): the two independent
// cube roots of the delta > 0 branch run on lanes 0 and 1 at once.
__device__ __forceinline__ int dev_cubic_wave(double a, double b, double c, double d, double *res) {
    const double A = b * b - 3 * a * c, B = b * c - 9 * a * d, C = c * c - 3 * b * d;
    const double delta = B * B - 4 * A * C;
    res[0] = res[1] = res[2] = 0.0;
    if (A == 0 && B == 0) { res[0] = fmax(res[0], -c / b); return 1; }
    if (delta > 0) {
        const double sq = sqrt(delta);
        const double Y1 = A * b + 1.5 * a * (-B + sq);
        const double Y2 = A * b + 1.5 * a * (-B - sq);
        const double y = (threadIdx.x & 1) ? Y2 : Y1;
        const double ay = y > 0 ? y : -y;
        double r = pow(ay, 1.0 / 3);
        r = y > 0 ? r : -r;
        const double Y13 = read_lane(r, 0), Y23 = read_lane(r, 1);
        res[0] = fmax(res[0], (-b - Y13 - Y23) / 3 / a);
        return 1;
    }
    if (delta == 0 && A != 0 && B != 0) {
        const double Kk = B / A;
        res[0] = -b / a + Kk; res[1] = -Kk / 2;
        return 2;
    }
    if (delta < 0) {
        const double sqA = sqrt(A);
        const double T = (A * b - 1.5 * a * B) / (A * sqA);
        const double th = acos(T);
        double sn, cs;
        sincos(th / 3, &sn, &cs);
        sn *= sqrt(3.0);
        res[0] = (-b - 2 * sqA * cs) / 3 / a;
        res[1] = (-b + sqA * (cs + sn)) / 3 / a;
        res[2] = (-b + sqA * (cs - sn)) / 3 / a;
        return 3;
    }
    return 0;
}

__device__ __forceinline__ double quartic(double a, double b, double c, double d, double x) {
    const double x2 = x * x;
    return a * (x2 * x2) + b * (x2 * x) + c * x2 + d * x;
}

// ALMLineSearch (lorads_alm.c:266-333) from the finals; writes ls[0..2]
__device__ void line_search_v(const double *__restrict__ par, double p1, double p2, const double *dots, double *ls);
__device__ void line_search(const double *__restrict__ par, int K, const double *__restrict__ fin, double *ls) {
    double p1 = 0.0, p2 = 0.0;
    for (int k = 0; k < K; ++k) { p1 += fin[FIN_SD + 2 * k]; p2 += fin[FIN_SD + 2 * k + 1]; }
    double dots[5];
    for (int q = 0; q < 5; ++q) dots[q] = fin[FIN_Q + q];
    line_search_v(par, p1, p2, dots, ls);
}
// ------------------------------------------------------------------------
// Split ALM inner iteration: FOUR launches per iteration (lorads_alm.c:1302-1379).
//   S1 k_it_dir_sddmm<G,E> control (folds the previous iteration's dots), the
//                          A(RR^T) refresh + residual of the previous iteration
//                          (primalInfeasibility, lorads_alg_common.c:386-394), the
//                          L-BFGS direction D = -H G (rows recomputed for the
//                          neighbours instead of a launch boundary) and sym(RD^T),
//                          DD^T on the pattern with the objective partials
//   S2 k_it_q              phase-1 test on the residual (lorads_alm.c:1359-1364),
//                          q1 = 2A(sym RD^T), q2 = A(DD^T), five line-search dots
//   S3 k_it_update         line search, R += tau D, S = C + A^*(M1) with M1 formed
//                          per constraint on the fly (ALMSetGrad, lorads_alm.c:38-57)
//   S4 k_it_grad<G,E>      G = 2 S R, A(RR^T) slots, L-BFGS pair, nine dots
// Cross-block sums: every producer block writes its partials; EVERY block of the
// consuming launch reduces them in the same fixed order.  No in-launch hand-off, no
// fences; the launch boundary is the only synchronisation.  Bitwise reproducible.
// ------------------------------------------------------------------------
// Block sums of NV accumulators into part[v][slot]: wave sums meet in LDS, then thread v
// adds value v over the waves in wave order (the order of block_reduce) and stores it --
// one barrier, the NV sums in parallel.
template <int NV, int NT = kBlock>
__device__ __forceinline__ void write_partials(double (&acc)[NV], double *__restrict__ part, int slot) {
    __shared__ double sh[NV][NT / 64];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const double t = wave_sum(acc[v]);
        if (lane == 0) sh[v][wid] = t;
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        const int v = threadIdx.x;
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) t += sh[v][w];
        part[v * kMaxPartialBlocks + slot] = t;
    }
}

// write_partials for a block of nw <= 8 waves (the latency kernels' run-time block size): the
// same wave-order sums
template <int NV>
__device__ __forceinline__ void write_partials_nw(double (&acc)[NV], double *__restrict__ part, int slot, int nw) {
    __shared__ double sh[NV][8];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const double t = wave_sum(acc[v]);
        if (lane == 0) sh[v][wid] = t;
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        const int v = threadIdx.x;
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < 8; ++w)
            if (w < nw) t += sh[v][w];
        part[v * kMaxPartialBlocks + slot] = t;
    }
}

template <int NV, int NT = kBlock>
__device__ __forceinline__ void write_partials_range(double (&acc)[NV], double *__restrict__ part, int slot, int v0,
                                                     int v1) {
    double s[NV];
    block_reduce<NV, NT>(acc, s);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (v >= v0 && v < v1) part[v * kMaxPartialBlocks + slot] = s[v];
    }
}

// all threads; generic nblk
template <int NV, int NT = kBlock>
__device__ __forceinline__ void reduce_partials(const double *__restrict__ part, int nblk, double *out,
                                                int pstr = kMaxPartialBlocks) {
    double a[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) a[v] = 0.0;
    for (int b = threadIdx.x; b < nblk; b += NT) {
#pragma unroll
        for (int v = 0; v < NV; ++v) a[v] += part[v * pstr + b];
    }
    double s[NV];
    block_reduce<NV, NT>(a, s);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v) out[v] = s[v];
    }
    __syncthreads();
}

// ALMLineSearch (lorads_alm.c:266-333) from reduced values: p1, p2 objective parts
// (p1 before its factor 2), dots = {q2q2, q1q2, q0q2, q1q1, q0q1}.
template <bool WAVE, typename PB>
__device__ __forceinline__ void line_search_t(const PB &par, double p1, double p2, const double *dots, double *ls) {
    p1 *= 2.0;
    const double rho = par[P_RHO];
    const double a = rho * dots[0] / 2;
    const double b = rho * dots[1];
    const double c = p2 - rho * dots[2] + rho * dots[3] / 2;
    const double d = p1 - rho * dots[4];
    double roots[3];
    const int rn = WAVE ? dev_cubic_wave(4 * a, 3 * b, 2 * c, d, roots) : dev_cubic(4 * a, 3 * b, 2 * c, d, roots);
    double tau = 0.0;
    const double f0 = 0.0, f1 = quartic(a, b, c, d, 1.0);
    double fr1 = 1e30, fr2 = 1e30, fr3 = 1e30;
    if (rn >= 1 && roots[0] > 1e-20 && roots[0] <= 1.0) fr1 = quartic(a, b, c, d, roots[0]);
    if (rn >= 2 && roots[1] > 1e-20 && roots[1] <= 1.0) fr2 = quartic(a, b, c, d, roots[1]);
    if (rn == 3 && roots[2] > 1e-20 && roots[2] <= 1.0) fr3 = quartic(a, b, c, d, roots[2]);
    const double mn = fmin(fmin(fmin(fmin(f0, f1), fr1), fr2), fr3);
    if (fabs(mn - f0) < 1e-10) tau = 0.0;
    if (fabs(mn - f1) < 1e-10) tau = 1.0;
    if (fabs(mn - fr1) < 1e-10) tau = roots[0];
    if (fabs(mn - fr2) < 1e-10) tau = roots[1];
    if (fabs(mn - fr3) < 1e-10) tau = roots[2];
    if (!WAVE || (threadIdx.x & 63) == 0) {
        ls[LS_TAU] = tau;
        ls[LS_ROOTNUM] = rn;
        ls[LS_FLAG] = rn == 0 ? 1.0 : (fabs(tau) < par[P_ENDTAU] ? 2.0 : 0.0);
    }
}
__device__ void line_search_v(const double *__restrict__ par, double p1, double p2, const double *dots, double *ls) {
    line_search_t<false>(par, p1, p2, dots, ls);
}

// Control of one split iteration (thread 0).  c: shared copy of the previous control,
// updated in place.
// d = the nine dots of the previous gradient stage when `fold`.
// CB / PB: the control block and parameters as LDS / global pointers (in place on the shared
// copy: in k_it_a a register copy of the block would set the VGPR peak, and so the occupancy,
// of the whole row kernel), or as register arrays (k_lat_a's control wave: every word a
// register, no LDS round trip per access on the launch's critical path).
template <typename CB, typename PB>
__device__ __forceinline__ void ctrl_step(CB &&c, const PB &par, double lsflag, double lstau, int fold,
                                          const double *d, bool ph1) {
    const int L = (int)par[P_L];
    const double cninf = par[P_CNINF], rctol = par[P_RCTOL], endsub = par[P_ENDSUB], budget = par[P_BUDGET];
    c[C_ACTIVE] = c[C_ACT2];
    c[C_EXIT] = c[C_EXIT2];
    c[C_RRDONE] = 0.0;
    if (c[C_ACTIVE] != 0.0 && c[C_PENDING] == 1.0) {
        if (lsflag == 1.0) {                    // rootNum == 0: RET_CODE_NUM_ERR (lorads_alm.c:1327)
            c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_NUMERR;
            c[C_PENDING] = 0.0;
        } else if (lsflag == 2.0) {             // |tau| < endTauTol (lorads_alm.c:1331-1339)
            c[C_INNER] += 1; c[C_LOCAL] += 1; c[C_CLEAR] += 1;
            c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_TINYTAU;
            c[C_PENDING] = 0.0;
        } else if (fold) {
            const int h = (int)c[C_HEAD];
            // setlbfgsHisTwo (lorads_alm.c:861): beta = 1/<y,s>; ring head advances (:862)
            const double beta = 1.0 / d[1];
            if (h == 0) { c[C_BETA0] = beta; c[C_YY0] = d[2]; }
            else { c[C_BETA1] = beta; c[C_YY1] = d[2]; }
            c[C_HEAD] = (double)(h + 1 >= L ? 0 : h + 1);
            c[C_GCUR] = 1.0 - c[C_GCUR];
            c[C_LAG] = d[0];
            c[C_LASTTAU] = lstau;
            c[C_DSG] = d[3]; c[C_DYG] = d[4]; c[C_DSOG] = d[5]; c[C_DYOG] = d[6];
            c[C_DSOY] = d[7]; c[C_DYOY] = d[8];
            c[C_PENDING] = 2.0;
            c[C_RCUR] = 1.0 - c[C_RCUR];
            if (ph1) {
                // primalInfeasibility (lorads_alg_common.c:393), l_inf and the phase-1 exit
                // (lorads_alm.c:1359-1364), which takes precedence over the tests below
                const double pinf1 = sqrt(d[9]) / (1.0 + par[P_BN1]);
                c[C_PINF1] = pinf1;
                c[C_PINFINF] = pinf1 * (1.0 + par[P_BN1]) / (1.0 + par[P_BNINF]);
                c[C_INNER] += 1; c[C_LOCAL] += 1; c[C_CLEAR] += 1;
                if ((c[C_PINFINF] <= par[P_PH1TOL]) && ((par[P_GAP] <= par[P_PH1TOL]) || (par[P_HIGHACC] == 0.0))) {
                    c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_PHASE1;
                } else {
                    c[C_RCVAL] = sqrt(c[C_LAG]) / (1.0 + cninf);
                    if (c[C_LOCAL] > 800) { c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_LOCAL800; }
                }
            } else {
                // the phase-1 test on the refreshed residual (which takes precedence) runs in
                // the global-constraint stage
                c[C_RRDONE] = 1.0;
                c[C_RCVAL] = sqrt(c[C_LAG]) / (1.0 + cninf);
                c[C_INNER] += 1; c[C_LOCAL] += 1; c[C_CLEAR] += 1;
                if (c[C_LOCAL] > 800) { c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_LOCAL800; }
            }
        }
    } else if (c[C_PENDING] == 0.0) {
        c[C_DSG] = c[C_DYG] = c[C_DSOG] = c[C_DYOG] = c[C_DSOY] = c[C_DYOY] = 0.0;
    }
    if (c[C_ACTIVE] != 0.0) {
        if (!(c[C_RCVAL] - rctol > endsub)) { c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_CONVERGED; }
        else if (budget > 0 && c[C_INNER] >= budget) { c[C_ACTIVE] = 0.0; c[C_EXIT] = EXIT_BUDGET; }
    }
    if (c[C_ACTIVE] != 0.0) {
        // LBFGSDirection (lorads_alm.c:468-505) in coefficient space
        if (((int)c[C_LOCAL]) % 300 == 0) c[C_CLEAR] = 0;   // localIter <= 801
        const int clear = (int)c[C_CLEAR];
        const int nodeNum = clear == 0 ? 0 : (clear <= L - 1 ? clear : L);
        c[C_NODENUM] = nodeNum;
        const double GG = c[C_LAG];
        const double sG = c[C_DSG], yG = c[C_DYG], soG = c[C_DSOG], yoG = c[C_DYOG], soy = c[C_DSOY],
                     yoy = c[C_DYOY];
        const int hn = (int)c[C_HEAD] == 0 ? L - 1 : (int)c[C_HEAD] - 1;     // newest slot
        double cs0 = 0, cs1 = 0, cy0 = 0, cy1 = 0;
        double dg;
        if (nodeNum == 0) {
            dg = -GG;
        } else if (nodeNum == 1) {
            const double bn = hn ? c[C_BETA1] : c[C_BETA0], yyn = hn ? c[C_YY1] : c[C_YY0];
            const double a1 = bn * sG;
            const double w1 = a1 - bn * (yG - a1 * yyn);
            if (hn) { cy1 += -a1; cs1 += w1; } else { cy0 += -a1; cs0 += w1; }
            dg = -(GG - a1 * yG + w1 * sG);
        } else {
            // L == 2: the older slot is the other one
            const double bn = hn ? c[C_BETA1] : c[C_BETA0], yyn = hn ? c[C_YY1] : c[C_YY0];
            const double bo = hn ? c[C_BETA0] : c[C_BETA1], yyo = hn ? c[C_YY0] : c[C_YY1];
            const double a1 = bn * sG;
            const double a2 = bo * (soG - a1 * soy);
            const double w2 = a2 - bo * (yoG - a1 * yoy - a2 * yyo);
            const double w1 = a1 - bn * (yG - a1 * yyn - a2 * yoy + w2 * soy);
            if (hn) { cy1 += -a1; cy0 += -a2; cs0 += w2; cs1 += w1; }
            else { cy0 += -a1; cy1 += -a2; cs1 += w2; cs0 += w1; }
            dg = -(GG - a1 * yG - a2 * yoG + w2 * soG + w1 * sG);
        }
        c[C_CG] = 1.0;
        c[C_CS0] = cs0; c[C_CY0] = cy0; c[C_CS1] = cs1; c[C_CY1] = cy1;
        // LBFGSDirectionUseGrad (lorads_alm.c:618-626)
        if (dg >= 0) { c[C_CS0] = c[C_CY0] = c[C_CS1] = c[C_CY1] = 0.0; dg = -GG; }
        c[C_DG] = dg;
        c[C_PENDING] = 1.0;
    }
    if (ph1) { c[C_ACT2] = c[C_ACTIVE]; c[C_EXIT2] = c[C_EXIT]; }
}

// Batch-end mirror of the control block into pinned host memory (run_inner polls it
// instead of a device-to-host copy and a stream synchronisation): the first wave of block 0
// stores the NCTRL words, then the sequence number with a system-scope release.
__device__ __forceinline__ void mirror_ctrl(const double *__restrict__ ctrl, double *hm, double seq) {
    if (hm == nullptr || blockIdx.x != 0 || threadIdx.x >= 64) return;
    if (threadIdx.x < C_NCTRL) hm[threadIdx.x] = ctrl[threadIdx.x];
    if (threadIdx.x == 0) __hip_atomic_store(hm + C_NCTRL, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct DirCoef {
    double cg, cs0, cy0, cs1, cy1;
    bool u0, u1;
};

// one row of D = -(cg G + cs0 s0 + cy0 y0 + cs1 s1 + cy1 y1), same arithmetic as k_alm_dir;
// the operand rows are loaded by dir_load so that the loads can run ahead.
template <int E>
struct DirRow {
    double g[E], a0[E], b0[E], a1[E], b1[E];
    __device__ __forceinline__ void load(const DirCoef &k, const double *__restrict__ Gc,
                                         const double *__restrict__ s0, const double *__restrict__ y0,
                                         const double *__restrict__ s1, const double *__restrict__ y1, long off) {
        ld_row<E>(Gc + off, g);
        if (k.u0) { ld_row<E>(s0 + off, a0); ld_row<E>(y0 + off, b0); }
        if (k.u1) { ld_row<E>(s1 + off, a1); ld_row<E>(y1 + off, b1); }
    }
    __device__ __forceinline__ void eval(const DirCoef &k, double (&d)[E]) const {
#pragma unroll
        for (int e = 0; e < E; ++e) d[e] = k.cg * g[e];
        if (k.u0) {
#pragma unroll
            for (int e = 0; e < E; ++e) d[e] += k.cs0 * a0[e] + k.cy0 * b0[e];
        }
        if (k.u1) {
#pragma unroll
            for (int e = 0; e < E; ++e) d[e] += k.cs1 * a1[e] + k.cy1 * b1[e];
        }
#pragma unroll
        for (int e = 0; e < E; ++e) d[e] = -d[e];
    }
};

constexpr int kRowBlock = 512;   // threads per block of the row kernels S1 / S4

// Row order of the row kernels' team loops.  Large grids (the bandwidth regime): blocks b and
// b + 8 share an XCD under the round-robin dispatch (MI355X_MICROARCH.md, for speed only), so
// the blocks of XCD group x = b % 8 take the contiguous rows [x n / 8, (x + 1) n / 8) and
// stride over them together: a row's neighbours (i +- 1, and i +- w on a w-wide grid) are then
// read by the same XCD and re-read from its L2 instead of fetched again from HBM through
// another XCD's misses.  Small problems (n < 16384; the dense small cones run their teams on a
// few dozen rows) and small grids: every team strides over all rows.  Either way each row is
// visited exactly once; only the rows' grouping into blocks (their partial sums) changes.
struct RowRange { int first, end, stride; };
__device__ __forceinline__ RowRange row_range(int n, int tpb, int team_local) {
#ifndef LRS_NO_XCD_ROWS
    if (gridDim.x >= 64 && n >= 16384) {
        const int x = blockIdx.x & 7, q = blockIdx.x >> 3;
        const int nbx = ((int)gridDim.x - x + 7) >> 3;
        const int r0 = (int)((long)n * x / 8), r1 = (int)((long)n * (x + 1) / 8);
        return {r0 + q * tpb + team_local, r1, nbx * tpb};
    }
#endif
    return {(int)blockIdx.x * tpb + team_local, n, (int)gridDim.x * tpb};
}

// Rows of the lower pattern carry the single-slot ("local") constraints: whoever
// computes a slot value also evaluates the local constraints on that slot.
//
// A.  Partials written (8): objective part of <C, sym RD^T>, of <C, DD^T>, the five
//     line-search dots over the local constraints, residual of the global ones.
// MODE 0: the whole stage (latency regime).  Bandwidth regime (large n), split in two
// launches over the same grid: MODE 1 = control + D of the own rows (+ global residual,
// partial 7), MODE 2 = SDDMM with D read back instead of recomputed per neighbour,
// local constraints (partials 0..6).
template <int G, int E, int U, int MODE>
__global__ void __launch_bounds__(kRowBlock) k_it_a(
    int n, int ld, long foff, const int *__restrict__ adj_ptr, const int *__restrict__ adj_low,
    const int *__restrict__ adj_col, const int *__restrict__ adj_slot, const double *__restrict__ Cw,
    const double *__restrict__ Rb0, const double *__restrict__ Rb1, double *__restrict__ Dall,
    const double *__restrict__ G0, const double *__restrict__ G1, const double *__restrict__ s0a,
    const double *__restrict__ y0a, const double *__restrict__ s1a, const double *__restrict__ y1a,
    double *__restrict__ uRD, double *__restrict__ uDD, const int *__restrict__ loc_ptr,
    const int *__restrict__ loc_con, const double *__restrict__ loc_w, const double2 *__restrict__ loc1,
    const double *__restrict__ b,
    double *__restrict__ cvs, const double *__restrict__ lam, double *__restrict__ rec, int do_glob, int mg,
    const int *__restrict__ glob, int m, int K, const int *__restrict__ con_ptr, const int *__restrict__ con_slot,
    const double *__restrict__ con_w, const double *__restrict__ uRR, const double *__restrict__ par,
    const double *__restrict__ ctrl_prev, double *__restrict__ ctrl_cur, const double *__restrict__ ls_prev,
    const double *__restrict__ partC, int nblkC, double *__restrict__ partA, int pblk_off, int T, int gwide,
    int row0, int pstr) {
    __shared__ double c[C_NCTRL];
    __shared__ double red[10];
    __shared__ double lsv[2];
    LRS_TS(0, 0);
    LRS_BLK_BEGIN();
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int fold = 0;
    if constexpr (MODE == 2) {
        // second half of a split stage: the control the first half wrote
        if (threadIdx.x < C_NCTRL) c[threadIdx.x] = ctrl_cur[threadIdx.x];
        __syncthreads();
    } else {
    if (threadIdx.x < C_NCTRL) c[threadIdx.x] = ctrl_prev[threadIdx.x];
    if (threadIdx.x == 0) { lsv[0] = ls_prev[LS_FLAG]; lsv[1] = ls_prev[LS_TAU]; }
    __syncthreads();
    LRS_TS(0, 1);
    fold = (c[C_ACT2] != 0.0 && c[C_PENDING] == 1.0 && lsv[0] == 0.0) ? 1 : 0;
    if (fold) reduce_partials<10, kRowBlock>(partC, nblkC, red, pstr);
    else __syncthreads();   // every wave has read c[] before thread 0 rewrites it
    LRS_TS(0, 2);
    if (threadIdx.x == 0) ctrl_step(c, par, lsv[0], lsv[1], fold, red, mg == 0);
    if (fold && do_glob) {
        // global constraints: A(RR^T) from the slots and their residual (primalInfeasibility);
        // independent of this iteration's control, so it runs beside ctrl_step.  Long
        // constraints (gwide) take a whole wave each, lanes striding over the entries.
        if (gwide) {
            const int lane64 = threadIdx.x & 63;
            const int nw = gridDim.x * (kRowBlock / 64);
            for (int g = blockIdx.x * (kRowBlock / 64) + (threadIdx.x >> 6); g < mg; g += nw) {
                const int i = glob[g];
                double tot = 0.0;
                for (int k = 0; k < K; ++k) {
                    const long row = (long)k * m + i;
                    double v = 0.0;
                    for (int e = con_ptr[row] + lane64; e < con_ptr[row + 1]; e += 64) v += con_w[e] * uRR[con_slot[e]];
                    tot += wave_sum(v);
                }
                if (lane64 == 0) {
                    cvs[i] = tot;
                    const double dd = b[i] - tot;
                    acc[7] += dd * dd;
                }
            }
        } else {
            for (int g = blockIdx.x * kRowBlock + threadIdx.x; g < mg; g += gridDim.x * kRowBlock) {
                const int i = glob[g];
                double tot = 0.0;
                for (int k = 0; k < K; ++k) {
                    const long row = (long)k * m + i;
                    double v = 0.0;
                    for (int e = con_ptr[row]; e < con_ptr[row + 1]; ++e) v += con_w[e] * uRR[con_slot[e]];
                    tot += v;
                }
                cvs[i] = tot;
                const double dd = b[i] - tot;
                acc[7] += dd * dd;
            }
        }
    }
    __syncthreads();
    LRS_TS(0, 3);
    if (pblk_off == 0 && blockIdx.x == 0 && threadIdx.x < C_NCTRL) ctrl_cur[threadIdx.x] = c[threadIdx.x];
    }   // MODE != 2
    const bool active = c[C_ACTIVE] != 0.0;
    if constexpr (MODE == 2) {
        if (!active) return;
    } else {
        if (!active && !(fold && mg > 0)) return;
    }
    LRS_TS(0, 4);
    if (active) {
        DirCoef kc;
        kc.cg = c[C_CG]; kc.cs0 = c[C_CS0]; kc.cy0 = c[C_CY0]; kc.cs1 = c[C_CS1]; kc.cy1 = c[C_CY1];
        kc.u0 = (kc.cs0 != 0.0 || kc.cy0 != 0.0);
        kc.u1 = (kc.cs1 != 0.0 || kc.cy1 != 0.0);
        const double rho = par[P_RHO], rhoInv = 1.0 / rho;
        const double *__restrict__ R = (c[C_RCUR] == 0.0 ? Rb0 : Rb1) + foff;
        double *__restrict__ D = Dall + foff;
        const double *__restrict__ Gc = (c[C_GCUR] == 0.0 ? G0 : G1) + foff;
        const double *__restrict__ s0 = s0a + foff, *__restrict__ y0 = y0a + foff;
        const double *__restrict__ s1 = s1a + foff, *__restrict__ y1 = y1a + foff;
        // lane groups of G lanes; a team of T groups shares one row (dense rows)
        const int lane = threadIdx.x & (G - 1);
        const int grp = (blockIdx.x * kRowBlock + threadIdx.x) / G;
        const int team = grp / T, mem = grp % T;
        const int tpb = (kRowBlock / G) / T;
        const RowRange rr = row_range(n, tpb, team - blockIdx.x * tpb);
        // rows [row0, row0 + n): the whole cone, or this process's shard of it
        for (int i = row0 + rr.first; i < row0 + rr.end; i += rr.stride) {
            const long oi = (long)i * ld + lane * E;
            const int kb = adj_ptr[i], ke = adj_low[i];
            double xi[E], yi[E];
            if constexpr (MODE == 2) {
                ld_row<E>(D + oi, yi);
            } else {
                DirRow<E> dr;
                dr.load(kc, Gc, s0, y0, s1, y1, oi);
                dr.eval(kc, yi);
                if (mem == 0) st_row<E>(D + oi, yi);
                if constexpr (MODE == 1) continue;   // the direction only
            }
            ld_row<E>(R + oi, xi);
            // lower entries U at a time: the neighbours' operand loads in flight together
            // (indices clamped to the row; the extra lanes' results are not stored); the
            // team's members take interleaved chunks of U
            for (int k0 = kb + mem * U; k0 < ke; k0 += T * U) {
                int jj[U], ss[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int k = min(k0 + u, ke - 1);
                    jj[u] = adj_col[k];
                    ss[u] = adj_slot[k];
                }
                double xj[U][E], yj[U][E], cw[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const long oj = (long)jj[u] * ld + lane * E;
                    ld_row<E>(R + oj, xj[u]);
                    cw[u] = Cw[ss[u]];
                    if constexpr (MODE == 2) {
                        ld_row<E>(D + oj, yj[u]);
                    } else {
                        DirRow<E> dj;
                        dj.load(kc, Gc, s0, y0, s1, y1, oj);
                        dj.eval(kc, yj[u]);
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    double d0 = 0.0, d1 = 0.0;
                    if (jj[u] != i) {
#pragma unroll
                        for (int e = 0; e < E; ++e) d0 += xi[e] * yj[u][e] + xj[u][e] * yi[e];
                        d0 *= 0.5;
                    } else {
#pragma unroll
                        for (int e = 0; e < E; ++e) d0 += xi[e] * yi[e];
                    }
#pragma unroll
                    for (int e = 0; e < E; ++e) d1 += yi[e] * yj[u][e];
                    d0 = group_sum<G>(d0);
                    d1 = group_sum<G>(d1);
                    if (lane == 0 && k0 + u < ke) {
                        const int sl = ss[u];
                        uRD[sl] = d0;
                        uDD[sl] = d1;
                        acc[0] += cw[u] * d0;
                        acc[1] += cw[u] * d1;
                        // local constraints on this slot: q1 = 2 A(sym RD^T), q2 = A(DD^T)
                        // (ALMCalq12p12 lorads_alm.c:714-734) and the line-search dots (:269-277);
                        // a single one comes with the slot's record, several from the lists
                        const double2 l1u = loc1[sl];
                        const int c1 = (int)l1u.y;
                        const int e0 = c1 == -2 ? loc_ptr[sl] : 0, e1 = c1 == -2 ? loc_ptr[sl + 1] : (c1 >= 0 ? 1 : 0);
                        for (int e = e0; e < e1; ++e) {
                            const int ci = c1 >= 0 ? c1 : loc_con[e];
                            const double w = c1 >= 0 ? l1u.x : loc_w[e];
                            const double q1 = 2.0 * (w * d0), q2 = w * d1;
                            const double bi = b[ci], cv = cvs[ci], li = lam[ci];
                            const double q0 = (bi - cv) + rhoInv * li;
                            acc[2] += q2 * q2; acc[3] += q1 * q2; acc[4] += q0 * q2; acc[5] += q1 * q1;
                            acc[6] += q0 * q1;
                            double2 *r = reinterpret_cast<double2 *>(rec + 4L * ci);
                            r[0] = make_double2(cv, q1);
                            r[1] = make_double2(q2, (-li) + (-rho) * bi);
                        }
                    }
                }
            }
        }
    }
    LRS_TS(0, 5);
    if constexpr (MODE == 0) write_partials<8, kRowBlock>(acc, partA, pblk_off + blockIdx.x);
    else if constexpr (MODE == 1) write_partials_range<8, kRowBlock>(acc, partA, pblk_off + blockIdx.x, 7, 8);
    else write_partials_range<8, kRowBlock>(acc, partA, pblk_off + blockIdx.x, 0, 7);
    LRS_TS_END(0, 6);
    LRS_BLK_END(0);
}

// G (only with global constraints).  Phase-1 test on the full residual (local part
// from stage B's partials, global part from stage A's), then q1, q2, the five dots
// and rec for the global constraints.  Partials written (5).
__global__ void __launch_bounds__(kBlock) k_it_g(int mg, const int *__restrict__ glob, int m, int K,
                                                 const int *__restrict__ con_ptr, const int *__restrict__ con_slot,
                                                 const double *__restrict__ con_w, const double *__restrict__ uRD,
                                                 const double *__restrict__ uDD, const double *__restrict__ b,
                                                 const double *__restrict__ cvs, const double *__restrict__ lam,
                                                 const double *__restrict__ par, double *__restrict__ ctrl_cur,
                                                 const double *__restrict__ partC, int nblkC,
                                                 const double *__restrict__ partA, int nblkA,
                                                 double *__restrict__ rec, double *__restrict__ partB, int gwide,
                                                 const double2 *__restrict__ uvp) {
    __shared__ double cs[3];
    __shared__ double red[2];
    LRS_TS(1, 0);
    LRS_BLK_BEGIN();
    if (threadIdx.x == 0) { cs[0] = ctrl_cur[C_ACTIVE]; cs[1] = ctrl_cur[C_EXIT]; cs[2] = ctrl_cur[C_RRDONE]; }
    __syncthreads();
    bool act = cs[0] != 0.0;
    double ex = cs[1];
    if (cs[2] != 0.0) {
        reduce_partials<1>(partC + 9 * kMaxPartialBlocks, nblkC, red);
        reduce_partials<1>(partA + 7 * kMaxPartialBlocks, nblkA, red + 1);
        // primalInfeasibility (lorads_alg_common.c:393) and l_inf (lorads_alm.c:1359)
        const double pinf1 = sqrt(red[0] + red[1]) / (1.0 + par[P_BN1]);
        const double pinfinf = pinf1 * (1.0 + par[P_BN1]) / (1.0 + par[P_BNINF]);
        if ((pinfinf <= par[P_PH1TOL]) && ((par[P_GAP] <= par[P_PH1TOL]) || (par[P_HIGHACC] == 0.0))) {
            act = false;
            ex = EXIT_PHASE1;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) { ctrl_cur[C_PINF1] = pinf1; ctrl_cur[C_PINFINF] = pinfinf; }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) { ctrl_cur[C_ACT2] = act ? 1.0 : 0.0; ctrl_cur[C_EXIT2] = ex; }
    LRS_TS(1, 1);
    if (!act) return;
    const double rho = par[P_RHO];
    const double rhoInv = 1.0 / rho;
    double acc[5] = {0, 0, 0, 0, 0};
    // gwide: a wave per constraint, lanes striding over its entries
    const int lanes = gwide ? 64 : 1;
    const int sub = gwide ? (threadIdx.x & 63) : 0;
    const int gid = gwide ? blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6) : blockIdx.x * kBlock + threadIdx.x;
    const int gstride = gwide ? gridDim.x * (kBlock / 64) : gridDim.x * kBlock;
    for (int g = gid; g < mg; g += gstride) {
        const int i = glob[g];
        double v1 = 0.0, v2 = 0.0;
        for (int k = 0; k < K; ++k) {
            const long row = (long)k * m + i;
            double a1 = 0.0, a2 = 0.0;
            if (uvp) {   // the tiled stage A's (RD, DD) records: one 16-B read per entry
                for (int e = con_ptr[row] + sub; e < con_ptr[row + 1]; e += lanes) {
                    const double w = con_w[e];
                    const double2 v = uvp[con_slot[e]];
                    a1 += w * v.x;
                    a2 += w * v.y;
                }
            } else {
                for (int e = con_ptr[row] + sub; e < con_ptr[row + 1]; e += lanes) {
                    const double w = con_w[e];
                    const int s = con_slot[e];
                    a1 += w * uRD[s];
                    a2 += w * uDD[s];
                }
            }
            if (gwide) { a1 = wave_sum(a1); a2 = wave_sum(a2); }
            v1 += a1; v2 += a2;
        }
        if (sub != 0) continue;
        v1 *= 2.0;
        const double bi = b[i], ci = cvs[i], li = lam[i];
        const double q0 = (bi - ci) + rhoInv * li;
        acc[0] += v2 * v2; acc[1] += v1 * v2; acc[2] += q0 * v2; acc[3] += v1 * v1; acc[4] += q0 * v1;
        double2 *r = reinterpret_cast<double2 *>(rec + 4L * i);
        r[0] = make_double2(ci, v1);
        r[1] = make_double2(v2, (-li) + (-rho) * bi);
    }
    LRS_TS(1, 2);
    write_partials<5>(acc, partB, blockIdx.x);
    LRS_TS_END(1, 3);
    LRS_BLK_END(1);
}

// ---- sharded solve, global constraints (lrs_problem.h ShardPlan: shared constraints) ----
// G1: this shard's share of every global constraint: sums over its owned-slot entries (the
// others carry weight 0) of RR (the last stage B's slots), RD and DD (this stage A's) ->
// g3[3][m], or for a shared constraint its row of gpack[nsh][3] (zero-filled before; the
// holders' rows meet in an all-reduce).
__global__ void __launch_bounds__(kBlock) k_g_part(int mg, const int *__restrict__ glob, int m, int K,
                                                   const int *__restrict__ con_ptr, const int *__restrict__ con_slot,
                                                   const double *__restrict__ con_w, const double *__restrict__ uRR,
                                                   const double *__restrict__ uRD, const double *__restrict__ uDD,
                                                   const int *__restrict__ sh_idx, double *__restrict__ g3,
                                                   double *__restrict__ gpack, int gwide,
                                                   const double *__restrict__ ctrl_cur) {
    // k_it_g_sh reads these sums only while the loop runs or A(RR^T) was refreshed (RRDONE):
    // the no-op iterations after the exit inside a batch skip the ~6 gathers per constraint
    if (ctrl_cur[C_ACTIVE] == 0.0 && ctrl_cur[C_RRDONE] == 0.0) return;
    const int lanes = gwide ? 64 : 1;
    const int sub = gwide ? (threadIdx.x & 63) : 0;
    const int gid = gwide ? blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6) : blockIdx.x * kBlock + threadIdx.x;
    const int gstride = gwide ? gridDim.x * (kBlock / 64) : gridDim.x * kBlock;
    for (int g = gid; g < mg; g += gstride) {
        const int i = glob[g];
        double a0 = 0.0, a1 = 0.0, a2 = 0.0;
        for (int k = 0; k < K; ++k) {   // cone-major constraint rows k m + i
            const long row = (long)k * m + i;
            for (int e = con_ptr[row] + sub; e < con_ptr[row + 1]; e += lanes) {
                const double w = con_w[e];
                const int s = con_slot[e];
                a0 += w * uRR[s];
                a1 += w * uRD[s];
                a2 += w * uDD[s];
            }
        }
        if (gwide) { a0 = wave_sum(a0); a1 = wave_sum(a1); a2 = wave_sum(a2); }
        if (sub != 0) continue;
        const int q = sh_idx[i];
        if (q >= 0) {
            gpack[3L * q] = a0; gpack[3L * q + 1] = a1; gpack[3L * q + 2] = a2;
        } else {
            g3[i] = a0; g3[m + i] = a1; g3[2L * m + i] = a2;
        }
    }
}

// G2: from the totals, per global constraint: A(RR^T) and its residual (after a fold), q0,
// q1 = 2 A(sym RD^T), q2 = A(DD^T) and rec -- on every holder --, the line-search dots and
// the residual counted by the primary holder only (cmask).  Six partials.
__global__ void __launch_bounds__(kBlock) k_it_g_sh(int mg, const int *__restrict__ glob, int m,
                                                    const int *__restrict__ sh_idx, const double *__restrict__ g3,
                                                    const double *__restrict__ gpack,
                                                    const double *__restrict__ cmask, const double *__restrict__ b,
                                                    double *__restrict__ cvs, const double *__restrict__ lam,
                                                    const double *__restrict__ par, const double *__restrict__ ctrl_cur,
                                                    double *__restrict__ rec, double *__restrict__ partB) {
    const bool act = ctrl_cur[C_ACTIVE] != 0.0, rr = ctrl_cur[C_RRDONE] != 0.0;
    const double rho = par[P_RHO], rhoInv = 1.0 / rho;
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int g = blockIdx.x * kBlock + threadIdx.x; g < mg; g += gridDim.x * kBlock) {
        const int i = glob[g];
        const int q = sh_idx[i];
        const double t0 = q >= 0 ? gpack[3L * q] : g3[i];
        const double t1 = q >= 0 ? gpack[3L * q + 1] : g3[m + i];
        const double t2 = q >= 0 ? gpack[3L * q + 2] : g3[2L * m + i];
        const double pm = cmask[i], bi = b[i];
        if (rr) {
            cvs[i] = t0;
            const double dd = bi - t0;
            acc[5] += pm * (dd * dd);
        }
        if (!act) continue;
        const double v1 = 2.0 * t1, v2 = t2;
        const double ci = cvs[i], li = lam[i];
        const double q0 = (bi - ci) + rhoInv * li;
        acc[0] += pm * (v2 * v2); acc[1] += pm * (v1 * v2); acc[2] += pm * (q0 * v2);
        acc[3] += pm * (v1 * v1); acc[4] += pm * (q0 * v1);
        double2 *r = reinterpret_cast<double2 *>(rec + 4L * i);
        r[0] = make_double2(ci, v1);
        r[1] = make_double2(v2, (-li) + (-rho) * bi);
    }
    write_partials<6>(acc, partB, blockIdx.x);
}

// G3 (one thread): the phase-1 test of k_it_g on the summed residuals (stage B's local
// constraints, totC[9], and G2's global ones, totB[5]), then the stage-B activity.
__global__ void k_g_ph1(const double *__restrict__ par, double *__restrict__ ctrl_cur,
                        const double *__restrict__ totC, const double *__restrict__ totB) {
    if (threadIdx.x != 0) return;
    bool act = ctrl_cur[C_ACTIVE] != 0.0;
    double ex = ctrl_cur[C_EXIT];
    if (ctrl_cur[C_RRDONE] != 0.0) {
        const double pinf1 = sqrt(totC[9] + totB[5]) / (1.0 + par[P_BN1]);
        const double pinfinf = pinf1 * (1.0 + par[P_BN1]) / (1.0 + par[P_BNINF]);
        if ((pinfinf <= par[P_PH1TOL]) && ((par[P_GAP] <= par[P_PH1TOL]) || (par[P_HIGHACC] == 0.0))) {
            act = false;
            ex = EXIT_PHASE1;
        }
        ctrl_cur[C_PINF1] = pinf1;
        ctrl_cur[C_PINFINF] = pinfinf;
    }
    ctrl_cur[C_ACT2] = act ? 1.0 : 0.0;
    ctrl_cur[C_EXIT2] = ex;
}

// an m-vector's shared entries <-> the packed buffer (sum over shards in between)
__global__ void __launch_bounds__(kBlock) k_pack_shared(int m, const int *__restrict__ sh_idx, double *__restrict__ v,
                                                        double *__restrict__ pk, int unpack) {
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < m; i += gridDim.x * kBlock) {
        const int q = sh_idx[i];
        if (q < 0) continue;
        if (unpack) v[i] = pk[q];
        else pk[q] = v[i];
    }
}

// B.  Line search (every block, from A's and G's partials), then per row: R_new =
// R + tau D (written to the other factor buffer; neighbours' rows recomputed), S =
// C + A^*(M1) per neighbour slot with M1 = -lam - rho b + rho (A(RR^T) + tau q1 +
// tau^2 q2) from rec (ALMupdateVar lorads_alm.c:826-830, :1351-1353, ALMSetGrad
// :38-57), G_new = 2 S R_new, A(R_new R_new^T) on the lower slots with the local
// constraints' values and residual (primalInfeasibility), the L-BFGS pair s = tau D,
// y = G_new - G_old (setlbfgsHisTwo :842-863) and nine dots.  Partials written (10).
// MODE 0: the whole stage (small regime, and the bandwidth regime's plain rows: b_fused_on).
// Split in two launches where the second half is the long-row / tiled kernels or the solve is
// sharded: MODE 1 = line search + R_new = R + tau D of every row (own and halo), MODE 2 = the
// rest with the neighbours' R_new read back (one row per neighbour instead of R and D) and tau
// from MODE 1.
#ifndef LRS_BW_UB
#define LRS_BW_UB 1   // neighbours in flight per lane group in the bandwidth regime's fused stage B
#endif
#ifndef LRS_BW_UB_MINB
#define LRS_BW_UB_MINB 3
#endif
// Occupancy bound of k_it_b (the launch bound's second argument): the fused bandwidth-regime
// kernel (U == 1, MODE 0) holds the row's R, D, gradient and the L-BFGS operands at once and
// spilled 8-15 VGPRs at 6 / 5 waves a SIMD (44 B a lane of scratch at G81 r = 64: ~20 MB of
// extra writes per launch, profiles/r06a_g81_summary.md); one wave a SIMD less keeps it in
// registers.  E = 8 (r > 256) needs the whole file.
constexpr int itb_min_blocks(int E, int U, int MODE) {
    return U == 1 ? (E >= 8 ? 2 : MODE == 0 ? (E >= 3 ? 4 : 5) : (E >= 3 ? 5 : 6))
                  : (MODE == 0 && U == LRS_BW_UB ? LRS_BW_UB_MINB : 1);
}
template <int G, int E, int U, int MODE>
__global__ void __launch_bounds__(kRowBlock, itb_min_blocks(E, U, MODE)) k_it_b(
    int n, int ld, long foff, const int *__restrict__ adj_ptr, const int *__restrict__ adj_low,
    const int *__restrict__ adj_col, const int *__restrict__ adj_slot, double *Rb0, double *Rb1,
    const double *__restrict__ Dall, double *G0, double *G1, double *s0, double *y0, double *s1, double *y1,
    double *__restrict__ uRR, const double *__restrict__ Craw, const int *__restrict__ slot_ptr,
    const int *__restrict__ slot_con, const double *__restrict__ slot_a, const double2 *__restrict__ slot1,
    const double *__restrict__ rec,
    const int *__restrict__ loc_ptr, const int *__restrict__ loc_con, const double *__restrict__ loc_w,
    const double2 *__restrict__ loc1,
    const double *__restrict__ b, double *__restrict__ cvs, const double *__restrict__ par,
    const double *__restrict__ ctrl, const double *__restrict__ partA, int nblkA, const double *__restrict__ partB,
    int nblkB, double *__restrict__ ls_cur, int L, double *__restrict__ partC, int pblk_off, int T, int row0,
    int nall, int pstr, double *hmirror, double seq, double *CRb, const double *__restrict__ CDb) {
    __shared__ double gsh[kRowBlock * E];   // team reduction of the row gradient (T > 1)
    __shared__ double red[12];
    __shared__ double ls[LS_N];
    __shared__ double cs[4];
    LRS_TS(2, 0);
    LRS_BLK_BEGIN();
    if constexpr (MODE != 2) mirror_ctrl(ctrl, hmirror, seq);
    if (threadIdx.x == 0) { cs[0] = ctrl[C_ACT2]; cs[1] = ctrl[C_GCUR]; cs[2] = ctrl[C_HEAD]; cs[3] = ctrl[C_RCUR]; }
    __syncthreads();
    if (cs[0] == 0.0) return;
    if constexpr (MODE == 2) {
        // second half of a split stage: the line search the first half wrote
        if (threadIdx.x < LS_N) ls[threadIdx.x] = ls_cur[threadIdx.x];
        __syncthreads();
    } else {
    reduce_partials<7, kRowBlock>(partA, nblkA, red, pstr);
    if (nblkB > 0) {
        reduce_partials<5, kRowBlock>(partB, nblkB, red + 7, pstr);
        if (threadIdx.x == 0) {
#pragma unroll
            for (int q = 0; q < 5; ++q) red[2 + q] += red[7 + q];
        }
        __syncthreads();
    }
    LRS_TS(2, 1);
    if (threadIdx.x < 64) line_search_t<true>(par, red[0], red[1], red + 2, ls);   // wave 0
    __syncthreads();
    LRS_TS(2, 2);
    if (pblk_off == 0 && blockIdx.x == 0 && threadIdx.x < LS_N) ls_cur[threadIdx.x] = ls[threadIdx.x];
    }   // MODE != 2
    if (ls[LS_FLAG] != 0.0) return;
    const double tau = ls[LS_TAU], tau2 = tau * tau, rho = par[P_RHO];
    const int gcur = (int)cs[1], h = (int)cs[2];
    const double *__restrict__ R = (cs[3] == 0.0 ? Rb0 : Rb1) + foff;
    double *__restrict__ Rn = (cs[3] == 0.0 ? Rb1 : Rb0) + foff;
    const double *__restrict__ D = Dall + foff;
    double *__restrict__ Gold = (gcur == 0 ? G0 : G1) + foff;
    double *__restrict__ Gnew = (gcur == 0 ? G1 : G0) + foff;
    double *__restrict__ sh = (h == 0 ? s0 : s1) + foff;
    double *__restrict__ yh = (h == 0 ? y0 : y1) + foff;
    const double *__restrict__ so = (h == 0 ? s1 : s0) + foff;
    const double *__restrict__ yo = (h == 0 ? y1 : y0) + foff;
    const bool two = (L == 2);
    if constexpr (MODE == 1) {
        // R_new = R + tau D for every local row (the shard's halo included)
        const int lane1 = threadIdx.x & (G - 1);
        const int grp1 = (blockIdx.x * kRowBlock + threadIdx.x) / G;
        const int ngrp1 = gridDim.x * kRowBlock / G;
        for (int l = grp1; l < nall; l += ngrp1) {
            const long ol = (long)l * ld + lane1 * E;
            double rv[E], dv[E];
            ld_row<E>(R + ol, rv);
            ld_row<E>(D + ol, dv);
#pragma unroll
            for (int e = 0; e < E; ++e) rv[e] += tau * dv[e];
            st_row<E>(Rn + ol, rv);
        }
        return;
    }
    // lane groups of G lanes; a team of T groups shares one row (dense rows): member m
    // takes interleaved chunks of U neighbours, the partial gradients meet in LDS.  The
    // row loop runs the same trip count in every team of a block (barriers inside).
    const int lane = threadIdx.x & (G - 1);
    const int grp = (blockIdx.x * kRowBlock + threadIdx.x) / G;
    const int ngrp = gridDim.x * kRowBlock / G;
    const int team = grp / T, mem = grp % T;
    const int tpb = (kRowBlock / G) / T;                 // teams per block
    const int team_local = team - blockIdx.x * tpb;
    // block-uniform trip count (the team reduction has barriers inside the loop)
    const RowRange rr = row_range(n, tpb, 0);
    // acc: GG, ys, yy, sG, yG, soG, yoG, soy, yoy, residual
    double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int ib = rr.first; ib < rr.end; ib += rr.stride) {
    const int i = row0 + ib + team_local;   // rows [row0, row0 + n) (a shard: n = owned rows)
    const bool valid = ib + team_local < rr.end;
    double ri[E], di[E], g[E];
    const long oi = (long)(valid ? i : 0) * ld + lane * E;
#pragma unroll
    for (int e = 0; e < E; ++e) g[e] = 0.0;
    if (valid) {
        if constexpr (MODE == 2) {
            ld_row<E>(Rn + oi, ri);   // D of the row is read at the end (s = tau D): fewer live registers
        } else {
            ld_row<E>(D + oi, di);
            ld_row<E>(R + oi, ri);
#pragma unroll
            for (int e = 0; e < E; ++e) ri[e] += tau * di[e];
            if (mem == 0) st_row<E>(Rn + oi, ri);
        }
        const int kb = adj_ptr[i], kl = adj_low[i], ke = adj_ptr[i + 1];
#ifdef LRS_PHASE_TIMING
        if (threadIdx.x == 0 && ib == blockIdx.x * tpb && kb >= 0 && ri[0] != 12345.678) LRS_TS(2, 6);
#endif
        // neighbours U at a time (indices clamped to the row; extra lanes add 0)
        for (int k0 = kb + mem * U; k0 < ke; k0 += T * U) {
            int jj[U], ss[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = min(k0 + u, ke - 1);
                jj[u] = adj_col[k];
                ss[u] = adj_slot[k];
            }
            double rj[U][E], dj[U][E], sv[U];
            double2 s1[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (MODE == 2) {
                    ld_row<E>(Rn + (long)jj[u] * ld + lane * E, rj[u]);
                } else {
                    ld_row<E>(R + (long)jj[u] * ld + lane * E, rj[u]);
                    ld_row<E>(D + (long)jj[u] * ld + lane * E, dj[u]);
                }
                sv[u] = Craw[ss[u]];
                s1[u] = slot1[ss[u]];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                // S[slot] = C + sum_con M1(con) a  (addObjCoeff + sdpDataWSum); a single entry
                // comes with the slot's record, several from the slot lists
                const int c1 = (int)s1[u].y;
                const int e0 = c1 == -2 ? slot_ptr[ss[u]] : 0;
                const int e1 = c1 == -2 ? slot_ptr[ss[u] + 1] : (c1 >= 0 ? 1 : 0);
                for (int e = e0; e < e1; ++e) {
                    const int con = c1 >= 0 ? c1 : slot_con[e];
                    const double2 *r = reinterpret_cast<const double2 *>(rec + 4L * con);
                    const double2 ra = r[0], rb = r[1];
                    double cv = ra.x + tau * ra.y;
                    cv = cv + tau2 * rb.x;
                    const double M1 = rb.y + rho * cv;
                    sv[u] += M1 * (c1 >= 0 ? s1[u].x : slot_a[e]);
                }
                if constexpr (MODE != 2) {
#pragma unroll
                    for (int e = 0; e < E; ++e) rj[u][e] += tau * dj[u][e];
                }
            }
#ifdef LRS_PHASE_TIMING
            if (threadIdx.x == 0 && ib == blockIdx.x * tpb && rj[0][0] != 12345.678 && sv[0] != 12345.678)
                LRS_TS(2, k0 == kb ? 7 : 9);
#endif
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = k0 + u;
                if (k < ke) {
#pragma unroll
                    for (int e = 0; e < E; ++e) g[e] += sv[u] * rj[u][e];
                }
                if (k < kl) {   // lower entry (j <= i): A(RR^T) slot owned by this row
                    double d = 0.0;
#pragma unroll
                    for (int e = 0; e < E; ++e) d += ri[e] * rj[u][e];
                    d = group_sum<G>(d);
                    if (lane == 0) {
                        uRR[ss[u]] = d;
                        const double2 l1u = loc1[ss[u]];
                        const int c1 = (int)l1u.y;
                        const int e0 = c1 == -2 ? loc_ptr[ss[u]] : 0;
                        const int e1 = c1 == -2 ? loc_ptr[ss[u] + 1] : (c1 >= 0 ? 1 : 0);
                        for (int e = e0; e < e1; ++e) {
                            const int ci = c1 >= 0 ? c1 : loc_con[e];
                            const double tot = (c1 >= 0 ? l1u.x : loc_w[e]) * d;
                            cvs[ci] = tot;
                            const double dd = b[ci] - tot;
                            acc[9] += dd * dd;
                        }
                    }
                }
            }
#ifdef LRS_PHASE_TIMING
            if (threadIdx.x == 0 && ib == blockIdx.x * tpb && acc[9] != 12345.678) LRS_TS(2, k0 == kb ? 8 : 10);
#endif
        }
    }   // valid
    if (T > 1) {
        // team reduction: member 0 of each team sums the members' partials in order
#pragma unroll
        for (int e = 0; e < E; ++e) gsh[threadIdx.x * E + e] = g[e];
        __syncthreads();
        if (mem == 0 && valid) {
            const int base = (team_local * T) * G + lane;
#pragma unroll
            for (int e = 0; e < E; ++e) g[e] = gsh[base * E + e];
            for (int t = 1; t < T; ++t)
#pragma unroll
                for (int e = 0; e < E; ++e) g[e] += gsh[(base + t * G) * E + e];
        }
        __syncthreads();
    }
    if (mem == 0 && valid) {
        double sv[E], yv[E], go[E];
        if constexpr (MODE == 2) ld_row<E>(D + oi, di);
        ld_row<E>(Gold + oi, go);
        if (CRb) {
            // dense objective: C R_new = C R + tau C D (carried), S R_new += C R_new
            double cr[E], cd[E];
            ld_row<E>(CRb + foff + oi, cr);
            ld_row<E>(CDb + foff + oi, cd);
#pragma unroll
            for (int e = 0; e < E; ++e) {
                cr[e] += tau * cd[e];
                g[e] += cr[e];
            }
            st_row<E>(CRb + foff + oi, cr);
        }
#pragma unroll
        for (int e = 0; e < E; ++e) g[e] *= 2.0;
#pragma unroll
        for (int e = 0; e < E; ++e) { sv[e] = tau * di[e]; yv[e] = g[e] - go[e]; }
        st_row<E>(Gnew + oi, g);
        st_row<E>(sh + oi, sv);
        st_row<E>(yh + oi, yv);
#ifdef LRS_PHASE_TIMING
        if (threadIdx.x == 0 && ib == blockIdx.x * tpb && go[0] != 12345.678) LRS_TS(2, 11);
#endif
#pragma unroll
        for (int e = 0; e < E; ++e) {
            acc[0] += g[e] * g[e];
            acc[1] += yv[e] * sv[e];
            acc[2] += yv[e] * yv[e];
            acc[3] += sv[e] * g[e];
            acc[4] += yv[e] * g[e];
        }
        if (two) {
            double sov[E], yov[E];
            ld_row<E>(so + oi, sov);
            ld_row<E>(yo + oi, yov);
#pragma unroll
            for (int e = 0; e < E; ++e) {
                acc[5] += sov[e] * g[e];
                acc[6] += yov[e] * g[e];
                acc[7] += sov[e] * yv[e];
                acc[8] += yov[e] * yv[e];
            }
        }
    }   // mem == 0
    }   // rows
    // sharded solve: the halo rows (the other shards' rows this one reads) take the same
    // update R_new = R + tau D, D of the halo received after stage A's first half
    if (MODE == 0 && nall > n) {
        for (int q = grp; q < nall - n; q += ngrp) {
            const int l = q < row0 ? q : q + n;
            const long ol = (long)l * ld + lane * E;
            double rv[E], dv[E];
            ld_row<E>(R + ol, rv);
            ld_row<E>(D + ol, dv);
#pragma unroll
            for (int e = 0; e < E; ++e) rv[e] += tau * dv[e];
            st_row<E>(Rn + ol, rv);
        }
    }
    LRS_TS(2, 3);
    write_partials<10, kRowBlock>(acc, partC, pblk_off + blockIdx.x);
    LRS_TS_END(2, 4);
#ifdef LRS_PHASE_TIMING
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int q_ = 5; q_ < 12; ++q_) g_phase[2][q_] = g_phase_tmp[2][q_];
#endif
    LRS_BLK_END(2);
}

// ------------------------------------------------------------------------
// B, bandwidth regime, plain rows (T == 1): the fused stage of k_it_b<., ., 1, 0> restructured
// around its dependency chain.  k_it_b walks a row's entries one after another, each entry three
// dependent memory trips deep (adjacency -> R_j, D_j and the slot record -> the constraint
// record) plus two more on lower entries (the local constraints after the dot product): about
// 20 trips a row on G81, where every lane group holds one or two rows and the launch is latency-
// bound (32 us for 96 MB, 0.37 of HBM).  Here a row takes four trips, as in k_lat_b's row
// waves: (1) the row header and own operands, (2) the first NO + 1 entries' columns and slots,
// (3) their factor rows and, lane-distributed (lane u of the group: entry u, lane NO: the
// diagonal), each entry's slot, objective and local-constraint records, (4) the constraint
// records and b.  Lane u finishes entry u's S value (its multi-constraint slot list too); the
// entries are then summed in k_it_b's adjacency order and their slots finished by lane 0 with
// the records broadcast from their lanes -- the same arithmetic in the same order, bitwise
// k_it_b's results (tests/test_gpu_bw_kernels.py).  The further entries of a long row take
// k_it_b's walk.  (The first row's trips issued before the block's line search, as k_lat_b's
// row waves do beside its control wave, kept ~100 VGPRs live through the line search: 148-440 B
// a lane of spills.)
// ------------------------------------------------------------------------
constexpr int kBwNo = 4;   // off-diagonal entries prefetched per row (torus rows: all of them)
template <int G, int E, int NO>
struct BwRow {
    int i, kb, kl, ke, no, sd;
    bool dg;
    double ri[E], di[E];
    int ss[NO];
    bool lw[NO];
    double rjp[NO][E], djp[NO][E];
    // this lane's entry (lane u < NO: off-diagonal entry u; lane NO: the diagonal)
    int msl;
    double msv, mbq;
    double2 ms1, ml1, mra, mrb;
};

template <int G, int E, int NO>
__device__ __forceinline__ void bw_prefetch(BwRow<G, E, NO> &w, int i, int ld, int lane, int m,
                                            const int *__restrict__ adj_ptr, const int *__restrict__ adj_low,
                                            const int *__restrict__ adj_col, const int *__restrict__ adj_slot,
                                            const double *__restrict__ R, const double *__restrict__ D,
                                            const double *__restrict__ Craw, const double2 *__restrict__ slot1,
                                            const double2 *__restrict__ loc1, const double *__restrict__ rec,
                                            const double *__restrict__ b) {
    w.i = i;
    const long oi = (long)i * ld + lane * E;
    w.kb = adj_ptr[i];
    w.kl = adj_low[i];
    w.ke = adj_ptr[i + 1];
    ld_row<E>(R + oi, w.ri);
    ld_row<E>(D + oi, w.di);
    const int nt = w.ke - w.kb;
    const int kd = (nt > 0 && w.kl > w.kb) ? w.kl - 1 : w.kb;   // the diagonal is the last lower entry
    const int kdc = nt > 0 ? kd : 0;
    const int jd = adj_col[kdc];
    w.sd = adj_slot[kdc];
    int ja[NO + 1], sa[NO + 1];
#pragma unroll
    for (int u = 0; u <= NO; ++u) {
        const int k = nt > 0 ? w.kb + min(u, nt - 1) : 0;
        ja[u] = adj_col[k];
        sa[u] = adj_slot[k];
    }
    w.dg = nt > 0 && w.kl > w.kb && jd == i;
    w.no = nt - (w.dg ? 1 : 0);
    const int pd = w.dg ? w.kl - 1 - w.kb : NO + 1;   // the diagonal's position among the first
    int my = w.sd;
#pragma unroll
    for (int u = 0; u < NO; ++u) {
        const bool past = u >= pd;
        const int j = past ? ja[u + 1] : ja[u];
        w.ss[u] = past ? sa[u + 1] : sa[u];
        w.lw[u] = w.kb + u + (past ? 1 : 0) < w.kl;
        const long oj = (long)(u < w.no ? j : i) * ld + lane * E;
        ld_row<E>(R + oj, w.rjp[u]);
        ld_row<E>(D + oj, w.djp[u]);
        if (lane == u) my = w.ss[u];
    }
    w.msl = my;
    w.msv = Craw[my];
    w.ms1 = slot1[my];
    w.ml1 = loc1[my];
    // slots without a single constraint read the row's own (spread, cached) index instead of a
    // common one (k_lat_b)
    const int ispare = min(i, m - 1);
    const int c1 = (int)w.ms1.y >= 0 ? (int)w.ms1.y : ispare;
    const int cl = (int)w.ml1.y >= 0 ? (int)w.ml1.y : ispare;
    const double2 *r = reinterpret_cast<const double2 *>(rec + 4L * c1);
    w.mra = r[0];
    w.mrb = r[1];
    w.mbq = b[cl];
}

// occupancy bound: the row state without spills (E <= 2: 128 VGPRs, E = 3: 168, above: 256)
constexpr int bwb_min_blocks(int E) { return E <= 2 ? 4 : (E == 3 ? 3 : 2); }
template <int G, int E, int NO>
__global__ void __launch_bounds__(kRowBlock, bwb_min_blocks(E)) k_bw_b(
    int n, int ld, long foff, const int *__restrict__ adj_ptr, const int *__restrict__ adj_low,
    const int *__restrict__ adj_col, const int *__restrict__ adj_slot, double *Rb0, double *Rb1,
    const double *__restrict__ Dall, double *G0, double *G1, double *s0, double *y0, double *s1, double *y1,
    double *__restrict__ uRR, const double *__restrict__ Craw, const int *__restrict__ slot_ptr,
    const int *__restrict__ slot_con, const double *__restrict__ slot_a, const double2 *__restrict__ slot1,
    const double *__restrict__ rec, const int *__restrict__ loc_ptr, const int *__restrict__ loc_con,
    const double *__restrict__ loc_w, const double2 *__restrict__ loc1, const double *__restrict__ b,
    double *__restrict__ cvs, const double *__restrict__ par, const double *__restrict__ ctrl,
    const double *__restrict__ partA, int nblkA, const double *__restrict__ partB, int nblkB,
    double *__restrict__ ls_cur, int L, double *__restrict__ partC, int pblk_off, int row0, int m, int pstr,
    double *hmirror, double seq, double *CRb, const double *__restrict__ CDb) {
    static_assert(NO < G, "lane NO holds the diagonal's records");
    __shared__ double red[12];
    __shared__ double ls[LS_N];
    LRS_TS(2, 0);
    LRS_BLK_BEGIN();
    mirror_ctrl(ctrl, hmirror, seq);
    if (ctrl[C_ACT2] == 0.0) return;
    const int gcur = (int)ctrl[C_GCUR], h = (int)ctrl[C_HEAD];
    const bool r1 = ctrl[C_RCUR] != 0.0;
    const double *__restrict__ R = (r1 ? Rb1 : Rb0) + foff;
    double *__restrict__ Rn = (r1 ? Rb0 : Rb1) + foff;
    const double *__restrict__ D = Dall + foff;
    double *__restrict__ Gold = (gcur == 0 ? G0 : G1) + foff;
    double *__restrict__ Gnew = (gcur == 0 ? G1 : G0) + foff;
    double *__restrict__ sh = (h == 0 ? s0 : s1) + foff;
    double *__restrict__ yh = (h == 0 ? y0 : y1) + foff;
    const double *__restrict__ so = (h == 0 ? s1 : s0) + foff;
    const double *__restrict__ yo = (h == 0 ? y1 : y0) + foff;
    const bool two = (L == 2);
    const int lane = threadIdx.x & (G - 1);
    const RowRange rr = row_range(n, kRowBlock / G, (int)threadIdx.x / G);
    // the line search from stage A's (and G's) partials, every block (k_it_b MODE 0)
    reduce_partials<7, kRowBlock>(partA, nblkA, red, pstr);
    if (nblkB > 0) {
        reduce_partials<5, kRowBlock>(partB, nblkB, red + 7, pstr);
        if (threadIdx.x == 0) {
#pragma unroll
            for (int q = 0; q < 5; ++q) red[2 + q] += red[7 + q];
        }
        __syncthreads();
    }
    LRS_TS(2, 1);
    if (threadIdx.x < 64) line_search_t<true>(par, red[0], red[1], red + 2, ls);   // wave 0
    __syncthreads();
    LRS_TS(2, 2);
    if (pblk_off == 0 && blockIdx.x == 0 && threadIdx.x < LS_N) ls_cur[threadIdx.x] = ls[threadIdx.x];
    if (ls[LS_FLAG] != 0.0) return;
    const double tau = ls[LS_TAU], tau2 = tau * tau, rho = par[P_RHO];
    // acc: GG, ys, yy, sG, yG, soG, yoG, soy, yoy, residual
    double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int ib = rr.first; ib < rr.end; ib += rr.stride) {
        BwRow<G, E, NO> w;
        bw_prefetch<G, E, NO>(w, row0 + ib, ld, lane, m, adj_ptr, adj_low, adj_col, adj_slot, R, D, Craw, slot1, loc1,
                              rec, b);
        const int i = w.i;
        const long oi = (long)i * ld + lane * E;
        double go[E], sov[E], yov[E];
        ld_row<E>(Gold + oi, go);
        if (two) { ld_row<E>(so + oi, sov); ld_row<E>(yo + oi, yov); }
        double ri[E], g[E];
#pragma unroll
        for (int e = 0; e < E; ++e) { ri[e] = w.ri[e] + tau * w.di[e]; g[e] = 0.0; }
        st_row<E>(Rn + oi, ri);
        // this lane's entry: S = C + A^*(M1) on its slot (ALMSetGrad lorads_alm.c:38-57)
        double msv = w.msv;
        {
            const int c1 = (int)w.ms1.y;
            const int e0 = c1 == -2 ? slot_ptr[w.msl] : 0;
            const int e1 = c1 == -2 ? slot_ptr[w.msl + 1] : (c1 >= 0 ? 1 : 0);
            for (int e = e0; e < e1; ++e) {
                double2 x = w.mra, y = w.mrb;
                if (c1 < 0) {
                    const double2 *r = reinterpret_cast<const double2 *>(rec + 4L * slot_con[e]);
                    x = r[0];
                    y = r[1];
                }
                double cv = x.x + tau * x.y;
                cv = cv + tau2 * y.x;
                const double M1 = y.y + rho * cv;
                msv += M1 * (c1 >= 0 ? w.ms1.x : slot_a[e]);
            }
        }
        // k_it_b's order (and its lane-0 code for the slots): every entry in adjacency order, the
        // diagonal at its place (the last lower entry); positions [0, win) from the prefetch --
        // the first NO off-diagonal entries and a diagonal among them -- the rest walked
        const int nt = w.ke - w.kb;
        const int pd = w.dg ? w.kl - 1 - w.kb : (1 << 30);
        const int win = min(nt, pd <= NO ? NO + 1 : NO);
        auto lower_slot = [&](int sl, double d, double wx, int cl, double bq) {
            uRR[sl] = d;
            const int f0 = cl == -2 ? loc_ptr[sl] : 0;
            const int f1 = cl == -2 ? loc_ptr[sl + 1] : (cl >= 0 ? 1 : 0);
            for (int e = f0; e < f1; ++e) {
                const int ci = cl >= 0 ? cl : loc_con[e];
                const double tot = (cl >= 0 ? wx : loc_w[e]) * d;
                cvs[ci] = tot;
                const double dd = (cl >= 0 ? bq : b[ci]) - tot;
                acc[9] += dd * dd;
            }
        };
#pragma unroll
        for (int p = 0; p <= NO; ++p) {
            if (p < win) {
                const bool isd = p == pd, past = p > pd;
                double rj[E];
                if (isd) {   // R_new of the row itself as k_it_b sees it: a second copy
#pragma unroll
                    for (int e = 0; e < E; ++e) rj[e] = opaque(ri[e]);
                } else {
                    const int ua = p < NO ? p : NO - 1, ub = p > 0 ? p - 1 : 0;
#pragma unroll
                    for (int e = 0; e < E; ++e)
                        rj[e] = (past ? w.rjp[ub][e] : w.rjp[ua][e]) + tau * (past ? w.djp[ub][e] : w.djp[ua][e]);
                }
                const int o = isd ? NO : (past ? p - 1 : p);   // the lane holding this entry's records
                const double su = bcast_d<G>(msv, o);
#pragma unroll
                for (int e = 0; e < E; ++e) g[e] += su * rj[e];
                if (w.kb + p < w.kl) {   // lower entry (j <= i): A(RR^T) slot owned by this row
                    double d = 0.0;
#pragma unroll
                    for (int e = 0; e < E; ++e) d += ri[e] * rj[e];
                    d = group_sum<G>(d);
                    const int sl = bcast_i<G>(w.msl, o);
                    const double wx = bcast_d<G>(w.ml1.x, o), wy = bcast_d<G>(w.ml1.y, o), bq = bcast_d<G>(w.mbq, o);
                    if (lane == 0) lower_slot(sl, d, wx, (int)wy, bq);
                }
            }
        }
        // the rest of a long row (the diagonal among them when it lies past the window): k_it_b's walk
        for (int k = w.kb + win; k < w.ke; ++k) {
            const int j = adj_col[k], sl = adj_slot[k];
            const long oj = (long)j * ld + lane * E;
            double rj[E], dj[E];
            ld_row<E>(R + oj, rj);
            ld_row<E>(D + oj, dj);
#pragma unroll
            for (int e = 0; e < E; ++e) rj[e] += tau * dj[e];
            const double2 s1u = slot1[sl];
            const int c1 = (int)s1u.y;
            double sv = Craw[sl];
            const int e0 = c1 == -2 ? slot_ptr[sl] : 0;
            const int e1 = c1 == -2 ? slot_ptr[sl + 1] : (c1 >= 0 ? 1 : 0);
            for (int e = e0; e < e1; ++e) {
                const int con = c1 >= 0 ? c1 : slot_con[e];
                const double2 *r = reinterpret_cast<const double2 *>(rec + 4L * con);
                const double2 ra = r[0], rb = r[1];
                double cv = ra.x + tau * ra.y;
                cv = cv + tau2 * rb.x;
                const double M1 = rb.y + rho * cv;
                sv += M1 * (c1 >= 0 ? s1u.x : slot_a[e]);
            }
#pragma unroll
            for (int e = 0; e < E; ++e) g[e] += sv * rj[e];
            if (k < w.kl) {
                double d = 0.0;
#pragma unroll
                for (int e = 0; e < E; ++e) d += ri[e] * rj[e];
                d = group_sum<G>(d);
                if (lane == 0) {
                    const double2 l1u = loc1[sl];
                    const int cl = (int)l1u.y;
                    lower_slot(sl, d, l1u.x, cl, cl >= 0 ? b[cl] : 0.0);
                }
            }
        }
        // gradient G_new = 2 S R_new, L-BFGS pair s = tau D, y = G_new - G_old, dots
        if (CRb) {
            // dense objective: C R_new = C R + tau C D (carried), S R_new += C R_new
            double cr[E], cd[E];
            ld_row<E>(CRb + foff + oi, cr);
            ld_row<E>(CDb + foff + oi, cd);
#pragma unroll
            for (int e = 0; e < E; ++e) {
                cr[e] += tau * cd[e];
                g[e] += cr[e];
            }
            st_row<E>(CRb + foff + oi, cr);
        }
        double sv2[E], yv[E];
#pragma unroll
        for (int e = 0; e < E; ++e) g[e] *= 2.0;
#pragma unroll
        for (int e = 0; e < E; ++e) { sv2[e] = tau * w.di[e]; yv[e] = g[e] - go[e]; }
        st_row<E>(Gnew + oi, g);
        st_row<E>(sh + oi, sv2);
        st_row<E>(yh + oi, yv);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            acc[0] += g[e] * g[e];
            acc[1] += yv[e] * sv2[e];
            acc[2] += yv[e] * yv[e];
            acc[3] += sv2[e] * g[e];
            acc[4] += yv[e] * g[e];
        }
        if (two) {
#pragma unroll
            for (int e = 0; e < E; ++e) {
                acc[5] += sov[e] * g[e];
                acc[6] += yov[e] * g[e];
                acc[7] += sov[e] * yv[e];
                acc[8] += yov[e] * yv[e];
            }
        }
    }
    LRS_TS(2, 3);
    write_partials<10, kRowBlock>(acc, partC, pblk_off + blockIdx.x);
    LRS_TS_END(2, 4);
    LRS_BLK_END(2);
}

// ------------------------------------------------------------------------
// Latency regime (small n: every row's lane group resident at once).  Same work and
// arithmetic as k_it_a<.,.,.,0> / k_it_b<.,.,.,0>, restructured around the critical path
// of one launch: the last wave of each block is a CONTROL wave (the cross-block reduction
// of the previous stage's partials, then ctrl_step, resp. the line search); the other
// seven are ROW waves, one row per lane group.  Every load that does not depend on this
// iteration's control -- the row header, the first NB adjacency entries, the own row
// operands, the slot and constraint records -- is issued by the row waves before the
// block barrier, so its latency runs beside the reduction and the serial control instead
// of after them.  Only the neighbours' factor rows (U at a time) are loaded afterwards.
// ------------------------------------------------------------------------
// Row block of latency-kernel block b: the row blocks of group x = b % 8 (one XCD under the
// round-robin dispatch; speed only, any placement is correct) are the contiguous range
// [start(x), start(x) + count(x)), so a row's w-apart grid neighbours are read through the same
// L2 instead of being fetched again by another XCD (a bijection on [0, nrb); slice blocks
// b >= nrb unchanged).  G67: FETCH_SIZE per dispatch 12.6 -> 7.0 MB (k_lat_a), 7.7 -> 4.6 MB
// (k_lat_b), 42.4K -> 45.5K it/s (scripts/latxcd_check.sh).  LRS_NO_LAT_XCD: identity map.
__device__ __forceinline__ int lat_row_block(int b, int nrb) {
#ifndef LRS_NO_LAT_XCD
    if (b >= nrb || nrb < 16) return b;
    const int x = b & 7, q8 = nrb >> 3, rem = nrb & 7;
    const int start = x * q8 + min(x, rem);
    return start + (b >> 3);
#else
    (void)nrb;
    return b;
#endif
}
// Latency-kernel blocks: w row waves (1 <= w <= 7) and one control wave, w chosen per launch at
// run time (blockDim.x = 64 (w + 1)) so that the grid spreads the row waves over as many CUs as
// it can (<= 256 blocks): the row waves' vector memory instructions per CU bound the launch
// (G67: 7 row waves a block, 179 blocks -> 5, 250 blocks: k_lat_a 9.1 -> 8.7, k_lat_b 10.1 ->
// 9.55 us, scripts/gpu_r04v.sh).
constexpr int kLatNT = 512;                      // the largest block (launch bounds)
constexpr int kLatRowWaves = kLatNT / 64 - 1;
constexpr int kLatRows = kLatRowWaves * 64;      // row-wave threads of the largest block
constexpr int kLatMaxPartials = 256;             // producer blocks one control wave reduces
constexpr int kSliceA = 2;                       // lower entries per lane group in a dense-row slice of A
constexpr int kSliceB = 4;                       // entries per lane group in a dense-row slice of B

// control wave: NV partial vectors summed over 1 <= nblk <= kLatMaxPartials producer blocks
// (lane l takes blocks l, l+64, ...).  Split in two so that the loads can be issued first
// thing in the kernel (clamped, not branched): the wave then waits for one memory trip.
constexpr int kLatQ = kLatMaxPartials / 64;
template <int NV>
__device__ __forceinline__ void load_partials(const double *__restrict__ part, int nblk, double (&x)[kLatQ][NV]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < kLatQ; ++q) {
        const int bc = min(lane + 64 * q, nblk - 1);
#pragma unroll
        for (int v = 0; v < NV; ++v) x[q][v] = part[v * kMaxPartialBlocks + bc];
    }
}
// wave-uniform sums of what load_partials fetched
template <int NV>
__device__ __forceinline__ void sum_partials(const double (&x)[kLatQ][NV], int nblk, double (&out)[NV]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        double a = 0.0;
#pragma unroll
        for (int q = 0; q < kLatQ; ++q) a += (lane + 64 * q < nblk) ? x[q][v] : 0.0;
        out[v] = wave_sum(a);
    }
}
template <int NV>
__device__ __forceinline__ void wave_reduce_partials(const double *__restrict__ part, int nblk, double (&out)[NV]) {
    double x[kLatQ][NV];
    load_partials<NV>(part, nblk, x);
    __builtin_amdgcn_sched_barrier(0);
    sum_partials<NV>(x, nblk, out);
}

// A in the latency regime (k_it_a MODE 0).  NO: off-diagonal lower entries whose operand
// rows are prefetched before the barrier (the diagonal entry, the last lower one in the
// column-sorted adjacency, uses the row's own operands); further ones are loaded after it.
template <int G, int E, int NO>
__global__ void __launch_bounds__(kLatNT) k_lat_a(
    int n, int ld, long foff, const int *__restrict__ adj_ptr, const int *__restrict__ adj_low,
    const int *__restrict__ adj_col, const int *__restrict__ adj_slot, const double *__restrict__ Cw,
    const double *__restrict__ Rb0, const double *__restrict__ Rb1, double *__restrict__ Dall,
    const double *__restrict__ G0, const double *__restrict__ G1, const double *__restrict__ s0a,
    const double *__restrict__ y0a, const double *__restrict__ s1a, const double *__restrict__ y1a,
    double *__restrict__ uRD, double *__restrict__ uDD, const int *__restrict__ loc_ptr,
    const int *__restrict__ loc_con, const double *__restrict__ loc_w, const double2 *__restrict__ loc1,
    const double *__restrict__ b, double *__restrict__ cvs, const double *__restrict__ lam,
    double *__restrict__ rec, int do_glob, int mg, const int *__restrict__ glob, int m, int K,
    const int *__restrict__ con_ptr, const int *__restrict__ con_slot, const double *__restrict__ con_w,
    const double *__restrict__ uRR, const double *__restrict__ par, const double *__restrict__ ctrl_prev,
    double *__restrict__ ctrl_cur, const double *__restrict__ ls_prev, const double *__restrict__ partC, int nblkC,
    double *__restrict__ partA, int pblk_off, int gwide, int nrb, int lrw, int nda, const int *__restrict__ dra) {
    __shared__ double c[C_NCTRL];
    __shared__ double pl[P_NPAR];
    LRS_TS(0, 0);
    LRS_BLK_BEGIN();
    // lrw row waves + the control wave (an argument beside nrb, loaded in the first argument batch:
    // blockDim.x would be one more load before the first branch)
    const int nwv = lrw + 1, rpb = lrw * 64 / G;   // waves, rows of this block
    const bool ctrl_wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) == nwv - 1;   // wave-uniform
    const int lane = threadIdx.x & (G - 1);
    // blocks [0, nrb): one row per lane group.  Blocks past nrb: slices of the dense rows --
    // every lane group of the block takes kSliceA consecutive lower entries of one dense row
    // (the rows' own groups skip those entries; A's results are per slot, nothing to combine)
    const bool slice = (int)blockIdx.x >= nrb;
    int i = lat_row_block((int)blockIdx.x, nrb) * rpb + (int)threadIdx.x / G, sq = 0;
    if (slice) {
        const int per = rpb * kSliceA;
        int q = (int)blockIdx.x - nrb, L = 0;
        for (; L < nda - 1; ++L) {
            const int r = dra[L], ns = (adj_low[r] - adj_ptr[r] + per - 1) / per;
            if (q < ns) break;
            q -= ns;
        }
        i = dra[L];
        sq = q * per + ((int)threadIdx.x / G) * kSliceA;   // this group's first entry (offset in the row)
    }
    const bool valid = !ctrl_wave && i < n;
    const int ic = valid ? i : 0;
    // every load that needs nothing else goes out first, so that its memory trip overlaps
    // the one of the control words: the control wave's partials (used only when folding),
    // control block and parameters; the row waves' row header
    // (control block and parameters one word per lane: two vector loads, broadcast later)
    double px[kLatQ][10], ccv = 0.0, pvv = 0.0;
    int kb = 0, ke = 0;
    if (ctrl_wave) {
        load_partials<10>(partC, nblkC, px);
        const int l64 = threadIdx.x & 63;
        ccv = ctrl_prev[min(l64, C_NCTRL - 1)];
        pvv = par[min(l64, P_NPAR - 1)];
    } else {
        kb = adj_ptr[ic];
        ke = adj_low[ic];
    }
    __builtin_amdgcn_sched_barrier(0);
    // this iteration's operands: ctrl_step folds the previous stage (and flips the G and R
    // buffers) exactly when `fold` holds
    const double lsflag = ls_prev[LS_FLAG];
    const int fold = (ctrl_prev[C_ACT2] != 0.0 && ctrl_prev[C_PENDING] == 1.0 && lsflag == 0.0) ? 1 : 0;
#ifdef LRS_PHASE_TIMING
    // diagnostics: the row header (a vector load) and the control words (scalar loads) arrived
    if (blockIdx.x == 0 && threadIdx.x == 0 && kb != -12345) g_phase_tmp[0][10] = wall_clock64();
    if (blockIdx.x == 0 && threadIdx.x == 0 && fold != 12345) g_phase_tmp[0][9] = wall_clock64();
    if (blockIdx.x == 0 && ctrl_wave && (threadIdx.x & 63) == 0 && ccv != 12345.678) g_phase_tmp[0][11] = wall_clock64();
#endif
    const bool r1 = (ctrl_prev[C_RCUR] != 0.0) != (fold != 0);
    const bool g1 = (ctrl_prev[C_GCUR] != 0.0) != (fold != 0);
    const double *__restrict__ R = (r1 ? Rb1 : Rb0) + foff;
    const double *__restrict__ Gc = (g1 ? G1 : G0) + foff;
    const double *__restrict__ s0 = s0a + foff, *__restrict__ y0 = y0a + foff;
    const double *__restrict__ s1 = s1a + foff, *__restrict__ y1 = y1a + foff;
    double *__restrict__ D = Dall + foff;
    const long oi = (long)ic * ld + lane * E;
    // row-wave prefetch state: own operands, the NO off-diagonal entries (records and the
    // neighbours' direction operands), the diagonal entry's records
    DirRow<E> own;
    double xi[E];
    int no = 0;
    bool dg = false;
    int jj[NO], ss[NO];
    double cw[NO], bq[NO], cq[NO], lq[NO];
    double2 l1[NO];
    DirRow<E> nbr[NO];
    double xj[NO][E];
    int sd = 0;
    double cwd = 0.0, bd = 0.0, cd = 0.0, lmd = 0.0;
    double2 l1d = make_double2(0.0, -1.0);
    if (ctrl_wave) {
        // ---- control wave: the previous stage's dots, then the control of this iteration;
        // every lane runs ctrl_step on a register copy (uniform values), lane 0 publishes it
        const int l64 = threadIdx.x & 63;
        if (l64 < C_NCTRL) c[l64] = ccv;
        if (l64 < P_NPAR) pl[l64] = pvv;
        double s[10];
        if (fold) {
            sum_partials<10>(px, nblkC, s);
        } else {
#pragma unroll
            for (int v = 0; v < 10; ++v) s[v] = 0.0;
        }
#ifdef LRS_PHASE_TIMING
        if (blockIdx.x == 0 && l64 == 0 && s[9] != 12345.678 && ccv != 12345.678) g_phase_tmp[0][8] = wall_clock64();
#endif
        // (lane 0 on the LDS copy: a register copy of the block, every word read back from
        // its lane, measured 0.5 us slower on G67, scripts/gpu_r04h.sh)
        // the block and the parameters read back from LDS as one batch of loads (constant
        // indices: registers), the step on registers, lane 0 writes the block back (k_lat_a
        // 9.1 -> 8.95 us on G67, profiles/r04u_lat_ab.txt; LRS_NO_CTRL_LREG: on the LDS copy)
        {
            double cr[C_NCTRL], pr[P_NPAR];
#pragma unroll
            for (int q = 0; q < C_NCTRL; ++q) cr[q] = c[q];
#pragma unroll
            for (int q = 0; q < P_NPAR; ++q) pr[q] = pl[q];
            ctrl_step(cr, pr, lsflag, ls_prev[LS_TAU], fold, s, mg == 0);
            if (l64 == 0) {
#pragma unroll
                for (int q = 0; q < C_NCTRL; ++q) c[q] = cr[q];
            }
        }
#ifdef LRS_PHASE_TIMING
        if (blockIdx.x == 0 && l64 == 0) g_phase_tmp[0][7] = wall_clock64();
#endif
    } else {
        // ---- row waves: every load the control does not decide, one memory trip per
        // dependency level; loads clamped to valid addresses instead of branched
        ld_row<E>(Gc + oi, own.g);
        ld_row<E>(s0 + oi, own.a0); ld_row<E>(y0 + oi, own.b0);
        ld_row<E>(s1 + oi, own.a1); ld_row<E>(y1 + oi, own.b1);
        ld_row<E>(R + oi, xi);
        // entries of this group: the row's lower part (a dense row's own group: none), or its
        // slice of a dense row (no diagonal special case there)
        int eb = kb, nl = valid ? ke - kb : 0;
        if (slice) { eb = kb + sq; nl = valid ? max(0, min(kSliceA, ke - eb)) : 0; }
        else if (nl > kDenseRow) nl = 0;
        const int kd = nl > 0 ? eb + nl - 1 : 0;
        const int jd = adj_col[kd];
        sd = adj_slot[kd];
#pragma unroll
        for (int u = 0; u < NO; ++u) {
            const int k = nl > 0 ? eb + min(u, nl - 1) : 0;
            jj[u] = adj_col[k];
            ss[u] = adj_slot[k];
        }
        kb = eb;
        dg = !slice && nl > 0 && jd == i;
        no = nl - (dg ? 1 : 0);
        cwd = Cw[sd];
        l1d = loc1[sd];
#pragma unroll
        for (int u = 0; u < NO; ++u) {
            cw[u] = Cw[ss[u]];
            l1[u] = loc1[ss[u]];
            // entries past `no` read the own row again (cached) instead of another
            const long oj = (long)(u < no ? jj[u] : ic) * ld + lane * E;
            ld_row<E>(R + oj, xj[u]);
            ld_row<E>(Gc + oj, nbr[u].g);
            ld_row<E>(s0 + oj, nbr[u].a0); ld_row<E>(y0 + oj, nbr[u].b0);
            ld_row<E>(s1 + oj, nbr[u].a1); ld_row<E>(y1 + oj, nbr[u].b1);
        }
        // slots without a single local constraint read the row's own (spread, cached) index
        // instead of a common one: no hot line shared by every lane
        const int ispare = min(ic, m - 1);
#pragma unroll
        for (int u = 0; u < NO; ++u) {
            const int ci = (int)l1[u].y >= 0 ? (int)l1[u].y : ispare;
            bq[u] = b[ci];
            cq[u] = cvs[ci];
            lq[u] = lam[ci];
        }
        {
            const int ci = (int)l1d.y >= 0 ? (int)l1d.y : ispare;
            bd = b[ci];
            cd = cvs[ci];
            lmd = lam[ci];
        }
#ifdef LRS_PHASE_TIMING
        if (blockIdx.x == 0 && threadIdx.x == 0 && xi[0] != 12345.678) g_phase_tmp[0][1] = wall_clock64();
        if (blockIdx.x == 0 && threadIdx.x == 0 && bq[0] != 12345.678 && xj[0][0] != 12345.678 && bd != 12345.678)
            g_phase_tmp[0][2] = wall_clock64();
#endif
    }
    __syncthreads();
    LRS_TS(0, 3);
    if (pblk_off == 0 && blockIdx.x == 0 && threadIdx.x < C_NCTRL) ctrl_cur[threadIdx.x] = c[threadIdx.x];
    const bool active = c[C_ACTIVE] != 0.0;
    if (!active && !(fold && mg > 0)) return;
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (fold && do_glob) {
        // global constraints: A(RR^T) from the slots and their residual (as k_it_a)
        if (gwide) {
            const int lane64 = threadIdx.x & 63;
            const int nw = gridDim.x * nwv;
            for (int g = blockIdx.x * nwv + (threadIdx.x >> 6); g < mg; g += nw) {
                const int ig = glob[g];
                double tot = 0.0;
                for (int k = 0; k < K; ++k) {
                    const long row = (long)k * m + ig;
                    double v = 0.0;
                    for (int e = con_ptr[row] + lane64; e < con_ptr[row + 1]; e += 64) v += con_w[e] * uRR[con_slot[e]];
                    tot += wave_sum(v);
                }
                if (lane64 == 0) {
                    cvs[ig] = tot;
                    const double dd = b[ig] - tot;
                    acc[7] += dd * dd;
                }
            }
        } else {
            for (int g = blockIdx.x * nwv * 64 + threadIdx.x; g < mg; g += gridDim.x * nwv * 64) {
                const int ig = glob[g];
                double tot = 0.0;
                for (int k = 0; k < K; ++k) {
                    const long row = (long)k * m + ig;
                    double v = 0.0;
                    for (int e = con_ptr[row]; e < con_ptr[row + 1]; ++e) v += con_w[e] * uRR[con_slot[e]];
                    tot += v;
                }
                cvs[ig] = tot;
                const double dd = b[ig] - tot;
                acc[7] += dd * dd;
            }
        }
    }
    if (active && valid) {
        DirCoef kc;
        kc.cg = c[C_CG]; kc.cs0 = c[C_CS0]; kc.cy0 = c[C_CY0]; kc.cs1 = c[C_CS1]; kc.cy1 = c[C_CY1];
        kc.u0 = (kc.cs0 != 0.0 || kc.cy0 != 0.0);
        kc.u1 = (kc.cs1 != 0.0 || kc.cy1 != 0.0);
        const double rho = par[P_RHO], rhoInv = 1.0 / rho;
        double yi[E];
        own.eval(kc, yi);
        if (!slice) st_row<E>(D + oi, yi);
        // one lower entry (j, slot): sym(R D^T), D D^T, objective parts, local constraints
        auto entry = [&](int j, int sl, const double (&xjv)[E], const double (&yj)[E], double cwv, double2 l1v,
                         double bv, double cv, double lv) {
            double d0 = 0.0, d1 = 0.0;
            if (j != i) {
#pragma unroll
                for (int e = 0; e < E; ++e) d0 += xi[e] * yj[e] + xjv[e] * yi[e];
                d0 *= 0.5;
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e) d0 += xi[e] * yi[e];
            }
#pragma unroll
            for (int e = 0; e < E; ++e) d1 += yi[e] * yj[e];
            d0 = group_sum<G>(d0);
            d1 = group_sum<G>(d1);
            if (lane != 0) return;
            uRD[sl] = d0;
            uDD[sl] = d1;
            acc[0] += cwv * d0;
            acc[1] += cwv * d1;
            // local constraints on this slot (ALMCalq12p12 lorads_alm.c:714-734, dots :269-277)
            const int c1 = (int)l1v.y;
            const int e0 = c1 == -2 ? loc_ptr[sl] : 0, e1 = c1 == -2 ? loc_ptr[sl + 1] : (c1 >= 0 ? 1 : 0);
            for (int e = e0; e < e1; ++e) {
                const int ci = c1 >= 0 ? c1 : loc_con[e];
                const double w = c1 >= 0 ? l1v.x : loc_w[e];
                const double bi = c1 >= 0 ? bv : b[ci], cvi = c1 >= 0 ? cv : cvs[ci], li = c1 >= 0 ? lv : lam[ci];
                const double q1 = 2.0 * (w * d0), q2 = w * d1;
                const double q0 = (bi - cvi) + rhoInv * li;
                acc[2] += q2 * q2; acc[3] += q1 * q2; acc[4] += q0 * q2; acc[5] += q1 * q1;
                acc[6] += q0 * q1;
                double2 *r = reinterpret_cast<double2 *>(rec + 4L * ci);
                r[0] = make_double2(cvi, q1);
                r[1] = make_double2(q2, (-li) + (-rho) * bi);
            }
        };
        // adjacency order: the off-diagonal lower entries, then the diagonal (the last)
#pragma unroll
        for (int u = 0; u < NO; ++u) {
            if (u < no) {
                double yj[E];
                nbr[u].eval(kc, yj);
                entry(jj[u], ss[u], xj[u], yj, cw[u], l1[u], bq[u], cq[u], lq[u]);
            }
        }
        for (int k = kb + NO; k < kb + no; ++k) {
            const int j = adj_col[k], sl = adj_slot[k];
            const long oj = (long)j * ld + lane * E;
            double xjv[E], yj[E];
            ld_row<E>(R + oj, xjv);
            DirRow<E> dj;
            dj.load(kc, Gc, s0, y0, s1, y1, oj);
            dj.eval(kc, yj);
            const double2 l1v = loc1[sl];
            const int ci = (int)l1v.y;
            double bv = 0.0, cv = 0.0, lv = 0.0;
            if (ci >= 0) { bv = b[ci]; cv = cvs[ci]; lv = lam[ci]; }
            entry(j, sl, xjv, yj, Cw[sl], l1v, bv, cv, lv);
        }
        if (dg) entry(i, sd, xi, yi, cwd, l1d, bd, cd, lmd);
    }
    LRS_TS(0, 5);
    write_partials_nw<8>(acc, partA, pblk_off + blockIdx.x, nwv);
    LRS_TS_END(0, 6);
#ifdef LRS_PHASE_TIMING
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int q_ = 7; q_ < 12; ++q_) g_phase[0][q_] = g_phase_tmp[0][q_];
#endif
    LRS_BLK_END(0);
}

// B in the latency regime (k_it_b MODE 0): the control wave reduces A's (and G's)
// partials and solves the line search while the row waves prefetch the row header, the
// first NO off-diagonal entries (records and neighbour rows R_j, D_j) and the diagonal
// entry's records; after the barrier only the tau-dependent arithmetic and the stores run.
template <int G, int E, int NO>
__global__ void __launch_bounds__(kLatNT) k_lat_b(
    int n, int ld, long foff, const int *__restrict__ adj_ptr, const int *__restrict__ adj_low,
    const int *__restrict__ adj_col, const int *__restrict__ adj_slot, double *Rb0, double *Rb1,
    const double *__restrict__ Dall, double *G0, double *G1, double *s0, double *y0, double *s1, double *y1,
    double *__restrict__ uRR, const double *__restrict__ Craw, const int *__restrict__ slot_ptr,
    const int *__restrict__ slot_con, const double *__restrict__ slot_a, const double2 *__restrict__ slot1,
    const double *__restrict__ rec, const int *__restrict__ loc_ptr, const int *__restrict__ loc_con,
    const double *__restrict__ loc_w, const double2 *__restrict__ loc1, const double *__restrict__ b,
    double *__restrict__ cvs, const double *__restrict__ par, const double *__restrict__ ctrl,
    const double *__restrict__ partA, int nblkA, const double *__restrict__ partB, int nblkB,
    double *__restrict__ ls_cur, int L, double *__restrict__ partC, int pblk_off, int m, double *hmirror,
    double seq, int nrb, int lrw, int ndb, const int *__restrict__ drb, double *__restrict__ gl, double *CRb,
    const double *__restrict__ CDb) {
    __shared__ double red[12];
    __shared__ double ls[LS_N];
    __shared__ double pl[P_NPAR];
    __shared__ double gsh[kLatRows * E];   // slice blocks: the lane groups' partial gradients
    LRS_TS(2, 0);
    LRS_BLK_BEGIN();
    mirror_ctrl(ctrl, hmirror, seq);
    // lrw row waves + the control wave (an argument beside nrb, loaded in the first argument batch:
    // blockDim.x would be one more load before the first branch)
    const int nwv = lrw + 1, rpb = lrw * 64 / G;   // waves, rows of this block
    const bool ctrl_wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) == nwv - 1;   // wave-uniform
    const int lane = threadIdx.x & (G - 1);
    // blocks [0, nrb): one row per lane group.  Blocks past nrb: slices of the dense rows --
    // every lane group takes kSliceB consecutive entries of one dense row, the block's partial
    // gradient goes to gl[slice] and k_lat_f finishes the row (its own group skips the entries)
    const bool slice = (int)blockIdx.x >= nrb;
    int i = lat_row_block((int)blockIdx.x, nrb) * rpb + (int)threadIdx.x / G, sq = 0;
    if (slice) {
        const int per = rpb * kSliceB;
        int q = (int)blockIdx.x - nrb, Ld = 0;
        for (; Ld < ndb - 1; ++Ld) {
            const int r = drb[Ld], ns = (adj_ptr[r + 1] - adj_ptr[r] + per - 1) / per;
            if (q < ns) break;
            q -= ns;
        }
        i = drb[Ld];
        sq = q * per + ((int)threadIdx.x / G) * kSliceB;
    }
    const bool valid = !ctrl_wave && i < n;
    const int ic = valid ? i : 0;
    // loads that need nothing else first: the control wave's partials (A's, and G's) and
    // parameters, the row waves' row header
    double pa[kLatQ][7], pb[kLatQ][5], pvv = 0.0;
    int kb = 0, kl = 0, ke = 0;
    if (ctrl_wave) {
        load_partials<7>(partA, nblkA, pa);
        if (nblkB > 0) load_partials<5>(partB, nblkB, pb);
        pvv = par[min((int)(threadIdx.x & 63), P_NPAR - 1)];
    } else {
        kb = adj_ptr[ic];
        kl = adj_low[ic];
        ke = adj_ptr[ic + 1];
    }
    __builtin_amdgcn_sched_barrier(0);
    if (ctrl[C_ACT2] == 0.0) return;
    const int gcur = (int)ctrl[C_GCUR], h = (int)ctrl[C_HEAD];
    const bool r1 = ctrl[C_RCUR] != 0.0;
    const double *__restrict__ R = (r1 ? Rb1 : Rb0) + foff;
    double *__restrict__ Rn = (r1 ? Rb0 : Rb1) + foff;
    const double *__restrict__ D = Dall + foff;
    double *__restrict__ Gold = (gcur == 0 ? G0 : G1) + foff;
    double *__restrict__ Gnew = (gcur == 0 ? G1 : G0) + foff;
    double *__restrict__ sh = (h == 0 ? s0 : s1) + foff;
    double *__restrict__ yh = (h == 0 ? y0 : y1) + foff;
    const double *__restrict__ so = (h == 0 ? s1 : s0) + foff;
    const double *__restrict__ yo = (h == 0 ? y1 : y0) + foff;
    const bool two = (L == 2);
    const long oi = (long)ic * ld + lane * E;
    // row-wave prefetch state
    int no = 0;
    bool dg = false, dense = false;
    double ri[E], di[E], go[E], sov[E], yov[E];
    int ss[NO];
    bool lw[NO];
    double rjp[NO][E], djp[NO][E];
    double sv[NO], bq[NO];
    double2 s1v[NO], l1v[NO], ra[NO], rb[NO];
    int sd = 0;
    double svd = 0.0, bqd = 0.0;
    double2 s1d = make_double2(0.0, -1.0), l1d = s1d, rad = make_double2(0.0, 0.0), rbd = rad;
    const double *__restrict__ RA = R;
    if (ctrl_wave) {
        // ---- control wave: line search (ALMLineSearch lorads_alm.c:266-333)
        double sA[7];
        sum_partials<7>(pa, nblkA, sA);
        if (nblkB > 0) {
            double sB[5];
            sum_partials<5>(pb, nblkB, sB);
#pragma unroll
            for (int q = 0; q < 5; ++q) sA[2 + q] += sB[q];
        }
        if ((threadIdx.x & 63) == 0) {
#pragma unroll
            for (int v = 0; v < 7; ++v) red[v] = sA[v];
        }
        __builtin_amdgcn_wave_barrier();
#ifdef LRS_PHASE_TIMING
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && sA[6] != 12345.678) g_phase_tmp[2][8] = wall_clock64();
#endif
        // (sums and parameters through LDS: on register operands, every parameter read back
        // from its lane, the launch measured 0.4 us slower on G67, scripts/gpu_r04k.sh)
        if ((threadIdx.x & 63) < P_NPAR) pl[threadIdx.x & 63] = pvv;
        __builtin_amdgcn_wave_barrier();
        line_search_t<true>(pl, red[0], red[1], red + 2, ls);
#ifdef LRS_PHASE_TIMING
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) g_phase_tmp[2][7] = wall_clock64();
#endif
    } else {
        // ---- row waves: prefetch, one memory trip per dependency level, clamped loads
        ld_row<E>(R + oi, ri);
        ld_row<E>(D + oi, di);
        ld_row<E>(Gold + oi, go);
        if (two) { ld_row<E>(so + oi, sov); ld_row<E>(yo + oi, yov); }
        // entries of this group: the row's adjacency (a dense row's own group: none, it only
        // updates R), or its slice of a dense row (no diagonal special case there)
        int eb = kb, nt = valid ? ke - kb : 0;
        if (slice) { eb = kb + sq; nt = valid ? max(0, min(kSliceB, ke - eb)) : 0; }
        else if (nt > kDenseRow) { nt = 0; dense = true; }
        // the diagonal is the last lower entry (columns ascending); positions of the first
        // NO + 1 entries, the off-diagonal ones picked after the diagonal test
        const int kd = (!slice && nt > 0 && kl > kb) ? kl - 1 : 0;
        const int jd = adj_col[kd];
        sd = adj_slot[kd];
        int ja[NO + 1], sa[NO + 1];
#pragma unroll
        for (int u = 0; u <= NO; ++u) {
            const int k = nt > 0 ? eb + min(u, nt - 1) : 0;
            ja[u] = adj_col[k];
            sa[u] = adj_slot[k];
        }
        dg = !slice && nt > 0 && kl > kb && jd == i;
        no = nt - (dg ? 1 : 0);
        const int pd = dg ? kl - 1 - kb : NO + 1;    // the diagonal's position among the first
#pragma unroll
        for (int u = 0; u < NO; ++u) {
            const bool past = u >= pd;
            const int j = past ? ja[u + 1] : ja[u];
            ss[u] = past ? sa[u + 1] : sa[u];
            lw[u] = eb + u + (past ? 1 : 0) < kl;
            const long oj = (long)(u < no ? j : ic) * ld + lane * E;
            ld_row<E>(RA + oj, rjp[u]);
            ld_row<E>(D + oj, djp[u]);
            sv[u] = Craw[ss[u]];
            s1v[u] = slot1[ss[u]];
            l1v[u] = loc1[ss[u]];
        }
        svd = Craw[sd];
        s1d = slot1[sd];
        l1d = loc1[sd];
        // slots without a single constraint read the row's own (spread, cached) index instead
        // of a common one: no hot line shared by every lane
        const int ispare = min(ic, m - 1);
#pragma unroll
        for (int u = 0; u < NO; ++u) {
            const int c1 = (int)s1v[u].y >= 0 ? (int)s1v[u].y : ispare;
            const int cl = (int)l1v[u].y >= 0 ? (int)l1v[u].y : ispare;
            const double2 *r = reinterpret_cast<const double2 *>(rec + 4L * c1);
            ra[u] = r[0];
            rb[u] = r[1];
            bq[u] = b[cl];
        }
        {
            const int c1 = (int)s1d.y >= 0 ? (int)s1d.y : ispare;
            const int cl = (int)l1d.y >= 0 ? (int)l1d.y : ispare;
            const double2 *r = reinterpret_cast<const double2 *>(rec + 4L * c1);
            rad = r[0];
            rbd = r[1];
            bqd = b[cl];
        }
#ifdef LRS_PHASE_TIMING
        if (blockIdx.x == 0 && threadIdx.x == 0 && ri[0] != 12345.678 && sv[0] != 12345.678)
            g_phase_tmp[2][5] = wall_clock64();
        if (blockIdx.x == 0 && threadIdx.x == 0 && bq[0] != 12345.678 && ra[0].x != 12345.678 && rjp[0][0] != 12345.678)
            g_phase_tmp[2][6] = wall_clock64();
#endif
    }
    __syncthreads();
    LRS_TS(2, 2);
    if (pblk_off == 0 && blockIdx.x == 0 && threadIdx.x < LS_N) ls_cur[threadIdx.x] = ls[threadIdx.x];
    if (ls[LS_FLAG] != 0.0) return;
    const double tau = ls[LS_TAU], tau2 = tau * tau, rho = par[P_RHO];
    double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    double g[E];
#pragma unroll
    for (int e = 0; e < E; ++e) g[e] = 0.0;
    if (valid) {
#pragma unroll
        for (int e = 0; e < E; ++e) ri[e] += tau * di[e];
        if (!slice) st_row<E>(Rn + oi, ri);
        // one entry (j, slot) with R_new,j: S_ij = C + A^*(M1) (ALMSetGrad lorads_alm.c:38-57),
        // the gradient, and on lower slots A(R_new R_new^T) with the local constraints
        auto entry = [&](int sl, bool lower, const double (&rj)[E], double svv, double2 s1u, double2 ra_, double2 rb_,
                         double2 l1u, double bv) {
            const int c1 = (int)s1u.y;
            const int e0 = c1 == -2 ? slot_ptr[sl] : 0;
            const int e1 = c1 == -2 ? slot_ptr[sl + 1] : (c1 >= 0 ? 1 : 0);
            for (int e = e0; e < e1; ++e) {
                double2 x = ra_, y = rb_;
                if (c1 < 0) {
                    const double2 *r = reinterpret_cast<const double2 *>(rec + 4L * slot_con[e]);
                    x = r[0];
                    y = r[1];
                }
                double cv = x.x + tau * x.y;
                cv = cv + tau2 * y.x;
                const double M1 = y.y + rho * cv;
                svv += M1 * (c1 >= 0 ? s1u.x : slot_a[e]);
            }
#pragma unroll
            for (int e = 0; e < E; ++e) g[e] += svv * rj[e];
            if (!lower) return;
            double d = 0.0;
#pragma unroll
            for (int e = 0; e < E; ++e) d += ri[e] * rj[e];
            d = group_sum<G>(d);
            if (lane != 0) return;
            uRR[sl] = d;
            const int cl = (int)l1u.y;
            const int f0 = cl == -2 ? loc_ptr[sl] : 0;
            const int f1 = cl == -2 ? loc_ptr[sl + 1] : (cl >= 0 ? 1 : 0);
            for (int e = f0; e < f1; ++e) {
                const int ci = cl >= 0 ? cl : loc_con[e];
                const double tot = (cl >= 0 ? l1u.x : loc_w[e]) * d;
                cvs[ci] = tot;
                const double dd = (cl >= 0 ? bv : b[ci]) - tot;
                acc[9] += dd * dd;
            }
        };
        // the off-diagonal entries in adjacency order (prefetched, then the rest), the diagonal last
#pragma unroll
        for (int u = 0; u < NO; ++u) {
            if (u < no) {
                double rj[E];
#pragma unroll
                for (int e = 0; e < E; ++e) rj[e] = rjp[u][e] + tau * djp[u][e];
                entry(ss[u], lw[u], rj, sv[u], s1v[u], ra[u], rb[u], l1v[u], bq[u]);
            }
        }
        if (!slice && no > NO) {
            int cnt = 0;
            for (int k = kb; k < ke; ++k) {
                if (dg && k == kl - 1) continue;
                if (cnt++ < NO) continue;
                const int j = adj_col[k], sl = adj_slot[k];
                const long oj = (long)j * ld + lane * E;
                double rj[E], dj[E];
                ld_row<E>(R + oj, rj);
                ld_row<E>(D + oj, dj);
#pragma unroll
                for (int e = 0; e < E; ++e) rj[e] += tau * dj[e];
                const double2 s1u = slot1[sl];
                const int c1 = (int)s1u.y;
                double2 x = make_double2(0.0, 0.0), y = x;
                if (c1 >= 0) {
                    const double2 *r = reinterpret_cast<const double2 *>(rec + 4L * c1);
                    x = r[0];
                    y = r[1];
                }
                const bool lower = k < kl;
                const double2 l1u = lower ? loc1[sl] : make_double2(0.0, -1.0);
                const int cl = (int)l1u.y;
                entry(sl, lower, rj, Craw[sl], s1u, x, y, l1u, cl >= 0 ? b[cl] : 0.0);
            }
        }
        if (dg) entry(sd, true, ri, svd, s1d, rad, rbd, l1d, bqd);
        if (!slice && !dense) {
            // gradient G_new = 2 S R_new, L-BFGS pair s = tau D, y = G_new - G_old, dots
            double sv2[E], yv[E];
            if (CRb) {
                // dense objective: C R_new = C R + tau C D (carried), S R_new += C R_new (as k_it_b)
                double cr[E], cd[E];
                ld_row<E>(CRb + foff + oi, cr);
                ld_row<E>(CDb + foff + oi, cd);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    cr[e] += tau * cd[e];
                    g[e] += cr[e];
                }
                st_row<E>(CRb + foff + oi, cr);
            }
#pragma unroll
            for (int e = 0; e < E; ++e) g[e] *= 2.0;
#pragma unroll
            for (int e = 0; e < E; ++e) { sv2[e] = tau * di[e]; yv[e] = g[e] - go[e]; }
            st_row<E>(Gnew + oi, g);
            st_row<E>(sh + oi, sv2);
            st_row<E>(yh + oi, yv);
#pragma unroll
            for (int e = 0; e < E; ++e) {
                acc[0] += g[e] * g[e];
                acc[1] += yv[e] * sv2[e];
                acc[2] += yv[e] * yv[e];
                acc[3] += sv2[e] * g[e];
                acc[4] += yv[e] * g[e];
            }
            if (two) {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    acc[5] += sov[e] * g[e];
                    acc[6] += yov[e] * g[e];
                    acc[7] += sov[e] * yv[e];
                    acc[8] += yov[e] * yv[e];
                }
            }
        }
    }
    if (slice) {
        // the block's partial gradient of its dense row: groups summed in group order
        if (!ctrl_wave) {
#pragma unroll
            for (int e = 0; e < E; ++e) gsh[threadIdx.x * E + e] = g[e];
        }
        __syncthreads();
        if ((int)threadIdx.x < G * E) {
            const int ln = threadIdx.x / E, e = threadIdx.x % E;
            double t = 0.0;
            for (int q = 0; q < rpb; ++q) t += gsh[(q * G + ln) * E + e];
            gl[(long)((int)blockIdx.x - nrb) * ld + threadIdx.x] = t;
        }
    }
    LRS_TS(2, 3);
    write_partials_nw<10>(acc, partC, pblk_off + blockIdx.x, nwv);
    LRS_TS_END(2, 4);
#ifdef LRS_PHASE_TIMING
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int q_ = 5; q_ < 12; ++q_) g_phase[2][q_] = g_phase_tmp[2][q_];
#endif
    LRS_BLK_END(2);
}

// Dense rows of stage B after the slice blocks: one block per row sums the row's slice
// gradients (slice order), then the epilogue of k_lat_b (gradient G_new = 2 S R_new, the
// L-BFGS pair, the dots); the block's partials go to slot pblk_off + blockIdx.x.
__global__ void __launch_bounds__(kRowBlock) k_lat_f(
    int ld, int w, long foff, const int *__restrict__ adj_ptr, const int *__restrict__ drb, int per,
    const double *__restrict__ gl, const double *__restrict__ Dall, double *G0, double *G1, double *s0, double *y0,
    double *s1, double *y1, const double *__restrict__ ctrl, const double *__restrict__ ls_cur, int L,
    double *__restrict__ partC, int pblk_off, double *CRb, const double *__restrict__ CDb) {
    if (ctrl[C_ACT2] == 0.0 || ls_cur[LS_FLAG] != 0.0) return;
    const int gcur = (int)ctrl[C_GCUR], h = (int)ctrl[C_HEAD];
    const double *__restrict__ D = Dall + foff;
    const double *__restrict__ Gold = (gcur == 0 ? G0 : G1) + foff;
    double *__restrict__ Gnew = (gcur == 0 ? G1 : G0) + foff;
    double *__restrict__ sh = (h == 0 ? s0 : s1) + foff;
    double *__restrict__ yh = (h == 0 ? y0 : y1) + foff;
    const double *__restrict__ so = (h == 0 ? s1 : s0) + foff;
    const double *__restrict__ yo = (h == 0 ? y1 : y0) + foff;
    const double tau = ls_cur[LS_TAU];
    int sl0 = 0;
    for (int q = 0; q < (int)blockIdx.x; ++q) {
        const int r = drb[q];
        sl0 += (adj_ptr[r + 1] - adj_ptr[r] + per - 1) / per;
    }
    const int i = drb[blockIdx.x], ns = (adj_ptr[i + 1] - adj_ptr[i] + per - 1) / per;
    double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const int t = threadIdx.x;
    if (t < w) {
        const long oi = (long)i * ld + t;
        double g = 0.0;
        for (int q = 0; q < ns; ++q) g += gl[(long)(sl0 + q) * ld + t];
        if (CRb) {   // dense objective (as k_lat_b)
            const double cr = CRb[foff + oi] + tau * CDb[foff + oi];
            CRb[foff + oi] = cr;
            g += cr;
        }
        g *= 2.0;
        const double sv2 = tau * D[oi], yv = g - Gold[oi];
        Gnew[oi] = g;
        sh[oi] = sv2;
        yh[oi] = yv;
        acc[0] = g * g;
        acc[1] = yv * sv2;
        acc[2] = yv * yv;
        acc[3] = sv2 * g;
        acc[4] = yv * g;
        if (L == 2) {
            const double sov = so[oi], yov = yo[oi];
            acc[5] = sov * g;
            acc[6] = yov * g;
            acc[7] = sov * yv;
            acc[8] = yov * yv;
        }
    }
    write_partials<10, kRowBlock>(acc, partC, pblk_off + blockIdx.x);
}

// ------------------------------------------------------------------------
// Bandwidth regime, long rows (a random sparse SDP has ~10^3 pattern entries per row): the
// neighbour halves of stages A and B (k_it_a / k_it_b MODE 2) with the per-entry metadata
// fetched lane-parallel -- a lane group takes G entries of its row at a time and every lane
// gathers one entry's column, slot and records (three memory trips for G entries instead
// of three per entry) -- then the entries' factor rows U at a time, the column broadcast
// from the lane that fetched it, which also stores the entry's results.
// ------------------------------------------------------------------------

// Column tiles (TL): the random long-row pattern (C5) reads ~10^3 neighbour rows per row from
// anywhere in the factor, and a 10 MB factor does not fit one XCD's 4 MB L2, so nearly every
// gather missed to the Infinity Cache (~12 GB per launch).  TL splits every row's entries by
// column block x = 0..7 (colseg: the row's first entry at or past column x n / 8) and gives
// column block x to the blocks of group b % 8 (one XCD under the round-robin dispatch; speed
// only): an XCD then reads neighbour rows from one n / 8 range of the factor -- 1.25 MB per
// operand at C5 -- through its own L2, and each row's own operands once per group.  Every
// entry is still visited once; B's per-row gradient becomes eight column-block partials
// (GP), summed in block order by k_wide_bf with the row epilogue.
__device__ __forceinline__ void tile_rows(bool tl, int &grp, int &ngrp, int &xg, int G) {
    if (tl) {
        xg = blockIdx.x & (kNX - 1);
        const int bq = blockIdx.x / kNX, nbq = ((int)gridDim.x - xg + kNX - 1) / kNX;
        grp = (bq * kRowBlock + (int)threadIdx.x) / G;
        ngrp = nbq * kRowBlock / G;
    } else {
        xg = 0;
        grp = (blockIdx.x * kRowBlock + (int)threadIdx.x) / G;
        ngrp = gridDim.x * kRowBlock / G;
    }
}

// A, second half (SDDMM sym(RD^T), DD^T on the lower slots, local constraints' q1/q2 and
// dots), D read back; partials 0..6 as k_it_a MODE 2
template <int G, int E, int U, bool TL>
__global__ void __launch_bounds__(kRowBlock) k_wide_a(
    int n, int ld, long foff, const int *__restrict__ adj_ptr, const int *__restrict__ adj_low,
    const int *__restrict__ adj_col, const int *__restrict__ adj_slot, const double *__restrict__ Cw,
    const double *__restrict__ Rb0, const double *__restrict__ Rb1, const double *__restrict__ Dall,
    double *__restrict__ uRD, double *__restrict__ uDD, const int *__restrict__ loc_ptr,
    const int *__restrict__ loc_con, const double *__restrict__ loc_w, const double2 *__restrict__ loc1,
    const double *__restrict__ b, const double *__restrict__ cvs, const double *__restrict__ lam,
    double *__restrict__ rec, const double *__restrict__ par, const double *__restrict__ ctrl_cur,
    double *__restrict__ partA, int pblk_off, int row0, int m, const int *__restrict__ colseg) {
    if (ctrl_cur[C_ACTIVE] == 0.0) return;
    const double *__restrict__ R = (ctrl_cur[C_RCUR] == 0.0 ? Rb0 : Rb1) + foff;
    const double *__restrict__ D = Dall + foff;
    const double rho = par[P_RHO], rhoInv = 1.0 / rho;
    const int lane = threadIdx.x & (G - 1);
    int grp, ngrp, xg;
    tile_rows(TL, grp, ngrp, xg, G);
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = row0 + grp; i < row0 + n; i += ngrp) {
        int kb = adj_ptr[i], ke = adj_low[i];
        if constexpr (TL) {
            kb = max(kb, colseg[(long)i * (kNX + 1) + xg]);
            ke = min(ke, colseg[(long)i * (kNX + 1) + xg + 1]);
            if (kb >= ke) continue;   // lane-group uniform
        }
        const long oi = (long)i * ld + lane * E;
        double xi[E], yi[E];
        ld_row<E>(R + oi, xi);
        ld_row<E>(D + oi, yi);
        const int ispare = min(i, m - 1);
        for (int c0 = kb; c0 < ke; c0 += G) {
            // this lane's entry of the chunk: column, slot, records
            const int kc = c0 + lane < ke ? c0 + lane : c0;
            const int jl = adj_col[kc], sl = adj_slot[kc];
            const double cwl = Cw[sl];
            const double2 l1l = loc1[sl];
            const int cil = (int)l1l.y >= 0 ? (int)l1l.y : ispare;
            const double bl = b[cil], cvl = cvs[cil], lml = lam[cil];
            const int nc = min(G, ke - c0);
            for (int u0 = 0; u0 < nc; u0 += U) {
                double xj[U][E], yj[U][E];
#pragma unroll
                for (int v = 0; v < U; ++v) {
                    const int j = bcast_i<G>(jl, min(u0 + v, nc - 1));
                    const long oj = (long)j * ld + lane * E;
                    ld_row<E>(R + oj, xj[v]);
                    ld_row<E>(D + oj, yj[v]);
                }
#pragma unroll
                for (int v = 0; v < U; ++v) {
                    const int u = u0 + v;
                    if (u >= nc) break;
                    const int j = bcast_i<G>(jl, u);
                    double d0 = 0.0, d1 = 0.0;
                    if (j != i) {
#pragma unroll
                        for (int e = 0; e < E; ++e) d0 += xi[e] * yj[v][e] + xj[v][e] * yi[e];
                        d0 *= 0.5;
                    } else {
#pragma unroll
                        for (int e = 0; e < E; ++e) d0 += xi[e] * yi[e];
                    }
#pragma unroll
                    for (int e = 0; e < E; ++e) d1 += yi[e] * yj[v][e];
                    d0 = group_sum<G>(d0);
                    d1 = group_sum<G>(d1);
                    if (lane == u) {
                        uRD[sl] = d0;
                        uDD[sl] = d1;
                        acc[0] += cwl * d0;
                        acc[1] += cwl * d1;
                        // local constraints on this slot (ALMCalq12p12 lorads_alm.c:714-734)
                        const int c1 = (int)l1l.y;
                        const int e0 = c1 == -2 ? loc_ptr[sl] : 0, e1 = c1 == -2 ? loc_ptr[sl + 1] : (c1 >= 0 ? 1 : 0);
                        for (int e = e0; e < e1; ++e) {
                            const int ci = c1 >= 0 ? c1 : loc_con[e];
                            const double w = c1 >= 0 ? l1l.x : loc_w[e];
                            const double bi = c1 >= 0 ? bl : b[ci], cvi = c1 >= 0 ? cvl : cvs[ci];
                            const double li = c1 >= 0 ? lml : lam[ci];
                            const double q1 = 2.0 * (w * d0), q2 = w * d1;
                            const double q0 = (bi - cvi) + rhoInv * li;
                            acc[2] += q2 * q2; acc[3] += q1 * q2; acc[4] += q0 * q2; acc[5] += q1 * q1;
                            acc[6] += q0 * q1;
                            double2 *r = reinterpret_cast<double2 *>(rec + 4L * ci);
                            r[0] = make_double2(cvi, q1);
                            r[1] = make_double2(q2, (-li) + (-rho) * bi);
                        }
                    }
                }
            }
        }
    }
    write_partials_range<8, kRowBlock>(acc, partA, pblk_off + blockIdx.x, 0, 7);
}

// k_wide_a's work over 2-D tiles of the lower pattern (cones with DevCone::sa_items, e.g. C5's
// ~570 lower slots per row): per (row tile I, column tile J) of kAuvT rows each, R and D of both
// tiles are staged in LDS kAuvC columns at a time and each thread evaluates its slots'
// sym(R D^T) and D D^T from there (auv_chunk<2>), instead of every lane group gathering ~570
// neighbour rows of R and D per row; the per-slot epilogue (slot values, C and local-constraint
// terms, rec) is k_wide_a's.  Work: the tile pairs' slots cut into sub-items of kTileSub (one
// slot a thread), in groups of at most kTileGrp sub-items of one row tile (the I side staged once
// per column chunk for the group, each new J side after it); the resident blocks (nwork) stride
// over the groups in order, so the groups in flight are neighbours and share their tiles in L2;
// the blocks past nwork write zero partials (same grid and partial slots as k_wide_a).  Staging,
// not the LDS reads, bounds it (C5, profiles/r05q_c5_tile_a_ab.txt: 0.27 ms of the 0.47 ms stage
// the tiles, 0.15 ms sum them), and the staging rounds' latency more than their bytes: groups of
// 4 / 6 / 8 sub-items (a third to a half fewer staged bytes) measured no faster (616 / 640 / 665
// against 610 us for stage A), register prefetch of the next round at 512 threads slower (806).
__device__ __forceinline__ void tile_side_fetch(double2 (&v)[2][auv_per<1024>()], int row0, int c0, int n, int r,
                                                int ld, const double *__restrict__ X, const double *__restrict__ Y) {
#pragma unroll
    for (int k = 0; k < auv_per<1024>(); ++k) {
        const int x = threadIdx.x + k * 1024;
        const int row = row0 + x / (kAuvC / 2), col = c0 + 2 * (x % (kAuvC / 2));
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            double2 t = make_double2(0.0, 0.0);
            if (row < n && col < r) {
                t = *reinterpret_cast<const double2 *>((a == 0 ? X : Y) + (long)row * ld + col);
                if (col + 1 >= r) t.y = 0.0;
            }
            v[a][k] = t;
        }
    }
}
__device__ __forceinline__ void tile_side_put(double (*tl)[kAuvT * kAuvS], int side,
                                              const double2 (&v)[2][auv_per<1024>()]) {
#pragma unroll
    for (int k = 0; k < auv_per<1024>(); ++k) {
        const int x = threadIdx.x + k * 1024;
        const int o = (x / (kAuvC / 2)) * kAuvS + 2 * (x % (kAuvC / 2));
        *reinterpret_cast<double2 *>(&tl[side][o]) = v[0][k];       // X side: tl[0] (I) / tl[1] (J)
        *reinterpret_cast<double2 *>(&tl[side + 2][o]) = v[1][k];   // Y side: tl[2] / tl[3]
    }
}
__global__ void __launch_bounds__(1024) k_tile_a(
    int n, int r, int ld, long foff, int ngrp, const int *__restrict__ grp, int nwork, const int4 *__restrict__ subs,
    const unsigned *__restrict__ pq, const int *__restrict__ tslot, const double *__restrict__ Cw,
    const double *__restrict__ Rb0, const double *__restrict__ Rb1, const double *__restrict__ Dall,
    double *__restrict__ uRD, double *__restrict__ uDD, const int *__restrict__ loc_ptr,
    const int *__restrict__ loc_con, const double *__restrict__ loc_w, const double2 *__restrict__ loc1,
    const double *__restrict__ b, const double *__restrict__ cvs, const double *__restrict__ lam,
    double *__restrict__ rec, const double *__restrict__ par, const double *__restrict__ ctrl_cur,
    double *__restrict__ partA, int pblk_off, double2 *__restrict__ uvp) {
    constexpr int NT = 1024, KM = kTileGrp;
    static_assert(kTileSub == NT, "k_tile_a: one slot of a sub-item a thread");
    if (ctrl_cur[C_ACTIVE] == 0.0) return;
    const double *__restrict__ R = (ctrl_cur[C_RCUR] == 0.0 ? Rb0 : Rb1) + foff;
    const double *__restrict__ D = Dall + foff;
    const double rho = par[P_RHO], rhoInv = 1.0 / rho;
    __shared__ double tl[4][kAuvT * kAuvS];
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int g = blockIdx.x; g < ngrp && (int)blockIdx.x < nwork; g += nwork) {   // block-uniform
        {
            const int g0 = grp[g], g1 = grp[g + 1];
            const int I0 = subs[g0].x;
            int pl[KM], ql[KM];
            double s0[KM], s1[KM];
#pragma unroll
            for (int j = 0; j < KM; ++j) {
                const int4 it = g0 + j < g1 ? subs[g0 + j] : make_int4(0, 0, 0, 0);
                const int t = it.z + (int)threadIdx.x;
                const unsigned w = t < it.w ? pq[t] : 0u;
                pl[j] = (int)(w >> 16) * kAuvS;
                ql[j] = (int)(w & 0xffffu) * kAuvS;
                s0[j] = 0.0;
                s1[j] = 0.0;
            }
            for (int c0 = 0; c0 < r; c0 += kAuvC) {
                int Jprev = -1;
#pragma unroll
                for (int j = 0; j < KM; ++j) {
                    if (g0 + j >= g1) break;
                    const int4 it = subs[g0 + j];
                    if (it.y != Jprev) {   // a new column tile (and, first, the row tile's chunk)
                        double2 vj[2][auv_per<1024>()];
                        tile_side_fetch(vj, it.y, c0, n, r, ld, R, D);
                        if (j == 0) {
                            double2 vi[2][auv_per<1024>()];
                            tile_side_fetch(vi, I0, c0, n, r, ld, R, D);
                            __syncthreads();
                            tile_side_put(tl, 0, vi);
                        } else {
                            __syncthreads();
                        }
                        tile_side_put(tl, 1, vj);
                        __syncthreads();
                        Jprev = it.y;
                    }
                    if (it.z + (int)threadIdx.x < it.w) auv_chunk<2>(tl, pl[j], ql[j], s0[j], s1[j]);
                }
            }
#pragma unroll
            for (int j = 0; j < KM; ++j) {
                if (g0 + j >= g1) break;
                const int4 it = subs[g0 + j];
                const int t = it.z + (int)threadIdx.x;
                if (t >= it.w) continue;
                const int sl = tslot[t];
                const double d0 = 0.5 * s0[j], d1 = s1[j];
                if (uvp) {
                    uvp[sl] = make_double2(d0, d1);
                } else {
                    uRD[sl] = d0;
                    uDD[sl] = d1;
                }
                const double cwl = Cw[sl];
                acc[0] += cwl * d0;
                acc[1] += cwl * d1;
                // local constraints on this slot (ALMCalq12p12 lorads_alm.c:714-734), as k_wide_a
                const double2 l1l = loc1[sl];
                const int c1 = (int)l1l.y;
                const int e0 = c1 == -2 ? loc_ptr[sl] : 0, e1 = c1 == -2 ? loc_ptr[sl + 1] : (c1 >= 0 ? 1 : 0);
                for (int e = e0; e < e1; ++e) {
                    const int ci = c1 >= 0 ? c1 : loc_con[e];
                    const double w = c1 >= 0 ? l1l.x : loc_w[e];
                    const double bi = b[ci], cvi = cvs[ci], li = lam[ci];
                    const double q1 = 2.0 * (w * d0), q2 = w * d1;
                    const double q0 = (bi - cvi) + rhoInv * li;
                    acc[2] += q2 * q2; acc[3] += q1 * q2; acc[4] += q0 * q2; acc[5] += q1 * q1;
                    acc[6] += q0 * q1;
                    double2 *rr = reinterpret_cast<double2 *>(rec + 4L * ci);
                    rr[0] = make_double2(cvi, q1);
                    rr[1] = make_double2(q2, (-li) + (-rho) * bi);
                }
            }
        }
    }
    write_partials_range<8, NT>(acc, partA, pblk_off + blockIdx.x, 0, 7);
}

// row epilogue of stage B: G_new = 2 (S R_new [+ C R_new]), s = tau D, y = G_new - G_old
// (setlbfgsHisTwo lorads_alm.c:842-863) and the nine L-BFGS dots
template <int E>
__device__ __forceinline__ void wide_b_epilogue(double (&g)[E], long oi, long foff, double tau, const double *D,
                                                const double *Gold, double *Gnew, double *sh, double *yh,
                                                const double *so, const double *yo, bool two, double *CRb,
                                                const double *CDb, double (&acc)[10]) {
    double di[E], go[E], sv2[E], yv[E];
    ld_row<E>(D + oi, di);
    ld_row<E>(Gold + oi, go);
    if (CRb) {
        // dense objective: C R_new = C R + tau C D (carried), S R_new += C R_new (as k_it_b)
        double cr[E], cd[E];
        ld_row<E>(CRb + foff + oi, cr);
        ld_row<E>(CDb + foff + oi, cd);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            cr[e] += tau * cd[e];
            g[e] += cr[e];
        }
        st_row<E>(CRb + foff + oi, cr);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) g[e] *= 2.0;
#pragma unroll
    for (int e = 0; e < E; ++e) { sv2[e] = tau * di[e]; yv[e] = g[e] - go[e]; }
    st_row<E>(Gnew + oi, g);
    st_row<E>(sh + oi, sv2);
    st_row<E>(yh + oi, yv);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        acc[0] += g[e] * g[e];
        acc[1] += yv[e] * sv2[e];
        acc[2] += yv[e] * yv[e];
        acc[3] += sv2[e] * g[e];
        acc[4] += yv[e] * g[e];
    }
    if (two) {
        double sov[E], yov[E];
        ld_row<E>(so + oi, sov);
        ld_row<E>(yo + oi, yov);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            acc[5] += sov[e] * g[e];
            acc[6] += yov[e] * g[e];
            acc[7] += sov[e] * yv[e];
            acc[8] += yov[e] * yv[e];
        }
    }
}

// B, second half (adjoint S = C + A^*(M1), G = 2 S R_new, A(R_new R_new^T) on the lower
// slots, L-BFGS pair, nine dots + residual) over the updated factor; as k_it_b MODE 2.
// TL: the row's entries of column block b % 8 only; the partial S R_new row goes to
// GP[x] and k_wide_bf runs the epilogue (partials: the residual only here).
template <int G, int E, int U, bool TL>
__global__ void __launch_bounds__(kRowBlock) k_wide_b(
    int n, int ld, long foff, const int *__restrict__ adj_ptr, const int *__restrict__ adj_low,
    const int *__restrict__ adj_col, const int *__restrict__ adj_slot, const double *Rb0, const double *Rb1,
    const double *__restrict__ Dall, double *G0, double *G1, double *s0, double *y0, double *s1, double *y1,
    double *__restrict__ uRR, const double *__restrict__ Craw, const int *__restrict__ slot_ptr,
    const int *__restrict__ slot_con, const double *__restrict__ slot_a, const double2 *__restrict__ slot1,
    const double *__restrict__ rec, const int *__restrict__ loc_ptr, const int *__restrict__ loc_con,
    const double *__restrict__ loc_w, const double2 *__restrict__ loc1, const double *__restrict__ b,
    double *__restrict__ cvs, const double *__restrict__ par, const double *__restrict__ ctrl,
    const double *__restrict__ ls_cur, int L, double *__restrict__ partC, int pblk_off, int row0, int m, double *CRb,
    const double *__restrict__ CDb, const int *__restrict__ colseg, double *__restrict__ GP, long gstride) {
    if (ctrl[C_ACT2] == 0.0 || ls_cur[LS_FLAG] != 0.0) return;
    const double tau = ls_cur[LS_TAU], tau2 = tau * tau, rho = par[P_RHO];
    const int gcur = (int)ctrl[C_GCUR], h = (int)ctrl[C_HEAD];
    const double *__restrict__ Rn = (ctrl[C_RCUR] == 0.0 ? Rb1 : Rb0) + foff;
    const double *__restrict__ D = Dall + foff;
    const double *__restrict__ Gold = (gcur == 0 ? G0 : G1) + foff;
    double *__restrict__ Gnew = (gcur == 0 ? G1 : G0) + foff;
    double *__restrict__ sh = (h == 0 ? s0 : s1) + foff;
    double *__restrict__ yh = (h == 0 ? y0 : y1) + foff;
    const double *__restrict__ so = (h == 0 ? s1 : s0) + foff;
    const double *__restrict__ yo = (h == 0 ? y1 : y0) + foff;
    const bool two = (L == 2);
    const int lane = threadIdx.x & (G - 1);
    int grp, ngrp, xg;
    tile_rows(TL, grp, ngrp, xg, G);
    double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = row0 + grp; i < row0 + n; i += ngrp) {
        const long oi = (long)i * ld + lane * E;
        double ri[E], g[E];
        ld_row<E>(Rn + oi, ri);
#pragma unroll
        for (int e = 0; e < E; ++e) g[e] = 0.0;
        int kb = adj_ptr[i], ke = adj_ptr[i + 1];
        const int kl = adj_low[i];
        if constexpr (TL) {
            kb = colseg[(long)i * (kNX + 1) + xg];
            ke = colseg[(long)i * (kNX + 1) + xg + 1];
        }
        const int ispare = min(i, m - 1);
        for (int c0 = kb; c0 < ke; c0 += G) {
            // this lane's entry: column, slot, S = C + A^*(M1) on the slot (ALMSetGrad
            // lorads_alm.c:38-57 with M1 formed from rec), its local constraint records
            const int kc = c0 + lane < ke ? c0 + lane : c0;
            const int jl = adj_col[kc], sl = adj_slot[kc];
            double svl = Craw[sl];
            const double2 s1l = slot1[sl];
            const int c1 = (int)s1l.y;
            {
                const double2 *r = reinterpret_cast<const double2 *>(rec + 4L * (c1 >= 0 ? c1 : ispare));
                const double2 ra = r[0], rb = r[1];
                if (c1 >= 0) {
                    double cv = ra.x + tau * ra.y;
                    cv = cv + tau2 * rb.x;
                    svl += (rb.y + rho * cv) * s1l.x;
                } else if (c1 == -2) {
                    for (int e = slot_ptr[sl]; e < slot_ptr[sl + 1]; ++e) {
                        const double2 *q = reinterpret_cast<const double2 *>(rec + 4L * slot_con[e]);
                        const double2 x = q[0], y = q[1];
                        double cv = x.x + tau * x.y;
                        cv = cv + tau2 * y.x;
                        svl += (y.y + rho * cv) * slot_a[e];
                    }
                }
            }
            const bool lowl = kc < kl;
            const double2 l1l = lowl ? loc1[sl] : make_double2(0.0, -1.0);
            const double bl = b[(int)l1l.y >= 0 ? (int)l1l.y : ispare];
            const int nc = min(G, ke - c0);
            for (int u0 = 0; u0 < nc; u0 += U) {
                double rj[U][E];
#pragma unroll
                for (int v = 0; v < U; ++v) {
                    const int j = bcast_i<G>(jl, min(u0 + v, nc - 1));
                    ld_row<E>(Rn + (long)j * ld + lane * E, rj[v]);
                }
#pragma unroll
                for (int v = 0; v < U; ++v) {
                    const int u = u0 + v;
                    if (u >= nc) break;
                    const double sv = bcast_d<G>(svl, u);
#pragma unroll
                    for (int e = 0; e < E; ++e) g[e] += sv * rj[v][e];
                    if (c0 + u < kl) {   // lower entry: A(R_new R_new^T) slot owned by this row
                        double d = 0.0;
#pragma unroll
                        for (int e = 0; e < E; ++e) d += ri[e] * rj[v][e];
                        d = group_sum<G>(d);
                        if (lane == u) {
                            uRR[sl] = d;
                            const int cl = (int)l1l.y;
                            const int f0 = cl == -2 ? loc_ptr[sl] : 0;
                            const int f1 = cl == -2 ? loc_ptr[sl + 1] : (cl >= 0 ? 1 : 0);
                            for (int e = f0; e < f1; ++e) {
                                const int ci = cl >= 0 ? cl : loc_con[e];
                                const double tot = (cl >= 0 ? l1l.x : loc_w[e]) * d;
                                cvs[ci] = tot;
                                const double dd = (cl >= 0 ? bl : b[ci]) - tot;
                                acc[9] += dd * dd;
                            }
                        }
                    }
                }
            }
        }
        if constexpr (TL) st_row<E>(GP + xg * gstride + foff + oi, g);
        else wide_b_epilogue<E>(g, oi, foff, tau, D, Gold, Gnew, sh, yh, so, yo, two, CRb, CDb, acc);
    }
    write_partials<10, kRowBlock>(acc, partC, pblk_off + blockIdx.x);
}

// k_wide_b over 2-D tiles (cones with DevCone::sb_blocks), in two kernels and k_wide_bf:
// k_tile_b1 -- per lower slot of the A-tiles, S = C + A^*(M1) from rec (ALMSetGrad
//   lorads_alm.c:38-57 as k_wide_b) into sa_S, and A(R_new R_new^T) from R_new staged in LDS
//   (uRR, local constraints' new A(.) and residual partial);
// k_tile_b2 -- G partials: block (row tile I, column group x) stages R_new of each column tile
//   J of its group in LDS, 64 columns at a time, and thread (row, quarter) sums S_ij R_new,j
//   over its row's entries of the tile pair in column order, 16 columns at a time, into GP[x];
// k_wide_bf sums the kNX partial rows in group order and runs the row epilogue.
__global__ void __launch_bounds__(kRowBlock, 4) k_tile_b1(   // <= 128 VGPRs: two blocks a CU (68 KB LDS each)
    int n, int r, int ld, long foff, int nitems, const int4 *__restrict__ items, const unsigned *__restrict__ pq,
    const int *__restrict__ tslot, const double *Rb0, const double *Rb1, double *__restrict__ uRR,
    double *__restrict__ Sv, const double *__restrict__ Craw, const int *__restrict__ slot_ptr,
    const int *__restrict__ slot_con, const double *__restrict__ slot_a, const double2 *__restrict__ slot1,
    const double *__restrict__ rec, const int *__restrict__ loc_ptr, const int *__restrict__ loc_con,
    const double *__restrict__ loc_w, const double2 *__restrict__ loc1, const double *__restrict__ b,
    double *__restrict__ cvs, const double *__restrict__ par, const double *__restrict__ ctrl,
    const double *__restrict__ ls_cur, double *__restrict__ partC, int pblk_off, int nwork) {
    if (ctrl[C_ACT2] == 0.0 || ls_cur[LS_FLAG] != 0.0) return;
    const double tau = ls_cur[LS_TAU], tau2 = tau * tau, rho = par[P_RHO];
    const double *__restrict__ Rn = (ctrl[C_RCUR] == 0.0 ? Rb1 : Rb0) + foff;
    __shared__ double tl[2][kAuvT * kAuvS];
    double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int itx = blockIdx.x; itx < nitems && (int)blockIdx.x < nwork; itx += nwork) {   // block-uniform
        const int4 it = items[itx];
        const int I0 = it.x, J0 = it.y, eb = it.z, ee = it.w;
        int pl[kAuvNpt], ql[kAuvNpt];
        double dv[kAuvNpt];
#pragma unroll
        for (int j = 0; j < kAuvNpt; ++j) {
            const int t = eb + (int)threadIdx.x + j * kAuvThreads;
            const unsigned w = t < ee ? pq[t] : 0u;
            pl[j] = (int)(w >> 16) * kAuvS;
            ql[j] = (int)(w & 0xffffu) * kAuvS;
            dv[j] = 0.0;
        }
        for (int c0 = 0; c0 < r; c0 += kAuvC) {
            double2 v[2][kAuvPer];
            auv_fetch<2>(v, I0, J0, c0, n, r, ld, Rn, Rn);
            __syncthreads();
            auv_put<2>(tl, v);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kAuvNpt; ++j) {
                if (eb + (int)threadIdx.x + j * kAuvThreads >= ee) break;
                double unused = 0.0;
                auv_chunk<1>(tl, pl[j], ql[j], dv[j], unused);
            }
        }
        // the slot epilogue, kB1H slots at a time with their loads issued before the arithmetic
        // (branch-free indices: entries past the item read the item's first slot, store nothing)
        constexpr int kB1H = 4;
#pragma unroll
        for (int h = 0; h < kAuvNpt; h += kB1H) {
        int slv[kB1H];
        double2 s1v[kB1H], l1v[kB1H];
        double crv[kB1H];
#pragma unroll
        for (int j = 0; j < kB1H; ++j) {
            const int t = eb + (int)threadIdx.x + (h + j) * kAuvThreads;
            slv[j] = tslot[t < ee ? t : eb];
        }
#pragma unroll
        for (int j = 0; j < kB1H; ++j) {
            s1v[j] = slot1[slv[j]];
            l1v[j] = loc1[slv[j]];
            crv[j] = Craw[slv[j]];
        }
        double2 rav[kB1H], rbv[kB1H];
#pragma unroll
        for (int j = 0; j < kB1H; ++j) {
            const int c1 = (int)s1v[j].y;
            const double2 *q = reinterpret_cast<const double2 *>(rec + 4L * (c1 >= 0 ? c1 : 0));
            rav[j] = q[0];
            rbv[j] = q[1];
        }
#pragma unroll
        for (int j = 0; j < kB1H; ++j) {
            const int t = eb + (int)threadIdx.x + (h + j) * kAuvThreads;
            if (t >= ee) break;
            const int sl = slv[j];
            double svl = crv[j];
            const double2 s1l = s1v[j];
            const int c1 = (int)s1l.y;
            if (c1 >= 0) {
                double cv = rav[j].x + tau * rav[j].y;
                cv = cv + tau2 * rbv[j].x;
                svl += (rbv[j].y + rho * cv) * s1l.x;
            } else if (c1 == -2) {
                for (int e = slot_ptr[sl]; e < slot_ptr[sl + 1]; ++e) {
                    const double2 *q = reinterpret_cast<const double2 *>(rec + 4L * slot_con[e]);
                    const double2 x = q[0], y = q[1];
                    double cv = x.x + tau * x.y;
                    cv = cv + tau2 * y.x;
                    svl += (y.y + rho * cv) * slot_a[e];
                }
            }
            Sv[sl] = svl;
            const double d = dv[h + j];
            uRR[sl] = d;
            const double2 l1l = l1v[j];
            const int cl = (int)l1l.y;
            const int f0 = cl == -2 ? loc_ptr[sl] : 0, f1 = cl == -2 ? loc_ptr[sl + 1] : (cl >= 0 ? 1 : 0);
            for (int e = f0; e < f1; ++e) {
                const int ci = cl >= 0 ? cl : loc_con[e];
                const double tot = (cl >= 0 ? l1l.x : loc_w[e]) * d;
                cvs[ci] = tot;
                const double dd = b[ci] - tot;
                acc[9] += dd * dd;
            }
        }
        }
    }
    write_partials<10, kRowBlock>(acc, partC, pblk_off + blockIdx.x);
}

constexpr int kTbC = 64;            // R_new columns staged per pass in k_tile_b2
// LDS row stride: unpadded, so every staged row starts on bank 0 and the two rows a
// ds_read_b128 service group mixes ({0-3,12-15} of one 16-lane row, {20-27} of the next,
// MI355X_MICROARCH.md §LDS) fall on disjoint banks whichever rows they are
constexpr int kTbS = kTbC;
constexpr int kTbPer = kAuvT * kTbC / 2 / kRowBlock;   // double2 per thread per staged tile
constexpr int kTbL = 16;            // lanes per tile row in k_tile_b2 (one 256-B LDS row read per 16 lanes)
constexpr int kTbRows = kAuvT / (kRowBlock / kTbL);     // tile rows per lane group
__device__ __forceinline__ void tb_fetch(double2 (&v)[kTbPer], int J0, int c0, int n, int r, int ld,
                                         const double *__restrict__ Rn) {
#pragma unroll
    for (int k = 0; k < kTbPer; ++k) {
        const int y = threadIdx.x + k * kRowBlock;
        const int grow = J0 + y / (kTbC / 2), col = c0 + 2 * (y % (kTbC / 2));
        double2 t = make_double2(0.0, 0.0);
        if (grow < n && col < r) {
            t = *reinterpret_cast<const double2 *>(Rn + (long)grow * ld + col);
            if (col + 1 >= r) t.y = 0.0;
        }
        v[k] = t;
    }
}
// Row broadcast (DPP row_newbcast, gfx90a+): every lane of each 16-lane row gets lane K's value.
template <int K>
__device__ __forceinline__ int nbc_i(int v) { return __builtin_amdgcn_mov_dpp(v, 0x150 + K, 0xF, 0xF, false); }
// one entry of a k_tile_b2 row batch: column and S from lane K of the lane group, the staged
// neighbour row's two 16-B pieces of this lane, four FMAs
template <int K>
__device__ __forceinline__ void b2_entry(const double *rj, int l, int colv, double sv, double (&g)[4]) {
    const int j = nbc_i<K>(colv);
    const double s = dpp_mov<0x150 + K>(sv);
    const double2 *p = reinterpret_cast<const double2 *>(&rj[j * kTbS]) + l;
    const double2 a0 = p[0], a1 = p[kTbL];
    g[0] += s * a0.x; g[1] += s * a0.y; g[2] += s * a1.x; g[3] += s * a1.y;
}
template <int... K>
__device__ __forceinline__ void b2_batch(std::integer_sequence<int, K...>, int kmax, const double *rj, int l, int colv,
                                         double sv, double (&g)[4]) {
    ((K < kmax ? b2_entry<K>(rj, l, colv, sv, g) : void()), ...);
}
// grid: (row tile I, column group x) x column chunk; the chunk's kTbC columns of each tile
// pair's R_new staged in LDS (the next pair's loads in flight during the current one).  A lane
// group of kTbL lanes takes kTbRows rows of the tile; lane l holds the chunk's columns 2l, 2l+1,
// 32+2l, 33+2l, so the group's two ds_read_b128 of a neighbour row read it whole, 256 B each
// (no bank conflicts, whatever the row).  A row's entries come 16 at a time, lane k loading
// entry k's column and slot and the slot's S (the four rows' batches in flight together), and
// the group walks them with a DPP row broadcast of lane k.  Each column's sum runs over the
// row's entries in column order, tile pair by tile pair.
__global__ void __launch_bounds__(kRowBlock) k_tile_b2(int n, int ld, long foff, const int2 *__restrict__ blk,
                                                       const int2 *__restrict__ tp, const int *__restrict__ rp,
                                                       const int2 *__restrict__ ent, const double *__restrict__ Sv,
                                                       const double *Rb0, const double *Rb1, double *__restrict__ GP,
                                                       long gstride, int r, const double *__restrict__ ctrl,
                                                       const double *__restrict__ ls_cur, int tI0) {
    static_assert(kTbC == 4 * kTbL && kTbL == 16, "k_tile_b2: four columns per lane, 16-lane DPP rows");
    // ctrl == nullptr: the standalone S X of launch_spmm (X in Rb0)
    if (ctrl && (ctrl[C_ACT2] == 0.0 || ls_cur[LS_FLAG] != 0.0)) return;
    const double *__restrict__ Rn = ((ctrl && ctrl[C_RCUR] == 0.0) ? Rb1 : Rb0) + foff;
    __shared__ double rj[kAuvT * kTbS];
    const int nch = (ld + kTbC - 1) / kTbC;
    const int bx = blockIdx.x / nch, c0 = (blockIdx.x % nch) * kTbC;
    const int I = tI0 + bx / kNX, x = bx % kNX;   // tI0: a shard's first owned row tile
    const int grp = threadIdx.x / kTbL, l = threadIdx.x % kTbL;
    const int2 br = blk[bx];
    double g[kTbRows][4];
#pragma unroll
    for (int w = 0; w < kTbRows; ++w)
#pragma unroll
        for (int c = 0; c < 4; ++c) g[w][c] = 0.0;
    double2 pre[kTbPer];
    int2 t = br.x < br.y ? tp[br.x] : make_int2(0, 0);
    if (br.x < br.y) tb_fetch(pre, t.x, c0, n, r, ld, Rn);
    for (int q = br.x; q < br.y; ++q) {   // block-uniform
        const int2 cur = t;
        if (q + 1 < br.y) t = tp[q + 1];
        // this tile pair's row ranges and first 16 entries of each row, in flight over the staging
        int e0[kTbRows], e1[kTbRows], cv[kTbRows];
        double sv[kTbRows];
#pragma unroll
        for (int w = 0; w < kTbRows; ++w) {
            const int pl = grp + w * (kRowBlock / kTbL);
            e0[w] = rp[cur.y + pl];
            e1[w] = rp[cur.y + pl + 1];
        }
#pragma unroll
        for (int w = 0; w < kTbRows; ++w) {
            const int e = e0[w] + l;
            const bool ok = e < e1[w];
            const int2 en = ent[ok ? e : e0[w] < e1[w] ? e0[w] : 0];
            cv[w] = en.x;
            sv[w] = ok ? Sv[en.y] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kTbPer; ++k) {
            const int y = threadIdx.x + k * kRowBlock;
            *reinterpret_cast<double2 *>(&rj[(y / (kTbC / 2)) * kTbS + 2 * (y % (kTbC / 2))]) = pre[k];
        }
        __syncthreads();
        if (q + 1 < br.y) tb_fetch(pre, t.x, c0, n, r, ld, Rn);
#pragma unroll
        for (int w = 0; w < kTbRows; ++w) {
            int base = e0[w], colv = cv[w];
            double s = sv[w];
            for (;;) {   // wave-uniform: batches of 16 until the wave's longest row is done
                int rem = e1[w] - base;
                rem = rem < 0 ? 0 : (rem > kTbL ? kTbL : rem);
                const int kmax = max(max(__builtin_amdgcn_readlane(rem, 0), __builtin_amdgcn_readlane(rem, 16)),
                                     max(__builtin_amdgcn_readlane(rem, 32), __builtin_amdgcn_readlane(rem, 48)));
                b2_batch(std::make_integer_sequence<int, kTbL>{}, kmax, rj, l, colv, s, g[w]);
                if (kmax < kTbL) break;
                base += kTbL;
                const int e = base + l;
                const bool ok = e < e1[w];
                const int2 en = ent[ok ? e : (e0[w] < e1[w] ? e0[w] : 0)];   // empty padding rows: entry 0
                colv = en.x;
                s = ok ? Sv[en.y] : 0.0;
            }
        }
    }
#pragma unroll
    for (int w = 0; w < kTbRows; ++w) {
        const int i = I * kAuvT + grp + w * (kRowBlock / kTbL);
        if (i < n) {
            double2 *dst = reinterpret_cast<double2 *>(GP + x * gstride + foff + (long)i * ld + c0) + l;
            if (c0 + 2 * l < ld) dst[0] = make_double2(g[w][0], g[w][1]);
            if (c0 + 2 * (l + kTbL) < ld) dst[kTbL] = make_double2(g[w][2], g[w][3]);
        }
    }
}

// Sharded long-row B over the tiles: S = C + A^*(M1) (k_tile_b1's slot epilogue, lorads_alm.c:38-57)
// on the slots whose lower row is a halo row -- k_tile_b2 reads them as owned rows' upper entries;
// their A(R_new R_new^T) belongs to the shard owning the lower row.
// sx == nullptr: the slots [s0, s0 + nx) (every slot of a cone); partZ: this
// launch's partial blocks of stage B (pblk_off on) written as zeros, the partial slots it stands in for.
__global__ void __launch_bounds__(kBlock) k_slot_sv(int nx, const int *__restrict__ sx, int s0, double *__restrict__ Sv,
                                                    const double *__restrict__ Craw, const int *__restrict__ slot_ptr,
                                                    const int *__restrict__ slot_con, const double *__restrict__ slot_a,
                                                    const double2 *__restrict__ slot1, const double *__restrict__ rec,
                                                    const double *__restrict__ par, const double *__restrict__ ctrl,
                                                    const double *__restrict__ ls_cur, double *__restrict__ partZ,
                                                    int pblk_off) {
    if (ctrl[C_ACT2] == 0.0 || ls_cur[LS_FLAG] != 0.0) return;
    const double tau = ls_cur[LS_TAU], tau2 = tau * tau, rho = par[P_RHO];
    if (partZ && threadIdx.x < 10) partZ[threadIdx.x * kMaxPartialBlocks + pblk_off + blockIdx.x] = 0.0;
    for (int t = blockIdx.x * kBlock + threadIdx.x; t < nx; t += gridDim.x * kBlock) {
        const int sl = sx ? sx[t] : s0 + t;
        double svl = Craw[sl];
        const double2 s1l = slot1[sl];
        const int c1 = (int)s1l.y;
        if (c1 >= 0) {
            const double2 *q = reinterpret_cast<const double2 *>(rec + 4L * c1);
            const double2 ra = q[0], rb = q[1];
            double cv = ra.x + tau * ra.y;
            cv = cv + tau2 * rb.x;
            svl += (rb.y + rho * cv) * s1l.x;
        } else if (c1 == -2) {
            for (int e = slot_ptr[sl]; e < slot_ptr[sl + 1]; ++e) {
                const double2 *q = reinterpret_cast<const double2 *>(rec + 4L * slot_con[e]);
                const double2 x = q[0], y = q[1];
                double cv = x.x + tau * x.y;
                cv = cv + tau2 * y.x;
                svl += (y.y + rho * cv) * slot_a[e];
            }
        }
        Sv[sl] = svl;
    }
}

// B, column-tiled: the eight partial S R_new rows summed in block order, then the row epilogue
template <int G, int E>
__global__ void __launch_bounds__(kRowBlock) k_wide_bf(int n, int ld, long foff, const double *__restrict__ Dall,
                                                       double *G0, double *G1, double *s0, double *y0, double *s1,
                                                       double *y1, const double *__restrict__ ctrl,
                                                       const double *__restrict__ ls_cur, int L,
                                                       double *__restrict__ partC, int pblk_off, int row0, double *CRb,
                                                       const double *__restrict__ CDb, const double *__restrict__ GP,
                                                       long gstride) {
    if (ctrl[C_ACT2] == 0.0 || ls_cur[LS_FLAG] != 0.0) return;
    const double tau = ls_cur[LS_TAU];
    const int gcur = (int)ctrl[C_GCUR], h = (int)ctrl[C_HEAD];
    const double *__restrict__ D = Dall + foff;
    const double *__restrict__ Gold = (gcur == 0 ? G0 : G1) + foff;
    double *__restrict__ Gnew = (gcur == 0 ? G1 : G0) + foff;
    double *__restrict__ sh = (h == 0 ? s0 : s1) + foff;
    double *__restrict__ yh = (h == 0 ? y0 : y1) + foff;
    const double *__restrict__ so = (h == 0 ? s1 : s0) + foff;
    const double *__restrict__ yo = (h == 0 ? y1 : y0) + foff;
    const int lane = threadIdx.x & (G - 1);
    const int grp = (blockIdx.x * kRowBlock + threadIdx.x) / G;
    const int ngrp = gridDim.x * kRowBlock / G;
    double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = row0 + grp; i < row0 + n; i += ngrp) {
        const long oi = (long)i * ld + lane * E;
        double g[E], t[E];
        ld_row<E>(GP + foff + oi, g);
#pragma unroll
        for (int x = 1; x < kNX; ++x) {
            ld_row<E>(GP + x * gstride + foff + oi, t);
#pragma unroll
            for (int e = 0; e < E; ++e) g[e] += t[e];
        }
        wide_b_epilogue<E>(g, oi, foff, tau, D, Gold, Gnew, sh, yh, so, yo, L == 2, CRb, CDb, acc);
    }
    write_partials<10, kRowBlock>(acc, partC, pblk_off + blockIdx.x);
}

// ------------------------------------------------------------------------
// Dual infeasibility (calculate_dual_infeasibility_solver, data/lorads_solver.c:1396-1426):
// lambda_min of S = C - sum_i lambda_i A_i per cone.  The reference runs ARPACK dsaupd
// ("SA", ncv 40, tol 1e-2; dual_infeasible, data/lorads_sdp_conic.c:1636-1699).  Here: a
// Lanczos process with full reorthogonalisation on the device -- S x over the cone's
// symmetric adjacency, Q^T w and w - Q h as row-blocked kernels -- the host keeps the
// tridiagonal and its smallest eigenvalue (lrs_solver.cpp lanczos_min).
// ------------------------------------------------------------------------
// y = S x on one cone (S on the pattern slots): a thread per row, or a wave per row (WAVE)
template <bool WAVE>
__global__ void __launch_bounds__(kBlock) k_symv(int n, const int *__restrict__ adj_ptr, const int *__restrict__ adj_col,
                                                 const int *__restrict__ adj_slot, const double *__restrict__ S,
                                                 const double *__restrict__ x, double *__restrict__ y) {
    if constexpr (WAVE) {
        const int lane = threadIdx.x & 63;
        const int nw = gridDim.x * (kBlock / 64);
        for (int i = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); i < n; i += nw) {
            double acc = 0.0;
            for (int k = adj_ptr[i] + lane; k < adj_ptr[i + 1]; k += 64) acc += S[adj_slot[k]] * x[adj_col[k]];
            acc = wave_sum(acc);
            if (lane == 0) y[i] = acc;
        }
    } else {
        for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
            double acc = 0.0;
            for (int k = adj_ptr[i]; k < adj_ptr[i + 1]; ++k) acc += S[adj_slot[k]] * x[adj_col[k]];
            y[i] = acc;
        }
    }
}
// part[c][blockIdx.x] = sum over this block's rows of Q[c][i] w[i]   (grid.y = column c)
__global__ void __launch_bounds__(kBlock) k_gemvt_part(int n, const double *__restrict__ Q, long ldq,
                                                       const double *__restrict__ w, double *__restrict__ part) {
    const int c = blockIdx.y;
    double a[1] = {0.0};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) a[0] += Q[c * ldq + i] * w[i];
    double s[1];
    block_reduce<1>(a, s);
    if (threadIdx.x == 0) part[(long)c * gridDim.x + blockIdx.x] = s[0];
}
// h[c] = sum over the blocks' partials in block order
__global__ void __launch_bounds__(kBlock) k_gemvt_fin(int k, int nb, const double *__restrict__ part,
                                                      double *__restrict__ h) {
    for (int c = blockIdx.x * kBlock + threadIdx.x; c < k; c += gridDim.x * kBlock) {
        double t = 0.0;
        for (int b = 0; b < nb; ++b) t += part[(long)c * nb + b];
        h[c] = t;
    }
}
// w -= Q h (k columns)
__global__ void __launch_bounds__(kBlock) k_gemv_sub(int n, int k, const double *__restrict__ Q, long ldq,
                                                     const double *__restrict__ h, double *__restrict__ w) {
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        double t = 0.0;
        for (int c = 0; c < k; ++c) t += Q[c * ldq + i] * h[c];
        w[i] -= t;
    }
}

// ---- Thick-restart Lanczos steps (dual infeasibility, lrs_solver.cpp trl_min).  The host
// drives step j of a cycle with plain launches (no captured graphs: every argument,
// dense_scale included, is the current one).  Vectors are the cone's local rows (a sharded
// solve: owned + halo, the kernels touch the owned rows [r0, r0 + nown) only); the basis
// V holds ncv + 1 vectors of ldv doubles.  Step j: v_j = w / beta_{j-1} (beta^2 read from
// device memory; 0 -> v_j = 0, so a breakdown never produces NaN), y = S v_j, two passes of
// classical Gram-Schmidt against v_0..v_j whose coefficients (the entries of V^T S V) go to
// column j of H, and ||y||^2 (beta_j^2) to bw2[j].
__device__ __forceinline__ double trl_inv(const double *b2) {
    if (!b2) return 1.0;
    const double v = *b2;
    return v > 1e-300 ? 1.0 / sqrt(v) : 0.0;
}
// vj[i] = w[i] * inv over rows [0, n) (pointers pre-offset to the first owned row)
__global__ void __launch_bounds__(kBlock) k_trl_norm(int n, const double *__restrict__ w,
                                                     const double *__restrict__ b2, double *__restrict__ vj) {
    const double inv = trl_inv(b2);
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) vj[i] = w[i] * inv;
}
// y = S (x inv) over rows [r0, r0 + n) (x read at any local row); vj (optional) = x inv on
// those rows.  A thread per row, or a wave per row (WAVE, long rows).
template <bool WAVE>
__global__ void __launch_bounds__(kBlock) k_trl_symv(int n, int r0, const int *__restrict__ adj_ptr,
                                                     const int *__restrict__ adj_col, const int *__restrict__ adj_slot,
                                                     const double *__restrict__ S, const double *x,
                                                     const double *__restrict__ b2, double *vj, double *__restrict__ y) {
    const double inv = trl_inv(b2);
    if constexpr (WAVE) {
        const int lane = threadIdx.x & 63;
        const int nw = gridDim.x * (kBlock / 64);
        for (int i = r0 + blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); i < r0 + n; i += nw) {
            double t = 0.0;
            for (int k = adj_ptr[i] + lane; k < adj_ptr[i + 1]; k += 64) t += S[adj_slot[k]] * x[adj_col[k]];
            t = wave_sum(t);
            if (lane == 0) {
                y[i] = t * inv;
                if (vj) vj[i] = x[i] * inv;
            }
        }
    } else {
        for (int i = r0 + blockIdx.x * kBlock + threadIdx.x; i < r0 + n; i += gridDim.x * kBlock) {
            double t = 0.0;
            for (int k = adj_ptr[i]; k < adj_ptr[i + 1]; ++k) t += S[adj_slot[k]] * x[adj_col[k]];
            y[i] = t * inv;
            if (vj) vj[i] = x[i] * inv;
        }
    }
}
// dense objective: y += scale C v over the cone's row block (rows r0 .. r0 + nr - 1, C row t
// holding row r0 + t's n columns; one wave per row)
__global__ void __launch_bounds__(kBlock) k_trl_dense(int n, int nr, int r0, double scale, const double *__restrict__ Cd,
                                                      const double *__restrict__ v, double *__restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int nw = gridDim.x * (kBlock / 64);
    for (int i = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); i < nr; i += nw) {
        const double *__restrict__ ci = Cd + (long)i * n;
        double t = 0.0;
        for (int k = lane; k < n; k += 64) t += ci[k] * v[k];
        t = wave_sum(t);
        if (lane == 0) y[r0 + i] += scale * t;
    }
}
// constant objective: y += sa sum(v) (one block, fixed order)
__global__ void __launch_bounds__(kBlock) k_trl_cj(int n, double sa, const double *__restrict__ v,
                                                   double *__restrict__ y) {
    double a[1] = {0.0};
    for (int i = threadIdx.x; i < n; i += kBlock) a[0] += v[i];
    double s[1];
    block_reduce<1>(a, s);
    __shared__ double tot;
    if (threadIdx.x == 0) tot = sa * s[0];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kBlock) y[i] += tot;
}
// part[c][blockIdx.x] = sum over this block's rows of V[c][i] y[i], c = blockIdx.y
__global__ void __launch_bounds__(kBlock) k_trl_dots(int n, const double *__restrict__ V, long ldv,
                                                     const double *__restrict__ y, double *__restrict__ part) {
    const int c = blockIdx.y;
    double a[1] = {0.0};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) a[0] += V[c * ldv + i] * y[i];
    double s[1];
    block_reduce<1>(a, s);
    if (threadIdx.x == 0) part[(long)c * gridDim.x + blockIdx.x] = s[0];
}
// tot[c] = sum of column c's nb partials in block order (sharded: before the all-reduce)
__global__ void __launch_bounds__(kBlock) k_trl_fold(int k, int nb, const double *__restrict__ part,
                                                     double *__restrict__ tot) {
    for (int c = threadIdx.x; c < k; c += kBlock) {
        double t = 0.0;
        for (int b = 0; b < nb; ++b) t += part[(long)c * nb + b];
        tot[c] = t;
    }
}
// y -= V h, h[c] = sum of column c's partials (block order), c < k <= kTrlMaxV.  A block takes
// 64 rows; its four waves split the columns (wave w: c = w, w + 4, ...), a lane per row, and
// the waves' sums meet in LDS in wave order.  Pass 0 stores h into H's column, pass 1 adds its
// h and reduces ||y||^2 into *bw2 (the last block sums the block partials in order).
__global__ void __launch_bounds__(kBlock) k_trl_sub(int n, const double *__restrict__ V, long ldv, int k,
                                                    const double *__restrict__ part, int nb, double *__restrict__ y,
                                                    double *__restrict__ Hc, int pass, double *npart, unsigned *ticket,
                                                    double *bw2) {
    static_assert(kBlock == 256, "four waves per block");
    __shared__ double h[kTrlMaxV];
    __shared__ double ws[4][64];
    for (int c = threadIdx.x; c < k; c += kBlock) {
        double t = 0.0;
        for (int b = 0; b < nb; ++b) t += part[(long)c * nb + b];
        h[c] = t;
        if (blockIdx.x == 0) Hc[c] = pass == 0 ? t : Hc[c] + t;
    }
    __syncthreads();
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double acc[1] = {0.0};
    for (int i0 = blockIdx.x * 64; i0 < n; i0 += gridDim.x * 64) {   // block-uniform
        const int i = i0 + lane;
        double t = 0.0;
        if (i < n)
            for (int c = wv; c < k; c += 4) t += V[c * ldv + i] * h[c];
        ws[wv][lane] = t;
        __syncthreads();
        if (wv == 0 && i < n) {
            const double v = y[i] - (((ws[0][lane] + ws[1][lane]) + ws[2][lane]) + ws[3][lane]);
            y[i] = v;
            acc[0] += v * v;
        }
        __syncthreads();
    }
    if (pass == 1) partials_finalize<1>(acc, npart, ticket, bw2);
}
// thick restart: Vt[c][i] = sum_q V[q][i] Y[q][c] (Y: m x kk row-major), c < kk
__global__ void __launch_bounds__(kBlock) k_trl_restart(int n, const double *__restrict__ V, long ldv, int m,
                                                        const double *__restrict__ Y, int kk, double *__restrict__ Vt) {
    const int c = blockIdx.y;
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        double t = 0.0;
        for (int q = 0; q < m; ++q) t += V[q * ldv + i] * Y[q * kk + c];
        Vt[c * ldv + i] = t;
    }
}

static unsigned *ticket_ptr(int id);
int trl_nblk(int n) { return std::max(1, std::min(64, (n + kBlock * 8 - 1) / (kBlock * 8))); }

int launch_trl_norm(int n, const double *w, const double *b2, double *vj, hipStream_t st) {
    hipLaunchKernelGGL(k_trl_norm, dim3(grid_elems(n, 4)), dim3(kBlock), 0, st, n, w, b2, vj);
    LRS_CHECK_LAUNCH();
    return 0;
}

int launch_trl_symv(const DevProblem &P, int cone, const double *S, const double *x, const double *b2, double *vj,
                    double *y, hipStream_t st) {
    const DevCone &c = P.cones[cone];
    const int n = c.nown, r0 = c.row0;
    const double deg = c.n > 0 ? (double)c.adj_nnz / c.n : 0.0;
    if (deg > 32.0) {
        const int ga = std::max(1, std::min(4096, (n + kBlock / 64 - 1) / (kBlock / 64)));
        hipLaunchKernelGGL(k_trl_symv<true>, dim3(ga), dim3(kBlock), 0, st, n, r0, c.adj_ptr, c.adj_col, c.adj_slot, S,
                           x, b2, vj, y);
    } else {
        hipLaunchKernelGGL(k_trl_symv<false>, dim3(grid_elems(n, 1)), dim3(kBlock), 0, st, n, r0, c.adj_ptr, c.adj_col,
                           c.adj_slot, S, x, b2, vj, y);
    }
    LRS_CHECK_LAUNCH();
    if (c.dense_c) {   // y += scale C v (v = vj, already normalized by the caller)
        if (!vj && b2) {
            snprintf(g_err, sizeof(g_err), "trl: dense cone needs the normalized vector");
            return -1;
        }
        if (c.dense_c == 2) {   // y += scale alpha 1 (1^T v)
            hipLaunchKernelGGL(k_trl_cj, dim3(1), dim3(kBlock), 0, st, c.n, P.dense_scale * c.c_alpha, vj ? vj : x, y);
        } else {
            const int grid = std::max(1, std::min(2048, (c.nown + kBlock / 64 - 1) / (kBlock / 64)));
            hipLaunchKernelGGL(k_trl_dense, dim3(grid), dim3(kBlock), 0, st, c.n, c.nown, c.row0, P.dense_scale, c.Cd,
                               vj ? vj : x, y);
        }
        LRS_CHECK_LAUNCH();
    }
    return 0;
}

int launch_trl_dots(int n, const double *V, long ldv, int k, const double *y, double *part, hipStream_t st) {
    hipLaunchKernelGGL(k_trl_dots, dim3(trl_nblk(n), k), dim3(kBlock), 0, st, n, V, ldv, y, part);
    LRS_CHECK_LAUNCH();
    return 0;
}

int launch_trl_fold(int k, int nb, const double *part, double *tot, hipStream_t st) {
    hipLaunchKernelGGL(k_trl_fold, dim3(1), dim3(kBlock), 0, st, k, nb, part, tot);
    LRS_CHECK_LAUNCH();
    return 0;
}

int launch_trl_sub(int n, const double *V, long ldv, int k, const double *part, int nb, double *y, double *Hc,
                   int pass, double *npart, double *bw2, hipStream_t st) {
    if (k > kTrlMaxV) {
        snprintf(g_err, sizeof(g_err), "trl: %d basis vectors past %d", k, kTrlMaxV);
        return -1;
    }
    hipLaunchKernelGGL(k_trl_sub, dim3(std::max(1, std::min((n + 63) / 64, kMaxPartialBlocks))), dim3(kBlock), 0, st, n,
                       V, ldv, k, part, nb, y, Hc, pass, npart, ticket_ptr(T_DOT), bw2);
    LRS_CHECK_LAUNCH();
    return 0;
}

int launch_trl_restart(int n, const double *V, long ldv, int m, const double *Y, int kk, double *Vt, hipStream_t st) {
    hipLaunchKernelGGL(k_trl_restart, dim3(grid_elems(n, 1), kk), dim3(kBlock), 0, st, n, V, ldv, m, Y, kk, Vt);
    LRS_CHECK_LAUNCH();
    return 0;
}

int launch_symv(const DevProblem &P, int cone, const double *S, const double *x, double *y, hipStream_t st) {
    const DevCone &c = P.cones[cone];
    const double deg = c.n > 0 ? (double)c.adj_nnz / c.n : 0.0;
    if (deg > 32.0) {
        const int grid = std::max(1, std::min(4096, (c.n + kBlock / 64 - 1) / (kBlock / 64)));
        hipLaunchKernelGGL(k_symv<true>, dim3(grid), dim3(kBlock), 0, st, c.n, c.adj_ptr, c.adj_col, c.adj_slot, S, x, y);
    } else {
        hipLaunchKernelGGL(k_symv<false>, dim3(grid_elems(c.n, 1)), dim3(kBlock), 0, st, c.n, c.adj_ptr, c.adj_col,
                           c.adj_slot, S, x, y);
    }
    LRS_CHECK_LAUNCH();
    return 0;
}
int launch_reorth(int n, int k, const double *Q, long ldq, double *w, double *part, double *h, hipStream_t st) {
    if (k <= 0) return 0;
    const int nb = std::max(1, std::min(64, (n + kBlock * 8 - 1) / (kBlock * 8)));
    hipLaunchKernelGGL(k_gemvt_part, dim3(nb, k), dim3(kBlock), 0, st, n, Q, ldq, w, part);
    LRS_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_gemvt_fin, dim3((k + kBlock - 1) / kBlock), dim3(kBlock), 0, st, k, nb, part, h);
    LRS_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_gemv_sub, dim3(grid_elems(n, 1)), dim3(kBlock), 0, st, n, k, Q, ldq, h, w);
    LRS_CHECK_LAUNCH();
    return 0;
}

// ------------------------------------------------------------------------
// Device-resident CG (CGSolve, linalg/lorads_cgs.c:128-287) for one cone's ADMM
// half-step system M X = b, M x = x + A^*(A(sym(x V^T))) V (linSysProduct,
// lorads_admm.c:471-486).  Scalars live in cgc[] (CgIdx); every kernel after the
// initial residual is guarded by cgc[CG_ACTIVE], so a batch of iterations enqueued
// past convergence does nothing.  Same partial-sum scheme as the ALM iteration.
// ------------------------------------------------------------------------
// sum |b| over the cone's factor rows (bNorm, lorads_cgs.c: nrm1 of the RHS)
__global__ void __launch_bounds__(kBlock) k_cg_nrm1(long nr, const double *__restrict__ b, double *__restrict__ part) {
    double acc[1] = {0.0};
    for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < nr; i += (long)gridDim.x * kBlock) acc[0] += fabs(b[i]);
    write_partials<1>(acc, part, blockIdx.x);
}

// Q = A^*(w) V + Xin on the cone's rows (S on the fly from the slot lists), optional
// partial <Xin, Q>.  Teams of T lane groups per row for dense rows (as k_it_b).
template <int G, int E, int U>
__global__ void __launch_bounds__(kRowBlock) k_cg_mv(int n, int ld, const int *__restrict__ adj_ptr,
                                                     const int *__restrict__ adj_col, const int *__restrict__ adj_slot,
                                                     const int *__restrict__ slot_ptr,
                                                     const int *__restrict__ slot_con,
                                                     const double *__restrict__ slot_a, const double *__restrict__ w,
                                                     const double *__restrict__ V, const double *__restrict__ Xin,
                                                     double *__restrict__ Q, double *__restrict__ part,
                                                     const double *__restrict__ cgc, int guarded, int T) {
    __shared__ double gsh[kRowBlock * E];
    if (guarded && cgc[CG_ACTIVE] == 0.0) return;
    const int lane = threadIdx.x & (G - 1);
    const int grp = (blockIdx.x * kRowBlock + threadIdx.x) / G;
    const int ngrp = gridDim.x * kRowBlock / G;
    const int team = grp / T, mem = grp % T, nteams = ngrp / T;
    const int tpb = (kRowBlock / G) / T;
    const int team_local = team - blockIdx.x * tpb;
    double acc[1] = {0.0};
    for (int ib = blockIdx.x * tpb; ib < n; ib += nteams) {
        const int i = ib + team_local;
        const bool valid = i < n;
        double g[E];
#pragma unroll
        for (int e = 0; e < E; ++e) g[e] = 0.0;
        if (valid) {
            const int kb = adj_ptr[i], ke = adj_ptr[i + 1];
            for (int k0 = kb + mem * U; k0 < ke; k0 += T * U) {
                int jj[U], ss[U], eb[U], ee[U];
                double yj[U][E], sv[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int k = min(k0 + u, ke - 1);
                    jj[u] = adj_col[k];
                    ss[u] = adj_slot[k];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    ld_row<E>(V + (long)jj[u] * ld + lane * E, yj[u]);
                    eb[u] = slot_ptr[ss[u]];
                    ee[u] = slot_ptr[ss[u] + 1];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    // S[slot] = sum_con w[con] a  (sdpDataWSum without C)
                    double v = 0.0;
                    for (int e = eb[u]; e < ee[u]; ++e) v += w[slot_con[e]] * slot_a[e];
                    sv[u] = v;
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (k0 + u < ke) {
#pragma unroll
                        for (int e = 0; e < E; ++e) g[e] += sv[u] * yj[u][e];
                    }
            }
        }
        if (T > 1) {
#pragma unroll
            for (int e = 0; e < E; ++e) gsh[threadIdx.x * E + e] = g[e];
            __syncthreads();
            if (mem == 0 && valid) {
                const int base = (team_local * T) * G + lane;
#pragma unroll
                for (int e = 0; e < E; ++e) g[e] = gsh[base * E + e];
                for (int t = 1; t < T; ++t)
#pragma unroll
                    for (int e = 0; e < E; ++e) g[e] += gsh[(base + t * G) * E + e];
            }
            __syncthreads();
        }
        if (mem == 0 && valid) {
            const long oi = (long)i * ld + lane * E;
            double x[E];
            ld_row<E>(Xin + oi, x);
#pragma unroll
            for (int e = 0; e < E; ++e) { g[e] *= 1.0; g[e] += 1.0 * x[e]; }
            st_row<E>(Q + oi, g);
            if (part) {
#pragma unroll
                for (int e = 0; e < E; ++e) acc[0] += x[e] * g[e];
            }
        }
    }
    if (part) write_partials<1, kRowBlock>(acc, part, blockIdx.x);
}

// alpha = qTr / <p, Q>; X += alpha p; r -= alpha Q; partial <r, r>; ITERS = it + 1
__global__ void __launch_bounds__(kBlock) k_cg_upd(long nr, double *__restrict__ X, double *__restrict__ r,
                                                   const double *__restrict__ p, const double *__restrict__ Q,
                                                   const double *__restrict__ partB, int nblkB,
                                                   double *__restrict__ partC, double *__restrict__ cgc, int par,
                                                   int it) {
    __shared__ double red[1];
    __shared__ int act;
    if (threadIdx.x == 0) act = cgc[CG_ACTIVE] != 0.0;
    __syncthreads();
    if (!act) return;
    reduce_partials<1>(partB, nblkB, red);
    const double alpha = cgc[CG_QTR0 + par] / red[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) cgc[CG_ITERS] = it + 1;
    double acc[1] = {0.0};
    for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < nr; i += (long)gridDim.x * kBlock) {
        X[i] = alpha * p[i] + 1.0 * X[i];
        const double ri = -alpha * Q[i] + 1.0 * r[i];
        r[i] = ri;
        acc[0] += ri * ri;
    }
    write_partials<1>(acc, partC, blockIdx.x);
}

// convergence test on ||r||_2 / ||b||_1; unless restarting: beta = rr / qTr,
// p = r + beta p, qTr <- rr (next parity)
__global__ void __launch_bounds__(kBlock) k_cg_conv(long nr, const double *__restrict__ r, double *__restrict__ p,
                                                    const double *__restrict__ partC, int nblkC,
                                                    double *__restrict__ cgc, double tol, int par, int restart) {
    __shared__ double red[1];
    __shared__ int act;
    if (threadIdx.x == 0) act = cgc[CG_ACTIVE] != 0.0;
    __syncthreads();
    if (!act) return;
    reduce_partials<1>(partC, nblkC, red);
    const double rr = red[0];
    const double resi = sqrt(rr);
    if (resi / cgc[CG_BNORM] < tol || resi != resi) {
        if (blockIdx.x == 0 && threadIdx.x == 0) { cgc[CG_ACTIVE] = 0.0; cgc[CG_RR] = rr; }
        return;
    }
    if (restart) return;
    const double beta = rr / cgc[CG_QTR0 + par];
    for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < nr; i += (long)gridDim.x * kBlock)
        p[i] = 1.0 * r[i] + beta * p[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) { cgc[CG_QTR0 + (par ^ 1)] = rr; cgc[CG_RR] = rr; }
}

// r = b - Q (Q = M X), p = r, partial <r, r>.  init: also bNorm from the nrm1 partials
__global__ void __launch_bounds__(kBlock) k_cg_resid(long nr, const double *__restrict__ b,
                                                     const double *__restrict__ Q, double *__restrict__ r,
                                                     double *__restrict__ p, double *__restrict__ partC,
                                                     double *__restrict__ cgc, const double *__restrict__ partA,
                                                     int nblkA, int init) {
    __shared__ double red[1];
    __shared__ int act;
    if (threadIdx.x == 0) act = init || cgc[CG_ACTIVE] != 0.0;
    __syncthreads();
    if (!act) return;
    if (init) {
        reduce_partials<1>(partA, nblkA, red);
        if (blockIdx.x == 0 && threadIdx.x == 0) cgc[CG_BNORM] = red[0];
    }
    double acc[1] = {0.0};
    for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < nr; i += (long)gridDim.x * kBlock) {
        const double ri = 1.0 * b[i] + -1.0 * Q[i];
        r[i] = ri;
        p[i] = ri;
        acc[0] += ri * ri;
    }
    write_partials<1>(acc, partC, blockIdx.x);
}

// init: resi test (ACTIVE), qTr[0] = rr.  restart (lorads_cgs.c restart every 20):
// qTr = rr, beta = rr / qTr, p = r + beta p, qTr[next] = rr
__global__ void __launch_bounds__(kBlock) k_cg_resid2(long nr, const double *__restrict__ r, double *__restrict__ p,
                                                      const double *__restrict__ partC, int nblkC,
                                                      double *__restrict__ cgc, double tol, int par, int init) {
    __shared__ double red[1];
    __shared__ int act;
    if (threadIdx.x == 0) act = init || cgc[CG_ACTIVE] != 0.0;
    __syncthreads();
    if (!act) return;
    reduce_partials<1>(partC, nblkC, red);
    const double rr = red[0];
    if (init) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const double resi = sqrt(rr);
            cgc[CG_ACTIVE] = (resi / cgc[CG_BNORM] < tol) ? 0.0 : 1.0;
            cgc[CG_QTR0] = rr;
            cgc[CG_RR] = rr;
            cgc[CG_ITERS] = 0;
        }
        return;
    }
    const double qTr = rr;
    const double beta = rr / qTr;
    for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < nr; i += (long)gridDim.x * kBlock)
        p[i] = 1.0 * r[i] + beta * p[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) { cgc[CG_QTR0 + (par ^ 1)] = rr; cgc[CG_RR] = rr; }
}

// ------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------
// Per-context scratch of the standalone reductions (tickets, finals, the line search's and
// the fused direction kernel's finals, residual partials), bound to the calling thread by
// the context's every C-ABI entry (several contexts may run concurrently in one process,
// e.g. the shards of the loopback transport, or two solves on two host threads).  There is
// no module-level fallback: the launchers only run inside a bound entry point.
static thread_local unsigned *t_tickets = nullptr;
static thread_local double *t_tmpfin = nullptr, *t_rpart = nullptr, *t_fin = nullptr;
void bind_scratch(unsigned *tickets, double *tmpfin, double *rpart, double *fin) {
    t_tickets = tickets;
    t_tmpfin = tmpfin;
    t_rpart = rpart;
    t_fin = fin;
}
static unsigned *ticket_ptr(int id) { return t_tickets + id; }
static double *fin_ptr() { return t_fin; }
static double *tmpfin_ptr() { return t_tmpfin; }
double *device_tmpfin() { return tmpfin_ptr(); }
double *device_fin() { return fin_ptr(); }

#define LRS_LAYOUT_SWITCH(Gv, Ev, BODY)                                                        \
    switch ((Gv) * 8 + (Ev)) {                                                                 \
    case 8 * 8 + 1: { constexpr int GG = 8, EE = 1; BODY; } break;                             \
    case 8 * 8 + 2: { constexpr int GG = 8, EE = 2; BODY; } break;                             \
    case 8 * 8 + 3: { constexpr int GG = 8, EE = 3; BODY; } break;                             \
    case 8 * 8 + 4: { constexpr int GG = 8, EE = 4; BODY; } break;                             \
    case 16 * 8 + 1: { constexpr int GG = 16, EE = 1; BODY; } break;                           \
    case 16 * 8 + 2: { constexpr int GG = 16, EE = 2; BODY; } break;                           \
    case 16 * 8 + 3: { constexpr int GG = 16, EE = 3; BODY; } break;                           \
    case 16 * 8 + 4: { constexpr int GG = 16, EE = 4; BODY; } break;                           \
    case 32 * 8 + 1: { constexpr int GG = 32, EE = 1; BODY; } break;                           \
    case 32 * 8 + 2: { constexpr int GG = 32, EE = 2; BODY; } break;                           \
    case 32 * 8 + 3: { constexpr int GG = 32, EE = 3; BODY; } break;                           \
    case 32 * 8 + 4: { constexpr int GG = 32, EE = 4; BODY; } break;                           \
    case 64 * 8 + 1: { constexpr int GG = 64, EE = 1; BODY; } break;                           \
    case 64 * 8 + 2: { constexpr int GG = 64, EE = 2; BODY; } break;                           \
    case 64 * 8 + 3: { constexpr int GG = 64, EE = 3; BODY; } break;                           \
    case 64 * 8 + 4: { constexpr int GG = 64, EE = 4; BODY; } break;                           \
    case 64 * 8 + 8: { constexpr int GG = 64, EE = 8; BODY; } break;                           \
    default:                                                                                   \
        snprintf(g_err, sizeof(g_err), "unsupported layout G=%d E=%d", (Gv), (Ev));            \
        return -1;                                                                             \
    }

// Team size (lane groups per row) of the standalone SDDMM / SpMM on cone c: 1 for sparse
// rows (the row loop unchanged); for dense rows up to the block's groups, about 8 entries
// per member (lower entries for the SDDMM).
static int small_team(const DevCone &c, bool lower) {
    const double deg = c.nown > 0 ? (double)c.adj_nnz / c.n : 0.0;
    const double ent = lower ? 0.5 * deg : deg;
    int T = 1;
    while (T * 2 <= kBlock / c.G && T * 2 * 8 <= ent && (long)c.nown * T * 2 * c.G <= 256L * 2048) T *= 2;
    return T;
}

// <C, out0> (and <C, out1>) over one cone's slots after the tiled SDDMM (k_sddmm's fin values)
__global__ void __launch_bounds__(kBlock) k_slot_cdot(int s0, int P, const double *__restrict__ Cw,
                                                      const double *__restrict__ out0,
                                                      const double *__restrict__ out1, double *part,
                                                      unsigned *ticket, double *fin) {
    double acc[2] = {0.0, 0.0};
    for (int s = s0 + blockIdx.x * kBlock + threadIdx.x; s < s0 + P; s += gridDim.x * kBlock) {
        acc[0] += Cw[s] * out0[s];
        if (out1) acc[1] += Cw[s] * out1[s];
    }
    partials_finalize<2>(acc, part, ticket, fin);
}

// a shard's tiled slots only (its owned rows' lower slots, sa_slot), in tile order
__global__ void __launch_bounds__(kBlock) k_slot_cdot_list(int nl, const int *__restrict__ sl, const double *__restrict__ Cw,
                                                           const double *__restrict__ out0,
                                                           const double *__restrict__ out1, double *part,
                                                           unsigned *ticket, double *fin) {
    double acc[2] = {0.0, 0.0};
    for (int t = blockIdx.x * kBlock + threadIdx.x; t < nl; t += gridDim.x * kBlock) {
        const int s = sl[t];
        acc[0] += Cw[s] * out0[s];
        if (out1) acc[1] += Cw[s] * out1[s];
    }
    partials_finalize<2>(acc, part, ticket, fin);
}

int launch_sddmm(const DevProblem &P, int cone, int mode, const double *X, const double *Y, double *out0,
                 double *out1, double *part, int pblk_off, int *nblk_used, hipStream_t st) {
    (void)pblk_off;
    const DevCone &c = P.cones[cone];
    if (c.sa_items > 0) {
        // long-row cone: the pattern SDDMM over the 2-D LDS tiles (k_auv_tile on the slot tiles,
        // values stored per slot), then the objective sums in slot order
        const double *Xc = X + c.foff, *Yc = Y ? Y + c.foff : nullptr;
        const int4 *it = reinterpret_cast<const int4 *>(c.sa_item);
        if (mode == 1)
            hipLaunchKernelGGL((k_auv_tile<1>), dim3(c.sa_items), dim3(kAuvThreads), 0, st, c.n, c.r, c.ld, it,
                               c.sa_pq, c.sa_slot, Xc, Xc, out0, nullptr);
        else
            hipLaunchKernelGGL((k_auv_tile<0>), dim3(c.sa_items), dim3(kAuvThreads), 0, st, c.n, c.r, c.ld, it,
                               c.sa_pq, c.sa_slot, Xc, Yc, out0, nullptr);
        LRS_CHECK_LAUNCH();
        if (mode == 2) {
            hipLaunchKernelGGL((k_auv_tile<1>), dim3(c.sa_items), dim3(kAuvThreads), 0, st, c.n, c.r, c.ld, it,
                               c.sa_pq, c.sa_slot, Yc, Yc, out1, nullptr);
            LRS_CHECK_LAUNCH();
        }
        if (P.shard) {   // the owned rows' lower slots only, as k_sddmm over the owned rows
            const int grid = grid_elems(std::max(1, c.sa_n), 4);
            hipLaunchKernelGGL(k_slot_cdot_list, dim3(grid), dim3(kBlock), 0, st, c.sa_n, c.sa_slot, P.Cw, out0,
                               mode == 2 ? out1 : nullptr, part, ticket_ptr(T_SDDMM),
                               tmpfin_ptr() + TF_SD + 2 * cone);
            LRS_CHECK_LAUNCH();
            if (nblk_used) *nblk_used = grid;
            return 0;
        }
        const int grid = grid_elems(c.P, 4);
        hipLaunchKernelGGL(k_slot_cdot, dim3(grid), dim3(kBlock), 0, st, c.slot_off, c.P, P.Cw, out0,
                           mode == 2 ? out1 : nullptr, part, ticket_ptr(T_SDDMM), tmpfin_ptr() + TF_SD + 2 * cone);
        LRS_CHECK_LAUNCH();
        if (nblk_used) *nblk_used = grid;
        return 0;
    }
    const int T = small_team(c, true);
    const int grid = grid_rows((long)c.nown * T, c.G);
    double *fin = tmpfin_ptr() + TF_SD + 2 * cone;
    const double *Xc = X + c.foff;
    const double *Yc = Y ? Y + c.foff : nullptr;
    LRS_LAYOUT_SWITCH(c.G, c.E, {
        if (mode == 0)
            hipLaunchKernelGGL((k_sddmm<GG, EE, 0>), dim3(grid), dim3(kBlock), 0, st, c.nown, c.ld, c.adj_ptr,
                               c.adj_low, c.adj_col, c.adj_slot, Xc, Yc, out0, out1, P.Cw, part,
                               ticket_ptr(T_SDDMM), fin, nullptr, c.row0, T);
        else if (mode == 1)
            hipLaunchKernelGGL((k_sddmm<GG, EE, 1>), dim3(grid), dim3(kBlock), 0, st, c.nown, c.ld, c.adj_ptr,
                               c.adj_low, c.adj_col, c.adj_slot, Xc, Yc, out0, out1, P.Cw, part,
                               ticket_ptr(T_SDDMM), fin, nullptr, c.row0, T);
        else
            hipLaunchKernelGGL((k_sddmm<GG, EE, 2>), dim3(grid), dim3(kBlock), 0, st, c.nown, c.ld, c.adj_ptr,
                               c.adj_low, c.adj_col, c.adj_slot, Xc, Yc, out0, out1, P.Cw, part,
                               ticket_ptr(T_SDDMM), fin, nullptr, c.row0, T);
    });
    LRS_CHECK_LAUNCH();
    if (nblk_used) *nblk_used = grid;
    return 0;
}

// <C, X Y^T> over a cone's C entries only (DevCone::cobj_slot): a lane group per entry reads
// its two factor rows (auv_entry, as k_auv_con), sum of Cw d -> tmpfin TF_SD + 2 cone [0]
template <int G, int E, int MODE>
__global__ void __launch_bounds__(kBlock) k_cobj(int nl, const int *__restrict__ sl, const int *__restrict__ slot_rc,
                                                 const double *__restrict__ Cw, int ld, const double *__restrict__ X,
                                                 const double *__restrict__ Y, double *part, unsigned *ticket,
                                                 double *fin) {
    const int lane = threadIdx.x & (G - 1);
    const int grp = (blockIdx.x * kBlock + threadIdx.x) / G, ngrp = gridDim.x * kBlock / G;
    double acc[2] = {0.0, 0.0};
    for (int t = grp; t < nl; t += ngrp) {
        const int s = sl[t];
        double d = auv_entry<E, MODE>(X, Y, ld, lane, slot_rc[2 * s], slot_rc[2 * s + 1]);
        d = group_sum<G>(d);
        if (lane == 0) acc[0] += Cw[s] * d;
    }
    partials_finalize<2>(acc, part, ticket, fin);
}
int launch_cobj(const DevProblem &P, int cone, int mode, const double *X, const double *Y, double *part,
                hipStream_t st) {
    const DevCone &c = P.cones[cone];
    const int grid = std::max(1, std::min(grid_rows(std::max(1, c.cobj_n), c.G), 512));
    const double *Xc = X + c.foff, *Yc = Y ? Y + c.foff : X + c.foff;
    LRS_LAYOUT_SWITCH(c.G, c.E, {
        if (mode == 1)
            hipLaunchKernelGGL((k_cobj<GG, EE, 1>), dim3(grid), dim3(kBlock), 0, st, c.cobj_n, c.cobj_slot, P.slot_rc,
                               P.Cw, c.ld, Xc, Xc, part, ticket_ptr(T_SDDMM), tmpfin_ptr() + TF_SD + 2 * cone);
        else
            hipLaunchKernelGGL((k_cobj<GG, EE, 0>), dim3(grid), dim3(kBlock), 0, st, c.cobj_n, c.cobj_slot, P.slot_rc,
                               P.Cw, c.ld, Xc, Yc, part, ticket_ptr(T_SDDMM), tmpfin_ptr() + TF_SD + 2 * cone);
    });
    LRS_CHECK_LAUNCH();
    return 0;
}

int launch_gather(const DevProblem &P, const double *uvt, double scale, double *out, const double *b_for_vio,
                  double *vio_part, hipStream_t st, int *nblk_used) {
    const int grid = grid_elems(P.m, 1);
    hipLaunchKernelGGL(k_gather, dim3(grid), dim3(kBlock), 0, st, P.m, P.K, -1, P.con_ptr, P.con_slot, P.con_w,
                       uvt, scale, out, b_for_vio, vio_part, ticket_ptr(T_GATHER), tmpfin_ptr() + TF_GATHER);
    LRS_CHECK_LAUNCH();
    if (nblk_used) *nblk_used = grid;
    return 0;
}

int launch_gather_cone(const DevProblem &P, int cone, const double *uvt, double *out, hipStream_t st) {
    const int grid = grid_elems(P.m, 1);
    hipLaunchKernelGGL(k_gather, dim3(grid), dim3(kBlock), 0, st, P.m, P.K, cone, P.con_ptr, P.con_slot, P.con_w,
                       uvt, 1.0, out, nullptr, nullptr, ticket_ptr(T_GATHER), tmpfin_ptr() + TF_GATHER);
    LRS_CHECK_LAUNCH();
    return 0;
}

int launch_auv_con(const DevProblem &P, int cone, int mode, const double *X, const double *Y, double scale,
                   int accumulate, double *out, const double *b_for_vio, double *vio_part, hipStream_t st,
                   const double *guard, double *sum_upd) {
    const DevCone &c = P.cones[cone];
    const double *Xc = X + c.foff;
    const double *Yc = Y ? Y + c.foff : nullptr;
    unsigned *tk = ticket_ptr(T_GATHER);
    double *fin = tmpfin_ptr() + TF_GATHER;
    if (c.auv_items > 0 && !P.shard) {
        // 2-D tiles through LDS, then the per-constraint sums
        if (mode == 1)
            hipLaunchKernelGGL((k_auv_tile<1>), dim3(c.auv_items), dim3(kAuvThreads), 0, st, c.n, c.r, c.ld,
                               reinterpret_cast<const int4 *>(c.auv_item), c.auv_pq, c.auv_pos, Xc, Xc, c.auv_val, guard);
        else
            hipLaunchKernelGGL((k_auv_tile<0>), dim3(c.auv_items), dim3(kAuvThreads), 0, st, c.n, c.r, c.ld,
                               reinterpret_cast<const int4 *>(c.auv_item), c.auv_pq, c.auv_pos, Xc, Yc, c.auv_val, guard);
        LRS_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_auv_tsum, dim3(grid_elems(P.m, 1)), dim3(kBlock), 0, st, P.m, cone, P.con_ptr,
                           P.con_w, c.auv_ebase, c.auv_val, scale, accumulate, out, b_for_vio, vio_part,
                           tk, fin, guard, sum_upd);
        LRS_CHECK_LAUNCH();
        return 0;
    }
    if (c.auv_diag && !P.shard && !getenv("LRS_NO_AUV_DIAG")) {
        static int U = -1, BSv = 256;
        if (U < 0) {
            const char *e = getenv("LRS_DIAG_U"); U = e ? atoi(e) : kDiagU;
            const char *f = getenv("LRS_DIAG_BS"); BSv = f ? atoi(f) : 256;
        }
        const int BSx = vio_part ? 256 : BSv;   // the residual's partials: kBlock-thread blocks
        const long thr = (long)((P.m + U - 1) / U) * c.G;
        const int grid = (int)std::max(1L, std::min((long)kMaxPartialBlocks, (thr + BSx - 1) / BSx));
#define LRS_DIAG(UU, BB)                                                                                          \
    LRS_LAYOUT_SWITCH(c.G, c.E, {                                                                                 \
        if (mode == 1)                                                                                            \
            hipLaunchKernelGGL((k_auv_diag<GG, EE, 1, UU, BB>), dim3(grid), dim3(BB), 0, st, P.m, (long)cone * P.m, \
                               c.ld, P.con1_w, Xc, Xc, scale, accumulate, out, b_for_vio, vio_part, tk, fin, guard,  \
                               sum_upd);                                                                          \
        else                                                                                                      \
            hipLaunchKernelGGL((k_auv_diag<GG, EE, 0, UU, BB>), dim3(grid), dim3(BB), 0, st, P.m, (long)cone * P.m, \
                               c.ld, P.con1_w, Xc, Yc, scale, accumulate, out, b_for_vio, vio_part, tk, fin, guard,  \
                               sum_upd);                                                                          \
    })
        if (BSx == 1024) {
            if (U == 1) { LRS_DIAG(1, 1024); }
            else if (U == 2) { LRS_DIAG(2, 1024); }
            else { LRS_DIAG(4, 1024); }
        } else if (BSx == 512) {
            if (U == 1) { LRS_DIAG(1, 512); }
            else if (U == 2) { LRS_DIAG(2, 512); }
            else { LRS_DIAG(4, 512); }
        } else {
            if (U == 1) { LRS_DIAG(1, 256); }
            else if (U == 2) { LRS_DIAG(2, 256); }
            else { LRS_DIAG(4, 256); }
        }
#undef LRS_DIAG
        LRS_CHECK_LAUNCH();
        return 0;
    }
    const int l0 = P.long_ptr_h.empty() ? 0 : P.long_ptr_h[cone];
    const int nlong = P.long_ptr_h.empty() ? 0 : P.long_ptr_h[cone + 1] - l0;
    if (nlong > 0 && b_for_vio) {
        snprintf(g_err, sizeof(g_err), "auv_con: residual with long constraint rows is not supported");
        return -1;
    }
    // row blocks, then a block per long row (at most 64 of them, striding past that)
    const int nlb = std::min(nlong, 64);
    const int grid = std::min(grid_rows(P.m, c.G), kMaxPartialBlocks - nlb);
    const int *lrows = nlong > 0 ? P.long_rows + l0 : nullptr;
    LRS_LAYOUT_SWITCH(c.G, c.E, {
        if (mode == 1)
            hipLaunchKernelGGL((k_auv_con<GG, EE, 1>), dim3(grid + nlb), dim3(kBlock), 0, st, P.m, P.K, cone, c.ld,
                               P.con_ptr, P.con_slot, P.con_w, P.slot_rc, P.con1_pq, P.con1_w, Xc, Yc, scale,
                               accumulate, out, b_for_vio, vio_part, tk, fin, guard, grid, nlong, lrows, sum_upd);
        else
            hipLaunchKernelGGL((k_auv_con<GG, EE, 0>), dim3(grid + nlb), dim3(kBlock), 0, st, P.m, P.K, cone, c.ld,
                               P.con_ptr, P.con_slot, P.con_w, P.slot_rc, P.con1_pq, P.con1_w, Xc, Yc, scale,
                               accumulate, out, b_for_vio, vio_part, tk, fin, guard, grid, nlong, lrows, sum_upd);
    });
    LRS_CHECK_LAUNCH();
    return 0;
}

int launch_wsum(const DevProblem &P, const double *w, int withC, double *S, hipStream_t st) {
    const int grid = grid_elems(P.Ptot, 1);
    hipLaunchKernelGGL(k_wsum, dim3(grid), dim3(kBlock), 0, st, P.Ptot, P.slot_ptr, P.slot_con, P.slot_a, P.Craw,
                       withC, w, S, nullptr, nullptr);
    LRS_CHECK_LAUNCH();
    return 0;
}

// launch_spmm over the tiles: out = scale (sum of the kNX partial rows in group order) +
// addScale addX over the cone's n x ld block, and the partial ||out||^2 (k_spmm's epilogue)
__global__ void __launch_bounds__(kBlock) k_spmm_fin(long len, const double *__restrict__ GP, long gstride,
                                                     double scale, const double *__restrict__ addX,
                                                     double addScale, double *__restrict__ out, double *part,
                                                     unsigned *ticket, double *fin) {
    double nrm[1] = {0.0};
    for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < len; i += (long)gridDim.x * kBlock) {
        double g = GP[i];
#pragma unroll
        for (int x = 1; x < kNX; ++x) g += GP[x * gstride + i];
        double v = g * scale;
        if (addX) v += addScale * addX[i];
        out[i] = v;
        nrm[0] += v * v;
    }
    if (part) partials_finalize<1>(nrm, part, ticket, fin);
}

int launch_spmm(const DevProblem &P, int cone, const double *S, const double *X, double scale, const double *addX,
                double addScale, double *out, double *part, int pblk_off, int *nblk_used, hipStream_t st) {
    (void)pblk_off;
    const DevCone &c = P.cones[cone];
    if (c.sb_blocks > 0 && P.gp) {
        // long-row cone: S X per (row tile, column group) from staged X tiles into P.gp's kNX
        // partial rows (k_tile_b2 without the iteration's control), then the sum and epilogue
        // over the rows the context owns (a shard: [row0, row0 + nown))
        hipLaunchKernelGGL(k_tile_b2, dim3(c.sb_blocks * ((c.ld + kTbC - 1) / kTbC)), dim3(kRowBlock), 0, st, c.n,
                           c.ld, c.foff, reinterpret_cast<const int2 *>(c.sb_blk),
                           reinterpret_cast<const int2 *>(c.sb_tp), c.sb_rp, reinterpret_cast<const int2 *>(c.sb_ent),
                           S, X, X, P.gp, P.NRpad, c.r, nullptr, nullptr, c.sb_I0);
        LRS_CHECK_LAUNCH();
        const long o0 = c.foff + (long)c.row0 * c.ld, len = (long)c.nown * c.ld;
        const int grid = grid_elems(len, 8);
        hipLaunchKernelGGL(k_spmm_fin, dim3(grid), dim3(kBlock), 0, st, len, P.gp + o0, P.NRpad, scale,
                           addX ? addX + o0 : nullptr, addScale, out + o0, part, ticket_ptr(T_SPMM),
                           tmpfin_ptr() + TF_SPMM + cone);
        LRS_CHECK_LAUNCH();
        if (nblk_used) *nblk_used = grid;
        return 0;
    }
    const int T = small_team(c, false);
    const int grid = grid_rows((long)c.nown * T, c.G);
    double *fin = tmpfin_ptr() + TF_SPMM + cone;
    LRS_LAYOUT_SWITCH(c.G, c.E, {
        hipLaunchKernelGGL((k_spmm<GG, EE>), dim3(grid), dim3(kBlock), 0, st, c.nown, c.ld, c.adj_ptr, c.adj_col,
                           c.adj_slot, S, X + c.foff, scale, addX ? addX + c.foff : nullptr, addScale,
                           out + c.foff, part, ticket_ptr(T_SPMM), fin, c.row0, T);
    });
    LRS_CHECK_LAUNCH();
    if (nblk_used) *nblk_used = grid;
    return 0;
}

int launch_axpby(long n, double a, const double *x, double b, double *y, hipStream_t st) {
    hipLaunchKernelGGL(k_axpby, dim3(grid_elems(n, 4)), dim3(kBlock), 0, st, n, a, x, b, y);
    LRS_CHECK_LAUNCH();
    return 0;
}
int launch_fill(long n, double v, double *x, hipStream_t st) {
    hipLaunchKernelGGL(k_fill, dim3(grid_elems(n, 4)), dim3(kBlock), 0, st, n, v, x);
    LRS_CHECK_LAUNCH();
    return 0;
}
int launch_dot(long n, const double *x, const double *y, double *part, hipStream_t st, int *nblk_used, int fin) {
    const int grid = grid_elems(n, 8);
    hipLaunchKernelGGL(k_dot, dim3(grid), dim3(kBlock), 0, st, n, x, y, part, ticket_ptr(T_DOT),
                       tmpfin_ptr() + fin);
    LRS_CHECK_LAUNCH();
    if (nblk_used) *nblk_used = grid;
    return 0;
}
int launch_dual_update(const DevProblem &P, double rho, double *lam, const double *cvs, hipStream_t st) {
    hipLaunchKernelGGL(k_dual_update, dim3(grid_elems(P.m, 1)), dim3(kBlock), 0, st, P.m, rho, P.b, lam, cvs);
    LRS_CHECK_LAUNCH();
    return 0;
}
int launch_alm_m1(const DevProblem &P, double rho, const double *lam, const double *cvs, double *M1,
                  hipStream_t st) {
    hipLaunchKernelGGL(k_alm_m1, dim3(grid_elems(P.m, 1)), dim3(kBlock), 0, st, P.m, rho, P.b, lam, cvs, M1);
    LRS_CHECK_LAUNCH();
    return 0;
}
static int num_cus();
// the FP64 matrix-core ceiling the Gram is measured against (bench.py): back-to-back
// v_mfma_f64_16x16x4f64 on 8 independent accumulators, 2 waves a SIMD on every CU
// FP64 matrix-core probe: every wave issues `iters` rounds of CH independent
// v_mfma_f64_16x16x4f64 (no dependence between consecutive MFMAs of a round), blocks of one
// wave per SIMD, `wps` blocks per CU.  Block 0's wave 0 stamps the shader clock (s_memtime)
// and the 100 MHz wall clock at its start and end: the clock under load and, from it, the
// cycles one SIMD spends per MFMA (an MFMA rate, not a FLOP rate, independent of the clock).
template <int CH>
__global__ void __launch_bounds__(kBlock) k_mfma_peak(int iters, double *out, unsigned long long *clk) {
    gram_acc_t acc[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = gram_acc_t{0.0, 0.0, 0.0, 0.0};
    const double a = 1.0 + 1e-9 * threadIdx.x, b = 1.0 - 1e-9 * threadIdx.x;
    unsigned long long c0 = 0, w0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { c0 = __builtin_amdgcn_s_memtime(); w0 = wall_clock64(); }
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int k = 0; k < CH; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < CH; ++k) s += (acc[k][0] + acc[k][1]) + (acc[k][2] + acc[k][3]);
    out[(long)blockIdx.x * kBlock + threadIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0 && s != 12345.678) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), w1 = wall_clock64();
        clk[0] = c1 - c0;
        clk[1] = w1 - w0;
    }
}
// waves per SIMD wps (1..8 blocks of four waves per CU), chains CH in {4, 8}
int mfma_f64_probe(hipStream_t st, int wps, int chains, double *tflops, double *mhz, double *cyc_per_mfma) {
    const int blocks = std::max(1, std::min(8, wps)) * num_cus(), iters = 4000;
    double *out = nullptr;
    unsigned long long *clk = nullptr;
    hipEvent_t e0, e1;
    if (hipMalloc((void **)&out, sizeof(double) * blocks * kBlock) != hipSuccess ||
        hipMalloc((void **)&clk, 2 * sizeof(unsigned long long)) != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "mfma_f64_probe: hipMalloc");
        return -1;
    }
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto go = [&]() {
        if (chains <= 4) hipLaunchKernelGGL(k_mfma_peak<4>, dim3(blocks), dim3(kBlock), 0, st, iters, out, clk);
        else hipLaunchKernelGGL(k_mfma_peak<8>, dim3(blocks), dim3(kBlock), 0, st, iters, out, clk);
    };
    go();   // warm (clocks up)
    (void)hipEventRecord(e0, st);
    go();
    (void)hipEventRecord(e1, st);
    const hipError_t e = hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2] = {0, 0};
    (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(out);
    (void)hipFree(clk);
    if (e != hipSuccess || ms <= 0.f) {
        snprintf(g_err, sizeof(g_err), "mfma_f64_probe: %s", hipGetErrorString(e));
        return -1;
    }
    const int ch = chains <= 4 ? 4 : 8;
    const double flop = (double)blocks * (kBlock / 64) * iters * ch * 2048.0;
    *tflops = flop / (ms * 1e-3) / 1e12;
    const double wall_s = h[1] * 1e-8;   // 100 MHz
    if (mhz) *mhz = wall_s > 0 ? h[0] / wall_s / 1e6 : 0.0;
    // a SIMD runs one wave of each of its CU's blocks: its MFMA count over the launch, in
    // cycles of the measured clock
    const double per_simd = (double)blocks / num_cus() * iters * ch;
    if (cyc_per_mfma) *cyc_per_mfma = (mhz && *mhz > 0) ? ms * 1e-3 * (*mhz * 1e6) / per_simd : 0.0;
    return 0;
}
int mfma_f64_peak(hipStream_t st, double *tflops) { return mfma_f64_probe(st, 2, 8, tflops, nullptr, nullptr); }

// ---- dense objective on the FP64 matrix cores.  The reference's dense
// branches form sym(U V^T) in full (fds_syr2k, LORADSUVt lorads_alg_common.c:72-89) and multiply
// by a packed C (dataMatDenseMultiRkMat lorads_sdp_data.c:948-973); here C stays a full n x n
// row-major matrix and every C-term is a product with it: <C, sym R D^T> = <R, C D>,
// <C, D D^T> = <D, C D>, S R = (C + A^*(M1)) R = C R + A^*(M1) R.
// k_cgemm: Y = scale C X (+ beta Y) on the rows of one cone, X / Y row-major n x ld; C is the
// cone's row block of nr rows (row r0 + t of the cone: C row t, n columns; unsharded nr = n,
// r0 = 0; a shard: its owned rows, DevCone row0 / nown).  Output
// tiles of kCgBM rows x kCgBN columns, four waves as 2 x 2, a wave 16 rows x 32 columns (two
// v_mfma_f64_16x16x4f64 accumulators); C and X staged through double-buffered LDS tiles of
// kCgBK k-rows, the next tile's global loads issued before the current tile's MFMAs.  With
// `ctrl` (the ALM iteration): nothing when the iteration is inactive, X = D, and the block's
// partials <R, Y>, <X, Y> (R the current iterate) in slots 0 and 1 of stage A's 8.
constexpr int kCgBM = 32, kCgBN = 64, kCgBK = 32, kCgMaxGrid = 1024;
__global__ void __launch_bounds__(kBlock) k_cgemm(int n, int nr, int r0, int r, int ld, double scale,
                                                  const double *__restrict__ Cd, const double *__restrict__ X,
                                                  double *__restrict__ Y, double beta, const double *__restrict__ ctrl,
                                                  const double *__restrict__ Rb0, const double *__restrict__ Rb1,
                                                  double *__restrict__ part, int poff) {
    __shared__ double Cs[2][kCgBM][kCgBK + 1];
    __shared__ double Xs[2][kCgBK][kCgBN + 1];
    const double *__restrict__ R = nullptr;
    if (ctrl) {
        if (ctrl[C_ACTIVE] == 0.0) return;   // grid-uniform
        R = ctrl[C_RCUR] == 0.0 ? Rb0 : Rb1;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
    const int ntm = (nr + kCgBM - 1) / kCgBM, ntn = (r + kCgBN - 1) / kCgBN;
    const int nk = (n + kCgBK - 1) / kCgBK;
    // staging maps: C tile row t >> 3, k (t & 7) * 4 .. +3; X tile k-row t >> 3, columns (t & 7) * 8 .. +7
    const int crow = threadIdx.x >> 3, ck = (threadIdx.x & 7) * 4;
    const int xrow = threadIdx.x >> 3, xc = (threadIdx.x & 7) * 8;
    double dots[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int tile = blockIdx.x; tile < ntm * ntn; tile += gridDim.x) {
        const int m0 = (tile / ntn) * kCgBM, n0 = (tile % ntn) * kCgBN;
        gram_acc_t acc[2] = {gram_acc_t{0.0, 0.0, 0.0, 0.0}, gram_acc_t{0.0, 0.0, 0.0, 0.0}};
        double cr[4], xr[8];
        auto gload = [&](int k0) {
            const int gi = m0 + crow;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int gk = k0 + ck + t;
                cr[t] = (gi < nr && gk < n) ? Cd[(long)gi * n + gk] : 0.0;
            }
            const int gk = k0 + xrow;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int col = n0 + xc + t;
                xr[t] = (gk < n && col < r) ? X[(long)gk * ld + col] : 0.0;
            }
        };
        auto sstore = [&](int buf) {
#pragma unroll
            for (int t = 0; t < 4; ++t) Cs[buf][crow][ck + t] = cr[t];
#pragma unroll
            for (int t = 0; t < 8; ++t) Xs[buf][xrow][xc + t] = xr[t];
        };
        gload(0);
        sstore(0);
        __syncthreads();
        for (int kt = 0; kt < nk; ++kt) {
            const int cur = kt & 1;
            if (kt + 1 < nk) gload((kt + 1) * kCgBK);
#pragma unroll
            for (int ks = 0; ks < kCgBK / 4; ++ks) {
                const double a = Cs[cur][wm * 16 + (lane & 15)][ks * 4 + (lane >> 4)];
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const double b = Xs[cur][ks * 4 + (lane >> 4)][wn * 32 + t * 16 + (lane & 15)];
                    acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
                }
            }
            if (kt + 1 < nk) sstore(cur ^ 1);
            __syncthreads();
        }
        // D fragment: col = lane & 15, row = (lane >> 4) + 4 q
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = m0 + wm * 16 + (lane >> 4) + 4 * q;
                const int col = n0 + wn * 32 + t * 16 + (lane & 15);
                if (row < nr && col < r) {
                    const long o = (long)(r0 + row) * ld + col;
                    double v = scale * acc[t][q];
                    if (beta != 0.0) v += beta * Y[o];
                    Y[o] = v;
                    if (R) {
                        dots[0] += R[o] * v;
                        dots[1] += X[o] * v;
                    }
                }
            }
    }
    if (part) write_partials<8, kBlock>(dots, part, poff + blockIdx.x);
}
// constant objective C = alpha J (DevCone::dense_c == 2, Lovász theta's -J): Y = sa 1 (1^T X)
// (+ beta Y) with sa = scale alpha; one block of kCjThreads (the theta-class cones are small).
// Column sums: thread t takes column t % ld over rows t / ld, t / ld + G, ... (G = threads per
// column, four independent partial sums), then the G partials of a column are added in order:
// fixed summation order.  With `ctrl` as k_cgemm: X = D and the partials <R, Y>, <X, Y> in
// slots 0 and 1 of stage A's 8, at partial block `poff`.
constexpr int kCjThreads = 1024;
__global__ void __launch_bounds__(kCjThreads) k_cjx(int n, int r, int ld, double sa, const double *__restrict__ X,
                                                    double *__restrict__ Y, double beta, const double *__restrict__ ctrl,
                                                    const double *__restrict__ Rb0, const double *__restrict__ Rb1,
                                                    double *__restrict__ part, int poff) {
    __shared__ double ps[kCjThreads];
    __shared__ double cs[kMaxRankLd];
    const double *__restrict__ R = nullptr;
    if (ctrl) {
        if (ctrl[C_ACTIVE] == 0.0) return;
        R = ctrl[C_RCUR] == 0.0 ? Rb0 : Rb1;
    }
    const int G = kCjThreads / ld;   // ld <= kMaxRankLd = kCjThreads / 2
    const int c = threadIdx.x % ld, g = threadIdx.x / ld;
    if (g < G) {
        double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
        int i = g;
        for (; i + 3 * G < n; i += 4 * G) {
            t0 += X[(long)i * ld + c];
            t1 += X[(long)(i + G) * ld + c];
            t2 += X[(long)(i + 2 * G) * ld + c];
            t3 += X[(long)(i + 3 * G) * ld + c];
        }
        for (; i < n; i += G) t0 += X[(long)i * ld + c];
        ps[g * ld + c] = (t0 + t1) + (t2 + t3);
    }
    __syncthreads();
    for (int q = threadIdx.x; q < ld; q += kCjThreads) {
        double t = 0.0;
        if (q < r)
            for (int h = 0; h < G; ++h) t += ps[h * ld + q];
        cs[q] = sa * t;
    }
    __syncthreads();
    double dots[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const long tot = (long)n * ld;
    for (long t = threadIdx.x; t < tot; t += kCjThreads) {
        const int cc = (int)(t % ld);
        if (cc >= r) continue;
        double v = cs[cc];
        if (beta != 0.0) v += beta * Y[t];
        Y[t] = v;
        if (R) {
            dots[0] += R[t] * v;
            dots[1] += X[t] * v;
        }
    }
    if (part) write_partials<8, kCjThreads>(dots, part, poff);
}
// k_cgemm2: the same product as k_cgemm at full column width -- output tiles of kC2BM rows x
// kC2BN = 128 columns (a wave 16 x 64: four 16 x 16 MFMA accumulators off one A fragment), so
// C streams from HBM once per 128 factor columns instead of once per 64 -- and split over K:
// block (tile, s) sums k-tiles [s K / S, (s + 1) K / S) into the scratch slab s (raw sums),
// k_cgemm2_fin adds the S slabs in slab order (deterministic), scales, applies beta and takes
// the objective dots.  S = 1: the epilogue is fused (no scratch).  X's LDS rows are padded to
// 144 doubles so the two k-rows of a ds_read_b64 lane group sit 32 banks apart; C's to 17.
constexpr int kC2BM = 32, kC2BN = 128, kC2BK = 16, kC2XS = 144, kCgSplitMax = kCgSplitSlabs;
template <bool SPLIT>
__global__ void __launch_bounds__(kBlock) k_cgemm2(int n, int nr, int r0, int r, int ld, double scale,
                                                   const double *__restrict__ Cd, const double *__restrict__ X,
                                                   double *__restrict__ Y, double beta, const double *__restrict__ ctrl,
                                                   const double *__restrict__ Rb0, const double *__restrict__ Rb1,
                                                   double *__restrict__ part, int poff, int S,
                                                   double *__restrict__ Pk) {
    __shared__ double Cs[2][kC2BM][kC2BK + 1];
    __shared__ double Xs[2][kC2BK][kC2XS];
    const double *__restrict__ R = nullptr;
    if (ctrl) {
        if (ctrl[C_ACTIVE] == 0.0) return;   // grid-uniform
        R = ctrl[C_RCUR] == 0.0 ? Rb0 : Rb1;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
    const int ntm = (nr + kC2BM - 1) / kC2BM, ntn = (r + kC2BN - 1) / kC2BN;
    const int nk = (n + kC2BK - 1) / kC2BK, kper = (nk + S - 1) / S;
    // staging maps: C tile row t >> 3, k (t & 7) * 2 .. +1; X tile k-row t >> 4, columns (t & 15) * 8 .. +7
    const int crow = threadIdx.x >> 3, ck = (threadIdx.x & 7) * 2;
    const int xrow = threadIdx.x >> 4, xc = (threadIdx.x & 15) * 8;
    double dots[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int item = blockIdx.x; item < ntm * ntn * S; item += gridDim.x) {
        const int tile = item / S, sk = item - tile * S;
        const int m0 = (tile / ntn) * kC2BM, n0 = (tile % ntn) * kC2BN;
        const int kt0 = sk * kper, kt1 = min(nk, kt0 + kper);
        gram_acc_t acc[4] = {gram_acc_t{0.0, 0.0, 0.0, 0.0}, gram_acc_t{0.0, 0.0, 0.0, 0.0},
                             gram_acc_t{0.0, 0.0, 0.0, 0.0}, gram_acc_t{0.0, 0.0, 0.0, 0.0}};
        double cr[2];
        double2 xr[4];
        auto gload = [&](int k0) {
            const int gi = m0 + crow;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int gk = k0 + ck + t;
                cr[t] = (gi < nr && gk < n) ? Cd[(long)gi * n + gk] : 0.0;
            }
            const int gk = k0 + xrow, col = n0 + xc;
            const bool ok = gk < n && col < ld;   // padded columns are zero in the factor layout
            const double2 *xp = reinterpret_cast<const double2 *>(X + (long)(ok ? gk : 0) * ld + (ok ? col : 0));
#pragma unroll
            for (int t = 0; t < 4; ++t) xr[t] = ok ? xp[t] : make_double2(0.0, 0.0);
        };
        auto sstore = [&](int buf) {
#pragma unroll
            for (int t = 0; t < 2; ++t) Cs[buf][crow][ck + t] = cr[t];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                Xs[buf][xrow][xc + 2 * t] = xr[t].x;
                Xs[buf][xrow][xc + 2 * t + 1] = xr[t].y;
            }
        };
        if (kt0 < kt1) {
            gload(kt0 * kC2BK);
            sstore(0);
        }
        __syncthreads();
        for (int kt = kt0; kt < kt1; ++kt) {
            const int cur = (kt - kt0) & 1;
            if (kt + 1 < kt1) gload((kt + 1) * kC2BK);
#pragma unroll
            for (int ks = 0; ks < kC2BK / 4; ++ks) {
                const double a = Cs[cur][wm * 16 + (lane & 15)][ks * 4 + (lane >> 4)];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const double b = Xs[cur][ks * 4 + (lane >> 4)][wn * 64 + t * 16 + (lane & 15)];
                    acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
                }
            }
            if (kt + 1 < kt1) sstore(cur ^ 1);
            __syncthreads();
        }
        // D fragment: col = lane & 15, row = (lane >> 4) + 4 q
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = m0 + wm * 16 + (lane >> 4) + 4 * q;
                const int col = n0 + wn * 64 + t * 16 + (lane & 15);
                if (row < nr && col < r) {
                    if (SPLIT) {
                        Pk[((long)sk * nr + row) * ld + col] = acc[t][q];
                    } else {
                        const long o = (long)(r0 + row) * ld + col;
                        double v = scale * acc[t][q];
                        if (beta != 0.0) v += beta * Y[o];
                        Y[o] = v;
                        if (R) {
                            dots[0] += R[o] * v;
                            dots[1] += X[o] * v;
                        }
                    }
                }
            }
    }
    if (!SPLIT && part) write_partials<8, kBlock>(dots, part, poff + blockIdx.x);
}
// the S slabs of k_cgemm2<true> in slab order -> Y (scale, beta) and the objective dots
__global__ void __launch_bounds__(kBlock) k_cgemm2_fin(int nr, int r0, int r, int ld, int S, double scale,
                                                       const double *__restrict__ Pk, const double *__restrict__ X,
                                                       double *__restrict__ Y, double beta,
                                                       const double *__restrict__ ctrl, const double *__restrict__ Rb0,
                                                       const double *__restrict__ Rb1, double *__restrict__ part,
                                                       int poff) {
    const double *__restrict__ R = nullptr;
    if (ctrl) {
        if (ctrl[C_ACTIVE] == 0.0) return;
        R = ctrl[C_RCUR] == 0.0 ? Rb0 : Rb1;
    }
    double dots[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const long tot = (long)nr * ld;
    for (long t = (long)blockIdx.x * kBlock + threadIdx.x; t < tot; t += (long)gridDim.x * kBlock) {
        const int col = (int)(t % ld);
        if (col >= r) continue;
        double a = Pk[t];
        for (int q = 1; q < S; ++q) a += Pk[(long)q * tot + t];
        const long o = (long)r0 * ld + t;
        double v = scale * a;
        if (beta != 0.0) v += beta * Y[o];
        Y[o] = v;
        if (R) {
            dots[0] += R[o] * v;
            dots[1] += X[o] * v;
        }
    }
    if (part) write_partials<8, kBlock>(dots, part, poff + blockIdx.x);
}
// Which product a dense cone takes: k_cgemm2 for cones of at least kC2MinN rows (C5b-size:
// C streamed once per 128 columns, split over K to fill the chip), k_cgemm below (theta-size:
// one launch of small tiles).  S from the tile count (about 3 blocks per CU), LRS_CG_SPLIT.
constexpr int kC2MinN = 2048, kC2FinGrid = 512;
struct CgPlan { bool big; int S, grid, fin_grid; };
static CgPlan cg_plan(const DevCone &c, bool scratch) {
    CgPlan p{false, 1, 0, 0};
    if (c.n < kC2MinN || getenv("LRS_CG_OLD")) return p;
    p.big = true;
    const long tiles = (long)((c.nown + kC2BM - 1) / kC2BM) * ((c.r + kC2BN - 1) / kC2BN);
    static int env = -2;
    if (env == -2) { const char *e = getenv("LRS_CG_SPLIT"); env = e ? atoi(e) : -1; }
    int S = env > 0 ? env : (int)std::max(1L, std::min((long)kCgSplitMax, (1536 + tiles - 1) / tiles));
    if (!scratch) S = 1;
    p.S = std::max(1, std::min(kCgSplitMax, S));
    p.grid = (int)std::min((long)kMaxPartialBlocks, tiles * p.S);
    p.fin_grid = p.S > 1 ? kC2FinGrid : 0;
    return p;
}
static int cgemm_grid(const DevCone &c) {
    const long tiles = (long)((c.nown + kCgBM - 1) / kCgBM) * ((c.r + kCgBN - 1) / kCgBN);
    return (int)std::max(1L, std::min((long)kCgMaxGrid, tiles));
}
int launch_dense_cx(const DevProblem &P, int cone, const double *X, double *Y, double beta, hipStream_t st) {
    const DevCone &c = P.cones[cone];
    if (!c.dense_c) return 0;
    if (c.dense_c == 2 && c.nown != c.n) {
        snprintf(g_err, sizeof(g_err), "constant objective: sharded cones take the slot path");
        return -1;
    }
    if (c.dense_c == 2) {
        hipLaunchKernelGGL(k_cjx, dim3(1), dim3(kCjThreads), 0, st, c.n, c.r, c.ld, P.dense_scale * c.c_alpha, X + c.foff,
                           Y + c.foff, beta, nullptr, nullptr, nullptr, nullptr, 0);
        LRS_CHECK_LAUNCH();
        return 0;
    }
    const CgPlan cp = cg_plan(c, P.cgk != nullptr);
    if (cp.big && cp.S > 1) {
        hipLaunchKernelGGL((k_cgemm2<true>), dim3(cp.grid), dim3(kBlock), 0, st, c.n, c.nown, c.row0, c.r, c.ld,
                           P.dense_scale, c.Cd, X + c.foff, Y + c.foff, beta, nullptr, nullptr, nullptr, nullptr, 0,
                           cp.S, P.cgk);
        LRS_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_cgemm2_fin, dim3(cp.fin_grid), dim3(kBlock), 0, st, c.nown, c.row0, c.r, c.ld, cp.S,
                           P.dense_scale, P.cgk, X + c.foff, Y + c.foff, beta, nullptr, nullptr, nullptr, nullptr, 0);
    } else if (cp.big) {
        hipLaunchKernelGGL((k_cgemm2<false>), dim3(cp.grid), dim3(kBlock), 0, st, c.n, c.nown, c.row0, c.r, c.ld,
                           P.dense_scale, c.Cd, X + c.foff, Y + c.foff, beta, nullptr, nullptr, nullptr, nullptr, 0, 1,
                           nullptr);
    } else {
        hipLaunchKernelGGL(k_cgemm, dim3(cgemm_grid(c)), dim3(kBlock), 0, st, c.n, c.nown, c.row0, c.r, c.ld,
                           P.dense_scale, c.Cd, X + c.foff, Y + c.foff, beta, nullptr, nullptr, nullptr, nullptr, 0);
    }
    LRS_CHECK_LAUNCH();
    return 0;
}
int dense_cd_blocks(const DevProblem &P) {
    int nb = 0;
    for (const DevCone &c : P.cones) {
        if (!c.dense_c) continue;
        if (c.dense_c == 2) { nb += 1; continue; }
        const CgPlan cp = cg_plan(c, P.cgk != nullptr);
        nb += !cp.big ? cgemm_grid(c) : (cp.S > 1 ? cp.fin_grid : cp.grid);
    }
    return nb;
}
int launch_dense_cd(const DevProblem &P, const DevWork &W, const double *ctrl, int off, hipStream_t st) {
    for (const DevCone &c : P.cones) {
        if (!c.dense_c) continue;
        if (c.dense_c == 2) {
            hipLaunchKernelGGL(k_cjx, dim3(1), dim3(kCjThreads), 0, st, c.n, c.r, c.ld, P.dense_scale * c.c_alpha,
                               W.D + c.foff, W.CD + c.foff, 0.0, ctrl, W.R + c.foff, W.R2 + c.foff, W.part, off);
            LRS_CHECK_LAUNCH();
            off += 1;
            continue;
        }
        const CgPlan cp = cg_plan(c, P.cgk != nullptr);
        if (cp.big && cp.S > 1) {
            hipLaunchKernelGGL((k_cgemm2<true>), dim3(cp.grid), dim3(kBlock), 0, st, c.n, c.nown, c.row0, c.r, c.ld,
                               P.dense_scale, c.Cd, W.D + c.foff, W.CD + c.foff, 0.0, ctrl, nullptr, nullptr, nullptr,
                               0, cp.S, P.cgk);
            LRS_CHECK_LAUNCH();
            hipLaunchKernelGGL(k_cgemm2_fin, dim3(cp.fin_grid), dim3(kBlock), 0, st, c.nown, c.row0, c.r, c.ld, cp.S,
                               P.dense_scale, P.cgk, W.D + c.foff, W.CD + c.foff, 0.0, ctrl, W.R + c.foff,
                               W.R2 + c.foff, W.part, off);
            off += cp.fin_grid;
        } else if (cp.big) {
            hipLaunchKernelGGL((k_cgemm2<false>), dim3(cp.grid), dim3(kBlock), 0, st, c.n, c.nown, c.row0, c.r, c.ld,
                               P.dense_scale, c.Cd, W.D + c.foff, W.CD + c.foff, 0.0, ctrl, W.R + c.foff,
                               W.R2 + c.foff, W.part, off, 1, nullptr);
            off += cp.grid;
        } else {
            const int grid = cgemm_grid(c);
            hipLaunchKernelGGL(k_cgemm, dim3(grid), dim3(kBlock), 0, st, c.n, c.nown, c.row0, c.r, c.ld, P.dense_scale,
                               c.Cd, W.D + c.foff, W.CD + c.foff, 0.0, ctrl, W.R + c.foff, W.R2 + c.foff, W.part, off);
            off += grid;
        }
        LRS_CHECK_LAUNCH();
    }
    return 0;
}

// register blocking of the Gram: NB x NB tiles per wave (16 NB columns a side)
static int gram_nb(int r) { return r > 16 ? 2 : 1; }
static long gram_subtiles(int r, int nb) {
    const long nbc = (r + 16 * nb - 1) / (16 * nb);
    return nbc * (nbc + 1) / 2 * nb * nb;
}
size_t gram_buf_len(int rmax) {
    long sub = 0;
    for (int nb = 1; nb <= 4; nb *= 2) sub = std::max(sub, gram_subtiles(rmax, nb));
    return (size_t)rmax * rmax + (size_t)kGramMaxChunks * sub * 256;
}
int launch_gram(const DevProblem &P, int cone, const double *X, const double *Y, int avg, double *gram,
                int *nblk_used, hipStream_t st, bool reduce) {
    const DevCone &c = P.cones[cone];
    if (c.r > 512) {
        snprintf(g_err, sizeof(g_err), "gram: rank %d above 512", c.r);
        return -1;
    }
    int nb = gram_nb(c.r);
#ifdef LRS_GRAM_DIAG
    if (getenv("LRS_GRAM_NB")) nb = atoi(getenv("LRS_GRAM_NB"));
#endif
    const int nbc = (c.r + 16 * nb - 1) / (16 * nb);
    const int npair = nbc * (nbc + 1) / 2;
    // row chunks: a multiple of 8 (chunk x's pairs share an XCD), >= 64 rows each, at most
    // kGramMaxChunks (the partial buffer), about 1024 workgroups in all (the partials' bytes
    // grow with the chunk count)
    int gx = std::max(1, std::min({kGramMaxChunks, (c.nown + 63) / 64, std::max(8, 1024 / npair)}));
#ifdef LRS_GRAM_DIAG
    if (getenv("LRS_GRAM_C")) gx = std::min(gx, atoi(getenv("LRS_GRAM_C")));
#endif
    if (gx >= 8) gx &= ~7;
    const double *Xs = X + c.foff + (long)c.row0 * c.ld;
    const double *Ys = Y ? Y + c.foff + (long)c.row0 * c.ld : nullptr;
    double *part = gram + (long)c.r * c.r;
    const dim3 grid(gx, npair);
#define LRS_GRAM_GO(NB_, U_)                                                                                      \
    do {                                                                                                          \
        if (avg)                                                                                                  \
            hipLaunchKernelGGL((k_gram<NB_, U_, true>), grid, dim3(kBlock), 0, st, c.nown, c.r, c.ld, nbc, Xs, Ys,  \
                               part);                                                                             \
        else                                                                                                      \
            hipLaunchKernelGGL((k_gram<NB_, U_, false>), grid, dim3(kBlock), 0, st, c.nown, c.r, c.ld, nbc, Xs, Ys, \
                               part);                                                                             \
    } while (0)
    if (nb == 4) LRS_GRAM_GO(4, 2);
    else if (nb == 2 && (c.nown + 16L * gx - 1) / (16L * gx) <= 12) LRS_GRAM_GO(2, 4);   // <= 12 k-steps a wave
    else if (nb == 2) LRS_GRAM_GO(2, 8);
    else LRS_GRAM_GO(1, 8);
#undef LRS_GRAM_GO
    LRS_CHECK_LAUNCH();
    if (!reduce) return 0;
    hipLaunchKernelGGL(k_gram_fin, dim3(npair * nb * nb * 4), dim3(kGramFinThreads), 0, st, c.r, nb, nbc, gx, part,
                       gram);
    LRS_CHECK_LAUNCH();
    if (nblk_used) *nblk_used = gx;
    return 0;
}

// Row-kernel grids of the split iteration, sized from the occupancy query: a stage
// launches min(rows' lane groups, blocks resident on the whole chip).  When one
// resident wave of groups covers every row (latency regime, small n) the neighbour
// loops are unrolled so that their gathers overlap; otherwise (bandwidth regime) the
// unroll-1 variant keeps registers low and occupancy high, and groups stride over rows.
static int num_cus() {
    static int cus[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    if (cus[dev] <= 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        cus[dev] = v;
    }
    return cus[dev];
}
template <typename KernelT>
static int resident_blocks(KernelT kern, int *cache, int nt = kRowBlock) {
    if (*cache <= 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void *>(kern), nt, 0) !=
                hipSuccess || nb < 1)
            nb = 1;
        *cache = nb * num_cus();
    }
    return *cache;
}
// Stage A as ONE launch in the bandwidth regime (k_it_a<., ., 1, 0>: the lower neighbours' D
// recomputed from G and the pairs instead of written by a first launch and read back by a second)
// on plain rows (T = 1, not the long-row kernels), unsharded, while a factor is at most 32 MB:
// the neighbours' five operand rows then come from L2 / the Infinity Cache.  G81 r = 64 (10 MB
// factors): stage A 35.7 -> 31.6-32.2 us, 14.6K -> 15.6-15.8K it/s; the 2000^2 torus (512 MB
// factors) 1 240 -> 1 551 us, so it stays split (profiles/r06m_stage_a_fused_ab.txt).
// LRS_A_FUSED=0 / 1 forces it off / on (where the rows allow).
static int a_fused_env() {
    static int v = -2;
    if (v == -2) {
        const char *e = getenv("LRS_A_FUSED");
        v = !e ? -1 : (e[0] == '1' ? 1 : 0);
    }
    return v;
}
constexpr long kAFusedMaxFactor = 32L << 20;   // bytes of one factor (n x ld doubles)
static bool a_fused_rows(const DevCone &c, int T, bool wide_rows, bool sharded) {
    if (sharded || wide_rows || T != 1) return false;
    const int e = a_fused_env();
    return e >= 0 ? e == 1 : 8L * c.nown * c.ld <= kAFusedMaxFactor;
}
template <int GG, int EE, int UU>
static int res_a(bool fused = false) {
    static int c = 0, c0 = 0;
    if constexpr (UU == 1) {
        // bandwidth regime: the split halves (MODE 1 / 2), or the fused launch (MODE 0)
        const int r = resident_blocks(k_it_a<GG, EE, 1, 2>, &c);
        return fused ? std::min(r, resident_blocks(k_it_a<GG, EE, 1, 0>, &c0)) : r;
    }
    return resident_blocks(k_it_a<GG, EE, UU, UU == 1 ? 2 : 0>, &c);
}
// k_bw_b (the bandwidth regime's fused stage B on plain rows); LRS_BW_B=0: k_it_b<., ., 1, 0>
static bool bw_b_on() {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("LRS_BW_B");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    return v != 0;
}
template <int GG, int EE, int UU>
static int res_b(bool fused = false) {
    static int c = 0;
    if constexpr (UU == 1) {
        // the bandwidth regime's grid: a fused stage B (one launch, not sharded) runs k_bw_b or
        // k_it_b MODE 0, a split one k_it_b MODE 1 / 2 (or the long-row kernels); the fused
        // kernels' smaller residency, so that no block waits for a second round
        static int c0 = 0, c1 = 0;
        const int r = resident_blocks(k_it_b<GG, EE, 1, 2>, &c);
        if (!fused) return r;
        const int r0 = std::min(r, resident_blocks(k_it_b<GG, EE, LRS_BW_UB, 0>, &c0));
        return bw_b_on() ? std::min(r0, resident_blocks(k_bw_b<GG, EE, kBwNo>, &c1)) : r0;
    }
    return resident_blocks(k_it_b<GG, EE, UU, (UU == 1 ? 2 : 0)>, &c);
}

constexpr int kWideU = 8;   // factor rows in flight per lane group in k_wide_a / k_wide_b
struct StagePlan {
    int grid = 1;
    bool small = true;
    int T = 1;         // lane groups per row (team)
    bool wide = false; // bandwidth regime, long rows: the neighbour half unrolled by 4 (more
                       // gathers in flight per lane group; E <= 2 keeps the registers low)
    bool afused = false;   // bandwidth regime, stage A as one MODE 0 launch (a_fused_rows)
};
// Team size for rows of average degree `deg`: split a row's neighbour list over T lane
// groups while every group still gets two unrolled chunks and the chip is not
// oversubscribed (dense rows, e.g. the Lovasz theta objective, n ~ 100s).
static int team_size(const DevCone &c, double deg, int U) {
    // largest power of two with at least one full U-unrolled round of entries per member
    // (theta3's 150-entry rows: T = 16, stages A/B 13.6/17.1 -> 12.0/13.7 us against T = 8)
    const long cap_threads = 256L * 2048;
    int T = 1;
    while (T * 2 <= kRowBlock / c.G && (double)(T * 2 * U) <= deg && (long)c.nown * T * 2 * c.G <= cap_threads)
        T *= 2;
    return T;
}
// LRS_FORCE_REGIME=small|large overrides the choice (tests run the bandwidth-regime code
// paths on small instances that way)
static int forced_regime() {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("LRS_FORCE_REGIME");
        v = !e ? 0 : (strcmp(e, "small") == 0 ? 1 : (strcmp(e, "large") == 0 ? 2 : 0));
    }
    return v;
}
// force: the context's kernel path (lrs_set_kernel_path): >= 2 forces the bandwidth regime
// neighbours in flight per lane group in the bandwidth regime's second halves (MODE 2)
#ifndef LRS_BW_U
#define LRS_BW_U 1
#endif
constexpr int kBwU = LRS_BW_U;
static StagePlan plan_stage(long rows_threads, int res_small, int res_large, int K, int T, int force) {
    StagePlan p;
    p.T = T;
    const long need = std::max(1L, (rows_threads * T + kRowBlock - 1) / kRowBlock);
    const int cap = std::max(1, kMaxPartialBlocks / std::max(1, K));
    const int fr = force >= 2 ? 2 : forced_regime();
    if (fr == 2) { p.grid = (int)std::max(1L, std::min<long>(std::min<long>(need, res_large), cap)); p.small = false; return p; }
    if (fr == 1) { p.grid = (int)std::max(1L, std::min<long>(need, cap)); p.small = true; return p; }
    if (need <= res_small) { p.grid = (int)std::min<long>(need, cap); p.small = true; }
    else { p.grid = (int)std::min<long>(std::min<long>(need, res_large), cap); p.small = false; }
    p.grid = std::max(1, p.grid);
    return p;
}
// force == 3 (lrs_set_kernel_path): the long-row neighbour kernels k_wide_a / k_wide_b on
// every row the layout allows (tests run them on short rows that way)
static int plan_a(const DevCone &c, int K, StagePlan &p, int force, bool sharded) {
    const double deg = c.nown > 0 ? (double)c.P / c.nown : 0.0;    // lower entries per row
    const int T = team_size(c, deg, 2);
    const bool wide_rows = (deg / T >= 32.0 || force == 3) && c.E <= 2;   // p.wide below, but for the grid
    const bool fused = a_fused_rows(c, T, wide_rows, sharded);
    LRS_LAYOUT_SWITCH(c.G, c.E, {
        p = plan_stage((long)c.nown * c.G, res_a<GG, EE, 2>(), res_a<GG, EE, 1>(fused), K, T, force);
    });
    p.wide = !p.small && wide_rows;
    p.afused = !p.small && fused;
    return 0;
}
static int plan_b(const DevCone &c, int K, StagePlan &p, int force, bool fused) {
    const double deg = c.nown > 0 ? (double)c.adj_nnz / c.nown : 0.0;
    const int T = team_size(c, deg, 4);
    const bool wide_rows = (deg / T >= 64.0 || force == 3) && c.E <= 2;   // p.wide below, but for the grid
    LRS_LAYOUT_SWITCH(c.G, c.E, {
        p = plan_stage((long)c.nown * c.G, res_b<GG, EE, 4>(), res_b<GG, EE, 1>(fused && !wide_rows), K, T, force);
    });
    p.wide = !p.small && (deg / T >= 64.0 || force == 3) && c.E <= 2;
    return 0;
}

// Latency-regime kernels (k_lat_a / k_lat_b): one row per lane group, every group
// resident, no teams (T == 1), and each stage's producer partials within one control
// wave's reach.  NB (prefetched entries) from the most entries of one row.
constexpr int kLatNoA = 2, kLatNoB = 4;   // off-diagonal entries prefetched (A: lower, B: all)
template <int GG, int EE>
static int res_la() {
    static int c = 0;
    return resident_blocks(k_lat_a<GG, EE, kLatNoA>, &c, kLatNT);
}
template <int GG, int EE>
static int res_lb() {
    static int c = 0;
    return resident_blocks(k_lat_b<GG, EE, kLatNoB>, &c, kLatNT);
}
static bool lat_disabled() {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("LRS_NO_LAT");
        v = (e && atoi(e) != 0) ? 1 : 0;
    }
    return v != 0;
}
// Launch plan of the latency kernels for one cone: nrb row blocks (one row per lane group),
// then sa / sb slice blocks over the dense rows' entries (A: lower, B: all) and nf k_lat_f
// blocks.  nrb == 0: they do not apply.
struct LatPlan {
    int nrb = 0, sa = 0, sb = 0, nf = 0, nt = kLatNT;   // nt: threads a block (w row waves + 1)
};
static int lat_slices(const std::vector<int> &cnt, int per) {
    int s = 0;
    for (int x : cnt) s += (x + per - 1) / per;
    return s;
}
static int lat_resident(const DevCone &c, int &ra, int &rb) {
    LRS_LAYOUT_SWITCH(c.G, c.E, { ra = (res_la<GG, EE>)(); rb = (res_lb<GG, EE>)(); });
    return 0;
}
static LatPlan lat_plan(const DevCone &c, const StagePlan &pa, const StagePlan &pb, int w = kLatRowWaves) {
    LatPlan lp;
    if (lat_disabled() || forced_regime() == 2 || c.maxdeg <= 0 || !pa.small || !pb.small || pa.T != 1 || pb.T != 1)
        return lp;
    if ((int)c.dra_h.size() > kMaxDenseRows || (int)c.drb_h.size() > kMaxDenseRows) return lp;
    const int rows = 64 * w;   // row-wave threads a block
    const long need = std::max(1L, ((long)c.nown * c.G + rows - 1) / rows);
    const int sa = lat_slices(c.dra_n, (rows / c.G) * kSliceA);
    const int sb = lat_slices(c.drb_n, (rows / c.G) * kSliceB);
    int ra = 0, rb = 0;
    if (lat_resident(c, ra, rb)) return lp;
    if (need + sa > ra || need + sb > rb || need + sa > kLatMaxPartials) return lp;
    if (need + sb + (long)c.drb_h.size() > kLatMaxPartials) return lp;
    lp.nrb = (int)need;
    lp.sa = sa;
    lp.sb = sb;
    lp.nf = (int)c.drb_h.size();
    lp.nt = 64 * (w + 1);
    return lp;
}
// LRS_LAT_ROWWAVES = 1..7 forces the row waves per latency block (0: chosen per launch)
static int lat_forced_waves() {
    static int forced = -1;
    if (forced < 0) {
        const char *e = getenv("LRS_LAT_ROWWAVES");
        forced = e ? std::max(0, std::min(kLatRowWaves, atoi(e))) : 0;
    }
    return forced;
}

// the multi-launch kernel family forced by lrs_set_kernel_path (4, the single-workgroup inner
// loop, counts as auto here: where that kernel does not fit, the iteration runs as with 0)
static int multi_path(const DevProblem &P) { return P.no_lat == 4 ? 0 : P.no_lat; }

// Whether stage A runs as two launches (bandwidth regime) for the current layouts.
bool alm_stage_a_split(const DevProblem &P) {
    for (int k = 0; k < P.K; ++k) {
        StagePlan pa;
        if (plan_a(P.cones[k], P.K, pa, multi_path(P), P.shard != nullptr)) return false;
        if (!pa.small && !pa.afused) return true;
    }
    return false;
}

// Stage B in the bandwidth regime on the plain row kernel (not the long-row / tiled kernels,
// not sharded): ONE launch (k_it_b MODE 0: every block's line search from the stage-A / G
// partials, the neighbours' R_new = R + tau D recomputed per entry) instead of the two of the
// split form (R_new written by the first, read back by the second).  G81-like r = 64: 14.5K ->
// 15.2K it/s; 2000^2 torus +2 % (profiles/r05zk_bfused_ab.txt).  LRS_B_FUSED=0: the split form.
static bool b_fused_on() {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("LRS_B_FUSED");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    return v != 0;
}
// Whether stage B runs as two launches (bandwidth regime).
bool alm_stage_b_split(const DevProblem &P) {
    for (int k = 0; k < P.K; ++k) {
        StagePlan pb;
        if (plan_b(P.cones[k], P.K, pb, multi_path(P), !P.shard && b_fused_on())) return false;
        if (!pb.small && (pb.wide || P.shard || !b_fused_on())) return true;
    }
    return false;
}

// One ALM inner iteration = two launches (A, B), three with global constraints
// (A, G, B).  Parity selects the control buffers.
int enqueue_alm_iteration(const AlmIterArgs &a, int parity, hipStream_t st) {
    return enqueue_alm_stages(a, parity, 7, st);
}

// Sharded solve: one block folds a stage's per-block partials (fixed order) into NV
// contiguous totals, which the shards then sum (ShardHooks::allreduce); the next stage
// reads the totals as a single "block" with stride 1.
template <int NV, int NT = kRowBlock>
__global__ void __launch_bounds__(NT) k_fold_partials(const double *__restrict__ part, int nblk,
                                                      double *__restrict__ out) {
    // the consumers' own reduction tree (reduce_partials<NV, NT>: the row kernels' kRowBlock, the
    // CG kernels' kBlock): a total read back by a consumer is bitwise the sum that consumer would
    // have formed from the partials
    __shared__ double red[NV];
    reduce_partials<NV, NT>(part, nblk, red);
    if (threadIdx.x < NV) out[threadIdx.x] = red[threadIdx.x];
}
// sharded: an m-vector's shared entries summed over the shards (the holders' partial sums of
// A(.) over their owned entries)
int sync_shared(const DevProblem &P, double *v, hipStream_t st) {
    if (!P.shard || P.nsh == 0) return 0;
    const ShardHooks *sh = P.shard;
    hipLaunchKernelGGL(k_fill, dim3(grid_elems(P.nsh, 4)), dim3(kBlock), 0, st, (long)P.nsh, 0.0, P.spack);
    hipLaunchKernelGGL(k_pack_shared, dim3(grid_elems(P.m, 1)), dim3(kBlock), 0, st, P.m, P.sh_idx, v, P.spack, 0);
    LRS_CHECK_LAUNCH();
    if (sh->allreduce(sh->self, P.spack, P.nsh, st)) return -1;
    hipLaunchKernelGGL(k_pack_shared, dim3(grid_elems(P.m, 1)), dim3(kBlock), 0, st, P.m, P.sh_idx, v, P.spack, 1);
    LRS_CHECK_LAUNCH();
    return 0;
}
// the inner loop's parameters and control block into device memory as kernel arguments: one
// queued launch instead of two host-to-device copies (each a DMA / blit round trip the host
// waits on before the first iteration of a run_inner call can start)
struct CtrlPut { double v[P_NPAR + C_NCTRL]; };
__global__ void k_put_ctrl(CtrlPut c, double *__restrict__ par, double *__restrict__ ctl) {
    const int t = threadIdx.x;
    if (t < P_NPAR) par[t] = c.v[t];
    if (t < C_NCTRL) ctl[t] = c.v[P_NPAR + t];
}
int launch_put_ctrl(const double *par, const double *ctl, double *dpar, double *dctl, hipStream_t st) {
    CtrlPut c;
    for (int q = 0; q < P_NPAR; ++q) c.v[q] = par[q];
    for (int q = 0; q < C_NCTRL; ++q) c.v[P_NPAR + q] = ctl[q];
    hipLaunchKernelGGL(k_put_ctrl, dim3(1), dim3(64), 0, st, c, dpar, dctl);
    LRS_CHECK_LAUNCH();
    return 0;
}

// one scalar's partials (the sharded CG's <p, Q>, <r, r>, ||b||_1) -> out[0]
int launch_fold1(const double *part, int nblk, double *out, hipStream_t st) {
    hipLaunchKernelGGL((k_fold_partials<1, kBlock>), dim3(1), dim3(kBlock), 0, st, part, nblk, out);
    LRS_CHECK_LAUNCH();
    return 0;
}

int enqueue_alm_stages(const AlmIterArgs &a, int parity, int mask, hipStream_t st) {
    const DevProblem &P = *a.P;
    DevWork &W = *a.W;
    double *ctrl_prev = W.ctrl + (parity ^ 1) * C_NCTRL;
    double *ctrl_cur = W.ctrl + parity * C_NCTRL;
    double *ls_prev = W.lsres + (parity ^ 1) * LS_N;
    double *ls_cur = W.lsres + parity * LS_N;
    const int L = 2;
    const ShardHooks *sh = P.shard;
    if (sh && !W.tot) {
        snprintf(g_err, sizeof(g_err), "sharded iteration: no totals buffer");
        return -1;
    }
    // one launch over the merged row space when every cone has the same row layout (not in a
    // sharded solve: a shard's owned rows are a range per cone)
    bool merge = P.K > 1 && P.has_merged && !sh;
    for (int k = 1; k < P.K && merge; ++k)
        merge = P.cones[k].G == P.cones[0].G && P.cones[k].E == P.cones[0].E && P.cones[k].ld == P.cones[0].ld;
    DevCone mc;
    if (merge) {
        mc = P.merged;
        mc.G = P.cones[0].G; mc.E = P.cones[0].E; mc.ld = P.cones[0].ld; mc.r = P.cones[0].r;
        mc.foff = 0;
    }
    const int KL = merge ? 1 : P.K;                       // launches per stage
    auto cone_of = [&](int k) -> const DevCone & { return merge ? mc : P.cones[k]; };
    StagePlan pa[kMaxCones], pb[kMaxCones];
    int nblkA = 0, nblkB = 0;
    bool split = sh != nullptr;   // stage A as two launches (bandwidth regime; always when sharded)
    for (int k = 0; k < KL; ++k) {
        if (plan_a(cone_of(k), KL, pa[k], multi_path(P), sh != nullptr) ||
            plan_b(cone_of(k), KL, pb[k], multi_path(P), !sh && b_fused_on()))
            return -1;
        nblkA += pa[k].grid;
        nblkB += pb[k].grid;
        if (!pa[k].small && !pa[k].afused) split = true;
    }
    // long-row kernels in column tiles (k_wide_a / k_wide_b TL): the cone's column segments and
    // the partial-gradient buffer exist, one cone per launch, not sharded; B adds k_wide_bf's blocks
    bool tla[kMaxCones], tlb[kMaxCones];
    auto bfused = [&](const StagePlan &pl, bool tiled) { return b_fused_on() && !sh && !pl.small && !pl.wide && !tiled; };
    int offBF = nblkB;
    for (int k = 0; k < KL; ++k) {
        // measured slower (C5: A 2.05 -> 2.95 ms, B 1.68 -> 2.08 ms) although the Infinity-Cache fetch
        // drops 16x (A) / 3x (B): off unless LRS_TILES=1
        const bool can = P.tiles && !merge && !sh && W.GP && cone_of(k).colseg && cone_of(k).nown >= kNX;
        tla[k] = can && pa[k].wide && pa[k].grid >= kNX;
        tlb[k] = can && pb[k].wide && pb[k].grid >= kNX;
        if (tlb[k]) nblkB += pb[k].grid;
    }
    // long-row B over 2-D LDS tiles (k_tile_b1 / k_tile_b2, then k_wide_bf's epilogue blocks)
    bool tbt[kMaxCones];
    for (int k = 0; k < KL; ++k) {
        tbt[k] = !merge && !tlb[k] && pb[k].wide && W.GP && cone_of(k).sb_blocks > 0 && cone_of(k).sa_items > 0;
        if (tbt[k]) nblkB += pb[k].grid;
    }
    if (nblkB > kMaxPartialBlocks) {
        snprintf(g_err, sizeof(g_err), "stage B: %d partial blocks past %d", nblkB, kMaxPartialBlocks);
        return -1;
    }
    // one tiled cone, unsharded: stage A's slot values go to k_it_g as (RD, DD) records
    const bool use_uvp = !sh && !merge && KL == 1 && W.uvp && split && pa[0].wide && !tla[0] &&
                         cone_of(0).sa_items > 0;
    double2 *uvp = use_uvp ? reinterpret_cast<double2 *>(W.uvp) : nullptr;
    const int gwide = P.glob_maxlen >= 32 ? 1 : 0;   // long global constraints: a wave each
    const int gg = gwide ? std::min((std::max(1, P.mg) + kBlock / 64 - 1) / (kBlock / 64), kMaxPartialBlocks)
                         : std::min(grid_elems(std::max(1, P.mg), 1), kMaxPartialBlocks);
    // latency regime: every launch of both stages on the k_lat kernels, or none
    LatPlan lg[kMaxCones];
    const int ngd = P.ndense ? dense_cd_blocks(P) : 0;   // dense objective: C D's partial blocks
    bool lat = !sh && !split && !multi_path(P);
    int nla = 0, nlb = 0, nlf = 0;
    for (int k = 0; k < KL && lat; ++k) {
        lg[k] = lat_plan(cone_of(k), pa[k], pb[k]);
        if (lg[k].nrb <= 0) lat = false;
    }
    if (lat) {
        // row waves per block: the fewest whose grids (every cone's row and slice blocks, the
        // dense objective's and k_lat_f's partial blocks) stay within min(kLatMaxPartials, CUs)
        // blocks a stage -- one block a CU with as few row waves as the grid allows; else 7
        const int cap = std::min(kLatMaxPartials, num_cus());
        const int wf = lat_forced_waves();
        for (int w = wf > 0 ? wf : 1; w <= kLatRowWaves; ++w) {
            nla = nlb = nlf = 0;
            bool fits = true;
            for (int k = 0; k < KL; ++k) {
                lg[k] = lat_plan(cone_of(k), pa[k], pb[k], w);
                if (lg[k].nrb <= 0) fits = false;
                nla += lg[k].nrb + lg[k].sa;
                nlb += lg[k].nrb + lg[k].sb;
                nlf += lg[k].nf;
            }
            if (wf > 0 || w == kLatRowWaves) {
                lat = fits;
                break;
            }
            if (fits && nla + ngd <= cap && nlb + nlf <= cap && (P.mg == 0 || gg <= cap)) break;
        }
    }
    if (lat && (nla + ngd > kLatMaxPartials || nlb + nlf > kLatMaxPartials || (P.mg > 0 && gg > kLatMaxPartials)))
        lat = false;
    P.last_path = lat ? 0 : 1;
    P.last_tiles = 0;
    for (int k = 0; k < KL; ++k)
        if (tbt[k] || (pa[k].wide && !merge && !tla[k] && cone_of(k).sa_items > 0)) P.last_tiles = 1;
    if (lat) {
        nblkA = nla;
        nblkB = nlb + nlf;   // the C partials: B's blocks, then k_lat_f's
        for (int k = 0; k < KL; ++k) {
            pa[k].grid = lg[k].nrb + lg[k].sa;
            pb[k].grid = lg[k].nrb + lg[k].sb;
        }
    }
    // dense-objective cones: C D and its two objective partials after stage A's blocks
    const int offCD = nblkA;
    if (ngd) {
        nblkA += ngd;
        if (nblkA > kMaxPartialBlocks) {
            snprintf(g_err, sizeof(g_err), "dense objective: %d partial blocks past %d", nblkA, kMaxPartialBlocks);
            return -1;
        }
    }
    // what the consumers read: every producer block's partials, or (sharded) the summed totals
    // sharded: each stage's per-block partials folded once into the stage totals (k_fold_partials,
    // the consumers' reduction tree), which take the all-reduce; the next stage reads the totals
    // (measured unsharded at G81 / C5 size, where every consumer block re-reads every producer's
    // partials: no faster, profiles/r05f_g81_ab.txt)
    const bool totals = sh != nullptr;
    double *totA = totals ? W.tot : nullptr, *totC = totals ? W.tot + 16 : nullptr;
    const double *inC = totals ? totC : W.partC;
    const int nC = totals ? 1 : nblkB, pstr = totals ? 1 : kMaxPartialBlocks;
    const double *inA = totals ? totA : W.part;
    const int nA = totals ? 1 : nblkA;
    auto mark = [&](int q) -> int {
        if (a.ev && hipEventRecord(a.ev[q], st) != hipSuccess) {
            snprintf(g_err, sizeof(g_err), "hipEventRecord failed");
            return -1;
        }
        return 0;
    };
#define LRS_WIDE_A(TL_)                                                                                        \
    hipLaunchKernelGGL((k_wide_a<GG, EE, kWideU, TL_>), dim3(grid), dim3(kRowBlock), 0, st, c.nown, c.ld, c.foff,   \
                       c.adj_ptr, c.adj_low, c.adj_col, c.adj_slot, P.Cw, W.R, W.R2, W.D, W.uvt0, W.uvt1, P.loc_ptr,  \
                       P.loc_con, P.loc_w, reinterpret_cast<const double2 *>(P.loc1), P.b, W.cvs, W.lam, W.rec,      \
                       W.par, ctrl_cur, W.part, off, c.row0, P.m, c.colseg)
#define LRS_WIDE_B(TL_)                                                                                        \
    hipLaunchKernelGGL((k_wide_b<GG, EE, kWideU, TL_>), dim3(grid), dim3(kRowBlock), 0, st, c.nown, c.ld, c.foff,   \
                       c.adj_ptr, c.adj_low, c.adj_col, c.adj_slot, W.R, W.R2, W.D, W.G[0], W.G[1], W.ls[0], W.ly[0], \
                       W.ls[1], W.ly[1], W.uvt2, P.Craw, P.slot_ptr, P.slot_con, P.slot_a,                          \
                       reinterpret_cast<const double2 *>(P.slot1), W.rec, P.loc_ptr, P.loc_con, P.loc_w,             \
                       reinterpret_cast<const double2 *>(P.loc1), P.b, W.cvs, W.par, ctrl_cur, ls_cur, L, W.partC,   \
                       off, c.row0, P.m, P.ndense ? W.CR : nullptr, W.CD, c.colseg, W.GP, P.NRpad)
    if (mark(0)) return -1;
    // A: control, direction, sym(RD^T) / DD^T, local constraints' q and dots
    int off = 0;
    for (int k = 0; k < KL && (mask & 1); ++k) {
        const DevCone &c = cone_of(k);
        const int grid = pa[k].grid;
#define LRS_LAUNCH_A(UU, MM)                                                                               \
    hipLaunchKernelGGL((k_it_a<GG, EE, UU, MM>), dim3(grid), dim3(kRowBlock), 0, st, c.nown, c.ld, c.foff,     \
                       c.adj_ptr, c.adj_low, c.adj_col, c.adj_slot, P.Cw, W.R, W.R2, W.D, W.G[0], W.G[1], W.ls[0], \
                       W.ly[0], W.ls[1], W.ly[1], W.uvt0, W.uvt1, P.loc_ptr, P.loc_con, P.loc_w,                \
                       reinterpret_cast<const double2 *>(P.loc1), P.b, W.cvs,                                     \
                       W.lam, W.rec, (k == 0 && !sh) ? 1 : 0, P.mg, P.glob, P.m, P.K, P.con_ptr, P.con_slot,       \
                       P.con_w,                                                                                   \
                       W.uvt2, W.par, ctrl_prev, ctrl_cur, ls_prev, inC, nC, W.part, off, pa[k].T, gwide, c.row0, \
                       pstr)
        if (lat) {
            LRS_LAYOUT_SWITCH(c.G, c.E, {
                hipLaunchKernelGGL((k_lat_a<GG, EE, kLatNoA>), dim3(grid), dim3(lg[k].nt), 0, st, c.nown,
                                   c.ld, c.foff, c.adj_ptr, c.adj_low, c.adj_col, c.adj_slot, P.Cw, W.R, W.R2, W.D,
                                   W.G[0], W.G[1], W.ls[0], W.ly[0], W.ls[1], W.ly[1], W.uvt0, W.uvt1, P.loc_ptr,
                                   P.loc_con, P.loc_w, reinterpret_cast<const double2 *>(P.loc1), P.b, W.cvs, W.lam,
                                   W.rec, k == 0 ? 1 : 0, P.mg, P.glob, P.m, P.K, P.con_ptr, P.con_slot, P.con_w,
                                   W.uvt2, W.par, ctrl_prev, ctrl_cur, ls_prev, inC, nC, W.part, off, gwide,
                                   lg[k].nrb, lg[k].nt / 64 - 1, (int)c.dra_h.size(), c.dra);
            });
        } else {
            LRS_LAYOUT_SWITCH(c.G, c.E, {
                if (split) LRS_LAUNCH_A(1, 1);
                else if (pa[k].small) LRS_LAUNCH_A(2, 0);
                else LRS_LAUNCH_A(1, 0);
            });
        }
        LRS_CHECK_LAUNCH();
        off += grid;
    }
    // sharded: the direction rows of the halo from their owners before the SDDMM half
    if (sh && (mask & 1) && sh->halo(sh->self, W.D, st)) return -1;
    off = 0;
    for (int k = 0; k < KL && (mask & 1) && split; ++k) {
        const DevCone &c = cone_of(k);
        const int grid = pa[k].grid;
        if (pa[k].wide && !merge && !tla[k] && c.sa_items > 0) {
            // lower pattern in 2-D LDS tiles (k_tile_a): the resident blocks work, the rest write zero partials
            static int rca = 0;
            const int nwork = std::min(grid, resident_blocks(k_tile_a, &rca, 1024));
            hipLaunchKernelGGL(k_tile_a, dim3(grid), dim3(1024), 0, st, c.n, c.r, c.ld, c.foff, c.sa_ngrp, c.sa_grp,
                               nwork, reinterpret_cast<const int4 *>(c.sa_sub), c.sa_pq, c.sa_slot, P.Cw, W.R, W.R2,
                               W.D, W.uvt0, W.uvt1, P.loc_ptr, P.loc_con, P.loc_w,
                               reinterpret_cast<const double2 *>(P.loc1), P.b, W.cvs, W.lam, W.rec, W.par, ctrl_cur,
                               W.part, off, uvp);
        } else if (pa[k].wide) {
            LRS_LAYOUT_SWITCH(c.G, c.E, {
                if (tla[k]) LRS_WIDE_A(true);
                else LRS_WIDE_A(false);
            });
        } else {
            LRS_LAYOUT_SWITCH(c.G, c.E, { LRS_LAUNCH_A(kBwU, 2); });
        }
        LRS_CHECK_LAUNCH();
        off += grid;
    }
#undef LRS_LAUNCH_A
    if (ngd && (mask & 1) && launch_dense_cd(P, W, ctrl_cur, offCD, st)) return -1;
    if (totals && (mask & 1)) {
        hipLaunchKernelGGL(k_fold_partials<8>, dim3(1), dim3(kRowBlock), 0, st, W.part, nblkA, totA);
        LRS_CHECK_LAUNCH();
        if (sh && sh->allreduce(sh->self, totA, 8, st)) return -1;
    }
    if (mark(1)) return -1;
    // G: phase-1 test and the global constraints' q and dots
    double *totB = totals ? W.tot + 8 : nullptr;
    if (sh && P.mg > 0 && (mask & 2)) {
        // sharded: each holder's owned-entry sums, the shared constraints' summed over the
        // shards, then q / rec / dots from the totals, the dots and residual summed, the
        // phase-1 test on the summed residual
        const int g1 = gwide ? gg : std::min(grid_elems(P.mg, 1), kMaxPartialBlocks);
        if (P.nsh > 0) {
            hipLaunchKernelGGL(k_fill, dim3(grid_elems(3L * P.nsh, 4)), dim3(kBlock), 0, st, 3L * P.nsh, 0.0, P.gpack);
            LRS_CHECK_LAUNCH();
        }
        hipLaunchKernelGGL(k_g_part, dim3(g1), dim3(kBlock), 0, st, P.mg, P.glob, P.m, P.K, P.con_ptr, P.con_slot, P.con_w,
                           W.uvt2, W.uvt0, W.uvt1, P.sh_idx, P.g3, P.gpack, gwide, ctrl_cur);
        LRS_CHECK_LAUNCH();
        if (P.nsh > 0 && sh->allreduce(sh->self, P.gpack, 3 * P.nsh, st)) return -1;
        const int g2 = std::min(grid_elems(P.mg, 1), kMaxPartialBlocks);
        hipLaunchKernelGGL(k_it_g_sh, dim3(g2), dim3(kBlock), 0, st, P.mg, P.glob, P.m, P.sh_idx, P.g3, P.gpack, P.cmask,
                           P.b, W.cvs, W.lam, W.par, ctrl_cur, W.rec, W.partB);
        LRS_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_fold_partials<6>, dim3(1), dim3(kRowBlock), 0, st, W.partB, g2, totB);
        LRS_CHECK_LAUNCH();
        if (sh->allreduce(sh->self, totB, 6, st)) return -1;
        hipLaunchKernelGGL(k_g_ph1, dim3(1), dim3(64), 0, st, W.par, ctrl_cur, totC, totB);
        LRS_CHECK_LAUNCH();
    } else if (P.mg > 0 && (mask & 2)) {
        hipLaunchKernelGGL(k_it_g, dim3(gg), dim3(kBlock), 0, st, P.mg, P.glob, P.m, P.K, P.con_ptr, P.con_slot,
                           P.con_w, W.uvt0, W.uvt1, P.b, W.cvs, W.lam, W.par, ctrl_cur, W.partC, nblkB, W.part,
                           nblkA, W.rec, W.partB, gwide, uvp);
        LRS_CHECK_LAUNCH();
    }
    if (mark(2)) return -1;
    // B: line search, R update, adjoint, gradient, A(RR^T), L-BFGS pair, dots
    off = 0;
    long glo = 0;   // latency kernels: this launch's slice gradients in W.gl
    for (int k = 0; k < KL && (mask & 4); ++k) {
        const DevCone &c = cone_of(k);
        const int grid = pb[k].grid;
#define LRS_LAUNCH_B(UU, MM)                                                                               \
    hipLaunchKernelGGL((k_it_b<GG, EE, UU, MM>), dim3(grid), dim3(kRowBlock), 0, st, c.nown, c.ld, c.foff, c.adj_ptr, \
                       c.adj_low, c.adj_col, c.adj_slot, W.R, W.R2, W.D, W.G[0], W.G[1], W.ls[0], W.ly[0],        \
                       W.ls[1], W.ly[1], W.uvt2, P.Craw, P.slot_ptr, P.slot_con, P.slot_a,                        \
                       reinterpret_cast<const double2 *>(P.slot1), W.rec, P.loc_ptr, P.loc_con, P.loc_w,           \
                       reinterpret_cast<const double2 *>(P.loc1), P.b, W.cvs, W.par, ctrl_cur, inA, nA,            \
                       sh ? totB : W.partB, P.mg > 0 ? (sh ? 1 : gg) : 0, ls_cur, L, W.partC, off, pb[k].T, c.row0, \
                       c.n, pstr,                                                                                 \
                       (MM) != 2 && k == 0 ? a.hmirror : nullptr, a.seq, P.ndense ? W.CR : nullptr, W.CD)
        const bool small = pb[k].small;
        if (lat) {
            LRS_LAYOUT_SWITCH(c.G, c.E, {
                hipLaunchKernelGGL((k_lat_b<GG, EE, kLatNoB>), dim3(grid), dim3(lg[k].nt), 0, st, c.nown,
                                   c.ld, c.foff, c.adj_ptr, c.adj_low, c.adj_col, c.adj_slot, W.R, W.R2, W.D, W.G[0],
                                   W.G[1], W.ls[0], W.ly[0], W.ls[1], W.ly[1], W.uvt2, P.Craw, P.slot_ptr, P.slot_con,
                                   P.slot_a, reinterpret_cast<const double2 *>(P.slot1), W.rec, P.loc_ptr, P.loc_con,
                                   P.loc_w, reinterpret_cast<const double2 *>(P.loc1), P.b, W.cvs, W.par, ctrl_cur,
                                   inA, nA, W.partB, P.mg > 0 ? gg : 0, ls_cur, L, W.partC, off, P.m,
                                   k == 0 ? a.hmirror : nullptr, a.seq, lg[k].nrb, lg[k].nt / 64 - 1, (int)c.drb_h.size(), c.drb,
                                   W.gl + glo, P.ndense ? W.CR : nullptr, W.CD);
            });
            glo += (long)lg[k].sb * c.ld;
        } else {
            LRS_LAYOUT_SWITCH(c.G, c.E, {
                if (small) LRS_LAUNCH_B(4, 0);
                else if (bfused(pb[k], tbt[k]) && pb[k].T == 1 && bw_b_on())
                    hipLaunchKernelGGL((k_bw_b<GG, EE, kBwNo>), dim3(grid), dim3(kRowBlock), 0, st, c.nown, c.ld, c.foff,
                                       c.adj_ptr, c.adj_low, c.adj_col, c.adj_slot, W.R, W.R2, W.D, W.G[0], W.G[1],
                                       W.ls[0], W.ly[0], W.ls[1], W.ly[1], W.uvt2, P.Craw, P.slot_ptr, P.slot_con,
                                       P.slot_a, reinterpret_cast<const double2 *>(P.slot1), W.rec, P.loc_ptr,
                                       P.loc_con, P.loc_w, reinterpret_cast<const double2 *>(P.loc1), P.b, W.cvs,
                                       W.par, ctrl_cur, inA, nA, sh ? totB : W.partB, P.mg > 0 ? (sh ? 1 : gg) : 0,
                                       ls_cur, L, W.partC, off, c.row0, P.m, pstr, k == 0 ? a.hmirror : nullptr, a.seq,
                                       P.ndense ? W.CR : nullptr, W.CD);
                else if (bfused(pb[k], tbt[k])) LRS_LAUNCH_B(LRS_BW_UB, 0);
                else LRS_LAUNCH_B(1, 1);
            });
        }
        LRS_CHECK_LAUNCH();
        off += grid;
    }
    // latency regime: the dense rows' epilogues after their slices
    glo = 0;
    for (int k = 0; k < KL && (mask & 4) && lat; ++k) {
        const DevCone &c = cone_of(k);
        if (lg[k].nf > 0) {
            hipLaunchKernelGGL(k_lat_f, dim3(lg[k].nf), dim3(kRowBlock), 0, st, c.ld, c.G * c.E, c.foff, c.adj_ptr,
                               c.drb, ((lg[k].nt - 64) / c.G) * kSliceB, W.gl + glo, W.D, W.G[0], W.G[1], W.ls[0], W.ly[0],
                               W.ls[1], W.ly[1], ctrl_cur, ls_cur, L, W.partC, off, P.ndense ? W.CR : nullptr, W.CD);
            LRS_CHECK_LAUNCH();
        }
        glo += (long)lg[k].sb * c.ld;
        off += lg[k].nf;
    }
    // bandwidth regime: the gradient half over the updated factor
    off = 0;
    for (int k = 0; k < KL && (mask & 4); ++k) {
        const DevCone &c = cone_of(k);
        const int grid = pb[k].grid;
        if (pb[k].small || bfused(pb[k], tbt[k])) { off += grid; continue; }
        if (tbt[k]) {
            static int rcb = 0;   // the resident blocks stride over the items (stage B 864 -> 803 us on C5)
            const int nwb = std::min(grid, resident_blocks(k_tile_b1, &rcb, kRowBlock));
            hipLaunchKernelGGL(k_tile_b1, dim3(grid), dim3(kRowBlock), 0, st, c.n, c.r, c.ld, c.foff, c.sa_items,
                               reinterpret_cast<const int4 *>(c.sa_item), c.sa_pq, c.sa_slot, W.R, W.R2, W.uvt2,
                               c.sa_S - c.slot_off, P.Craw, P.slot_ptr,
                               P.slot_con, P.slot_a,
                               reinterpret_cast<const double2 *>(P.slot1), W.rec, P.loc_ptr, P.loc_con, P.loc_w,
                               reinterpret_cast<const double2 *>(P.loc1), P.b, W.cvs, W.par, ctrl_cur, ls_cur,
                               W.partC, off, nwb);
            LRS_CHECK_LAUNCH();
            if (c.sx_n > 0) {   // sharded: S on the halo rows' lower slots
                hipLaunchKernelGGL(k_slot_sv, dim3(std::min(grid_elems(c.sx_n, 1), 2048)), dim3(kBlock), 0, st, c.sx_n,
                                   c.sx_slot, 0, c.sa_S - c.slot_off, P.Craw,
                                   P.slot_ptr, P.slot_con, P.slot_a,
                                   reinterpret_cast<const double2 *>(P.slot1), W.rec, W.par, ctrl_cur, ls_cur, nullptr, 0);
                LRS_CHECK_LAUNCH();
            }
            hipLaunchKernelGGL(k_tile_b2, dim3(c.sb_blocks * ((c.ld + kTbC - 1) / kTbC)), dim3(kRowBlock), 0, st, c.n, c.ld, c.foff,
                               reinterpret_cast<const int2 *>(c.sb_blk), reinterpret_cast<const int2 *>(c.sb_tp),
                               c.sb_rp, reinterpret_cast<const int2 *>(c.sb_ent), c.sa_S - c.slot_off, W.R, W.R2,
                               W.GP, P.NRpad, c.r, ctrl_cur, ls_cur, c.sb_I0);
            LRS_CHECK_LAUNCH();
            LRS_LAYOUT_SWITCH(c.G, c.E, {
                hipLaunchKernelGGL((k_wide_bf<GG, EE>), dim3(grid), dim3(kRowBlock), 0, st, c.nown, c.ld, c.foff, W.D,
                                   W.G[0], W.G[1], W.ls[0], W.ly[0], W.ls[1], W.ly[1], ctrl_cur, ls_cur, L, W.partC,
                                   offBF, c.row0, P.ndense ? W.CR : nullptr, W.CD, W.GP, P.NRpad);
            });
            offBF += grid;
        } else if (pb[k].wide) {
            LRS_LAYOUT_SWITCH(c.G, c.E, {
                if (tlb[k]) {
                    LRS_WIDE_B(true);
                    LRS_CHECK_LAUNCH();
                    hipLaunchKernelGGL((k_wide_bf<GG, EE>), dim3(grid), dim3(kRowBlock), 0, st, c.nown, c.ld, c.foff,
                                       W.D, W.G[0], W.G[1], W.ls[0], W.ly[0], W.ls[1], W.ly[1], ctrl_cur, ls_cur, L,
                                       W.partC, offBF, c.row0, P.ndense ? W.CR : nullptr, W.CD, W.GP, P.NRpad);
                    offBF += grid;
                } else {
                    LRS_WIDE_B(false);
                }
            });
        } else {
            LRS_LAYOUT_SWITCH(c.G, c.E, { LRS_LAUNCH_B(kBwU, 2); });
        }
        LRS_CHECK_LAUNCH();
        off += grid;
    }
#undef LRS_LAUNCH_B
#undef LRS_WIDE_A
#undef LRS_WIDE_B
    if (totals && (mask & 4)) {
        hipLaunchKernelGGL(k_fold_partials<10>, dim3(1), dim3(kRowBlock), 0, st, W.partC, nblkB, totC);
        LRS_CHECK_LAUNCH();
        if (sh && sh->allreduce(sh->self, totC, 10, st)) return -1;
    }
    if (mark(3)) return -1;
    return mark(4);
}

// ------------------------------------------------------------------------
// Single-workgroup persistent ALM inner loop (small problems: theta-class cones, tiny MaxCut).
// The whole inner L-BFGS loop (lorads_alm.c:1302-1379) of one run_inner call runs in ONE
// launch of one workgroup: the trips are separated by workgroup barriers instead of kernel
// boundaries (no grid barrier, no inter-workgroup hand-off), the factor R and the direction D
// stay in LDS, the control block in LDS, the rest (G, the L-BFGS pairs, the per-constraint
// records) in global memory, which this one CU's L1 / the XCD's L2 serve.  Per trip, the same
// arithmetic as k_it_a / k_it_g / k_it_b (MODE 0) with the dense objective's carried C R
// (constant objectives C = alpha J: column sums): ctrl_step (fold of the previous trip's ten
// dots, L-BFGS coefficients), D, the pattern SDDMM with the local constraints' q1 / q2 and
// records, the global constraints', the wave-parallel line search, R += tau D, S R_new and
// A(R_new R_new^T) per row, the new L-BFGS pair and the ten dots.  The loop ends where the
// multi-launch iteration's control would (ctrl_step's exits), so every run_inner call is one
// launch and one host synchronisation.
// ------------------------------------------------------------------------
#ifndef LRS_SMALL_NT
#define LRS_SMALL_NT 512
#endif
constexpr int kSmallThreads = LRS_SMALL_NT;   // the single workgroup's threads
constexpr int kSmallMaxConst = 4;     // constant-objective cones the kernel carries
constexpr int kSmallMaxWg = 8;        // cones of a one-workgroup-per-cone launch
constexpr int kSmallXcds = 8;         // block stride between those cones' workgroups (MI355X: 8 XCDs)
constexpr int kSmallMaxLd = 64;       // widest factor row
constexpr int kSmallMaxRows = 1024;   // rows of a workgroup's cone(s): the rows phase's order in LDS
struct SmallWg {
    int n, r0, s0, P, nadj;                      // rows, first (all-cone) row, first slot, slots, adjacency
    const int *adj_ptr, *adj_low, *adj_col, *adj_slot;
};
struct SmallArgs {
    int N, K, m, Ptot, mg, nadj, al;
    const int2 *slot_g;                      // [Ptot] merged-space (row, col) of each slot (row >= col)
    const double *Cw, *Craw;
    const double2 *loc1, *slot1;
    const int *loc_ptr, *loc_con, *slot_ptr, *slot_con;
    const double *loc_w, *slot_a;
    const int *glob, *con_ptr, *con_slot;
    const double *con_w;
    const double *b, *lam;
    double *cvs, *rec, *uRD, *uDD, *uRR;
    double *R, *G0, *G1, *s0, *y0, *s1, *y1;
    const double *par;
    const double *ctrl_in;
    double *ctrl_out, *ls_out;
    int nconst;
    int cst_row0[kSmallMaxConst], cst_n[kSmallMaxConst];
    double cst_sa[kSmallMaxConst];
    // one workgroup per cone (nwg > 1; cones whose constraints each lie in one cone): workgroup k
    // at block k * xs runs cone k's rows [r0, r0 + n) and slots [s0, s0 + P) over the cone's own
    // adjacency; the per-trip sums are exchanged through xbuf ([2][kSmallMaxWg][16]) and the
    // arrival counter xcnt
    int nwg, xs;
    int spin_log2;             // the exchange's spin limit, 2^spin_log2 polls (LRS_XWG_SPIN; default 26; -1 none)
    int row_sort;              // rows phase in adjacency-length order (LRS_SMALL_ROWSORT; default 1)
    SmallWg wg[kSmallMaxWg];   // [0]: the single workgroup's (all cones, merged adjacency) when nwg == 1
    double *xbuf;
    unsigned *xcnt;
};
// The per-trip sums of the workgroups of one multi-cone launch (SmallArgs::nwg > 1), by wave 0
// of each: lane q stores partial sum q (a relaxed device-scope store: write-through to the
// coherence point), the wave waits for its stores, lane 0 counts the workgroup in and polls the
// counter until every workgroup of this exchange has arrived, then lane (k, q) loads workgroup
// k's sum q (device-scope loads, all in flight together) into xr and lane q adds them in
// workgroup order -- every workgroup gets the same totals (MI355X_MICROARCH.md, the hand-off
// table's first row: sc1 payload, drained, one counter add per workgroup, an sc1 poll, the
// polling wave's own loads after the match).  Two parities of the buffer: a workgroup cannot
// reach exchange e + 2 before every workgroup has read exchange e.  xs: this workgroup's nv
// sums (LDS); out: the totals (LDS); returns false when the others do not arrive within the
// spin limit (the caller ends the loop).
__device__ __forceinline__ bool xwg_sum(const SmallArgs &A, int wg, unsigned &xe, int nv, const double *xs,
                                        double *xr, double *out) {
    const int lane = threadIdx.x & 63;
    double *buf = A.xbuf + (long)(xe & 1u) * kSmallMaxWg * 16;
    if (lane < nv) __hip_atomic_store(buf + wg * 16 + lane, xs[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);   // the wave's stores acknowledged before the arrival is counted
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const unsigned target = (xe + 1u) * (unsigned)A.nwg;
    xe++;
    int ok = 1;
    if (lane == 0) {
        __hip_atomic_fetch_add(A.xcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (long spin = 0; __hip_atomic_load(A.xcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin) {
            if (spin > (A.spin_log2 < 0 ? -1L : (1L << A.spin_log2))) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    ok = __builtin_amdgcn_readfirstlane(ok);
    if (!ok) return false;
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    for (int k = lane / 16, q = lane % 16; k < A.nwg; k += 4)
        if (q < nv) xr[k * 16 + q] = __hip_atomic_load(buf + k * 16 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_wave_barrier();
    if (lane < nv) {
        double t = 0.0;
        for (int k = 0; k < A.nwg; ++k) t += xr[k * 16 + lane];
        out[lane] = t;
    }
    return true;
}

// diagnostics build: thread 0 adds each phase's wall-clock ticks (100 MHz) into g_phase[3][q]
// (q: 0 control, 1 direction, 2 slots, 3 global + reduction, 4 line search, 5 R / S update,
// 6 rows, 7 global + reduction; 15 the trips)
#ifdef LRS_PHASE_TIMING
#define LRS_SM_T(q) do { if (tid == 0) { const unsigned long long t_ = wall_clock64(); sm_t[q] += t_ - sm_last; sm_last = t_; } } while (0)
#define LRS_SM_MARK(v) unsigned long long v = tid == 0 ? wall_clock64() : 0
#define LRS_SM_SUB(q, v) do { if (tid == 0) sm_t[q] += wall_clock64() - v; } while (0)
#else
#define LRS_SM_T(q) do { } while (0)
#define LRS_SM_MARK(v) do { } while (0)
#define LRS_SM_SUB(q, v) do { } while (0)
#endif
template <int LD, bool AL, bool MC>
__global__ void __launch_bounds__(kSmallThreads) k_small_alm(SmallArgs A) {
    constexpr int LS = LD + 2;          // LDS row stride (doubles): 16-B aligned rows
    constexpr int H = LD / 2;           // double2 per row
    constexpr int LS2 = LS / 2;
    // row phases: TPR threads per row, H2 double2 each (pair p of lane l: columns 2 (l + TPR p), + 1);
    // few lanes per row: the cross-lane sums of the per-entry dots cost VALU issue per lane
    // (the loops are VALU-bound, not LDS-bound, at two waves per SIMD)
    constexpr int TPR = LD <= 32 ? 4 : 8;
    constexpr int H2 = H / TPR, RPP = kSmallThreads / TPR;
    static_assert(H2 * TPR == H, "row split");
    constexpr int T = kSmallThreads;
    // dynamic LDS 16-B aligned whatever the static arrays' size: R / D rows are read 16 B at a time
    extern __shared__ __attribute__((aligned(16))) double dyn[];
    // one workgroup per cone (A.nwg > 1): this block's cone, its rows, slots and adjacency; the
    // blocks between the cones' (blockIdx % xs != 0) leave at once
    // (MC: A.wg[wg] and the kernel arguments are re-read where used: the loop holds no copies)
    constexpr bool mc = MC;
    if (MC && blockIdx.x % A.xs != 0) return;
    const int wg = MC ? (int)blockIdx.x / A.xs : 0;
    const int N = MC ? A.wg[wg].n : A.N, tid = threadIdx.x;
    const int rb = MC ? A.wg[wg].r0 : 0, sb = MC ? A.wg[wg].s0 : 0, Pn = MC ? A.wg[wg].P : A.Ptot;
    const int nadj = MC ? A.wg[wg].nadj : A.nadj;
    const long rbo = (long)rb * LD;   // this cone's first factor element
    // this workgroup's slot-indexed arrays and adjacency (MC == false: the arguments themselves)
    const int2 *__restrict__ slot_g = MC ? A.slot_g + sb : A.slot_g;
    const double *__restrict__ Cw = MC ? A.Cw + sb : A.Cw;
    const double *__restrict__ Craw = MC ? A.Craw + sb : A.Craw;
    const double2 *__restrict__ loc1 = MC ? A.loc1 + sb : A.loc1;
    const double2 *__restrict__ slot1 = MC ? A.slot1 + sb : A.slot1;
    const int *__restrict__ loc_ptr = MC ? A.loc_ptr + sb : A.loc_ptr;
    const int *__restrict__ slot_ptr = MC ? A.slot_ptr + sb : A.slot_ptr;
    const int *__restrict__ adj_ptr = A.wg[wg].adj_ptr, *__restrict__ adj_low = A.wg[wg].adj_low;
    const int *__restrict__ adj_col = A.wg[wg].adj_col, *__restrict__ adj_slot = A.wg[wg].adj_slot;
    auto own_c = [&](int q) { return A.cst_row0[q] >= rb && A.cst_row0[q] < rb + N; };   // this cone's constant C
    // LDS: R, D; per-slot X1 (uDD, then S); with AL a second per-slot array (uRD, then uRR)
    // and the adjacency ((column, slot) pairs, row pointers, lower-entry ends), without AL
    // (the lean layout, larger cones) those stay in global memory
    double *Rs = dyn, *Ds = dyn + (long)N * LS, *X1 = dyn + 2L * N * LS, *X2 = X1 + Pn;
    int2 *Ladj = reinterpret_cast<int2 *>(X2 + Pn);
    int *Lptr = reinterpret_cast<int *>(Ladj + nadj), *Llow = Lptr + N + 1;
    double *XA = AL ? X2 : A.uRD + sb, *XB = AL ? X2 : A.uRR + sb;
    auto adj = [&](int q) -> int2 {
        if constexpr (AL) return Ladj[q];
        else return make_int2(adj_col[q], adj_slot[q] - sb);
    };
    auto aptr = [&](int i) -> int {
        if constexpr (AL) return Lptr[i];
        else return adj_ptr[i];
    };
    auto alow = [&](int i) -> int {
        if constexpr (AL) return Llow[i];
        else return adj_low[i];
    };
    const double2 *Rs2 = reinterpret_cast<const double2 *>(Rs), *Ds2 = reinterpret_cast<const double2 *>(Ds);
    __shared__ double c[C_NCTRL];
    __shared__ double red[16];
    __shared__ double ls[LS_N];
    __shared__ double csR[kSmallMaxConst][kSmallMaxLd], csD[kSmallMaxConst][kSmallMaxLd];
    __shared__ double cpart[kSmallThreads];
    __shared__ int xfail;
    __shared__ int Lord[kSmallMaxRows];   // the rows phase's row order
    __shared__ double xsum[16], xrecv[kSmallMaxWg * 16];   // the exchange's own sums, the received ones
    unsigned xe = 0;   // exchanges so far (wave 0)
    const int lane = tid & 63, wv = tid >> 6, sl_lane = tid % TPR;
    const double rho = A.par[P_RHO], rhoInv = 1.0 / rho;
    if (tid < LS_N) ls[tid] = 0.0;
    if (tid == 0) xfail = 0;
    // R into LDS, the control block, the adjacency
    for (int e = tid; e < N * H; e += T) {
        const int i = e / H, q = e - i * H;
        reinterpret_cast<double2 *>(Rs + (long)i * LS)[q] = reinterpret_cast<const double2 *>((MC ? A.R + rbo : A.R) + (long)i * LD)[q];
    }
    if (tid < C_NCTRL) c[tid] = A.ctrl_in[tid];
    if (AL) {
        for (int e = tid; e < nadj; e += T) Ladj[e] = make_int2(adj_col[e], adj_slot[e] - sb);
        for (int e = tid; e <= N; e += T) {
            Lptr[e] = adj_ptr[e];
            if (e < N) Llow[e] = adj_low[e];
        }
    }
    __syncthreads();
    // the rows phase's order (row_sort): rows by adjacency length, longest first (ties by index),
    // dealt to the row groups in alternating directions pass by pass -- a wave's pass lasts as
    // long as its longest row, so the long rows share the first pass's waves and the short ones
    // fill the last, partial pass beside the first pass's shortest; a row's own sums keep their order
    constexpr int RK = (kSmallMaxRows + T - 1) / T;
    for (int i = tid; i < N; i += T) Lord[i] = A.row_sort ? aptr(i + 1) - aptr(i) : 0;
    __syncthreads();
    int rk[RK];
#pragma unroll
    for (int u = 0; u < RK; ++u) {
        const int i = tid + u * T;
        rk[u] = i;
        if (i >= N || !A.row_sort) continue;
        const int di = Lord[i];
        int k = 0;
        for (int j = 0; j < N; ++j) {
            const int dj = Lord[j];
            k += (dj > di || (dj == di && j < i)) ? 1 : 0;
        }
        rk[u] = k;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < RK; ++u)
        if (tid + u * T < N) Lord[rk[u]] = tid + u * T;
    __syncthreads();
    // constant objectives: column sums (C R = sa 1 (1^T R), carried with tau like C R)
    auto colsums = [&](const double *X, double (*cs)[kSmallMaxLd]) {
        constexpr int G = kSmallThreads / LD;
        for (int q = 0; q < A.nconst; ++q) {
            if (!own_c(q)) continue;   // block-uniform
            const int col = tid % LD, g = tid / LD;
            double t = 0.0;
            if (g < G)
                for (int i = g; i < A.cst_n[q]; i += G) t += X[(long)(A.cst_row0[q] - rb + i) * LS + col];
            __syncthreads();
            cpart[tid] = t;
            __syncthreads();
            if (tid < LD) {
                double s = 0.0;
                for (int h = 0; h < G; ++h) s += cpart[h * LD + tid];
                cs[q][tid] = s;
            }
        }
        __syncthreads();
    };
    __syncthreads();
    if (A.nconst) colsums(Rs, csR);
    double lsflag = 0.0, lstau = 0.0;
    int fold = 0;
#ifdef LRS_PHASE_TIMING
    unsigned long long sm_t[16] = {0}, sm_last = wall_clock64();
#endif
    for (;;) {
        // ---- control (k_it_a's fold + ctrl_step, the phase-1 test on the whole residual)
        if (tid == 0) ctrl_step(c, A.par, lsflag, lstau, fold, red, true);
        __syncthreads();
        LRS_SM_T(0);
        if (c[C_ACTIVE] == 0.0) break;
#ifdef LRS_PHASE_TIMING
        sm_t[15]++;
#endif
        const double cg = c[C_CG], cs0 = c[C_CS0], cy0 = c[C_CY0], cs1 = c[C_CS1], cy1 = c[C_CY1];
        const bool u0 = (cs0 != 0.0 || cy0 != 0.0), u1 = (cs1 != 0.0 || cy1 != 0.0);
        const double *__restrict__ Gc = c[C_GCUR] == 0.0 ? (MC ? A.G0 + rbo : A.G0) : (MC ? A.G1 + rbo : A.G1);
        // ---- D = -(cg G + cs0 s0 + cy0 y0 + cs1 s1 + cy1 y1)  (DirRow's arithmetic), 16-B loads
        // two elements a thread at a time, every operand load issued before the arithmetic
        // (one memory trip per pair instead of one per element and operand)
        for (int e0 = tid; e0 < N * H; e0 += 2 * T) {
            double2 gv[2], a0[2], b0[2], a1[2], b1[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int e = min(e0 + u * T, N * H - 1), i = e / H, q = e - i * H;
                const long o = (long)i * LD + 2 * q;
                gv[u] = *reinterpret_cast<const double2 *>(Gc + o);
                a0[u] = *reinterpret_cast<const double2 *>((MC ? A.s0 + rbo : A.s0) + o);
                b0[u] = *reinterpret_cast<const double2 *>((MC ? A.y0 + rbo : A.y0) + o);
                a1[u] = *reinterpret_cast<const double2 *>((MC ? A.s1 + rbo : A.s1) + o);
                b1[u] = *reinterpret_cast<const double2 *>((MC ? A.y1 + rbo : A.y1) + o);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int e = e0 + u * T;
                if (e >= N * H) break;
                const int i = e / H, q = e - i * H;
                double dx = cg * gv[u].x, dy = cg * gv[u].y;
                if (u0) {
                    dx += cs0 * a0[u].x + cy0 * b0[u].x;
                    dy += cs0 * a0[u].y + cy0 * b0[u].y;
                }
                if (u1) {
                    dx += cs1 * a1[u].x + cy1 * b1[u].x;
                    dy += cs1 * a1[u].y + cy1 * b1[u].y;
                }
                reinterpret_cast<double2 *>(Ds + (long)i * LS)[q] = make_double2(-dx, -dy);
            }
        }
        __syncthreads();
        if (A.nconst) colsums(Ds, csD);
        LRS_SM_T(1);
        // ---- A: the pattern's lower slots (k_it_a's per-slot arithmetic), a thread per slot
        // (by rows instead -- a group of lanes per row, each lower entry's R_j / D_j read once --
        // measured slower: the per-entry cross-lane sums and a second per-slot pass for the
        // constraints outweigh the halved LDS reads); uRD -> XA, uDD -> X1
        double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        // software-pipelined: the next slot's records and this slot's single constraint's
        // values are in flight while this slot's dots run on LDS (one memory trip a slot, not
        // two); loads clamped, not branched
        // (Ptot == 0: index 0 of the >= 1-element arrays, never used -- the loop does not run)
        const int s0c = max(0, min(tid, Pn - 1));
        int2 ijn = slot_g[s0c];
        double cwn = Cw[s0c];
        double2 l1n = loc1[s0c];
        for (int s = tid; s < Pn; s += T) {
            const int2 ij = make_int2(ijn.x - rb, ijn.y - rb);
            const double cw = cwn;
            const double2 l1u = l1n;
            {
                const int sn = min(s + T, Pn - 1);
                ijn = slot_g[sn];
                cwn = Cw[sn];
                l1n = loc1[sn];
            }
            const int c1p = (int)l1u.y >= 0 ? (int)l1u.y : 0;
            const double bp = A.b[c1p], cvp = A.cvs[c1p], lp = A.lam[c1p];
            const double2 *ri = Rs2 + (long)ij.x * LS2, *di = Ds2 + (long)ij.x * LS2;
            const double2 *rj = Rs2 + (long)ij.y * LS2, *dj = Ds2 + (long)ij.y * LS2;
            double d0 = 0.0, d1 = 0.0;
            if (ij.x != ij.y) {
#pragma unroll 4
                for (int q = 0; q < H; ++q) {
                    const double2 a = ri[q], bq = dj[q], cq = rj[q], dq = di[q];
                    d0 += a.x * bq.x + cq.x * dq.x;
                    d0 += a.y * bq.y + cq.y * dq.y;
                    d1 += dq.x * bq.x;
                    d1 += dq.y * bq.y;
                }
                d0 *= 0.5;
            } else {
#pragma unroll 4
                for (int q = 0; q < H; ++q) {
                    const double2 a = ri[q], dq = di[q];
                    d0 += a.x * dq.x;
                    d0 += a.y * dq.y;
                    d1 += dq.x * dq.x;
                    d1 += dq.y * dq.y;
                }
            }
            XA[s] = d0;
            X1[s] = d1;
            acc[0] += cw * d0;
            acc[1] += cw * d1;
            const int c1 = (int)l1u.y;
            const int e0 = c1 == -2 ? loc_ptr[s] : 0, e1 = c1 == -2 ? loc_ptr[s + 1] : (c1 >= 0 ? 1 : 0);
            for (int e = e0; e < e1; ++e) {
                const int ci = c1 >= 0 ? c1 : A.loc_con[e];
                const double w = c1 >= 0 ? l1u.x : A.loc_w[e];
                const double q1 = 2.0 * (w * d0), q2 = w * d1;
                double bi = bp, cv = cvp, li = lp;
                if (c1 < 0) { bi = A.b[ci]; cv = A.cvs[ci]; li = A.lam[ci]; }
                const double q0 = (bi - cv) + rhoInv * li;
                acc[2] += q2 * q2; acc[3] += q1 * q2; acc[4] += q0 * q2; acc[5] += q1 * q1; acc[6] += q0 * q1;
                double2 *rc = reinterpret_cast<double2 *>(A.rec + 4L * ci);
                rc[0] = make_double2(cv, q1);
                rc[1] = make_double2(q2, (-li) + (-rho) * bi);
            }
        }
        __syncthreads();   // uRD / uDD of every slot before the global constraints read them
        LRS_SM_T(2);
        // ---- G: the global (multi-slot) constraints, a wave each (k_it_g's arithmetic)
        for (int g = wv; g < A.mg; g += T / 64) {
            const int i = A.glob[g];
            // one workgroup per cone: the constraint is this cone's, or another's (wave-uniform)
            if (mc && A.con_ptr[(long)wg * A.m + i] == A.con_ptr[(long)wg * A.m + i + 1]) continue;
            double v1 = 0.0, v2 = 0.0;
            for (int k = mc ? wg : 0; k < (mc ? wg + 1 : A.K); ++k) {
                const long row = (long)k * A.m + i;
                double a1 = 0.0, a2 = 0.0;
                // four entries a lane in flight, summed in entry order
                const int eb = A.con_ptr[row], ee = A.con_ptr[row + 1];
                for (int e0 = eb + lane; e0 < ee; e0 += 256) {
                    double w[4], xa[4], x1[4];
                    int sl[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int e = min(e0 + 64 * u, ee - 1);
                        w[u] = A.con_w[e];
                        sl[u] = A.con_slot[e];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        xa[u] = XA[sl[u] - sb];
                        x1[u] = X1[sl[u] - sb];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const bool ok = e0 + 64 * u < ee;
                        a1 = ok ? a1 + w[u] * xa[u] : a1;
                        a2 = ok ? a2 + w[u] * x1[u] : a2;
                    }
                }
                v1 += wave_sum(a1);
                v2 += wave_sum(a2);
            }
            if (lane != 0) continue;
            v1 *= 2.0;
            const double bi = A.b[i], ci = A.cvs[i], li = A.lam[i];
            const double q0 = (bi - ci) + rhoInv * li;
            acc[2] += v2 * v2; acc[3] += v1 * v2; acc[4] += q0 * v2; acc[5] += v1 * v1; acc[6] += q0 * v1;
            double2 *rc = reinterpret_cast<double2 *>(A.rec + 4L * i);
            rc[0] = make_double2(ci, v1);
            rc[1] = make_double2(v2, (-li) + (-rho) * bi);
        }
        {
            double s7[8];
            block_reduce<8, kSmallThreads>(acc, s7);
            if (tid == 0) {
                // constant objectives: <C, sym R D^T> = sa (1^T R).(1^T D), <C, D D^T> = sa |1^T D|^2
                for (int q = 0; q < A.nconst; ++q) {
                    if (!own_c(q)) continue;
                    double a = 0.0, bb = 0.0;
                    for (int e = 0; e < LD; ++e) {
                        const double y = A.cst_sa[q] * csD[q][e];
                        a += csR[q][e] * y;
                        bb += csD[q][e] * y;
                    }
                    s7[0] += a;
                    s7[1] += bb;
                }
                for (int q = 0; q < 7; ++q) (mc ? xsum : red)[q] = s7[q];
            }
        }
        if (mc) {
            __syncthreads();
            if (wv == 0 && !xwg_sum(A, wg, xe, 7, xsum, xrecv, red) && lane == 0) xfail = 1;
        }
        __syncthreads();   // every rec written, the reduced sums in red
        if (xfail) break;
        LRS_SM_T(3);
        if (tid < 64) line_search_t<true>(A.par, red[0], red[1], red + 2, ls);   // wave 0
        __syncthreads();
        LRS_SM_T(4);
        lsflag = ls[LS_FLAG];
        lstau = ls[LS_TAU];
        fold = 0;
        if (lsflag != 0.0) continue;   // rootNum 0 / tiny tau: the next ctrl_step exits
        const double tau = lstau, tau2 = tau * tau;
        const int gcur = (int)c[C_GCUR], h = (int)c[C_HEAD];
        // ---- R_new = R + tau D (in place), S = C + A^*(M1) per slot -> X1 (k_it_b's per-entry
        // arithmetic, once per slot instead of per adjacency entry), the column sums carried
        for (int e = tid; e < N * H; e += T) {
            const int i = e / H, q = e - i * H;
            double2 *rp = reinterpret_cast<double2 *>(Rs + (long)i * LS) + q;
            const double2 dv = reinterpret_cast<const double2 *>(Ds + (long)i * LS)[q];
            double2 rv = *rp;
            rv.x += tau * dv.x;
            rv.y += tau * dv.y;
            *rp = rv;
        }
        for (int s0 = tid; s0 < Pn; s0 += 2 * T) {
            double craw[2];
            double2 s1u[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int s = s0 + u * T < Pn ? s0 + u * T : s0;
                craw[u] = Craw[s];
                s1u[u] = slot1[s];
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int s = s0 + u * T;
                if (s >= Pn) break;
                double sv = craw[u];
                const int c1 = (int)s1u[u].y;
                const int e0 = c1 == -2 ? slot_ptr[s] : 0, e1 = c1 == -2 ? slot_ptr[s + 1] : (c1 >= 0 ? 1 : 0);
                for (int e = e0; e < e1; ++e) {
                    const int con = c1 >= 0 ? c1 : A.slot_con[e];
                    const double2 *rc = reinterpret_cast<const double2 *>(A.rec + 4L * con);
                    const double2 ra = rc[0], rb = rc[1];
                    double cv = ra.x + tau * ra.y;
                    cv = cv + tau2 * rb.x;
                    const double M1 = rb.y + rho * cv;
                    sv += M1 * (c1 >= 0 ? s1u[u].x : A.slot_a[e]);
                }
                X1[s] = sv;
            }
        }
        if (tid < LD)
            for (int q = 0; q < A.nconst; ++q)
                if (own_c(q)) csR[q][tid] += tau * csD[q][tid];
        __syncthreads();
        LRS_SM_T(5);
        // ---- B: per row, S R_new over the adjacency and A(R_new R_new^T) on the lower slots
        // (k_it_b's arithmetic); uRR -> XB
        double *__restrict__ Gold = gcur == 0 ? (MC ? A.G0 + rbo : A.G0) : (MC ? A.G1 + rbo : A.G1), *__restrict__ Gnew = gcur == 0 ? (MC ? A.G1 + rbo : A.G1) : (MC ? A.G0 + rbo : A.G0);
        double *__restrict__ sh = h == 0 ? (MC ? A.s0 + rbo : A.s0) : (MC ? A.s1 + rbo : A.s1), *__restrict__ yh = h == 0 ? (MC ? A.y0 + rbo : A.y0) : (MC ? A.y1 + rbo : A.y1);
        const double *__restrict__ so = h == 0 ? (MC ? A.s1 + rbo : A.s1) : (MC ? A.s0 + rbo : A.s0), *__restrict__ yo = h == 0 ? (MC ? A.y1 + rbo : A.y1) : (MC ? A.y0 + rbo : A.y0);
        double bacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i0 = 0; i0 < N; i0 += RPP) {
            const int gi = tid / TPR;
            const int pos = i0 + ((A.row_sort && ((i0 / RPP) & 1)) ? RPP - 1 - gi : gi);
            const bool valid = pos < N;
            const int ii = Lord[valid ? pos : N - 1];
            double2 g[H2], rii[H2];
            const long ob = ((long)ii * LD) / 2 + sl_lane;     // double2 index of this lane's first pair
#pragma unroll
            for (int p = 0; p < H2; ++p) {
                g[p] = make_double2(0.0, 0.0);
                rii[p] = Rs2[(long)ii * LS2 + sl_lane + TPR * p];
            }
            LRS_SM_MARK(t_adj);
            const int kb = aptr(ii), kl = alow(ii), ke = valid ? aptr(ii + 1) : kb;
            int2 jn[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) jn[u] = adj(kb + u < ke ? kb + u : kb);
            for (int k = kb; k < ke; k += 4) {   // four entries per pass, the next four's indices in flight
                int2 js[4];
                double sv[4], d[4];
                double2 x[4][H2];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    js[u] = jn[u];
                    const int kn = k + 4 + u;
                    jn[u] = adj(kn < ke ? kn : kb);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double t = X1[js[u].y];
                    sv[u] = k + u < ke ? t : 0.0;
#pragma unroll
                    for (int p = 0; p < H2; ++p) x[u][p] = Rs2[(long)js[u].x * LS2 + sl_lane + TPR * p];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    d[u] = 0.0;
#pragma unroll
                    for (int p = 0; p < H2; ++p) {
                        g[p].x += sv[u] * x[u][p].x;
                        g[p].y += sv[u] * x[u][p].y;
                        d[u] += rii[p].x * x[u][p].x;
                        d[u] += rii[p].y * x[u][p].y;
                    }
                }
                // lower entries: A(R R^T) on this row's slots (their constraints after the barrier)
                if constexpr (TPR == 4) {
                    const double v = group_sum4<4>(d, sl_lane);   // lane u: entry u
                    const int u = sl_lane;
                    const int su = u == 0 ? js[0].y : (u == 1 ? js[1].y : (u == 2 ? js[2].y : js[3].y));
                    if (k + u < kl) XB[su] = v;
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) d[u] = group_sum<TPR>(d[u]);
                    if (sl_lane == 0)
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (k + u < kl) XB[js[u].y] = d[u];
                }
            }
            LRS_SM_SUB(8, t_adj);
            if (!valid) continue;
            LRS_SM_MARK(t_epi);
            // row epilogue (k_it_b): [C R_new], G_new = 2 (...), s = tau D, y = G_new - G_old
            int cq = -1;
            for (int q = 0; q < A.nconst; ++q)
                if (ii + rb >= A.cst_row0[q] && ii + rb < A.cst_row0[q] + A.cst_n[q]) cq = q;
            double2 go[H2], sov[H2], yov[H2];
#pragma unroll
            for (int p = 0; p < H2; ++p) {
                go[p] = reinterpret_cast<const double2 *>(Gold)[ob + TPR * p];
                sov[p] = reinterpret_cast<const double2 *>(so)[ob + TPR * p];
                yov[p] = reinterpret_cast<const double2 *>(yo)[ob + TPR * p];
            }
#pragma unroll
            for (int p = 0; p < H2; ++p) {
                const int col = 2 * (sl_lane + TPR * p);
                double2 gv = g[p];
                if (cq >= 0) {
                    gv.x += A.cst_sa[cq] * csR[cq][col];
                    gv.y += A.cst_sa[cq] * csR[cq][col + 1];
                }
                gv.x *= 2.0;
                gv.y *= 2.0;
                const double2 dv = Ds2[(long)ii * LS2 + sl_lane + TPR * p];
                const double2 sv = make_double2(tau * dv.x, tau * dv.y);
                const double2 yv = make_double2(gv.x - go[p].x, gv.y - go[p].y);
                const long o = ob + TPR * p;
                reinterpret_cast<double2 *>(Gnew)[o] = gv;
                reinterpret_cast<double2 *>(sh)[o] = sv;
                reinterpret_cast<double2 *>(yh)[o] = yv;
#pragma unroll
                for (int h2 = 0; h2 < 2; ++h2) {
                    const double G_ = h2 ? gv.y : gv.x, S_ = h2 ? sv.y : sv.x, Y_ = h2 ? yv.y : yv.x;
                    const double SO = h2 ? sov[p].y : sov[p].x, YO = h2 ? yov[p].y : yov[p].x;
                    bacc[0] += G_ * G_; bacc[1] += Y_ * S_; bacc[2] += Y_ * Y_; bacc[3] += S_ * G_; bacc[4] += Y_ * G_;
                    bacc[5] += SO * G_; bacc[6] += YO * G_; bacc[7] += SO * Y_; bacc[8] += YO * Y_;
                }
            }
            LRS_SM_SUB(9, t_epi);
        }
        __syncthreads();   // uRR of every slot before the constraints read them
        LRS_SM_T(6);
        // single-slot constraints: A(R_new R_new^T) and their residual, a thread per slot
        // software-pipelined as the slot phase: the next slot's record and this slot's b in flight
        double2 l1nx = loc1[max(0, min(tid, Pn - 1))];
        for (int s = tid; s < Pn; s += T) {
            const double d = XB[s];
            const double2 l1u = l1nx;
            l1nx = loc1[min(s + T, Pn - 1)];
            const int c1 = (int)l1u.y;
            const double bc = A.b[c1 >= 0 ? c1 : 0];
            if (AL) A.uRR[sb + s] = d;
            if (c1 >= 0) {
                const double tot = l1u.x * d, dd = bc - tot;
                A.cvs[c1] = tot;
                bacc[9] += dd * dd;
                continue;
            }
            if (c1 == -2)
                for (int e = loc_ptr[s]; e < loc_ptr[s + 1]; ++e) {
                    const int ci = A.loc_con[e];
                    const double tot = A.loc_w[e] * d, dd = A.b[ci] - tot;
                    A.cvs[ci] = tot;
                    bacc[9] += dd * dd;
                }
        }
        // global constraints: A(R_new R_new^T) from the slots and their residual
        for (int g = wv; g < A.mg; g += T / 64) {
            const int i = A.glob[g];
            if (mc && A.con_ptr[(long)wg * A.m + i] == A.con_ptr[(long)wg * A.m + i + 1]) continue;
            double tot = 0.0;
            for (int k = mc ? wg : 0; k < (mc ? wg + 1 : A.K); ++k) {
                const long row = (long)k * A.m + i;
                double v = 0.0;
                // four entries a lane in flight, summed in entry order
                const int eb = A.con_ptr[row], ee = A.con_ptr[row + 1];
                for (int e0 = eb + lane; e0 < ee; e0 += 256) {
                    double w[4], xv[4];
                    int sl[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int e = min(e0 + 64 * u, ee - 1);
                        w[u] = A.con_w[e];
                        sl[u] = A.con_slot[e];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) xv[u] = XB[sl[u] - sb];
#pragma unroll
                    for (int u = 0; u < 4; ++u) v = e0 + 64 * u < ee ? v + w[u] * xv[u] : v;
                }
                tot += wave_sum(v);
            }
            if (lane == 0) {
                A.cvs[i] = tot;
                const double dd = A.b[i] - tot;
                bacc[9] += dd * dd;
            }
        }
        {
            double s10[10];
            block_reduce<10, kSmallThreads>(bacc, s10);
            if (tid == 0)
                for (int q = 0; q < 10; ++q) (mc ? xsum : red)[q] = s10[q];
        }
        if (mc) {
            __syncthreads();
            if (wv == 0 && !xwg_sum(A, wg, xe, 10, xsum, xrecv, red) && lane == 0) xfail = 1;
        }
        __syncthreads();
        if (xfail) break;
        LRS_SM_T(7);
        fold = 1;
    }
    // R back to global memory (the iterate stays in W.R: RCUR 0), the control block out
    for (int e = tid; e < N * H; e += T) {
        const int i = e / H, q = e - i * H;
        reinterpret_cast<double2 *>((MC ? A.R + rbo : A.R) + (long)i * LD)[q] = reinterpret_cast<const double2 *>(Rs + (long)i * LS)[q];
    }
    if (tid == 0) {
        c[C_RCUR] = 0.0;
        if (xfail) { c[C_ACTIVE] = 0.0; c[C_EXIT] = (double)EXIT_XWG; }
    }
    if (MC) {
        // the control block goes out through the buffer it came in by (ctrl_out == ctrl_in): every
        // workgroup counts itself out once more, and workgroup 0 writes only after all have --
        // each read ctrl_in at its start, so none can still be reading it
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_fetch_add(A.xcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (wg == 0 && !xfail) {
                const unsigned target = (xe + 1u) * (unsigned)A.nwg;
                for (long spin = 0; __hip_atomic_load(A.xcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin) {
                    if (spin > (A.spin_log2 < 0 ? -1L : (1L << A.spin_log2))) { c[C_ACTIVE] = 0.0; c[C_EXIT] = (double)EXIT_XWG; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
        }
    }
    __syncthreads();
    if (wg == 0 && tid < C_NCTRL) A.ctrl_out[tid] = c[tid];
    if (wg == 0 && tid < LS_N) A.ls_out[tid] = ls[tid];
#ifdef LRS_PHASE_TIMING
    if (tid == 0 && wg == 0)
        for (int q = 0; q < 16; ++q) g_phase[3][q] += sm_t[q];
#endif
}

static size_t small_lds_bytes(int N, int ld, int Ptot, long nadj, bool al) {
    if (!al) return (2UL * N * (ld + 2) + (size_t)Ptot) * sizeof(double);
    return (2UL * N * (ld + 2) + 2UL * Ptot + (size_t)nadj) * sizeof(double) + (2UL * N + 2) * sizeof(int);
}
constexpr size_t kSmallMaxDynLds = 136 * 1024;   // beside ~15 KB of the kernel's static LDS
static bool small_ld_ok(int ld) { return ld == 8 || ld == 16 || ld == 24 || ld == 32 || ld == 48 || ld == 64; }

// Whether the whole inner loop fits the single-workgroup kernel; fills the launch arguments.
static bool small_alm_args(const DevProblem &P, DevWork &W, SmallArgs &A, int *ldo) {
    if (P.shard || !P.slot_g || P.K > kMaxCones) return false;
    const int ld = P.cones[0].ld;
    int N = 0, nconst = 0;
    for (int k = 0; k < P.K; ++k) {
        const DevCone &c = P.cones[k];
        if (c.ld != ld || c.dense_c == 1) return false;
        if (c.dense_c == 2) {
            if (nconst >= kSmallMaxConst) return false;
            A.cst_row0[nconst] = N;
            A.cst_n[nconst] = c.n;
            A.cst_sa[nconst] = P.dense_scale * c.c_alpha;
            nconst++;
        }
        N += c.n;
    }
    if (!small_ld_ok(ld) || N <= 0) return false;
    const DevCone &a = P.K > 1 && P.has_merged ? P.merged : P.cones[0];
    A.nwg = 1;
    A.xs = 1;
    // LRS_SMALL_MC=1 (tests): one workgroup per cone wherever that applies, also where all fit one
    const bool force_mc = getenv("LRS_SMALL_MC") && atoi(getenv("LRS_SMALL_MC")) != 0;
    if ((P.K == 1 || P.has_merged) && !(force_mc && P.K >= 2 && P.cone_sep) &&
        N <= kSmallMaxRows && small_lds_bytes(N, ld, P.Ptot, a.adj_nnz, false) <= kSmallMaxDynLds) {
        A.al = small_lds_bytes(N, ld, P.Ptot, a.adj_nnz, true) <= kSmallMaxDynLds;
    } else {
        // one workgroup per cone: every constraint within one cone, each cone in one CU's LDS
        if (P.K < 2 || P.K > kSmallMaxWg || !P.cone_sep) return false;
        bool al = true;
        for (int k = 0; k < P.K; ++k) {
            const DevCone &ck = P.cones[k];
            if (ck.n > kSmallMaxRows || small_lds_bytes(ck.n, ld, ck.P, ck.adj_nnz, false) > kSmallMaxDynLds) return false;
            al = al && small_lds_bytes(ck.n, ld, ck.P, ck.adj_nnz, true) <= kSmallMaxDynLds;
        }
        A.al = al;
        A.nwg = P.K;
        A.xs = kSmallXcds;
        int r0 = 0;
        for (int k = 0; k < P.K; ++k) {
            const DevCone &ck = P.cones[k];
            A.wg[k] = SmallWg{ck.n, r0, ck.slot_off, ck.P, (int)ck.adj_nnz, ck.adj_ptr, ck.adj_low, ck.adj_col, ck.adj_slot};
            r0 += ck.n;
        }
        A.xbuf = W.partB;
        A.xcnt = reinterpret_cast<unsigned *>(W.partB + 2 * kSmallMaxWg * 16);
    }
    A.N = N; A.K = P.K; A.m = P.m; A.Ptot = P.Ptot; A.mg = P.mg; A.nadj = (int)a.adj_nnz;
    A.slot_g = reinterpret_cast<const int2 *>(P.slot_g);
    if (A.nwg == 1) A.wg[0] = SmallWg{N, 0, 0, P.Ptot, (int)a.adj_nnz, a.adj_ptr, a.adj_low, a.adj_col, a.adj_slot};
    A.Cw = P.Cw; A.Craw = P.Craw;
    A.loc1 = reinterpret_cast<const double2 *>(P.loc1); A.slot1 = reinterpret_cast<const double2 *>(P.slot1);
    A.loc_ptr = P.loc_ptr; A.loc_con = P.loc_con; A.slot_ptr = P.slot_ptr; A.slot_con = P.slot_con;
    A.loc_w = P.loc_w; A.slot_a = P.slot_a;
    A.glob = P.glob; A.con_ptr = P.con_ptr; A.con_slot = P.con_slot; A.con_w = P.con_w;
    A.b = P.b; A.lam = W.lam;
    A.cvs = W.cvs; A.rec = W.rec; A.uRD = W.uvt0; A.uDD = W.uvt1; A.uRR = W.uvt2;
    A.R = W.R; A.G0 = W.G[0]; A.G1 = W.G[1]; A.s0 = W.ls[0]; A.y0 = W.ly[0]; A.s1 = W.ls[1]; A.y1 = W.ly[1];
    A.par = W.par;
    A.nconst = nconst;
    if (ldo) *ldo = ld;
    return true;
}
bool small_alm_fits(const DevProblem &P, DevWork &W) {
    if (P.lp_cone >= 0) return false;   // an LP block: the multi-launch iteration (its own ADMM sweep)
    SmallArgs A{};
    return small_alm_args(P, W, A, nullptr);
}
int small_alm_workgroups(const DevProblem &P, DevWork &W) {
    SmallArgs A{};
    return small_alm_args(P, W, A, nullptr) ? A.nwg : 0;
}
template <int LD, bool AL, bool MC>
static int launch_small_ld(const SmallArgs &A, size_t lds, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(k_small_alm<LD, AL, MC>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSmallMaxDynLds) != hipSuccess) {
            snprintf(g_err, sizeof(g_err), "single-workgroup inner loop: LDS attribute refused");
            return -1;
        }
        attr = true;
    }
    if (A.nwg > 1 && hipMemsetAsync(A.xcnt, 0, sizeof(unsigned), st) != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "single-workgroup inner loop: exchange counter reset failed");
        return -1;
    }
    // one workgroup per cone at blocks 0, xs, 2 xs, ...: consecutive blocks go to consecutive XCDs,
    // so the cones' workgroups share one XCD's L2 (the blocks between leave at once)
    const int grid = A.nwg > 1 ? (A.nwg - 1) * A.xs + 1 : 1;
    hipLaunchKernelGGL((k_small_alm<LD, AL, MC>), dim3(grid), dim3(kSmallThreads), lds, st, A);
    LRS_CHECK_LAUNCH();
    return 0;
}
// One launch: the inner loop from the control block at ctrl_in to its exit; the final control
// block to ctrl_out, the last line search to ls_out, the iterate to W.R.
int launch_small_alm(const DevProblem &P, DevWork &W, const double *ctrl_in, double *ctrl_out, double *ls_out,
                     hipStream_t st) {
    SmallArgs A{};
    int ld = 0;
    if (!small_alm_args(P, W, A, &ld)) {
        snprintf(g_err, sizeof(g_err), "single-workgroup inner loop: the problem does not fit");
        return -1;
    }
    A.ctrl_in = ctrl_in;
    A.ctrl_out = ctrl_out;
    A.ls_out = ls_out;
    {
        const char *e = getenv("LRS_XWG_SPIN");
        A.spin_log2 = e ? std::max(-1, std::min(40, atoi(e))) : 26;   // -1: no wait at all (tests)
        const char *o = getenv("LRS_SMALL_ROWSORT");
        A.row_sort = o ? (atoi(o) != 0) : 1;
    }
    size_t lds = small_lds_bytes(A.N, ld, A.Ptot, A.nadj, A.al != 0);
    if (A.nwg > 1) {   // the largest cone's
        lds = 0;
        for (int k = 0; k < A.nwg; ++k) lds = std::max(lds, small_lds_bytes(A.wg[k].n, ld, A.wg[k].P, A.wg[k].nadj, A.al != 0));
    }
#define LRS_SMALL_LD(AL, MC)                                      \
    switch (ld) {                                                 \
    case 8: return launch_small_ld<8, AL, MC>(A, lds, st);        \
    case 16: return launch_small_ld<16, AL, MC>(A, lds, st);      \
    case 24: return launch_small_ld<24, AL, MC>(A, lds, st);      \
    case 32: return launch_small_ld<32, AL, MC>(A, lds, st);      \
    case 48: return launch_small_ld<48, AL, MC>(A, lds, st);      \
    default: return launch_small_ld<64, AL, MC>(A, lds, st);      \
    }
    if (A.nwg > 1) {
        if (A.al) { LRS_SMALL_LD(true, true) }
        LRS_SMALL_LD(false, true)
    }
    if (A.al) { LRS_SMALL_LD(true, false) }
    LRS_SMALL_LD(false, false)
#undef LRS_SMALL_LD
}

// Sharded solve: pack the listed rows (ld doubles each) into a contiguous buffer.
__global__ void __launch_bounds__(kBlock) k_pack_rows(int nrows, int ld, const int *__restrict__ rows,
                                                      const double *__restrict__ src, double *__restrict__ dst) {
    const long tot = (long)nrows * ld;
    for (long t = (long)blockIdx.x * kBlock + threadIdx.x; t < tot; t += (long)gridDim.x * kBlock) {
        const long q = t / ld, e = t - q * ld;
        dst[t] = src[(long)rows[q] * ld + e];
    }
}
int launch_pack_rows(int nrows, int ld, const int *rows, const double *src, double *dst, hipStream_t st) {
    if (nrows <= 0) return 0;
    hipLaunchKernelGGL(k_pack_rows, dim3(grid_elems((long)nrows * ld, 4)), dim3(kBlock), 0, st, nrows, ld, rows,
                       src, dst);
    LRS_CHECK_LAUNCH();
    return 0;
}
// Loopback transport (tests: several shards in one process on one GPU): out = sum of
// the shards' buffers in rank order.
struct SumSrc { const double *p[kMaxShards]; };
__global__ void __launch_bounds__(kBlock) k_sum_shards(int n, int world, SumSrc src, double *__restrict__ out) {
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        double v = 0.0;
        for (int q = 0; q < world; ++q) v += src.p[q][i];
        out[i] = v;
    }
}
int launch_sum_shards(int n, int world, const double *const *src, double *out, hipStream_t st) {
    if (world > kMaxShards) { snprintf(g_err, sizeof(g_err), "sum_shards: world %d", world); return -1; }
    SumSrc s{};
    for (int q = 0; q < world; ++q) s.p[q] = src[q];
    hipLaunchKernelGGL(k_sum_shards, dim3(grid_elems(n, 1)), dim3(kBlock), 0, st, n, world, s, out);
    LRS_CHECK_LAUNCH();
    return 0;
}

// ------------------------------------------------------------------------
// small helper kernels used by the host-driven phases
// ------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_resid(int m, const double *__restrict__ b, const double *__restrict__ x,
                                                  const double *__restrict__ mask, double *part, unsigned *ticket,
                                                  double *fin) {
    double acc[1] = {0.0};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < m; i += gridDim.x * kBlock) {
        const double d = b[i] - x[i];
        acc[0] += mask ? mask[i] * (d * d) : d * d;
    }
    partials_finalize<1>(acc, part, ticket, fin);
}
// averageUV (lorads_admm.c:372-377)
__global__ void __launch_bounds__(kBlock) k_avg(long n, const double *__restrict__ U, const double *__restrict__ V,
                                                double *__restrict__ R) {
    for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long)gridDim.x * kBlock)
        R[i] = (U[i] + V[i]) / 2;
}
// M1 = rho (cvs - cv - b) - lam in the reference's operation order (lorads_admm.c:568-581)
__global__ void __launch_bounds__(kBlock) k_admm_m1(int m, double rho, const double *__restrict__ b,
                                                    const double *__restrict__ cvs, const double *__restrict__ cv,
                                                    const double *__restrict__ lam, double *__restrict__ M1) {
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < m; i += gridDim.x * kBlock) {
        double v = -b[i];
        v = v + cvs[i];
        v = v + (-1.0) * cv[i];
        v = v * rho;
        M1[i] = v + (-1.0) * lam[i];
    }
}
__global__ void k_ls_only(const double *__restrict__ par, int K, const double *__restrict__ fin,
                          double *__restrict__ lsout) {
    __shared__ double ls[LS_N];
    if (threadIdx.x == 0) line_search(par, K, fin, ls);
    __syncthreads();
    if (threadIdx.x < LS_N) lsout[threadIdx.x] = ls[threadIdx.x];
}

int launch_resid(int m, const double *b, const double *x, hipStream_t st, const double *mask) {
    double *part = t_rpart;
    if (!part) {
        snprintf(g_err, sizeof(g_err), "launch_resid: no context scratch bound");
        return -1;
    }
    hipLaunchKernelGGL(k_resid, dim3(grid_elems(m, 1)), dim3(kBlock), 0, st, m, b, x, mask, part, ticket_ptr(T_RR + 40),
                       tmpfin_ptr() + TF_RESID);
    LRS_CHECK_LAUNCH();
    return 0;
}
int launch_avg(long n, const double *U, const double *V, double *R, hipStream_t st) {
    hipLaunchKernelGGL(k_avg, dim3(grid_elems(n, 4)), dim3(kBlock), 0, st, n, U, V, R);
    LRS_CHECK_LAUNCH();
    return 0;
}
int launch_admm_m1(int m, double rho, const double *b, const double *cvs, const double *cv, const double *lam,
                   double *M1, hipStream_t st) {
    hipLaunchKernelGGL(k_admm_m1, dim3(grid_elems(m, 1)), dim3(kBlock), 0, st, m, rho, b, cvs, cv, lam, M1);
    LRS_CHECK_LAUNCH();
    return 0;
}
// gather_q on the current (uvt0, uvt1, cvs, lam) + device line search -> lsres[0..]
int launch_ls_only(const DevProblem &P, DevWork &W, hipStream_t st) {
    double one[C_NCTRL] = {0};
    one[C_ACTIVE] = 1.0;
    if (hipMemcpyAsync(W.ctrl, one, sizeof(one), hipMemcpyHostToDevice, st) != hipSuccess) return -1;
    double *fin = fin_ptr();
    hipLaunchKernelGGL(k_alm_gather_q, dim3(grid_elems(P.m, 1)), dim3(kBlock), 0, st, P.m, P.K, P.con_ptr,
                       P.con_slot, P.con_w, W.uvt0, W.uvt1, P.b, W.cvs, W.lam, W.par, W.q1, W.q2, W.partB,
                       ticket_ptr(T_Q), fin + FIN_Q, W.ctrl);
    LRS_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_ls_only, dim3(1), dim3(64), 0, st, W.par, P.K, fin, W.lsres);
    LRS_CHECK_LAUNCH();
    return 0;
}
// direction kernel alone, reading ctrl[1] and writing ctrl[0] (white-box tests)
int launch_alm_dir_only(const DevProblem &P, DevWork &W, hipStream_t st) {
    hipLaunchKernelGGL(k_alm_dir, dim3(grid_elems(P.NRpad, 2)), dim3(kBlock), 0, st, P.NRpad, W.par,
                       W.ctrl + C_NCTRL, W.ctrl, W.lsres + LS_N, P.K, W.D, W.G[0], W.G[1], W.ls[0], W.ly[0],
                       W.ls[1], W.ly[1], fin_ptr());
    LRS_CHECK_LAUNCH();
    return 0;
}

// ---- device CG launchers
static StagePlan plan_cg_mv(const DevCone &c) {
    const double deg = c.n > 0 ? (double)c.adj_nnz / c.n : 0.0;
    const int T = team_size(c, deg, 4);
    StagePlan p;
    p.T = T;
    const long need = std::max(1L, ((long)c.nown * c.G * T + kRowBlock - 1) / kRowBlock);
    p.grid = (int)std::min<long>(need, kMaxPartialBlocks);
    p.small = true;
    return p;
}
int launch_cg_mv(const DevProblem &P, int cone, const double *w, const double *V, const double *Xin, double *Q,
                 double *part, const double *cgc, int guarded, hipStream_t st, int *nblk) {
    const DevCone &c = P.cones[cone];
    const StagePlan pl = plan_cg_mv(c);
    LRS_LAYOUT_SWITCH(c.G, c.E, {
        // the cone's computed rows [row0, row0 + nown) (a sharded solve's owned rows); the
        // neighbours' rows of V are addressed from the cone's first local row
        const long o = c.foff + (long)c.row0 * c.ld;
        hipLaunchKernelGGL((k_cg_mv<GG, EE, 4>), dim3(pl.grid), dim3(kRowBlock), 0, st, c.nown, c.ld,
                           c.adj_ptr + c.row0, c.adj_col, c.adj_slot, P.slot_ptr, P.slot_con, P.slot_a, w,
                           V + c.foff, Xin + o, Q + o, part, cgc, guarded, pl.T);
    });
    LRS_CHECK_LAUNCH();
    if (nblk) *nblk = pl.grid;
    return 0;
}
static inline int cg_grid(long nr) { return std::min(grid_elems(nr, 2), 1024); }
int launch_cg_nrm1(long nr, const double *b, double *part, hipStream_t st, int *nblk) {
    const int g = cg_grid(nr);
    hipLaunchKernelGGL(k_cg_nrm1, dim3(g), dim3(kBlock), 0, st, nr, b, part);
    LRS_CHECK_LAUNCH();
    *nblk = g;
    return 0;
}
int launch_cg_upd(long nr, double *X, double *r, const double *p, const double *Q, const double *partB, int nblkB,
                  double *partC, double *cgc, int par, int it, hipStream_t st, int *nblk) {
    const int g = cg_grid(nr);
    hipLaunchKernelGGL(k_cg_upd, dim3(g), dim3(kBlock), 0, st, nr, X, r, p, Q, partB, nblkB, partC, cgc, par, it);
    LRS_CHECK_LAUNCH();
    *nblk = g;
    return 0;
}
int launch_cg_conv(long nr, const double *r, double *p, const double *partC, int nblkC, double *cgc, double tol,
                   int par, int restart, hipStream_t st) {
    hipLaunchKernelGGL(k_cg_conv, dim3(cg_grid(nr)), dim3(kBlock), 0, st, nr, r, p, partC, nblkC, cgc, tol, par,
                       restart);
    LRS_CHECK_LAUNCH();
    return 0;
}
int launch_cg_resid(long nr, const double *b, const double *Q, double *r, double *p, double *partC, double *cgc,
                    const double *partA, int nblkA, int init, hipStream_t st, int *nblk) {
    const int g = cg_grid(nr);
    hipLaunchKernelGGL(k_cg_resid, dim3(g), dim3(kBlock), 0, st, nr, b, Q, r, p, partC, cgc, partA, nblkA, init);
    LRS_CHECK_LAUNCH();
    *nblk = g;
    return 0;
}
int launch_cg_resid2(long nr, const double *r, double *p, const double *partC, int nblkC, double *cgc, double tol,
                     int par, int init, hipStream_t st) {
    hipLaunchKernelGGL(k_cg_resid2, dim3(cg_grid(nr)), dim3(kBlock), 0, st, nr, r, p, partC, nblkC, cgc, tol, par,
                       init);
    LRS_CHECK_LAUNCH();
    return 0;
}


// ------------------------------------------------------------------------
// Single-workgroup ADMM half-step (small cones: the theta class).  ONE launch of one workgroup
// runs LORADSUpdateSDPVarOne (lorads_admm.c:564-616) for one cone and side -- the right-hand
// side, the whole CGSolve (linalg/lorads_cgs.c:128-287, as the device-resident CG above: the
// same tolerance test, restart every 20 iterations and iteration count) -- and the cone's
// constraint refresh of LORADSUpdateSDPVar (lorads_alg_common.c:310-314 / :321-323), where the
// multi-launch path takes four launches per CG iteration and a host poll per batch (theta3x3:
// ~20 us a CG iteration).  Layout: the fixed factor Y in LDS (rows of r doubles,
// odd pitch); the operand x (p, or X at a restart and for the refresh), X, r, p, Q and b of a row
// in the registers of the 16-lane group that owns it (row i: group i % kScG; column c: lane
// c % 16, element c / 16); the constraint values (compact order), the per-slot products and the
// lists of DevCone::cg_* in LDS.  The operator x -> x + A*(A(sym(x Y^T))) Y (linSysProduct,
// lorads_admm.c:471-486) runs in four phases: (A) every row's group forms x_i . Y_j for each
// constraint slot (i, j) of its row, so a slot's 1/2 (x_p . Y_q + x_q . Y_p) comes from its two
// rows' halves; (B) the constraint values from the slots (a thread per short constraint, a wave
// per long one); (C) A*(w) on the constraint slots; (D) Q_i = sum_j S_ij Y_j + x_i in the
// adjacency's column order (k_cg_mv's order).  Sums over the block: wave sums, then the eight
// wave values in wave order (deterministic).
// ------------------------------------------------------------------------
#ifndef LRS_SC_NT
#define LRS_SC_NT 1024
#endif
constexpr int kScT = LRS_SC_NT;          // threads
constexpr int kScL = 16;                 // lanes per factor row
constexpr int kScG = kScT / kScL;        // row groups
constexpr int kScW = kScT / 64;          // waves
constexpr int kScMaxDynLds = 152 * 1024;

struct SmallCgArgs {
    int n, r, ld, rS, side, maxit, ncs, ncl, ns, nce, nsc, nadj, cconst, cslot;
    long foff;
    double rho, tol, calpha;
    const int *cadj_ptr, *cadj, *cl_con, *cl_ptr, *ce, *sp, *sj, *cc_ptr, *cc;
    const double *ce_w, *sa, *Craw, *b, *lam;
    double *cvs, *cvc, *U, *V, *cg_b, *cgc;
};
// One launch of k_small_cg: block k runs the half-step of a[k] (several cones' half-steps side
// by side where no constraint spans two cones: their solves and refreshes touch disjoint rows
// and constraints, so the reference's cone-by-cone sweep gives the same values)
struct SmallCgBatch {
    SmallCgArgs a[kSmallMaxWg];
};

static size_t small_cg_lds(int n, int rS, int ncl, int ncs, int nce, int nsc, int nadj) {
    const size_t dbl = (size_t)n * rS + ncl + 2 * (size_t)ncs + nce + nsc + rS + 2 * kScW;
    const size_t in = (size_t)(n + 1) + nadj + (ncl + 1) + nce + (ncs + 1) + nsc;
    return dbl * sizeof(double) + in * sizeof(int);
}

// block-wide global -> LDS copy with KB loads in flight per thread: a loop of one load per
// iteration (trip count unknown to the compiler) waits one memory trip per element it copies
template <int KB, typename T>
__device__ __forceinline__ void sc_stage(T *dst, const T *__restrict__ src, int n) {
    for (int t0 = (int)threadIdx.x; t0 < n; t0 += KB * kScT) {
        T v[KB];
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            const int t = t0 + u * kScT;
            v[u] = src[t < n ? t : t0];
        }
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            const int t = t0 + u * kScT;
            if (t < n) dst[t] = v[u];
        }
    }
}

// acc += sum_e S_e Y_j over one row's constraint slots e in [e0, e1) in entry order, four
// entries a pass (their indices, S values and operand rows loaded together)
template <int EL>
__device__ __forceinline__ void sc_row_apply(int e0, int e1, const int *cadj, const double *T, const double *Ys,
                                             int rS, int r, int l, double (&acc)[EL]) {
    for (int e = e0; e < e1; e += 4) {
        int pk[4];
        double sv[4], y[4][EL];
#pragma unroll
        for (int u = 0; u < 4; ++u) pk[u] = cadj[min(e + u, e1 - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            sv[u] = T[pk[u] & 0xffff];
#pragma unroll
            // unconditional (selects below); columns past the row pitch clamped into the row, whose
            // words are finite (Y or the zeroed pad), so a masked column adds 0 * finite = +-0
            for (int k = 0; k < EL; ++k) y[u][k] = Ys[(pk[u] >> 16) * rS + min(l + kScL * k, rS - 1)];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < EL; ++k) {
                // the test selects the coefficient, not the load (see prod_pass): a masked
                // entry or column adds +-0
                const double sc = (e + u < e1 && l + kScL * k < r) ? sv[u] : 0.0;
                acc[k] += sc * y[u][k];
            }
    }
}

template <int EL, int RPG>
__global__ void __launch_bounds__(kScT) k_small_cg(SmallCgBatch Bt) {
    const SmallCgArgs &A = Bt.a[blockIdx.x];
    extern __shared__ double smem[];
    const int n = A.n, r = A.r, rS = A.rS;
    double *Ys = smem;                         // [n][rS] the fixed factor
    double *wv = Ys + (long)n * rS;            // [ncl] constraint values (or M1), compact order
    double *T = wv + A.ncl;                    // [ncs][2] half products; then S on [0, ncs)
    double *cew = T + 2 * A.ncs;               // [nce]
    double *sav = cew + A.nce;                 // [nsc]
    double *csum = sav + A.nsc;                // [rS] column sums of Y (constant objective)
    double *red = csum + rS;                   // [2][kScW]
    int *cap = reinterpret_cast<int *>(red + 2 * kScW);   // [n + 1]
    int *cadj = cap + n + 1;                   // [nadj]
    int *clp = cadj + A.nadj;                  // [ncl + 1]
    int *ce = clp + A.ncl + 1;                 // [nce]
    int *sp = ce + A.nce;                      // [ncs + 1]
    int *sj = sp + A.ncs + 1;                  // [nsc]
    const int tid = threadIdx.x, g = tid / kScL, l = tid % kScL, wid = tid >> 6, lane = tid & 63;
    // diagnostics build: thread 0 adds its phases' wall-clock ticks into g_phase[1][8..13]
    // (staging, right-hand side, first residual, CG iterations, refresh), iterations into
    // [1][14], launches into [1][15]
#ifdef LRS_PHASE_TIMING
    unsigned long long sc_t = wall_clock64();
#define LRS_SC_T(q) do { if (tid == 0) { const unsigned long long t_ = wall_clock64(); g_phase[1][q] += t_ - sc_t; sc_t = t_; } } while (0)
#else
#define LRS_SC_T(q) do { } while (0)
#endif
    double *X = (A.side ? A.V : A.U) + A.foff;
    const double *Yg = (A.side ? A.U : A.V) + A.foff;
    // stage the fixed factor and the lists (batched loads: one memory trip per ~4K elements)
    for (int t0 = tid; t0 < n * r; t0 += 8 * kScT) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = min(t0 + u * kScT, n * r - 1), i = t / r, c = t - i * r;
            v[u] = Yg[(long)i * A.ld + c];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = t0 + u * kScT, i = t / r, c = t - i * r;
            if (t < n * r) Ys[i * rS + c] = v[u];
        }
    }
    if (rS > r)   // the pad columns [r, rS): zero (the row loops read them unmasked)
        for (int t = tid; t < n * (rS - r); t += kScT) Ys[(t / (rS - r)) * rS + r + t % (rS - r)] = 0.0;
    sc_stage<8>(cap, A.cadj_ptr, n + 1);
    sc_stage<8>(cadj, A.cadj, A.nadj);
    sc_stage<8>(clp, A.cl_ptr, A.ncl + 1);
    sc_stage<8>(ce, A.ce, A.nce);
    sc_stage<8>(cew, A.ce_w, A.nce);
    sc_stage<8>(sp, A.sp, A.ncs + 1);
    sc_stage<8>(sj, A.sj, A.nsc);
    sc_stage<8>(sav, A.sa, A.nsc);
    // this group's rows of X (zero past r and n)
    double x[RPG][EL], rv[RPG][EL], pv[RPG][EL], Q[RPG][EL], bv[RPG][EL];
#pragma unroll
    for (int q = 0; q < RPG; ++q)
#pragma unroll
        for (int k = 0; k < EL; ++k) {
            const int i = g + kScG * q, c = l + kScL * k;
            x[q][k] = (i < n && c < r) ? X[(long)i * A.ld + c] : 0.0;
            rv[q][k] = pv[q][k] = Q[q][k] = bv[q][k] = 0.0;
        }
    int rp = 0;
    auto block_sum = [&](double v) -> double {
        v = wave_sum(v);
        if (lane == 0) red[rp * kScW + wid] = v;
        __syncthreads();
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kScW; ++w) s += red[rp * kScW + w];
        rp ^= 1;
        return s;
    };
    // (A) x_i . Y_j per constraint slot (i, j): half 0 from the slot's lower row, 1 from its upper
    // the operand is p (usep) or x: selected per row, not copied (a copy of the block's rows
    // spills at EL 2 / RPG 8)
    auto prod_pass = [&](bool usep) {
#pragma unroll
        for (int q = 0; q < RPG; ++q) {
            const int i = g + kScG * q;
            if (i >= n) continue;   // group-uniform
            double xq[EL];
#pragma unroll
            for (int k = 0; k < EL; ++k) xq[k] = usep ? pv[q][k] : x[q][k];
            // four entries a pass: their index, operand loads and cross-lane sums overlap
            const int e1 = cap[i + 1];
            for (int e = cap[i]; e < e1; e += 4) {
                int pk[4];
                double d[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) pk[u] = cadj[min(e + u, e1 - 1)];
                // no branch around a load (the compiler sinks a load into its branch and then
                // waits for it before the next one issues: eight serial LDS round trips a pass):
                // columns past r hold x = 0 exactly and read the zeroed pad, or (past the row
                // pitch) are clamped into the row: finite words, so their products are +-0 (an
                // unclamped read past the last row would reach wv / T, not yet written)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int j = pk[u] >> 16;
                    d[u] = 0.0;
#pragma unroll
                    for (int k = 0; k < EL; ++k) d[u] += xq[k] * Ys[j * rS + min(l + kScL * k, rS - 1)];
                }
                {
                    // entry u's total in lanes 4u..4u+3; lane 4u stores it
                    const double v = group_sum4<kScL>(d, l);
                    const int u = l >> 2;
                    const int pku = u == 0 ? pk[0] : (u == 1 ? pk[1] : (u == 2 ? pk[2] : pk[3]));
                    if ((l & 3) == 0 && e + u < e1) T[2 * (pku & 0xffff) + ((pku >> 16) <= i ? 0 : 1)] = v;
                }
            }
        }
    };
    // (B) constraint values sum_e w_e d_e (k_auv_con's entry order)
    auto con_pass = [&]() {
        for (int j = tid; j < A.ns; j += kScT) {
            double v = 0.0;
            for (int e = clp[j]; e < clp[j + 1]; ++e) {
                const int pk = ce[e], cs = pk >> 1;
                const double d = (pk & 1) ? T[2 * cs] : 0.5 * (T[2 * cs] + T[2 * cs + 1]);
                v += cew[e] * d;
            }
            wv[j] = v;
        }
        for (int j = A.ns + wid; j < A.ncl; j += kScW) {   // wave-uniform
            double v = 0.0;
            for (int e = clp[j] + lane; e < clp[j + 1]; e += 64) {
                const int pk = ce[e], cs = pk >> 1;
                const double d = (pk & 1) ? T[2 * cs] : 0.5 * (T[2 * cs] + T[2 * cs + 1]);
                v += cew[e] * d;
            }
            v = wave_sum(v);
            if (lane == 0) wv[j] = v;
        }
    };
    // (C) S = A*(w) on the constraint slots (sdpDataWSum without C), into T[0, ncs)
    auto slot_pass = [&]() {
        for (int t = tid; t < A.ncs; t += kScT) {
            double v = 0.0;
            for (int e = sp[t]; e < sp[t + 1]; ++e) v += wv[sj[e]] * sav[e];
            T[t] = v;
        }
    };
    // (D) Q = S Y + x on the group's rows; returns this thread's part of <x, Q>
    auto apply_pass = [&](bool usep, double (&Qv)[RPG][EL]) -> double {
        double dot = 0.0;
#pragma unroll
        for (int q = 0; q < RPG; ++q) {
            const int i = g + kScG * q;
            double acc[EL];
#pragma unroll
            for (int k = 0; k < EL; ++k) acc[k] = 0.0;
            if (i < n) sc_row_apply<EL>(cap[i], cap[i + 1], cadj, T, Ys, rS, r, l, acc);
#pragma unroll
            for (int k = 0; k < EL; ++k) {
                const double xk = usep ? pv[q][k] : x[q][k];
                double v = acc[k] * 1.0;
                v += 1.0 * xk;
                Qv[q][k] = v;
                dot += xk * v;
            }
        }
        return dot;
    };

    // ---- right-hand side (lorads_admm.c:566-598): M1 = rho (cvs - A_k - b) - lam (compact),
    // S = A*(M1) on the constraint slots, M2 = S Y + C Y - rho Y, b = -M2 / rho
    const double rho = A.rho;
    for (int j0 = tid; j0 < A.ncl; j0 += 4 * kScT) {   // four constraints a thread in flight
        int gi[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) gi[u] = A.cl_con[min(j0 + u * kScT, A.ncl - 1)];
        double bq[4], cq[4], kq[4], lq[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            bq[u] = A.b[gi[u]];
            cq[u] = A.cvs[gi[u]];
            kq[u] = A.cvc[gi[u]];
            lq[u] = A.lam[gi[u]];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + u * kScT;
            if (j >= A.ncl) break;
            double v = -bq[u];
            v = v + cq[u];
            v = v + (-1.0) * kq[u];
            v = v * rho;
            wv[j] = v + (-1.0) * lq[u];
        }
    }
    __syncthreads();   // Ys and the lists staged, M1 formed
    LRS_SC_T(8);
    if (A.cconst)
        for (int c = tid; c < r; c += kScT) {
            double s = 0.0;
            for (int i = 0; i < n; ++i) s += Ys[i * rS + c];
            csum[c] = s;
        }
    slot_pass();
    __syncthreads();
    {
        const double alpha = A.cconst == 1 ? A.Craw[A.cslot] : A.calpha;
        double bn = 0.0;
#pragma unroll
        for (int q = 0; q < RPG; ++q) {
            const int i = g + kScG * q;
            double acc[EL];
#pragma unroll
            for (int k = 0; k < EL; ++k) acc[k] = 0.0;
            if (i < n) {
                sc_row_apply<EL>(cap[i], cap[i + 1], cadj, T, Ys, rS, r, l, acc);
                if (!A.cconst)
                    for (int e = A.cc_ptr[i]; e < A.cc_ptr[i + 1]; ++e) {
                        const int j = A.cc[2 * e];
                        const double cv = A.Craw[A.cc[2 * e + 1]];
#pragma unroll
                        for (int k = 0; k < EL; ++k) {
                            const int c = l + kScL * k;
                            if (c < r) acc[k] += cv * Ys[j * rS + c];
                        }
                    }
            }
#pragma unroll
            for (int k = 0; k < EL; ++k) {
                const int c = l + kScL * k;
                const bool ok = i < n && c < r;
                double m2 = acc[k] * 1.0;
                m2 += (-rho) * (ok ? Ys[i * rS + c] : 0.0);
                if (A.cconst && ok) m2 = alpha * csum[c] + 1.0 * m2;
                const double bvk = ok ? (-1.0 / rho) * m2 : 0.0;
                bv[q][k] = bvk;
                if (ok) A.cg_b[A.foff + (long)i * A.ld + c] = bvk;
                bn += fabs(bvk);
            }
        }
        bn = block_sum(bn);
        LRS_SC_T(9);

        // ---- CGSolve with ONE operator site (the whole operator inlined once keeps the kernel
        // inside the instruction cache; three inlined copies made it 96 KB and every CG iteration
        // missed): mode 0 the first residual r = b - M X, 1 an iteration's M p, 2 the restart's
        // r = b - M X (lorads_cgs.c: every 20 iterations, then its beta = 1 step p = r + p),
        // 3 the cone's refresh A_k <- A_k(sym(U V^T)) from the solved side (the operator's
        // first two passes).  The arithmetic and the block sums' order are CGSolve's.
        int mode = 0, it = 0, iters = 0;   // block-uniform
        double qtr[2] = {0.0, 0.0};
        for (;;) {
            const bool usep = mode == 1;
            __syncthreads();   // T free (the previous apply pass is done)
#ifdef LRS_PHASE_TIMING
            // diagnostics: the operator's four passes of the first residual into g_phase[1][4..7]
            const bool pt = mode == 0 && tid == 0;
            unsigned long long p_t = pt ? wall_clock64() : 0;
#define LRS_SC_P(q) do { if (pt) { const unsigned long long t_ = wall_clock64(); g_phase[1][q] += t_ - p_t; p_t = t_; } } while (0)
#else
#define LRS_SC_P(q) do { } while (0)
#endif
            prod_pass(usep);
            __syncthreads();
            LRS_SC_P(4);
            con_pass();
            if (mode == 3) break;
            __syncthreads();
            LRS_SC_P(5);
            slot_pass();
            __syncthreads();
            LRS_SC_P(6);
            const double dot = apply_pass(usep, Q);
#ifdef LRS_PHASE_TIMING
            __syncthreads();
#endif
            LRS_SC_P(7);
#undef LRS_SC_P
            if (mode == 1) {
                const int par = it & 1;
                const double pq = block_sum(dot);
                const double alph = qtr[par] / pq;
                iters = it + 1;
                double rr1 = 0.0;
#pragma unroll
                for (int q = 0; q < RPG; ++q)
#pragma unroll
                    for (int kk = 0; kk < EL; ++kk) {
                        x[q][kk] = alph * pv[q][kk] + 1.0 * x[q][kk];
                        const double ri = -alph * Q[q][kk] + 1.0 * rv[q][kk];
                        rv[q][kk] = ri;
                        rr1 += ri * ri;
                    }
                rr1 = block_sum(rr1);
                const double resi = sqrt(rr1);
                if (resi / bn < A.tol || resi != resi) {
                    mode = 3;
                } else if (it % 20 != 0) {
                    const double beta = rr1 / qtr[par];
#pragma unroll
                    for (int q = 0; q < RPG; ++q)
#pragma unroll
                        for (int kk = 0; kk < EL; ++kk) pv[q][kk] = 1.0 * rv[q][kk] + beta * pv[q][kk];
                    qtr[par ^ 1] = rr1;
                    ++it;
                    mode = it < A.maxit ? 1 : 3;
                } else {
                    mode = 2;
                }
            } else {   // r = b - M X, p = r
                double rr = 0.0;
#pragma unroll
                for (int q = 0; q < RPG; ++q)
#pragma unroll
                    for (int kk = 0; kk < EL; ++kk) {
                        const double ri = 1.0 * bv[q][kk] + -1.0 * Q[q][kk];
                        rv[q][kk] = ri;
                        pv[q][kk] = ri;
                        rr += ri * ri;
                    }
                rr = block_sum(rr);
                if (mode == 0) {
                    qtr[0] = rr;
                    mode = (!(sqrt(rr) / bn < A.tol) && A.maxit > 0) ? 1 : 3;
                    LRS_SC_T(10);
                } else {
                    const int par = it & 1;
                    const double beta = rr / rr;
#pragma unroll
                    for (int q = 0; q < RPG; ++q)
#pragma unroll
                        for (int kk = 0; kk < EL; ++kk) pv[q][kk] = 1.0 * rv[q][kk] + beta * pv[q][kk];
                    qtr[par ^ 1] = rr;
                    ++it;
                    mode = it < A.maxit ? 1 : 3;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < RPG; ++q)
#pragma unroll
            for (int kk = 0; kk < EL; ++kk) {
                const int i = g + kScG * q, c = l + kScL * kk;
                if (i < n && c < r) X[(long)i * A.ld + c] = x[q][kk];
            }
        LRS_SC_T(11);
        if (tid == 0) {
            // a batch launch (one block per cone, launch_small_cg_batch) has no single count to report:
            // CG_ITERS is the one-cone launch's (lrs_op_admm_half reads it); every launch adds its
            // cones' counts to CG_TOTAL, the one the ADMM log and lrs_result use
            if (gridDim.x == 1) A.cgc[CG_ITERS] = iters;
            atomicAdd(A.cgc + CG_TOTAL, (double)iters);   // several cones' blocks: integers, exact in any order
#ifdef LRS_PHASE_TIMING
            g_phase[1][14] += iters;
            g_phase[1][15] += 1;
#endif
        }
    }
    // ---- the refresh's writes: CVS += new - old per constraint of the cone (values from mode 3)
    __syncthreads();
    for (int j0 = tid; j0 < A.ncl; j0 += 4 * kScT) {
        int gi[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) gi[u] = A.cl_con[min(j0 + u * kScT, A.ncl - 1)];
        double cq[4], kq[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            cq[u] = A.cvs[gi[u]];
            kq[u] = A.cvc[gi[u]];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + u * kScT;
            if (j >= A.ncl) break;
            const double v = wv[j];
            A.cvs[gi[u]] = (cq[u] - kq[u]) + v;
            A.cvc[gi[u]] = v;
        }
    }
    LRS_SC_T(12);
#undef LRS_SC_T
}

// The instantiated (elements per lane, rows per group) for a cone, 0 if none: EL 1 with up to
// 8 rows a group, EL 2 up to 6, EL 3 up to 4, EL 4 up to 2 (five register arrays of EL x RPG
// doubles at two waves a SIMD; the larger products spill)
static int small_cg_rpg(int EL, int RPG) {
    if constexpr (kScT == 1024) {
        // 128 VGPRs a lane at 1024 threads: the variants that do not spill
        const int lim = EL == 1 ? 6 : (EL == 2 ? 3 : (EL == 3 ? 2 : 0));
        const int rpg = RPG <= 2 ? 2 : (RPG <= 3 ? 3 : (RPG <= 4 ? 4 : (RPG <= 6 ? 6 : 8)));
        return (RPG >= 1 && rpg <= lim) ? rpg : 0;
    }
    const int lim = EL == 1 ? 8 : (EL == 2 ? 6 : (EL == 3 ? 4 : (EL == 4 ? 2 : 0)));
    const int rpg = RPG <= 2 ? 2 : (RPG <= 4 ? 4 : (RPG <= 6 ? 6 : 8));
    return (RPG >= 1 && rpg <= lim) ? rpg : 0;
}
bool small_cg_fits(const DevProblem &P, int cone) {
    const DevCone &c = P.cones[cone];
    if (P.shard || !c.cg_ok || c.dense_c == 1 || c.r < 1) return false;
    const int EL = (c.r + kScL - 1) / kScL, RPG = (c.n + kScG - 1) / kScG;
    if (!small_cg_rpg(EL, RPG)) return false;
    const int rS = c.r | 1;
    return small_cg_lds(c.n, rS, c.cg_ncl, c.cg_ncs, c.cg_nce, c.cg_nsc, c.cg_nadj) <= (size_t)kScMaxDynLds;
}

template <int EL, int RPG>
static int launch_small_cg_t(const SmallCgBatch &A, int nb, size_t lds, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(k_small_cg<EL, RPG>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kScMaxDynLds) != hipSuccess) {
            snprintf(g_err, sizeof(g_err), "single-workgroup ADMM half-step: LDS attribute refused");
            return -1;
        }
        attr = true;
    }
    hipLaunchKernelGGL((k_small_cg<EL, RPG>), dim3(nb), dim3(kScT), lds, st, A);
    LRS_CHECK_LAUNCH();
    return 0;
}

static void small_cg_args(const DevProblem &P, DevWork &W, int cone, int side, double rho, double tol, int maxit,
                          SmallCgArgs &A) {
    const DevCone &c = P.cones[cone];
    A = SmallCgArgs{};
    A.n = c.n; A.r = c.r; A.ld = c.ld; A.rS = c.r | 1; A.side = side; A.maxit = maxit;
    A.ncs = c.cg_ncs; A.ncl = c.cg_ncl; A.ns = c.cg_ns; A.nce = c.cg_nce; A.nsc = c.cg_nsc; A.nadj = c.cg_nadj;
    A.cconst = c.dense_c == 2 ? 2 : c.cg_cconst;
    A.cslot = c.cg_cslot;
    A.foff = c.foff;
    A.rho = rho; A.tol = tol;
    A.calpha = P.dense_scale * c.c_alpha;
    A.cadj_ptr = c.cg_cadj_ptr; A.cadj = c.cg_cadj; A.cl_con = c.cg_cl_con; A.cl_ptr = c.cg_cl_ptr; A.ce = c.cg_ce;
    A.sp = c.cg_sp; A.sj = c.cg_sj; A.cc_ptr = c.cg_cc_ptr; A.cc = c.cg_cc; A.ce_w = c.cg_ce_w; A.sa = c.cg_sa;
    A.Craw = P.Craw; A.b = P.b; A.lam = W.lam;
    A.cvs = W.cvs; A.cvc = W.cvc + (long)cone * P.m; A.U = W.U; A.V = W.V; A.cg_b = W.cg_b; A.cgc = W.cgc;
}
static int small_cg_variant(const DevCone &c) {   // EL * 16 + rows per group, 0 if none
    const int EL = (c.r + kScL - 1) / kScL, RPG = (c.n + kScG - 1) / kScG;
    const int rpg = small_cg_rpg(EL, RPG);
    return rpg ? EL * 16 + rpg : 0;
}
static int launch_small_cg_v(int v, const SmallCgBatch &B, int nb, size_t lds, hipStream_t st) {
    switch (v) {
    case 1 * 16 + 2: return launch_small_cg_t<1, 2>(B, nb, lds, st);
    case 1 * 16 + 4: return launch_small_cg_t<1, 4>(B, nb, lds, st);
    case 1 * 16 + 6: return launch_small_cg_t<1, 6>(B, nb, lds, st);
    case 1 * 16 + 8: return launch_small_cg_t<1, 8>(B, nb, lds, st);
    case 2 * 16 + 2: return launch_small_cg_t<2, 2>(B, nb, lds, st);
#if LRS_SC_NT == 1024
    case 1 * 16 + 3: return launch_small_cg_t<1, 3>(B, nb, lds, st);
    case 2 * 16 + 3: return launch_small_cg_t<2, 3>(B, nb, lds, st);
#endif
    case 2 * 16 + 4: return launch_small_cg_t<2, 4>(B, nb, lds, st);
    case 2 * 16 + 6: return launch_small_cg_t<2, 6>(B, nb, lds, st);
    case 3 * 16 + 2: return launch_small_cg_t<3, 2>(B, nb, lds, st);
    case 3 * 16 + 4: return launch_small_cg_t<3, 4>(B, nb, lds, st);
    case 4 * 16 + 2: return launch_small_cg_t<4, 2>(B, nb, lds, st);
    default:
        snprintf(g_err, sizeof(g_err), "single-workgroup ADMM half-step: no variant %d", v);
        return -1;
    }
}

int launch_small_cg(const DevProblem &P, DevWork &W, int cone, int side, double rho, double tol, int maxit,
                    hipStream_t st) {
    if (!small_cg_fits(P, cone)) {
        snprintf(g_err, sizeof(g_err), "single-workgroup ADMM half-step: cone %d does not fit", cone);
        return -1;
    }
    const DevCone &c = P.cones[cone];
    SmallCgBatch B{};
    small_cg_args(P, W, cone, side, rho, tol, maxit, B.a[0]);
    const SmallCgArgs &A = B.a[0];
    const size_t lds = small_cg_lds(c.n, A.rS, A.ncl, A.ncs, A.nce, A.nsc, A.nadj);
    return launch_small_cg_v(small_cg_variant(c), B, 1, lds, st);
}

// Every cone's half-step on one side in one launch (a block a cone): the cones each fit the
// single-workgroup kernel with the same variant, no constraint spans two cones (DevProblem::cone_sep).
bool small_cg_batch_fits(const DevProblem &P) {
    if (P.K < 2 || P.K > kSmallMaxWg || !P.cone_sep || P.lp_cone >= 0) return false;
    const int v = small_cg_fits(P, 0) ? small_cg_variant(P.cones[0]) : 0;
    if (!v) return false;
    for (int k = 1; k < P.K; ++k)
        if (!small_cg_fits(P, k) || small_cg_variant(P.cones[k]) != v) return false;
    return true;
}
int launch_small_cg_batch(const DevProblem &P, DevWork &W, int side, double rho, double tol, int maxit,
                          hipStream_t st) {
    if (!small_cg_batch_fits(P)) {
        snprintf(g_err, sizeof(g_err), "single-workgroup ADMM half-steps: the cones do not fit one launch");
        return -1;
    }
    SmallCgBatch B{};
    size_t lds = 0;
    for (int k = 0; k < P.K; ++k) {
        small_cg_args(P, W, k, side, rho, tol, maxit, B.a[k]);
        const SmallCgArgs &A = B.a[k];
        lds = std::max(lds, small_cg_lds(A.n, A.rS, A.ncl, A.ncs, A.nce, A.nsc, A.nadj));
    }
    return launch_small_cg_v(small_cg_variant(P.cones[0]), B, P.K, lds, st);
}

// ------------------------------------------------------------------------
// The ADMM iteration's evaluation for small cones in one launch (LORADSCalObjUV_ADMM
// lorads_admm.c:398-410 + update_dimacs_admm on R = (U + V) / 2): block k takes cone k --
// R = (U + V) / 2 of its rows (into W.R and LDS), R_p . R_q on its constraint slots (the
// k_small_cg lists, DevCone::cg_*), each of its constraints' A(R R^T) in entry order (the
// gather's arithmetic) into A(X) and the cone's share, and the cone's partial sums
// {sum (b - A(X))^2, <C, R R^T>, sum b lambda} over its constraints.  Cones whose constraints
// each lie in one cone (DevProblem::cone_sep) and together cover all m; the host adds the
// cones' partials in cone order.
// ------------------------------------------------------------------------
struct SmallEvalCone {
    int n, r, ld, ncs, ncl, cconst, cslot;
    long foff;
    double calpha;
    const int *cadj_ptr, *cadj, *cl_con, *cl_ptr, *ce, *cc_ptr, *cc;
    const double *ce_w;
};
struct SmallEvalArgs {
    SmallEvalCone c[kSmallMaxWg];
    int m;
    const double *U, *V, *b, *lam, *Craw;
    double *R, *cvs, *cvc, *out;   // out: [K][4]
};
constexpr int kSeT = 256;
__global__ void __launch_bounds__(kSeT) k_small_eval(SmallEvalArgs A) {
    const int k = blockIdx.x, tid = threadIdx.x;
    const SmallEvalCone &C = A.c[k];
    const int n = C.n, r = C.r;
    extern __shared__ __attribute__((aligned(16))) double se[];
    double *Rs = se;                   // [n][r]
    double *T = Rs + (long)n * r;      // [ncs] slot values
    double *cs = T + C.ncs;            // [r] column sums (constant objective)
    for (int t = tid; t < n * C.ld; t += kSeT) {   // every column of the rows, as k_avg
        const int i = t / C.ld, c = t - i * C.ld;
        const long o = C.foff + t;
        const double v = (A.U[o] + A.V[o]) / 2;
        A.R[o] = v;
        if (c < r) Rs[(long)i * r + c] = v;
    }
    __syncthreads();
    // the lower constraint slots of each row: T[slot] = R_i . R_j (a thread a row)
    for (int i = tid; i < n; i += kSeT)
        for (int q = C.cadj_ptr[i]; q < C.cadj_ptr[i + 1]; ++q) {
            const int w = C.cadj[q], j = w >> 16;
            if (j > i) continue;
            double d = 0.0;
            for (int c = 0; c < r; ++c) d += Rs[(long)i * r + c] * Rs[(long)j * r + c];
            T[w & 0xffff] = d;
        }
    if (C.cconst && tid < r) {
        double t = 0.0;
        for (int i = 0; i < n; ++i) t += Rs[(long)i * r + tid];
        cs[tid] = t;
    }
    __syncthreads();
    double acc[3] = {0.0, 0.0, 0.0};
    for (int j = tid; j < C.ncl; j += kSeT) {
        double v = 0.0;
        for (int e = C.cl_ptr[j]; e < C.cl_ptr[j + 1]; ++e) v += C.ce_w[e] * T[C.ce[e] >> 1];
        const int gi = C.cl_con[j];
        A.cvs[gi] = v;
        A.cvc[(long)k * A.m + gi] = v;
        const double d = A.b[gi] - v;
        acc[0] += d * d;
        acc[2] += A.b[gi] * A.lam[gi];
    }
    if (C.cconst) {
        if (tid == 0) {
            const double a = C.cconst == 2 ? C.calpha : A.Craw[C.cslot];
            double t = 0.0;
            for (int c = 0; c < r; ++c) t += cs[c] * cs[c];
            acc[1] = a * t;
        }
    } else {
        for (int i = tid; i < n; i += kSeT)
            for (int q = C.cc_ptr[i]; q < C.cc_ptr[i + 1]; ++q) {
                const int j = C.cc[2 * q], sl = C.cc[2 * q + 1];
                double d = 0.0;
                for (int c = 0; c < r; ++c) d += Rs[(long)i * r + c] * Rs[(long)j * r + c];
                acc[1] += A.Craw[sl] * d;
            }
    }
    double s3[3];
    block_reduce<3, kSeT>(acc, s3);
    if (tid == 0)
        for (int q = 0; q < 3; ++q) A.out[4 * k + q] = s3[q];
}
static size_t small_eval_lds(const DevCone &c) { return ((size_t)c.n * c.r + c.cg_ncs + c.r) * sizeof(double); }
bool small_eval_fits(const DevProblem &P) {
    if (P.shard || P.K > kSmallMaxWg || (P.K > 1 && !P.cone_sep) || P.lp_cone >= 0) return false;
    long ncl = 0;
    for (int k = 0; k < P.K; ++k) {
        const DevCone &c = P.cones[k];
        if (!c.cg_ok || c.dense_c == 1 || c.n > kScMaxN || small_eval_lds(c) > 64 * 1024) return false;
        ncl += c.cg_ncl;
    }
    return ncl == P.m;   // every constraint in one cone's list
}
int launch_small_eval(const DevProblem &P, DevWork &W, const double *U, const double *V, double *out, hipStream_t st) {
    if (!small_eval_fits(P)) {
        snprintf(g_err, sizeof(g_err), "single-workgroup ADMM evaluation: the cones do not fit");
        return -1;
    }
    SmallEvalArgs A{};
    size_t lds = 0;
    for (int k = 0; k < P.K; ++k) {
        const DevCone &c = P.cones[k];
        A.c[k] = SmallEvalCone{c.n, c.r, c.ld, c.cg_ncs, c.cg_ncl, c.dense_c == 2 ? 2 : c.cg_cconst, c.cg_cslot, c.foff,
                               P.dense_scale * c.c_alpha, c.cg_cadj_ptr, c.cg_cadj, c.cg_cl_con, c.cg_cl_ptr, c.cg_ce,
                               c.cg_cc_ptr, c.cg_cc, c.cg_ce_w};
        lds = std::max(lds, small_eval_lds(c));
    }
    A.m = P.m; A.U = U; A.V = V; A.b = P.b; A.lam = W.lam; A.Craw = P.Craw;
    A.R = W.R; A.cvs = W.cvs; A.cvc = W.cvc; A.out = out;
    hipLaunchKernelGGL(k_small_eval, dim3(P.K), dim3(kSeT), lds, st, A);
    LRS_CHECK_LAUNCH();
    return 0;
}


// ---- the LP block's ADMM update (LORADSUpdateSDPLPVar's LP loop, lorads_alg_common.c:352-372):
// for every LP column j in column order, LORADSUpdateLPVarOne (lorads_admm.c:759-792) for u_j with
// v_j fixed, the constraint sums refreshed, then the same for v_j with u_j fixed.  The update is
// closed form (a 1 x 1 system), but each column reads the constraint sums its predecessors left
// (Gauss-Seidel), so the sweep is one thread's ordered loop: the block stages the operands the
// chain touches -- the constraint sums, lambda and b, the columns' (u, v, c, ||a||^2) and their
// entries -- in LDS with coalesced loads, one thread walks the columns from LDS, and the block
// writes u, v and the sums back.  Arithmetic in the reference's operation order:
//   M1_i = ((-b_i + cvs_i) + (-1) (u v) a_ij) rho + (-1) lambda_i   (scal/axpy sequence :764-779)
//   w = c_j + sum_i a_ij M1_i (entry order, lp_cone_ObjCoeffSum + LPdataMatSparseWeightSum)
//   x = (-1 (w y - rho y)) / rho / (1 + ||a_j||^2 y y)
//   cvs_i += (-1) (u v)_old a_ij; cvs_i += (u v)_new a_ij   (constrValLP add / recompute / add)
// The LP cone's own total A_lp(U V^T) (cvc[lp]) takes the same two adds.
constexpr int kLpT = 256;
constexpr size_t kLpMaxDynLds = 152 * 1024;
struct LpSweepArgs {
    int m, n, ld, slot_off, P;
    long foff, e0, ne;          // the cone's entries: slot CSR range [e0, e0 + ne)
    const int *lp_slot, *slot_ptr, *slot_con;
    const double *slot_a, *lp_nrm2, *Craw, *b, *lam;
    double *U, *V, *cvs, *cvc;
    double rho;
};
__device__ inline void lp_sweep_serial(int m, int n, double rho, const int *__restrict__ lslot,
                                       const int *__restrict__ ebeg, const int *__restrict__ econ,
                                       const double *__restrict__ ea, const double *__restrict__ cj,
                                       const double *__restrict__ nr, const double *__restrict__ b,
                                       const double *__restrict__ lam, double *u, double *v, double *cvs,
                                       double *cvc) {
    for (int j = 0; j < n; ++j) {
        const int t = lslot[j];
        const int a0 = t >= 0 ? ebeg[t] : 0, a1 = t >= 0 ? ebeg[t + 1] : 0;
        const double c = t >= 0 ? cj[t] : 0.0, n2 = nr[j];
        for (int side = 0; side < 2; ++side) {
            const double uv = u[j] * v[j];
            double w = 0.0;
            w += c;
            for (int e = a0; e < a1; ++e) {
                const int i = econ[e];
                const double a = ea[e];
                double m1 = -b[i];
                m1 = m1 + cvs[i];
                m1 = m1 + (-1.0) * (uv * a);
                m1 = m1 * rho;
                m1 = m1 + (-1.0) * lam[i];
                w += a * m1;
            }
            const double y = side == 0 ? v[j] : u[j];
            double M2 = w * y;
            M2 = M2 - rho * y;
            const double blin = -1.0 * M2 / rho;
            const double x = blin / (1 + n2 * y * y);
            if (side == 0) u[j] = x;
            else v[j] = x;
            const double uvn = u[j] * v[j];
            for (int e = a0; e < a1; ++e) {
                const int i = econ[e];
                const double a = ea[e];
                cvs[i] += (-1.0) * (uv * a);
                cvc[i] += (-1.0) * (uv * a);
            }
            for (int e = a0; e < a1; ++e) {
                const int i = econ[e];
                const double a = ea[e];
                cvs[i] += 1.0 * (uvn * a);
                cvc[i] += 1.0 * (uvn * a);
            }
        }
    }
}
// STAGED: operands in LDS (lp_sweep_lds bytes fit kLpMaxDynLds); else straight from global
// memory with a scratch copy of the (u, v) columns and per-slot entry starts in W.lpw.
template <bool STAGED>
__global__ void __launch_bounds__(kLpT) k_lp_admm(LpSweepArgs A, double *__restrict__ scratch) {
    extern __shared__ __align__(16) double lds_lp[];
    const int m = A.m, n = A.n, P = A.P;
    double *cvs, *cvc, *lam, *b, *u, *v, *cj, *nr, *ea;
    int *econ, *ebeg, *lslot;
    if (STAGED) {
        cvs = lds_lp; cvc = cvs + m; lam = cvc + m; b = lam + m; u = b + m; v = u + n; cj = v + n; nr = cj + P;
        ea = nr + n;
        econ = reinterpret_cast<int *>(ea + A.ne);
        ebeg = econ + A.ne;
        lslot = ebeg + (P + 1);
        for (int i = threadIdx.x; i < m; i += kLpT) { cvs[i] = A.cvs[i]; cvc[i] = A.cvc[i]; lam[i] = A.lam[i]; b[i] = A.b[i]; }
        for (long e = threadIdx.x; e < A.ne; e += kLpT) { econ[e] = A.slot_con[A.e0 + e]; ea[e] = A.slot_a[A.e0 + e]; }
        for (int t = threadIdx.x; t < P; t += kLpT) cj[t] = A.Craw[A.slot_off + t];
        for (int t = threadIdx.x; t <= P; t += kLpT) ebeg[t] = A.slot_ptr[A.slot_off + t] - (int)A.e0;
        for (int j = threadIdx.x; j < n; j += kLpT) {
            lslot[j] = A.lp_slot[j];
            nr[j] = A.lp_nrm2[j];
            u[j] = A.U[A.foff + (long)j * A.ld];
            v[j] = A.V[A.foff + (long)j * A.ld];
        }
    } else {
        cvs = A.cvs; cvc = A.cvc; lam = const_cast<double *>(A.lam); b = const_cast<double *>(A.b);
        u = scratch; v = scratch + n; cj = const_cast<double *>(A.Craw) + A.slot_off;
        nr = const_cast<double *>(A.lp_nrm2); ea = const_cast<double *>(A.slot_a) + A.e0;
        econ = const_cast<int *>(A.slot_con) + A.e0;
        ebeg = reinterpret_cast<int *>(scratch + 2L * n);
        lslot = const_cast<int *>(A.lp_slot);
        for (int t = threadIdx.x; t <= P; t += kLpT) ebeg[t] = A.slot_ptr[A.slot_off + t] - (int)A.e0;
        for (int j = threadIdx.x; j < n; j += kLpT) {
            u[j] = A.U[A.foff + (long)j * A.ld];
            v[j] = A.V[A.foff + (long)j * A.ld];
        }
        __threadfence_block();
    }
    __syncthreads();
    if (threadIdx.x == 0) lp_sweep_serial(m, n, A.rho, lslot, ebeg, econ, ea, cj, nr, b, lam, u, v, cvs, cvc);
    __syncthreads();
    if (!STAGED) __threadfence_block();
    for (int j = threadIdx.x; j < n; j += kLpT) {
        A.U[A.foff + (long)j * A.ld] = u[j];
        A.V[A.foff + (long)j * A.ld] = v[j];
    }
    if (STAGED)
        for (int i = threadIdx.x; i < m; i += kLpT) { A.cvs[i] = cvs[i]; A.cvc[i] = cvc[i]; }
}
static size_t lp_sweep_lds(int m, int n, int P, long ne) {
    return sizeof(double) * (4L * m + 3L * n + P + ne) + sizeof(int) * (ne + P + 1 + n);
}
long lp_sweep_scratch(const DevProblem &P) {   // doubles of W.lpw the unstaged sweep needs
    if (P.lp_cone < 0) return 0;
    const DevCone &c = P.cones[P.lp_cone];
    return 2L * c.n + (c.P + 2) / 2 + 1;
}
int launch_lp_admm(const DevProblem &P, DevWork &W, double rho, hipStream_t st) {
    if (P.lp_cone < 0) return 0;
    const DevCone &c = P.cones[P.lp_cone];
    LpSweepArgs A{};
    A.m = P.m; A.n = c.n; A.ld = c.ld; A.slot_off = c.slot_off; A.P = c.P; A.foff = c.foff;
    std::vector<int> sp(2);
    if (hipMemcpy(sp.data(), P.slot_ptr + c.slot_off, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(sp.data() + 1, P.slot_ptr + c.slot_off + c.P, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "launch_lp_admm: slot range read failed");
        return -1;
    }
    A.e0 = sp[0]; A.ne = sp[1] - sp[0];
    A.lp_slot = c.lp_slot; A.slot_ptr = P.slot_ptr; A.slot_con = P.slot_con; A.slot_a = P.slot_a;
    A.lp_nrm2 = c.lp_nrm2; A.Craw = P.Craw; A.b = P.b; A.lam = W.lam;
    A.U = W.U; A.V = W.V; A.cvs = W.cvs; A.cvc = W.cvc + (long)P.lp_cone * P.m; A.rho = rho;
    const size_t lds = lp_sweep_lds(P.m, c.n, c.P, A.ne);
    if (lds <= kLpMaxDynLds) {
        static bool attr = false;
        if (!attr) {
            if (hipFuncSetAttribute(reinterpret_cast<const void *>(k_lp_admm<true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLpMaxDynLds) != hipSuccess) {
                snprintf(g_err, sizeof(g_err), "launch_lp_admm: LDS attribute");
                return -1;
            }
            attr = true;
        }
        hipLaunchKernelGGL(k_lp_admm<true>, dim3(1), dim3(kLpT), lds, st, A, W.lpw);
    } else {
        if (!W.lpw) {
            snprintf(g_err, sizeof(g_err), "launch_lp_admm: no scratch for the unstaged sweep");
            return -1;
        }
        hipLaunchKernelGGL(k_lp_admm<false>, dim3(1), dim3(kLpT), 0, st, A, W.lpw);
    }
    LRS_CHECK_LAUNCH();
    return 0;
}

}  // namespace lrs
