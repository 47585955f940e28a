// Diagnostics (GPU box): cost of a stage boundary for the latency-regime loop.
// (a) a hipGraph of S dependent launches of a stage kernel (179 blocks x 512 threads,
//     each block reads a 64 KB slice written by ANOTHER block in the previous stage and
//     writes its own), (b) the same S stages inside one cooperative launch separated by a
//     grid barrier (agent-scope release/acquire around one counter per barrier), and
//     (c) both with an empty stage body.  The barrier spin is bounded: a block that waits
//     too long sets an error word and leaves, so the grid always drains.
// Build: hipcc -O3 --offload-arch=gfx950 -o barrier_probe scripts/barrier_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kThreads = 512;
constexpr int kChunk = 8192;   // doubles per block slice (64 KB)

__device__ __forceinline__ void stage_body(const double *__restrict__ in, double *__restrict__ out, int blk, int nblk,
                                           int s, int work) {
    if (!work) return;
    const int src = (blk * 37 + s * 11 + 5) % nblk;   // another block's slice
    const double *a = in + (long)src * kChunk;
    double *o = out + (long)blk * kChunk;
    if (work == 2) {
        for (int q = threadIdx.x; q < kChunk; q += kThreads) __builtin_nontemporal_store(a[q] * 0.5 + 1.0, o + q);
    } else {
        for (int q = threadIdx.x; q < kChunk; q += kThreads) o[q] = a[q] * 0.5 + 1.0;
    }
}
struct Big { const double *p[48]; };
__global__ void __launch_bounds__(kThreads) k_stage_big(const double *in, double *out, int s, int work, Big b) {
    stage_body(in, out, blockIdx.x, gridDim.x, s, work + (b.p[47] == in ? 1 : 0) * 0);
}

__global__ void __launch_bounds__(kThreads) k_stage(const double *in, double *out, int s, int work) {
    stage_body(in, out, blockIdx.x, gridDim.x, s, work);
}

__device__ __forceinline__ bool grid_barrier(unsigned *count, unsigned *gen, unsigned nblk, unsigned *err) {
    __syncthreads();
    __shared__ int bad;
    if (threadIdx.x == 0) {
        bad = 0;
        const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned prev = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == nblk - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            long spins = 0;
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1L << 24)) {
                    __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    bad = 1;
                    break;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return bad == 0;
}

// Hierarchical variant ("re-measure a hierarchical, XCD-local grid barrier"): the
// blocks of group x = blockIdx % 8 (one XCD under the round-robin dispatch; speed only, the
// protocol does not rely on it) count on their own counter (its own 256-byte line); the last
// arriver of a group counts on the top counter; the last of those bumps the top generation,
// which the group leaders wait for and pass on through a per-group generation the group's
// blocks wait on.  Every spin bounded (err word, early exit).
template <bool FENCE>
__device__ __forceinline__ bool wait_gen(unsigned *gen, unsigned g, unsigned *err) {
    long spins = 0;
    while (__hip_atomic_load(gen, FENCE ? __ATOMIC_ACQUIRE : __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1L << 24)) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
    }
    return true;
}
// FENCE = false: relaxed counters and spins, no release / acquire fences -- the cost of the
// synchronisation alone (data handed off through it would need sc1 stores and loads instead,
// cdna_hip_programming G16's valid forms)
template <bool FENCE>
__device__ __forceinline__ bool grid_barrier_h(unsigned *bar, unsigned nblk, unsigned *err) {
    // layout (unsigned words, 64 apart = 256 bytes): [0] top count, [64] top gen,
    // [128 + 128 x] group count, [192 + 128 x] group gen
    __syncthreads();
    __shared__ int bad;
    if (threadIdx.x == 0) {
        bad = 0;
        const unsigned x = blockIdx.x & 7;
        const unsigned gsz = (nblk - x + 7) / 8;
        unsigned *gc = bar + 128 + 128 * x, *gg = bar + 192 + 128 * x;
        unsigned *tc = bar, *tg = bar + 64;
        const unsigned g0 = __hip_atomic_load(gg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned prev = __hip_atomic_fetch_add(gc, 1u, FENCE ? __ATOMIC_ACQ_REL : __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gsz - 1) {   // group leader: the top level
            __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned t0 = __hip_atomic_load(tg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned ngroups = nblk < 8 ? nblk : 8;
            const unsigned tp = __hip_atomic_fetch_add(tc, 1u, FENCE ? __ATOMIC_ACQ_REL : __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
            if (tp == ngroups - 1) {
                __hip_atomic_store(tc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(tg, t0 + 1, FENCE ? __ATOMIC_RELEASE : __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (!wait_gen<FENCE>(tg, t0, err)) {
                bad = 1;
            }
            __hip_atomic_store(gg, g0 + 1, FENCE ? __ATOMIC_RELEASE : __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (!wait_gen<FENCE>(gg, g0, err)) {
            bad = 1;
        }
        if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return bad == 0;
}
template <bool FENCE>
__global__ void __launch_bounds__(kThreads) k_persist_h(double *b0, double *b1, int S, int work, unsigned *bar,
                                                        unsigned *err) {
    for (int s = 0; s < S; ++s) {
        const double *in = (s & 1) ? b1 : b0;
        double *out = (s & 1) ? b0 : b1;
        stage_body(in, out, blockIdx.x, gridDim.x, s, work);
        if (!grid_barrier_h<FENCE>(bar, gridDim.x, err)) return;
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    }
}

__global__ void __launch_bounds__(kThreads) k_persist(double *b0, double *b1, int S, int work, unsigned *bar,
                                                      unsigned *err) {
    for (int s = 0; s < S; ++s) {
        const double *in = (s & 1) ? b1 : b0;
        double *out = (s & 1) ? b0 : b1;
        stage_body(in, out, blockIdx.x, gridDim.x, s, work);
        if (!grid_barrier(bar, bar + 1, gridDim.x, err)) return;
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    }
}

int main(int argc, char **argv) {
    const int nblk = argc > 1 ? atoi(argv[1]) : 179;
    const int S = 64, reps = 20;
    double *b0, *b1;
    unsigned *bar, *err;
    CK(hipMalloc(&b0, sizeof(double) * kChunk * nblk));
    CK(hipMalloc(&b1, sizeof(double) * kChunk * nblk));
    CK(hipMalloc(&bar, 8192));
    CK(hipMalloc(&err, 64));
    CK(hipMemset(b0, 0, sizeof(double) * kChunk * nblk));
    CK(hipMemset(b1, 0, sizeof(double) * kChunk * nblk));
    CK(hipMemset(bar, 0, 8192));
    CK(hipMemset(err, 0, 64));
    int dev = 0, coop = 0, per_cu = 0, ncu = 0;
    CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_persist, kThreads, 0));
    printf("cooperative=%d CUs=%d blocks/CU=%d grid=%d\n", coop, ncu, per_cu, nblk);
    if (!coop || per_cu * ncu < nblk) { printf("grid cannot be co-resident; stop\n"); return 0; }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    Big big;
    for (int q = 0; q < 48; ++q) big.p[q] = b0;
    for (int mode = 0; mode < 4; ++mode) {
        const int work = mode == 3 ? 1 : mode;
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int s = 0; s < S; ++s) {
            if (mode == 3)
                hipLaunchKernelGGL(k_stage_big, dim3(nblk), dim3(kThreads), 0, st, (s & 1) ? b1 : b0, (s & 1) ? b0 : b1, s,
                                   work, big);
            else
                hipLaunchKernelGGL(k_stage, dim3(nblk), dim3(kThreads), 0, st, (s & 1) ? b1 : b0, (s & 1) ? b0 : b1, s,
                                   work);
        }
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const char *nm[4] = {"empty", "copy", "copy, nontemporal stores", "copy, 400-byte kernarg"};
        printf("graph, %-26s %.3f us per stage\n", nm[mode], ms * 1e3 / (reps * S));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    // the persistent forms: S stages in one cooperative launch, flat and hierarchical barriers
    for (int h = 0; h < 3; ++h)
        for (int work = 0; work < 2; ++work) {
            unsigned herr = 0;
            CK(hipMemset(bar, 0, 8192));
            CK(hipMemset(err, 0, 64));
            void *args[] = {&b0, &b1, (void *)&S, &work, &bar, &err};
            const void *fn = h == 0 ? (const void *)k_persist
                             : h == 1 ? (const void *)k_persist_h<true> : (const void *)k_persist_h<false>;
            CK(hipLaunchCooperativeKernel(fn, dim3(nblk), dim3(kThreads), args, 0, st));   // warm
            CK(hipStreamSynchronize(st));
            CK(hipEventRecord(e0, st));
            for (int r = 0; r < reps; ++r) CK(hipLaunchCooperativeKernel(fn, dim3(nblk), dim3(kThreads), args, 0, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            CK(hipMemcpy(&herr, err, sizeof(unsigned), hipMemcpyDeviceToHost));
            printf("persistent, %s barrier, %s: %.3f us per stage%s\n",
                   h == 0 ? "flat" : h == 1 ? "hierarchical (8 groups)" : "hierarchical, no fences",
                   work ? "copy" : "empty", ms * 1e3 / (reps * S), herr ? " (SPIN LIMIT HIT)" : "");
            if (herr) return 1;
        }
    printf("done\n");
    return 0;
}
