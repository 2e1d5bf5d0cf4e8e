// Does an LDS-DMA prefetch ring move a column sweep's streams faster than a register ring at one
// wave per SIMD? Lab, not product code.
//
// The column kernels (codegen/column.py) run one 256-thread block per CU because their LDS tail
// cache takes the whole 160 KB, i.e. ONE wave per SIMD; each wave keeps its load ring (the next
// P levels of every window front) in VGPRs. This lab isolates the stream side of vadv's forward
// sweep -- 5 f64 fields read per level, a loop-carried recurrence, 1 field written -- and times:
//
//   R<P>   fronts in a register ring of P levels (the product's scheme; P = 8 is its default)
//   D<Q>   fronts landed in LDS by global_load_lds_dwordx4 (no VGPR destination), Q levels ahead:
//          one wave-instruction moves one field's 64 columns for TWO levels (lanes 0-31 level k,
//          32-63 level k+1, 16 B each), a thread then reads its own column with ds_read_b64;
//          waits are counted by hand (s_waitcnt vmcnt(N), N = the memory operations issued since)
//   *h     the same without the 160-KB LDS reservation (occupancy set by registers: the stream
//          mix's rate when latency is hidden by waves instead)
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o ldsring_lab ldsring_lab.hip
// Run:   ./ldsring_lab [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

constexpr int NI = 1024, NJ = 1024, NK = 160;
constexpr long long SK = (long long)NI * NJ;  // level stride (elements)
constexpr int NF = 5;                         // fields read per level

struct Args {
    const double* f[NF];
    double* out;
};

__device__ __forceinline__ double level_op(double a, double b, double c, double d, double e, double& x) {
    // a loop-carried recurrence in the shape of the Thomas forward sweep
    const double den = d - e * x;
    x = (a * b + c) / den;
    return x;
}

// ------------------------------------------------------------------------ register ring
template <int P>
__global__ void __launch_bounds__(256, 1) k_reg(Args a) {
    static_assert(NK % P == 0, "whole blocks of P levels");
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    const long long c = (long long)j * NI + i;
    double r[P][NF];
#pragma unroll
    for (int u = 0; u < P; ++u)
#pragma unroll
        for (int f = 0; f < NF; ++f) r[u][f] = __builtin_nontemporal_load(a.f[f] + c + u * SK);
    double x = 0.0;
    int k = 0;
    // full blocks: every level refills its slot P levels ahead, no branch around a load
    for (; k + P < NK; k += P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const double v = level_op(r[u][0], r[u][1], r[u][2], r[u][3] + 4.0, r[u][4], x);
#pragma unroll
            for (int f = 0; f < NF; ++f) r[u][f] = __builtin_nontemporal_load(a.f[f] + c + (k + u + P) * SK);
            __builtin_nontemporal_store(v, a.out + c + (k + u) * SK);
        }
    }
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const double v = level_op(r[u][0], r[u][1], r[u][2], r[u][3] + 4.0, r[u][4], x);
        __builtin_nontemporal_store(v, a.out + c + (k + u) * SK);
    }
}

// ------------------------------------------------------------------------ LDS-DMA ring
// s_waitcnt immediates (gfx9): vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14
// ROUND 0: the first Q levels (their DMAs came from the prologue), 1: steady state, 2: the last Q
// levels (no DMAs issued). Operations issued after slot s's DMAs until its wait, for the count:
//   round 0: the prologue's later slots (NF each) + this round's earlier steps (NF DMAs + 2 stores)
//   round 1: its own step's 2 stores + the S-1 steps after it (NF + 2 each)
//   round 2: its own step's 2 stores + the previous round's later steps + this round's earlier
//            steps (2 stores each)
template <int Q, int ROUND, int s>
__device__ __forceinline__ void dma_step(const Args& a, char* wbase, long long dma_off, long long c, int lane, int kb,
                                         double& x) {
    constexpr int S = Q / 2;
    constexpr int n = ROUND == 0 ? NF * (S - 1 - s) + (NF + 2) * s
                    : ROUND == 1 ? 2 + (NF + 2) * (S - 1)
                                 : 2 + (NF + 2) * (S - 1 - s) + 2 * s;
    static_assert(n >= 0 && n <= 63, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((n & 15) | (7 << 4) | (15 << 8) | (((n >> 4) & 3) << 14));
    const int k = kb + 2 * s;
    double v[2][NF];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int f = 0; f < NF; ++f)
            v[h][f] = *(const double*)(wbase + (s * NF + f) * 1024 + h * 512 + lane * 8);
    __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0): the slot is read
    __asm__ volatile("" ::: "memory");
    if (ROUND != 2) {
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            const double* g = a.f[f] + dma_off + (long long)(k + Q) * SK;
            __builtin_amdgcn_global_load_lds((const void*)g,
                                             (__attribute__((address_space(3))) void*)(wbase + (s * NF + f) * 1024),
                                             16, 0, 0);
        }
    }
    // keep the stores after this step's DMAs: the hand counts assume this issue order
    __asm__ volatile("" ::: "memory");
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const double y = level_op(v[h][0], v[h][1], v[h][2], v[h][3] + 4.0, v[h][4], x);
        __builtin_nontemporal_store(y, a.out + c + (long long)(k + h) * SK);
    }
}

template <int Q, int ROUND, int... s>
__device__ __forceinline__ void dma_round(const Args& a, char* wbase, long long dma_off, long long c, int lane, int kb,
                                          double& x, std::integer_sequence<int, s...>) {
    (dma_step<Q, ROUND, s>(a, wbase, dma_off, c, lane, kb, x), ...);
}

template <int Q>
__global__ void __launch_bounds__(256, 1) k_dma(Args a) {
    static_assert(Q % 2 == 0 && NK % Q == 0 && NK / Q >= 2, "levels come in pairs, whole rounds");
    constexpr int S = Q / 2;  // ring slots (level pairs)
    static_assert(2 + (NF + 2) * (S - 1) <= 63, "vmcnt is 6 bits");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int lane = threadIdx.x, wv = threadIdx.y;
    const int i0 = blockIdx.x * 64, j = blockIdx.y * 4 + wv;
    const long long c = (long long)j * NI + i0 + lane;
    // per wave: S slots x NF fields x 1 KiB (two levels of 64 doubles)
    char* wbase = lds + (size_t)wv * S * NF * 1024;
    // DMA lane mapping: lanes 0-31 -> level k, columns 2l, 2l+1; lanes 32-63 -> level k+1
    const long long dma_off = (long long)j * NI + i0 + 2 * (lane & 31) + (lane >> 5) * SK;
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
        for (int f = 0; f < NF; ++f)
            __builtin_amdgcn_global_load_lds((const void*)(a.f[f] + dma_off + (long long)(2 * s) * SK),
                                             (__attribute__((address_space(3))) void*)(wbase + (s * NF + f) * 1024),
                                             16, 0, 0);
    double x = 0.0;
    using seq = std::make_integer_sequence<int, S>;
    dma_round<Q, 0>(a, wbase, dma_off, c, lane, 0, x, seq{});
    for (int kb = Q; kb < NK - Q; kb += Q) dma_round<Q, 1>(a, wbase, dma_off, c, lane, kb, x, seq{});
    dma_round<Q, 2>(a, wbase, dma_off, c, lane, NK - Q, x, seq{});
    __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (15 << 8));
}

// ------------------------------------------------------------------------ host
static void reference(const std::vector<std::vector<double>>& f, std::vector<double>& out) {
    for (long long c = 0; c < SK; ++c) {
        double x = 0.0;
        for (int k = 0; k < NK; ++k) {
            const long long o = c + k * SK;
            const double den = (f[3][o] + 4.0) - f[4][o] * x;
            x = (f[0][o] * f[1][o] + f[2][o]) / den;
            out[o] = x;
        }
    }
}

template <typename K>
static float run(K kern, Args a, size_t lds, int reps) {
    dim3 grid(NI / 64, NJ / 4), block(64, 4);
    if (lds) CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int r = 0; r < reps + 2; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, grid, block, lds, 0, a);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const size_t n = (size_t)SK * NK;
    std::vector<std::vector<double>> h(NF, std::vector<double>(n));
    unsigned s = 12345;
    for (int f = 0; f < NF; ++f)
        for (size_t q = 0; q < n; ++q) {
            s = s * 1664525u + 1013904223u;
            h[f][q] = (double)(s >> 8) / 16777216.0 - 0.5;
        }
    std::vector<double> ref(n), got(n);
    reference(h, ref);
    Args a;
    for (int f = 0; f < NF; ++f) {
        double* d;
        CK(hipMalloc(&d, n * 8));
        CK(hipMemcpy(d, h[f].data(), n * 8, hipMemcpyHostToDevice));
        a.f[f] = d;
    }
    CK(hipMalloc(&a.out, n * 8));
    const double gb = (double)n * 8 * (NF + 1) / 1e9;
    const size_t FULL = 160 * 1024;
    auto check = [&](const char* name, float ms) {
        CK(hipMemcpy(got.data(), a.out, n * 8, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t q = 0; q < n; ++q) bad += memcmp(&got[q], &ref[q], 8) != 0;
        printf("%-6s %8.4f ms  %6.3f TB/s of %.2f GB  %s\n", name, ms, gb / ms, gb,
               bad ? "MISMATCH" : "bit-exact");
        CK(hipMemset(a.out, 0, n * 8));
    };
    for (int round = 0; round < 2; ++round) {
        check("R8", run(k_reg<8>, a, FULL, reps));
        check("R10", run(k_reg<10>, a, FULL, reps));
        check("R16", run(k_reg<16>, a, FULL, reps));
        check("R8h", run(k_reg<8>, a, 0, reps));
        check("D8h", run(k_dma<8>, a, 4 * 4 * NF * 1024, reps));
        check("D8", run(k_dma<8>, a, FULL, reps));
        check("D10", run(k_dma<10>, a, FULL, reps));
        check("D16", run(k_dma<16>, a, FULL, reps));
    }
    return 0;
}
