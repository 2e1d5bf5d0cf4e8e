// Can a column sweep's scratch levels live in L2 instead of HBM? Lab, not product code
// (VERDICT r05 item 1 / DESIGN.md §3 K2: vadv's 24 scratch levels of ccol/dcol).
//
// vadv's column kernel keeps 136 of 160 levels of ccol/dcol on chip (96 in VGPRs, 40 in LDS) and
// sends the other S = 24 through a full-domain scratch array: written in the forward sweep, read
// back in the backward sweep, 32 B per scratch level and column, 4.8 B/cell of its 1.27x traffic.
// Between that write and that read each CU streams ~136 levels x 256 columns of the five input
// fields, far more than its share of L2 or the Infinity Cache, so the scratch goes to HBM.
//
// Here the scratch is indexed by the BLOCK, not by the column: a persistent grid (one 256-thread
// block per CU, as the 160-KB LDS tail forces anyway) walks its column tiles one after another
// and reuses one 96-KB scratch slot for all of them. Correct by construction (a block owns its
// slot whatever CU it runs on); the question is only whether 32 blocks x 96 KB = 3 MB per XCD
// stays in that XCD's 4-MB L2 while the read-once streams (non-temporal) pass through it.
//
// Variants (same arithmetic, bit-identical outputs):
//   G<S>    grid of 4096 blocks, column-indexed scratch of S levels (the product's scheme)
//   P<S>    persistent grid of 256 blocks, column-indexed scratch
//   Q<S>    persistent grid, block-slot scratch
//   Qn<S>   the same, with the scratch accessed non-temporally (should behave like P)
// S = 0 is the no-scratch bound (all levels on chip, which the product cannot afford).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o slotscratch_lab slotscratch_lab.hip
// Run:   ./slotscratch_lab [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
constexpr int NF = 5;                         // fields read per level in the forward sweep
constexpr int P = 8;                          // load ring depth (levels)
constexpr int TL = 40;                        // LDS tail levels (2 f64 x 256 threads x 40 = 160 KB)
constexpr int TILES = (NI / 64) * (NJ / 4);   // 4096 tiles of 64 x 4 columns
constexpr int NSLOT = 256;                    // persistent blocks

struct Args {
    const double* f[NF];  // f[3] plays u_pos: read again by the backward sweep
    double* out;
    double* sc;  // scratch c / d
    double* sd;
    double dtr;
};

template <bool NT, typename T> __device__ __forceinline__ T ld(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}
template <bool NT, typename T> __device__ __forceinline__ void st(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}

// one 64x4 tile of columns; SLOT: scratch indexed by block slot, SNT: scratch non-temporal
template <int S, bool SLOT, bool SNT>
__device__ __forceinline__ void tile(const Args& a, int t, double* lds) {
    const int tid = threadIdx.y * 64 + threadIdx.x;
    const int i = (t % (NI / 64)) * 64 + threadIdx.x, j = (t / (NI / 64)) * 4 + threadIdx.y;
    const long long c = (long long)j * NI + i;
    const long long s0 = SLOT ? (long long)blockIdx.x * 256 + tid : c;
    const long long sst = SLOT ? (long long)NSLOT * 256 : SK;
    double* lc = lds;
    double* ldd = lds + TL * 256;
    // ---- forward sweep: 5 read-once streams, a division-carried recurrence, S levels to scratch
    double r[P][NF];
#pragma unroll
    for (int u = 0; u < P; ++u)
#pragma unroll
        for (int f = 0; f < NF; ++f) r[u][f] = ld<true>(a.f[f] + c + u * SK);
    double x = 0.0, y = 0.0;
#pragma unroll 1
    for (int kb = 0; kb < NK; kb += P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int k = kb + u;
            const double inv = 1.0 / (r[u][3] + 4.0 - r[u][4] * x);
            x = r[u][0] * r[u][1] * inv;
            y = (r[u][2] - y * r[u][4]) * inv;
            if (kb + P < NK) {
#pragma unroll
                for (int f = 0; f < NF; ++f) r[u][f] = ld<true>(a.f[f] + c + (k + P) * SK);
            }
            if (k < S) {
                st<SNT>(a.sc + s0 + k * sst, x);
                st<SNT>(a.sd + s0 + k * sst, y);
            } else if (k < S + TL) {
                lc[(k - S) * 256 + tid] = x;
                ldd[(k - S) * 256 + tid] = y;
            }
        }
    }
    // ---- backward sweep: u_pos again (normal loads), scratch c/d for k < S, LDS for the tail
    // levels; the register band's levels (k >= S + TL) use the LDS tail again (timing only)
    double q[P][3];
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const int k = NK - 1 - u;
        q[u][0] = ld<false>(a.f[3] + c + k * SK);
        if (k < S) {
            q[u][1] = ld<SNT>(a.sc + s0 + k * sst);
            q[u][2] = ld<SNT>(a.sd + s0 + k * sst);
        }
    }
    double dc = 0.0;
#pragma unroll 1
    for (int kb = NK - 1; kb >= 0; kb -= P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int k = kb - u;
            double cc, dd;
            if (k < S) {
                cc = q[u][1];
                dd = q[u][2];
            } else {
                const int sl = (k - S) % TL;
                cc = lc[sl * 256 + tid];
                dd = ldd[sl * 256 + tid];
            }
            const double up = q[u][0];
            if (kb - P >= 0) {
                const int kn = k - P;
                q[u][0] = ld<false>(a.f[3] + c + kn * SK);
                if (kn < S) {
                    q[u][1] = ld<SNT>(a.sc + s0 + kn * sst);
                    q[u][2] = ld<SNT>(a.sd + s0 + kn * sst);
                }
            }
            dc = dd - cc * dc;
            st<true>(a.out + c + k * SK, a.dtr * (dc - up));
        }
    }
}

template <int S, bool SLOT, bool SNT>
__global__ void __launch_bounds__(256, 1) k_grid(Args a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    // XCD-aware: the 8 XCDs take contiguous tile ranges (as the product's remap)
    const int b = blockIdx.x, nb = gridDim.x;
    const int t = (b & 7) * (nb >> 3) + (b >> 3);
    tile<S, SLOT, SNT>(a, t, lds);
}

template <int S, bool SLOT, bool SNT>
__global__ void __launch_bounds__(256, 1) k_persist(Args a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    // block b (on XCD b & 7) walks tiles of that XCD's contiguous range
    const int b = blockIdx.x, per_xcd = TILES / 8, blk_per_xcd = NSLOT / 8;
    const int xcd = b & 7, sub = b >> 3;
#pragma unroll 1
    for (int n = sub; n < per_xcd; n += blk_per_xcd) tile<S, SLOT, SNT>(a, xcd * per_xcd + n, lds);
}

template <typename K>
static float run(K kern, int grid, Args a, int reps) {
    const size_t lds = (size_t)TL * 256 * 16;
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int r = 0; r < reps + 2; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(64, 4), lds, 0, a);
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
    std::vector<double> h(n);
    Args a;
    a.dtr = 3.0;
    unsigned s = 12345;
    for (int f = 0; f < NF; ++f) {
        for (size_t q = 0; q < n; ++q) {
            s = s * 1664525u + 1013904223u;
            h[q] = (double)(s >> 8) / 16777216.0 - 0.5;
        }
        double* d;
        CK(hipMalloc(&d, n * 8));
        CK(hipMemcpy(d, h.data(), n * 8, hipMemcpyHostToDevice));
        a.f[f] = d;
    }
    CK(hipMalloc(&a.out, n * 8));
    // scratch: big enough for the column-indexed 40-level case
    const size_t ns = (size_t)SK * 40;
    CK(hipMalloc(&a.sc, ns * 8));
    CK(hipMalloc(&a.sd, ns * 8));
    std::vector<double> got(n);
    std::vector<std::vector<double>> ref(3);  // per scratch depth S (it changes which levels are exact)
    const double gb = (double)n * 8 * (NF + 1) / 1e9;  // 48 B/cell, the algorithmic bytes of vadv
    auto check = [&](const char* name, int sidx, float ms) {
        CK(hipMemcpy(got.data(), a.out, n * 8, hipMemcpyDeviceToHost));
        const char* verdict = "reference";
        if (ref[sidx].empty()) {
            ref[sidx] = got;
        } else {
            size_t bad = 0;
            for (size_t q = 0; q < n; ++q) bad += memcmp(&got[q], &ref[sidx][q], 8) != 0;
            verdict = bad ? "MISMATCH" : "bit-identical";
        }
        printf("%-6s %8.4f ms  %6.3f TB/s algorithmic  %s\n", name, ms, gb / ms, verdict);
        fflush(stdout);
        CK(hipMemset(a.out, 0, n * 8));
    };
    for (int round = 0; round < 2; ++round) {
        check("G24", 0, run(k_grid<24, false, false>, TILES, a, reps));
        check("P24", 0, run(k_persist<24, false, false>, NSLOT, a, reps));
        check("Q24", 0, run(k_persist<24, true, false>, NSLOT, a, reps));
        check("Qn24", 0, run(k_persist<24, true, true>, NSLOT, a, reps));
        check("G40", 1, run(k_grid<40, false, false>, TILES, a, reps));
        check("Q40", 1, run(k_persist<40, true, false>, NSLOT, a, reps));
        check("G0", 2, run(k_grid<0, false, false>, TILES, a, reps));
        check("Q0", 2, run(k_persist<0, true, false>, NSLOT, a, reps));
    }
    return 0;
}
