// Which levels of a FORWARD->BACKWARD column sweep should stay on chip? Lab, not product code.
//
// The Thomas solve (tridiagonal_solver) at 1024x1024x160 f64 re-reads c'/d'
// (sup/rhs) in the backward sweep for every level the LDS does not hold. The product kernel
// (codegen/column.py) keeps the LAST forward levels on chip (the first ones the backward sweep
// needs), so it re-reads the FIRST forward levels -- the ones written longest ago, after ~all
// of the live columns' traffic has gone by (beyond the 256-MB Infinity Cache). Keeping the FIRST
// levels on chip instead re-reads the LAST ones, written just before the turn.
//
//   tail<L>  the last L forward levels of (c', d') in LDS, levels [0, NK-L) re-read
//   head<L>  the first L forward levels in LDS, levels [L, NK) re-read
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o headtail_lab headtail_lab.hip
// Run:   ./headtail_lab [reps] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

constexpr int NK = 160;
constexpr int P = 8;  // load ring depth (levels in flight)

struct Args {
    const double* inf;
    const double* diag;
    double* sup;
    double* rhs;
    double* out;
    int ni, nj;
    long long S;
};

// HEAD = false: LDS holds levels [NK-L, NK); HEAD = true: levels [0, L)
template <int L, bool HEAD>
__global__ void __launch_bounds__(256, 1) k_sweep(Args a) {
    extern __shared__ double2 lds[];  // [L][256]
    const int tid = threadIdx.y * 64 + threadIdx.x;
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    if (i >= a.ni || j >= a.nj) return;
    const long long c = (long long)j * a.ni + i;
    const long long S = a.S;
    const double* inf = a.inf + c;
    const double* diag = a.diag + c;
    double* sup = a.sup + c;
    double* rhs = a.rhs + c;
    double* out = a.out + c;
    constexpr int C0 = HEAD ? 0 : NK - L, C1 = HEAD ? L : NK;  // cached levels [C0, C1)
    double cp = 0, dp = 0;
    double ri[P], rd[P], rs[P], rr[P];
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const long long o = (long long)u * S;
        ri[u] = inf[o];
        rd[u] = diag[o];
        rs[u] = sup[o];
        rr[u] = rhs[o];
    }
    for (int kb = 0; kb < NK; kb += P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int k = kb + u;
            double ncp, ndp;
            if (k == 0) {
                ncp = rs[u] / rd[u];
                ndp = rr[u] / rd[u];
            } else {
                const double den = rd[u] - cp * ri[u];
                ncp = rs[u] / den;
                ndp = (rr[u] - ri[u] * dp) / den;
            }
            cp = ncp;
            dp = ndp;
            const long long o = (long long)k * S;
            sup[o] = cp;
            rhs[o] = dp;
            if (k >= C0 && k < C1) lds[(k - C0) * 256 + tid] = make_double2(cp, dp);
            const int kn = min(k + P, NK - 1);
            const long long on = (long long)kn * S;
            ri[u] = inf[on];
            rd[u] = diag[on];
            rs[u] = sup[on];
            rr[u] = rhs[on];
        }
    }
    double o = dp;
    out[(long long)(NK - 1) * S] = o;
    // backward over levels NK-2 .. 0; memory levels through a P-deep ring (a cached level's slot
    // loads nothing useful: its value comes from LDS)
    double bs[P], br[P];
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const long long q = (long long)max(NK - 2 - u, 0) * S;
        bs[u] = sup[q];
        br[u] = rhs[q];
    }
    for (int kb = NK - 2; kb >= 0; kb -= P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int k = kb - u;
            if (k >= 0) {
                double s_, r_;
                if (k >= C0 && k < C1) {
                    const double2 v = lds[(k - C0) * 256 + tid];
                    s_ = v.x;
                    r_ = v.y;
                } else {
                    s_ = bs[u];
                    r_ = br[u];
                }
                o = r_ - s_ * o;
                out[(long long)k * S] = o;
                const int kn = max(k - P, 0);
                if (!(kn >= C0 && kn < C1)) {
                    const long long q = (long long)kn * S;
                    bs[u] = sup[q];
                    br[u] = rhs[q];
                }
            }
        }
    }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int ni = 1024, nj = 1024;
    const long long S = (long long)ni * nj, N = S * NK;
    std::vector<double> h(N);
    double* d[5];
    double* keep[2];
    unsigned seed = 1337;
    auto rnd = [&]() { seed = seed * 1664525u + 1013904223u; return (seed >> 8) / 16777216.0; };
    const double lo[5] = {-1, 4, -1, -10, 0}, hi[5] = {1, 5, 1, 10, 0};
    for (int f = 0; f < 5; ++f) {
        CK(hipMalloc(&d[f], N * sizeof(double)));
        for (long long x = 0; x < N; ++x) h[x] = lo[f] + (hi[f] - lo[f]) * rnd();
        CK(hipMemcpy(d[f], h.data(), N * sizeof(double), hipMemcpyHostToDevice));
    }
    for (int q = 0; q < 2; ++q) {
        CK(hipMalloc(&keep[q], N * sizeof(double)));
        CK(hipMemcpy(keep[q], d[2 + q], N * sizeof(double), hipMemcpyDeviceToDevice));
    }
    Args a{d[0], d[1], d[2], d[3], d[4], ni, nj, S};
    dim3 grid(ni / 64, nj / 4), block(64, 4);
    constexpr int L = 40;
    const size_t lds = (size_t)L * 256 * sizeof(double2);
    CK(hipFuncSetAttribute((const void*)k_sweep<L, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)k_sweep<L, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    auto restore = [&]() {
        CK(hipMemcpy(d[2], keep[0], N * sizeof(double), hipMemcpyDeviceToDevice));
        CK(hipMemcpy(d[3], keep[1], N * sizeof(double), hipMemcpyDeviceToDevice));
    };
    // one checked call of each (sup/rhs are solved in place): the results must be identical
    std::vector<double> r0(N), r1(N);
    restore();
    hipLaunchKernelGGL((k_sweep<L, false>), grid, block, lds, 0, a);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r0.data(), d[4], N * sizeof(double), hipMemcpyDeviceToHost));
    restore();
    hipLaunchKernelGGL((k_sweep<L, true>), grid, block, lds, 0, a);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r1.data(), d[4], N * sizeof(double), hipMemcpyDeviceToHost));
    long long bad = 0;
    for (long long x = 0; x < N; ++x) bad += (r0[x] != r1[x]);
    printf("{\"check\": \"head vs tail out\", \"mismatches\": %lld}\n", bad);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t[2];
    for (int r = 0; r < rounds; ++r) {
        for (int v = 0; v < 2; ++v) {
            CK(hipEventRecord(e0));
            for (int q = 0; q < reps; ++q) {
                if (v) hipLaunchKernelGGL((k_sweep<L, true>), grid, block, lds, 0, a);
                else hipLaunchKernelGGL((k_sweep<L, false>), grid, block, lds, 0, a);
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / reps);
        }
    }
    for (int v = 0; v < 2; ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("{\"variant\": \"%s<%d>\", \"median_ms\": %.4f, \"min_ms\": %.4f}\n", v ? "head" : "tail", L,
               t[v][t[v].size() / 2], t[v][0]);
    }
    return 0;
}
