// HBM ceiling lab: what MI355X sustains for the access mixes of the hot-path stencils, with the
// same 16-B lanes the plane kernel uses. Not product code; it anchors the roofline discussion in
// DESIGN.md (what fraction of 8 TB/s a perfect kernel of each read:write mix reaches).
//
//   read1   1 stream read  (sum kept live)          copy   1R 1W  (copy_stencil)
//   r2w1    2R 1W  out = a - 0.025 * b  (hdiff's field mix: in + coeff -> out)
//   r4w3    4R 3W  (tridiag's forward mix, pointwise)
//
// Build: hipcc --offload-arch=gfx950 -O3 -o stream_lab stream_lab.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ d2 ld(const d2* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(d2* p, d2 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool NT>
__global__ void __launch_bounds__(256) k_read1(const d2* a, long long n, double* sink) {
    d2 s = {0, 0};
    for (long long q = blockIdx.x * 256LL + threadIdx.x; q < n; q += (long long)gridDim.x * 256) s += ld<NT>(a + q);
    if (s.x == 12345.678) sink[0] = s.y;  // never true: keeps the loads live
}

template <bool NT>
__global__ void __launch_bounds__(256) k_copy(const d2* a, d2* b, long long n) {
    for (long long q = blockIdx.x * 256LL + threadIdx.x; q < n; q += (long long)gridDim.x * 256) st<NT>(b + q, ld<NT>(a + q));
}

template <bool NT>
__global__ void __launch_bounds__(256) k_r2w1(const d2* a, const d2* b, d2* c, long long n) {
    for (long long q = blockIdx.x * 256LL + threadIdx.x; q < n; q += (long long)gridDim.x * 256)
        st<NT>(c + q, ld<NT>(a + q) - 0.025 * ld<NT>(b + q));
}

template <bool NT>
__global__ void __launch_bounds__(256) k_r4w3(const d2* a, const d2* b, d2* c, d2* d, d2* e, long long n) {
    for (long long q = blockIdx.x * 256LL + threadIdx.x; q < n; q += (long long)gridDim.x * 256) {
        const d2 x = ld<NT>(a + q), y = ld<NT>(b + q), z = ld<false>(c + q), w = ld<false>(d + q);
        st<false>(c + q, z / y);
        st<false>(d + q, (w - x) / y);
        st<NT>(e + q, x + w);
    }
}

int main(int argc, char** argv) {
    const long long n = (argc > 1 ? atoll(argv[1]) : 2048LL * 2048 * 160) / 2;  // d2 elements per array
    const int mode = argc > 2 ? atoi(argv[2]) : 0;  // 1: relative-offset sweep (HBM channel aliasing)
    const int reps = 20;
    const size_t B = n * sizeof(d2);
    d2* f[5];
    for (int i = 0; i < 5; ++i) {
        f[i] = nullptr;
        if (mode == 1) continue;
        CK(hipMalloc(&f[i], B));
        CK(hipMemset(f[i], 0x3f, B));
    }
    double* sink;
    CK(hipMalloc(&sink, 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        std::vector<float> ms;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        printf("%-22s median %.4f ms  %.1f GB/s  frac %.3f\n", name, med, bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12);
        fflush(stdout);
    };
    if (mode == 1) {
        // arrays carved from one arena at base + q * (B + d): the relative offset of the streams
        // modulo the HBM interleave decides whether they collide on the same channels
        const size_t maxd = 8ull << 20;
        char* arena;
        CK(hipMalloc(&arena, 3 * (B + maxd) + (4 << 20)));
        CK(hipMemset(arena, 0x3f, 3 * (B + maxd)));
        const int grid = ncu * 8;
        for (long long d : {0LL, 4096LL, 65536LL, 262144LL, 524288LL, 786432LL, 1LL << 20, 1536LL << 10, 2LL << 20,
                            3LL << 20, 4LL << 20, 5LL << 20, 6LL << 20, 7LL << 20}) {
            d2* a = (d2*)(arena);
            d2* b = (d2*)(arena + (B + d));
            d2* c = (d2*)(arena + 2 * (B + d));
            char label[64];
            snprintf(label, sizeof label, "copy d=%lld", d);
            timeit(label, 2.0 * B, [&] { hipLaunchKernelGGL(k_copy<true>, dim3(grid), dim3(256), 0, 0, a, b, n); });
            snprintf(label, sizeof label, "r2w1 d=%lld", d);
            timeit(label, 3.0 * B, [&] { hipLaunchKernelGGL(k_r2w1<true>, dim3(grid), dim3(256), 0, 0, a, b, c, n); });
        }
        return 0;
    }
    for (int occ : {8, 16, 32}) {
        const int grid = ncu * occ;
        printf("-- grid %d blocks of 256 (%d per CU), %.2f GB per array\n", grid, occ, B / 1e9);
        timeit("read1", 1.0 * B, [&] { hipLaunchKernelGGL(k_read1<false>, dim3(grid), dim3(256), 0, 0, f[0], n, sink); });
        timeit("read1 nt", 1.0 * B, [&] { hipLaunchKernelGGL(k_read1<true>, dim3(grid), dim3(256), 0, 0, f[0], n, sink); });
        timeit("copy", 2.0 * B, [&] { hipLaunchKernelGGL(k_copy<false>, dim3(grid), dim3(256), 0, 0, f[0], f[1], n); });
        timeit("copy nt", 2.0 * B, [&] { hipLaunchKernelGGL(k_copy<true>, dim3(grid), dim3(256), 0, 0, f[0], f[1], n); });
        timeit("r2w1", 3.0 * B, [&] { hipLaunchKernelGGL(k_r2w1<false>, dim3(grid), dim3(256), 0, 0, f[0], f[1], f[2], n); });
        timeit("r2w1 nt", 3.0 * B, [&] { hipLaunchKernelGGL(k_r2w1<true>, dim3(grid), dim3(256), 0, 0, f[0], f[1], f[2], n); });
        timeit("r4w3 nt", 7.0 * B, [&] { hipLaunchKernelGGL(k_r4w3<true>, dim3(grid), dim3(256), 0, 0, f[0], f[1], f[2], f[3], f[4], n); });
    }
    return 0;
}
