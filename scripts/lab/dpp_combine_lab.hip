// Do VALU instructions with a folded DPP wave rotate compute what the ISA says on gfx950? Lab,
// not product code (found by the mixed-precision differential fuzz, seed 9130: an int32 I-offset
// difference came out wrong in the odd elements of 2-element lanes).
//
// The stencil kernels move I neighbours with a DPP wave rotate (`wave_rol:1` / `wave_ror:1`,
// __builtin_amdgcn_update_dpp -> v_mov_b32_dpp). LLVM's DPP combiner folds such a move into the
// VALU instruction that consumes it (v_subrev_u32_dpp, v_add_f32_dpp, ...). Each kernel here
// computes one lane-pair expression twice -- once with the move left foldable, once behind an
// empty asm that keeps it a separate v_mov_b32_dpp -- and counts lanes that differ from the host.
//
// Result on the MI355X (profiles/r06/r06n/dpp_combine_lab.log): every lane of the folded
// `v_subrev_u32_dpp` (int32 y - rot(x)) that should differ from its separate form is wrong (3843
// of 4096); the folded v_sub_u32 / v_add_u32 / v_add_f32 / v_sub_f32 / v_subrev_f32 forms and
// every separate v_mov_b32_dpp are right. The JIT therefore compiles with
// -mllvm -amdgpu-dpp-combine=false (runtime/jit.py).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o dpp_combine_lab dpp_combine_lab.hip
//        (add --save-temps to see which instructions the combiner produced)
// Run:   ./dpp_combine_lab
#include <hip/hip_runtime.h>

#include <cmath>
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

constexpr int WAVES = 64, N = WAVES * 64;

template <bool OPAQUE, int CTRL> __device__ __forceinline__ int rot(int v) {
    int r = __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
    if constexpr (OPAQUE) __asm__ volatile("" : "+v"(r));
    return r;
}
template <bool OPAQUE, int CTRL> __device__ __forceinline__ float rotf(float v) {
    return __int_as_float(rot<OPAQUE, CTRL>(__float_as_int(v)));
}

// case 0: |y - rol(x)| on int32 pairs (the fuzz program's shape)
// case 1: y - rol(x) int32      case 2: rol(x) - y int32      case 3: y + rol(x) int32
// case 4: y + rol(x) f32        case 5: y - rol(x) f32        case 6: rol(x) - y f32
// case 7: y + ror(x) f32        case 8: |y - ror(x)| int32
template <bool OPAQUE>
__global__ void k(const int* __restrict__ xi, const int* __restrict__ yi, const float* __restrict__ xf,
                  const float* __restrict__ yf, int* __restrict__ oi, float* __restrict__ of) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int x = xi[t], y = yi[t];
    const float u = xf[t], v = yf[t];
    int d = y - rot<OPAQUE, 0x134>(x);
    oi[9 * t + 0] = d < 0 ? -d : d;
    oi[9 * t + 1] = y - rot<OPAQUE, 0x134>(x);
    oi[9 * t + 2] = rot<OPAQUE, 0x134>(x) - y;
    oi[9 * t + 3] = y + rot<OPAQUE, 0x134>(x);
    of[9 * t + 4] = v + rotf<OPAQUE, 0x134>(u);
    of[9 * t + 5] = v - rotf<OPAQUE, 0x134>(u);
    of[9 * t + 6] = rotf<OPAQUE, 0x134>(u) - v;
    of[9 * t + 7] = v + rotf<OPAQUE, 0x13C>(u);
    int e = y - rot<OPAQUE, 0x13C>(x);
    oi[9 * t + 8] = e < 0 ? -e : e;
}

int main() {
    std::vector<int> xi(N), yi(N);
    std::vector<float> xf(N), yf(N);
    srand(7);
    for (int q = 0; q < N; ++q) {
        xi[q] = rand() % 11 - 5;
        yi[q] = rand() % 11 - 5;
        xf[q] = (float)(rand() % 2001 - 1000) / 256.0f;
        yf[q] = (float)(rand() % 2001 - 1000) / 256.0f;
    }
    int *dxi, *dyi, *doi;
    float *dxf, *dyf, *dof;
    CK(hipMalloc(&dxi, N * 4));
    CK(hipMalloc(&dyi, N * 4));
    CK(hipMalloc(&dxf, N * 4));
    CK(hipMalloc(&dyf, N * 4));
    CK(hipMalloc(&doi, 9 * N * 4));
    CK(hipMalloc(&dof, 9 * N * 4));
    CK(hipMemcpy(dxi, xi.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dyi, yi.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dxf, xf.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dyf, yf.data(), N * 4, hipMemcpyHostToDevice));
    const char* names[9] = {"|y-rol(x)| i32", "y-rol(x) i32", "rol(x)-y i32", "y+rol(x) i32", "y+rol(x) f32",
                            "y-rol(x) f32",   "rol(x)-y f32", "y+ror(x) f32", "|y-ror(x)| i32"};
    for (int opaque = 0; opaque < 2; ++opaque) {
        CK(hipMemset(doi, 0, 9 * N * 4));
        CK(hipMemset(dof, 0, 9 * N * 4));
        if (opaque)
            hipLaunchKernelGGL(k<true>, dim3(N / 256), dim3(256), 0, 0, dxi, dyi, dxf, dyf, doi, dof);
        else
            hipLaunchKernelGGL(k<false>, dim3(N / 256), dim3(256), 0, 0, dxi, dyi, dxf, dyf, doi, dof);
        CK(hipDeviceSynchronize());
        std::vector<int> oi(9 * N);
        std::vector<float> of(9 * N);
        CK(hipMemcpy(oi.data(), doi, 9 * N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(of.data(), dof, 9 * N * 4, hipMemcpyDeviceToHost));
        printf("%s DPP moves:\n", opaque ? "separate (opaque)" : "foldable");
        for (int c = 0; c < 9; ++c) {
            int bad = 0, first = -1;
            for (int t = 0; t < N; ++t) {
                const int l = t & 63, base = t - l;
                const int nx = base + ((l + 1) & 63), px = base + ((l + 63) & 63);  // rol: lane+1, ror: lane-1
                double want;
                switch (c) {
                    case 0: want = std::abs(yi[t] - xi[nx]); break;
                    case 1: want = yi[t] - xi[nx]; break;
                    case 2: want = xi[nx] - yi[t]; break;
                    case 3: want = yi[t] + xi[nx]; break;
                    case 4: want = yf[t] + xf[nx]; break;
                    case 5: want = yf[t] - xf[nx]; break;
                    case 6: want = xf[nx] - yf[t]; break;
                    case 7: want = yf[t] + xf[px]; break;
                    default: want = std::abs(yi[t] - xi[px]); break;
                }
                const double got = (c >= 4 && c <= 7) ? (double)of[9 * t + c] : (double)oi[9 * t + c];
                if (got != want) {
                    ++bad;
                    if (first < 0) first = t;
                }
            }
            printf("  %-16s %5d of %d lanes wrong", names[c], bad, N);
            if (first >= 0) printf("  (first: thread %d)", first);
            printf("\n");
        }
    }
    return 0;
}
