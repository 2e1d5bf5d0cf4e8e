// Cross-stream ordering cost lab: what an event record costs on the producing stream.
// A dirty-L2 writer kernel is followed on the same stream by a second kernel; in between, one of
//   none | hipEventRecord (default flags = system-scope release) | a hipEventReleaseToDevice
//   event | both + a wait of a second stream on it.
// Reports the median wall time of N (writer, marker, writer) iterations over the plain pair.
// Not product code: it sizes the hand-offs in DESIGN.md §6.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o event_lab event_lab.hip
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

__global__ void __launch_bounds__(256) k_fill(double* a, long long n, double v) {
    for (long long q = blockIdx.x * 256LL + threadIdx.x; q < n; q += (long long)gridDim.x * 256) a[q] = v + q;
}

int main(int argc, char** argv) {
    const long long n = argc > 1 ? atoll(argv[1]) : (16LL << 20) / 8;  // 16 MiB: fits the L2s + MALL
    const int iters = 200;
    double* a;
    CK(hipMalloc(&a, n * 8));
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, -1));
    hipEvent_t t0, t1, e_sys, e_dev;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    CK(hipEventCreateWithFlags(&e_sys, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e_dev, hipEventDisableTiming | hipEventReleaseToDevice));
    const int grid = 256 * 8;
    const char* names[] = {"none", "record sys", "record dev", "record sys + wait", "record dev + wait"};
    for (int rep = 0; rep < 2; ++rep) {
        for (int mode = 0; mode < 5; ++mode) {
            std::vector<float> ms;
            for (int r = 0; r < 7; ++r) {
                CK(hipEventRecord(t0, s));
                for (int it = 0; it < iters; ++it) {
                    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(256), 0, s, a, n, 1.0 * it);
                    if (mode == 1 || mode == 3) CK(hipEventRecord(e_sys, s));
                    if (mode == 2 || mode == 4) CK(hipEventRecord(e_dev, s));
                    if (mode == 3) CK(hipStreamWaitEvent(s2, e_sys, 0));
                    if (mode == 4) CK(hipStreamWaitEvent(s2, e_dev, 0));
                }
                CK(hipEventRecord(t1, s));
                CK(hipEventSynchronize(t1));
                CK(hipStreamSynchronize(s2));
                float t;
                CK(hipEventElapsedTime(&t, t0, t1));
                ms.push_back(t * 1000.f / iters);
            }
            std::sort(ms.begin(), ms.end());
            printf("%-20s %.2f us per kernel (+marker)\n", names[mode], ms[ms.size() / 2]);
            fflush(stdout);
        }
    }
    return 0;
}
