// gtmi_halo.hip -- batched strided-box <-> contiguous-buffer copies for the halo exchanges.
//
// One launch handles up to GTMI_HALO_LAUNCH_BOXES faces (blockIdx.y = box); a box is walked
// I-fastest so field reads/writes are coalesced along the contiguous I axis of the (2,1,0)
// layout and the buffer side is fully contiguous. Grid-stride over the largest box.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "gtmi_roctx.h"

#include "gtmi_halo.h"

#define GTMI_HALO_LAUNCH_BOXES 16  // boxes passed by value per launch (kernel-argument budget)

struct LaunchBoxes {
    gtmi_box b[GTMI_HALO_LAUNCH_BOXES];
};

static thread_local char g_err[512];

template <typename T>
__device__ __forceinline__ void copy_box(const gtmi_box& bx, int direction) {
    const int64_t ei = bx.extent[0], ej = bx.extent[1], ek = bx.extent[2];
    const int64_t n = ei * ej * ek;
    T* __restrict__ f = (T*)bx.field;
    T* __restrict__ buf = (T*)bx.buffer;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e % ei;
        const int64_t r = e / ei;
        const int64_t j = r % ej;
        const int64_t k = r / ej;
        const int64_t off = (bx.start[0] + i) * bx.strides[0] + (bx.start[1] + j) * bx.strides[1] +
                            (bx.start[2] + k) * bx.strides[2];
        if (direction == 0)
            buf[e] = f[off];
        else
            f[off] = buf[e];
    }
}

__global__ void __launch_bounds__(256) gtmi_halo_kernel(const LaunchBoxes boxes, int n_boxes, int direction) {
    const int b = (int)blockIdx.y;
    if (b >= n_boxes) return;
    const gtmi_box& bx = boxes.b[b];
    if (bx.itemsize == 8)
        copy_box<uint64_t>(bx, direction);
    else if (bx.itemsize == 4)
        copy_box<uint32_t>(bx, direction);
    else if (bx.itemsize == 2)
        copy_box<uint16_t>(bx, direction);
    else
        copy_box<uint8_t>(bx, direction);
}

extern "C" const char* gtmi_halo_last_error(void) { return g_err; }
extern "C" int gtmi_halo_abi_version(void) { return GTMI_HALO_ABI_VERSION; }

static int halo_copy_impl(const gtmi_box* boxes, int32_t n_boxes, int32_t direction, void* stream_ptr);

extern "C" int gtmi_halo_copy(const gtmi_box* boxes, int32_t n_boxes, int32_t direction, void* stream_ptr) {
    GTMI_RANGE_PUSH(direction == 0 ? "gtmi_halo:pack" : "gtmi_halo:unpack");
    const int rc = halo_copy_impl(boxes, n_boxes, direction, stream_ptr);
    GTMI_RANGE_POP();
    return rc;
}

static int halo_copy_impl(const gtmi_box* boxes, int32_t n_boxes, int32_t direction, void* stream_ptr) {
    g_err[0] = 0;
    if (n_boxes < 0 || n_boxes > GTMI_HALO_MAX_BOXES || (direction != 0 && direction != 1)) {
        snprintf(g_err, sizeof(g_err), "bad arguments: n_boxes=%d direction=%d", (int)n_boxes, (int)direction);
        return 1;
    }
    hipStream_t stream = (hipStream_t)stream_ptr;
    for (int32_t first = 0; first < n_boxes; first += GTMI_HALO_LAUNCH_BOXES) {
        LaunchBoxes lb;
        memset(&lb, 0, sizeof(lb));
        int nb = n_boxes - first < GTMI_HALO_LAUNCH_BOXES ? n_boxes - first : GTMI_HALO_LAUNCH_BOXES;
        int64_t maxn = 0;
        for (int b = 0; b < nb; ++b) {
            lb.b[b] = boxes[first + b];
            const int64_t n = lb.b[b].extent[0] * lb.b[b].extent[1] * lb.b[b].extent[2];
            if (n < 0 || lb.b[b].field == NULL || lb.b[b].buffer == NULL) {
                snprintf(g_err, sizeof(g_err), "box %d: null pointer or negative extent", first + b);
                return 1;
            }
            if (n > maxn) maxn = n;
        }
        if (maxn == 0) continue;
        int64_t blocks = (maxn + 255) / 256;
        if (blocks > 2048) blocks = 2048;  // grid-stride beyond: ~8 waves per CU per box
        hipLaunchKernelGGL(gtmi_halo_kernel, dim3((unsigned)blocks, (unsigned)nb), dim3(256), 0, stream, lb, nb,
                           (int)direction);
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "HIP launch failed: %s", hipGetErrorString(err));
        return (int)err;
    }
    return 0;
}
