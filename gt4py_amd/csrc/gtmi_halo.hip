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

// A box is ej*ek ROWS of ei elements contiguous along I (the field's I stride) and along the
// buffer. Narrow boxes (the I faces of a 2-D exchange: ei = halo width, one or two 8-B cells per
// row) take one 16-B row per lane when the face row is 16 B and aligned, else one element per
// lane with 32-bit index math (the lanes of a row share its line; the buffer side is contiguous); wide
// boxes (J faces: whole rows) take 64-element chunks of a row per wave, coalesced along I. Row and
// chunk indices are computed once per lane (narrow, 32-bit when the box allows) or once per wave
// in scalar registers (wide), not per element: the round-2 kernel's three 64-bit divisions per
// element dominated the narrow I faces.
#define GTMI_HALO_NARROW 16

template <typename T>
__device__ __forceinline__ void copy_row(const gtmi_box& bx, int64_t row, int64_t i0, int64_t n, int direction,
                                         int64_t step) {
    const int64_t ej = bx.extent[1], ei = bx.extent[0];
    const int64_t j = row % ej, k = row / ej;
    T* __restrict__ f = (T*)bx.field +
                        ((bx.start[1] + j) * bx.strides[1] + (bx.start[2] + k) * bx.strides[2] + bx.start[0] * bx.strides[0]);
    T* __restrict__ buf = (T*)bx.buffer + row * ei;
    const int64_t si = bx.strides[0];
    if (direction == 0) {
        for (int64_t i = i0; i < n; i += step) buf[i] = f[i * si];
    } else {
        for (int64_t i = i0; i < n; i += step) f[i * si] = buf[i];
    }
}

template <typename T>
__device__ __forceinline__ void copy_box(const gtmi_box& bx, int direction) {
    const int64_t ei = bx.extent[0], ej = bx.extent[1], ek = bx.extent[2];
    const int64_t rows = ej * ek;
    if (ei <= 0 || rows <= 0) return;
    if (ei <= GTMI_HALO_NARROW) {
        const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
        const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        const int64_t si = bx.strides[0], sj = bx.strides[1], sk = bx.strides[2];
        const int64_t base = bx.start[0] * si + bx.start[1] * sj + bx.start[2] * sk;
        // a 16-B face row (two 8-B or four 4-B cells) moved as ONE 16-B access per lane: the
        // lanes of a wave then fill 1 KB of the buffer contiguously
        const bool vec16 = ei * (int64_t)sizeof(T) == 16 && si == 1 &&
                           ((uintptr_t)((T*)bx.field + base) % 16) == 0 && (sj * (int64_t)sizeof(T)) % 16 == 0 &&
                           (sk * (int64_t)sizeof(T)) % 16 == 0 && ((uintptr_t)bx.buffer % 16) == 0;
        if (vec16 && rows <= 0xffffffffLL) {
            const uint32_t uej = (uint32_t)ej;
            for (int64_t r = t0; r < rows; r += nthreads) {
                const uint32_t ur = (uint32_t)r, j = ur % uej, k = ur / uej;
                ulonglong2* f = (ulonglong2*)((T*)bx.field + base + (int64_t)j * sj + (int64_t)k * sk);
                ulonglong2* b = (ulonglong2*)bx.buffer + r;
                if (direction == 0)
                    *b = *f;
                else
                    *f = *b;
            }
            return;
        }
        const int64_t n = rows * ei;  // one element per lane: lanes of a row share its line
        if (n <= 0xffffffffLL) {
            const uint32_t uei = (uint32_t)ei, uej = (uint32_t)ej;
            for (int64_t e = t0; e < n; e += nthreads) {
                const uint32_t ue = (uint32_t)e, r = ue / uei, i = ue - r * uei, j = r % uej, k = r / uej;
                T* f = (T*)bx.field + base + (int64_t)i * si + (int64_t)j * sj + (int64_t)k * sk;
                T* b = (T*)bx.buffer + e;
                if (direction == 0)
                    *b = *f;
                else
                    *f = *b;
            }
        } else {
            for (int64_t r = t0; r < rows; r += nthreads) copy_row<T>(bx, r, 0, ei, direction, 1);
        }
        return;
    }
    // wide: one wave per (row, 64-element chunk); wave-uniform indices in scalar registers
    const int lane = (int)(threadIdx.x & 63);
    const int64_t cpr = (ei + 63) / 64;
    const int64_t units = rows * cpr;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    for (int64_t u = w0; u < units; u += nwaves) {
        const int64_t row = u / cpr, c = u - row * cpr;
        const int64_t i0 = c * 64 + lane;
        const int64_t n = (c + 1) * 64 < ei ? (c + 1) * 64 : ei;
        copy_row<T>(bx, row, i0, n, direction, 64);
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
        // work units of the largest box: rows (narrow boxes, one per lane) or 64-element row
        // chunks (wide boxes, one per wave)
        int64_t units = 0;
        for (int b = 0; b < nb; ++b) {
            const int64_t ei = lb.b[b].extent[0], rows = lb.b[b].extent[1] * lb.b[b].extent[2];
            const int64_t lanes = ei <= GTMI_HALO_NARROW ? rows * ei : rows * ((ei + 63) / 64) * 64;
            if (lanes > units) units = lanes;
        }
        int64_t blocks = (units + 255) / 256;
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
