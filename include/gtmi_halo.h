/*
 * gtmi_halo.h -- C ABI of the halo pack/unpack library used by the multi-GPU drivers
 * (gt4py_amd/distributed/{halo,decomp2d}.py).
 *
 * The reference has no multi-device support; there is no reference
 * interface this replaces. One call moves every face of one exchange phase -- all fields, all
 * directions -- between the strided fields and the contiguous message buffers handed to RCCL,
 * in a single kernel launch on `stream` (instead of one copy kernel per face and field).
 */
#ifndef GTMI_HALO_H
#define GTMI_HALO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GTMI_HALO_ABI_VERSION 1
#define GTMI_HALO_MAX_BOXES 64

typedef struct gtmi_box {
    void* field;         /* device address of the field's element (0,0,0) */
    int64_t strides[3];  /* element strides along I, J, K */
    int64_t start[3];    /* first index of the box along I, J, K */
    int64_t extent[3];   /* box size along I, J, K */
    void* buffer;        /* contiguous device buffer: box element (i,j,k) at ((k*ej + j)*ei + i) */
    int32_t itemsize;    /* 4 or 8 bytes */
    int32_t reserved;
} gtmi_box;

/* direction 0: field -> buffer (pack); 1: buffer -> field (unpack). Returns 0 on success. */
int gtmi_halo_copy(const gtmi_box* boxes, int32_t n_boxes, int32_t direction, void* stream);

const char* gtmi_halo_last_error(void);
int gtmi_halo_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GTMI_HALO_H */
