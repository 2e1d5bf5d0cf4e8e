/*
 * gtmi.h -- C ABI of gt:mi355x generated stencil libraries.
 *
 * Every stencil built by the gt:mi355x backend is one shared library (hipcc, gfx950) that
 * exports exactly the five entry points below. They replace the pybind11 extension that the
 * reference's GridTools backends generate per stencil:
 *
 *   reference: backend/gtc_common.py:65-103  (bindings_main_template)
 *       m.def("run_computation", [](std::array<gt::uint_t,3> domain,
 *                                   <field: py::buffer|py::object>, std::array<gt::int_t,N> origin, ...,
 *                                   <scalar>..., py::object exec_info) {...});
 *   reference caller: backend/gtc_common.py:144-168 (PyExtModuleGenerator.generate_implementation)
 *       pyext_module.run_computation(list(_domain_), field, list(_origin_["field"]), ..., exec_info)
 *
 * Mapping: `domain` -> domain[3]; every (field, origin) pair -> one gtmi_field (borrowed device
 * pointer, per-axis element strides, origin, shape, data-dimension strides/extents); scalars -> gtmi_scalar slots in the
 * stencil's parameter order (gtir.params order, gtc_common.py:148-163); the CUDA/HIP stream
 * (the reference syncs with cupy, gtc_common.py:288-296) -> `stream`. exec_info timing stays
 * on the Python side (run_cpp_start_time / run_cpp_end_time around the call).
 *
 * Ownership: all arrays are borrowed; outputs are written in place inside the compute domain
 * (scratch temporaries, appended after the API fields, are owned by the caller too).
 * Errors: nonzero return (1 = bad arguments, 2 = launch geometry, otherwise a hipError_t);
 * gtmi_last_error() returns a thread-local message for the last failing call.
 * No implicit synchronisation: the kernels are enqueued on `stream`.
 */
#ifndef GTMI_H
#define GTMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GTMI_ABI_VERSION 3
#define GTMI_MAX_DATA_DIMS 4

/* dtype ids = gt4py DataType ids (gtc/common.py:105-118) */
enum gtmi_dtype {
    GTMI_BOOL = 10,
    GTMI_INT8 = 11,
    GTMI_INT16 = 12,
    GTMI_INT32 = 14,
    GTMI_INT64 = 18,
    GTMI_FLOAT32 = 104,
    GTMI_FLOAT64 = 108
};

typedef struct gtmi_field {
    void* data;          /* device address of array element (0,0,0) (NOT origin-shifted) */
    int64_t strides[3];  /* element strides along I, J, K (0 for an axis the field lacks) */
    int64_t origin[3];   /* index of the compute-domain origin inside the array */
    int64_t shape[3];    /* array extent along I, J, K (1 for an absent axis) */
    int32_t dtype;       /* enum gtmi_dtype */
    int32_t ndim;        /* number of spatial axes the field has */
    int32_t n_data_dims; /* trailing data dimensions (Field[(dtype, (n, ...))], GlobalTable) */
    int32_t reserved;
    int64_t data_strides[GTMI_MAX_DATA_DIMS]; /* element strides of the data dimensions */
    int64_t data_shape[GTMI_MAX_DATA_DIMS];   /* their extents (indices are clamped to them) */
} gtmi_field;

typedef union gtmi_scalar {
    double f64;
    float f32;
    int64_t i64;
    int32_t i32;
    int16_t i16;
    int8_t i8;
    uint8_t b;
} gtmi_scalar;

/* Enqueue the stencil over `domain` (ni, nj, nk) on `stream` (a hipStream_t; NULL = default).
 * fields: API fields in definition order (unused optional fields: data = NULL), followed by the
 * scratch temporaries listed in gtmi_stencil_signature(). Returns 0 on success. */
int gtmi_stencil_run(const int64_t* domain, const gtmi_field* fields, int32_t n_fields,
                     const gtmi_scalar* scalars, int32_t n_scalars, void* stream);

/* gtmi_stencil_run over the rows [0, j_split) and [j_split + j_skip, domain[1]) of `domain`
 * only; the rows in between are not touched. One launch per kernel when every kernel of the
 * stencil is a plane kernel without scratch temporaries or horizontal regions, otherwise two
 * passes (the second with every field's J origin advanced by j_split + j_skip).
 * No reference counterpart: the reference has no multi-device path (users cut the domain by
 * hand through origin/domain, stencil_object.py:155-175); this serves the two boundary strips
 * of a J-strip rank after its halo exchange (gt4py_amd/distributed/halo.py). */
int gtmi_stencil_run_jsplit(const int64_t* domain, int64_t j_split, int64_t j_skip, const gtmi_field* fields,
                            int32_t n_fields, const gtmi_scalar* scalars, int32_t n_scalars, void* stream);

/* JSON self-description of the library (codegen/hip.py emits it):
 *   {"abi": 3,
 *    "fields":  [{"name", "dtype", "axes": ["I","J","K"], "data_dims": [...]}, ...]   API fields, in
 *               the order of the gtmi_field array gtmi_stencil_run takes,
 *    "scratch": [{"name", "dtype", "extent": [[i_lo,i_hi],[j_lo,j_hi]], "axes"}, ...] temporaries
 *               the caller allocates (domain + extent) and passes after the API fields,
 *    "scalars": [{"name", "dtype", "used": bool}, ...]                                  in the order of
 *               the gtmi_scalar array,
 *    "kernels": ["PlaneKernel" | "ColumnKernel", ...]}                                   launches, in order.
 * "abi" equals GTMI_ABI_VERSION. */
const char* gtmi_stencil_signature(void);

/* Message of the last failing gtmi_stencil_run on this thread ("" if none). */
const char* gtmi_last_error(void);

/* GTMI_ABI_VERSION the library was built against. */
int gtmi_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GTMI_H */
