// Prepared launches: the native half of the StencilObject / FrozenStencil fast path.
//
// A repeated stencil call with the same arrays, domain and origin needs no argument extraction,
// validation or packing (the reference caches the validated signature in
// `_domain_origin_cache`, src/gt4py/cartesian/stencil_object.py:579-593, and still rebuilds the
// pybind11 argument list per call, gtc_common.py:79-101). `Prepared` holds what one such call
// signature needs -- the packed gtmi_field array, the domain, the scalar slots and the
// library's gtmi_stencil_run -- and a call
//
//     prepared(fields: tuple, params: tuple) -> bool
//
// checks that every field argument is still the tensor the entry was made for (same object via
// its weak reference, same data pointer, sizes, strides and dtype -- a tensor re-strided in place by
// transpose_/as_strided_ keeps its identity, pointer and sizes), stores the scalar parameters with the
// ordinary path's conversions, reads the caller's current HIP stream from c10 and launches.
// Parameter values are not re-validated, as in the reference, whose _validate_args runs only
// when the (shapes, origins, parameter names, domain) cache misses (stencil_object.py:578-591).
// False means "take the ordinary path" (another tensor, another current device, a parameter the
// conversions would treat differently); a failing launch raises RuntimeError with
// gtmi_last_error(). The GIL is held during the (non-blocking) launch, as the reference's
// binding does.
#include <Python.h>

#include <c10/hip/HIPFunctions.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>
#include <cstring>
#include <vector>

#include "gtmi.h"

namespace {

typedef int (*run_fn)(const int64_t*, const gtmi_field*, int32_t, const gtmi_scalar*, int32_t, void*);
typedef const char* (*err_fn)(void);

enum Kind { K_F64 = 0, K_F32, K_I64, K_I32, K_I16, K_I8, K_BOOL };

struct Setter {
    int pos;   // index in the params tuple
    int slot;  // gtmi_scalar slot
    int kind;
};

struct Check {
    PyObject* wr;  // weak reference to the tensor (owned)
    const void* ptr;
    std::vector<int64_t> sizes;
    std::vector<int64_t> strides;
    c10::ScalarType dtype;
};

struct Prepared {
    PyObject_HEAD
    run_fn run;
    err_fn err;
    int64_t dom[3];
    std::vector<gtmi_field>* fields;
    std::vector<gtmi_scalar>* scalars;
    std::vector<Setter>* setters;
    std::vector<Check>* checks;
    int32_t n_scalars;  // slots the stencil declares (the array holds at least one)
    int n_params;
    int device;
    int sync;
    PyObject* name;
};

bool set_scalar(gtmi_scalar& s, int kind, PyObject* v) {
    // the conversions of the ordinary path (ffi.SCALAR_SLOTS: float(v), int(v) on integers, truth
    // value); a value they would treat differently (a float for an integer parameter) returns
    // false and takes the ordinary path
    switch (kind) {
    case K_F64:
    case K_F32: {
        double d = PyFloat_AsDouble(v);
        if (d == -1.0 && PyErr_Occurred()) { PyErr_Clear(); return false; }
        if (kind == K_F64) s.f64 = d;
        else s.f32 = (float)d;
        return true;
    }
    case K_BOOL: {
        int b = PyObject_IsTrue(v);
        if (b < 0) { PyErr_Clear(); return false; }
        s.b = (uint8_t)b;
        return true;
    }
    default: {
        if (PyFloat_Check(v)) return false;
        int overflow = 0;
        long long x = PyLong_AsLongLongAndOverflow(v, &overflow);  // ints and __index__ objects
        if (overflow || (x == -1 && PyErr_Occurred())) { PyErr_Clear(); return false; }
        if (kind == K_I64) s.i64 = x;
        else if (kind == K_I32) s.i32 = (int32_t)x;
        else if (kind == K_I16) s.i16 = (int16_t)x;
        else s.i8 = (int8_t)x;
        return true;
    }
    }
}

PyObject* prepared_call(PyObject* self_, PyObject* args, PyObject* kwargs) {
    Prepared* self = (Prepared*)self_;
    PyObject *fields, *params;
    if (kwargs || PyTuple_GET_SIZE(args) != 2) {
        PyErr_SetString(PyExc_TypeError, "prepared launch takes (fields, params)");
        return nullptr;
    }
    fields = PyTuple_GET_ITEM(args, 0);
    params = PyTuple_GET_ITEM(args, 1);
    if (!PyTuple_Check(fields) || !PyTuple_Check(params)) Py_RETURN_FALSE;
    const std::vector<Check>& checks = *self->checks;
    if ((size_t)PyTuple_GET_SIZE(fields) != checks.size() || PyTuple_GET_SIZE(params) != self->n_params)
        Py_RETURN_FALSE;
    for (size_t i = 0; i < checks.size(); ++i) {
        PyObject* obj = PyTuple_GET_ITEM(fields, i);
        if (PyWeakref_GetObject(checks[i].wr) != obj || !THPVariable_CheckExact(obj)) Py_RETURN_FALSE;
        const at::Tensor& t = THPVariable_Unpack(obj);
        if (t.data_ptr() != checks[i].ptr) Py_RETURN_FALSE;
        c10::IntArrayRef sz = t.sizes();
        if (sz.size() != checks[i].sizes.size() ||
            std::memcmp(sz.data(), checks[i].sizes.data(), sz.size() * sizeof(int64_t)) != 0)
            Py_RETURN_FALSE;
        c10::IntArrayRef st = t.strides();  // same rank as the sizes
        if (std::memcmp(st.data(), checks[i].strides.data(), st.size() * sizeof(int64_t)) != 0 ||
            t.scalar_type() != checks[i].dtype)
            Py_RETURN_FALSE;
    }
    if ((int)c10::hip::current_device() != self->device) Py_RETURN_FALSE;
    gtmi_scalar* sc = self->scalars->data();
    for (const Setter& s : *self->setters)
        if (!set_scalar(sc[s.slot], s.kind, PyTuple_GET_ITEM(params, s.pos))) Py_RETURN_FALSE;
    hipStream_t stream = c10::hip::getCurrentHIPStream((c10::DeviceIndex)self->device).stream();
    int rc = self->run(self->dom, self->fields->data(), (int32_t)self->fields->size(), sc, self->n_scalars,
                       (void*)stream);
    if (rc != 0) {
        PyErr_Format(PyExc_RuntimeError, "gt:mi355x stencil '%U' failed: %s", self->name, self->err());
        return nullptr;
    }
    if (self->sync) {
        hipError_t e;
        Py_BEGIN_ALLOW_THREADS
        e = hipStreamSynchronize(stream);
        Py_END_ALLOW_THREADS
        if (e != hipSuccess) {
            PyErr_Format(PyExc_RuntimeError, "gt:mi355x stencil '%U': %s", self->name, hipGetErrorString(e));
            return nullptr;
        }
    }
    Py_RETURN_TRUE;
}

void prepared_dealloc(PyObject* self_) {
    Prepared* self = (Prepared*)self_;
    if (self->checks)
        for (Check& c : *self->checks) Py_XDECREF(c.wr);
    delete self->fields;
    delete self->scalars;
    delete self->setters;
    delete self->checks;
    Py_XDECREF(self->name);
    Py_TYPE(self_)->tp_free(self_);
}

// Prepared(run_addr, err_addr, domain(3), fields_addr, n_fields, scalars_addr (max(1, n) slots), n_scalars,
//          setters: [(param_pos, slot, kind)], n_params, tensors: [tensor], device, sync, name)
// The field and scalar arrays are copied: the ctypes objects they come from need not outlive it.
PyObject* prepared_new(PyTypeObject* type, PyObject* args, PyObject* kwargs) {
    unsigned long long run_addr, err_addr, fields_addr, scal_addr;
    long long d0, d1, d2;
    int n_fields, n_sc, n_params, device, sync;
    PyObject *setters, *tensors, *name;
    if (!PyArg_ParseTuple(args, "KK(LLL)KiKiOiOipU", &run_addr, &err_addr, &d0, &d1, &d2, &fields_addr, &n_fields,
                          &scal_addr, &n_sc, &setters, &n_params, &tensors, &device, &sync, &name))
        return nullptr;
    if (n_fields < 0 || n_sc < 0 || !PyList_Check(setters) || !PyList_Check(tensors)) {
        PyErr_SetString(PyExc_ValueError, "bad prepared-launch arguments");
        return nullptr;
    }
    Prepared* self = (Prepared*)type->tp_alloc(type, 0);
    if (!self) return nullptr;
    self->run = (run_fn)(uintptr_t)run_addr;
    self->err = (err_fn)(uintptr_t)err_addr;
    self->dom[0] = d0;
    self->dom[1] = d1;
    self->dom[2] = d2;
    const gtmi_field* fsrc = (const gtmi_field*)(uintptr_t)fields_addr;
    self->fields = new std::vector<gtmi_field>(fsrc, fsrc + n_fields);
    const gtmi_scalar* ssrc = (const gtmi_scalar*)(uintptr_t)scal_addr;
    self->scalars = new std::vector<gtmi_scalar>(ssrc, ssrc + (n_sc > 0 ? n_sc : 1));
    self->n_scalars = n_sc;
    self->setters = new std::vector<Setter>();
    self->checks = new std::vector<Check>();
    self->n_params = n_params;
    self->device = device;
    self->sync = sync;
    Py_INCREF(name);
    self->name = name;
    for (Py_ssize_t i = 0; i < PyList_GET_SIZE(setters); ++i) {
        Setter s;
        if (!PyArg_ParseTuple(PyList_GET_ITEM(setters, i), "iii", &s.pos, &s.slot, &s.kind)) goto fail;
        if (s.pos < 0 || s.pos >= n_params || s.slot < 0 || s.slot >= n_sc || s.kind < K_F64 || s.kind > K_BOOL) {
            PyErr_SetString(PyExc_ValueError, "bad scalar setter");
            goto fail;
        }
        self->setters->push_back(s);
    }
    for (Py_ssize_t i = 0; i < PyList_GET_SIZE(tensors); ++i) {
        PyObject* t = PyList_GET_ITEM(tensors, i);
        if (!THPVariable_CheckExact(t)) {
            PyErr_SetString(PyExc_TypeError, "prepared launches take torch.Tensor fields");
            goto fail;
        }
        Check c;
        c.wr = PyWeakref_NewRef(t, nullptr);
        if (!c.wr) goto fail;
        const at::Tensor& tt = THPVariable_Unpack(t);
        c.ptr = tt.data_ptr();
        c.sizes.assign(tt.sizes().begin(), tt.sizes().end());
        c.strides.assign(tt.strides().begin(), tt.strides().end());
        c.dtype = tt.scalar_type();
        self->checks->push_back(std::move(c));
    }
    return (PyObject*)self;
fail:
    Py_DECREF(self);
    return nullptr;
}

PyTypeObject PreparedType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyModuleDef module_def = {PyModuleDef_HEAD_INIT, "_gtmi_fastcall",
                          "Prepared gt:mi355x stencil launches (StencilObject fast path).", -1, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__gtmi_fastcall(void) {
    PreparedType.tp_name = "gt4py_amd._gtmi_fastcall.Prepared";
    PreparedType.tp_basicsize = sizeof(Prepared);
    PreparedType.tp_flags = Py_TPFLAGS_DEFAULT;
    PreparedType.tp_new = prepared_new;
    PreparedType.tp_dealloc = prepared_dealloc;
    PreparedType.tp_call = prepared_call;
    PreparedType.tp_doc = "Prepared(...)(fields, params) -> bool: a launch prepared for one call signature";
    if (PyType_Ready(&PreparedType) < 0) return nullptr;
    PyObject* m = PyModule_Create(&module_def);
    if (!m) return nullptr;
    Py_INCREF(&PreparedType);
    if (PyModule_AddObject(m, "Prepared", (PyObject*)&PreparedType) < 0) {
        Py_DECREF(&PreparedType);
        Py_DECREF(m);
        return nullptr;
    }
    PyModule_AddIntConstant(m, "ABI", 2);
    return m;
}
