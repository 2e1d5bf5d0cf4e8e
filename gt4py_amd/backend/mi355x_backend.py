"""``gt:mi355x`` backend: GTScript stencils as hand-written-skeleton HIP kernels for MI355X.

Plugs into the same registry/StencilObject contract as the reference backends
(``src/gt4py/cartesian/backend/gtcpp_backend.py:168-183`` ``GTGpuBackend``): ``generate()``
plans the launches (``codegen/plan.py``), emits one HIP translation unit
(``codegen/hip.py``), compiles it with hipcc for gfx950 (``runtime/jit.py``) and returns a
``StencilObject`` subclass whose ``run`` calls ``gtmi_stencil_run`` through ctypes.

Storage: I-first layout ``(2, 1, 0)`` (I contiguous, then J, then K), 32-element alignment of
the aligned index, device = ROCm GPU via torch tensors -- the layout the reference uses for
``gt:gpu`` (``storage/cartesian/layout_registry.py:87-122``), minus CuPy.

There is no CPU fallback: without the compiled library or a ROCm device the call raises.
"""

from __future__ import annotations

import ctypes
import time
from typing import Any, Dict, Tuple

import numpy as np

from gt4py_amd.backend.base import BaseBackend, register
from gt4py_amd.codegen import hip as hipgen
from gt4py_amd.codegen.plan import make_plan
from gt4py_amd.runtime import ffi, jit
from gt4py_amd.storage.layout import layout_checker_factory, layout_maker_factory

_layout = layout_maker_factory((2, 1, 0))


def _tensor_of(obj):
    import torch

    if isinstance(obj, torch.Tensor):
        t = obj
    elif hasattr(obj, "__cuda_array_interface__"):
        t = torch.as_tensor(obj, device="cuda")
    else:
        raise TypeError(
            f"gt:mi355x expects device arrays (torch ROCm tensors or objects with __cuda_array_interface__), "
            f"got {type(obj).__name__}; allocate with gt4py_amd.storage.*(backend='gt:mi355x')"
        )
    if not t.is_cuda:
        raise TypeError("gt:mi355x expects tensors on the ROCm device (tensor.is_cuda is False)")
    return t


class _Compiled:
    """Everything a call needs: the library and the argument layout."""

    def __init__(self, analysis, plan, source, signature, lib_path, options):
        self.analysis = analysis
        self.plan = plan
        self.source = source
        self.signature = signature
        self.lib_path = lib_path
        self.options = options
        self._lib = None
        st = analysis.stencil
        self.field_params = st.field_params()
        self.scalar_params = st.scalar_params()
        self.n_fields = len(self.field_params) + len(plan.scratch)
        self.scratch_decls = [(t, st.decl(t).dtype) for t in plan.scratch]
        self._scratch_cache: Dict[Tuple, Any] = {}

    @property
    def lib(self):
        if self._lib is None:
            self._lib = ffi.load_library(self.lib_path)
        return self._lib

    def _scratch(self, domain, device):
        key = (tuple(domain), str(device))
        if key not in self._scratch_cache:
            import torch

            from gt4py_amd.storage import torch_dtype

            ni, nj, nk = domain
            out = []
            for name, dtype in self.scratch_decls:
                (ilo, ihi), (jlo, jhi) = self.plan.scratch_extent[name]
                si = ni + ilo + ihi
                sj = nj + jlo + jhi
                pi = -(-si // 32) * 32
                buf = torch.empty(pi * sj * nk, dtype=torch_dtype(dtype.np_dtype), device=device)
                out.append((buf, (si, sj, nk), (1, pi, pi * sj), (ilo, jlo, 0)))
            self._scratch_cache[key] = out
        return self._scratch_cache[key]

    def __call__(self, domain, origin, exec_info, kwargs):
        import torch

        ni, nj, nk = (int(d) for d in domain)
        fields = (ffi.GtmiField * self.n_fields)()
        device = None
        for idx, decl in enumerate(self.field_params):
            arr = kwargs.get(decl.name)
            f = fields[idx]
            if arr is None:
                f.data = None
                continue
            t = _tensor_of(arr)
            device = t.device
            want = decl.dtype.np_dtype
            from gt4py_amd.storage import numpy_dtype_of

            if numpy_dtype_of(t) != want:
                raise TypeError(f"The dtype of field '{decl.name}' is '{numpy_dtype_of(t)}' instead of '{want}'")
            if decl.data_dims:
                raise NotImplementedError("data dimensions are not supported by gt:mi355x yet")
            org = origin[decl.name]
            mask = decl.mask
            st = t.stride()
            sh = t.shape
            d = 0
            for ax in range(3):
                if mask[ax]:
                    f.strides[ax] = st[d]
                    f.shape[ax] = sh[d]
                    f.origin[ax] = int(org[d])
                    d += 1
                else:
                    f.strides[ax] = 0
                    f.shape[ax] = 1
                    f.origin[ax] = 0
            f.data = t.data_ptr()
            f.dtype = ffi.DTYPE_IDS[want.name]
            f.ndim = sum(mask)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        base = len(self.field_params)
        for j, (buf, shape, strides, org) in enumerate(self._scratch((ni, nj, nk), device)):
            f = fields[base + j]
            f.data = buf.data_ptr()
            for ax in range(3):
                f.strides[ax] = strides[ax]
                f.shape[ax] = shape[ax]
                f.origin[ax] = org[ax]
            f.ndim = 3
            f.dtype = ffi.DTYPE_IDS[self.scratch_decls[j][1].np_dtype.name]
        n_sc = len(self.scalar_params)
        scalars = (ffi.GtmiScalar * max(1, n_sc))()
        for j, s in enumerate(self.scalar_params):
            v = kwargs.get(s.name)
            if v is None:
                v = 0
            ffi.set_scalar(scalars[j], s.dtype.np_dtype.name, v)
        dom = (ctypes.c_int64 * 3)(ni, nj, nk)
        with torch.cuda.device(device):
            stream = torch.cuda.current_stream(device)
            if exec_info is not None:
                torch.cuda.synchronize(device)
                exec_info["run_cpp_start_time"] = time.perf_counter()
            rc = self.lib.run(dom, fields, self.n_fields, scalars, n_sc, ctypes.c_void_p(stream.cuda_stream))
            if rc != 0:
                raise RuntimeError(f"gt:mi355x stencil '{self.analysis.stencil.name}' failed: {self.lib.last_error()}")
            if self.options.get("device_sync", True) or exec_info is not None:
                stream.synchronize()
            if exec_info is not None:
                exec_info["run_cpp_end_time"] = time.perf_counter()


@register
class Mi355xBackend(BaseBackend):
    name = "gt:mi355x"
    options = {
        "device_sync": {"versioning": False, "type": bool, "description": "synchronize the stream after each call"},
        "jchunk": {"versioning": True, "type": int, "description": "J rows per wavefront in plane kernels"},
        "vector": {"versioning": True, "type": int, "description": "I elements per lane in plane kernels (1, 2, 4)"},
        "prefetch": {"versioning": True, "type": int, "description": "rows loaded ahead in plane kernels"},
        "kprefetch": {"versioning": True, "type": int, "description": "levels loaded ahead in column kernels"},
        "col_occupancy": {"versioning": True, "type": int, "description": "max column-kernel blocks per CU (0 = hw)"},
        "strip_align": {"versioning": True, "type": int, "description": "round plane-strip width to a multiple"},
        "order": {"versioning": True, "type": int, "description": "plane work order (0 xcd, 1 k-fast, 2 scatter, 3 natural)"},
        "verbose": {"versioning": False, "type": bool, "description": "print the hipcc command"},
        "oir_pipeline": {"versioning": True, "type": object, "description": "accepted for compatibility"},
    }
    storage_info = {
        "alignment": 32,
        "device": "gpu",
        "layout_map": _layout,
        "is_optimal_layout": layout_checker_factory(_layout),
    }
    languages = {"computation": "hip", "bindings": ["python"]}

    def compile(self) -> _Compiled:
        b = self.builder
        opts = dict(b.options.backend_opts)
        t0 = time.perf_counter()
        plan = make_plan(b.analysis)
        source, signature = hipgen.generate(b.analysis, plan, opts)
        t1 = time.perf_counter()
        path = jit.compile_source(source, verbose=bool(opts.get("verbose")))
        t2 = time.perf_counter()
        if b.options.build_info is not None:
            b.options.build_info["codegen_time"] = t1 - t0
            b.options.build_info["build_time"] = t2 - t1
        return _Compiled(b.analysis, plan, source, signature, path, opts)

    def make_run_impl(self):
        compiled = self.compile()

        def run_impl(domain, origin, exec_info, kwargs):
            compiled(domain, origin, exec_info, kwargs)

        run_impl.compiled = compiled
        return run_impl

    def make_stencil_class(self):
        cls = super().make_stencil_class()
        return cls
