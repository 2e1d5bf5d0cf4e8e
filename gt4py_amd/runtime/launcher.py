"""Host-side launcher of a generated stencil library, driven by its self-description.

Every library exports ``gtmi_stencil_signature()`` (JSON: API fields with dtype/axes, scratch
temporaries with dtype/extent, scalars with dtype). ``StencilLauncher`` needs nothing else:
it is shared by the native ``gt:mi355x`` StencilObject and by the adapter that registers the
backend inside the reference gt4py (``gt4py_amd.gt4py_plugin``).

Per call: pack one ``gtmi_field`` per API field (borrowed device pointer, element strides,
origin, shape), append the cached scratch buffers, pack the scalars, call
``gtmi_stencil_run`` on torch's current HIP stream, optionally synchronize.
"""

from __future__ import annotations

import ctypes
import time
import weakref
from typing import Any, Dict, Tuple

import numpy as np

from gt4py_amd.runtime import ffi

_AXES = ("I", "J", "K")
_NEVER = object()


def _layout(a):
    """(data pointer, shape, strides) of a device array: a cached pack is reused only when all
    three still match (a tensor changed in place by set_/resize_/as_strided_ keeps its identity)."""
    st = getattr(a, "stride", None)
    if st is not None:
        return a.data_ptr(), tuple(a.shape), tuple(st())
    cai = a.__cuda_array_interface__
    return cai["data"][0], tuple(cai["shape"]), tuple(cai.get("strides") or ())


def device_tensor(obj):
    """The torch view of a device array argument (torch tensor or __cuda_array_interface__)."""
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


def _np_dtype_of(t) -> np.dtype:
    from gt4py_amd.storage import numpy_dtype_of

    return numpy_dtype_of(t)


# dtype name -> scalar kind of the native prepared launch (csrc/gtmi_fastcall.cpp, enum Kind)
_SCALAR_KIND = {"float64": 0, "float32": 1, "int64": 2, "int32": 3, "int16": 4, "int8": 5, "bool": 6}


_LAUNCHERS = weakref.WeakSet()


def drop_pack_caches() -> None:
    """Forget the packed argument arrays of every launcher (see ``drop_prepared_launches``)."""
    for la in list(_LAUNCHERS):
        la._pack_cache.clear()


class StencilLauncher:
    def __init__(self, lib_path: str, name: str = ""):
        self.lib_path = lib_path
        self.name = name
        self._lib = None
        self._scratch_cache: Dict[Tuple, Any] = {}
        self._pack_cache: Dict[Tuple, Any] = {}
        _LAUNCHERS.add(self)

    @property
    def lib(self) -> ffi.StencilLibrary:
        if self._lib is None:
            self._lib = ffi.load_library(self.lib_path)
            sig = self._lib.signature
            self.fields = sig["fields"]
            self.scratch = sig["scratch"]
            self.scalars = sig["scalars"]
            self.n_fields = len(self.fields) + len(self.scratch)
        return self._lib

    def _scratch_buffers(self, domain, device):
        key = (tuple(domain), str(device))
        if key not in self._scratch_cache:
            from gt4py_amd.storage import staggered_device_buffer

            ni, nj, nk = domain
            out = []
            for s in self.scratch:
                (ilo, ihi), (jlo, jhi) = s["extent"]
                si, sj = ni + ilo + ihi, nj + jlo + jhi
                pi = -(-si // 32) * 32
                if "K" in s.get("axes", ("I", "J", "K")):
                    buf = staggered_device_buffer(pi * sj * nk, np.dtype(s["dtype"]), device)
                    out.append((buf, (si, sj, nk), (1, pi, pi * sj), (ilo, jlo, 0), s["dtype"]))
                else:  # IJ temporary: one plane shared by every level (K stride 0)
                    buf = staggered_device_buffer(pi * sj, np.dtype(s["dtype"]), device)
                    out.append((buf, (si, sj, 1), (1, pi, 0), (ilo, jlo, 0), s["dtype"]))
            self._scratch_cache[key] = out
        return self._scratch_cache[key]

    def pack_fields(self, domain, origin, arrays: Dict[str, Any]):
        """The ``gtmi_field`` array for a call (+ the device), cached per (arrays, origins, domain).

        A repeated call with the same tensor objects, origins and domain reuses the packed structs:
        the entry holds weak references to the arrays and their data pointers, shapes and strides,
        so a freed, re-allocated or re-strided tensor never matches a stale entry.
        """
        lib = self.lib  # noqa: F841  (loads the signature)
        key = (tuple(domain),) + tuple(
            (id(arrays.get(d["name"])), tuple(origin.get(d["name"], ()))) for d in self.fields
        )
        ent = self._pack_cache.get(key)
        if ent is not None:
            refs, ptrs, fields, device = ent
            ok = True
            for d, r, p in zip(self.fields, refs, ptrs):
                a = arrays.get(d["name"])
                if (r is None) != (a is None) or (r is not None and (r() is not a or _layout(a) != p)):
                    ok = False
                    break
            if ok:
                return fields, device
        fields, device, refs, ptrs = self._pack(domain, origin, arrays)
        if len(self._pack_cache) >= 64:
            self._pack_cache.clear()
        self._pack_cache[key] = (refs, ptrs, fields, device)
        return fields, device

    def _pack(self, domain, origin, arrays):
        import torch

        ni, nj, nk = (int(d) for d in domain)
        fields = (ffi.GtmiField * self.n_fields)()
        device = None
        refs, ptrs = [], []
        for idx, decl in enumerate(self.fields):
            name = decl["name"]
            arr = arrays.get(name)
            f = fields[idx]
            if arr is None:
                f.data = None
                refs.append(None)
                ptrs.append(None)
                continue
            t = device_tensor(arr)
            try:
                refs.append(weakref.ref(arr))
            except TypeError:  # not weak-referenceable: never reuse this entry
                refs.append(lambda: _NEVER)
            ptrs.append(_layout(arr))
            device = t.device
            want = np.dtype(decl["dtype"])
            got = _np_dtype_of(t)
            if got != want:
                raise TypeError(f"The dtype of field '{name}' is '{got}' instead of '{want}'")
            org = origin[name]
            axes = decl["axes"]
            ddims = decl.get("data_dims", [])
            st = t.stride()
            sh = t.shape
            if len(sh) != len(axes) + len(ddims):
                raise ValueError(
                    f"Storage for '{name}' has {len(sh)} dimensions, expected {len(axes) + len(ddims)} "
                    f"({axes} + data dimensions {ddims})"
                )
            if len(ddims) > ffi.MAX_DATA_DIMS:
                raise ValueError(f"'{name}': at most {ffi.MAX_DATA_DIMS} data dimensions are supported")
            f.n_data_dims = len(ddims)
            for d in range(len(ddims)):
                f.data_strides[d] = st[len(axes) + d]
                f.data_shape[d] = sh[len(axes) + d]
            d = 0
            for ax in range(3):
                if _AXES[ax] in axes:
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
            f.ndim = len(axes)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        base = len(self.fields)
        for j, (buf, shape, strides, org, dt) in enumerate(self._scratch_buffers((ni, nj, nk), device)):
            f = fields[base + j]
            f.data = buf.data_ptr()
            for ax in range(3):
                f.strides[ax] = strides[ax]
                f.shape[ax] = shape[ax]
                f.origin[ax] = org[ax]
            f.ndim = 3
            f.dtype = ffi.DTYPE_IDS[np.dtype(dt).name]
        return fields, device, refs, ptrs

    def bind(self, domain, origin, arrays: Dict[str, Any], param_names, tensors, *, device_sync=True):
        """A prepared launch for repeated calls with these arrays, origins and domain: the fast
        path of ``StencilObject.__call__`` / ``FrozenStencil.__call__``.

        ``tensors``: the field arguments in call order (plain torch tensors). Returns
        ``launch(fields, params) -> bool`` -- ``fields`` the field arguments of a call in the same
        order, ``params`` its scalar values in ``param_names`` order -- which launches and returns
        True when every field is still the same tensor (same object, data pointer, sizes, strides and
        dtype) and
        the current device is the arrays' one, else returns False (take the ordinary path); or
        None when this call cannot be prepared. Everything a call does not change (the packed
        ``gtmi_field`` array, the domain, the scalar slots, the foreign function) is built here
        once. With the native extension (``runtime/fastcall.py``) the whole launch is one C++
        call; without it, a ctypes closure does the same.
        """
        import torch

        from gt4py_amd.runtime import fastcall

        lib = self.lib
        fields, device = self.pack_fields(domain, origin, arrays)
        if device is None or device.index is None:
            return None
        idx = device.index
        n_sc = len(self.scalars)
        scalars = (ffi.GtmiScalar * max(1, n_sc))()
        setters = []
        for j, s in enumerate(self.scalars):
            if s["name"] in param_names:
                setters.append((param_names.index(s["name"]), j, s["dtype"]))
            elif s.get("used", True):
                return None
            else:
                ffi.set_scalar(scalars[j], s["dtype"], 0)
        ni, nj, nk = (int(d) for d in domain)
        name = self.name
        native = fastcall.module()
        if native is not None:
            return native.Prepared(
                ctypes.cast(lib.run, ctypes.c_void_p).value, ctypes.cast(lib.lib.gtmi_last_error, ctypes.c_void_p).value,
                (ni, nj, nk), ctypes.addressof(fields), self.n_fields, ctypes.addressof(scalars), n_sc,
                [(pos, j, _SCALAR_KIND[dt]) for pos, j, dt in setters], len(param_names),
                list(tensors), idx,
                bool(device_sync), name)
        import weakref

        dom = (ctypes.c_int64 * 3)(ni, nj, nk)
        run = lib.run
        n_fields = self.n_fields
        raw_stream = torch._C._cuda_getCurrentRawStream
        current_device = torch._C._cuda_getDevice
        slots = [(scalars[j], pos, *ffi.SCALAR_SLOTS[dt]) for pos, j, dt in setters]
        # strides and dtype too: transpose_/as_strided_ re-stride a tensor in place and keep its
        # identity, data pointer and sizes
        checks = [(weakref.ref(t), t.data_ptr(), t.shape, t.stride(), t.dtype) for t in tensors]
        n_params = len(param_names)

        def launch(fields_now, params) -> bool:
            if len(fields_now) != len(checks) or len(params) != n_params:
                return False
            for a, (ref, ptr, shape, stride, dtype) in zip(fields_now, checks):
                if (ref() is not a or a.data_ptr() != ptr or a.shape != shape or a.stride() != stride
                        or a.dtype != dtype):
                    return False
            if current_device() != idx:
                return False
            for slot, pos, attr, conv in slots:
                setattr(slot, attr, conv(params[pos]))
            rc = run(dom, fields, n_fields, scalars, n_sc, raw_stream(idx))
            if rc != 0:
                raise RuntimeError(f"gt:mi355x stencil '{name}' failed: {lib.last_error()}")
            if device_sync:
                torch.cuda.current_stream(device).synchronize()
            return True

        launch.keep = (fields, scalars, dom)  # the foreign call borrows these
        return launch

    def __call__(self, domain, origin, arrays: Dict[str, Any], params: Dict[str, Any], *, device_sync=True,
                 exec_info=None, rows=None) -> None:
        """``rows=(j_split, j_skip)``: only rows [0, j_split) and [j_split + j_skip, nj) of ``domain``
        (``gtmi_stencil_run_jsplit``)."""
        import torch

        lib = self.lib
        ni, nj, nk = (int(d) for d in domain)
        fields, device = self.pack_fields(domain, origin, arrays)
        n_sc = len(self.scalars)
        scalars = (ffi.GtmiScalar * max(1, n_sc))()
        for j, s in enumerate(self.scalars):
            v = params.get(s["name"])
            if v is None and s.get("used", True):
                raise TypeError(
                    f"The type of parameter '{s['name']}' is '{type(v)}' instead of '{np.dtype(s['dtype'])}'"
                )
            ffi.set_scalar(scalars[j], s["dtype"], 0 if v is None else v)
        dom = (ctypes.c_int64 * 3)(ni, nj, nk)
        if device.index is not None and device.index != torch.cuda.current_device():
            with torch.cuda.device(device):
                self._run(lib, dom, fields, scalars, n_sc, device, device_sync, exec_info, rows)
        else:
            self._run(lib, dom, fields, scalars, n_sc, device, device_sync, exec_info, rows)

    def _run(self, lib, dom, fields, scalars, n_sc, device, device_sync, exec_info, rows=None):
        import torch

        stream = torch.cuda.current_stream(device)
        if exec_info is not None:
            stream.synchronize()
            exec_info["run_cpp_start_time"] = time.perf_counter()
        if rows is None:
            rc = lib.run(dom, fields, self.n_fields, scalars, n_sc, ctypes.c_void_p(stream.cuda_stream))
        else:
            rc = lib.run_jsplit(dom, int(rows[0]), int(rows[1]), fields, self.n_fields, scalars, n_sc,
                                ctypes.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"gt:mi355x stencil '{self.name}' failed: {lib.last_error()}")
        if device_sync or exec_info is not None:
            stream.synchronize()
        if exec_info is not None:
            exec_info["run_cpp_end_time"] = time.perf_counter()
