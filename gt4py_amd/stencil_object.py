"""Runtime call path: ``StencilObject`` / ``FrozenStencil``.

Same contract as ``src/gt4py/cartesian/stencil_object.py``:
- singleton, frozen subclasses (``:194-204``),
- ``_call_run`` (``:534-605``): extract arrays, domain/origin cache keyed like ``:38-49``,
  ``_normalize_origins`` (``:499-532``), ``_get_max_domain`` (``:298-343``),
  ``_validate_args`` (``:345-497``) with the same error types and messages,
- ``freeze`` -> ``FrozenStencil`` (``:94-128``) which skips validation,
- ``exec_info`` timestamps and ``__aggregate_data`` counters
  (``backend/templates/stencil_module.py.in:91-169``).

Arrays are borrowed. Device arrays are torch tensors (ROCm) or any object exposing
``__cuda_array_interface__``; host arrays are numpy arrays.
"""

from __future__ import annotations

import abc
import collections.abc
import sys
import time
import warnings
from dataclasses import dataclass
from pickle import dumps
from typing import Any, Callable, ClassVar, Dict, Optional, Tuple

import numpy as np

from gt4py_amd import definitions as gd
from gt4py_amd.definitions import AccessKind, DomainInfo, FieldInfo, ParameterInfo
from gt4py_amd.storage import array_info as storage_array_info


@dataclass
class ArgsInfo:
    device: str
    array: Any
    original_object: Any = None
    origin: Optional[Tuple[int, ...]] = None
    dimensions: Optional[Tuple[str, ...]] = None

    @property
    def shape(self):
        return tuple(self.array.shape)


def _compute_domain_origin_cache_key(field_args_info, parameter_args, domain, origin) -> int:
    field_data = tuple(
        (name, tuple(arg.array.shape), arg.origin or (0, 0, 0)) for name, arg in field_args_info.items() if arg is not None
    )
    return hash((field_data, *parameter_args.keys(), dumps(domain), dumps(origin)))


def _extract_array_infos(field_args, device) -> Dict[str, Optional[ArgsInfo]]:
    infos: Dict[str, Optional[ArgsInfo]] = {}
    for name, arg in field_args.items():
        if arg is None:
            infos[name] = None
            continue
        array, dims, origin = storage_array_info(arg)
        if dims is not None:
            sorted_dims = [d for d in "IJK" if d in dims]
            data_dims = sorted(int(d) for d in dims if str(d).isdigit())
            sorted_dims += [str(d) for d in data_dims]
            perm = [dims.index(sd) for sd in sorted_dims]
            if perm != list(range(len(perm))):
                array = array.permute(*perm) if hasattr(array, "permute") else array.transpose(perm)
            dims = tuple(sorted_dims)
        infos[name] = ArgsInfo(device=device, array=array, original_object=arg, dimensions=dims, origin=origin)
    return infos


def _nt_lt(a, b) -> bool:
    """NumericTuple '<': no element greater and at least one smaller (gtc/definitions.py:141-147)."""
    return any(x < y for x, y in zip(a, b)) and not any(x > y for x, y in zip(a, b))


def _nt_gt(a, b) -> bool:
    return any(x > y for x, y in zip(a, b)) and not any(x < y for x, y in zip(a, b))


def _nt_le(a, b) -> bool:
    return all(x <= y for x, y in zip(a, b))


# ---------------------------------------------------------------------------------- fast path
# A repeated call with the same arrays (same objects, data pointers and shapes), domain and
# origin skips argument extraction, the domain/origin cache key and the argument packing: the
# backend prepares the launch once (``run_impl.bind``, gt:mi355x: ``StencilLauncher.bind``) and
# the generated ``__call__`` checks the arguments inline. The reference has no such layer; its
# validation semantics are kept, because an entry is only made after an ordinary call has
# passed (or, with validate_args=False, skipped) validation for exactly this signature, as the
# reference's ``_domain_origin_cache`` does (stencil_object.py:579-593).

_FAST_MEMO_MAX = 64
_FAST_SIGS_PER_ARGS = 8

# every StencilObject class with a prepared-launch memo (``_gt_fast_memo_``; the memos hold weak
# references to the argument tensors, drop_prepared_launches). Weak: a class that is no longer
# used takes its memo, closures and packed arguments with it
_MEMO_CLASSES = None
_FROZEN = None  # id -> FrozenStencil (weak values; frozen stencils are not hashable), made on first use


def _memo_classes():
    global _MEMO_CLASSES
    if _MEMO_CLASSES is None:
        import weakref

        _MEMO_CLASSES = weakref.WeakSet()
    return _MEMO_CLASSES


def _frozen_set():
    global _FROZEN
    if _FROZEN is None:
        import weakref

        _FROZEN = weakref.WeakValueDictionary()
    return _FROZEN


def drop_prepared_launches() -> None:
    """Forget every prepared launch and packed argument array (they hold weak references to and
    borrowed pointers of the argument tensors): the next call of each signature prepares it
    again. Used before tensors are re-homed in place (``storage.placement.tune_in_place``)."""
    for cls in list(_memo_classes()):
        cls._gt_fast_memo_.clear()
    for fz in list(_frozen_set().values()):
        fz._memo.clear()
    from gt4py_amd.runtime.launcher import drop_pack_caches

    drop_pack_caches()


def _plain_value(v) -> bool:
    """A domain / origin value the fast path may compare with ``==`` (ints, tuples, dicts)."""
    if v is None or type(v) is int:
        return True
    if isinstance(v, (tuple, list)):
        return all(type(x) is int for x in v)
    if isinstance(v, dict):
        return all(isinstance(k, str) and isinstance(x, (tuple, list)) and _plain_value(x) for k, x in v.items())
    return False


def _fast_tensors(field_args, arrays):
    """The field arguments (call order) when a fast-path entry can be made for them: every one a
    plain CUDA torch tensor passed through unchanged (no gt4py dims/origin metadata, no view
    made); else None. The prepared launch re-checks object, data pointer and sizes per call."""
    try:
        import torch
    except ImportError:  # pragma: no cover
        return None
    out = []
    for name, a in field_args.items():
        if type(a) is not torch.Tensor or arrays.get(name) is not a or not a.is_cuda:
            return None
        if getattr(a, "__gt_dims__", None) is not None or getattr(a, "__gt_origin__", None) is not None:
            return None
        out.append(a)
    return out


def _tuple_src(names) -> str:
    return "(" + "".join(f"{n}, " for n in names) + ")"


def _ids_src(field_names) -> str:
    return "(" + "".join(f"id({n}), " for n in field_names) + ")"


@dataclass(frozen=True)
class FrozenStencil:
    """Stencil with pre-computed domain and origin for each field argument."""

    stencil_object: "StencilObject"
    origin: Dict[str, Tuple[int, ...]]
    domain: Tuple[int, ...]

    def __post_init__(self):
        for name, field_info in self.stencil_object.field_info.items():
            if name not in self.origin or len(self.origin[name]) != field_info.ndim:
                raise ValueError(
                    f"'{name}' origin {self.origin.get(name)} is not a {field_info.ndim}-dimensional integer tuple"
                )
        # fast path (see _fast_tensors): entry = prepared launch(fields, params) -> bool
        fnames = list(self.stencil_object.field_info.keys())
        pnames = list(self.stencil_object.parameter_info.keys())
        memo: Dict[tuple, tuple] = {}
        src = (
            "def _fast(kwargs):\n"
            + f"    if len(kwargs) != {len(fnames) + len(pnames)}:\n        return False\n"
            + "    try:\n"
            + "".join(f"        {n} = kwargs[{n!r}]\n" for n in fnames + pnames)
            + "    except KeyError:\n        return False\n"
            + f"    _gt_e = _memo.get({_ids_src(fnames)})\n"
            + f"    return _gt_e is not None and _gt_e({_tuple_src(fnames)}, {_tuple_src(pnames)})\n"
        )
        ns: Dict[str, Any] = {"_memo": memo}
        exec(compile(src, "<gt4py_amd:FrozenStencil._fast>", "exec"), ns)  # noqa: S102 - generated code
        object.__setattr__(self, "_memo", memo)
        object.__setattr__(self, "_fast", ns["_fast"])
        _frozen_set()[id(self)] = self

    def tune_placement(self, *, candidates: int = 3, reps: int = 10, scope: str = "written",
                       **kwargs) -> Dict[str, Any]:
        """Re-home the fields this stencil writes (``scope="all"``: all its fields), in place, to
        the fastest of ``candidates + 1`` HBM buffer sets for this frozen domain/origin
        (``storage.placement.tune_in_place``): takes the keyword arguments of a call; the tensors
        stay the same objects. Returns the report (every set's kernel time, set 0 = the current
        allocation)."""
        from gt4py_amd.storage.placement import tune_in_place

        so = self.stencil_object
        fields = {n: kwargs[n] for n in so.field_info}
        params = {n: kwargs[n] for n in so.parameter_info if n in kwargs}
        return tune_in_place(so, fields, origin=self.origin, domain=self.domain, params=params,
                             candidates=candidates, reps=reps, scope=scope)

    def __call__(self, **kwargs) -> None:
        if self._fast(kwargs):  # exactly the field and parameter arguments, a prepared launch
            return
        assert "origin" not in kwargs and "domain" not in kwargs
        exec_info = kwargs.get("exec_info")
        if exec_info is not None:
            exec_info["call_run_start_time"] = time.perf_counter()
        field_args = {name: kwargs[name] for name in self.stencil_object.field_info.keys()}
        parameter_args = {name: kwargs[name] for name in self.stencil_object.parameter_info.keys()}
        self.stencil_object.run(
            _domain_=self.domain, _origin_=self.origin, exec_info=exec_info, **field_args, **parameter_args
        )
        if exec_info is not None:
            exec_info["call_run_end_time"] = time.perf_counter()
        else:
            self._remember(field_args, parameter_args)

    def _remember(self, field_args, parameter_args) -> None:
        bind = getattr(type(self.stencil_object)._gt_run_impl_, "bind", None)
        if bind is None or any(a is None for a in field_args.values()):
            return
        tensors = _fast_tensors(field_args, field_args)
        if tensors is None:
            return
        launch = bind(self.domain, self.origin, field_args, tuple(parameter_args), tensors)
        if launch is None:
            return
        if len(self._memo) >= _FAST_MEMO_MAX:
            self._memo.clear()
        self._memo[tuple(id(a) for a in tensors)] = launch


_UNSET = object()


def _frozen_class(fnames, pnames) -> type:
    """A ``FrozenStencil`` subclass whose ``__call__`` takes the stencil's arguments as named
    keywords, so a prepared call needs no keyword dict: the fast path of ``FrozenStencil``
    generated for one argument list (any other call goes to ``FrozenStencil.__call__``)."""
    names = fnames + pnames
    params = ", ".join(f"{n}=_UNSET" for n in names)
    src = (
        f"def __call__(self, *, {params}{', ' if names else ''}exec_info=None, **_gt_rest):\n"
        f"    if exec_info is None and not _gt_rest:\n"
        f"        _gt_e = self._memo.get({_ids_src(fnames)})\n"
        f"        if _gt_e is not None and _gt_e({_tuple_src(fnames)}, {_tuple_src(pnames)}):\n"
        f"            return\n"
        f"    _gt_kw = {{k: v for k, v in (" + "".join(f"({n!r}, {n}), " for n in names) + ") if v is not _UNSET}\n"
        f"    if exec_info is not None:\n"
        f"        _gt_kw['exec_info'] = exec_info\n"
        f"    _gt_kw.update(_gt_rest)\n"
        f"    return _FrozenStencil.__call__(self, **_gt_kw)\n"
    )
    ns: Dict[str, Any] = {"_UNSET": _UNSET, "_FrozenStencil": FrozenStencil}
    exec(compile(src, "<gt4py_amd:FrozenStencil.__call__>", "exec"), ns)  # noqa: S102 - generated code
    return type("FrozenStencil", (FrozenStencil,), {"__call__": ns["__call__"], "__module__": __name__})


class StencilObject(abc.ABC):
    """Generic singleton implementation of a stencil callable (see module docstring)."""

    _gt_id_: str
    definition_func: Callable[..., Any]
    _domain_origin_cache: ClassVar[Dict[int, Tuple[Tuple[int, ...], Dict[str, Tuple[int, ...]]]]]

    # filled in by the backend's class factory
    _gt_backend_: ClassVar[str]
    _gt_source_: ClassVar[str]
    _gt_domain_info_: ClassVar[DomainInfo]
    _gt_field_info_: ClassVar[Dict[str, FieldInfo]]
    _gt_parameter_info_: ClassVar[Dict[str, ParameterInfo]]
    _gt_constants_: ClassVar[Dict[str, Any]]
    _gt_options_: ClassVar[Dict[str, Any]]

    def __new__(cls, *args, **kwargs):
        if cls.__dict__.get("_instance") is None:
            inst = object.__new__(cls)
            type.__setattr__(cls, "_instance", inst)
            type.__setattr__(cls, "_domain_origin_cache", {})
        return cls.__dict__["_instance"]

    def __setattr__(self, key, value) -> None:
        raise AttributeError("Attempting a modification of an attribute in a frozen class")

    def __delattr__(self, item) -> None:
        raise AttributeError("Attempting a deletion of an attribute in a frozen class")

    def __eq__(self, other) -> bool:
        return type(self) is type(other)

    def __hash__(self) -> int:
        return int.from_bytes(type(self)._gt_id_.encode()[:16], byteorder="little")

    def __str__(self) -> str:
        return (
            f"<StencilObject: {self.options['module']}.{self.options['name']}> [backend=\"{self.backend}\"]\n"
            f"    - I/O fields: {self.field_info}\n    - Parameters: {self.parameter_info}\n"
            f"    - Constants: {self.constants}\n    - Version: {self._gt_id_}\n"
        )

    @property
    def backend(self) -> str:
        return type(self)._gt_backend_

    @property
    def source(self) -> str:
        return type(self)._gt_source_

    @property
    def domain_info(self) -> DomainInfo:
        return type(self)._gt_domain_info_

    @property
    def field_info(self) -> Dict[str, FieldInfo]:
        return type(self)._gt_field_info_

    @property
    def parameter_info(self) -> Dict[str, ParameterInfo]:
        return type(self)._gt_parameter_info_

    @property
    def constants(self) -> Dict[str, Any]:
        return type(self)._gt_constants_

    @property
    def options(self) -> Dict[str, Any]:
        return type(self)._gt_options_

    @abc.abstractmethod
    def run(self, _domain_, _origin_, exec_info, **kwargs) -> None:
        pass

    # ------------------------------------------------------------------ call path
    def _call_impl(self, field_args, parameter_args, domain, origin, validate_args, exec_info):
        if exec_info is not None:
            exec_info["call_start_time"] = time.perf_counter()
        self._call_run(
            field_args=field_args,
            parameter_args=parameter_args,
            domain=domain,
            origin=origin,
            validate_args=validate_args,
            exec_info=exec_info,
        )
        if exec_info is not None:
            exec_info["call_end_time"] = time.perf_counter()
            if exec_info.setdefault("__aggregate_data", False):
                info = exec_info.setdefault(type(self).__name__, {})
                info["call_start_time"] = exec_info["call_start_time"]
                info["call_end_time"] = exec_info["call_end_time"]
                info["call_time"] = info["call_end_time"] - info["call_start_time"]
                info["total_call_time"] = info.get("total_call_time", 0.0) + info["call_time"]
                info["ncalls"] = info.get("ncalls", 0) + 1
                info["run_time"] = exec_info["run_end_time"] - exec_info["run_start_time"]
                info["total_run_time"] = info.get("total_run_time", 0.0) + info["run_time"]
                if "run_cpp_start_time" in exec_info:
                    info["run_cpp_time"] = exec_info["run_cpp_end_time"] - exec_info["run_cpp_start_time"]
                    info["total_run_cpp_time"] = info.get("total_run_cpp_time", 0.0) + info["run_cpp_time"]

    @staticmethod
    def _make_origin_dict(origin) -> Dict[str, Tuple[int, ...]]:
        try:
            if isinstance(origin, dict):
                return {str(k): tuple(v) for k, v in origin.items()}
            if origin is None:
                return {}
            if isinstance(origin, collections.abc.Iterable):
                return {"_all_": tuple(int(x) for x in origin)}
            if isinstance(origin, int):
                return {"_all_": (0, 0, origin)}
        except Exception:
            pass
        raise ValueError("Invalid 'origin' value ({})".format(origin))

    @staticmethod
    def _get_max_domain(array_infos, domain_infos, field_infos, origin, *, squeeze=True):
        domain_ndim = domain_infos.ndim
        max_size = sys.maxsize
        max_domain = [max_size] * domain_ndim
        for name, field_info in field_infos.items():
            if field_info.access != AccessKind.NONE:
                info = array_infos.get(name, None)
                assert info is not None, f"Invalid value for '{name}' field."
                mask = field_info.domain_mask
                upper = gd.filter_mask(field_info.boundary.upper_indices, mask)
                forigin = tuple(origin[name])
                fdomain = tuple(info.shape[i] - (forigin[i] + upper[i]) for i in range(field_info.domain_ndim))
                full = gd.interpolate_mask(fdomain, mask, max_size)
                max_domain = [min(a, b) for a, b in zip(max_domain, full)]
        if squeeze:
            return tuple(i if i != max_size else 1 for i in max_domain)
        return tuple(max_domain)

    def _validate_args(self, arg_infos, param_args, domain, origin) -> None:
        from gt4py_amd.backend import from_name

        domain_ndim = self.domain_info.ndim
        if len(domain) != domain_ndim:
            raise ValueError(f"Invalid 'domain' value '{domain}'")
        try:
            domain = tuple(int(d) for d in domain)
        except Exception as ex:
            raise ValueError("Invalid 'domain' value ({})".format(domain)) from ex
        if not _nt_gt(domain, (0,) * domain_ndim):
            raise ValueError(f"Compute domain contains zero sizes '{domain}')")
        max_domain = self._get_max_domain(arg_infos, self.domain_info, self.field_info, origin, squeeze=False)
        if not _nt_le(domain, max_domain):
            offending = []
            for name, info in self.field_info.items():
                used = self._get_max_domain(arg_infos, self.domain_info, {name: info}, origin, squeeze=False)
                if _nt_lt(used, domain):
                    offending.append((name, used))
            raise ValueError(
                f"Compute domain too large for stencil {self.options['name']}: \n"
                f"  Stencil domain is {domain} but field indexation leads to read outside of bounds.\n"
                f"  Check region/horizontal offsets or interval/vertical offsets, or stencil domain.\n"
                f"  Offending fields (name, size with offset removed): {offending}"
            )
        if domain[2] < self.domain_info.min_sequential_axis_size:
            raise ValueError(
                f"Compute domain too small. Sequential axis is {domain[2]}, but must be at least "
                f"{self.domain_info.min_sequential_axis_size}."
            )
        backend_cls = from_name(self.backend)
        for name, field_info in self.field_info.items():
            if field_info.access == AccessKind.NONE:
                continue
            if name not in arg_infos or arg_infos[name] is None:
                raise ValueError(f"Missing value for '{name}' field.")
            arg_info = arg_infos[name]
            dims = tuple(list(field_info.axes) + [str(d) for d in range(len(field_info.data_dims))])
            if not backend_cls.storage_info["is_optimal_layout"](arg_info.array, dims):
                warnings.warn(
                    f"The layout of the field '{name}' is not recommended for this backend."
                    f"This may lead to performance degradation. Please consider using the"
                    f"provided allocators in `gt4py_amd.storage`.",
                    stacklevel=2,
                )
            adtype = _array_dtype(arg_info.array)
            if adtype != field_info.dtype:
                raise TypeError(f"The dtype of field '{name}' is '{adtype}' instead of '{field_info.dtype}'")
            mask = field_info.domain_mask
            fndim = field_info.domain_ndim
            forigin = gd.filter_mask(origin[name], mask[:domain_ndim]) if len(origin[name]) == 3 else tuple(
                origin[name][:fndim]
            )
            if len(arg_info.shape) != fndim + len(field_info.data_dims):
                raise ValueError(
                    f"Storage for '{name}' has {len(arg_info.shape)} dimensions but the API signature "
                    f"expects {fndim + len(field_info.data_dims)} ('{field_info.axes}[{field_info.data_dims}]')"
                )
            if arg_info.dimensions is not None and (
                *field_info.axes,
                *(str(d) for d in range(len(field_info.data_dims))),
            ) != tuple(arg_info.dimensions):
                raise ValueError(
                    f"Storage for '{name}' has dimensions '{arg_info.dimensions}' but the API signature "
                    f"expects '[{', '.join(field_info.axes)}]'"
                    + (f" and {len(field_info.data_dims)}" if field_info.data_dims else "")
                )
            if tuple(arg_info.shape[fndim:]) != tuple(field_info.data_dims):
                raise ValueError(
                    f"Field '{name}' expects data dimensions {field_info.data_dims} but got "
                    f"{tuple(arg_info.shape[fndim:])}"
                )
            lower = gd.filter_mask(field_info.boundary.lower_indices, mask)
            min_origin = gd.interpolate_mask(lower, mask, 0)
            forigin_full = gd.interpolate_mask(forigin, mask, 0)
            if _nt_lt(forigin_full, min_origin):
                raise ValueError(
                    f"Origin for field {name} too small. Must be at least {min_origin}, is {forigin_full}"
                )
            spatial = gd.filter_mask(domain, mask)
            upper = gd.filter_mask(field_info.boundary.upper_indices, mask)
            min_shape = tuple(lb + d + ub for lb, d, ub in zip(lower, spatial, upper))
            if min_shape > tuple(arg_info.shape):
                raise ValueError(
                    f"Shape of field {name} is {tuple(arg_info.shape)} but must be at least {min_shape} "
                    f"for given domain and origin."
                )
        for name, parameter_info in self.parameter_info.items():
            if parameter_info.access != AccessKind.NONE:
                if name not in param_args:
                    raise ValueError(f"Missing value for '{name}' parameter.")
                parameter = param_args[name]
                if np.dtype(type(parameter)) != parameter_info.dtype:
                    raise TypeError(
                        f"The type of parameter '{name}' is '{type(parameter)}' instead of '{parameter_info.dtype}'"
                    )

    @staticmethod
    def _normalize_origins(array_infos, field_infos, origin) -> Dict[str, Tuple[int, ...]]:
        origin = StencilObject._make_origin_dict(origin)
        all_origin = origin.get("_all_", None)
        for name, field_info in field_infos.items():
            assert name in array_infos, f"Missing value for '{name}' field."
            field_origin = origin.get(name, None)
            if field_origin is not None:
                if len(field_origin) != field_info.ndim:
                    assert len(field_origin) == field_info.domain_ndim, (
                        f"Invalid origin specification ({field_origin}) for '{name}' field."
                    )
                    origin[name] = (*field_origin, *((0,) * len(field_info.data_dims)))
            elif all_origin is not None:
                origin[name] = (
                    *gd.filter_mask(all_origin, field_info.domain_mask),
                    *((0,) * len(field_info.data_dims)),
                )
            elif (info_origin := getattr(array_infos.get(name), "origin", None)) is not None:
                origin[name] = tuple(info_origin)
            else:
                origin[name] = (0,) * field_info.ndim
        return origin

    def call_rows(self, j_split: int, j_skip: int, *, domain, origin, validate_args=True, exec_info=None, **kwargs):
        """Run over the rows ``[0, j_split)`` and ``[j_split + j_skip, nj)`` of ``domain`` only (a
        gt4py_amd extension, no reference counterpart): the two boundary strips of a J-strip rank
        after its halo exchange (``distributed/halo.py``). gt:mi355x computes both in one launch
        per kernel when it can (``gtmi_stencil_run_jsplit``, include/gtmi.h); other backends make
        two calls. Arguments as ``__call__``; ``domain`` is the full (ni, nj, nk) region."""
        unknown = sorted(set(kwargs) - set(self.field_info) - set(self.parameter_info))
        if unknown:
            raise TypeError(f"call_rows() got unexpected keyword argument(s) {unknown}")
        field_args = {n: kwargs.get(n) for n in self.field_info}
        parameter_args = {n: kwargs.get(n) for n in self.parameter_info}
        self._call_run(field_args, parameter_args, domain, origin, validate_args=validate_args, exec_info=exec_info,
                       rows=(int(j_split), int(j_skip)))

    def _call_run(self, field_args, parameter_args, domain, origin, *, validate_args=True, exec_info=None, rows=None):
        if exec_info is not None:
            exec_info["call_run_start_time"] = time.perf_counter()
        from gt4py_amd.backend import from_name

        user_domain, user_origin = domain, origin
        device = from_name(self.backend).storage_info["device"]
        array_infos = _extract_array_infos(field_args, device)
        cache_key = _compute_domain_origin_cache_key(array_infos, parameter_args, domain, origin)
        cache = type(self)._domain_origin_cache
        if cache_key not in cache:
            origin = self._normalize_origins(array_infos, self.field_info, origin)
            if domain is None:
                domain = self._get_max_domain(array_infos, self.domain_info, self.field_info, origin)
            if validate_args:
                self._validate_args(array_infos, parameter_args, domain, origin)
            cache[cache_key] = (domain, origin)
        else:
            domain, origin = cache[cache_key]
        arrays = {name: (info.array if info is not None else None) for name, info in array_infos.items()}
        if rows is None:
            self.run(_domain_=domain, _origin_=origin, exec_info=exec_info, **arrays, **parameter_args)
            if exec_info is None:
                self._remember_call(field_args, parameter_args, user_domain, user_origin, domain, origin, arrays)
        else:
            self._run_rows(domain, origin, exec_info, arrays, parameter_args, *rows)
        if exec_info is not None:
            exec_info["call_run_end_time"] = time.perf_counter()

    def _remember_call(self, field_args, parameter_args, user_domain, user_origin, domain, origin, arrays) -> None:
        """Make the fast-path entry of this call signature (see ``_fast_tensors``)."""
        cls = type(self)
        memo = cls.__dict__.get("_gt_fast_memo_")
        bind = getattr(cls._gt_run_impl_, "bind", None)
        if memo is None or bind is None or any(a is None for a in field_args.values()):
            return
        if not (_plain_value(user_domain) and _plain_value(user_origin)):
            return
        tensors = _fast_tensors(field_args, arrays)
        if tensors is None:
            return
        launch = bind(domain, origin, arrays, tuple(parameter_args), tensors)
        if launch is None:
            return
        import copy

        if len(memo) >= _FAST_MEMO_MAX:
            memo.clear()
        # a few (domain, origin) signatures per argument tuple, most recent first: callers that
        # alternate domains/origins on the same arrays (row bands, boundary regions) keep hitting
        key = tuple(id(a) for a in tensors)
        entries = [e for e in memo.get(key, ()) if not (e[0] == user_domain and e[1] == user_origin)]
        entries.insert(0, (copy.deepcopy(user_domain), copy.deepcopy(user_origin), launch))
        memo[key] = entries[:_FAST_SIGS_PER_ARGS]

    def _run_rows(self, domain, origin, exec_info, arrays, parameter_args, j_split, j_skip):
        ni, nj, nk = domain
        if j_split < 0 or j_skip < 0 or j_split + j_skip > nj:
            raise ValueError(f"row split {j_split} + {j_skip} does not fit {nj} rows")
        impl = type(self)._gt_run_impl_
        if getattr(impl, "supports_rows", False):
            if exec_info is not None:
                exec_info["domain"], exec_info["origin"] = domain, origin
                exec_info["run_start_time"] = time.perf_counter()
            impl(domain, origin, exec_info, {**arrays, **parameter_args}, rows=(j_split, j_skip))
            if exec_info is not None:
                exec_info["run_end_time"] = time.perf_counter()
            return
        if j_split > 0:
            self.run(_domain_=(ni, j_split, nk), _origin_=origin, exec_info=exec_info, **arrays, **parameter_args)
        rows_b = nj - j_split - j_skip
        if rows_b > 0:
            shifted = {}
            for name, org in origin.items():
                axes = self.field_info[name].axes if name in self.field_info and self.field_info[name] else ()
                if "J" in axes:
                    q = list(axes).index("J")
                    org = tuple(o + (j_split + j_skip if d == q else 0) for d, o in enumerate(org))
                shifted[name] = org
            self.run(_domain_=(ni, rows_b, nk), _origin_=shifted, exec_info=exec_info, **arrays, **parameter_args)

    def freeze(self, *, origin: Dict[str, Tuple[int, ...]], domain: Tuple[int, ...]) -> FrozenStencil:
        cls = type(self).__dict__.get("_gt_frozen_cls_")
        if cls is None:
            cls = _frozen_class(list(self.field_info), list(self.parameter_info))
            type.__setattr__(type(self), "_gt_frozen_cls_", cls)
        return cls(self, origin, domain)

    def tune_placement(self, *args, candidates: int = 3, reps: int = 10, origin=None, domain=None,
                       scope: str = "written", **kwargs) -> Dict[str, Any]:
        """Opt-in HBM placement for the drop-in path (DESIGN.md §5 "HBM placement"): called with
        the arguments of an ordinary call, it re-homes the fields the stencil writes (``scope=
        "all"``: every field it accesses, for column stencils whose read streams decide too) IN
        PLACE to the fastest of ``candidates + 1`` buffer sets (``storage.placement.tune_in_place``) --
        the caller's tensors stay the same objects with the same contents, on other pages. Once,
        after allocating the fields; returns the report (every set's kernel time in ms, set 0 =
        the current allocation)."""
        import inspect

        from gt4py_amd.storage.placement import tune_in_place

        bound = inspect.signature(self.definition_func).bind(*args, **kwargs)
        bound.apply_defaults()
        fields = {n: v for n, v in bound.arguments.items() if n in self.field_info}
        params = {n: v for n, v in bound.arguments.items() if n in self.parameter_info}
        return tune_in_place(self, fields, origin=origin, domain=domain, params=params, candidates=candidates,
                             reps=reps, scope=scope)

    def clean_call_args_cache(self) -> None:
        type(self)._domain_origin_cache.clear()
        memo = type(self).__dict__.get("_gt_fast_memo_")
        if memo is not None:
            memo.clear()

    def __deepcopy__(self, memodict=None):
        return self


def _array_dtype(array) -> np.dtype:
    dt = getattr(array, "dtype", None)
    if isinstance(dt, np.dtype):
        return dt
    try:
        import torch

        if isinstance(dt, torch.dtype):
            return np.dtype(str(dt).replace("torch.", "").replace("bool", "bool_"))
    except ImportError:  # pragma: no cover
        pass
    return np.dtype(dt)


def make_stencil_class(
    *,
    class_name: str,
    backend_name: str,
    stencil_id: str,
    definition_func,
    source: str,
    domain_info: DomainInfo,
    field_info: Dict[str, FieldInfo],
    parameter_info: Dict[str, ParameterInfo],
    constants: Dict[str, Any],
    options: Dict[str, Any],
    run_impl: Callable,
    module: str,
) -> type:
    """Create the per-stencil ``StencilObject`` subclass.

    ``__call__`` gets the definition's own signature (as the reference template does,
    ``stencil_module.py.in:91-93``) plus ``domain=None, origin=None, validate_args=True,
    exec_info=None``.
    """
    import inspect

    sig = inspect.signature(definition_func)
    field_names = [n for n in sig.parameters if n in field_info]
    param_names = [n for n in sig.parameters if n in parameter_info]
    parts = []
    seen_kwonly = False
    ns: Dict[str, Any] = {}
    for p in sig.parameters.values():
        if p.kind == p.KEYWORD_ONLY and not seen_kwonly:
            parts.append("*")
            seen_kwonly = True
        if p.default is inspect.Parameter.empty:
            parts.append(p.name)
        else:  # the definition's default value (module_generator.py:258-284)
            ns[f"_default_{p.name}"] = p.default
            parts.append(f"{p.name}=_default_{p.name}")
    if not seen_kwonly:
        parts.append("*")
    parts += ["domain=None", "origin=None", "validate_args=True", "exec_info=None"]
    fdict = ", ".join(f"{n}={n}" for n in field_names)
    pdict = ", ".join(f"{n}={n}" for n in param_names)
    # fast path (see _fast_tensors): id tuple -> [(domain, origin, prepared launch(fields, params) -> bool)]
    memo: Dict[tuple, tuple] = {}
    ns["_memo"] = memo
    src = (
        f"def __call__(self, {', '.join(parts)}):\n"
        f"    if exec_info is None:\n"
        f"        for _gt_e in _memo.get({_ids_src(field_names)}, ()):\n"
        f"            if _gt_e[0] == domain and _gt_e[1] == origin:\n"
        f"                if _gt_e[2]({_tuple_src(field_names)}, {_tuple_src(param_names)}):\n"
        f"                    return\n"
        f"                break\n"
        f"    self._call_impl(dict({fdict}), dict({pdict}), domain, origin, validate_args, exec_info)\n"
    )
    exec(compile(src, f"<gt4py_amd:{class_name}.__call__>", "exec"), ns)  # noqa: S102 - generated code

    def run(self, _domain_, _origin_, exec_info, **kwargs):
        if exec_info is not None:
            exec_info["domain"] = _domain_
            exec_info["origin"] = _origin_
            exec_info["run_start_time"] = time.perf_counter()
        run_impl(_domain_, _origin_, exec_info, kwargs)
        if exec_info is not None:
            exec_info["run_end_time"] = time.perf_counter()

    attrs = {
        "__call__": ns["__call__"],
        "run": run,
        "_gt_backend_": backend_name,
        "_gt_source_": source,
        "_gt_domain_info_": domain_info,
        "_gt_field_info_": field_info,
        "_gt_parameter_info_": parameter_info,
        "_gt_constants_": constants,
        "_gt_options_": options,
        "_gt_id_": stencil_id,
        "_gt_run_impl_": staticmethod(run_impl),  # backend hook (gt:mi355x: .compiled.lib_path)
        "definition_func": staticmethod(definition_func),
        "__module__": module,
        "__doc__": inspect.getdoc(definition_func) or "",
        "_instance": None,
        "_gt_fast_memo_": memo,
    }
    cls = type(class_name, (StencilObject,), attrs)
    _memo_classes().add(cls)
    return cls
