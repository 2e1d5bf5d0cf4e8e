"""Register ``gt:mi355x`` inside the reference ``gt4py.cartesian`` (drop-in adapter).

With ``gt4py`` importable, ``gt4py_amd.gt4py_plugin.register()`` adds a backend class to the
reference registry exactly like the in-tree backends do (``backend/base.py:142-152``
``@register``; ``gtcpp_backend.py:168-183`` is the GPU backend it stands beside):

* ``generate()`` takes the reference's own typed GTIR (``builder.gtir_pipeline.full()``: the
  frontend, dtype resolution and upcasting of the reference), translates it to
  ``gt4py_amd.ir`` (``gtir_to_ir``), plans/generates/compiles the HIP kernels of
  ``gt:mi355x`` and renders the reference's ``stencil_module.py.in`` with a ``run()`` that
  calls the generated library through ``StencilLauncher`` (C ABI of ``include/gtmi.h``);
* ``field_info`` / ``parameter_info`` / ``domain_info`` come from the reference's
  ``make_args_data_from_gtir`` (``module_generator.py:56-106``), i.e. they are the reference's;
* the generated class derives from ``GTMIStencilObject``, a ``StencilObject`` whose
  ``_call_run`` accepts torch ROCm tensors (the reference's ``storage_utils.asarray`` requires
  CuPy for GPU devices, ``storage/cartesian/utils.py:176-215``) and otherwise reuses the
  reference's origin normalisation, max-domain and validation code unchanged.

See INTEGRATION.md for the maintainer-side steps.
"""

from __future__ import annotations

import time
from typing import Any, Dict, List

from gt4py_amd import ir
from gt4py_amd.ir import DataType

_REGISTERED = None


# ------------------------------------------------------------------------------------------
# GTIR -> gt4py_amd IR
# ------------------------------------------------------------------------------------------


def _dt(d) -> DataType:
    return DataType(int(d))


def _bound(b) -> ir.AxisBound:
    lvl = ir.LevelMarker.START if str(b.level.value).lower() == "start" else ir.LevelMarker.END
    if not isinstance(b.offset, int):
        raise NotImplementedError("runtime interval bounds are not supported by gt:mi355x")
    return ir.AxisBound(lvl, int(b.offset))


def _literal(node) -> ir.Literal:
    dt = _dt(node.dtype)
    v = node.value
    sv = str(getattr(v, "value", v)).lower()
    if dt == DataType.BOOL:
        return ir.Literal(sv in ("true", "1"), dt)
    if dt.isinteger():
        return ir.Literal(int(sv) if sv not in ("max", "min") else 0, dt)
    return ir.Literal(float(getattr(v, "value", v)), dt)


def _expr(node) -> ir.Expr:
    from gt4py.cartesian.gtc import gtir

    if isinstance(node, gtir.Literal):
        return _literal(node)
    if isinstance(node, gtir.FieldAccess):
        off = node.offset
        didx = [_expr(x) for x in (node.data_index or [])]
        if isinstance(off, gtir.VariableKOffset):
            return ir.FieldAccess(node.name, (0, 0, 0), _dt(node.dtype), didx, _expr(off.k))
        if isinstance(off, gtir.AbsoluteKIndex):
            koff = ir.BinaryOp("-", ir.NativeCall("int64", [_expr(off.k)]), ir.AxisIndex(2))
            return ir.FieldAccess(node.name, (0, 0, 0), _dt(node.dtype), didx, koff)
        if not hasattr(off, "i"):
            raise NotImplementedError(f"GTIR offset {type(off).__name__}")
        return ir.FieldAccess(node.name, (int(off.i), int(off.j), int(off.k)), _dt(node.dtype), didx)
    if isinstance(node, gtir.ScalarAccess):
        return ir.ScalarAccess(node.name, _dt(node.dtype))
    if isinstance(node, gtir.IteratorAccess):
        return ir.AxisIndex("IJK".index(str(node.name.value).upper()))
    if isinstance(node, gtir.BinaryOp):
        return ir.BinaryOp(str(node.op.value), _expr(node.left), _expr(node.right), _dt(node.dtype))
    if isinstance(node, gtir.UnaryOp):
        return ir.UnaryOp(str(node.op.value), _expr(node.expr), _dt(node.dtype))
    if isinstance(node, gtir.TernaryOp):
        return ir.TernaryOp(_expr(node.cond), _expr(node.true_expr), _expr(node.false_expr), _dt(node.dtype))
    if isinstance(node, gtir.Cast):
        return ir.Cast(_dt(node.dtype), _expr(node.expr))
    if isinstance(node, gtir.NativeFuncCall):
        return ir.NativeCall(str(node.func.value), [_expr(a) for a in node.args], _dt(node.dtype))
    raise NotImplementedError(f"GTIR expression {type(node).__name__}")


def _hinterval(h) -> ir.HorizontalInterval:
    def b(x):
        if x is None:
            return None
        lvl = ir.LevelMarker.START if str(x.level.value).lower() == "start" else ir.LevelMarker.END
        if abs(int(x.offset)) >= 10000:  # the frontend's "unbounded" marker (gtscript_frontend.py:146-150)
            return None
        return ir.AxisBound(lvl, int(x.offset))

    return ir.HorizontalInterval(b(h.start), b(h.end))


def _stmts(body) -> List[ir.Stmt]:
    from gt4py.cartesian.gtc import gtir

    out: List[ir.Stmt] = []
    for s in body:
        if isinstance(s, gtir.ParAssignStmt):
            tgt = _expr(s.left)
            out.append(ir.Assign(tgt, _expr(s.right)))
        elif isinstance(s, (gtir.FieldIfStmt, gtir.ScalarIfStmt)):
            orelse = _stmts(s.false_branch.body) if s.false_branch is not None else []
            out.append(ir.If(_expr(s.cond), _stmts(s.true_branch.body), orelse))
        elif isinstance(s, gtir.While):
            out.append(ir.While(_expr(s.cond), _stmts(s.body)))
        elif isinstance(s, gtir.HorizontalRestriction):
            m = s.mask
            out.append(ir.HorizontalRegion([ir.HorizontalMask(_hinterval(m.i), _hinterval(m.j))], _stmts(s.body)))
        elif isinstance(s, gtir.BlockStmt):
            out.extend(_stmts(s.body))
        else:
            raise NotImplementedError(f"GTIR statement {type(s).__name__}")
    return out


def _ordered(prev: ir.Interval, nxt: ir.Interval, order: ir.LoopOrder) -> bool:
    """Can ``nxt`` follow ``prev`` as another section of the same vertical loop?"""
    a, b = (prev.end, nxt.start) if order != ir.LoopOrder.BACKWARD else (nxt.end, prev.start)
    return a.level == b.level and b.offset >= a.offset


def gtir_to_ir(node) -> ir.Stencil:
    """Translate the reference's typed GTIR stencil (after its pipeline) to gt4py_amd IR."""
    from gt4py.cartesian.gtc import gtir

    params = []
    for d in node.params:
        if isinstance(d, gtir.FieldDecl):
            axes = tuple(a for a, m in zip("IJK", d.dimensions) if m)
            params.append(ir.FieldDecl(d.name, _dt(d.dtype), axes, tuple(d.data_dims)))
        else:
            params.append(ir.ScalarDecl(d.name, _dt(d.dtype)))
    temps: Dict[str, ir.FieldDecl] = {}
    loops: List[ir.VerticalLoop] = []
    for vl in node.vertical_loops:
        for t in vl.temporaries:
            temps[t.name] = ir.FieldDecl(t.name, _dt(t.dtype), ("I", "J", "K"), tuple(t.data_dims), True)
        order = ir.LoopOrder[str(vl.loop_order.name)]
        sec = ir.Section(ir.Interval(_bound(vl.interval.start), _bound(vl.interval.end)), _stmts(vl.body))
        if loops and loops[-1].loop_order == order and _ordered(loops[-1].sections[-1].interval, sec.interval, order):
            loops[-1].sections.append(sec)
        else:
            loops.append(ir.VerticalLoop(order, [sec]))
    st = ir.Stencil(
        name=node.name,
        api_signature=[a.name for a in node.api_signature],
        params=params,
        temporaries=list(temps.values()),
        vertical_loops=loops,
        externals={},
        docstring=node.docstring or "",
    )
    st.temp_declared_dtype = {n: t.dtype for n, t in temps.items()}
    return st


# ------------------------------------------------------------------------------------------
# runtime pieces referenced by the generated modules
# ------------------------------------------------------------------------------------------

_LAUNCHERS: Dict[str, Any] = {}


def launcher_for(lib_path: str, name: str):
    from gt4py_amd.runtime.launcher import StencilLauncher

    if lib_path not in _LAUNCHERS:
        _LAUNCHERS[lib_path] = StencilLauncher(lib_path, name)
    return _LAUNCHERS[lib_path]


class _DeviceArrayView:
    """numpy-like metadata of a device tensor, for the reference's validation code."""

    def __init__(self, tensor):
        from gt4py_amd.storage import numpy_dtype_of

        self.tensor = tensor
        self.shape = tuple(tensor.shape)
        self.ndim = tensor.dim()
        self.dtype = numpy_dtype_of(tensor)
        self.strides = tuple(s * tensor.element_size() for s in tensor.stride())


def _stencil_object_base():
    from gt4py.cartesian import stencil_object as so
    from gt4py.storage.cartesian import utils as storage_utils

    from gt4py_amd.runtime.launcher import device_tensor

    class GTMIStencilObject(so.StencilObject):
        """Reference StencilObject with a CuPy-free array extraction for ROCm tensors."""

        def _call_run(self, field_args, parameter_args, domain, origin, *, validate_args=True, exec_info=None):
            if exec_info is not None:
                exec_info["call_run_start_time"] = time.perf_counter()
            infos = {}
            for name, arg in field_args.items():
                if arg is None:
                    infos[name] = None
                    continue
                t = device_tensor(arg)
                infos[name] = so.ArgsInfo(
                    device="gpu",
                    array=_DeviceArrayView(t),
                    original_object=arg,
                    origin=storage_utils.get_origin(arg),
                    dimensions=storage_utils.get_dims(arg),
                )
            key = so._compute_domain_origin_cache_key(infos, parameter_args, domain, origin)
            cache = type(self)._domain_origin_cache
            if key not in cache:
                origin = self._normalize_origins(infos, self.field_info, origin)
                if domain is None:
                    domain = self._get_max_domain(infos, self.domain_info, self.field_info, origin)
                if validate_args:
                    self._validate_args(infos, parameter_args, domain, origin)
                cache[key] = (domain, origin)
            else:
                domain, origin = cache[key]
            arrays = {n: (None if i is None else i.array.tensor) for n, i in infos.items()}
            self.run(_domain_=domain, _origin_=origin, exec_info=exec_info, **arrays, **parameter_args)
            if exec_info is not None:
                exec_info["call_run_end_time"] = time.perf_counter()

    return GTMIStencilObject


GTMIStencilObject = None


def register():
    """Register ``gt:mi355x`` in ``gt4py.cartesian.backend.REGISTRY`` (idempotent)."""
    global _REGISTERED, GTMIStencilObject
    if _REGISTERED is not None:
        return _REGISTERED
    from gt4py.cartesian import backend as gt_backend
    from gt4py.cartesian.backend.module_generator import BaseModuleGenerator
    from gt4py.storage.cartesian import layout as gt_layout

    from gt4py_amd import passes
    from gt4py_amd.backend.mi355x_backend import Mi355xBackend, generate_source
    from gt4py_amd.runtime import jit

    GTMIStencilObject = _stencil_object_base()
    globals()["GTMIStencilObject"] = GTMIStencilObject

    class GTMIModuleGenerator(BaseModuleGenerator):
        def generate_imports(self) -> str:
            return "from gt4py_amd.gt4py_plugin import GTMIStencilObject, launcher_for"

        def generate_base_class_name(self) -> str:
            return "GTMIStencilObject"

        def generate_module_members(self) -> str:
            lib = self.builder.backend_data["gtmi:lib"]
            return f"_gtmi_launcher = launcher_for({lib!r}, {self.builder.gtir.name!r})"

        def generate_implementation(self) -> str:
            fields = ", ".join(f"{n}={n}" for n in self.args_data.field_names)
            params = ", ".join(f"{n}={n}" for n in self.args_data.parameter_names)
            sync = bool(self.builder.options.backend_opts.get("device_sync", True))
            return (
                f"_gtmi_launcher(_domain_, _origin_, dict({fields}), dict({params}), "
                f"device_sync={sync}, exec_info=exec_info)"
            )

    layout_map = gt_layout.layout_maker_factory((2, 1, 0))

    class GT4PyMi355xBackend(gt_backend.BaseBackend):
        """gt:mi355x as a reference gt4py backend (HIP kernels for MI355X via the gtmi C ABI)."""

        name = "gt:mi355x"
        options = dict(Mi355xBackend.options)
        storage_info = {
            "alignment": 32,
            "device": "gpu",
            "layout_map": layout_map,
            "is_optimal_layout": gt_layout.layout_checker_factory(layout_map),
        }
        languages = {"computation": "hip", "bindings": ["python"]}
        MODULE_GENERATOR_CLASS = GTMIModuleGenerator

        def compile_library(self) -> str:
            opts = dict(self.builder.options.backend_opts)
            stencil_ir = gtir_to_ir(self.builder.gtir_pipeline.full())
            analysis = passes.run_pipeline(stencil_ir)
            _, source, _ = generate_source(analysis, opts)
            return jit.compile_source(source, verbose=bool(opts.get("verbose")))

        def generate(self):
            self.check_options(self.builder.options)
            t0 = time.perf_counter()
            lib = self.compile_library()
            if self.builder.options.build_info is not None:
                self.builder.options.build_info["build_time"] = time.perf_counter() - t0
            self.builder.with_backend_data({"gtmi:lib": lib})
            return self.make_module()

    _REGISTERED = gt_backend.register(GT4PyMi355xBackend)
    return _REGISTERED
