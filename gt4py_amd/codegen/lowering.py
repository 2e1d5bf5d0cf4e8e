"""IR lowerings applied before kernel planning (gt:mi355x only).

Data dimensions (``Field[(dtype, (n,))]``, ``GlobalTable``) are lowered to *component fields*:
every distinct data index of a field becomes one virtual 3-D field whose base address is the
field's address plus ``sum(index_d * data_stride_d)``, computed by the host code at launch time.
With the ``(2, 1, 0)`` I-first layout the data dimensions are the outermost ones
(``storage/layout.py``), so each component is itself a dense I-first 3-D array: the plane and
column kernels stream it like any other field.

The indices must be launch-uniform (integer literals and scalar parameters, e.g.
``vec[0, 0, 0][2]`` or ``vec[0, 0, 0][idx]``; reference ``test_code_generation.py:309-361,
463-510, 664-716, 894-917, 1096-1109``). A written data-dimension field must use literal indices
only (or a single index), so that two components never alias.
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Tuple

from gt4py_amd import ir, passes
from gt4py_amd.codegen.plan import UnsupportedStencil
from gt4py_amd.passes import StencilAnalysis


@dataclasses.dataclass
class Component:
    base: str  # API field name
    index: List[ir.Expr]  # launch-uniform index expression per data dimension


def _uniform(e: ir.Expr) -> bool:
    for n in ir.walk(e):
        if isinstance(n, (ir.FieldAccess, ir.AxisIndex)):
            return False
    return True


def _key(index: List[ir.Expr]) -> str:
    return repr([(type(x).__name__, dataclasses.astuple(x) if dataclasses.is_dataclass(x) else x) for x in index])


def lower_data_dims(analysis: StencilAnalysis) -> Tuple[StencilAnalysis, Dict[str, Component]]:
    st = analysis.stencil
    dd_fields = {p.name: p for p in st.field_params() if p.data_dims}
    dd_temps = {t.name: t for t in st.temporaries if t.data_dims}
    if not dd_fields and not dd_temps:
        return analysis, {}
    temp_comps: Dict[Tuple[str, Tuple[int, ...]], str] = {}

    def temp_comp(acc: ir.FieldAccess) -> str:
        if not all(isinstance(x, ir.Literal) for x in acc.data_index):
            raise UnsupportedStencil(f"run-time data index into temporary '{acc.name}'")
        idx = tuple(int(x.value) for x in acc.data_index)
        k = (acc.name, idx)
        if k not in temp_comps:
            temp_comps[k] = f"{acc.name}__t{'_'.join(str(i) for i in idx)}"
        return temp_comps[k]

    comps: Dict[str, Component] = {}
    by_key: Dict[Tuple[str, str], str] = {}
    written: Dict[str, set] = {}

    def comp_name(acc: ir.FieldAccess) -> str:
        if not all(_uniform(x) for x in acc.data_index):
            raise UnsupportedStencil(f"data index of '{acc.name}' varies across grid points")
        k = (acc.name, _key(acc.data_index))
        if k not in by_key:
            vname = f"{acc.name}__c{sum(1 for b in by_key if b[0] == acc.name)}"
            by_key[k] = vname
            comps[vname] = Component(acc.name, list(acc.data_index))
        return by_key[k]

    def fn(e):
        if isinstance(e, ir.FieldAccess) and e.name in dd_fields:
            return ir.FieldAccess(comp_name(e), e.offset, e.dtype, [], e.k_offset)
        if isinstance(e, ir.FieldAccess) and e.name in dd_temps:
            return ir.FieldAccess(temp_comp(e), e.offset, e.dtype, [], e.k_offset)
        return e

    # a written field: its components must be provably distinct (literal indices) or just one
    keys: Dict[str, set] = {}
    runtime: Dict[str, bool] = {}
    for vl in st.vertical_loops:
        for sec in vl.sections:
            for acc, w in passes.iter_accesses(sec.body):
                if isinstance(acc, ir.FieldAccess) and acc.name in dd_fields:
                    keys.setdefault(acc.name, set()).add(_key(acc.data_index))
                    if not all(isinstance(x, ir.Literal) for x in acc.data_index):
                        runtime[acc.name] = True
                    if w:
                        written[acc.name] = set()
    for name in written:
        if runtime.get(name) and len(keys[name]) > 1:
            raise UnsupportedStencil(f"'{name}' is written with run-time data indices that may alias")

    loops = [ir.map_expr(vl, fn) for vl in st.vertical_loops]
    params = []
    virtual_decls = []
    for p in st.params:
        if isinstance(p, ir.FieldDecl) and p.name in dd_fields:
            for vname, c in comps.items():
                if c.base == p.name:
                    virtual_decls.append(ir.FieldDecl(vname, p.dtype, p.axes, (), False))
            continue
        params.append(p)
    params += virtual_decls
    temps = [t for t in st.temporaries if t.name not in dd_temps]
    temps += [ir.FieldDecl(v, dd_temps[n].dtype, dd_temps[n].axes, (), True) for (n, _), v in temp_comps.items()]
    lowered = ir.Stencil(st.name, st.api_signature, params, temps, loops, st.externals, st.docstring)
    extents = passes.compute_extents(lowered)
    out = StencilAnalysis(
        lowered,
        passes.compute_access_kinds(lowered),
        extents,
        passes.compute_k_boundary(lowered),
        analysis.min_k_size,
    )
    return out, comps
