"""HIP C++ code generation for gt:mi355x (gfx950).

Emits, per stencil, one ``.hip`` translation unit holding the kernels of the plan
(``codegen/plan.py``) instantiated from two hand-written skeletons, plus the C-ABI entry
points declared in ``include/gtmi.h``. Replaces the reference's GridTools C++ generation
(``gtc/gtcpp/gtcpp_codegen.py:291-319``) and pybind11 bindings (``backend/gtc_common.py:65-103``).

K1 -- J-streaming plane kernel (PARALLEL sections with IJ offsets)
    block = 256 threads = 4 independent wavefronts; wave w of block b owns I strip
    ``4*s + w`` (64 lanes, ``64 - H_lo - H_hi`` output columns, H = I halo), a chunk of
    ``JC`` rows and one K level. Per row step every value of the section is produced at
    row ``t + lead`` into a register ring (depth = J offsets read); I offsets are wave64
    shuffles hoisted out of divergent control flow. Loads are I-contiguous (coalesced),
    one row ahead (prefetch), rows/levels are wave-uniform (scalar address math).
    Block -> work mapping is XCD-aware: consecutive work items land on the same XCD.

K2 -- column kernel (K sweeps and pointwise PARALLEL loops)
    one thread per (i, j) column, 64 x 4 threads per block (I-contiguous waves), walks the
    levels of each vertical loop in loop order; every (name, di, dj) accessed in a loop
    has a register K-window covering its K offsets, so each level loads only the window
    front and writes go straight through to memory.

Numerics: expressions are emitted with the exact association and cast points of the typed
IR (``passes.upcast``) and compiled with ``-ffp-contract=off`` (no FMA contraction), IEEE
division and correctly rounded sqrt, so f64 results are bit-identical to the reference
numpy backend for + - * / comparisons and selects.
"""

from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional, Set, Tuple

from gt4py_amd import ir
from gt4py_amd.codegen.plan import ColumnKernel, KernelPlan, PlaneKernel, UnsupportedStencil
from gt4py_amd.ir import DataType
from gt4py_amd.passes import ZERO_EXTENT, StencilAnalysis, iter_accesses
from gt4py_amd.codegen.column import ColumnGen
from gt4py_amd.codegen.common import (  # noqa: F401  (re-exported)
    COLUMN_BLOCK, PLANE_BLOCK_WAVES, PLANE_MIN_JCHUNK, PLANE_TARGET_BLOCKS, WAVE, ExprRenderer, FieldSlot, cname,
    host_fill, interval_bounds, kparam_decl, literal, region_condition,
)
from gt4py_amd.codegen.plane import PlaneGen

# ------------------------------------------------------------------------------------------
# translation unit
# ------------------------------------------------------------------------------------------


def jsplit_native(analysis: StencilAnalysis, plan: KernelPlan) -> bool:
    """``gtmi_stencil_run_jsplit`` runs in one launch per kernel: plane kernels only (their J
    chunks are mapped around the gap), no scratch (a producer's J halo would straddle it), no
    horizontal regions (their conditions are relative to the call's domain)."""
    if plan.scratch or not all(isinstance(k, PlaneKernel) for k in plan.kernels):
        return False
    st = analysis.stencil
    return not any(
        isinstance(n, ir.HorizontalRegion) for vl in st.vertical_loops for sec in vl.sections for n in ir.walk(sec.body)
    )


def generate(
    analysis: StencilAnalysis, plan: KernelPlan, opts: Dict, abi_fields=None, components=None
) -> Tuple[str, Dict]:
    """``abi_fields``: the API field declarations in ABI order (default: the stencil's);
    ``components``: data-dimension components from ``lowering.lower_data_dims``."""
    st = analysis.stencil
    components = components or {}
    abi_fields = list(abi_fields) if abi_fields is not None else st.field_params()
    slots: Dict[str, FieldSlot] = {}
    idx = 0
    host_scalar = ExprRenderer(lambda acc: "0", lambda n: f"hs_{cname(n)}", lambda ax: "0")
    for p in abi_fields:
        slots[p.name] = FieldSlot(p.name, idx, p.dtype, False)
        for vname, comp in components.items():
            if comp.base == p.name:
                slots[vname] = FieldSlot(vname, idx, p.dtype, False, tuple(host_scalar(x) for x in comp.index))
        idx += 1
    for t in plan.scratch:
        slots[t] = FieldSlot(t, idx, st.decl(t).dtype, True)
        idx += 1
    n_fields = idx
    kernels_src = []
    launches = []
    for kid, k in enumerate(plan.kernels):
        if isinstance(k, PlaneKernel):
            ks, hs = PlaneGen(analysis, plan, k, slots, kid, opts).render()
        else:
            ks, hs = ColumnGen(analysis, plan, k, slots, kid, opts).render()
        kernels_src.append(ks)
        launches.append(hs)
    import json

    used_scalars = {
        n.name for vl in st.vertical_loops for sec in vl.sections for n in ir.walk(sec.body) if isinstance(n, ir.ScalarAccess)
    }
    for comp in components.values():
        used_scalars |= {n.name for x in comp.index for n in ir.walk(x) if isinstance(n, ir.ScalarAccess)}
    signature = {
        "abi": 3,
        "fields": [
            {"name": p.name, "dtype": p.dtype.name.lower(), "axes": list(p.axes), "data_dims": list(p.data_dims)}
            for p in abi_fields
        ],
        "scratch": [
            {
                "name": t,
                "dtype": st.decl(t).dtype.name.lower(),
                "extent": [list(e) for e in plan.scratch_extent[t]],
                "axes": list(st.decl(t).axes),
            }
            for t in plan.scratch
        ],
        "scalars": [
            {"name": s.name, "dtype": s.dtype.name.lower(), "used": s.name in used_scalars} for s in st.scalar_params()
        ],
        "kernels": [type(k).__name__ for k in plan.kernels],
    }
    sig_json = json.dumps(signature).replace("\\", "\\\\").replace('"', '\\"')
    roctx_name = "gtmi:" + "".join(c if (c.isalnum() or c in "._-") else "_" for c in st.name)
    n_scalars = len(st.scalar_params())
    host_scalars = [
        f"    {sp.dtype.ctype} hs_{cname(sp.name)}; memcpy(&hs_{cname(sp.name)}, &sc[{i}], sizeof(hs_{cname(sp.name)})); "
        f"(void)hs_{cname(sp.name)};"
        for i, sp in enumerate(st.scalar_params())
    ]
    if jsplit_native(analysis, plan):
        # every kernel is a plane kernel without scratch or regions: one launch per kernel over both row ranges
        jsplit_body = "    return gtmi_run_rows(domain, (int)j_split, (int)j_skip, f, sc, stream);"
    else:
        # two ordinary passes; the second sees every field (and scratch buffer) shifted by the gap
        jsplit_body = f"""    if (j_split > 0) {{
        const int64_t da[3] = {{domain[0], j_split, domain[2]}};
        if (int rc = gtmi_run_rows(da, (int)j_split, 0, f, sc, stream)) return rc;
    }}
    if (rows_b == 0) return 0;
    gtmi_field g[{max(1, n_fields)}];
    for (int q = 0; q < {n_fields}; ++q) {{
        g[q] = f[q];
        if (g[q].strides[1] != 0) g[q].origin[1] += j_split + j_skip;
    }}
    const int64_t db[3] = {{domain[0], rows_b, domain[2]}};
    return gtmi_run_rows(db, (int)rows_b, 0, g, sc, stream);"""
    src = f"""// Generated by gt4py_amd (gt:mi355x). Do not edit.
#include "gtmi_device.h"
#include "gtmi.h"
#include "gtmi_roctx.h"
#include <string.h>
#include <stdio.h>

static thread_local char g_gtmi_err[512];
static void gtmi_set_error(const char* msg) {{ snprintf(g_gtmi_err, sizeof(g_gtmi_err), "%s", msg); }}

{chr(10).join(kernels_src)}

extern "C" const char* gtmi_last_error(void) {{ return g_gtmi_err; }}
extern "C" int gtmi_abi_version(void) {{ return GTMI_ABI_VERSION; }}
extern "C" const char* gtmi_stencil_signature(void) {{ return "{sig_json}"; }}

// Rows [0, jsplit) and [jsplit + jskip, nj) of the domain; an ordinary call has jsplit = nj.
static int gtmi_run_rows(const int64_t* domain, int jsplit, int jskip, const gtmi_field* f, const gtmi_scalar* sc,
                         hipStream_t stream) {{
    (void)sc; (void)f;
    const int ni = (int)domain[0], nj = (int)domain[1], nk = (int)domain[2];
    (void)ni; (void)nj; (void)nk; (void)jsplit; (void)jskip;
    GTMI_RANGE_PUSH("{roctx_name}");  // ROCTX range around the launches (rocprofv3 --marker-trace)
{chr(10).join(host_scalars)}
{chr(10).join("    " + line for h in launches for line in h.splitlines())}
    GTMI_RANGE_POP();
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {{
        snprintf(g_gtmi_err, sizeof(g_gtmi_err), "HIP launch failed: %s", hipGetErrorString(err));
        return (int)err;
    }}
    return 0;
}}

static int gtmi_check_counts(int32_t n_fields, int32_t n_scalars) {{
    g_gtmi_err[0] = 0;
    if (n_fields != {n_fields} || n_scalars != {n_scalars}) {{
        snprintf(g_gtmi_err, sizeof(g_gtmi_err), "expected {n_fields} fields / {n_scalars} scalars, got %d / %d",
                 (int)n_fields, (int)n_scalars);
        return 1;
    }}
    return 0;
}}

extern "C" int gtmi_stencil_run(const int64_t* domain, const gtmi_field* f, int32_t n_fields,
                                const gtmi_scalar* sc, int32_t n_scalars, void* stream_ptr) {{
    if (int rc = gtmi_check_counts(n_fields, n_scalars)) return rc;
    return gtmi_run_rows(domain, (int)domain[1], 0, f, sc, (hipStream_t)stream_ptr);
}}

extern "C" int gtmi_stencil_run_jsplit(const int64_t* domain, int64_t j_split, int64_t j_skip, const gtmi_field* f,
                                       int32_t n_fields, const gtmi_scalar* sc, int32_t n_scalars, void* stream_ptr) {{
    if (int rc = gtmi_check_counts(n_fields, n_scalars)) return rc;
    if (j_split < 0 || j_skip < 0 || j_split + j_skip > domain[1]) {{
        snprintf(g_gtmi_err, sizeof(g_gtmi_err), "bad row split %lld + %lld of %lld rows", (long long)j_split,
                 (long long)j_skip, (long long)domain[1]);
        return 1;
    }}
    hipStream_t stream = (hipStream_t)stream_ptr;
    const int64_t rows_b = domain[1] - j_split - j_skip;
    if (j_split == 0 && rows_b == 0) return 0;
{jsplit_body}
}}
"""
    return src, signature
