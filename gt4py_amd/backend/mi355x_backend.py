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

import time

from gt4py_amd.backend.base import BaseBackend, register
from gt4py_amd.codegen import hip as hipgen
from gt4py_amd.codegen.lowering import fuse_parallel_loops, fuse_sequential_loops, lower_data_dims, split_phases
from gt4py_amd.codegen.plan import UnsupportedStencil, make_plan
from gt4py_amd.runtime import jit
from gt4py_amd.runtime.launcher import StencilLauncher
from gt4py_amd.storage.layout import layout_checker_factory, layout_maker_factory

_layout = layout_maker_factory((2, 1, 0))


def generate_source(analysis, opts):
    """(plan, HIP source, signature) of a typed stencil analysis: data-dimension lowering,
    kernel planning, code generation."""
    lowered, components = lower_data_dims(analysis)
    abi = analysis.stencil.field_params()
    fused = fuse_parallel_loops(lowered) if int(opts.get("fuse", 1)) else lowered
    if fused is not lowered:
        try:
            plan = make_plan(fused, pointwise_plane=bool(opts.get("pointwise_plane", 1)))
            source, signature = hipgen.generate(fused, plan, opts, abi_fields=abi, components=components)
            return plan, source, signature
        except UnsupportedStencil:
            pass  # the computations as written
    try:
        plan = make_plan(lowered, pointwise_plane=bool(opts.get("pointwise_plane", 1)))
        source, signature = hipgen.generate(lowered, plan, opts, abi_fields=abi, components=components)
    except UnsupportedStencil as direct_failure:
        # tile kernels: sequential computations fused into one K sweep where legal, and a sweep
        # that reads its own products across columns runs on overlapping 2-D tiles with an LDS
        # plane per level (the reference's IJ caches, oir_optimizations/caches.py:44-90)
        if int(opts.get("tile", 1)):
            try:
                seq = fuse_sequential_loops(lowered)
                plan = make_plan(seq, pointwise_plane=bool(opts.get("pointwise_plane", 1)), tile=True)
                if any(getattr(k, "tile", False) for k in plan.kernels):
                    source, signature = hipgen.generate(seq, plan, opts, abi_fields=abi, components=components)
                    return plan, source, signature
            except UnsupportedStencil:
                pass
        # staged fallback: split computations into phases, column kernels + scratch temporaries
        try:
            staged = split_phases(lowered)
            plan = make_plan(staged, column_only=True)
            source, signature = hipgen.generate(staged, plan, opts, abi_fields=abi, components=components)
        except UnsupportedStencil as staged_failure:
            raise UnsupportedStencil(f"{direct_failure}; staged lowering: {staged_failure}") from None
    return plan, source, signature


class _Compiled:
    """The generated source, its library and the launcher that calls it."""

    def __init__(self, analysis, plan, source, signature, lib_path, options):
        self.analysis = analysis
        self.plan = plan
        self.source = source
        self.signature = signature
        self.lib_path = lib_path
        self.options = options
        self.launcher = StencilLauncher(lib_path, analysis.stencil.name)

    def __call__(self, domain, origin, exec_info, kwargs, rows=None):
        self.launcher(
            domain,
            origin,
            kwargs,
            kwargs,
            device_sync=bool(self.options.get("device_sync", True)),
            exec_info=exec_info,
            rows=rows,
        )

    def bind(self, domain, origin, arrays, param_names, tensors):
        """Prepared launch for the StencilObject fast path (``StencilLauncher.bind``)."""
        return self.launcher.bind(domain, origin, arrays, param_names, tensors,
                                  device_sync=bool(self.options.get("device_sync", True)))


@register
class Mi355xBackend(BaseBackend):
    name = "gt:mi355x"
    options = {
        "device_sync": {"versioning": False, "type": bool, "description": "synchronize the stream after each call"},
        "jchunk": {"versioning": True, "type": int, "description": "J rows per wavefront in plane kernels (0 = auto)"},
        "vector": {"versioning": True, "type": int, "description": "I elements per lane in plane kernels (1, 2, 4)"},
        "prefetch": {"versioning": True, "type": int, "description": "rows loaded ahead in plane kernels"},
        "strip_align": {"versioning": True, "type": int, "description": "round plane-strip width to a multiple"},
        "min_blocks": {"versioning": True, "type": int, "description": "plane kernels: __launch_bounds__ min blocks per CU"},
        "pointwise_plane": {"versioning": True, "type": int, "description": "stream pointwise PARALLEL loops with K1"},
        "order": {"versioning": True, "type": int, "description": "plane work order (0 xcd, 1 k-fast, 2 scatter, 3 natural, 4 chunk-slow, 5 level-synchronous xcd, 6 auto: 5 for small launches else 0, default)"},
        "nt_store": {"versioning": True, "type": int, "description": "non-temporal stores of API fields"},
        "nt_load": {"versioning": True, "type": int, "description": "non-temporal loads of read-once streams"},
        "kring": {"versioning": True, "type": int, "description": "column kernels: window-front loads in flight (levels)"},
        "ktail_lds": {"versioning": True, "type": int, "description": "column kernels: LDS bytes for the sweep-to-sweep tail cache (0 = off)"},
        "ktail_all": {"versioning": True, "type": int, "description": "column kernels: tail-cache every eligible field (1) or only write-free scratch when there is any (0)"},
        "dpp": {"versioning": True, "type": int, "description": "plane kernels: +-1-lane I shuffles as DPP wave rotates (1, default) instead of ds_bpermute (0)"},
        "fuse": {"versioning": True, "type": int, "description": "merge adjacent PARALLEL computations over identical intervals into one launch (1, default)"},
        "kreg": {"versioning": True, "type": int, "description": "column kernels: levels of the sweep-to-sweep tail cache held in registers (register band next to the LDS band)"},
        "kreg_pf": {"versioning": True, "type": int, "description": "column kernels: register-band levels whose memory fronts are loaded ahead (default: the load ring depth + 2; 0 = at their level)"},
        "ktail_head": {"versioning": True, "type": int, "description": "column kernels: keep the FIRST levels of the writer's sweep on chip (1), the last (0), or auto (-1: first for cached API outputs, last for write-free scratch)"},
        "col_bx": {"versioning": True, "type": int, "description": "column kernels: threads per block along I (64/128/256)"},
        "col_order": {"versioning": True, "type": int, "description": "column kernels: block order (0 natural, 1 xcd-aware, default)"},
        "jmirror": {"versioning": True, "type": int, "description": "plane kernels: odd J chunks stream top-down"},
        "row_unroll": {"versioning": True, "type": int, "description": "plane kernels: row steps per loop trip (ring rotations become renames; 0 = off, -1 = auto: 4 for small register state, default)"},
        "bufld": {"versioning": True, "type": int, "description": "plane kernels: interior strips load rows through buffer descriptors, branch-free, so prefetched rows stay in flight (1 on, 0 off, -1 auto: on for 4-cell lanes, default)"},
        "tile": {"versioning": True, "type": int, "description": "sequential sweeps that read their own products across columns: tile kernels with LDS planes (1, default) instead of the staged lowering (0)"},
        "tile_by": {"versioning": True, "type": int, "description": "tile kernels: J rows of threads per block (4, 8, 16; -1 auto, default: 16 for a one-row J halo on 8-byte cells, else 8)"},
        "tile_lblock": {"versioning": True, "type": int, "description": "tile kernels: levels per LDS barrier in the steady-state loop (1, 2, 4)"},
        "tile_bx": {"versioning": True, "type": int, "description": "tile kernels: I lanes per block (64 or 128)"},
        "tile_rows": {"versioning": True, "type": int, "description": "tile kernels: J rows per thread (1, default; 2: each thread carries two columns, by rows apart, so the block covers 2 x tile_by rows)"},
        "tile_order": {"versioning": True, "type": int, "description": "tile kernels: work order of the tiles within an XCD's range (0 I-fast, default; 1 J-fast; 2 pairs of J rows, I-fast)"},
        "tile_ti": {"versioning": True, "type": int, "description": "tile kernels: output columns per tile in I (default: 64 minus the sweep's I extent)"},
        "exact_fma": {"versioning": True, "type": int, "description": "f64 add/sub of an exact product (power-of-two literal x a value widened from f32 or a <= 32-bit int) as one fma: bit-identical, one instruction fewer (1, default)"},
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
        plan, source, signature = generate_source(b.analysis, opts)
        t1 = time.perf_counter()
        path = jit.compile_source(source, verbose=bool(opts.get("verbose")))
        t2 = time.perf_counter()
        if b.options.build_info is not None:
            b.options.build_info["codegen_time"] = t1 - t0
            b.options.build_info["build_time"] = t2 - t1
        return _Compiled(b.analysis, plan, source, signature, path, opts)

    def make_run_impl(self):
        compiled = self.compile()

        def run_impl(domain, origin, exec_info, kwargs, rows=None):
            compiled(domain, origin, exec_info, kwargs, rows)

        run_impl.compiled = compiled
        run_impl.bind = compiled.bind  # fast path of repeated calls (stencil_object.py)
        run_impl.supports_rows = True  # gtmi_stencil_run_jsplit
        return run_impl

    def make_stencil_class(self):
        cls = super().make_stencil_class()
        return cls
