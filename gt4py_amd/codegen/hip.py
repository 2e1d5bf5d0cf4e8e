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

WAVE = 64
PLANE_BLOCK_WAVES = 4
PLANE_TARGET_BLOCKS = 60000  # auto J-chunk: aim for at least this many workgroups
PLANE_MIN_JCHUNK = 4
COLUMN_BLOCK = (64, 4)


def cname(name: str) -> str:
    out = "".join(c if c.isalnum() else "_" for c in name)
    return out


# ------------------------------------------------------------------------------------------
# expression rendering
# ------------------------------------------------------------------------------------------


def literal(value, dtype: DataType) -> str:
    if dtype == DataType.BOOL:
        return "true" if value else "false"
    if dtype.isinteger():
        v = int(value)
        if dtype == DataType.INT64:
            if v == -(2**63):
                return "((int64_t)(-9223372036854775807LL - 1))"
            return f"((int64_t){v}LL)"
        return f"(({dtype.ctype}){v})"
    v = float(value)
    if math.isnan(v):
        s = "__builtin_nan(\"\")"
    elif math.isinf(v):
        s = "__builtin_inf()" if v > 0 else "(-__builtin_inf())"
    else:
        s = v.hex()
    return f"(({dtype.ctype})({s}))"


_MATH1 = {
    "sin": "sin",
    "cos": "cos",
    "tan": "tan",
    "arcsin": "asin",
    "arccos": "acos",
    "arctan": "atan",
    "sinh": "sinh",
    "cosh": "cosh",
    "tanh": "tanh",
    "arcsinh": "asinh",
    "arccosh": "acosh",
    "arctanh": "atanh",
    "sqrt": "sqrt",
    "exp": "exp",
    "log": "log",
    "log10": "log10",
    "gamma": "tgamma",
    "cbrt": "cbrt",
    "floor": "floor",
    "ceil": "ceil",
    "trunc": "trunc",
    "erf": "erf",
    "erfc": "erfc",
}


class ExprRenderer:
    """Renders typed IR expressions to C++; ``resolve(FieldAccess) -> str`` is supplied."""

    def __init__(self, resolve, scalar_name, axis_index=None):
        self.resolve = resolve
        self.scalar_name = scalar_name
        self.axis_index = axis_index

    def __call__(self, e: ir.Expr) -> str:
        return self.r(e)

    def r(self, e) -> str:
        if isinstance(e, ir.Literal):
            return literal(e.value, e.dtype)
        if isinstance(e, ir.FieldAccess):
            return self.resolve(e)
        if isinstance(e, ir.ScalarAccess):
            return self.scalar_name(e.name)
        if isinstance(e, ir.Cast):
            return f"(({e.dtype.ctype})({self.r(e.expr)}))"
        if isinstance(e, ir.BinaryOp):
            a, b = self.r(e.left), self.r(e.right)
            if e.op in ("and", "or"):
                return f"({a} {'&&' if e.op == 'and' else '||'} {b})"
            if e.op in ir.COMPARE_OPS:
                return f"({a} {e.op} {b})"
            expr = f"({a} {e.op} {b})"
            if not e.dtype.isfloat():
                return f"(({e.dtype.ctype}){expr})"
            return expr
        if isinstance(e, ir.UnaryOp):
            a = self.r(e.expr)
            if e.op == "not":
                return f"(!{a})"
            if e.op == "-":
                return f"(({e.dtype.ctype})(-{a}))" if not e.dtype.isfloat() else f"(-{a})"
            return f"(+{a})" if e.dtype.isfloat() else f"(({e.dtype.ctype})(+{a}))"
        if isinstance(e, ir.TernaryOp):
            return f"({self.r(e.cond)} ? {self.r(e.true_expr)} : {self.r(e.false_expr)})"
        if isinstance(e, ir.NativeCall):
            return self.native(e)
        if isinstance(e, ir.AxisIndex):
            return self.axis_index(e.axis)
        raise TypeError(type(e))

    def native(self, e: ir.NativeCall) -> str:
        f = e.func
        args = [self.r(a) for a in e.args]
        t = e.dtype.ctype
        if f in ("int32", "int64", "float32", "float64"):
            return f"(({t})({args[0]}))"
        if f == "abs":
            return f"gtmi::absolute({args[0]})"
        if f == "min":
            return f"gtmi::minimum<{t}>({args[0]}, {args[1]})"
        if f == "max":
            return f"gtmi::maximum<{t}>({args[0]}, {args[1]})"
        if f == "mod":
            return f"gtmi::remainder_(({t}){args[0]}, ({t}){args[1]})"
        if f == "pow":
            if e.dtype.isfloat():
                return f"(({t})pow(({t})({args[0]}), ({t})({args[1]})))"
            return f"gtmi::ipow<{t}>(({t})({args[0]}), ({t})({args[1]}))"
        if f in ("isfinite", "isinf", "isnan"):
            at = e.args[0].dtype
            if not at.isfloat():
                return "true" if f == "isfinite" else "false"
            return f"((bool)__builtin_{f}({args[0]}))"
        if f == "round":
            return f"gtmi::round_half_even({args[0]})"
        if f == "round_away_from_zero":
            return f"gtmi::round_away({args[0]})"
        if f in _MATH1:
            at = e.args[0].dtype
            if not at.isfloat():
                return f"(({t}){_MATH1[f]}((double)({args[0]})))"
            return f"(({t}){_MATH1[f]}({args[0]}))"
        raise UnsupportedStencil(f"native function {f}")


# ------------------------------------------------------------------------------------------
# shared field-argument model
# ------------------------------------------------------------------------------------------


@dataclasses.dataclass
class FieldSlot:
    """A memory-backed field visible to kernels: an API field or a scratch temporary."""

    name: str
    index: int  # index in the gtmi_field array
    dtype: DataType
    is_scratch: bool
    data_index: Tuple[str, ...] = ()  # host C expressions: component of a data-dimension field

    @property
    def c(self) -> str:
        return cname(self.name)


def kparam_decl(slot: FieldSlot, writable: bool) -> List[str]:
    c = slot.c
    const = "" if writable else "const "
    return [
        f"{const}{slot.dtype.ctype}* __restrict__ p_{c};",
        f"int64_t sI_{c}, sJ_{c}, sK_{c};",
        f"int32_t ilo_{c}, ihi_{c}, jlo_{c}, jhi_{c}, klo_{c}, khi_{c};",
    ]


def host_fill(slot: FieldSlot, pvar: str, writable: bool) -> List[str]:
    c = slot.c
    t = slot.dtype.ctype
    cast = f"({t}*)" if writable else f"(const {t}*)"
    f = f"f[{slot.index}]"
    comp = "".join(
        f" + (int64_t)gtmi_clamp_index((int64_t)({x}), {f}.data_shape[{d}]) * {f}.data_strides[{d}]"
        for d, x in enumerate(slot.data_index)
    )
    return [
        f"{pvar}.p_{c} = {cast}{f}.data + ({f}.origin[0] * {f}.strides[0] + {f}.origin[1] * {f}.strides[1] + "
        f"{f}.origin[2] * {f}.strides[2]{comp});",
        f"{pvar}.sI_{c} = {f}.strides[0]; {pvar}.sJ_{c} = {f}.strides[1]; {pvar}.sK_{c} = {f}.strides[2];",
        f"{pvar}.ilo_{c} = (int32_t)(-{f}.origin[0]); {pvar}.ihi_{c} = (int32_t)({f}.shape[0] - {f}.origin[0] - 1);",
        f"{pvar}.jlo_{c} = (int32_t)(-{f}.origin[1]); {pvar}.jhi_{c} = (int32_t)({f}.shape[1] - {f}.origin[1] - 1);",
        f"{pvar}.klo_{c} = (int32_t)(-{f}.origin[2]); {pvar}.khi_{c} = (int32_t)({f}.shape[2] - {f}.origin[2] - 1);",
    ]


def interval_bounds(itv: ir.Interval) -> Tuple[str, str]:
    def b(x):
        return f"{x.offset}" if x.level == ir.LevelMarker.START else f"(nk + ({x.offset}))"

    return b(itv.start), b(itv.end)


# ------------------------------------------------------------------------------------------
# K1: J-streaming plane kernel
# ------------------------------------------------------------------------------------------


@dataclasses.dataclass
class Val:
    vid: int
    name: str
    dtype: DataType
    kind: str  # "load" | "stage" | "undef"
    lead: int = 0
    dk: int = 0
    min_read: Optional[int] = None
    max_read: Optional[int] = None
    needed_lo: int = 0
    stage: int = -1
    conditional: bool = False

    needed_ilo: int = 0
    needed_ihi: int = 0

    def note_read(self, row: int, reader_needed_lo: int, dj: int, reader_iext=(0, 0), di: int = 0):
        self.min_read = row if self.min_read is None else min(self.min_read, row)
        self.max_read = row if self.max_read is None else max(self.max_read, row)
        self.needed_lo = max(self.needed_lo, reader_needed_lo - dj)
        self.needed_ilo = max(self.needed_ilo, reader_iext[0] - di)
        self.needed_ihi = max(self.needed_ihi, reader_iext[1] + di)

    @property
    def depth(self) -> int:
        if self.min_read is None:
            return 1
        return max(1, self.lead - self.min_read + 1)

    @property
    def c(self) -> str:
        return f"v{self.vid}_{cname(self.name)}"


@dataclasses.dataclass
class VRef(ir.Expr):
    val: Val
    di: int
    dj: int
    dtype: DataType = DataType.AUTO


@dataclasses.dataclass
class VAssign(ir.Stmt):
    val: Val
    value: ir.Expr
    top_level: bool


@dataclasses.dataclass
class VInit(ir.Stmt):
    """Declare the new version of a conditionally written name, initialised from ``prev``."""

    val: Val
    prev: Optional[VRef]


class PlaneGen:
    def __init__(self, analysis: StencilAnalysis, plan: KernelPlan, kernel: PlaneKernel, slots, kid: int, opts):
        self.a = analysis
        self.st = analysis.stencil
        self.plan = plan
        self.kernel = kernel
        self.slots: Dict[str, FieldSlot] = slots
        self.kid = kid
        self.opts = opts
        self.vl = self.st.vertical_loops[kernel.loop]
        self.sec = self.vl.sections[kernel.section]
        for acc, w in iter_accesses(self.sec.body):
            if isinstance(acc, ir.FieldAccess) and w and not self.st.decl(acc.name).mask[2]:
                # one value per column written from every level of a PARALLEL section: only a
                # sequential column sweep defines which level is the last writer
                raise UnsupportedStencil(f"'{acc.name}' has no K axis and is written in a PARALLEL section")
        self.vals: List[Val] = []
        self.loads: Dict[Tuple[str, int], Val] = {}
        self.current: Dict[str, Val] = {}
        self.api = {p.name for p in self.st.field_params()}
        self.scratch = set(plan.scratch)
        self.stage_ext = []
        for ti in range(len(self.sec.body)):
            self.stage_ext.append(analysis.extents.blocks[(kernel.loop, kernel.section, ti)])

    # -------------------------------------------------------------- value bookkeeping
    def _new_val(self, name, dtype, kind, **kw) -> Val:
        v = Val(len(self.vals), name, dtype, kind, **kw)
        self.vals.append(v)
        return v

    def _mem_backed(self, name) -> bool:
        return name in self.api or name in self.scratch

    def _load(self, name, dk, dtype) -> Val:
        key = (name, dk)
        if key not in self.loads:
            self.loads[key] = self._new_val(name, dtype, "load", dk=dk)
        return self.loads[key]

    def _read(self, acc: ir.FieldAccess, ti: int, written_here: Set[str]) -> VRef:
        di, dj, dk = acc.offset
        lead = self.stage_ext[ti][1][1]
        needed_lo = self.stage_ext[ti][1][0]
        if acc.name in written_here:
            if di or dj or dk:
                raise UnsupportedStencil(
                    f"'{acc.name}' is read at offset {acc.offset} in the statement that writes it"
                )
            v = self.current[acc.name]
        elif acc.name in self.current:
            if dk:
                raise UnsupportedStencil(f"K-offset read of '{acc.name}' written in the same PARALLEL section")
            v = self.current[acc.name]
        elif self._mem_backed(acc.name):
            v = self._load(acc.name, dk, acc.dtype)
        else:
            v = self._new_val(acc.name, acc.dtype, "undef")
        v.note_read(lead + dj, needed_lo, dj, self.stage_ext[ti][0], di)
        return VRef(v, di, dj, acc.dtype)

    # -------------------------------------------------------------- SSA construction
    def build(self):
        self.stage_code = []
        for ti, stmt in enumerate(self.sec.body):
            lead = self.stage_ext[ti][1][1]
            needed_lo = self.stage_ext[ti][1][0]
            out: List[ir.Stmt] = []
            if isinstance(stmt, ir.Assign):
                value = self._rewrite_expr(stmt.value, ti, set())
                nv = self._new_val(stmt.target.name, stmt.target.dtype, "stage", lead=lead, stage=ti)
                nv.needed_lo = needed_lo
                out.append(VAssign(nv, value, True))
                self.current[stmt.target.name] = nv
            else:
                written = []
                for n in ir.walk([stmt]):
                    if isinstance(n, ir.Assign) and n.target.name not in written:
                        written.append(n.target.name)
                new_vals = {}
                for name in written:
                    dtype = self.st.decl(name).dtype
                    if name in self.current:
                        prev = self.current[name]
                        prev.note_read(lead, needed_lo, 0, self.stage_ext[ti][0], 0)
                        pref = VRef(prev, 0, 0, dtype)
                    elif self._mem_backed(name):
                        prev = self._load(name, 0, dtype)
                        prev.note_read(lead, needed_lo, 0, self.stage_ext[ti][0], 0)
                        pref = VRef(prev, 0, 0, dtype)
                    else:
                        pref = None
                    nv = self._new_val(name, dtype, "stage", lead=lead, stage=ti, conditional=True)
                    nv.needed_lo = needed_lo
                    out.append(VInit(nv, pref))
                    new_vals[name] = nv
                body = self._rewrite_stmt(stmt, ti, new_vals, set(), in_loop=False)
                out.append(body)
                for name, nv in new_vals.items():
                    self.current[name] = nv
            self.stage_code.append(out)
        # finalize load leads
        for v in self.loads.values():
            v.lead = v.max_read if v.max_read is not None else 0
        return self

    def _rewrite_expr(self, e, ti, written_here: Set[str], new_vals=None):
        def fn(x):
            if isinstance(x, ir.FieldAccess):
                if new_vals is not None and x.name in new_vals and x.name in written_here:
                    if any(x.offset):
                        raise UnsupportedStencil(
                            f"'{x.name}' is read at offset {x.offset} in the statement that writes it"
                        )
                    return VRef(new_vals[x.name], 0, 0, x.dtype)
                return self._read(x, ti, set())
            return x

        return ir.map_expr(e, fn)

    def _rewrite_stmt(self, s, ti, new_vals, written: Set[str], in_loop: bool):
        if isinstance(s, ir.Assign):
            value = self._rewrite_expr(s.value, ti, written, new_vals)
            written.add(s.target.name)
            return VAssign(new_vals[s.target.name], value, False)
        if isinstance(s, ir.If):
            cond = self._rewrite_expr(s.cond, ti, written, new_vals)
            w_body = set(written)
            body = [self._rewrite_stmt(x, ti, new_vals, w_body, in_loop) for x in s.body]
            w_else = set(written)
            orelse = [self._rewrite_stmt(x, ti, new_vals, w_else, in_loop) for x in s.orelse]
            written |= w_body | w_else
            return ir.If(cond, body, orelse)
        if isinstance(s, ir.While):
            inner = {n.target.name for n in ir.walk(s.body) if isinstance(n, ir.Assign)}
            written |= inner
            cond = self._rewrite_expr(s.cond, ti, written, new_vals)
            body = [self._rewrite_stmt(x, ti, new_vals, written, True) for x in s.body]
            return ir.While(cond, body)
        if isinstance(s, ir.HorizontalRegion):
            body = [self._rewrite_stmt(x, ti, new_vals, written, in_loop) for x in s.body]
            return ir.HorizontalRegion(s.masks, body)
        raise TypeError(type(s))

    # -------------------------------------------------------------- geometry
    def geometry(self, V: int):
        """I halo (rounded to the vector width), strip width, first row step, per-value ranges."""
        h_lo = h_hi = 0
        for ti, code in enumerate(self.stage_code):
            ilo, ihi = self.stage_ext[ti][0]
            h_lo, h_hi = max(h_lo, ilo), max(h_hi, ihi)
            for ref in _vrefs_in(code):
                h_lo = max(h_lo, ilo - ref.di)
                h_hi = max(h_hi, ihi + ref.di)
        for name, (ie, _) in self.plan.scratch_extent.items():
            if name in self.current:
                h_lo, h_hi = max(h_lo, ie[0]), max(h_hi, ie[1])
        h_lo = -(-h_lo // V) * V
        h_hi = -(-h_hi // V) * V
        self.V = V
        self.h_lo, self.h_hi = h_lo, h_hi
        self.npos = WAVE * V
        self.w_out = self.npos - h_lo - h_hi
        # align output strips to 128-B lines of the widest stored field (measured: +5-10% on MI355X)
        stored = [self.st.decl(n).dtype.itemsize for n in self.current if self._mem_backed(n)]
        align = int(self.opts.get("strip_align", 128 // max(stored) if stored else 0))
        if align > 1 and self.w_out >= 2 * align:
            self.w_out = (self.w_out // align) * align
        if self.w_out < 8:
            raise UnsupportedStencil(f"I halo {h_lo}+{h_hi} too wide for a {self.npos}-wide strip")
        t_start = 0
        for v in self.vals:
            if v.kind == "undef":
                continue
            t_start = min(t_start, -(v.needed_lo + v.lead))
        self.t_start = t_start

    def _nt_load(self, v: Val) -> bool:
        """Non-temporal loads for streams read once (no IJ offsets), if enabled."""
        if not self.opts.get("nt_load", 1):
            return False
        return v.needed_ilo == 0 and v.needed_ihi == 0 and v.depth == 1

    def _lane_range(self, v: Val) -> Tuple[int, int]:
        """Lanes whose elements hold positions the value is needed at (inclusive)."""
        lo_pos = self.h_lo - v.needed_ilo
        hi_pos = self.h_lo + self.w_out - 1 + v.needed_ihi
        return max(0, lo_pos // self.V), min(WAVE - 1, hi_pos // self.V)

    # -------------------------------------------------------------- rendering
    def render(self) -> Tuple[str, str]:
        self.build()
        variants = [1]
        if "vector" in self.opts:
            vec = int(self.opts["vector"])
        else:  # 16 B per lane for the widest memory-backed type of the section
            sizes = [self.st.decl(n).dtype.itemsize for (n, _dk) in self.loads] + [
                self.st.decl(n).dtype.itemsize for n in self.current if self._mem_backed(n)
            ]
            vec = max(1, min(4, 16 // max(sizes))) if sizes else 1
        if vec > 1:
            variants.append(vec)
        srcs = []
        launches = {}
        for V in variants:
            self.geometry(V)
            src, launch = self._render_variant(V)
            srcs.append(src)
            launches[V] = launch
        return "\n\n".join(srcs), self._render_host(launches)

    def _used_slots(self):
        used, written = [], set()
        for (name, _dk) in self.loads:
            if self.slots[name] not in used:
                used.append(self.slots[name])
        for name in self.current:
            if self._mem_backed(name):
                written.add(name)
                if self.slots[name] not in used:
                    used.append(self.slots[name])
        return used, written

    def _render_variant(self, V: int) -> Tuple[str, dict]:
        k = self.kid
        P = int(self.opts.get("prefetch", 4 if V <= 2 else 2))
        used_slots, written_slots = self._used_slots()
        scalars = self.st.scalar_params()
        L = []
        if V == 1:
            L.append(f"struct K{k}Params {{")
            for s in used_slots:
                L += ["    " + x for x in kparam_decl(s, s.name in written_slots)]
            for s in scalars:
                L.append(f"    {s.dtype.ctype} s_{cname(s.name)};")
            L.append("    int32_t ni, nj, nk, k0, nks, jc, n_strips, n_chunks, n_sgroups, perm_a;")
            L.append("};")
            L.append("")
        kname = f"k{k}_plane_v{V}"
        mb = int(self.opts.get("min_blocks", 0))  # blocks per CU the register budget must allow
        lb = f"{WAVE * PLANE_BLOCK_WAVES}, {mb}" if mb > 0 else f"{WAVE * PLANE_BLOCK_WAVES}"
        L.append(f"__global__ void __launch_bounds__({lb}) {kname}(const K{k}Params p) {{")
        B = []
        B.append("const int lane = (int)__lane_id();")
        B.append("const int wave = (int)(threadIdx.x >> 6);")
        order = int(self.opts.get("order", 0))
        B.append("const int nb = (int)gridDim.x, b = (int)blockIdx.x;")
        if order == 3:
            B.append("const int w = b;  // natural dispatch order")
        else:
            B.append("// XCD-aware block remap: consecutive work items share an XCD (8 XCDs, round-robin dispatch)")
            B.append("const int q = nb >> 3, r = nb & 7, xcd = b & 7, slot = b >> 3;")
            B.append("const int w0x = (xcd < r) ? xcd * (q + 1) + slot : r * (q + 1) + (xcd - r) * q + slot;")
            if order == 2:
                B.append("const int w = (int)(((long long)w0x * p.perm_a) % nb);  // bijective scatter")
            else:
                B.append("const int w = w0x;")
        if order == 4:  # chunks slowest: chunk c+1 starts as chunk c ends on the same XCD (halo rows warm)
            B.append("const int sg = w % p.n_sgroups;")
            B.append("const int rest = w / p.n_sgroups;")
            B.append("const int kk = p.k0 + rest % p.nks;")
            B.append("const int chunk = rest / p.nks;")
        elif order == 1:
            B.append("const int kk = p.k0 + w % p.nks;")
            B.append("const int rest = w / p.nks;")
            B.append("const int sg = rest % p.n_sgroups;")
            B.append("const int chunk = rest / p.n_sgroups;")
        else:
            B.append("const int sg = w % p.n_sgroups;")
            B.append("const int rest = w / p.n_sgroups;")
            B.append("const int chunk = rest % p.n_chunks;")
            B.append("const int kk = p.k0 + rest / p.n_chunks;")
        B.append(f"const int strip = sg * {PLANE_BLOCK_WAVES} + wave;")
        B.append("if (strip >= p.n_strips) return;")
        B.append(f"const int ib = strip * {self.w_out};")
        B.append("const int jb = chunk * p.jc;")
        B.append("const int jce = min(p.jc, p.nj - jb);")
        B.append(f"const int w0 = ib - {self.h_lo};")
        B.append(f"const int pos = w0 + lane * {V};  // position of element 0 of this lane")
        for e in range(V):
            B.append(f"const int i_{e} = pos + {e};")
            B.append(f"const int rel_{e} = lane * {V} + {e} - {self.h_lo};")
            B.append(f"const bool own_{e} = (rel_{e} >= 0) && (rel_{e} < {self.w_out}) && (i_{e} < p.ni);")
        for s in scalars:
            B.append(f"const {s.dtype.ctype} s_{cname(s.name)} = p.s_{cname(s.name)};")
        for s in used_slots:
            c = s.c
            if V == 1:
                B.append(f"const int64_t li_{c} = (int64_t)gtmi::clampi(pos, p.ilo_{c}, p.ihi_{c}) * p.sI_{c};")
            else:
                B.append(f"const bool vok_{c} = (pos >= p.ilo_{c}) && (pos + {V - 1} <= p.ihi_{c});")
        # rings (+ per-element registers)
        for v in self.vals:
            if v.kind == "undef":
                continue
            for a in range(v.depth):
                for e in range(V):
                    B.append(f"{v.dtype.ctype} {v.c}_{a}_{e} = ({v.dtype.ctype})0;")
        loads = list(self.loads.values())
        for v in loads:
            lo, hi = self._lane_range(v)
            B.append(f"const bool ln_{v.c} = (lane >= {lo}) && (lane <= {hi});")
            for pp in range(P):
                for e in range(V):
                    B.append(f"{v.dtype.ctype} pf{pp}_{v.c}_{e} = ({v.dtype.ctype})0;")

        def emit_load(v: Val, row_expr: str, dests: List[str]) -> List[str]:
            c = cname(v.name)
            kexpr = f"kk + ({v.dk})" if v.dk else "kk"
            out = [
                "{",
                f"    const int64_t ro = (int64_t)gtmi::clampi({row_expr}, p.jlo_{c}, p.jhi_{c}) * p.sJ_{c} + "
                f"(int64_t)gtmi::clampi({kexpr}, p.klo_{c}, p.khi_{c}) * p.sK_{c};",
                f"    if (ln_{v.c}) {{",
            ]
            if V == 1:
                nt = "true" if self._nt_load(v) else "false"
                out.append(f"        {dests[0]} = gtmi::sload<{v.dtype.ctype}, {nt}>(p.p_{c} + li_{c} + ro);")
            else:
                t = v.dtype.ctype
                nt = "true" if self._nt_load(v) else "false"
                out.append(f"        if (vok_{c}) {{")
                if v.dtype.itemsize >= 4:
                    out.append(f"            {t} tmp[{V}];")
                    out.append(f"            gtmi::vload<{t}, {V}, {nt}>(p.p_{c} + pos + ro, tmp);")
                    for e in range(V):
                        out.append(f"            {dests[e]} = tmp[{e}];")
                else:
                    out.append(
                        f"            const gtmi::vec<{t}, {V}> tmp = "
                        f"*reinterpret_cast<const gtmi::vec<{t}, {V}>*>(p.p_{c} + pos + ro);"
                    )
                    for e in range(V):
                        out.append(f"            {dests[e]} = tmp.v[{e}];")
                out.append("        } else {")
                for e in range(V):
                    out.append(
                        f"            {dests[e]} = p.p_{c}[(int64_t)gtmi::clampi(pos + {e}, p.ilo_{c}, p.ihi_{c}) * "
                        f"p.sI_{c} + ro];"
                    )
                out.append("        }")
            out.append("    }")
            out.append("}")
            return out

        # initial prefetch
        for v in loads:
            first = -(v.needed_lo + v.lead)
            for pp in range(P):
                B.append(f"if ({self.t_start + pp} >= {first} && {self.t_start + pp} < jce)")
                B += ["    " + x for x in emit_load(v, f"jb + ({self.t_start + pp}) + ({v.lead})",
                                                   [f"pf{pp}_{v.c}_{e}" for e in range(V)])]
        B.append(f"for (int t = {self.t_start}; t < jce; ++t) {{")
        S = []
        for v in loads:
            first = -(v.needed_lo + v.lead)
            if P == 0:
                S.append(f"if (t >= {first})")
                S += ["    " + x for x in emit_load(v, f"jb + t + ({v.lead})", [f"{v.c}_0_{e}" for e in range(V)])]
            else:
                for e in range(V):
                    S.append(f"{v.c}_0_{e} = pf0_{v.c}_{e};")
                for pp in range(P - 1):
                    for e in range(V):
                        S.append(f"pf{pp}_{v.c}_{e} = pf{pp + 1}_{v.c}_{e};")
                S.append(f"if (t + {P} >= {first} && t + {P} < jce)")
                S += ["    " + x for x in emit_load(v, f"jb + t + {P} + ({v.lead})",
                                                   [f"pf{P - 1}_{v.c}_{e}" for e in range(V)])]
        for ti, code in enumerate(self.stage_code):
            lead = self.stage_ext[ti][1][1]
            S.append(f"{{  // stage {ti}: row t + {lead}")
            S += ["    " + x for x in self._render_stage(ti, code, lead)]
            S.append("}")
        S += self._render_stores()
        for v in self.vals:
            if v.kind == "undef":
                continue
            for a in range(v.depth - 1, 0, -1):
                for e in range(V):
                    S.append(f"{v.c}_{a}_{e} = {v.c}_{a - 1}_{e};")
        B += ["    " + x for x in S]
        B.append("}")
        L += ["    " + x for x in B]
        L.append("}")
        geo = {"w_out": self.w_out, "V": V, "kname": kname, "used": used_slots}
        return "\n".join(L), geo

    def _render_stores(self) -> List[str]:
        V = self.V
        S = []
        for name, v in self.current.items():
            if not self._mem_backed(name):
                continue
            c = cname(name)
            row = f"jb + t + ({v.lead})"
            if name in self.scratch:
                (eilo, eihi), (ejlo, ejhi) = self.plan.scratch_extent[name]
                rcond = (
                    f"(t + ({v.lead}) >= (chunk == 0 ? -jb - {ejlo} : 0)) && "
                    f"(t + ({v.lead}) < (chunk == p.n_chunks - 1 ? p.nj - jb + {ejhi} : jce))"
                )
                econd = [
                    f"((strip == 0 ? (rel_{e} >= -{eilo}) : (rel_{e} >= 0)) && "
                    f"(strip == p.n_strips - 1 ? (i_{e} < p.ni + {eihi}) : (rel_{e} < {self.w_out})))"
                    for e in range(V)
                ]
            else:
                rcond = f"(t + ({v.lead}) >= 0) && (t + ({v.lead}) < jce)"
                econd = [f"own_{e}" for e in range(V)]
            S.append(f"if ({rcond}) {{")
            S.append(f"    const int64_t ro = (int64_t)({row}) * p.sJ_{c} + (int64_t)kk * p.sK_{c};")
            nts = "true" if (self.opts.get("nt_store", 1) and name not in self.scratch) else "false"
            if V == 1:
                S.append(
                    f"    if ({econd[0]}) gtmi::sstore<{v.dtype.ctype}, {nts}>(p.p_{c} + (int64_t)i_0 * p.sI_{c} + ro, "
                    f"{v.c}_0_0);"
                )
            else:
                t = v.dtype.ctype
                allc = " && ".join(f"({x})" for x in econd)
                S.append(f"    if (vok_{c} && {allc}) {{")
                if v.dtype.itemsize >= 4:
                    S.append(f"        const {t} tmp[{V}] = {{{', '.join(f'{v.c}_0_{e}' for e in range(V))}}};")
                    S.append(f"        gtmi::vstore<{t}, {V}, {nts}>(p.p_{c} + pos + ro, tmp);")
                else:
                    S.append(f"        gtmi::vec<{t}, {V}> tmp;")
                    for e in range(V):
                        S.append(f"        tmp.v[{e}] = {v.c}_0_{e};")
                    S.append(f"        *reinterpret_cast<gtmi::vec<{t}, {V}>*>(p.p_{c} + pos + ro) = tmp;")
                S.append("    } else {")
                for e in range(V):
                    S.append(f"        if ({econd[e]}) p.p_{c}[(int64_t)i_{e} * p.sI_{c} + ro] = {v.c}_0_{e};")
                S.append("    }")
            S.append("}")
        return S

    def _render_host(self, launches: Dict[int, dict]) -> str:
        k = self.kid
        used_slots, written_slots = self._used_slots()
        H = []
        lo, hi = interval_bounds(self.sec.interval)
        H.append(f"{{  // kernel {k}: plane, loop {self.kernel.loop} section {self.kernel.section}")
        H.append(f"    int k0 = {lo}, k1 = {hi};")
        H.append("    if (k0 < 0) k0 = 0; if (k1 > nk) k1 = nk;")
        H.append("    if (k1 > k0 && ni > 0 && nj > 0) {")
        H.append(f"        K{k}Params p;")
        for s in used_slots:
            H += ["        " + x for x in host_fill(s, "p", s.name in written_slots)]
        for i_s, s in enumerate(self.st.scalar_params()):
            H.append(f"        memcpy(&p.s_{cname(s.name)}, &sc[{i_s}], sizeof(p.s_{cname(s.name)}));")
        H.append("        p.ni = ni; p.nj = nj; p.nk = nk; p.k0 = k0; p.nks = k1 - k0;")
        jchunk = int(self.opts.get("jchunk", 0))
        vecs = sorted(launches, reverse=True)
        H.append("        int vsel = 1;")
        for V in vecs:
            if V == 1:
                continue
            conds = ["(gtmi_env_vector() != 1)"]
            for s in used_slots:
                c = s.c
                isz = s.dtype.itemsize
                conds.append(
                    f"(p.sI_{c} == 1 && (p.sJ_{c} % {V}) == 0 && (p.sK_{c} % {V}) == 0 && "
                    f"(((uintptr_t)p.p_{c}) % {V * isz}) == 0)"
                )
            H.append(f"        if ({' && '.join(conds)}) vsel = {V};")
        for V in vecs:
            g = launches[V]
            H.append(f"        {'if' if V == vecs[0] else 'else if'} (vsel == {V}) {{")
            H.append(f"            p.n_strips = (ni + {g['w_out']} - 1) / {g['w_out']};")
            H.append(f"            p.n_sgroups = (p.n_strips + {PLANE_BLOCK_WAVES - 1}) / {PLANE_BLOCK_WAVES};")
            if jchunk > 0:
                H.append(f"            p.jc = {jchunk};")
            else:
                # auto: the longest J chunk (<= 32 rows, >= 4) that still gives ~64K workgroups; shorter
                # chunks trade halo-row re-reads for more concurrent row streams and a shorter tail
                # (MI355X sweeps: hdiff 2048^2x160 best at 16, lap5 1024^2x80 at 4, hdiff f32 at 16)
                H.append("            p.jc = 32;")
                H.append(
                    f"            while (p.jc > {PLANE_MIN_JCHUNK} && (long long)p.n_sgroups * ((nj + p.jc - 1) / p.jc) * "
                    f"p.nks < {PLANE_TARGET_BLOCKS}LL) p.jc >>= 1;"
                )
            H.append("            p.n_chunks = (nj + p.jc - 1) / p.jc;")
            H.append("            const long long nblocks = (long long)p.n_sgroups * p.n_chunks * p.nks;")
            H.append("            if (nblocks > 0x7fffffffLL) { gtmi_set_error(\"grid too large\"); return 2; }")
            H.append("            p.perm_a = gtmi_coprime_multiplier((long long)nblocks);")
            H.append(
                f"            hipLaunchKernelGGL({g['kname']}, dim3((unsigned)nblocks), "
                f"dim3({WAVE * PLANE_BLOCK_WAVES}), 0, stream, p);"
            )
            H.append("        }")
        H.append("    }")
        H.append("}")
        return "\n".join(H)

    def _render_stage(self, ti, code, lead) -> List[str]:
        V = self.V
        out: List[str] = []
        shuffles: Dict[Tuple[int, int, int, int], str] = {}
        refs = []
        for s in code:
            refs += _vrefs_in(s)
        # hoist every cross-lane read of the stage out of divergent control flow
        for ref in refs:
            if ref.val.kind == "undef" or (ref.val.conditional and ref.val.stage == ti):
                continue
            slot = ref.val.lead - (lead + ref.dj)
            for e in range(V):
                src = e + ref.di
                qd, r = src // V, src % V
                if qd == 0:
                    continue
                key = (ref.val.vid, slot, r, qd)
                if key not in shuffles:
                    nm = f"sh{len(shuffles)}"
                    shuffles[key] = nm
                    out.append(f"const {ref.val.dtype.ctype} {nm} = gtmi::shfl({ref.val.c}_{slot}_{r}, {qd});")

        for e in range(V):

            def resolve(ref, e=e) -> str:
                if ref.val.kind == "undef":
                    return f"(({ref.val.dtype.ctype})0)"
                if ref.val.conditional and ref.val.stage == ti:
                    return f"{ref.val.c}_{e}"
                slot = ref.val.lead - (lead + ref.dj)
                assert 0 <= slot < ref.val.depth, (ref.val, slot, lead, ref.dj)
                src = e + ref.di
                qd, r = src // V, src % V
                if qd != 0:
                    return shuffles[(ref.val.vid, slot, r, qd)]
                return f"{ref.val.c}_{slot}_{r}"

            rend = _VRenderer(resolve, lambda n: f"s_{cname(n)}", self._axis_index(lead, e))
            if V > 1:
                out.append(f"// element {e}")
            for s in code:
                out += self._stmt(s, rend, e, lead)
            for s in code:
                if isinstance(s, VInit):
                    out.append(f"{s.val.c}_0_{e} = {s.val.c}_{e};")
        return out

    def _axis_index(self, lead, e):
        def ax(axis):
            return [f"i_{e}", f"(jb + t + ({lead}))", "kk"][axis]

        return ax

    def _stmt(self, s, rend, e, lead) -> List[str]:
        if isinstance(s, VInit):
            t = s.val.dtype.ctype
            init = rend(s.prev) if s.prev is not None else f"({t})0"
            return [f"{t} {s.val.c}_{e} = {init};"]
        if isinstance(s, VAssign):
            target = f"{s.val.c}_{e}" if not s.top_level else f"{s.val.c}_0_{e}"
            return [f"{target} = {rend(s.value)};"]
        if isinstance(s, ir.If):
            out = [f"if ({rend(s.cond)}) {{"]
            for x in s.body:
                out += ["    " + y for y in self._stmt(x, rend, e, lead)]
            if s.orelse:
                out.append("} else {")
                for x in s.orelse:
                    out += ["    " + y for y in self._stmt(x, rend, e, lead)]
            out.append("}")
            return out
        if isinstance(s, ir.While):
            out = [f"while ({rend(s.cond)}) {{"]
            for x in s.body:
                out += ["    " + y for y in self._stmt(x, rend, e, lead)]
            out.append("}")
            return out
        if isinstance(s, ir.HorizontalRegion):
            cond = region_condition(s.masks, f"i_{e}", f"(jb + t + ({lead}))", "p.ni", "p.nj")
            out = [f"if ({cond}) {{"]
            for x in s.body:
                out += ["    " + y for y in self._stmt(x, rend, e, lead)]
            out.append("}")
            return out
        raise TypeError(type(s))


def region_condition(masks, iv, jv, ni, nj) -> str:
    def bound(b, n):
        return f"{b.offset}" if b.level == ir.LevelMarker.START else f"({n} + ({b.offset}))"

    parts = []
    for m in masks:
        conds = []
        for itv, var, n in ((m.i, iv, ni), (m.j, jv, nj)):
            if itv.start is not None:
                conds.append(f"({var} >= {bound(itv.start, n)})")
            if itv.end is not None:
                conds.append(f"({var} < {bound(itv.end, n)})")
        parts.append("(" + (" && ".join(conds) if conds else "true") + ")")
    return " || ".join(parts) if parts else "false"


def _vrefs_in(node) -> List[VRef]:
    out = []
    stack = [node]
    while stack:
        n = stack.pop()
        if isinstance(n, VRef):
            out.append(n)
            continue
        if isinstance(n, list):
            stack.extend(n)
            continue
        if isinstance(n, VInit):
            if n.prev is not None:
                stack.append(n.prev)
            continue
        if isinstance(n, VAssign):
            stack.append(n.value)
            continue
        if dataclasses.is_dataclass(n):
            for f in dataclasses.fields(n):
                v = getattr(n, f.name)
                if isinstance(v, (ir.Expr, ir.Stmt, list)):
                    stack.append(v)
    return out


class _VRenderer(ExprRenderer):
    def r(self, e):
        if isinstance(e, VRef):
            return self.resolve(e)
        return super().r(e)


# ------------------------------------------------------------------------------------------
# K2: column kernel
# ------------------------------------------------------------------------------------------


class ColumnGen:
    def __init__(self, analysis: StencilAnalysis, plan: KernelPlan, kernel: ColumnKernel, slots, kid, opts):
        self.a = analysis
        self.st = analysis.stencil
        self.plan = plan
        self.kernel = kernel
        self.slots = slots
        self.kid = kid
        self.opts = opts
        self.api = {p.name for p in self.st.field_params()}
        self.scratch = set(plan.scratch)
        # compute region: the union of the IJ extents of the kernel's statements (temporaries that a
        # later kernel reads at IJ offsets are produced on their halo too, passes.compute_extents)
        ilo = ihi = jlo = jhi = 0
        for li in kernel.loops:
            for si, sec in enumerate(self.st.vertical_loops[li].sections):
                for ti in range(len(sec.body)):
                    (a, b), (c, d) = analysis.extents.blocks.get((li, si, ti), ((0, 0), (0, 0)))
                    ilo, ihi, jlo, jhi = max(ilo, a), max(ihi, b), max(jlo, c), max(jhi, d)
        self.ext = (ilo, ihi, jlo, jhi)

    def _mem(self, name):
        return name in self.api or name in self.scratch

    def _guard(self, li, si, ti) -> Optional[str]:
        """Condition restricting top-level statement ti to its own extent (None: whole region)."""
        (a, b), (c, d) = self.a.extents.blocks.get((li, si, ti), ((0, 0), (0, 0)))
        ilo, ihi, jlo, jhi = self.ext
        conds = []
        if a < ilo:
            conds.append(f"i >= {-a}")
        if b < ihi:
            conds.append(f"i < p.ni + {b}")
        if c < jlo:
            conds.append(f"j >= {-c}")
        if d < jhi:
            conds.append(f"j < p.nj + {d}")
        return " && ".join(conds) if conds else None

    def render(self) -> Tuple[str, str]:
        k = self.kid
        st = self.st
        used: List[FieldSlot] = []
        written: Set[str] = set()
        for li in self.kernel.loops:
            for sec in st.vertical_loops[li].sections:
                for acc, w in iter_accesses(sec.body):
                    if isinstance(acc, ir.FieldAccess) and self._mem(acc.name):
                        if self.slots[acc.name] not in used:
                            used.append(self.slots[acc.name])
                        if w:
                            written.add(acc.name)
        # cache policy: non-temporal loads of read-once streams (never written here, one IJ offset)
        # and non-temporal stores of fields no other loop of this kernel reads back
        keys: Dict[str, Set[Tuple[int, int]]] = {}
        read_loops: Dict[str, Set[int]] = {}
        write_loops: Dict[str, Set[int]] = {}
        for li in self.kernel.loops:
            for sec in st.vertical_loops[li].sections:
                for acc, w in iter_accesses(sec.body):
                    if not isinstance(acc, ir.FieldAccess):
                        continue
                    (write_loops if w else read_loops).setdefault(acc.name, set()).add(li)
                    if not w:
                        keys.setdefault(acc.name, set()).add(acc.offset[:2])
        self.nt_loads = set()
        self.nt_stores = set()
        if self.opts.get("nt_load", 1):
            self.nt_loads = {n for n, ks in keys.items() if n not in write_loops and len(ks) == 1 and self._mem(n)}
        if self.opts.get("nt_store", 1):
            self.nt_stores = {
                n for n, wl in write_loops.items()
                if self._mem(n) and n not in self.scratch and not (read_loops.get(n, set()) - wl)
            }
        scalars = st.scalar_params()
        L = [f"struct K{k}Params {{"]
        for s in used:
            L += ["    " + x for x in kparam_decl(s, s.name in written)]
        for s in scalars:
            L.append(f"    {s.dtype.ctype} s_{cname(s.name)};")
        L.append("    int32_t ni, nj, nk;")
        L.append("};")
        L.append("")
        bx, by = COLUMN_BLOCK
        L.append(f"__global__ void __launch_bounds__({bx * by}) k{k}_column(const K{k}Params p) {{")
        if int(self.opts.get("col_occupancy", 0)) > 0:
            L.append("    extern __shared__ __attribute__((aligned(16))) char gtmi_lds_reserve[];")
            L.append("    if (p.ni < 0) gtmi_lds_reserve[threadIdx.x] = 0;  // keep the reservation alive")
        B = []
        eilo, eihi, ejlo, ejhi = self.ext
        B.append(f"const int i = (int)(blockIdx.x * {bx} + threadIdx.x) - {eilo};")
        B.append(f"const int j = (int)(blockIdx.y * {by} + threadIdx.y) - {ejlo};")
        B.append(f"if (i >= p.ni + {eihi} || j >= p.nj + {ejhi}) return;")
        B.append("const int nk = p.nk;")
        for s in scalars:
            B.append(f"const {s.dtype.ctype} s_{cname(s.name)} = p.s_{cname(s.name)};")
        for li in self.kernel.loops:
            B += self._render_loop(li)
        L += ["    " + x for x in B]
        L.append("}")
        H = [f"{{  // kernel {k}: column, loops {self.kernel.loops}"]
        H.append("    if (ni > 0 && nj > 0 && nk > 0) {")
        H.append(f"        K{k}Params p;")
        for s in used:
            H += ["        " + x for x in host_fill(s, "p", s.name in written)]
        for i_s, s in enumerate(scalars):
            H.append(f"        memcpy(&p.s_{cname(s.name)}, &sc[{i_s}], sizeof(p.s_{cname(s.name)}));")
        H.append("        p.ni = ni; p.nj = nj; p.nk = nk;")
        occ = int(self.opts.get("col_occupancy", 0))
        # blocks per CU capped through the LDS reservation: keeps the K-sweep working set of the
        # resident columns small enough to be re-read from the 256 MiB Infinity Cache
        lds = 0 if occ <= 0 else min(160 * 1024, (160 * 1024) // occ - 1024)
        H.append(
            f"        hipLaunchKernelGGL(k{k}_column, dim3((unsigned)((ni + {eilo + eihi + bx - 1}) / {bx}), "
            f"(unsigned)((nj + {ejlo + ejhi + by - 1}) / {by})), dim3({bx}, {by}), {lds}, stream, p);"
        )
        H.append("    }")
        H.append("}")
        return "\n".join(L), "\n".join(H)

    def _render_loop(self, li) -> List[str]:
        vl = self.st.vertical_loops[li]
        order = vl.loop_order
        fwd = order != ir.LoopOrder.BACKWARD
        # direct fields: read at a run-time K offset or written at a K offset in this loop; every
        # access to them goes to memory at its own address (no register window)
        direct: Set[str] = set()
        for sec in vl.sections:
            for acc, w in iter_accesses(sec.body):
                if isinstance(acc, ir.FieldAccess) and (acc.k_offset is not None or (w and acc.offset[2] != 0)):
                    if not self._mem(acc.name):
                        raise UnsupportedStencil(f"run-time or written K offset on temporary '{acc.name}'")
                    direct.add(acc.name)
        self.direct = direct
        # windows: key (name, di, dj) -> [dmin, dmax]
        win: Dict[Tuple[str, int, int], List[int]] = {}
        wnames: Set[str] = set()
        for sec in vl.sections:
            for acc, w in iter_accesses(sec.body):
                if not isinstance(acc, ir.FieldAccess) or acc.name in direct:
                    continue
                di, dj, dk = acc.offset
                key = (acc.name, di, dj)
                rng = win.setdefault(key, [dk, dk])
                rng[0], rng[1] = min(rng[0], dk), max(rng[1], dk)
                if w:
                    wnames.add(acc.name)
        for (name, di, dj), rng in win.items():
            if name in wnames:
                if di or dj:
                    raise UnsupportedStencil(f"'{name}' written and read at IJ offset in one column loop")
                rng[0], rng[1] = min(rng[0], 0), max(rng[1], 0)
            if vl.loop_order == ir.LoopOrder.PARALLEL and name in wnames and (rng[0] < 0 or rng[1] > 0):
                raise UnsupportedStencil(f"'{name}' written and read at a K offset in one PARALLEL loop")
        decl_dtype = {}
        for (name, di, dj) in win:
            decl_dtype[name] = self.st.decl(name).dtype
        for name in direct:
            decl_dtype[name] = self.st.decl(name).dtype

        def wvar(name, di, dj, d):
            rng = win[(name, di, dj)]
            return f"w{li}_{cname(name)}_{_sgn(di)}_{_sgn(dj)}_{d - rng[0]}"

        def mem_ptr(name, di, dj, kexpr):
            c = cname(name)
            return (
                f"p.p_{c} + ((int64_t)gtmi::clampi(i + ({di}), p.ilo_{c}, p.ihi_{c}) * p.sI_{c} + "
                f"(int64_t)gtmi::clampi(j + ({dj}), p.jlo_{c}, p.jhi_{c}) * p.sJ_{c} + "
                f"(int64_t)gtmi::clampi({kexpr}, p.klo_{c}, p.khi_{c}) * p.sK_{c})"
            )

        def mem_index(name, di, dj, kexpr):
            """A load expression (non-temporal for read-once streams)."""
            nt = "true" if (name in self.nt_loads and name not in direct) else "false"
            return f"gtmi::sload<{decl_dtype[name].ctype}, {nt}>({mem_ptr(name, di, dj, kexpr)})"

        def mem_store(name, kexpr, value):
            nt = "true" if (name in self.nt_stores and name not in direct) else "false"
            return f"gtmi::sstore<{decl_dtype[name].ctype}, {nt}>({mem_ptr(name, 0, 0, kexpr)}, {value});"

        P = int(self.opts.get("kprefetch", 0))
        step = "+" if fwd else "-"
        out = [f"{{  // vertical loop {li} ({order.name})"]
        for (name, di, dj), rng in win.items():
            t = decl_dtype[name].ctype
            for d in range(rng[0], rng[1] + 1):
                out.append(f"    {t} {wvar(name, di, dj, d)} = ({t})0;")
        out.append("    int k_next = -0x7fffffff;")
        front = {}
        for key, rng in win.items():
            front[key] = rng[1] if fwd else rng[0]

        def zero_needed_in(name, di, dj, sec) -> bool:
            """Is entry d == 0 of the window read at this level before an unconditional write?"""
            if not self._mem(name):
                return False
            if (di, dj) != (0, 0) or name not in wnames:
                return True
            for s in sec.body:
                for acc, w in iter_accesses([s]):
                    if acc.name == name and isinstance(acc, ir.FieldAccess) and acc.offset == (0, 0, 0):
                        if w:
                            return not isinstance(s, ir.Assign)
                        return True
            return True

        # which window fronts are loaded from memory at every level (loop-wide decision)
        front_load = {}
        for key in win:
            name, di, dj = key
            fd = front[key]
            if not self._mem(name):
                front_load[key] = False
            elif fd == 0 and name in wnames:
                front_load[key] = any(zero_needed_in(name, di, dj, sec) for sec in vl.sections)
            else:
                front_load[key] = True
        # prefetch registers: front values of the next P levels
        for key, fl in front_load.items():
            if fl:
                t = decl_dtype[key[0]].ctype
                for pp in range(1, P + 1):
                    out.append(f"    {t} pf{pp}_{wvar(*key, front[key])} = ({t})0;")

        for si, sec in enumerate(vl.sections):
            lo, hi = interval_bounds(sec.interval)
            out.append(f"    {{  // section {si}")
            out.append(f"        int ks = {lo}, ke = {hi};")
            out.append("        if (ks < 0) ks = 0; if (ke > nk) ke = nk;")
            if fwd:
                out.append("        for (int k = ks; k < ke; ++k) {")
            else:
                out.append("        for (int k = ke - 1; k >= ks; --k) {")
            body = []
            body.append("if (k != k_next) {  // (re)load the full K-window and the prefetch registers")
            for (name, di, dj), rng in win.items():
                if not self._mem(name):
                    continue
                for d in range(rng[0], rng[1] + 1):
                    if d == 0 and not zero_needed_in(name, di, dj, sec):
                        continue
                    body.append(f"    {wvar(name, di, dj, d)} = {mem_index(name, di, dj, f'k + ({d})')};")
            for key, fl in front_load.items():
                if fl:
                    fd = front[key]
                    for pp in range(1, P + 1):
                        body.append(
                            f"    pf{pp}_{wvar(*key, fd)} = {mem_index(*key, f'k {step} {pp} + ({fd})')};"
                        )
            body.append("} else {  // shift the window; its front comes from the prefetch registers")
            for key, rng in win.items():
                name, di, dj = key
                ds = list(range(rng[0], rng[1] + 1))
                if fwd:
                    for d in ds[:-1]:
                        body.append(f"    {wvar(name, di, dj, d)} = {wvar(name, di, dj, d + 1)};")
                else:
                    for d in reversed(ds[1:]):
                        body.append(f"    {wvar(name, di, dj, d)} = {wvar(name, di, dj, d - 1)};")
                if front_load[key]:
                    fd = front[key]
                    fv = wvar(name, di, dj, fd)
                    if P == 0:
                        body.append(f"    {fv} = {mem_index(name, di, dj, f'k + ({fd})')};")
                    else:
                        body.append(f"    {fv} = pf1_{fv};")
                        for pp in range(1, P):
                            body.append(f"    pf{pp}_{fv} = pf{pp + 1}_{fv};")
                        body.append(f"    pf{P}_{fv} = {mem_index(name, di, dj, f'k {step} {P} + ({fd})')};")
            body.append("}")
            body.append(f"k_next = k {step} 1;")

            def kaddr(acc: ir.FieldAccess) -> str:
                kexpr = f"k + ({acc.offset[2]})"
                if acc.k_offset is not None:
                    kexpr += f" + (int)({rend(acc.k_offset)})"
                return kexpr

            def resolve(acc: ir.FieldAccess) -> str:
                di, dj, dk = acc.offset
                if acc.name in direct:
                    return mem_index(acc.name, di, dj, kaddr(acc))
                return wvar(acc.name, di, dj, dk)

            rend = ExprRenderer(resolve, lambda n: f"s_{cname(n)}", lambda ax: ["i", "j", "k"][ax])
            self._kaddr = kaddr
            for ti, s in enumerate(sec.body):
                code = self._stmt(s, rend, wvar, mem_store)
                g = self._guard(li, si, ti)
                if g:
                    code = [f"if ({g}) {{"] + ["    " + x for x in code] + ["}"]
                body += code
            out += ["            " + x for x in body]
            out.append("        }")
            out.append("    }")
        out.append("}")
        return out

    def _stmt(self, s, rend, wvar, mem_store) -> List[str]:
        mem_index = mem_store
        if isinstance(s, ir.Assign):
            name = s.target.name
            if name in self.direct:
                st = mem_store(name, self._kaddr(s.target), rend(s.value))
                if name in self.api and any(self.ext):
                    st = f"if (i >= 0 && i < p.ni && j >= 0 && j < p.nj) {st}"
                return [st]
            tgt = wvar(name, 0, 0, 0)
            out = [f"{tgt} = {rend(s.value)};"]
            if self._mem(name):
                st = mem_store(name, "k", tgt)
                if name in self.api and any(self.ext):
                    st = f"if (i >= 0 && i < p.ni && j >= 0 && j < p.nj) {st}"
                out.append(st)
            return out
        if isinstance(s, ir.If):
            out = [f"if ({rend(s.cond)}) {{"]
            for x in s.body:
                out += ["    " + y for y in self._stmt(x, rend, wvar, mem_index)]
            if s.orelse:
                out.append("} else {")
                for x in s.orelse:
                    out += ["    " + y for y in self._stmt(x, rend, wvar, mem_index)]
            out.append("}")
            return out
        if isinstance(s, ir.While):
            out = [f"while ({rend(s.cond)}) {{"]
            for x in s.body:
                out += ["    " + y for y in self._stmt(x, rend, wvar, mem_index)]
            out.append("}")
            return out
        if isinstance(s, ir.HorizontalRegion):
            cond = region_condition(s.masks, "i", "j", "p.ni", "p.nj")
            out = [f"if ({cond}) {{"]
            for x in s.body:
                out += ["    " + y for y in self._stmt(x, rend, wvar, mem_index)]
            out.append("}")
            return out
        raise TypeError(type(s))


def _sgn(x: int) -> str:
    return f"m{-x}" if x < 0 else f"p{x}"


# ------------------------------------------------------------------------------------------
# translation unit
# ------------------------------------------------------------------------------------------


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
        "abi": 2,
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
    n_scalars = len(st.scalar_params())
    host_scalars = [
        f"    {sp.dtype.ctype} hs_{cname(sp.name)}; memcpy(&hs_{cname(sp.name)}, &sc[{i}], sizeof(hs_{cname(sp.name)})); "
        f"(void)hs_{cname(sp.name)};"
        for i, sp in enumerate(st.scalar_params())
    ]
    src = f"""// Generated by gt4py_amd (gt:mi355x). Do not edit.
#include "gtmi_device.h"
#include "gtmi.h"
#include <string.h>
#include <stdio.h>

static thread_local char g_gtmi_err[512];
static void gtmi_set_error(const char* msg) {{ snprintf(g_gtmi_err, sizeof(g_gtmi_err), "%s", msg); }}

{chr(10).join(kernels_src)}

extern "C" const char* gtmi_last_error(void) {{ return g_gtmi_err; }}
extern "C" int gtmi_abi_version(void) {{ return GTMI_ABI_VERSION; }}
extern "C" const char* gtmi_stencil_signature(void) {{ return "{sig_json}"; }}

extern "C" int gtmi_stencil_run(const int64_t* domain, const gtmi_field* f, int32_t n_fields,
                                const gtmi_scalar* sc, int32_t n_scalars, void* stream_ptr) {{
    g_gtmi_err[0] = 0;
    if (n_fields != {n_fields} || n_scalars != {n_scalars}) {{
        snprintf(g_gtmi_err, sizeof(g_gtmi_err), "expected {n_fields} fields / {n_scalars} scalars, got %d / %d",
                 (int)n_fields, (int)n_scalars);
        return 1;
    }}
    (void)sc; (void)f;
    hipStream_t stream = (hipStream_t)stream_ptr;
    const int ni = (int)domain[0], nj = (int)domain[1], nk = (int)domain[2];
    (void)ni; (void)nj; (void)nk;
{chr(10).join(host_scalars)}
{chr(10).join("    " + line for h in launches for line in h.splitlines())}
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {{
        snprintf(g_gtmi_err, sizeof(g_gtmi_err), "HIP launch failed: %s", hipGetErrorString(err));
        return (int)err;
    }}
    return 0;
}}
"""
    return src, signature
