"""K1 -- the J-streaming plane kernel generator (PARALLEL sections with IJ offsets).

See ``codegen/hip.py`` for the skeleton's description and DESIGN.md §3.
"""

from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional, Set, Tuple

from gt4py_amd import ir
from gt4py_amd.codegen.plan import ColumnKernel, KernelPlan, PlaneKernel, UnsupportedStencil
from gt4py_amd.ir import DataType
from gt4py_amd.passes import ZERO_EXTENT, StencilAnalysis, iter_accesses
from gt4py_amd.codegen.common import (  # noqa: F401
    COLUMN_BLOCK, PLANE_BLOCK_WAVES, PLANE_LVLSYNC_MAX_LEVELS, PLANE_LVLSYNC_MAX_PLANE, PLANE_MIN_JCHUNK, PLANE_ORDER_AUTO, PLANE_TARGET_BLOCKS, WAVE, ExprRenderer, FieldSlot, cname,
    host_fill, interval_bounds, kparam_decl, literal, region_condition,
)

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
    def __init__(self, analysis: StencilAnalysis, plan: KernelPlan, kernel: PlaneKernel, slots, kid: int, opts,
                 mirror: bool = False):
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
        # mirror=True generates the same section streamed in -J (the rows of a chunk visited
        # top-down): J offsets are negated, J extents swapped, and local row u is row jb + jce - 1 - u
        self.mirror = mirror
        self.body = ir.map_expr(self.sec.body, _negate_dj) if mirror else self.sec.body
        self.stage_ext = []
        for ti in range(len(self.sec.body)):
            (ilo, ihi), (jlo, jhi) = analysis.extents.blocks[(kernel.loop, kernel.section, ti)]
            self.stage_ext.append(((ilo, ihi), (jhi, jlo) if mirror else (jlo, jhi)))

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
        for ti, stmt in enumerate(self.body):
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
        if int(self.opts.get("nt_load", 1)) == 2:  # experiment: every load non-temporal
            return True
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
        mirrored = None
        if self._mirror_pays():
            mirrored = PlaneGen(self.a, self.plan, self.kernel, self.slots, self.kid, self.opts, mirror=True).build()
        srcs = []
        launches = {}
        for V in variants:
            self.geometry(V)
            if mirrored is not None:
                mirrored.geometry(V)
                assert (mirrored.h_lo, mirrored.w_out) == (self.h_lo, self.w_out)
            src, launch = self._render_variant(V, mirrored)
            srcs.append(src)
            launches[V] = launch
        return "\n\n".join(srcs), self._render_host(launches)

    def _mirror_pays(self) -> bool:
        """Stream odd J chunks top-down (option ``jmirror``, default on).

        Two chunks that meet at a boundary then read the rows they share (the J halo of the
        section, ``needed_lo + lead`` rows) at the same time -- both at the start or both at the
        end of their sweep -- so the second read hits the XCD's L2 instead of HBM. Chunks of one
        level are consecutive work items on one XCD (XCD-aware order), i.e. they run together.
        """
        if not int(self.opts.get("jmirror", 1)) or self.mirror:
            return False
        if any(n in self.scratch for n in self.current):
            return False  # scratch stores extend into the J halo of the edge chunks
        return any(isinstance(n, ir.FieldAccess) and n.offset[1] != 0 for n in ir.walk(self.sec.body))

    def _row(self, local: str) -> str:
        """Grid row of local row ``local`` of the chunk (``t + lead``)."""
        return f"(jb + jce - 1 - ({local}))" if self.mirror else f"(jb + ({local}))"

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

    def _render_variant(self, V: int, mirrored: Optional["PlaneGen"] = None) -> Tuple[str, dict]:
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
            L.append("    int32_t ni, nj, nk, k0, nks, jc, n_strips, n_chunks, n_sgroups, perm_a, jsplit, jskip, ca, lvlsync;")
            L.append("};")
            L.append("")
        kname = f"k{k}_plane_v{V}"
        mb = int(self.opts.get("min_blocks", 0))  # blocks per CU the register budget must allow
        lb = f"{WAVE * PLANE_BLOCK_WAVES}, {mb}" if mb > 0 else f"{WAVE * PLANE_BLOCK_WAVES}"
        L.append(f"__global__ void __launch_bounds__({lb}) {kname}(const K{k}Params p) {{")
        B = []
        B.append("const int lane = (int)__lane_id();")
        B.append("const int wave = (int)(threadIdx.x >> 6);")
        order = int(self.opts.get("order", PLANE_ORDER_AUTO))
        B.append("const int nb = (int)gridDim.x, b = (int)blockIdx.x;")

        def lvlsync():
            # level-synchronous XCD-aware order: every level's work items are cut into 8 contiguous
            # ranges, one per XCD (blocks are dispatched round-robin over the XCDs), so all XCDs
            # stream the same few levels at a time while each keeps its neighbours in its own L2
            return [
                "const int per_lvl = p.n_sgroups * p.n_chunks, m8 = (per_lvl + 7) >> 3;",
                "const int lvl = b / (m8 * 8), loc = b - lvl * m8 * 8;",
                "const int w = (loc & 7) * m8 + (loc >> 3);",
                "if (w >= per_lvl) return;  // padding block (whole workgroup)",
                "sg = w % p.n_sgroups;",
                "chunk = w / p.n_sgroups;",
                "kk = p.k0 + lvl;",
            ]

        def xcd_ranges(o):
            L2 = [
                "// XCD-aware block remap: consecutive work items share an XCD (8 XCDs, round-robin dispatch)",
                "const int q = nb >> 3, r = nb & 7, xcd = b & 7, slot = b >> 3;",
                "const int w0x = (xcd < r) ? xcd * (q + 1) + slot : r * (q + 1) + (xcd - r) * q + slot;",
            ]
            if o == 3:
                L2 = ["const int w = b;  // natural dispatch order"]
            elif o == 2:
                L2.append("const int w = (int)(((long long)w0x * p.perm_a) % nb);  // bijective scatter")
            else:
                L2.append("const int w = w0x;")
            if o == 4:  # chunks slowest: chunk c+1 starts as chunk c ends on the same XCD (halo rows warm)
                L2 += ["sg = w % p.n_sgroups;", "const int rest = w / p.n_sgroups;", "kk = p.k0 + rest % p.nks;",
                       "chunk = rest / p.nks;"]
            elif o == 1:
                L2 += ["kk = p.k0 + w % p.nks;", "const int rest = w / p.nks;", "sg = rest % p.n_sgroups;",
                       "chunk = rest / p.n_sgroups;"]
            else:
                L2 += ["sg = w % p.n_sgroups;", "const int rest = w / p.n_sgroups;", "chunk = rest % p.n_chunks;",
                       "kk = p.k0 + rest / p.n_chunks;"]
            return L2

        B.append("int sg, chunk, kk;")
        if order == 5:
            B.append("{")
            B += ["    " + x for x in lvlsync()]
            B.append("}")
        elif order == PLANE_ORDER_AUTO:
            # chosen per launch by the host (p.lvlsync, see _render_host): uniform branch
            B.append("if (p.lvlsync) {")
            B += ["    " + x for x in lvlsync()]
            B.append("} else {")
            B += ["    " + x for x in xcd_ranges(0)]
            B.append("}")
        else:
            B.append("{")
            B += ["    " + x for x in xcd_ranges(order)]
            B.append("}")
        B.append(f"const int strip = sg * {PLANE_BLOCK_WAVES} + wave;")
        B.append("if (strip >= p.n_strips) return;")
        B.append(f"const int ib = strip * {self.w_out};")
        # rows [0, jsplit) and [jsplit + jskip, nj): chunks never straddle the gap (jsplit = nj and
        # jskip = 0 for an ordinary call, gtmi_stencil_run_jsplit otherwise)
        B.append("const int jb = chunk < p.ca ? chunk * p.jc : p.jsplit + p.jskip + (chunk - p.ca) * p.jc;")
        B.append("const int jce = min(p.jc, (chunk < p.ca ? p.jsplit : p.nj) - jb);")
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
        if mirrored is None:
            B += self._render_body(V, P)
        else:  # wave-uniform branch: odd chunks stream top-down
            B.append("if ((chunk & 1) == 0) {")
            B += ["    " + x for x in self._render_body(V, P)]
            B.append("} else {")
            B += ["    " + x for x in mirrored._render_body(V, P)]
            B.append("}")
        L += ["    " + x for x in B]
        L.append("}")
        geo = {"w_out": self.w_out, "V": V, "kname": kname, "used": used_slots}
        return "\n".join(L), geo

    def _bufld_ok(self, V: int) -> bool:
        """Row loads through buffer descriptors (option ``bufld``): 16- or 8-B lanes of 4/8-B types."""
        mode = int(self.opts.get("bufld", -1))
        if mode < 0:
            # auto: 4-byte lanes (4 cells per lane). hdiff f32 8192x1024x160: +4..+11 % on every
            # one of 24 HBM placements, bit-identical; hdiff f64 (2 cells per lane): -0.5 %
            # (profiles/r03/r03c_bufld_ab_*.jsonl)
            mode = 1 if V >= 4 else 0
        if V < 2 or not mode or not self.loads:
            return False
        stored = [n for n in self.current if self._mem_backed(n)]
        if any(n in self.scratch for n in stored):
            return False  # scratch stores cover the extent halo (edge-dependent conditions)
        sizes = [v.dtype.itemsize for v in self.loads.values()] + [self.st.decl(n).dtype.itemsize for n in stored]
        return all(x >= 4 and V * x in (8, 16) for x in sizes)

    def _bufld_interior(self, V: int) -> str:
        """Wave-uniform condition under which every lane that needs a loaded value finds its whole
        vector inside the field's I range (all strips but the first and the last, typically)."""
        conds = []
        for v in self.loads.values():
            lo, hi = self._lane_range(v)
            c = cname(v.name)
            conds.append(f"(w0 + {lo * V} >= p.ilo_{c}) && (w0 + {hi * V + V - 1} <= p.ihi_{c})")
        # stores: the whole output strip inside the domain (every owned lane owns its whole vector:
        # h_lo and w_out are multiples of V)
        conds.append(f"(ib + {self.w_out} <= p.ni)")
        return " && ".join(conds)

    def _render_body(self, V: int, P: int) -> List[str]:
        """Register rings, prefetch and the row loop of one J direction; with ``bufld`` the row
        loop exists twice behind a wave-uniform branch: interior strips load every row through a
        buffer descriptor (no branches around the loads), edge strips keep the clamped loads."""
        if not self._bufld_ok(V):
            return self._render_body_v(V, P)
        B = [f"const bool bl_ok = __builtin_amdgcn_readfirstlane((int)({self._bufld_interior(V)})) != 0;",
             "if (bl_ok) {"]
        B += ["    " + x for x in self._render_body_slots(V, P)]
        B.append("} else {")
        B += ["    " + x for x in self._render_body_v(V, P)]
        B.append("}")
        return B

    def _emit_bload(self, v: Val, row_expr: str, dests: List[str], rcond: str) -> List[str]:
        """Unconditional row load: an invalid row gets a zero-record descriptor (no traffic), so
        every row step issues the same loads and hipcc counts them exactly (vmcnt(N) instead of
        vmcnt(0)), i.e. the prefetched rows really stay in flight."""
        V = self.V
        c = cname(v.name)
        kexpr = f"kk + ({v.dk})" if v.dk else "kk"
        nt = "true" if self._nt_load(v) else "false"
        t = v.dtype.ctype
        return [
            "{",
            f"    const int64_t ro = (int64_t)gtmi::clampi({row_expr}, p.jlo_{c}, p.jhi_{c}) * p.sJ_{c} + "
            f"(int64_t)gtmi::clampi({kexpr}, p.klo_{c}, p.khi_{c}) * p.sK_{c};",
            f"    const __amdgpu_buffer_rsrc_t rs = gtmi::row_rsrc(p.p_{c} + ro + p.ilo_{c}, ({rcond}) ? nr_{v.c} : 0);",
            f"    {t} tmp[{V}];",
            f"    gtmi::bload<{t}, {V}, {nt}>(rs, bo_{v.c}, tmp);",
        ] + [f"    {dests[e]} = tmp[{e}];" for e in range(V)] + ["}"]

    def _render_body_slots(self, V: int, P: int) -> List[str]:
        """Row loop of an interior strip with buffer-descriptor loads and slot rings.

        Every loaded value (field, K offset) keeps the rows it still needs -- the J ring of the
        section (``depth`` rows) plus the rows in flight (``P_v``) -- in ONE ring of ``R_v``
        register slots (``R_v`` divides ``U = max(depth) + P``), ``P_v = R_v - depth_v``; the loop
        is unrolled ``U`` times, so copy ``u`` reads ring position ``a`` from slot
        ``(u - a) mod R_v`` and loads row ``t + P_v`` into slot ``(u + P_v) mod R_v``, the slot
        its oldest row just left. No load
        result is ever moved (a move of a row in flight would make hipcc wait for it), every
        copy issues the same unconditional loads, and the waits count them exactly: each wave
        keeps ``P_v`` rows of every stream in flight.
        """
        loads = list(self.loads.values())
        U = max(v.depth for v in loads) + max(1, P)
        # ring size per value: the smallest divisor of U that holds its J ring plus at least
        # P - 1 rows in flight (U itself for the deepest ring): shallow streams (coeff) do not
        # pay U - 1 rows of registers
        ring: Dict[int, int] = {}
        for v in loads:
            need = v.depth + max(1, P - 1)
            ring[v.vid] = U if v.depth + max(1, P) >= U else min(d for d in range(1, U + 1) if U % d == 0 and d >= need)
        B = []
        for v in self.vals:  # rings of computed values (moves between VALU results only)
            if v.kind in ("undef", "load"):
                continue
            for a in range(v.depth):
                for e in range(V):
                    B.append(f"{v.dtype.ctype} {v.c}_{a}_{e} = ({v.dtype.ctype})0;")
        for v in loads:
            lo, hi = self._lane_range(v)
            c = cname(v.name)
            # byte offset of the lane's vector from the row's first element; lanes that do not
            # need the value point past the descriptor's range (the load returns 0, no traffic)
            B.append(f"const int32_t bo_{v.c} = ((lane >= {lo}) && (lane <= {hi})) ? (pos - p.ilo_{c}) * "
                     f"{v.dtype.itemsize} : (int32_t)0x40000000;")
            B.append(f"const int32_t nr_{v.c} = (p.ihi_{c} - p.ilo_{c} + 1) * {v.dtype.itemsize};")
            for k in range(ring[v.vid]):
                for e in range(V):
                    B.append(f"{v.dtype.ctype} sl{k}_{v.c}_{e} = ({v.dtype.ctype})0;")
        # prologue: rows t_start .. t_start + P_v - 1 into slots 0 .. P_v - 1
        for v in loads:
            first = -(v.needed_lo + v.lead)
            pv = ring[v.vid] - v.depth
            for k in range(pv):
                rcond = f"{self.t_start + k} >= {first} && {self.t_start + k} < jce"
                B += self._emit_bload(v, self._row(f"({self.t_start + k}) + ({v.lead})"),
                                      [f"sl{k}_{v.c}_{e}" for e in range(V)], rcond)
        # the row loop must not inherit pending prologue loads: at the loop header hipcc merges
        # the entry state with the back edge, and a prologue load still in flight there would
        # pin the loop's waits to the prologue's registers
        B.append("__builtin_amdgcn_s_waitcnt(0);  // prologue rows landed")
        B.append(f"for (int tt = {self.t_start}; ; tt += {U}) {{")
        for u in range(U):
            S = []
            for v in loads:
                first = -(v.needed_lo + v.lead)
                R = ring[v.vid]
                pv = R - v.depth
                for a in range(v.depth):
                    for e in range(V):
                        S.append(f"const {v.dtype.ctype} {v.c}_{a}_{e} = sl{(u - a) % R}_{v.c}_{e};")
                rcond = f"t + {pv} >= {first} && t + {pv} < jce"
                S += self._emit_bload(v, self._row(f"t + {pv} + ({v.lead})"),
                                      [f"sl{(u + pv) % R}_{v.c}_{e}" for e in range(V)], rcond)
            for ti, code in enumerate(self.stage_code):
                lead = self.stage_ext[ti][1][1]
                S.append(f"{{  // stage {ti}: row t + {lead}")
                S += ["    " + x for x in self._render_stage(ti, code, lead)]
                S.append("}")
            S += self._render_stores_buf()
            for v in self.vals:
                if v.kind in ("undef", "load"):
                    continue
                for a in range(v.depth - 1, 0, -1):
                    for e in range(V):
                        S.append(f"{v.c}_{a}_{e} = {v.c}_{a - 1}_{e};")
            B.append(f"    {{  // slot copy {u}")
            B.append(f"        const int t = tt + {u};")
            B.append("        if (t >= jce) break;")
            B += ["        " + x for x in S]
            B.append("    }")
        B.append("}")
        return B

    def _render_body_v(self, V: int, P: int) -> List[str]:
        B = []
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
                rcond = f"{self.t_start + pp} >= {first} && {self.t_start + pp} < jce"
                row = self._row(f"({self.t_start + pp}) + ({v.lead})")
                dests = [f"pf{pp}_{v.c}_{e}" for e in range(V)]
                B.append(f"if ({rcond})")
                B += ["    " + x for x in emit_load(v, row, dests)]
        # row_unroll=U: U copies of the row step per loop trip, each leaving the loop on its own
        # (uniform) bound check, so the ring rotations between copies become register renames.
        # Auto (-1, default): 4 when the rings and prefetch buffers hold <= 40 32-bit words per
        # lane (lap5: 32 words, +3 %; copy: neutral); kernels with more state lose occupancy
        # (hdiff f64 80 words: -2.4 % at U=6; profiles/r02za_sweep_row_unroll*.log).
        row_unroll = int(self.opts.get("row_unroll", -1))
        if row_unroll < 0:
            words = sum(v.depth * V * max(1, v.dtype.itemsize // 4) for v in self.vals if v.kind != "undef")
            words += sum(P * V * max(1, v.dtype.itemsize // 4) for v in loads)
            if V == 1:
                row_unroll = 0  # the 1-wide fallback stays rolled
            elif words <= 40:
                row_unroll = 4
            else:
                # 4 cells per lane (f32): 2x (+0.7 %, +3.5 % on two boxes); 2 cells per lane
                # (f64 hdiff): 2x/3x cost 3-4 % (profiles/r02za_sweep_row_unroll3.log)
                row_unroll = 2 if V >= 4 else 0
        if row_unroll > 1:
            B.append(f"for (int tt = {self.t_start}; ; tt += {row_unroll}) {{")
        else:
            B.append(f"for (int t = {self.t_start}; t < jce; ++t) {{")
        def step_code(u: int) -> List[str]:
            S = []
            for v in loads:
                first = -(v.needed_lo + v.lead)
                if P == 0:
                    S.append(f"if (t >= {first})")
                    S += ["    " + x for x in emit_load(v, self._row(f"t + ({v.lead})"),
                                                       [f"{v.c}_0_{e}" for e in range(V)])]
                    continue
                rcond = f"t + {P} >= {first} && t + {P} < jce"
                row = self._row(f"t + {P} + ({v.lead})")
                for e in range(V):
                    S.append(f"{v.c}_0_{e} = pf0_{v.c}_{e};")
                for pp in range(P - 1):
                    for e in range(V):
                        S.append(f"pf{pp}_{v.c}_{e} = pf{pp + 1}_{v.c}_{e};")
                dests = [f"pf{P - 1}_{v.c}_{e}" for e in range(V)]
                S.append(f"if ({rcond})")
                S += ["    " + x for x in emit_load(v, row, dests)]
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
            return S

        if row_unroll > 1:
            for u in range(row_unroll):
                B.append(f"    {{  // row copy {u}")
                B.append(f"        const int t = tt + {u};")
                B.append("        if (t >= jce) break;")
                B += ["        " + x for x in step_code(u)]
                B.append("    }")
        else:
            B += ["    " + x for x in step_code(0)]
        B.append("}")
        return B

    def _render_stores_buf(self) -> List[str]:
        """Stores of an interior strip: one unconditional buffer store per field and row; rows
        outside the chunk get a zero-record descriptor, lanes outside the output strip an
        offset past it (both dropped by the range check), so no branch surrounds a store."""
        V = self.V
        S = []
        for name, v in self.current.items():
            if not self._mem_backed(name):
                continue
            c = cname(name)
            isz = self.st.decl(name).dtype.itemsize
            t = v.dtype.ctype
            row = self._row(f"t + ({v.lead})")
            nts = "true" if self.opts.get("nt_store", 1) else "false"
            S.append("{")
            S.append(f"    const int64_t ro = (int64_t)({row}) * p.sJ_{c} + (int64_t)kk * p.sK_{c};")
            S.append(f"    const bool rv = (t + ({v.lead}) >= 0) && (t + ({v.lead}) < jce);")
            S.append(f"    const __amdgpu_buffer_rsrc_t rs = gtmi::row_rsrc(p.p_{c} + ro + p.ilo_{c}, "
                     f"rv ? (p.ihi_{c} - p.ilo_{c} + 1) * {isz} : 0);")
            S.append(f"    const {t} tmp[{V}] = {{{', '.join(f'{v.c}_0_{e}' for e in range(V))}}};")
            S.append(f"    gtmi::bstore<{t}, {V}, {nts}>(rs, own_0 ? (pos - p.ilo_{c}) * {isz} : (int32_t)0x40000000, tmp);")
            S.append("}")
        return S

    def _render_stores(self) -> List[str]:
        V = self.V
        S = []
        for name, v in self.current.items():
            if not self._mem_backed(name):
                continue
            c = cname(name)
            row = self._row(f"t + ({v.lead})")
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
        H.append("        p.ni = ni; p.nj = nj; p.nk = nk; p.k0 = k0; p.nks = k1 - k0; p.jsplit = jsplit; p.jskip = jskip;")
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
                    f"            while (p.jc > {PLANE_MIN_JCHUNK} && (long long)p.n_sgroups * ((nj - jskip + p.jc - 1) / p.jc) * "
                    f"p.nks < {PLANE_TARGET_BLOCKS}LL) p.jc >>= 1;"
                )
            H.append("            p.ca = (jsplit + p.jc - 1) / p.jc;  // chunks of the first row range")
            H.append("            p.n_chunks = p.ca + (nj - jsplit - jskip + p.jc - 1) / p.jc;")
            order = int(self.opts.get("order", PLANE_ORDER_AUTO))
            if order == PLANE_ORDER_AUTO:
                # level-synchronous order for small launches: measured faster for planes of <= 1M
                # cells over <= 80 levels (lap5 1024^2x80 +3.5 %, copy 1024^2x80 +4.6 %), slower or
                # mixed beyond (hdiff 2048^2x80 -1 %, lap5 2048^2x80 -0.4 %, copy 1024^2x160 -1.3 to
                # +2.5 %, hdiff 2048^2x160 -1 to -8.5 %): profiles/r02z_sweep_order_shapes.log
                H.append(
                    f"            p.lvlsync = ((long long)ni * nj <= {PLANE_LVLSYNC_MAX_PLANE}LL && p.nks <= "
                    f"{PLANE_LVLSYNC_MAX_LEVELS}) ? 1 : 0;"
                )
            else:
                H.append(f"            p.lvlsync = {1 if order == 5 else 0};")
            H.append("            const long long nblocks = p.lvlsync  // per level: padded to a multiple of the 8 XCDs")
            H.append("                ? (long long)(((p.n_sgroups * p.n_chunks + 7) >> 3) * 8) * p.nks")
            H.append("                : (long long)p.n_sgroups * p.n_chunks * p.nks;")
            H.append("            if (nblocks > 0x7fffffffLL) { gtmi_set_error(\"grid too large\"); GTMI_RANGE_POP(); return 2; }")
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
                    if int(self.opts.get("dpp", 1)):  # DPP wave rotate for +-1 lanes (gtmi_device.h)
                        out.append(f"const {ref.val.dtype.ctype} {nm} = gtmi::shfl_c<{qd}>({ref.val.c}_{slot}_{r});")
                    else:
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
            rend.exact_fma = bool(int(self.opts.get("exact_fma", 1)))
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
            return [f"i_{e}", self._row(f"t + ({lead})"), "kk"][axis]

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
            cond = region_condition(s.masks, f"i_{e}", self._row(f"t + ({lead})"), "p.ni", "p.nj")
            out = [f"if ({cond}) {{"]
            for x in s.body:
                out += ["    " + y for y in self._stmt(x, rend, e, lead)]
            out.append("}")
            return out
        raise TypeError(type(s))


def _negate_dj(x):
    if isinstance(x, ir.FieldAccess) and x.offset[1]:
        return dataclasses.replace(x, offset=(x.offset[0], -x.offset[1], x.offset[2]))
    return x


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
