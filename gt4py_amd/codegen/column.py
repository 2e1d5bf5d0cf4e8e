"""K2 -- the column kernel generator (FORWARD/BACKWARD sweeps, K-windows in registers).

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
    COLUMN_BLOCK, PLANE_BLOCK_WAVES, WAVE, ExprRenderer, FieldSlot, cname, host_fill, interval_bounds, kparam_decl,
    literal, region_condition,
)

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

    def _block(self) -> Tuple[int, int]:
        """Threads per block in I and J (option ``col_bx``: I width, 256 threads in total)."""
        bx = int(self.opts.get("col_bx", COLUMN_BLOCK[0]))
        if bx not in (64, 128, 256):
            raise ValueError(f"col_bx must be 64, 128 or 256, got {bx}")
        return bx, (COLUMN_BLOCK[0] * COLUMN_BLOCK[1]) // bx

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
        bx, by = self._block()
        L.append(f"__global__ void __launch_bounds__({bx * by}) k{k}_column(const K{k}Params p) {{")
        if int(self.opts.get("col_occupancy", 0)) > 0:
            L.append("    extern __shared__ __attribute__((aligned(16))) char gtmi_lds_reserve[];")
            L.append("    if (p.ni < 0) gtmi_lds_reserve[threadIdx.x] = 0;  // keep the reservation alive")
        B = []
        eilo, eihi, ejlo, ejhi = self.ext
        if int(self.opts.get("col_order", 0)) == 1:
            # XCD-aware: consecutive column blocks (along I, then J) run on one XCD (8 XCDs, round-robin dispatch)
            B.append("const int nbx = (int)gridDim.x, nb = nbx * (int)gridDim.y;")
            B.append("const int b = (int)(blockIdx.y * gridDim.x + blockIdx.x);")
            B.append("const int q = nb >> 3, r = nb & 7, xcd = b & 7, slot = b >> 3;")
            B.append("const int w = (xcd < r) ? xcd * (q + 1) + slot : r * (q + 1) + (xcd - r) * q + slot;")
            B.append(f"const int i = (w % nbx) * {bx} + (int)threadIdx.x - {eilo};")
            B.append(f"const int j = (w / nbx) * {by} + (int)threadIdx.y - {ejlo};")
        else:
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
        bx, by = self._block()
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
                if any(_parallel_k_race(sec, name) for sec in vl.sections):
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
        U = int(self.opts.get("kblock", 0))
        if U > 1:
            P = 0  # blocked loads replace the rotating prefetch registers
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

            def level_body(u: Optional[int]) -> List[str]:
                """One level: window (re)load or shift, then the statements. ``u``: the level's
                slot in a block of ``U`` levels whose window fronts were loaded together."""
                body = ["if (k != k_next) {  // (re)load the full K-window and the prefetch registers"]
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
                        if u is not None:
                            body.append(f"    {fv} = bf{u}_{fv};")
                        elif P == 0:
                            body.append(f"    {fv} = {mem_index(name, di, dj, f'k + ({fd})')};")
                        else:
                            body.append(f"    {fv} = pf1_{fv};")
                            for pp in range(1, P):
                                body.append(f"    pf{pp}_{fv} = pf{pp + 1}_{fv};")
                            body.append(f"    pf{P}_{fv} = {mem_index(name, di, dj, f'k {step} {P} + ({fd})')};")
                body.append("}")
                body.append(f"k_next = k {step} 1;")
                for ti, s in enumerate(sec.body):
                    code = self._stmt(s, rend, wvar, mem_store)
                    g = self._guard(li, si, ti)
                    if g:
                        code = [f"if ({g}) {{"] + ["    " + x for x in code] + ["}"]
                    body += code
                return body

            if U > 1:
                # blocked K loads: the window fronts of U levels are issued together (U independent
                # loads per stream in flight per wave), then the U levels are computed in order;
                # levels past the section end re-read its last level (a cache hit, no extra HBM bytes)
                if fwd:
                    out.append(f"        for (int kb = ks; kb < ke; kb += {U}) {{")
                else:
                    out.append(f"        for (int kb = ke - 1; kb >= ks; kb -= {U}) {{")
                for key, fl in front_load.items():
                    if not fl:
                        continue
                    fd = front[key]
                    fv = wvar(*key, fd)
                    t = decl_dtype[key[0]].ctype
                    for u in range(U):
                        kl = f"min(kb + {u}, ke - 1)" if fwd else f"max(kb - {u}, ks)"
                        out.append(f"            const {t} bf{u}_{fv} = {mem_index(*key, f'{kl} + ({fd})')};")
                for u in range(U):
                    cond = f"k < ke" if fwd else "k >= ks"
                    out.append(f"            {{  // level kb {step} {u}")
                    out.append(f"                const int k = kb {step} {u};")
                    out.append(f"                if ({cond}) {{")
                    out += ["                    " + x for x in level_body(u)]
                    out.append("                }")
                    out.append("            }")
                out.append("        }")
            else:
                if fwd:
                    out.append("        for (int k = ks; k < ke; ++k) {")
                else:
                    out.append("        for (int k = ke - 1; k >= ks; --k) {")
                out += ["            " + x for x in level_body(None)]
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


def _parallel_k_race(sec: ir.Section, name: str) -> bool:
    """``name`` written and read at a K offset in a PARALLEL section of more than one static
    level. A one-level section (``interval(0, 1)``, ``interval(-1, None)``) has no race: it
    writes its own level only (``gtc/gtir.py:252-262``), so the column sweep may run it."""
    iv = sec.interval
    if iv.start.level == iv.end.level and abs(iv.end.offset - iv.start.offset) == 1:
        return False
    writes = reads = False
    for acc, w in iter_accesses(sec.body):
        if isinstance(acc, ir.FieldAccess) and acc.name == name:
            writes |= w
            reads |= (not w) and acc.offset[2] != 0
    return writes and reads


def _sgn(x: int) -> str:
    return f"m{-x}" if x < 0 else f"p{x}"
