"""K2 -- the column kernel generator (FORWARD/BACKWARD sweeps, K-windows in registers).

One thread per (i, j) column, 64 x 4 threads per block; the thread walks the levels of each
vertical loop of the kernel in loop order. See ``codegen/hip.py`` and DESIGN.md §3.

* **K-windows** -- every accessed ``(name, di, dj)`` has a register window over the K offsets
  it is read at (the register-carried K-cache of the reference's ``KCacheDetection``,
  ``gtc/passes/oir_optimizations/caches.py:92``): a level loads only the window *front*.
* **Load ring** -- the fronts of the next ``kring`` levels are in flight at any time: each
  section runs in blocks of ``kring`` levels unrolled over statically indexed ring slots
  (slot ``u`` holds the front of level ``kb + u``); after level ``k`` computes, its slot is
  refilled with level ``k + kring``. Fronts never alias a pending write: a loop writes a
  field only at its own level, and fronts lie ahead of the sweep.
* **Sweep-to-sweep tail cache** -- when a FORWARD (or PARALLEL) loop is followed in the same
  kernel by a BACKWARD loop (or the reverse) that reads, at ``(0, 0)``, fields the first loop
  holds in its windows (the Thomas solve's ``c'``/``d'``: ``sup``/``rhs``; vadv's ``ccol``,
  ``dcol``, ``u_pos``), the values of the LAST ``L`` levels of the first sweep -- the FIRST
  levels of the second -- are kept in LDS, so the second sweep re-reads only the remaining
  ``nk - L`` levels from HBM. The reference's ``gt:gpu`` re-reads every level there (its
  backward multistage k-caches only the field it writes). ``L`` = LDS budget / (256 threads x
  cached bytes per level), capped at ``nk``; scratch temporaries only these two loops use are
  not written to memory at the cached levels at all.
"""

from __future__ import annotations

import dataclasses
import re
from typing import Dict, List, Optional, Set, Tuple

from gt4py_amd import ir
from gt4py_amd.codegen.plan import ColumnKernel, KernelPlan, UnsupportedStencil, sections_contiguous
from gt4py_amd.passes import StencilAnalysis, iter_accesses
from gt4py_amd.codegen.common import (  # noqa: F401
    COLUMN_BLOCK, ExprRenderer, FieldSlot, cname, host_fill, interval_bounds, kparam_decl, region_condition,
)

LDS_BYTES = 160 * 1024  # per CU (MI355X_MICROARCH.md); one 256-thread block may take all of it
DEFAULT_RING = 8
# register band levels (option ``kreg``; -1 = auto, see ColumnGen._plan_register_band)
DEFAULT_KREG = -1
AUTO_KREG = 96  # write-free scratch tails
AUTO_KREG_API = 48  # tails of API outputs
AUTO_KREG_API_PF = 6
# register band fronts prefetched across section and writer/reader boundaries, BAND_PF_OVER_RING
# levels beyond the ring depth: vadv 1024^2x160 1.763 ms against 1.800-1.810 (pf 10 per section) and
# 1.791 (pf 12 per section, the round-4 default, which spilled 9 registers); span pf 8 1.780,
# pf 12 1.791; tridiag -0.3 % (profiles/r04/r04n_sweep_*_span_*.log). Measured and removed in
# round 5: the per-section prefetch, deeper prefetch for light loops (kpf_adapt),
# I-neighbour lane shifts (nbr_shfl) and split cached/uncached writer segments (seg_tail).
BAND_PF_OVER_RING = 2
DEFAULT_TAIL_HEAD = -1  # auto: see ColumnGen._plan_tail
# tile mode: J rows of threads per block, halo included (option ``tile_by``; -1 = auto: 16 rows as
# one 1024-thread block when the tile's J halo is a single row and its cells are 8 bytes, else 8).
# A one-row halo costs a tile 1/8 of its rows at 8 and 1/16 at 16; with halo rows on both sides the
# 1024-thread block's 128-VGPR cap costs more than the halved re-read saves (profiles/r05/
# r05e_tile_probe.log, r05l_*: fwd_recurrence -4 %, staged -2.8 %; two_phase_chain, bwd_recurrence
# and tile_f32 +1.5-4 % at 16)
TILE_BY = -1
# tile mode: levels per LDS barrier in the steady-state loop (a level's statements after the barrier
# wait for the next level's before it; planes rotate over 2 x TILE_LBLOCK buffers). Every tile
# program at 1024^2x80 (profiles/r05/r05l_tile_probe.log): tile_f32 -6 %, bwd_recurrence -1.8 %,
# scratch_product -0.8 %, staged -0.6 %, the rest within +-0.4 %; kernels where no loop can be
# blocked keep two planes and one barrier per level.
TILE_LBLOCK = 2
# tile mode: J rows per thread (option ``tile_rows``): 2 makes a block of bx x by threads cover
# 2 x by rows, each thread carrying the state of two columns (the second one by rows further down,
# its code the first row's with the per-column names renamed), so 128 x 8 threads can hold a
# 112 x 15 tile -- the only way past the 1024-thread cap to a tile both wide and tall
TILE_ROWS = 1
_ROW1 = re.compile(r"\b(w\d+_\w+|rg\d+_\w+|cb_\w+|sn\d+_\w+|j|ty|alive|own)\b")


def _row1(line: str) -> str:
    """Tile mode, a thread's second row: the same code on its own column state (window, ring and
    snapshot registers, column bases, j, ty, alive and own renamed)."""
    return _ROW1.sub(r"\1_r1", line)
_KVAR = re.compile(r"\bk\b")
_WVAR = re.compile(r"\bw\d+_\w+")
_WASSIGN = re.compile(r"^\s*(w\d+_\w+) = ")
_CBVAR = re.compile(r"\bcb_\w+")


@dataclasses.dataclass
class _LoopInfo:
    fwd: bool
    direct: Set[str]
    win: Dict[Tuple[str, int, int], List[int]]  # (name, di, dj) -> [dmin, dmax]
    wnames: Set[str]  # window names written in the loop


@dataclasses.dataclass
class _Tail:
    """LDS tail cache between loops ``a`` and ``b`` (consecutive in the kernel, opposite sweeps)."""

    a: int
    b: int
    a_fwd: bool
    fields: List[str]
    no_store: Set[str]  # scratch fields whose cached levels are never written to memory
    # head: the FIRST levels of loop a's sweep stay on chip (the reader re-reads the last ones,
    # written just before the turn, from the Infinity Cache); else the LAST ones (tail)
    head: bool = False

    @property
    def low(self) -> bool:
        """The cached levels are the lowest ones, [0, kreg + L) (else the highest)."""
        return self.a_fwd == self.head

    def var(self, name):
        return f"tl_{cname(name)}"


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
        self.ring = max(0, int(opts.get("kring", DEFAULT_RING)))
        self.tile = bool(getattr(kernel, "tile", False))
        self.lds = set(getattr(kernel, "lds", ()))
        # tile mode: levels per LDS barrier in the steady-state loop (option ``tile_lblock``); the
        # planes rotate over 2 x that many buffers
        self.lblock = int(opts.get("tile_lblock", TILE_LBLOCK)) if self.tile else 1
        if self.lblock not in (1, 2, 4):
            raise ValueError(f"tile_lblock must be 1, 2 or 4, got {self.lblock}")
        self.pmask = "1" if self.lblock == 1 else str(2 * self.lblock - 1)
        self._by_cap = 16
        self.trows = int(opts.get("tile_rows", TILE_ROWS)) if self.tile else 1
        if self.trows not in (1, 2):
            raise ValueError(f"tile_rows must be 1 or 2, got {self.trows}")
        if self.tile:
            self._fit_tile_lds()
            bx, by = self._block()
            by *= self.trows
            if bx - ilo - ihi < 8 or by - jlo - jhi < 1:
                raise UnsupportedStencil(f"IJ extent {self.ext} too wide for a {bx}x{by} tile")
            ti = int(opts.get("tile_ti", 0))
            if ti and not 8 <= ti <= bx - ilo - ihi:
                raise ValueError(f"tile_ti must be in [8, {bx - ilo - ihi}] for IJ extent {self.ext}, got {ti}")
        self.info = {li: self._analyse_loop(li) for li in kernel.loops}
        self.kreg = 0
        self.band_pf_default = None
        self.tail = None if self.tile else self._plan_tail()

    def _mem(self, name):
        return name in self.api or name in self.scratch

    def tile_lds_bytes(self) -> int:
        """Tile mode: the block's static LDS, one plane per shared field and buffer
        (2 x ``lblock`` buffers of ``by`` x ``bx`` cells)."""
        bx, by = self._block()
        return sum(2 * self.lblock * by * self.trows * bx * self.st.decl(n).dtype.itemsize for n in self.lds)

    def _fit_tile_lds(self) -> None:
        """Keep the tile's LDS planes within the CU's 160 KB: fewer levels per
        barrier first, then 8-row blocks when the rows are the automatic choice; a sweep that
        still does not fit goes to the staged lowering (UnsupportedStencil)."""
        if self.tile_lds_bytes() <= LDS_BYTES:
            return
        if self.lblock > 1:
            self.lblock, self.pmask = 1, "1"
        if self.tile_lds_bytes() > LDS_BYTES and int(self.opts.get("tile_by", TILE_BY)) == -1:
            self._by_cap = 8
        if self.tile_lds_bytes() > LDS_BYTES:
            raise UnsupportedStencil(
                f"tile kernel needs {self.tile_lds_bytes()} B of LDS planes for {sorted(self.lds)} (limit {LDS_BYTES})")

    def _block(self) -> Tuple[int, int]:
        """Threads per block in I and J (option ``col_bx``: I width, 256 threads in total; tile
        mode: ``tile_bx`` x ``tile_by`` threads, halo included; defaults 64 x 8 for 8-byte cells,
        128 x 8 for narrower ones)."""
        if getattr(self.kernel, "tile", False):
            by = int(self.opts.get("tile_by", TILE_BY))
            if by == -1:
                by = 16 if self.ext[2] + self.ext[3] <= 1 and self._tile_item() >= 8 and self._by_cap >= 16 else 8
            # two waves per row for cells of 4 bytes or less (a row of 448 B of outputs, r03l sweep)
            bx = int(self.opts.get("tile_bx", 0)) or (128 if self._tile_item() <= 4 and by <= 8 else 64)
            if not 2 <= by <= 16 or bx not in (64, 128) or bx * by > 1024:
                raise ValueError(f"tile_bx x tile_by must be 64 or 128 x 2 ... 16 (at most 1024 threads), got {bx} x {by}")
            return bx, by
        bx = int(self.opts.get("col_bx", COLUMN_BLOCK[0]))
        if bx not in (64, 128, 256):
            raise ValueError(f"col_bx must be 64, 128 or 256, got {bx}")
        return bx, (COLUMN_BLOCK[0] * COLUMN_BLOCK[1]) // bx

    def _tile_geom(self) -> Tuple[int, int]:
        """Tile mode: output columns (I) and rows (J) per tile. ``tile_ti`` narrows the I width
        below the block's 64 lanes minus the halo (lanes past the tile's halo then repeat its
        last column: same addresses, no extra lines)."""
        bx, by = self._block()
        eilo, eihi, ejlo, ejhi = self.ext
        ti = int(self.opts.get("tile_ti", 0))
        if not ti:
            # widest tile whose output rows start on an aligned boundary (128 B for 8-byte cells,
            # 64 B for narrower ones), so the API stores write whole lines: unaligned 62-wide f64
            # tiles take 1.2-1.5x the time (profiles/r03/r03l_sweep_tile_geom*.log)
            ti = bx - eilo - eihi
            item = self._tile_item()
            unit = (128 if item >= 8 else 64) // item
            if ti >= unit:
                ti -= ti % unit
        return ti, by * self.trows - ejlo - ejhi

    def _tile_item(self) -> int:
        """Largest cell size among the API fields the tile kernel stores (8 if none)."""
        sizes = set()
        for li in self.kernel.loops:
            for sec in self.st.vertical_loops[li].sections:
                for acc, w in iter_accesses(sec.body):
                    if w and isinstance(acc, ir.FieldAccess) and acc.name in self.api:
                        sizes.add(self.st.decl(acc.name).dtype.itemsize)
        return max(sizes, default=8)

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
        if self.tile:
            conds.insert(0, "alive")
        return " && ".join(conds) if conds else None

    def _tile_local(self, li, si, ti) -> Optional[str]:
        """Tile mode: the lanes of the block on which top-level statement ti is valid -- the owned
        tile grown by the statement's own extent. Outside it a statement's cross-column reads
        reach past the tile (e.g. ``[tx-1]`` at tx = 0), so a halo lane that still passes the
        global ``_guard`` computes garbage; a store of that garbage to a scratch field would race
        with the tile that owns the column. Extent analysis makes every producer
        valid wherever its consumers are, so the guard never starves a valid lane."""
        (a, b), (c, d) = self.a.extents.blocks.get((li, si, ti), ((0, 0), (0, 0)))
        eilo, _, ejlo, _ = self.ext
        TI, TJ = self._tile_geom()
        conds = []
        if a < eilo:
            conds.append(f"tx >= {eilo - a}")
        conds.append(f"tx < {eilo + TI + b}")
        if c < ejlo:
            conds.append(f"ty >= {ejlo - c}")
        conds.append(f"ty < {ejlo + TJ + d}")
        return " && ".join(conds)

    # ------------------------------------------------------------------ analysis
    def _analyse_loop(self, li) -> _LoopInfo:
        vl = self.st.vertical_loops[li]
        # direct fields: read at a run-time K offset or written at a K offset in this loop; every
        # access to them goes to memory at its own address (no register window)
        direct: Set[str] = set()
        for sec in vl.sections:
            for acc, w in iter_accesses(sec.body):
                if isinstance(acc, ir.FieldAccess) and (acc.k_offset is not None or (w and acc.offset[2] != 0)):
                    if not self._mem(acc.name):
                        raise UnsupportedStencil(f"run-time or written K offset on temporary '{acc.name}'")
                    direct.add(acc.name)
        win: Dict[Tuple[str, int, int], List[int]] = {}
        wnames: Set[str] = set()
        for sec in vl.sections:
            for acc, w in iter_accesses(sec.body):
                if not isinstance(acc, ir.FieldAccess) or acc.name in direct:
                    continue
                di, dj, dk = acc.offset
                if acc.name in self.lds and (di or dj):
                    continue  # tile mode: read from the level's LDS plane
                rng = win.setdefault((acc.name, di, dj), [dk, dk])
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
            if not self._mem(name) and rng[0] != rng[1] and not _contiguous(vl):
                # the planner puts such temporaries in scratch (plan.make_plan); a register window
                # cannot carry a value across levels that never run
                raise UnsupportedStencil(f"register temporary '{name}' read at a K offset across a section gap")
        return _LoopInfo(vl.loop_order != ir.LoopOrder.BACKWARD, direct, win, wnames)

    def _plan_tail(self) -> Optional[_Tail]:
        budget = int(self.opts.get("ktail_lds", LDS_BYTES))
        if budget <= 0 or any(self.ext):
            return None
        loops = self.kernel.loops
        best = None
        for x in range(len(loops) - 1):
            la, lb = loops[x], loops[x + 1]
            A, B = self.info[la], self.info[lb]
            vla = self.st.vertical_loops[la]
            if A.fwd == B.fwd or not _covers_all_levels(vla, A.fwd):
                continue
            b_written = {acc.name for sec in self.st.vertical_loops[lb].sections
                         for acc, w in iter_accesses(sec.body) if w}
            fields = []
            for (name, di, dj) in B.win:
                if (di, dj) != (0, 0) or not self._mem(name) or name in b_written or name in B.direct:
                    continue
                if "K" not in self.st.decl(name).axes:  # one value for all levels: nothing per level to cache
                    continue
                if any(k[0] == name and (k[1], k[2]) != (0, 0) for k in B.win):
                    continue
                rng = A.win.get((name, 0, 0))
                if rng is None or name in A.direct or not (rng[0] <= 0 <= rng[1]):
                    continue
                fields.append(name)
            if fields and (best is None or len(fields) > len(best.fields)):
                # scratch values only these two loops touch need no memory copy of the cached levels
                no_store = set()
                for n in fields:
                    if n in self.scratch and self._touching_loops(n) <= {la, lb}:
                        no_store.add(n)
                if no_store and int(self.opts.get("ktail_all", 0)) == 0:
                    # a cached level of such a field saves its write AND its re-read (twice the HBM
                    # bytes per LDS byte of a field that is only re-read): give them all the LDS
                    fields = [n for n in fields if n in no_store]
                best = _Tail(la, lb, A.fwd, fields, no_store)
        if best is None:
            return None
        # which end of the writer's sweep stays on chip (option ``ktail_head``: 1 head, 0 tail,
        # -1 auto): a re-read level costs HBM bytes unless it was written recently enough to be
        # in the 256-MB Infinity Cache, i.e. unless it is one of the writer's LAST levels -- so
        # cached API outputs (re-read, never skipped) keep the FIRST levels on chip (lab:
        # scripts/lab/headtail_lab.hip, tridiag with 40 LDS levels 2.245 -> 2.152 ms). Write-free
        # scratch tails keep the last levels: their big register band would stay live through
        # both memory sweeps.
        head = int(self.opts.get("ktail_head", DEFAULT_TAIL_HEAD))
        if head < 0:
            head = 1 if not all(n in best.no_store for n in best.fields) else 0
        best.head = bool(head)
        per_level = 256 * sum(self.st.decl(n).dtype.itemsize for n in best.fields)
        self.tail_lmax = budget // per_level
        if self.tail_lmax < 1:
            return None
        self.tail_per_level = per_level
        self._plan_register_band(best)
        return best

    def _plan_register_band(self, t: _Tail) -> None:
        """Register band: the ``kreg`` levels at the END of loop ``a``'s sweep (the START of loop
        ``b``'s) keep the tail fields in registers ``rb_<name>_<u>`` instead of LDS; the LDS band
        moves next to it. The band code is unrolled with static register names, so every band
        level's section must be known statically: true for ``nk >= band_nmin`` (checked at run time;
        below it the kernel runs without the register band)."""
        self.kreg = 0
        self.band_pf_default = None
        R = int(self.opts.get("kreg", DEFAULT_KREG))
        if R < 0:
            # auto: a band of AUTO_KREG levels when every cached field is a scratch temporary that
            # the band keeps out of memory altogether (no write, no re-read: 32 B per level and
            # column for two f64 fields) and the cached bytes per level fit two f64: vadv
            # 1024^2x160 2.42 -> 1.885 ms (kreg 96, band fronts prefetched 8 levels ahead; 32: 2.11,
            # 64: 2.00, 112: 1.94 ms). When the cached fields are API outputs (tridiag's sup/rhs,
            # written anyway) the band saves only the re-read and costs more than it saves
            # (kreg 32: -1.3 %, 64: +5 %, 96: +35 %), so no band (profiles/r04/r04c_sweep_*_kreg.log)
            # Cached API outputs (tridiag's sup/rhs, written at every level anyway): the band saves
            # only the re-read; a moderate band with a shallow prefetch still pays a little
            # (tridiag 1024^2x160: kreg 48 / pf 6 1.826 ms vs 1.869 without; 16: 1.851, 32: 1.841;
            # 64 and beyond lose, profiles/r04/r04h_sweep_tridiag_band.log)
            per_level = sum(self.st.decl(n).dtype.itemsize for n in t.fields)
            if not t.fields or per_level > 16:
                R = 0
            elif all(n in t.no_store for n in t.fields):
                R = AUTO_KREG
            else:
                R = AUTO_KREG_API
                self.band_pf_default = AUTO_KREG_API_PF
        if R <= 0:
            return
        B = self.info[t.b]
        if any(B.win.get((n, 0, 0)) != [0, 0] for n in t.fields):
            return  # the reader's fronts must be the cached level itself
        maps = {}
        bounds = []
        for li in (t.a, t.b):
            secs = self.st.vertical_loops[li].sections
            m = []
            for u in range(R):
                lev = (ir.LevelMarker.START, u) if t.low else (ir.LevelMarker.END, u - R)
                hit = [si for si, sec in enumerate(secs)
                       if _ge(lev, sec.interval.start) and not _ge(lev, sec.interval.end)]
                m.append(hit[0] if hit else None)
            if li == t.a and any(x is None for x in m):
                return
            maps[li] = m
            for sec in secs:
                bounds += [sec.interval.start, sec.interval.end]
        nmin = R + 1
        for b in bounds:
            nmin = max(nmin, R + (b.offset if b.level == ir.LevelMarker.START else -b.offset) + 1)
        self.kreg = R
        self.band_map = maps
        self.band_nmin = nmin

    def _touching_loops(self, name) -> Set[int]:
        out = set()
        for li, vl in enumerate(self.st.vertical_loops):
            for sec in vl.sections:
                if any(acc.name == name for acc, _ in iter_accesses(sec.body)):
                    out.add(li)
        return out

    # ------------------------------------------------------------------ rendering
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
        # tile kernels: the halo lanes load the neighbouring tiles' columns, so every stream is read
        # by more than one block and stays cacheable (non-temporal: 1.15x the time, r03l sweep)
        if self.opts.get("nt_load", 0 if self.tile else 1):
            self.nt_loads = {n for n, ks in keys.items() if n not in write_loops and len(ks) == 1 and self._mem(n)}
        if self.opts.get("nt_store", 1):
            self.nt_stores = {
                n for n, wl in write_loops.items()
                if self._mem(n) and n not in self.scratch and not (read_loops.get(n, set()) - wl)
            }
        scalars = st.scalar_params()
        L = []
        L.append(f"struct K{k}Params {{")
        for s in used:
            L += ["    " + x for x in kparam_decl(s, s.name in written)]
        for s in scalars:
            L.append(f"    {s.dtype.ctype} s_{cname(s.name)};")
        L.append("    int32_t ni, nj, nk;")
        L.append("    int32_t tail_len;  // levels held in the LDS tail cache (0: none)")
        L.append("};")
        L.append("")
        bx, by = self._block()
        L.append(f"__global__ void __launch_bounds__({bx * by}) k{k}_column(const K{k}Params p) {{")
        B = []
        eilo, eihi, ejlo, ejhi = self.ext
        if self.tile:
            # overlapping tiles: block (ti, tj) owns output columns [ti*TI, ti*TI + TI) x
            # [tj*TJ, tj*TJ + TJ) and its threads cover them plus the loop's IJ extent as halo;
            # no thread returns early (every thread reaches every level's barrier)
            TI, TJ = self._tile_geom()
            B.append("const int nbx = (int)gridDim.x, nb = nbx * (int)gridDim.y;")
            B.append("const int b = (int)(blockIdx.y * gridDim.x + blockIdx.x);")
            B.append("const int q = nb >> 3, r = nb & 7, xcd = b & 7, slot = b >> 3;")
            B.append("const int w = (xcd < r) ? xcd * (q + 1) + slot : r * (q + 1) + (xcd - r) * q + slot;")
            B.append("const int tx = (int)threadIdx.x, ty = (int)threadIdx.y;")
            # tile order within an XCD's range (option ``tile_order``): 0 I-fast (neighbours in I are
            # consecutive work items), 1 J-fast, 2 pairs of J rows I-fast (tiles (ti, 2q) and (ti, 2q+1)
            # consecutive, so both sides of a J halo row run together)
            torder = int(self.opts.get("tile_order", 0))
            if torder == 1:
                B.append("const int nby = (int)gridDim.y, tti = w / nby, ttj = w % nby;")
            elif torder == 2:
                B.append("const int nby = (int)gridDim.y, pr = w / (2 * nbx), rem = w % (2 * nbx);")
                B.append("const bool pair = 2 * pr + 1 < nby;  // the last row of an odd count runs alone")
                B.append("const int tti = pair ? (rem >> 1) : rem, ttj = pair ? 2 * pr + (rem & 1) : 2 * pr;")
            else:
                B.append("const int tti = w % nbx, ttj = w / nbx;")
            if TI + eilo + eihi < bx:
                B.append(f"const int i = tti * {TI} + (tx < {TI + eilo + eihi} ? tx : {TI + eilo + eihi - 1}) - {eilo};")
            else:
                B.append(f"const int i = tti * {TI} + tx - {eilo};")
            B.append(f"const int j = ttj * {TJ} + ty - {ejlo};")
            B.append(f"const bool alive = i < p.ni + {eihi} && j < p.nj + {ejhi};")
            B.append(f"const bool own = tx >= {eilo} && tx < {eilo + TI} && ty >= {ejlo} && ty < {ejlo + TJ} && "
                     f"i < p.ni && j < p.nj;")
            if self.trows == 2:  # the thread's second row, by rows further down the tile
                B.append(f"const int ty_r1 = ty + {by}, j_r1 = j + {by};")
                B.append(_row1(f"const bool alive = i < p.ni + {eihi} && j < p.nj + {ejhi};"))
                B.append(_row1(f"const bool own = tx >= {eilo} && tx < {eilo + TI} && ty >= {ejlo} && "
                               f"ty < {ejlo + TJ} && i < p.ni && j < p.nj;"))
            for n in sorted(self.lds):
                ct = self.st.decl(n).dtype.ctype
                B.append(f"__shared__ {ct} lds_{cname(n)}[{2 * self.lblock}][{by * self.trows}][{bx}];  "
                         f"// this level's plane (k & {self.pmask})")
        elif int(self.opts.get("col_order", 1)) == 1:
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
        if not self.tile:
            B.append(f"if (i >= p.ni + {eihi} || j >= p.nj + {ejhi}) return;")
        B.append("const int nk = p.nk;")
        for s in scalars:
            B.append(f"const {s.dtype.ctype} s_{cname(s.name)} = p.s_{cname(s.name)};")
        # column base pointers: the i/j part of every address, computed once per thread
        self.bases: Dict[Tuple[str, int, int], str] = {}
        nb0 = len(B)
        for li in self.kernel.loops:
            inf = self.info[li]
            for (name, di, dj) in list(inf.win) + [(n, None, None) for n in sorted(inf.direct)]:
                if not self._mem(name):
                    continue
                if di is None:
                    continue  # direct accesses: offsets known per access, see _base()
                self._base(name, di, dj, B, name in written)
            for sec in self.st.vertical_loops[li].sections:
                for acc, w in iter_accesses(sec.body):
                    if isinstance(acc, ir.FieldAccess) and acc.name in inf.direct:
                        self._base(acc.name, acc.offset[0], acc.offset[1], B, acc.name in written)
        if self.trows == 2:
            B += [_row1(x) for x in B[nb0:]]
        if self.tail is not None:
            t = self.tail
            B.append(f"extern __shared__ __attribute__((aligned(16))) char gtmi_lds[];")
            B.append(f"const int tid = (int)(threadIdx.y * {bx} + threadIdx.x);")
            if self.kreg:
                R = self.kreg
                B.append(f"const bool regband = nk >= {self.band_nmin};  // register band of {R} levels")
                B.append(f"const int rbase = regband ? {R} : 0;")
                for n in t.fields:
                    ct = self.st.decl(n).dtype.ctype
                    B.append(f"{ct} " + ", ".join(f"rb_{cname(n)}_{u}" for u in range(R)) + ";")
            else:
                B.append("const int rbase = 0;")
            B.append("const int tlen = p.tail_len < nk - rbase ? p.tail_len : nk - rbase;")
            if not t.low:
                B.append("const int tc1 = nk - rbase, tc0 = tc1 - tlen;  // LDS-cached levels [tc0, tc1)")
            else:
                B.append("const int tc0 = rbase, tc1 = rbase + tlen;  // LDS-cached levels [tc0, tc1)")
            off = "0"
            for n in t.fields:
                ct = self.st.decl(n).dtype.ctype
                B.append(f"{ct}* __restrict__ {t.var(n)} = ({ct}*)(gtmi_lds + {off});")
                off = f"{off} + (size_t)p.tail_len * 256 * sizeof({ct})"
        # prefetch across the writer/reader boundary of the register band: the
        # reader is rendered first so that the writer's last band levels can issue the reader's
        # first band prefetches (declared here, at kernel scope)
        t_ = self.tail
        self._xpf = bool(self.kreg) and t_ is not None and not t_.head \
            and t_.a != t_.b and t_.b in self.kernel.loops and t_.a in self.kernel.loops \
            and self.kernel.loops.index(t_.b) == self.kernel.loops.index(t_.a) + 1
        if self._xpf:
            # a reader front the writer's band might still write (any reader window field the
            # writer writes, except the band-served tail fields) must not be fetched early
            wa = self.info[t_.a]
            clash = {n for (n, _, _) in self.info[t_.b].win} & (wa.wnames | wa.direct)
            self._xpf = not (clash - set(t_.fields))
        self._xpf_decls, self._xpf_loads = [], []
        order = [t_.b] + [x for x in self.kernel.loops if x != t_.b] if self._xpf else list(self.kernel.loops)
        self._blocked_any = False
        rendered = {li: self._render_loop(li) for li in order}
        if self.lblock > 1 and not self._blocked_any:
            # nothing could be blocked: two planes, as with tile_lblock=1
            self.lblock, self.pmask = 1, "1"
            return self.render()
        B += self._xpf_decls
        for li in self.kernel.loops:
            B += rendered[li]
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
        lds = "0"
        if self.tail is not None:
            H.append(f"        p.tail_len = nk < {self.tail_lmax} ? nk : {self.tail_lmax};")
            lds = f"(size_t)p.tail_len * {self.tail_per_level}"
            H.append("        static bool lds_attr = false;")
            H.append("        if (!lds_attr) {")
            H.append(f"            hipFuncSetAttribute((const void*)k{k}_column, hipFuncAttributeMaxDynamicSharedMemorySize, "
                     f"{LDS_BYTES});")
            H.append("            lds_attr = true;")
            H.append("        }")
        else:
            H.append("        p.tail_len = 0;")
        if self.tile:
            TI, TJ = self._tile_geom()
            H.append(
                f"        hipLaunchKernelGGL(k{k}_column, dim3((unsigned)((ni + {TI - 1}) / {TI}), "
                f"(unsigned)((nj + {TJ - 1}) / {TJ})), dim3({bx}, {by}), {lds}, stream, p);"
            )
        else:
            grid = (f"dim3((unsigned)((ni + {eilo + eihi + bx - 1}) / {bx}), "
                    f"(unsigned)((nj + {ejlo + ejhi + by - 1}) / {by})), dim3({bx}, {by}), {lds}, stream, p")
            H.append(f"        hipLaunchKernelGGL(k{k}_column, {grid});")
        H.append("    }")
        H.append("}")
        return "\n".join(L), "\n".join(H)

    def _base_fields(self) -> Dict[str, str]:
        """Column base pointer variable -> the field it addresses."""
        return {v: key[0] for key, v in self.bases.items()}

    @staticmethod
    def _blockable(levels: List[List[str]], shift: List[str], base_fields: Optional[Dict[str, str]] = None) -> bool:
        """Can a level's statements after its LDS barrier wait until the next level's statements
        before it have run? Exactly one barrier per level, no plane written after it, no window
        value assigned after it that the next level's shift or statements read, and no field
        stored to memory after it that the next level's shift or statements load (the caller also
        refuses loops with run-time K offsets, whose memory reads this text test cannot place)."""
        st = levels[0]
        bars = [q for q, x in enumerate(st) if x.startswith("gtmi::lds_barrier();")]
        if len(bars) != 1:
            return False
        post = st[bars[0] + 1:]
        if any("lds_" in x and "] = " in x for x in post):
            return False
        assigned = {m.group(1) for x in post for m in [_WASSIGN.match(x)] if m}
        later = "\n".join(shift + levels[1][:bars[0]])
        if any(re.search(r"\b" + re.escape(n) + r"\b", later) for n in assigned):
            return False
        if base_fields:
            stored = {base_fields[v] for x in post if "sstore<" in x for v in _CBVAR.findall(x) if v in base_fields}
            loaded = {base_fields[v] for v in _CBVAR.findall(later) if v in base_fields}
            if stored & loaded:
                return False
        return True

    def _base(self, name, di, dj, out: List[str], writable: bool) -> str:
        key = (name, di, dj)
        if key not in self.bases:
            c = cname(name)
            v = f"cb_{c}_{_sgn(di)}_{_sgn(dj)}"
            t = self.st.decl(name).dtype.ctype
            const = "" if writable else "const "
            out.append(
                f"{const}{t}* __restrict__ {v} = p.p_{c} + ((int64_t)gtmi::clampi(i + ({di}), p.ilo_{c}, p.ihi_{c}) * "
                f"p.sI_{c} + (int64_t)gtmi::clampi(j + ({dj}), p.jlo_{c}, p.jhi_{c}) * p.sJ_{c});"
            )
            self.bases[key] = v
        return self.bases[key]

    def _render_loop(self, li) -> List[str]:
        vl = self.st.vertical_loops[li]
        order = vl.loop_order
        info = self.info[li]
        fwd = info.fwd
        direct, win, wnames = info.direct, info.win, info.wnames
        self.direct = direct
        tail = self.tail
        tail_write = tail.fields if (tail is not None and tail.a == li) else []
        tail_read = set(tail.fields) if (tail is not None and tail.b == li) else set()
        no_store = tail.no_store if (tail is not None and tail.a == li) else set()
        R = self.kreg if (tail is not None and li in (tail.a, tail.b)) else 0
        band_map = self.band_map[li] if R else None
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
            return f"({self.bases[(name, di, dj)]} + (int64_t)gtmi::clampi({kexpr}, p.klo_{c}, p.khi_{c}) * p.sK_{c})"

        def mem_index(name, di, dj, kexpr):
            """A load expression (non-temporal for read-once streams)."""
            nt = "true" if (name in self.nt_loads and name not in direct) else "false"
            return f"gtmi::sload<{decl_dtype[name].ctype}, {nt}>({mem_ptr(name, di, dj, kexpr)})"

        def load_into(var, name, di, dj, kexpr, maybe_cached=True, reg=None) -> List[str]:
            """``var = F(level kexpr)``: from the LDS tail cache when this loop reads a cached level
            (a run-time test unless ``maybe_cached`` is False: the level is known not to be cached);
            ``reg``: the level's static register-band index (register band levels only)."""
            if reg is not None and name in tail_read and (di, dj) == (0, 0) and 0 <= reg < R:
                return [f"{var} = rb_{cname(name)}_{reg};"]
            if maybe_cached and name in tail_read and (di, dj) == (0, 0):
                return [
                    f"{{ const int lv_ = {kexpr};",
                    f"  if (lv_ >= tc0 && lv_ < tc1) {var} = {tail.var(name)}[(lv_ - tc0) * 256 + tid];",
                    f"  else {var} = {mem_index(name, di, dj, 'lv_')}; }}",
                ]
            return [f"{var} = {mem_index(name, di, dj, kexpr)};"]

        reg_now = [None]  # static register-band index of the level being generated
        band_now = [None]  # tail writer: None = run-time test per level, True/False = levels known in/out of the cache

        def mem_store(name, kexpr, value):
            nt = "true" if (name in self.nt_stores and name not in direct) else "false"
            st = f"gtmi::sstore<{decl_dtype[name].ctype}, {nt}>({mem_ptr(name, 0, 0, kexpr)}, {value});"
            if name in no_store and kexpr == "k":
                if band_now[0] == "reg":
                    return "// register band level: kept in registers only"
                if band_now[0] is True:
                    return "// cached level: kept in LDS only"
                if band_now[0] is None:
                    st = f"if (k < tc0 || k >= tc1) {st}"
            return st

        P = self.ring
        step = "+" if fwd else "-"

        def dup(code: List[str]) -> List[str]:
            """Per-column code for every row of the thread (tile_rows)."""
            return code + [_row1(x) for x in code] if self.trows == 2 else code

        def merged(stmts: List[str]) -> List[str]:
            """A level's statements for every row of the thread, interleaved between the LDS
            barriers (both rows' planes are written before any row reads across columns); the
            level's ``k_next`` update (stmts[0]) once."""
            if self.trows == 1:
                return stmts
            chunks, cur = [], []
            for x in stmts[1:]:
                if x.startswith("gtmi::lds_barrier();"):
                    chunks.append((cur, x))
                    cur = []
                else:
                    cur.append(x)
            res = stmts[:1]
            for c, bar in chunks:
                res += c + [_row1(x) for x in c] + [bar]
            return res + cur + [_row1(x) for x in cur]

        out = [f"{{  // vertical loop {li} ({order.name})"]
        decls = []
        for (name, di, dj), rng in win.items():
            t = decl_dtype[name].ctype
            for d in range(rng[0], rng[1] + 1):
                decls.append(f"    {t} {wvar(name, di, dj, d)} = ({t})0;")
        out += dup(decls)
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
        # ring keys: every loaded front, except fields this loop writes that have no K axis (IJ
        # temporaries/fields: every level is the same address, so a front fetched ahead would
        # miss the writes of the levels in between)
        ring_keys = [
            key for key, fl in front_load.items()
            if fl and not (key[0] in wnames and "K" not in self.st.decl(key[0]).axes)
        ] if P > 1 else []
        # fronts of tail-cached fields in the reading loop (LDS source in the cached segment)
        tail_keys = [key for key, fl in front_load.items() if fl and key[0] in tail_read and key[1:] == (0, 0)]

        sec_start = len(out)
        band_code: List[str] = []
        # register band fronts prefetched across the whole band: one sweep-order list of band
        # levels over all sections, each level prefetching the one ``Pb`` levels on whatever
        # section it lies in, and -- for the writer, whose band ends the sweep -- the prologue
        # issued at the start of the loop, so no band level (nor the first) waits for loads issued
        # at a section boundary
        if R:
            Pb = int(self.opts.get("kreg_pf", self.band_pf_default if self.band_pf_default is not None else P + BAND_PF_OVER_RING))
            kexpr_of = (lambda u_: f"{u_}") if tail.low else (lambda u_: f"nk - {R} + {u_}")  # noqa: E731
            all_us = sorted((u for u in range(R) if band_map[u] is not None), reverse=not fwd)
            mem_keys = {}
            for u in all_us:
                mk = []
                for key in win:
                    if not front_load[key] or not self._mem(key[0]):
                        continue
                    if key[0] in wnames and "K" not in self.st.decl(key[0]).axes:
                        continue  # as ring_keys: one address for every level, loaded at its level
                    if key[0] in tail_read and key[1:] == (0, 0) and 0 <= u + front[key] < R:
                        continue  # served by the register band
                    mk.append(key)
                mem_keys[u] = mk
            pfv = {}

            def prefetch(u_):
                return [f"{pfv[(u_, key)]} = {mem_index(key[0], key[1], key[2], f'({kexpr_of(u_)}) + ({front[key]})')};"
                        for key in mem_keys[u_]]

            def declare_pf(us_, indent):
                d = []
                for u in us_:
                    for key in mem_keys[u]:
                        pfv[(u, key)] = f"bp{u}_{wvar(*key, front[key])}"
                        d.append(f"{indent}{decl_dtype[key[0]].ctype} {pfv[(u, key)]};")
                return d

            # span schedule: ``pre`` levels are in flight when the band starts (the prologue, or for
            # the reader the writer's last levels: at most the default distance, which the writer's
            # registers afford); the rest are issued at most two per level, each ``Pb`` levels
            # ahead or as early as that allows, so a deeper distance ramps up within the band
            issue_at: Dict[int, List[int]] = {}
            if Pb > 0:
                pre = Pb
                if self._xpf and li == tail.b:
                    pre = min(Pb, int(self.opts.get("kreg_pf", P + BAND_PF_OVER_RING)))
                pre = min(pre, len(all_us))
                pend = list(range(pre, len(all_us)))
                for p_ in range(len(all_us)):
                    while pend and pend[0] - Pb <= p_ and len(issue_at.get(p_, ())) < 2:
                        issue_at.setdefault(p_, []).append(pend.pop(0))
            if Pb > 0 and self._xpf and li == tail.b:
                # reader: its first ``pre`` band levels are prefetched by the writer's last band levels
                self._xpf_decls = declare_pf(all_us[:pre], "")
                self._xpf_loads = [prefetch(u) for u in all_us[:pre]]
                out += declare_pf(all_us[pre:], "    ")
                sec_start = len(out)
            elif Pb > 0:
                out += declare_pf(all_us, "    ")
                out.append("    if (regband) {  // band prefetch prologue (whole band)")
                for u in all_us[:pre]:
                    out += ["        " + x for x in prefetch(u)]
                if self._xpf and li == tail.a:  # reader levels the writer's band is too short to reach
                    for j in range(max(0, len(self._xpf_loads) - len(all_us))):
                        out += ["        " + x for x in self._xpf_loads[j]]
                out.append("    }")
                sec_start = len(out)
        for si, sec in enumerate(vl.sections):
            lo, hi = interval_bounds(sec.interval)
            out.append(f"    {{  // section {si}")
            out.append(f"        int ks = {lo}, ke = {hi};")
            out.append("        if (ks < 0) ks = 0; if (ke > nk) ke = nk;")
            if R:  # the register band's levels run in the unrolled band code
                out.append("        if (ks < rbase) ks = rbase;" if tail.low else "        if (ke > nk - rbase) ke = nk - rbase;")

            def kaddr(acc: ir.FieldAccess) -> str:
                kexpr = f"k + ({acc.offset[2]})"
                if acc.k_offset is not None:
                    kexpr += f" + (int)({rend(acc.k_offset)})"
                return kexpr

            def resolve(acc: ir.FieldAccess) -> str:
                di, dj, dk = acc.offset
                if acc.name in direct:
                    return mem_index(acc.name, di, dj, kaddr(acc))
                if acc.name in self.lds and (di or dj):
                    return f"lds_{cname(acc.name)}[k & {self.pmask}][ty + ({dj})][tx + ({di})]"
                return wvar(acc.name, di, dj, dk)

            rend = ExprRenderer(resolve, lambda n: f"s_{cname(n)}", lambda ax: ["i", "j", "k"][ax])
            rend.exact_fma = bool(int(self.opts.get("exact_fma", 1)))
            self._kaddr = kaddr

            def shift_and_fronts(slot: Optional[int], mode: str, reg_u: Optional[int] = None,
                                 pf: Optional[Dict] = None) -> List[str]:
                """Shift every window one level and load each front: from ring ``slot``, from the
                LDS tail cache (``mode`` "lds"), from the register band (``reg_u``: the level's band
                index), from a band prefetch register (``pf``: key -> variable) or from memory here
                (``slot`` None)."""
                body = []
                for key, rng in win.items():
                    name, di, dj = key
                    ds = list(range(rng[0], rng[1] + 1))
                    if fwd:
                        for d in ds[:-1]:
                            body.append(f"{wvar(name, di, dj, d)} = {wvar(name, di, dj, d + 1)};")
                    else:
                        for d in reversed(ds[1:]):
                            body.append(f"{wvar(name, di, dj, d)} = {wvar(name, di, dj, d - 1)};")
                    if front_load[key]:
                        fd = front[key]
                        fv = wvar(name, di, dj, fd)
                        if pf is not None and key in pf:
                            body.append(f"{fv} = {pf[key]};")
                        elif reg_u is not None:
                            body += load_into(fv, name, di, dj, f"k + ({fd})", maybe_cached=False, reg=reg_u + fd)
                        elif mode == "lds" and key in tail_keys:
                            body.append(f"{fv} = {tail.var(name)}[(k + ({fd}) - tc0) * 256 + tid];")
                        elif slot is not None and key in ring_keys:
                            body.append(f"{fv} = rg{slot}_{fv};")
                        else:
                            body += load_into(fv, name, di, dj, f"k + ({fd})", maybe_cached=(mode == "mixed"))
                return body

            def reload(reg_u: Optional[int] = None, pf: Optional[Dict] = None) -> List[str]:
                body = []
                for (name, di, dj), rng in win.items():
                    if not self._mem(name):
                        continue
                    for d in range(rng[0], rng[1] + 1):
                        if d == 0 and not zero_needed_in(name, di, dj, sec):
                            continue
                        if pf is not None and (name, di, dj) in pf and d == front[(name, di, dj)]:
                            body.append(f"{wvar(name, di, dj, d)} = {pf[(name, di, dj)]};")  # prefetched
                            continue
                        body += load_into(wvar(name, di, dj, d), name, di, dj, f"k + ({d})",
                                          reg=None if reg_u is None else reg_u + d)
                return body

            def statements() -> List[str]:
                body = [f"k_next = k {step} 1;"]
                pending: Set[str] = set()  # LDS planes written since the last barrier (tile mode)
                for ti, s in enumerate(sec.body):
                    if self.lds:
                        reads = {a.name for a, w in iter_accesses([s])
                                 if not w and isinstance(a, ir.FieldAccess) and a.name in self.lds
                                 and (a.offset[0] or a.offset[1])}
                        if reads & pending:
                            body.append("gtmi::lds_barrier();  // the level's planes are complete")
                            pending.clear()
                    code = self._stmt(s, rend, wvar, mem_store)
                    g = self._guard(li, si, ti)
                    if self.tile and any(w and self._mem(a.name) and a.name not in self.api
                                         for a, w in iter_accesses([s])):
                        g = f"{g} && {self._tile_local(li, si, ti)}" if g else self._tile_local(li, si, ti)
                    if g:
                        code = [f"if ({g}) {{"] + ["    " + x for x in code] + ["}"]
                    body += code
                    if self.lds:
                        pending |= {a.name for a, w in iter_accesses([s]) if w and a.name in self.lds}
                if pending:
                    # planes written but not read across columns at this level: the next write of
                    # the same buffer (two levels on) must not overtake a slow reader
                    body.append("gtmi::lds_barrier();")
                if tail_write and band_now[0] == "reg":
                    body.append("// register band: this level's final values")
                    body += [f"rb_{cname(n)}_{reg_now[0]} = {wvar(n, 0, 0, 0)};" for n in tail_write]
                elif tail_write and band_now[0] is not False:
                    stores = [f"{tail.var(n)}[(k - tc0) * 256 + tid] = {wvar(n, 0, 0, 0)};" for n in tail_write]
                    if band_now[0] is True:
                        body.append("// LDS tail cache: this level's final values")
                        body += stores
                    else:
                        body.append("if (k >= tc0 && k < tc1) {  // LDS tail cache: this level's final values")
                        body += ["    " + x for x in stores]
                        body.append("}")
                return body

            def entry_level(slot, mode) -> List[str]:
                """A segment's first level, which may follow a gap: full window reload unless it
                continues the sweep (the only level with loads inside a branch)."""
                return (["if (k != k_next) {  // (re)load the full K-window"] + ["    " + x for x in dup(reload())]
                        + ["} else {"] + ["    " + x for x in dup(shift_and_fronts(slot, mode))] + ["}"]
                        + merged(statements()))

            def refill(slot, R, keys) -> List[str]:
                body = []
                for key in keys:
                    fv = wvar(*key, front[key])
                    body += load_into(f"rg{slot}_{fv}", *key, f"k {step} {R} + ({front[key]})", maybe_cached=False)
                return body

            def segment(ss, se, mode: str) -> List[str]:
                """Levels [ss, se) of the section in sweep order. ``mode``: "mem" (no front of
                these levels is tail-cached), "lds" (every tail-cached front is), "mixed"."""
                keys = [k_ for k_ in ring_keys if not (mode == "lds" and k_ in tail_keys)] if mode != "mixed" else []
                R = _section_ring(sec.interval, P) if keys else 0
                o = [f"{{  // levels [{ss}, {se}), {mode}"]
                o.append(f"    const int ss = {ss}, se = {se};")
                first = "ss" if fwd else "se - 1"
                o.append("    if (ss < se) {")
                if R <= 1:
                    # no ring: fronts loaded at their level (first level peeled: the loop itself has
                    # no branch around a load)
                    o.append("        {")
                    o.append(f"            const int k = {first};")
                    o += ["            " + x for x in entry_level(None, mode)]
                    o.append("        }")
                    if fwd:
                        o.append("        for (int k = ss + 1; k < se; ++k) {")
                    else:
                        o.append("        for (int k = se - 2; k >= ss; --k) {")
                    o += ["            " + x for x in dup(shift_and_fronts(None, mode)) + merged(statements())]
                    o.append("        }")
                    o.append("    }")
                    o.append("}")
                    return o
                pro = []
                for u in range(R):
                    for key in keys:
                        fv = wvar(*key, front[key])
                        t = decl_dtype[key[0]].ctype
                        pro.append(f"{t} rg{u}_{fv};")
                        pro += load_into(f"rg{u}_{fv}", *key, f"{first} {step} {u} + ({front[key]})", maybe_cached=False)
                o += ["        " + x for x in dup(pro)]
                # first level: reload or continue; ring slot 0
                o.append("        {")
                o.append(f"            const int k = {first};")
                o += ["            " + x for x in entry_level(0, mode)]
                o += ["            " + x for x in dup(refill(0, R, keys))]
                o.append("        }")
                # full blocks of R levels: shift only, no branches around loads (a load inside a
                # branch makes the compiler drain every load in flight at the join)
                if fwd:
                    o.append("        int kb = ss + 1;")
                    o.append(f"        for (; kb + {R - 1} < se; kb += {R}) {{")
                else:
                    o.append("        int kb = se - 2;")
                    o.append(f"        for (; kb - {R - 1} >= ss; kb -= {R}) {{")
                blocked = self.lblock > 1 and R % self.lblock == 0 and not direct and \
                    self._blockable([statements() for _ in range(2)], shift_and_fronts(1 % R, mode),
                                    self._base_fields())
                self._blocked_any |= blocked
                for g in range(0, R, self.lblock if blocked else 1):
                    if not blocked:
                        u, slot = g, (g + 1) % R
                        o.append(f"            {{  // ring slot {slot}")
                        o.append(f"                const int k = kb {step} {u};")
                        o += ["                " + x for x in dup(shift_and_fronts(slot, mode)) + merged(statements())
                              + dup(refill(slot, R, keys))]
                        o.append("            }")
                        continue
                    # tile mode, several levels per LDS barrier: every level's statements before
                    # the barrier (the plane writes), one barrier, then every level's statements
                    # after it on snapshots of the window values they read
                    o.append(f"            {{  // levels kb {step} {g} .. {g + self.lblock - 1}: one LDS barrier")
                    posts = []
                    for b in range(self.lblock):
                        u, slot = g + b, (g + b + 1) % R
                        kv = f"k{b}_"
                        ren = lambda x, kv=kv: _KVAR.sub(kv, x)  # noqa: E731
                        o.append(f"                const int {kv} = kb {step} {u};")
                        st = statements()
                        cut = next(q for q, x in enumerate(st) if x.startswith("gtmi::lds_barrier();"))
                        pre, post = st[:cut], st[cut + 1:]
                        names = sorted(set(_WVAR.findall("\n".join(post))))
                        # pre[0] is the level's k_next update: once for both rows of a thread
                        o += ["                " + ren(x) for x in dup(shift_and_fronts(slot, mode)) + pre[:1] + dup(pre[1:])]
                        o += ["                " + x for x in dup([f"auto sn{b}_{n} = {n};" for n in names])]
                        o += ["                " + ren(x) for x in dup(refill(slot, R, keys))]
                        snap = re.compile(r"\b(" + "|".join(map(re.escape, names)) + r")\b") if names else None
                        posts += dup([ren(snap.sub(lambda m, b=b: f"sn{b}_{m.group(1)}", x) if snap else x) for x in post])
                    o.append("                gtmi::lds_barrier();  // the block's planes are complete")
                    o += ["                " + x for x in posts]
                    o.append("            }")
                o.append("        }")
                # the last < R levels: their fronts are already in the ring
                for u in range(R - 1):
                    slot = (u + 1) % R
                    cond = f"kb + {u} < se" if fwd else f"kb - {u} >= ss"
                    o.append(f"        if ({cond}) {{  // ring slot {slot}")
                    o.append(f"            const int k = kb {step} {u};")
                    o += ["            " + x for x in dup(shift_and_fronts(slot, mode)) + merged(statements())]
                    o.append("        }")
                o.append("    }")
                o.append("}")
                return o

            if tail_keys:
                # split the section by where the tail-cached fronts come from. A front k + fd is
                # cached iff tc0 <= k + fd < tc1. With lo/hi the smallest/largest fd of the tail keys:
                # all fronts cached for k in [tc0 - lo, tc1 - hi), none below tc0 - hi or from
                # tc1 - lo on. Levels before the cached band in sweep order are run "mixed" (their
                # ring would look ahead into the cache); the band itself reads LDS; the levels after
                # it stream from memory with the ring.
                fds = [front[k_] for k_ in tail_keys]
                lo_fd, hi_fd = min(fds), max(fds)
                mn = lambda a, b: f"({a} < {b} ? {a} : {b})"  # noqa: E731
                mx = lambda a, b: f"({a} > {b} ? {a} : {b})"  # noqa: E731
                out.append(f"        const int x1 = tc0 - ({hi_fd}), x2 = {mx('x1', f'tc0 - ({lo_fd})')};")
                out.append(f"        const int x3 = {mx('x2', f'tc1 - ({hi_fd})')}, x4 = tc1 - ({lo_fd});  // x1 <= x2 <= x3 <= x4")
                x1, x2, x3, x4 = "x1", "x2", "x3", "x4"
                rng_ = lambda a, b: (mx("ks", a) if a else "ks", mn("ke", b) if b else "ke")  # noqa: E731
                if tail.head:
                    # the cache sits at the END of this (reading) sweep: stream the levels before
                    # it with the ring, each side of it the levels whose fronts straddle its edge
                    out.append("        const int x4b = x4 > x3 ? x4 : x3;")
                    if fwd:
                        parts = [(*rng_(None, x1), "mem"), (*rng_(x1, x2), "mixed"), (*rng_(x2, x3), "lds"),
                                 (*rng_(x3, "x4b"), "mixed"), (*rng_("x4b", None), "mem")]
                    else:
                        parts = [(*rng_("x4b", None), "mem"), (*rng_(x3, "x4b"), "mixed"), (*rng_(x2, x3), "lds"),
                                 (*rng_(x1, x2), "mixed"), (*rng_(None, x1), "mem")]
                elif fwd:
                    parts = [(*rng_(None, x2), "mixed"), (*rng_(x2, x3), "lds"), (*rng_(x3, x4), "mixed"),
                             (*rng_(x4, None), "mem")]
                else:
                    parts = [(*rng_(x3, None), "mixed"), (*rng_(x2, x3), "lds"), (*rng_(x1, x2), "mixed"),
                             (*rng_(None, x1), "mem")]
                for ss, se, mode in parts:
                    out += ["        " + x for x in segment(ss, se, mode)]
            else:
                out += ["        " + x for x in segment("ks", "ke", "mem")]
            out.append("    }")
            us = [u for u in range(R) if band_map[u] == si] if R else []
            if us:
                # this section's register-band levels: unrolled, static register names. The band
                # is straight-line code, so its memory fronts are software-pipelined explicitly:
                # band level n's fronts are loaded ``kreg_pf`` band levels earlier into registers
                # of their own (a level waiting for its own loads stalls a one-wave-per-SIMD kernel)
                order_us = sorted(us, reverse=not fwd)
                # prefetch distance: see BAND_PF_OVER_RING
                bc = [f"    if (regband) {{  // section {si}: register band levels"]
                seq = all_us
                for n_, u in enumerate(order_us):
                    kexpr = kexpr_of(u)
                    reg_now[0], band_now[0] = u, "reg"
                    pf = {key: pfv[(u, key)] for key in mem_keys[u]} if Pb > 0 else None
                    if n_ == 0:
                        body = (["if (k != k_next) {"] + ["    " + x for x in reload(u, pf)] + ["} else {"]
                                + ["    " + x for x in shift_and_fronts(None, "mem", u, pf)] + ["}"])
                    else:
                        body = shift_and_fronts(None, "mem", u, pf)
                    g_ = seq.index(u)
                    for t_ in issue_at.get(g_, ()):
                        body += prefetch(seq[t_])
                    if self._xpf and li == tail.a and Pb > 0:
                        # the reader's band level j is prefetched its own distance (len(_xpf_loads))
                        # before the reader starts
                        j_ = g_ + len(self._xpf_loads) - len(seq)
                        if 0 <= j_ < len(self._xpf_loads):
                            body += ["// the reader's band: prefetched here"] + self._xpf_loads[j_]
                    body += statements()
                    reg_now[0], band_now[0] = None, None
                    bc.append(f"        {{  const int k = {kexpr};")
                    bc += ["            " + x for x in body]
                    bc.append("        }")
                bc.append("    }")
                band_code += bc
        if band_code:
            if (li == tail.a) != tail.head:
                out += band_code  # the band ends the writer's sweep (tail) or the reader's (head)
            else:
                out[sec_start:sec_start] = band_code  # and starts the other one
        out.append("}")
        return out

    def _stmt(self, s, rend, wvar, mem_store) -> List[str]:
        if isinstance(s, ir.Assign):
            name = s.target.name
            if name in self.direct:
                st = mem_store(name, self._kaddr(s.target), rend(s.value))
                if name in self.api and self.tile:
                    st = f"if (own) {st}"
                elif name in self.api and any(self.ext):
                    st = f"if (i >= 0 && i < p.ni && j >= 0 && j < p.nj) {st}"
                return [st]
            tgt = wvar(name, 0, 0, 0)
            out = [f"{tgt} = {rend(s.value)};"]
            if name in self.lds:
                out.append(f"lds_{cname(name)}[k & {self.pmask}][ty][tx] = {tgt};")
            if self._mem(name):
                st = mem_store(name, "k", tgt)
                if name in self.api and self.tile:
                    st = f"if (own) {st}"  # overlapping tiles: each output column has one owner
                elif name in self.api and any(self.ext):
                    st = f"if (i >= 0 && i < p.ni && j >= 0 && j < p.nj) {st}"
                out.append(st)
            return out
        if isinstance(s, ir.If):
            out = [f"if ({rend(s.cond)}) {{"]
            for x in s.body:
                out += ["    " + y for y in self._stmt(x, rend, wvar, mem_store)]
            if s.orelse:
                out.append("} else {")
                for x in s.orelse:
                    out += ["    " + y for y in self._stmt(x, rend, wvar, mem_store)]
            out.append("}")
            return out
        if isinstance(s, ir.While):
            out = [f"while ({rend(s.cond)}) {{"]
            for x in s.body:
                out += ["    " + y for y in self._stmt(x, rend, wvar, mem_store)]
            out.append("}")
            return out
        if isinstance(s, ir.HorizontalRegion):
            cond = region_condition(s.masks, "i", "j", "p.ni", "p.nj")
            out = [f"if ({cond}) {{"]
            for x in s.body:
                out += ["    " + y for y in self._stmt(x, rend, wvar, mem_store)]
            out.append("}")
            return out
        raise TypeError(type(s))


def _bound_eq(a: ir.AxisBound, b: ir.AxisBound) -> bool:
    return a.level == b.level and a.offset == b.offset


_contiguous = sections_contiguous


def _covers_all_levels(vl: ir.VerticalLoop, fwd: bool) -> bool:
    """The loop's sections run every level of [0, nk) exactly once (statically provable)."""
    if not vl.sections or not _contiguous(vl):
        return False
    first, last = vl.sections[0].interval, vl.sections[-1].interval
    lo = first.start if fwd else last.start
    hi = last.end if fwd else first.end
    return _bound_eq(lo, ir.AxisBound(ir.LevelMarker.START, 0)) and _bound_eq(hi, ir.AxisBound(ir.LevelMarker.END, 0))


def _ge(level, bound: ir.AxisBound) -> bool:
    """``level >= bound`` for every ``nk >= band_nmin`` (``level`` = (marker, offset))."""
    lm, lo = level
    if lm == bound.level:
        return lo >= bound.offset
    return lm == ir.LevelMarker.END  # END + x >= START + c and not START + x >= END + c, for nk large


def _section_ring(itv: ir.Interval, P: int) -> int:
    """Ring depth of a section: ``P``, or its static length when that is shorter (a one-level
    section such as ``interval(0, 1)`` loads its fronts directly)."""
    if itv.start.level == itv.end.level:
        return max(0, min(P, itv.end.offset - itv.start.offset))
    return P


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
