"""Random GTScript program generator for differential testing (gt:mi355x vs the numpy backend).

``generate(seed)`` writes a stencil definition to a module source: three input fields with an
IJ halo of 2 (plus K slack), two outputs, a few temporaries; statements are random arithmetic
expression trees over fields/temporaries at random offsets, ternaries, if/else blocks and
min/max/abs; computations are PARALLEL (IJ offsets), or FORWARD/BACKWARD with K recurrences on
temporaries. Everything stays within the declared halos so the same inputs are valid for any
program, and only exactly-rounded operations are used, so results must be bit-identical.
"""

import random

HALO = 2
NAMES_IN = ("a", "b", "c")


class _Gen:
    def __init__(self, seed):
        self.r = random.Random(seed)
        self.temps = []  # (name, ij_extent_used)
        self.lines = []

    def leaf(self, allow_temps, kmode):
        r = self.r
        if allow_temps and self.temps and r.random() < 0.4:
            t = r.choice(self.temps)
            # temporaries at IJ offsets only from the outputs (extent stays within the halo of 2)
            di, dj = (r.randint(-1, 1), r.randint(-1, 1)) if (kmode == "par" and allow_temps == "offsets") else (0, 0)
            return f"{t}[{di}, {dj}, 0]"
        if r.random() < 0.15:
            return repr(round(r.uniform(-3, 3), 3))
        f = r.choice(NAMES_IN)
        di, dj = r.randint(-1, 1), r.randint(-1, 1)
        dk = r.choice((0, 0, 0, 1, -1)) if kmode == "par" else 0
        return f"{f}[{di}, {dj}, {dk}]"

    def expr(self, depth, allow_temps, kmode):
        r = self.r
        if depth == 0 or r.random() < 0.25:
            return self.leaf(allow_temps, kmode)
        kind = r.random()
        x = self.expr(depth - 1, allow_temps, kmode)
        y = self.expr(depth - 1, allow_temps, kmode)
        if kind < 0.55:
            op = r.choice(("+", "-", "*"))
            return f"({x} {op} {y})"
        if kind < 0.65:
            return f"({x} / (abs({y}) + 1.5))"
        if kind < 0.8:
            fn = r.choice(("min", "max"))
            return f"{fn}({x}, {y})"
        if kind < 0.9:
            z = self.expr(depth - 1, allow_temps, kmode)
            return f"({x} if {y} > {z} else {z})"
        return f"abs({x})"


def _generate_v3(seed):
    """Seeds >= 7000: the column-kernel schedules of round 5. A FORWARD sweep followed by a
    BACKWARD sweep that reads the first one's products at (0, 0) -- a write-free scratch
    temporary and/or an API output (sweep-to-sweep cache: tail placement for scratch, head
    placement for API outputs, register band when nk is large) -- or a FORWARD recurrence whose
    product a second FORWARD computation reads across columns (tile kernel, two levels per
    barrier)."""
    g = _Gen(seed)
    r = g.r
    name = f"fuzz_{seed}"
    L = [f"def {name}(a: Field[np.float64], b: Field[np.float64], c: Field[np.float64], "
         f"out1: Field[np.float64], out2: Field[np.float64], *, s: float):"]
    if r.random() < 0.6:
        temp, api = r.random() < 0.7, r.random() < 0.6
        if not (temp or api):
            temp = True
        L.append("    with computation(FORWARD):")
        L.append("        with interval(0, 1):")
        if temp:
            L.append(f"            cc = {g.expr(2, False, 'seq')}")
        if api:
            L.append(f"            out1 = {g.expr(2, False, 'seq')}")
        L.append("        with interval(1, None):")
        if temp:
            L.append(f"            cc = cc[0, 0, -1] * 0.5 + {g.expr(2, False, 'seq')}")
        if api:
            L.append(f"            out1 = {g.expr(1, False, 'seq')} - out1[0, 0, -1] * 0.25")
        rd = " + ".join((["cc"] if temp else []) + (["out1"] if api else []))
        L.append("    with computation(BACKWARD):")
        L.append("        with interval(-1, None):")
        L.append(f"            out2 = {rd} * s")
        L.append("        with interval(0, -1):")
        L.append(f"            out2 = ({rd}) * 0.5 - out2[0, 0, 1] * 0.25 + {g.expr(1, False, 'seq')}")
    else:
        L.append("    with computation(FORWARD):")
        L.append("        with interval(0, 1):")
        L.append(f"            ss = {g.expr(2, False, 'seq')}")
        L.append("        with interval(1, None):")
        L.append(f"            ss = ss[0, 0, -1] * 0.5 + {g.expr(2, False, 'seq')}")
        L.append("    with computation(FORWARD), interval(...):")
        L.append(f"        tt = ss * {round(r.uniform(0.5, 2), 3)} + {g.expr(1, False, 'seq')}")
        offs = [(1, 0), (-1, 0), (0, 1), (0, -1), (1, 1), (-1, -1)]
        picks = r.sample(offs, r.randint(2, 4))
        terms = " + ".join(f"tt[{di}, {dj}, 0]" for di, dj in picks)
        L.append(f"        out1 = {terms} - ss * {g.expr(1, False, 'seq')}")
    return "\n".join(L) + "\n", name


MIXED_BASE = 9000  # seeds >= MIXED_BASE: mixed-precision programs (_generate_mixed)
# field dtypes of the mixed-precision programs: f32 and f64 inputs, an int32 input, an f32 and an
# f64 output (the NumPy-ufunc upcasting of gtir_upcaster.py:80-143 and the cast on assignment)
MIXED_FIELDS = {"a": "float32", "b": "float64", "c": "float32", "m": "int32", "out1": "float32", "out2": "float64"}


LOWDIM_BASE = 9700  # seeds >= LOWDIM_BASE: lower-dimensional fields (_generate_lowdim)
LOWDIM_FIELDS = {"a": ("float64", "IJK"), "w": ("float32", "IJ"), "z": ("float64", "K"),
                 "out1": ("float64", "IJK"), "out2": ("float64", "IJ")}


TILE_BASE = 10000  # seeds >= TILE_BASE: mixed-precision tile programs with a vector field (_generate_tile)
TILE_FIELDS = {**MIXED_FIELDS, "v": "float64"}  # v: 2 data components per cell


FUNC_BASE = 10100  # seeds >= FUNC_BASE: gtscript functions and a vector output (_generate_func)
FUNC_FIELDS = {"a": "float64", "b": "float64", "c": "float32", "m": "int32", "out1": "float64", "out2": "float32",
               "outv": "float64"}  # outv: 2 data components per cell


def data_dims(seed):
    """{field: trailing data-dimension shape} of the fields that have data dimensions."""
    if seed >= VK_BASE:
        return {}
    if seed >= FUNC_BASE:
        return {"outv": (2,)}
    return {"v": (2,)} if seed >= TILE_BASE else {}


VK_BASE = 10200  # seeds >= VK_BASE: run-time K offsets (_generate_vk), mixed precision
IVL_BASE = 10300  # seeds >= IVL_BASE: interval partitions with absolute/relative bounds and gaps
ABSK_BASE = 10400  # seeds >= ABSK_BASE: absolute K indexing (_generate_absk), f64 (debug-backend oracle)
ABSK_FIELDS = {"a": "float64", "b": "float64", "c": "float64", "m": "int32", "out1": "float64", "out2": "float64"}


def field_dtypes(seed):
    """{field: numpy dtype name} of the program ``generate(seed)`` writes."""
    if seed >= ABSK_BASE:
        return dict(ABSK_FIELDS)
    if seed >= VK_BASE:
        return dict(MIXED_FIELDS)
    if seed >= FUNC_BASE:
        return dict(FUNC_FIELDS)
    if seed >= TILE_BASE:
        return dict(TILE_FIELDS)
    if seed >= OPS_BASE:
        return dict(MIXED_FIELDS)
    if seed >= LOWDIM_BASE:
        return {n: t for n, (t, _) in LOWDIM_FIELDS.items()}
    if seed >= MIXED_BASE:
        return dict(MIXED_FIELDS)
    return {n: "float64" for n in ("a", "b", "c", "out1", "out2")}


def field_axes(seed):
    """{field: axes} ("IJK", "IJ" or "K") of the program ``generate(seed)`` writes."""
    if LOWDIM_BASE <= seed < OPS_BASE:
        return {n: ax for n, (_, ax) in LOWDIM_FIELDS.items()}
    return {n: "IJK" for n in field_dtypes(seed)}


def make_inputs(seed, shape):
    """Deterministic inputs of program ``seed`` on domain ``shape``: (fields, origins). Inputs
    carry an IJ halo of 2; float inputs U(-4, 4), the int32 input U{-5..5}, outputs U(-1, 1) in
    their own dtype (cells outside the domain keep these values). Lower-dimensional fields have
    only their own axes."""
    import numpy as np

    rng = np.random.default_rng(20000 + seed)
    ni, nj, nk = shape
    dts, axes = field_dtypes(seed), field_axes(seed)
    fields, origin = {}, {}
    dd = data_dims(seed)
    for n, dt in dts.items():
        out = n.startswith("out")
        ext = {"I": ni if out else ni + 4, "J": nj if out else nj + 4, "K": nk}
        shp = tuple(ext[a] for a in axes[n]) + dd.get(n, ())
        origin[n] = tuple(0 if (out or a == "K") else 2 for a in axes[n])
        if out:
            fields[n] = rng.uniform(-1, 1, shp).astype(dt)
        elif dt == "int32":
            fields[n] = rng.integers(-5, 6, shp).astype(dt)
        else:
            fields[n] = rng.uniform(-4, 4, shp).astype(dt)
    return fields, origin


class _MixedGen(_Gen):
    """Leaves over f32/f64/int32 fields, float and int literals: every binary operation mixes
    dtypes at random, so the program exercises the upcasting rules, not one precision."""

    def leaf(self, allow_temps, kmode):
        r = self.r
        if allow_temps and self.temps and r.random() < 0.35:
            t = r.choice(self.temps)
            di, dj = (r.randint(-1, 1), r.randint(-1, 1)) if allow_temps == "offsets" else (0, 0)
            return f"{t}[{di}, {dj}, 0]"
        x = r.random()
        if x < 0.08:
            return repr(round(r.uniform(-3, 3), 3))
        if x < 0.14:
            return str(r.randint(-3, 3))
        f = r.choice(("a", "b", "c", "a", "c", "m"))
        di, dj = r.randint(-1, 1), r.randint(-1, 1)
        dk = r.choice((0, 0, 0, 1, -1)) if kmode == "kwin" else 0
        return f"{f}[{di}, {dj}, {dk}]"


def _generate_mixed(seed):
    """Seeds >= MIXED_BASE: PARALLEL computations split into K intervals (K offsets in the middle
    one), FORWARD/BACKWARD recurrences on temporaries whose dtype comes from their first
    assignment (later f64 values are cast back), and conditionals, over f32, f64 and int32
    fields with f64 and int literals."""
    g = _MixedGen(seed)
    r = g.r
    name = f"fuzz_{seed}"
    sig = ", ".join(f"{n}: Field[np.{t}]" for n, t in MIXED_FIELDS.items())
    L = [f"def {name}({sig}, *, s: float):"]
    for ci in range(r.randint(1, 3)):
        order = r.choice(("PARALLEL", "PARALLEL", "FORWARD", "BACKWARD"))
        out = r.choice(("out1", "out2"))
        if order == "PARALLEL":
            L.append("    with computation(PARALLEL):")
            L.append("        with interval(0, 1):")
            L.append(f"            {out} = {g.expr(2, False, 'par')}")
            L.append("        with interval(1, -1):")
            nst = r.randint(0, 2)
            for si in range(nst):
                t = f"t{ci}_{si}"
                L.append(f"            {t} = {g.expr(2, True, 'kwin')}")
                g.temps.append(t)
            if r.random() < 0.5:
                L.append(f"            if {g.expr(1, True, 'kwin')} > s:")
                L.append(f"                {out} = {g.expr(2, 'offsets', 'kwin')}")
                L.append("            else:")
                L.append(f"                {out} = {g.expr(2, 'offsets', 'kwin')} * s")
            else:
                L.append(f"            {out} = {g.expr(3, 'offsets', 'kwin')}")
            L.append("        with interval(-1, None):")
            L.append(f"            {out} = {g.expr(2, False, 'par')} + {out}")
            g.temps = []
        else:
            first, rest = ("interval(0, 1)", "interval(1, None)") if order == "FORWARD" else (
                "interval(-1, None)", "interval(0, -1)")
            dk = -1 if order == "FORWARD" else 1
            acc = f"acc{ci}"
            L.append(f"    with computation({order}):")
            L.append(f"        with {first}:")
            L.append(f"            {acc} = {g.expr(2, False, 'seq')}")
            L.append(f"            {out} = {acc}")
            L.append(f"        with {rest}:")
            L.append(f"            {acc} = {acc}[0, 0, {dk}] * {round(r.uniform(0.25, 0.75), 2)} + {g.expr(2, False, 'seq')}")
            L.append(f"            {out} = {acc} - {out}[0, 0, {dk}] * 0.25")
    return "\n".join(L) + "\n", name


KOFF_BASE = 9500  # seeds >= KOFF_BASE: K-offset programs (_generate_koff), mixed precision too


class _KoffGen(_MixedGen):
    """Leaves of the K-offset programs: ``kmode`` "k" reads fields (and the PARALLEL temporaries
    in ``self.ktemps``) at K offsets -1..1, optionally at IJ offsets too."""

    def leaf(self, allow_temps, kmode):
        r = self.r
        if kmode == "k" and self.ktemps and r.random() < 0.3:
            t = r.choice(self.ktemps)
            di, dj = (r.randint(-1, 1), r.randint(-1, 1)) if r.random() < 0.3 else (0, 0)
            return f"{t}[{di}, {dj}, {r.randint(-1, 1)}]"
        if kmode == "k":
            return super().leaf(allow_temps, "kwin")
        return super().leaf(allow_temps, kmode)


def _generate_koff(seed):
    """Seeds >= KOFF_BASE: PARALLEL temporaries over the whole column, then a FORWARD or BACKWARD
    sweep in three intervals whose middle one reads the fields and those temporaries at K
    offsets (K windows of the column kernel, staged phases when read at IJ offsets), then
    optionally a PARALLEL computation reading the temporaries at K offsets again."""
    g = _KoffGen(seed)
    g.ktemps = []
    r = g.r
    name = f"fuzz_{seed}"
    sig = ", ".join(f"{n}: Field[np.{t}]" for n, t in MIXED_FIELDS.items())
    L = [f"def {name}({sig}, *, s: float):"]
    L.append("    with computation(PARALLEL), interval(...):")
    for q in range(r.randint(1, 2)):
        L.append(f"        p{q} = {g.expr(2, False, 'par')}")
        g.ktemps.append(f"p{q}")
    order = r.choice(("FORWARD", "BACKWARD"))
    out = r.choice(("out1", "out2"))
    first, last = ("interval(0, 1)", "interval(-1, None)") if order == "FORWARD" else ("interval(-1, None)", "interval(0, 1)")
    dk = -1 if order == "FORWARD" else 1
    L.append(f"    with computation({order}):")
    L.append(f"        with {first}:")
    L.append(f"            acc = {g.expr(2, False, 'par')} + p0")
    L.append(f"            {out} = acc")
    L.append("        with interval(1, -1):")
    L.append(f"            acc = acc[0, 0, {dk}] * {round(r.uniform(0.25, 0.75), 2)} + {g.expr(2, False, 'k')}")
    if r.random() < 0.5:
        L.append(f"            if {g.expr(1, False, 'k')} > s:")
        L.append(f"                {out} = acc - {out}[0, 0, {dk}] * 0.25")
        L.append("            else:")
        L.append(f"                {out} = {g.expr(1, False, 'k')} + acc")
    else:
        L.append(f"            {out} = acc - {out}[0, 0, {dk}] * 0.25")
    L.append(f"        with {last}:")
    L.append(f"            acc = acc[0, 0, {dk}] * 0.5 + {g.expr(1, False, 'par')}")
    L.append(f"            {out} = acc * s")
    if r.random() < 0.6:
        other = "out2" if out == "out1" else "out1"
        L.append("    with computation(PARALLEL), interval(1, -1):")
        L.append(f"        {other} = {g.expr(3, False, 'k')}")
    return "\n".join(L) + "\n", name


class _LowdimGen(_Gen):
    """Leaves over a 3-D f64 field ``a``, a 2-D f32 field ``w`` and a 1-D K field ``z``."""

    def leaf(self, allow_temps, kmode):
        r = self.r
        x = r.random()
        if x < 0.1:
            return repr(round(r.uniform(-3, 3), 3))
        if x < 0.45:
            dk = r.choice((0, 0, 1, -1)) if kmode == "kwin" else 0
            return f"a[{r.randint(-1, 1)}, {r.randint(-1, 1)}, {dk}]"
        if x < 0.75:
            return f"w[{r.randint(-1, 1)}, {r.randint(-1, 1)}]"
        return f"z[{r.choice((0, 0, 1, -1)) if kmode == 'kwin' else 0}]"


def _generate_lowdim(seed):
    """Seeds >= LOWDIM_BASE: 2-D (IJ) and 1-D (K) fields read beside a 3-D one (K offsets of the
    K field in the middle interval), a 2-D output accumulated by a FORWARD sweep and optionally
    read back by a later PARALLEL computation."""
    g = _LowdimGen(seed)
    r = g.r
    name = f"fuzz_{seed}"
    ann = {"IJK": "Field[np.{t}]", "IJ": "Field[IJ, np.{t}]", "K": "Field[K, np.{t}]"}
    sig = ", ".join(f"{n}: " + ann[ax].format(t=t) for n, (t, ax) in LOWDIM_FIELDS.items())
    L = [f"def {name}({sig}, *, s: float):"]
    L.append("    with computation(PARALLEL):")
    L.append("        with interval(0, 1):")
    L.append(f"            out1 = {g.expr(2, False, 'par')}")
    L.append("        with interval(1, -1):")
    L.append(f"            out1 = {g.expr(3, False, 'kwin')}")
    L.append("        with interval(-1, None):")
    L.append(f"            out1 = {g.expr(2, False, 'par')} * s")
    L.append("    with computation(FORWARD):")
    L.append("        with interval(0, 1):")
    L.append(f"            out2 = {g.expr(2, False, 'par')}")
    L.append("        with interval(1, None):")
    L.append(f"            out2 = out2 * {round(r.uniform(0.25, 0.75), 2)} + {g.expr(2, False, 'par')}")
    if r.random() < 0.5:
        L.append("    with computation(PARALLEL), interval(...):")
        L.append(f"        out1 = out1 + out2 * {g.expr(1, False, 'par')}")
    return "\n".join(L) + "\n", name


OPS_BASE = 9800  # seeds >= OPS_BASE: operator programs (_generate_ops), mixed precision


class _OpsGen(_MixedGen):
    """Expressions over the exactly rounded builtins: mod, ** 2, sqrt, floor/ceil/trunc, round
    (half to even), round_away_from_zero, casts; conditions with and/or/not."""

    def expr(self, depth, allow_temps, kmode):
        r = self.r
        if depth == 0 or r.random() < 0.2:
            return self.leaf(allow_temps, kmode)
        x = self.expr(depth - 1, allow_temps, kmode)
        k = r.random()
        if k < 0.3:
            return f"({x} {r.choice(('+', '-', '*'))} {self.expr(depth - 1, allow_temps, kmode)})"
        if k < 0.38:
            return f"({x} % (abs({self.expr(depth - 1, allow_temps, kmode)}) + 0.75))"
        if k < 0.43:
            return f"((m[{r.randint(-1, 1)}, {r.randint(-1, 1)}, 0] + {r.randint(0, 9)}) % {r.randint(2, 5)})"
        if k < 0.5:
            return f"(min(max({x}, -30.0), 30.0) ** 2)"
        if k < 0.55:
            return f"sqrt(abs({x}))"
        if k < 0.67:
            fn = r.choice(("floor", "ceil", "trunc", "round", "round_away_from_zero"))
            return f"{fn}({x} * {r.choice((0.5, 1.5, 2.0, 0.25))})"
        if k < 0.72:
            ct = r.choice(("float32", "float64", "int32", "int64"))
            return f"{ct}(min(max({x}, -100.0), 100.0))"
        if k < 0.82:
            return f"{r.choice(('min', 'max'))}({x}, {self.expr(depth - 1, allow_temps, kmode)})"
        if k < 0.92:
            return f"({x} if {self.cond(allow_temps, kmode)} else {self.expr(depth - 1, allow_temps, kmode)})"
        return f"abs({x})"

    def cond(self, allow_temps, kmode):
        r = self.r
        a = f"{self.expr(1, allow_temps, kmode)} {r.choice(('>', '<', '>=', '<=', '==', '!='))} {self.expr(1, allow_temps, kmode)}"
        k = r.random()
        if k < 0.5:
            return a
        b = f"{self.expr(1, allow_temps, kmode)} > {self.expr(0, allow_temps, kmode)}"
        if k < 0.7:
            return f"({a}) and (not ({b}))"
        if k < 0.9:
            return f"({a}) or ({b})"
        return f"isfinite({self.expr(1, allow_temps, kmode)}) and ({a})"


def _generate_ops(seed):
    """Seeds >= OPS_BASE: PARALLEL if/elif/else chains (nested once) and a FORWARD sweep over the
    operator set of ``_OpsGen``, on the mixed-precision fields."""
    g = _OpsGen(seed)
    r = g.r
    name = f"fuzz_{seed}"
    sig = ", ".join(f"{n}: Field[np.{t}]" for n, t in MIXED_FIELDS.items())
    L = [f"def {name}({sig}, *, s: float):"]
    out = r.choice(("out1", "out2"))
    L.append("    with computation(PARALLEL), interval(...):")
    L.append(f"        t0 = {g.expr(2, False, 'par')}")
    g.temps.append("t0")
    L.append(f"        if {g.cond(True, 'par')}:")
    L.append(f"            {out} = {g.expr(2, True, 'par')}")
    if r.random() < 0.5:
        L.append(f"            if {g.cond(True, 'par')}:")
        L.append(f"                {out} = {out} * {g.expr(1, True, 'par')}")
    L.append(f"        elif {g.cond(True, 'par')}:")
    L.append(f"            {out} = {g.expr(2, True, 'par')}")
    L.append("        else:")
    L.append(f"            {out} = {g.expr(2, True, 'par')} + s")
    g.temps = []
    if r.random() < 0.6:
        other = "out2" if out == "out1" else "out1"
        L.append("    with computation(FORWARD):")
        L.append("        with interval(0, 1):")
        L.append(f"            {other} = {g.expr(2, False, 'seq')}")
        L.append("        with interval(1, None):")
        L.append(f"            {other} = {other}[0, 0, -1] * 0.5 + {g.expr(2, False, 'seq')}")
    return "\n".join(L) + "\n", name


CTRL_BASE = 9900  # seeds >= CTRL_BASE: while loops and horizontal regions (_generate_ctrl)
REGIONS = ("region[I[0] : I[0] + 2, :]", "region[:, J[-1] - 1 : J[-1]]", "region[I[0] : I[0] + 3, J[0] : J[0] + 2]",
           "region[I[-1] - 2 : I[-1], :]", "region[I[0] + 1 : I[-1] - 1, J[0] + 1 : J[0] + 2]")


def _generate_ctrl(seed):
    """Seeds >= CTRL_BASE: bounded while loops on temporaries (an int counter, optionally a value
    condition), horizontal regions in PARALLEL and FORWARD/BACKWARD computations, over the
    mixed-precision fields."""
    g = _MixedGen(seed)
    r = g.r
    name = f"fuzz_{seed}"
    sig = ", ".join(f"{n}: Field[np.{t}]" for n, t in MIXED_FIELDS.items())
    L = [f"def {name}({sig}, *, s: float):"]
    out = r.choice(("out1", "out2"))
    other = "out2" if out == "out1" else "out1"
    L.append("    with computation(PARALLEL), interval(...):")
    L.append("        n = 0")
    L.append(f"        acc = {g.expr(2, False, 'par')}")
    cond = f"n < {r.randint(1, 4)}"
    if r.random() < 0.5:
        cond += f" and acc {r.choice(('>', '<'))} {round(r.uniform(-2, 2), 2)}"
    L.append(f"        while {cond}:")
    L.append(f"            acc = acc * {round(r.uniform(0.25, 0.75), 2)} + {g.expr(2, False, 'par')}")
    L.append("            n = n + 1")
    L.append(f"        {out} = acc + n")
    if r.random() < 0.7:
        L.append(f"        with horizontal({r.choice(REGIONS)}):")
        L.append(f"            {out} = {g.expr(2, False, 'par')} + {out}")
    order = r.choice(("FORWARD", "BACKWARD"))
    first, rest = ("interval(0, 1)", "interval(1, None)") if order == "FORWARD" else ("interval(-1, None)", "interval(0, -1)")
    dk = -1 if order == "FORWARD" else 1
    L.append(f"    with computation({order}):")
    L.append(f"        with {first}:")
    L.append(f"            {other} = {g.expr(2, False, 'seq')}")
    L.append(f"        with {rest}:")
    L.append(f"            {other} = {other}[0, 0, {dk}] * 0.5 + {g.expr(2, False, 'seq')}")
    if r.random() < 0.7:
        L.append(f"            with horizontal({r.choice(REGIONS)}):")
        L.append(f"                {other} = {g.expr(2, False, 'seq')} - {other}[0, 0, {dk}]")
    return "\n".join(L) + "\n", name


class _TileGen(_MixedGen):
    """Mixed-precision leaves plus the components of the vector field ``v``."""

    def leaf(self, allow_temps, kmode):
        r = self.r
        if r.random() < 0.2:
            return f"v[{r.randint(-1, 1)}, {r.randint(-1, 1)}, 0][{r.randint(0, 1)}]"
        return super().leaf(allow_temps, kmode)


def _generate_tile(seed):
    """Seeds >= TILE_BASE: the tile-kernel shape (a FORWARD recurrence whose product a second
    FORWARD computation reads across columns, IJ caches in LDS) with an f32, f64 or int32
    recurrence, mixed-precision operands and the components of a vector field."""
    g = _TileGen(seed)
    r = g.r
    name = f"fuzz_{seed}"
    sig = ", ".join(f"{n}: Field[np.{t}]" for n, t in MIXED_FIELDS.items()) + ", v: Field[(np.float64, (2,))]"
    L = [f"def {name}({sig}, *, s: float):"]
    seedexpr = r.choice(("a[0, 0, 0]", "c[0, 0, 0] * 0.5", "m[0, 0, 0]", "b[0, 0, 0]", "v[0, 0, 0][1]"))
    L.append("    with computation(FORWARD):")
    L.append("        with interval(0, 1):")
    L.append(f"            ss = {seedexpr}")
    L.append("        with interval(1, None):")
    L.append(f"            ss = ss[0, 0, -1] * {round(r.uniform(0.25, 0.75), 2)} + {g.expr(2, False, 'seq')}")
    L.append("    with computation(FORWARD), interval(...):")
    L.append(f"        tt = ss * {round(r.uniform(0.5, 2), 3)} + {g.expr(1, False, 'seq')}")
    offs = [(1, 0), (-1, 0), (0, 1), (0, -1), (1, 1), (-1, -1), (1, -1)]
    picks = r.sample(offs, r.randint(2, 4))
    terms = " + ".join(f"tt[{di}, {dj}, 0]" for di, dj in picks)
    out = r.choice(("out1", "out2"))
    L.append(f"        {out} = {terms} - ss * {g.expr(1, False, 'seq')}")
    if r.random() < 0.5:
        other = "out2" if out == "out1" else "out1"
        L.append(f"        {other} = tt[{r.randint(-1, 1)}, {r.randint(-1, 1)}, 0] * v[0, 0, 0][0] + ss")
    return "\n".join(L) + "\n", name


class _FuncGen(_MixedGen):
    """Leaves over the f64/f32/int32 inputs of the function programs, and calls of the module's
    gtscript functions (``self.funcs``: name -> arity) on field arguments."""

    def leaf(self, allow_temps, kmode):
        r = self.r
        if self.funcs and r.random() < 0.25:
            fn, arity = r.choice(sorted(self.funcs.items()))
            args = ", ".join(r.choice(("a", "b", "c", "m")) for _ in range(arity))
            return f"{fn}({args})"
        x = r.random()
        if x < 0.1:
            return repr(round(r.uniform(-3, 3), 3))
        f = r.choice(("a", "b", "c", "m"))
        return f"{f}[{r.randint(-1, 1)}, {r.randint(-1, 1)}, 0]"


def _generate_func(seed):
    """Seeds >= FUNC_BASE: two or three @gtscript.function helpers (offset reads of their field
    arguments, one calling another, one returning through an if/else), called from PARALLEL and
    FORWARD computations, and a vector output written component by component."""
    g = _FuncGen(seed)
    g.funcs = {}
    r = g.r
    name = f"fuzz_{seed}"
    L = []
    L.append("@function")
    L.append("def f0(x, y):")
    L.append(f"    return (x[1, 0, 0] - y[0, 0, 0]) * {round(r.uniform(0.25, 2), 2)} + x[0, -1, 0]")
    g.funcs["f0"] = 2
    L.append("@function")
    L.append("def f1(x):")
    L.append(f"    return max(x[0, 1, 0], x[-1, 0, 0]) - f0(x, x) * 0.5")
    g.funcs["f1"] = 1
    if r.random() < 0.5:
        L.append("@function")
        L.append("def f2(x, y):")
        L.append(f"    if x[0, 0, 0] > y[0, 0, 0]:")
        L.append(f"        t = x[0, 0, 0] - y[1, 0, 0]")
        L.append("    else:")
        L.append(f"        t = y[0, 0, 0] * {round(r.uniform(0.5, 1.5), 2)}")
        L.append("    return t")
        g.funcs["f2"] = 2
    sig = ", ".join(f"{n}: Field[np.{t}]" for n, t in FUNC_FIELDS.items() if n != "outv")
    L.append(f"def {name}({sig}, outv: Field[(np.float64, (2,))], *, s: float):")
    L.append("    with computation(PARALLEL), interval(...):")
    L.append(f"        out1 = {g.expr(2, False, 'par')}")
    L.append(f"        outv[0, 0, 0][0] = {g.expr(2, False, 'par')}")
    L.append(f"        outv[0, 0, 0][1] = out1 * {g.expr(1, False, 'par')}")
    L.append("    with computation(FORWARD):")
    L.append("        with interval(0, 1):")
    L.append(f"            out2 = {g.expr(2, False, 'seq')}")
    L.append("        with interval(1, None):")
    L.append(f"            out2 = out2[0, 0, -1] * 0.5 + {g.expr(2, False, 'seq')}")
    return "\n".join(L) + "\n", name


class _VkGen(_MixedGen):
    """Mixed-precision leaves plus reads at a run-time K offset: ``(m[..] % 3) - 1`` in the middle
    interval (levels k-1..k+1), ``m[..] % 2`` in a FORWARD sweep's interval(1, -1) (k..k+1)."""

    def leaf(self, allow_temps, kmode):
        r = self.r
        if kmode in ("vk3", "vk2") and r.random() < 0.35:
            f = r.choice(("a", "b", "c"))
            idx = f"m[{r.randint(-1, 1)}, {r.randint(-1, 1)}, 0]"
            ko = f"({idx} % 3) - 1" if kmode == "vk3" else f"{idx} % 2"
            return f"{f}[{r.randint(-1, 1)}, {r.randint(-1, 1)}, {ko}]"
        return super().leaf(allow_temps, "kwin" if kmode == "vk3" else "seq")


def _generate_vk(seed):
    """Seeds >= VK_BASE: fields read at run-time K offsets computed from an int32 field (the
    column kernels' direct loads), in a PARALLEL computation and a FORWARD sweep."""
    g = _VkGen(seed)
    r = g.r
    name = f"fuzz_{seed}"
    sig = ", ".join(f"{n}: Field[np.{t}]" for n, t in MIXED_FIELDS.items())
    L = [f"def {name}({sig}, *, s: float):"]
    L.append("    with computation(PARALLEL):")
    L.append("        with interval(0, 1):")
    L.append(f"            out1 = {g.expr(1, False, 'par')}")
    L.append("        with interval(1, -1):")
    L.append(f"            out1 = {g.expr(3, False, 'vk3')}")
    L.append("        with interval(-1, None):")
    L.append(f"            out1 = {g.expr(1, False, 'par')} * s")
    L.append("    with computation(FORWARD):")
    L.append("        with interval(0, 1):")
    L.append(f"            out2 = {g.expr(2, False, 'seq')}")
    L.append("        with interval(1, -1):")
    L.append(f"            out2 = out2[0, 0, -1] * 0.5 + {g.expr(2, False, 'vk2')}")
    L.append("        with interval(-1, None):")
    L.append(f"            out2 = out2[0, 0, -1] * 0.25 + {g.expr(1, False, 'seq')}")
    return "\n".join(L) + "\n", name


class _IvlGen(_MixedGen):
    """Mixed-precision leaves with K offsets restricted to the ones the current interval allows
    (``self.kallowed``)."""

    def leaf(self, allow_temps, kmode):
        r = self.r
        if kmode == "ivl" and r.random() > 0.35:
            f = r.choice(("a", "b", "c", "m"))
            return f"{f}[{r.randint(-1, 1)}, {r.randint(-1, 1)}, {r.choice(self.kallowed)}]"
        return super().leaf(allow_temps, "par")


def _bounds(r):
    """A random partition of the K axis as consecutive (lo, hi) bound pairs: absolute bounds from
    the bottom, relative (negative) ones from the top, None = the end."""
    cuts = sorted(r.sample([1, 2, 3, -3, -2, -1], r.randint(1, 4)), key=lambda b: (b < 0, b))
    pts = [0] + cuts + [None]
    return list(zip(pts[:-1], pts[1:]))


def _generate_ivl(seed):
    """Seeds >= IVL_BASE: a PARALLEL computation over a random partition of K into 2-5 intervals
    (absolute and relative bounds, K offsets where the interval leaves room) and a FORWARD or
    BACKWARD sweep over another partition with one interval left out (its levels keep the
    output's previous values)."""
    g = _IvlGen(seed)
    r = g.r
    name = f"fuzz_{seed}"
    sig = ", ".join(f"{n}: Field[np.{t}]" for n, t in MIXED_FIELDS.items())
    L = [f"def {name}({sig}, *, s: float):"]

    def ivl(lo, hi):
        return f"interval({lo}, {hi})"

    def allowed(lo, hi):
        return [0] + ([-1] if lo != 0 else []) + ([1] if hi is not None else [])

    out = r.choice(("out1", "out2"))
    L.append("    with computation(PARALLEL):")
    for lo, hi in _bounds(r):
        g.kallowed = allowed(lo, hi)
        L.append(f"        with {ivl(lo, hi)}:")
        L.append(f"            {out} = {g.expr(2, False, 'ivl')}")
    other = "out2" if out == "out1" else "out1"
    order = r.choice(("FORWARD", "BACKWARD"))
    parts = _bounds(r)
    if len(parts) > 2:
        parts.pop(r.randrange(1, len(parts)))
    if order == "BACKWARD":
        parts = parts[::-1]
    dk = -1 if order == "FORWARD" else 1
    L.append(f"    with computation({order}):")
    for q, (lo, hi) in enumerate(parts):
        g.kallowed = allowed(lo, hi)
        L.append(f"        with {ivl(lo, hi)}:")
        # the neighbour level the sweep came from exists when this is not the sweep's first level
        carried = (lo != 0) if order == "FORWARD" else (hi is not None)
        if carried:
            L.append(f"            {other} = {other}[0, 0, {dk}] * 0.5 + {g.expr(2, False, 'ivl')}")
        else:
            L.append(f"            {other} = {g.expr(2, False, 'ivl')}")
    return "\n".join(L) + "\n", name


class _AbskGen(_MixedGen):
    """f64 leaves plus ``.at(K=...)`` reads at a constant level or at a level computed from m. No
    ternaries: the reference's debug backend (the oracle here) prints a ternary without parentheses
    (gtc/debug/debug_codegen.py:358-359), so `(x if c else y) - z` runs as `x if c else (y - z)`."""

    def expr(self, depth, allow_temps, kmode):
        r = self.r
        if depth == 0 or r.random() < 0.25:
            return self.leaf(allow_temps, kmode)
        x, y = self.expr(depth - 1, allow_temps, kmode), self.expr(depth - 1, allow_temps, kmode)
        k = r.random()
        if k < 0.6:
            return f"({x} {r.choice(('+', '-', '*'))} {y})"
        if k < 0.7:
            return f"({x} / (abs({y}) + 1.5))"
        if k < 0.9:
            return f"{r.choice(('min', 'max'))}({x}, {y})"
        return f"abs({x})"

    def leaf(self, allow_temps, kmode):
        r = self.r
        if r.random() < 0.3:
            f = r.choice(("a", "b", "c"))
            lev = r.choice((str(r.randint(0, 5)), f"(m[0, 0, 0] % 3) + {r.randint(0, 3)}"))
            return f"{f}.at(K={lev})"
        return super().leaf(allow_temps, kmode)


def _generate_absk(seed):
    """Seeds >= ABSK_BASE: reads at absolute levels (``field.at(K=...)``, constant or from an int32
    field) beside relative reads, in a PARALLEL computation and a FORWARD sweep; f64 fields so the
    reference's debug backend (its only backend for absolute K indexing) is an exact oracle."""
    g = _AbskGen(seed)
    r = g.r
    name = f"fuzz_{seed}"
    sig = ", ".join(f"{n}: Field[np.{t}]" for n, t in ABSK_FIELDS.items())
    L = [f"def {name}({sig}, *, s: float):"]
    L.append("    with computation(PARALLEL), interval(...):")
    L.append(f"        out1 = {g.expr(3, False, 'par')}")
    L.append("    with computation(FORWARD):")
    L.append("        with interval(0, 1):")
    L.append(f"            out2 = {g.expr(2, False, 'seq')}")
    L.append("        with interval(1, None):")
    L.append(f"            out2 = out2[0, 0, -1] * 0.5 + {g.expr(2, False, 'seq')}")
    return "\n".join(L) + "\n", name


def generate(seed):
    """Return (source, function name) of a random stencil; seeds >= 1000 add horizontal regions,
    cross-computation temporaries read at IJ offsets and sweeps needing the staged lowering;
    seeds >= 7000 are the sweep-pair and tile templates of ``_generate_v3``; seeds >=
    ``MIXED_BASE`` the mixed-precision programs of ``_generate_mixed``."""
    if seed >= ABSK_BASE:
        return _generate_absk(seed)
    if seed >= IVL_BASE:
        return _generate_ivl(seed)
    if seed >= VK_BASE:
        return _generate_vk(seed)
    if seed >= FUNC_BASE:
        return _generate_func(seed)
    if seed >= TILE_BASE:
        return _generate_tile(seed)
    if seed >= CTRL_BASE:
        return _generate_ctrl(seed)
    if seed >= OPS_BASE:
        return _generate_ops(seed)
    if seed >= LOWDIM_BASE:
        return _generate_lowdim(seed)
    if seed >= KOFF_BASE:
        return _generate_koff(seed)
    if seed >= MIXED_BASE:
        return _generate_mixed(seed)
    if seed >= 7000:
        return _generate_v3(seed)
    v2 = seed >= 1000
    g = _Gen(seed)
    r = g.r
    name = f"fuzz_{seed}"
    L = []
    L.append(f"def {name}(a: Field[np.float64], b: Field[np.float64], c: Field[np.float64], "
             f"out1: Field[np.float64], out2: Field[np.float64], *, s: float):")
    n_comp = r.randint(1, 3)
    used_out = set()
    for ci in range(n_comp):
        order = r.choice(("PARALLEL", "PARALLEL", "FORWARD", "BACKWARD"))
        kmode = "par" if order == "PARALLEL" else "seq"
        if order == "PARALLEL":
            L.append("    with computation(PARALLEL), interval(1, -1):")
            nst = r.randint(1, 4)
            for si in range(nst):
                t = f"t{ci}_{si}"
                L.append(f"        {t} = {g.expr(3, True, kmode)}")
                g.temps.append(t)
            if r.random() < 0.5:
                cond = g.expr(1, "offsets", kmode)
                L.append(f"        if {cond} > s:")
                L.append(f"            out1 = {g.expr(2, 'offsets', kmode)}")
                L.append("        else:")
                L.append(f"            out1 = {g.expr(2, 'offsets', kmode)} * s")
            else:
                L.append(f"        out1 = {g.expr(3, 'offsets', kmode)}")
            used_out.add("out1")
            if v2 and r.random() < 0.6:
                ib = r.choice(("region[I[0] : I[0] + 2, :]", "region[:, J[-1] - 1 : J[-1]]",
                               "region[I[0] : I[0] + 3, J[0] : J[0] + 2]", "region[I[-1] - 2 : I[-1], :]"))
                # no temporaries inside the region: a value written before and read at an IJ
                # offset in a horizontal region is refused by the reference frontend
                # (gtscript_frontend.py:1952-1956), and at offset 0 they add nothing new
                L.append(f"        with horizontal({ib}):")
                L.append(f"            out1 = {g.expr(2, False, kmode)} + out1")
            if v2:
                g.prev_temps = list(g.temps)  # readable (at IJ offsets) by a later sequential sweep
            g.temps = []  # temporaries are local to the computation
        else:
            first, rest = ("interval(0, 1)", "interval(1, None)") if order == "FORWARD" else (
                "interval(-1, None)", "interval(0, -1)")
            dk = -1 if order == "FORWARD" else 1
            L.append(f"    with computation({order}):")
            L.append(f"        with {first}:")
            L.append(f"            acc = {g.expr(2, False, kmode)}")
            L.append("            out2 = acc")
            L.append(f"        with {rest}:")
            L.append(f"            acc = acc[0, 0, {dk}] * 0.5 + {g.expr(2, False, kmode)}")
            L.append(f"            out2 = acc - out2[0, 0, {dk}] * 0.25")
            used_out.add("out2")
            if v2 and r.random() < 0.6:
                # a temporary produced and read at IJ offsets inside one sweep (staged lowering),
                # optionally mixed with a PARALLEL computation's temporary at an offset
                extra = ""
                if getattr(g, "prev_temps", None):  # at an offset: extent 1 (its fields) + 1
                    extra = f" + {r.choice(g.prev_temps)}[{r.randint(-1, 1)}, {r.randint(-1, 1)}, 0]"
                # a PARALLEL temporary is only defined on interval(1, -1): reading it elsewhere reads
                # uninitialised temporary storage (undefined in GTScript), so stay inside
                ivl = "interval(1, -1)" if extra else "interval(...)"
                # one name per computation: a temporary declared in an earlier computation and
                # written + read at an IJ offset here is illegal (gtc/gtir.py:226-240)
                L.append(f"    with computation({order}), {ivl}:")
                L.append(f"        u{ci} = {r.choice(NAMES_IN)}[{r.randint(-1, 1)}, {r.randint(-1, 1)}, 0] * 0.5 + 0.25")
                L.append(f"        out2 = out2 + 0.5 * (u{ci}[1, 0, 0] - u{ci}[0, -1, 0]){extra}")
    if not used_out:
        L.append("    with computation(PARALLEL), interval(...):")
        L.append("        out1 = a")
    return "\n".join(L) + "\n", name


# seeds whose programs take the tile-kernel path (checked by tests/test_tile.py::
# test_fuzz_golden_programs_take_the_tile_path); their sources are committed as
# tests/fuzz_golden_programs.py and pinned to reference-generated goldens (stencil_cases.py)
GOLDEN_SEEDS = [1003, 1005, 1011, 1014, 1029, 1045, 1057, 5001, 5002, 5010, 5069, 5089]


def emit(seeds) -> str:
    """The source of a module defining ``fuzz_<seed>`` for every seed (``SEEDS`` lists them)."""
    out = ['"""Generated by ``python tests/fuzz_stencils.py`` from tests/fuzz_stencils.py (do not edit):',
           "differential-fuzz programs that take the tile-kernel path, pinned to reference goldens",
           '(tests/stencil_cases.py, fuzz_tile_<seed>)."""', "",
           "import numpy as np",
           "from gt4py_amd.gtscript import BACKWARD, FORWARD, PARALLEL, Field, I, J, computation, horizontal, "
           "interval, region  # noqa: F401", "", f"SEEDS = {list(seeds)!r}", ""]
    for seed in seeds:
        src, _ = generate(seed)
        out += ["", src]
    return "\n".join(out).rstrip("\n") + "\n"


if __name__ == "__main__":
    import os

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fuzz_golden_programs.py")
    with open(path, "w") as f:
        f.write(emit(GOLDEN_SEEDS))
    print(path)
