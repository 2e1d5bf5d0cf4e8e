"""Stencil cases shared by the golden-fixture generator and the parity tests.

Every case is a GTScript definition written against ``gt4py_amd.gtscript`` plus a
deterministic input recipe (shapes, dtypes, value ranges, origin, domain, parameters).

``tests/golden/make_golden.py`` runs each definition through the *reference* numpy
backend (``gt4py.cartesian``, only in the build container) by aliasing
``gt4py_amd.gtscript`` to the reference module, and stores inputs + outputs as ``.npz``.
The parity tests build the very same definitions with ``gt4py_amd`` backends and compare.

The stencils restate the GTScript programs of the reference's own tests:
- ``tests/cartesian_tests/integration_tests/multi_feature_tests/stencil_definitions.py``
- ``tests/cartesian_tests/integration_tests/multi_feature_tests/test_suites.py``
- the demo notebook ``examples/cartesian/demo_horizontal_diffusion.ipynb`` (cells 7/9)
"""



import dataclasses
import zlib
from typing import Any, Callable, Dict, Optional, Tuple

import numpy as np

from gt4py_amd import gtscript
from gt4py_amd.gtscript import (
    BACKWARD,
    FORWARD,
    PARALLEL,
    IJ,
    Field,
    I,
    J,
    computation,
    horizontal,
    interval,
    region,
)
from gt4py_amd.gtscript import __INLINED  # noqa: F401  (used inside stencil bodies)
from gt4py_amd.gtscript import (  # noqa: F401  (math builtins used inside stencil bodies)
    acos,
    acosh,
    asin,
    asinh,
    atan,
    atanh,
    cbrt,
    ceil,
    cos,
    cosh,
    erf,
    erfc,
    exp,
    floor,
    gamma,
    isfinite,
    isinf,
    isnan,
    log,
    log10,
    mod,
    round,
    round_away_from_zero,
    sin,
    sinh,
    sqrt,
    tan,
    tanh,
    trunc,
)

F64 = Field[np.float64]
F32 = Field[np.float32]
FBool = Field[np.bool_]
F2D = Field[gtscript.IJ, np.float64]


@dataclasses.dataclass
class FieldSpec:
    shape: Tuple[int, ...]
    dtype: str = "f8"
    init: Any = ("u", -10.0, 10.0)  # ("u", lo, hi) | ("int", lo, hi) | "bool" | "zeros" | "demo" | ("const", v)
    nan_frac: float = 0.0


@dataclasses.dataclass
class Case:
    name: str
    definition: Callable
    fields: Dict[str, Optional[FieldSpec]]
    params: Dict[str, Any]
    externals: Dict[str, Any]
    origin: Any
    domain: Optional[Tuple[int, int, int]]
    rtol: float = 0.0  # 0 => bit-exact expected on every backend
    atol: float = 0.0
    features: Tuple[str, ...] = ()  # tags used by tests to select/skip cases

    @property
    def seed(self) -> int:
        return zlib.crc32(self.name.encode()) & 0x7FFFFFFF

    def make_inputs(self) -> Dict[str, Optional[np.ndarray]]:
        rng = np.random.default_rng(self.seed)
        out: Dict[str, Optional[np.ndarray]] = {}
        for name, spec in self.fields.items():
            if spec is None:
                out[name] = None
                continue
            out[name] = _make_array(spec, rng)
        return out


def _make_array(spec: FieldSpec, rng: np.random.Generator) -> np.ndarray:
    dt = np.dtype(spec.dtype)
    init = spec.init
    shape = tuple(spec.shape)
    if init == "zeros":
        arr = np.zeros(shape, dtype=dt)
    elif init == "bool":
        arr = rng.random(shape) > 0.5
    elif init == "demo":
        # demo_horizontal_diffusion.ipynb cell 9: in = 5 + 8*(2 + cos(pi*(x+1.5y)) + sin(2pi*(x+1.5y)))/4
        ni, nj = shape[0], shape[1]
        x = np.arange(ni)[:, None] / ni
        y = np.arange(nj)[None, :] / nj
        plane = 5.0 + 8.0 * (2.0 + np.cos(np.pi * (x + 1.5 * y)) + np.sin(2 * np.pi * (x + 1.5 * y))) / 4.0
        arr = np.empty(shape, dtype=np.float64)
        arr[...] = plane[:, :, None] if len(shape) == 3 else plane
    elif isinstance(init, tuple) and init[0] == "u":
        arr = rng.uniform(init[1], init[2], size=shape)
    elif isinstance(init, tuple) and init[0] == "int":
        arr = rng.integers(init[1], init[2], size=shape)
    elif isinstance(init, tuple) and init[0] == "ramp":
        # monotone along the last spatial axis (pressure-like columns), jittered across I/J
        nk = shape[2] if len(shape) >= 3 else shape[-1]
        kk = np.arange(nk) / max(nk - 1, 1)
        base = init[1] + (init[2] - init[1]) * kk
        jit = rng.uniform(0.0, 0.2 * (init[2] - init[1]) / max(nk, 1), size=shape[:2] + (1,) if len(shape) >= 3 else (1,))
        arr = np.broadcast_to(base + jit, shape).copy()
    elif isinstance(init, tuple) and init[0] == "const":
        arr = np.full(shape, init[1])
    elif isinstance(init, tuple) and init[0] == "special":
        # IEEE edge values among U(lo, hi) ("special", lo, hi[, fraction[, finite only]]): signed
        # zeros, denormals, the largest finite values and (unless finite only) NaN and infinities
        # of the field's type, each cell special with probability ``fraction`` (default 1/8)
        frac = init[3] if len(init) > 3 else 0.125
        pool = [0.0, -0.0, 1.0, -1.0, 0.5]
        if dt == np.float32:
            pool += [1.4e-45, -1.4e-45, 1.1754944e-38, -3.0e-39, 3.4028235e38, -3.4028235e38]
        else:
            pool += [5e-324, -5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, -1.7976931348623157e308]
        if not (len(init) > 4 and init[4]):
            pool += [np.nan, np.inf, -np.inf]
        special = rng.random(size=shape) < frac
        pick = rng.integers(0, len(pool), size=shape)
        rnd = rng.uniform(init[1], init[2], size=shape)
        arr = np.where(special, np.asarray(pool)[pick], rnd)
    else:
        raise ValueError(f"unknown init {init!r}")
    arr = np.asarray(arr).astype(dt)
    if spec.nan_frac:
        flat = arr.reshape(-1)
        n = max(1, int(spec.nan_frac * flat.size))
        idx = rng.choice(flat.size, size=3 * n, replace=False)
        flat[idx[:n]] = np.nan
        flat[idx[n : 2 * n]] = np.inf
        flat[idx[2 * n :]] = -np.inf
    return arr


CASES: Dict[str, Case] = {}


def case(
    name: Optional[str] = None,
    *,
    fields,
    params=None,
    externals=None,
    origin=None,
    domain=None,
    rtol=0.0,
    atol=0.0,
    features=(),
):
    def deco(func):
        n = name or func.__name__
        assert n not in CASES, n
        CASES[n] = Case(
            n,
            func,
            dict(fields),
            dict(params or {}),
            dict(externals or {}),
            origin,
            domain,
            rtol,
            atol,
            tuple(features),
        )
        return func

    return deco


def fs(*shape, dtype="f8", init=("u", -10.0, 10.0), nan_frac=0.0):
    return FieldSpec(tuple(shape), dtype, init, nan_frac)


# --------------------------------------------------------------------------------------
# Hot-path stencils
# --------------------------------------------------------------------------------------


def copy_stencil(field_a: F64, field_b: F64):
    with computation(PARALLEL), interval(...):
        field_b = field_a[0, 0, 0]


case("copy", fields={"field_a": fs(16, 12, 8), "field_b": fs(16, 12, 8)}, features=("hot",))(copy_stencil)
case(
    "copy_subdomain",
    fields={"field_a": fs(16, 12, 8), "field_b": fs(16, 12, 8)},
    origin=(1, 2, 1),
    domain=(10, 8, 5),
    features=("hot",),
)(copy_stencil)


def lap5(in_field: F64, out_field: F64):
    with computation(PARALLEL), interval(...):
        out_field = 4.0 * in_field[0, 0, 0] - (
            in_field[1, 0, 0] + in_field[-1, 0, 0] + in_field[0, 1, 0] + in_field[0, -1, 0]
        )


case(
    "lap5",
    fields={"in_field": fs(26, 22, 8), "out_field": fs(24, 20, 8, init="zeros")},
    origin={"in_field": (1, 1, 0), "out_field": (0, 0, 0)},
    domain=(24, 20, 8),
    features=("hot",),
)(lap5)


def _hdiff_body_factory(dtype):
    FT = Field[dtype]

    def horizontal_diffusion(in_field: FT, out_field: FT, coeff: FT):
        with computation(PARALLEL), interval(...):
            lap_field = 4.0 * in_field[0, 0, 0] - (
                in_field[1, 0, 0] + in_field[-1, 0, 0] + in_field[0, 1, 0] + in_field[0, -1, 0]
            )
            res = lap_field[1, 0, 0] - lap_field[0, 0, 0]
            flx_field = 0 if (res * (in_field[1, 0, 0] - in_field[0, 0, 0])) > 0 else res
            res = lap_field[0, 1, 0] - lap_field[0, 0, 0]
            fly_field = 0 if (res * (in_field[0, 1, 0] - in_field[0, 0, 0])) > 0 else res
            out_field = in_field[0, 0, 0] - coeff[0, 0, 0] * (
                flx_field[0, 0, 0] - flx_field[-1, 0, 0] + fly_field[0, 0, 0] - fly_field[0, -1, 0]
            )

    return horizontal_diffusion


hdiff_f64 = _hdiff_body_factory(np.float64)
hdiff_f32 = _hdiff_body_factory(np.float32)

_HD_ORIGIN = {"in_field": (2, 2, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}

case(
    "hdiff_f64",
    fields={
        "in_field": fs(28, 24, 8),
        "out_field": fs(24, 20, 8, init="zeros"),
        "coeff": fs(24, 20, 8, init=("u", 0.0, 0.5)),
    },
    origin=_HD_ORIGIN,
    domain=(24, 20, 8),
    features=("hot",),
)(hdiff_f64)
case(
    "hdiff_f64_demo",
    fields={
        "in_field": fs(36, 36, 6, init="demo"),
        "out_field": fs(32, 32, 6, init="zeros"),
        "coeff": fs(32, 32, 6, init=("const", 0.025)),
    },
    origin=_HD_ORIGIN,
    domain=(32, 32, 6),
    features=("hot",),
)(hdiff_f64)
case(
    "hdiff_f64_origin",
    fields={
        "in_field": fs(30, 27, 10),
        "out_field": fs(30, 27, 10),
        "coeff": fs(30, 27, 10, init=("u", 0.0, 0.5)),
    },
    origin=(3, 2, 1),
    domain=(21, 19, 7),
    features=("hot",),
)(hdiff_f64)
case(
    "hdiff_f64_ties",  # integer-valued inputs hit exact res*du == 0 limiter ties
    fields={
        "in_field": fs(20, 18, 4, init=("int", -3, 4)),
        "out_field": fs(16, 14, 4, init="zeros"),
        "coeff": fs(16, 14, 4, init=("int", 0, 2)),
    },
    origin=_HD_ORIGIN,
    domain=(16, 14, 4),
    features=("hot",),
)(hdiff_f64)
case(
    "hdiff_f64_nan",  # NaN/Inf propagation (numpy runs under errstate(ignore))
    fields={
        "in_field": fs(20, 18, 4, nan_frac=0.01),
        "out_field": fs(16, 14, 4, init="zeros"),
        "coeff": fs(16, 14, 4, init=("u", 0.0, 0.5)),
    },
    origin=_HD_ORIGIN,
    domain=(16, 14, 4),
    features=("hot",),
)(hdiff_f64)
case(
    "hdiff_f32",
    fields={
        "in_field": fs(28, 24, 8, dtype="f4"),
        "out_field": fs(24, 20, 8, dtype="f4", init="zeros"),
        "coeff": fs(24, 20, 8, dtype="f4", init=("u", 0.0, 0.5)),
    },
    origin=_HD_ORIGIN,
    domain=(24, 20, 8),
    features=("hot",),
)(hdiff_f32)
case(
    "hdiff_f32_demo",
    fields={
        "in_field": fs(36, 36, 6, dtype="f4", init="demo"),
        "out_field": fs(32, 32, 6, dtype="f4", init="zeros"),
        "coeff": fs(32, 32, 6, dtype="f4", init=("const", 0.025)),
    },
    origin=_HD_ORIGIN,
    domain=(32, 32, 6),
    features=("hot",),
)(hdiff_f32)


def tridiagonal_solver(inf: F64, diag: F64, sup: F64, rhs: F64, out: F64):
    with computation(FORWARD):
        with interval(0, 1):
            sup = sup / diag
            rhs = rhs / diag
        with interval(1, None):
            sup = sup / (diag - sup[0, 0, -1] * inf)
            rhs = (rhs - inf * rhs[0, 0, -1]) / (diag - sup[0, 0, -1] * inf)
    with computation(BACKWARD):
        with interval(-1, None):
            out = rhs
        with interval(0, -1):
            out = rhs - sup * out[0, 0, 1]


def _tridiag_fields(ni, nj, nk):
    return {
        "inf": fs(ni, nj, nk, init=("u", -1.0, 1.0)),
        "diag": fs(ni, nj, nk, init=("u", 4.0, 5.0)),
        "sup": fs(ni, nj, nk, init=("u", -1.0, 1.0)),
        "rhs": fs(ni, nj, nk, init=("u", -10.0, 10.0)),
        "out": fs(ni, nj, nk, init="zeros"),
    }


case("tridiag", fields=_tridiag_fields(8, 6, 32), features=("hot",))(tridiagonal_solver)


# IEEE edge values through the hot path (signed zeros, denormals, the largest finite values -- whose
# sums overflow -- NaN and infinities, mixed with ordinary values): the f32 cast tree, the limiter's
# comparisons and the Thomas solve's divisions, against the reference numpy backend
def _special(*shape, dtype="f8", lo=-10.0, hi=10.0, frac=0.125, finite=False):
    return fs(*shape, dtype=dtype, init=("special", lo, hi, frac, finite))


for _dt, _defn in (("f4", hdiff_f32), ("f8", hdiff_f64)):
    case(
        f"hdiff_{'f32' if _dt == 'f4' else 'f64'}_special",
        fields={
            "in_field": _special(41, 33, 5, dtype=_dt),
            "out_field": fs(37, 29, 5, dtype=_dt, init="zeros"),
            "coeff": _special(37, 29, 5, dtype=_dt, lo=0.0, hi=0.5),
        },
        origin=_HD_ORIGIN,
        domain=(37, 29, 5),
        features=("hot",),
    )(_defn)
case(
    "lap5_special",
    fields={"in_field": _special(39, 31, 5), "out_field": fs(37, 29, 5, init="zeros")},
    origin={"in_field": (1, 1, 0), "out_field": (0, 0, 0)},
    domain=(37, 29, 5),
    features=("hot",),
)(lap5)
case(
    "tridiag_special",
    fields={
        # finite edge values (a NaN would poison its whole column through both sweeps), a zero
        # or denormal pivot now and then (infinities and NaN made by the divisions themselves)
        "inf": _special(9, 7, 12, lo=-1.0, hi=1.0, frac=0.05, finite=True),
        "diag": _special(9, 7, 12, lo=4.0, hi=5.0, frac=0.03, finite=True),
        "sup": _special(9, 7, 12, lo=-1.0, hi=1.0, frac=0.05, finite=True),
        "rhs": _special(9, 7, 12, frac=0.05, finite=True),
        "out": fs(9, 7, 12, init="zeros"),
    },
    features=("hot",),
)(tridiagonal_solver)
case("tridiag_k2", fields=_tridiag_fields(5, 4, 2), features=("hot",))(tridiagonal_solver)
case(
    "tridiag_subdomain",
    fields=_tridiag_fields(9, 7, 12),
    origin=(1, 2, 1),
    domain=(7, 4, 9),
    features=("hot",),
)(tridiagonal_solver)


# --------------------------------------------------------------------------------------
# test_suites.py programs
# --------------------------------------------------------------------------------------


def suite_identity(field_a: F64):
    with computation(PARALLEL), interval(...):
        tmp = field_a
        field_a = tmp


case("suite_identity", fields={"field_a": fs(9, 7, 5)})(suite_identity)


def suite_aug_assign(field_a: F64, field_b: F64):
    with computation(PARALLEL), interval(...):
        field_a += 1.0
        field_a *= 2.0
        field_b -= 1.0
        field_b /= 2.0


case("suite_aug_assign", fields={"field_a": fs(9, 7, 5), "field_b": fs(9, 7, 5)})(suite_aug_assign)


def suite_global_scale(field_a: F64):
    from __externals__ import SCALE_FACTOR

    with computation(PARALLEL), interval(...):
        field_a = SCALE_FACTOR * field_a[0, 0, 0]


case("suite_global_scale", fields={"field_a": fs(8, 6, 5, init=("u", -1.0, 1.0))}, externals={"SCALE_FACTOR": 1e3})(
    suite_global_scale
)


def suite_parametric_scale(field_a: F64, *, scale: float):
    with computation(PARALLEL), interval(...):
        field_a = scale * field_a


case("suite_parametric_scale", fields={"field_a": fs(8, 6, 5)}, params={"scale": -37.25})(suite_parametric_scale)


def suite_parametric_mix(
    field_a: F64, field_b: F64, field_c: F64, field_out: F32, *, weight: np.float64, alpha_factor: np.float64
):
    from __externals__ import USE_ALPHA
    from __gtscript__ import __INLINED

    with computation(PARALLEL), interval(...):
        if __INLINED(USE_ALPHA):
            factor = alpha_factor
        else:
            factor = 1.0
        field_out = factor * field_a[0, 0, 0] - (1 - factor) * (field_b[0, 0, 0] - weight * field_c[0, 0, 0])


for _ua in (True, False):
    case(
        f"suite_parametric_mix_{int(_ua)}",
        fields={
            "field_a": fs(8, 7, 6),
            "field_b": fs(8, 7, 6),
            "field_c": fs(8, 7, 6),
            "field_out": fs(8, 7, 6, dtype="f4"),
        },
        params={"weight": 3.5, "alpha_factor": -0.75},
        externals={"USE_ALPHA": _ua},
    )(suite_parametric_mix)


def suite_heat_equation(u: F64, v: F64, u_new: F64, v_new: F64, *, ru: float, rv: float):
    with computation(PARALLEL), interval(...):
        u_new = u[0, 0, 0] + ru * (u[1, 0, 0] - 2 * u[0, 0, 0] + u[-1, 0, 0])
        v_new = v[0, 0, 0] + rv * (v[0, 1, 0] - 2 * v[0, 0, 0] + v[0, -1, 0])


case(
    "suite_heat_equation",
    fields={"u": fs(12, 9, 6), "v": fs(10, 11, 6), "u_new": fs(10, 9, 6), "v_new": fs(10, 9, 6)},
    params={"ru": 0.3, "rv": 0.125},
    origin={"u": (1, 0, 0), "v": (0, 1, 0), "u_new": (0, 0, 0), "v_new": (0, 0, 0)},
    domain=(10, 9, 6),
)(suite_heat_equation)


def suite_hdiff_weight(u: F64, diffusion: F64, *, weight: float):
    with computation(PARALLEL), interval(...):
        laplacian = 4.0 * u[0, 0, 0] - (u[1, 0, 0] + u[-1, 0, 0] + u[0, 1, 0] + u[0, -1, 0])
        flux_i = laplacian[1, 0, 0] - laplacian[0, 0, 0]
        flux_j = laplacian[0, 1, 0] - laplacian[0, 0, 0]
        diffusion = u[0, 0, 0] - weight * (flux_i[0, 0, 0] - flux_i[-1, 0, 0] + flux_j[0, 0, 0] - flux_j[0, -1, 0])


case(
    "suite_hdiff_weight",
    fields={"u": fs(17, 15, 5), "diffusion": fs(13, 11, 5)},
    params={"weight": 0.375},
    origin={"u": (2, 2, 0), "diffusion": (0, 0, 0)},
    domain=(13, 11, 5),
)(suite_hdiff_weight)


@gtscript.function
def lap_op(u):
    """Laplacian operator."""
    return 4.0 * u[0, 0, 0] - (u[1, 0, 0] + u[-1, 0, 0] + u[0, 1, 0] + u[0, -1, 0])


@gtscript.function
def fwd_diff_op_xy(field):
    dx = field[1, 0, 0] - field[0, 0, 0]
    dy = field[0, 1, 0] - field[0, 0, 0]
    return dx, dy


@gtscript.function
def wrap1arg2return(field):
    dx, dy = fwd_diff_op_xy(field=field)
    return dx, dy


@gtscript.function
def fwd_diff_op_x(field):
    dx = field[1, 0, 0] - field[0, 0, 0]
    return dx


@gtscript.function
def fwd_diff_op_y(field):
    dy = field[0, 1, 0] - field[0, 0, 0]
    return dy


def suite_hdiff_subroutines(u: F64, diffusion: F64, *, weight: float):
    from __externals__ import fwd_diff

    with computation(PARALLEL), interval(...):
        laplacian = lap_op(u=u)
        flux_i, flux_j = fwd_diff(field=laplacian)
        diffusion = u[0, 0, 0] - weight * (flux_i[0, 0, 0] - flux_i[-1, 0, 0] + flux_j[0, 0, 0] - flux_j[0, -1, 0])


case(
    "suite_hdiff_subroutines",
    fields={"u": fs(17, 15, 5), "diffusion": fs(13, 11, 5)},
    params={"weight": 0.25},
    externals={"fwd_diff": wrap1arg2return},
    origin={"u": (2, 2, 0), "diffusion": (0, 0, 0)},
    domain=(13, 11, 5),
)(suite_hdiff_subroutines)


def suite_hdiff_subroutines2(u: F64, diffusion: F64, *, weight: float):
    from __externals__ import BRANCH
    from __gtscript__ import __INLINED

    with computation(PARALLEL), interval(...):
        laplacian = lap_op(u=u)
        if __INLINED(BRANCH):
            flux_i = fwd_diff_op_x(field=laplacian)
            flux_j = fwd_diff_op_y(field=laplacian)
        else:
            flux_i, flux_j = fwd_diff_op_xy(field=laplacian)
        diffusion = u[0, 0, 0] - weight * (flux_i[0, 0, 0] - flux_i[-1, 0, 0] + flux_j[0, 0, 0] - flux_j[0, -1, 0])


for _br in (True, False):
    case(
        f"suite_hdiff_subroutines2_{int(_br)}",
        fields={"u": fs(17, 15, 5), "diffusion": fs(13, 11, 5)},
        params={"weight": 0.125},
        externals={"BRANCH": _br},
        origin={"u": (2, 2, 0), "diffusion": (0, 0, 0)},
        domain=(13, 11, 5),
    )(suite_hdiff_subroutines2)


def suite_runtime_if_flat(outfield: F64):
    with computation(PARALLEL), interval(...):
        if True:
            outfield = 1
        else:
            outfield = 2


case("suite_runtime_if_flat", fields={"outfield": fs(6, 5, 4)})(suite_runtime_if_flat)


def suite_runtime_if_nested(outfield: F64):
    with computation(PARALLEL), interval(...):
        if (outfield > 0 and outfield > 0) or (not outfield > 0 and not outfield > 0):
            if False:
                outfield = 1
            else:
                outfield = 2
        else:
            outfield = 3


case("suite_runtime_if_nested", fields={"outfield": fs(6, 5, 4)})(suite_runtime_if_nested)


def suite_3fold_nested_if(field_a: F64):
    with computation(PARALLEL), interval(...):
        if field_a >= 0.0:
            field_a = 0.0
            if field_a > 1:
                field_a = 1
                if field_a > 2:
                    field_a = 2


case("suite_3fold_nested_if", fields={"field_a": fs(5, 5, 5, init=("u", -1.0, 1.0))})(suite_3fold_nested_if)


@gtscript.function
def add_one(field_in):
    """Add 1 to each element of `field_in`."""
    return field_in + 1


def suite_runtime_if_data_dependent(field_a: F64, field_b: F64, field_c: F64, *, factor: float):
    with computation(PARALLEL), interval(...):
        if factor > 0:
            if field_a < 0:
                field_b = -field_a
            else:
                field_b = field_a
        else:
            if field_a < 0:
                field_c = -field_a
            else:
                field_c = field_a
        field_a = add_one(field_a)


for _fac in (12.5, -3.0):
    case(
        f"suite_runtime_if_data_dependent_{'p' if _fac > 0 else 'm'}",
        fields={"field_a": fs(5, 4, 3, init=("u", -1.0, 1.0)), "field_b": fs(5, 4, 3), "field_c": fs(5, 4, 3)},
        params={"factor": _fac},
    )(suite_runtime_if_data_dependent)


def suite_runtime_if_nested_while(infield: F64, outfield: F64):
    with computation(PARALLEL), interval(...):
        if infield < 10:
            outfield = 1
            done = False
            while not done:
                outfield = 2
                done = True
        else:
            condition = True
            while condition:
                outfield = 4
                condition = False
            outfield = 3


case(
    "suite_runtime_if_nested_while",
    fields={"infield": fs(6, 5, 4, init=("u", -20.0, 20.0)), "outfield": fs(6, 5, 4)},
)(suite_runtime_if_nested_while)


def suite_ternary_op(infield: F64, outfield: F64):
    with computation(PARALLEL), interval(...):
        outfield = infield if infield > 0.0 else -infield[0, 1, 0]


case(
    "suite_ternary_op",
    fields={"infield": fs(7, 9, 4), "outfield": fs(7, 8, 4)},
    domain=(7, 8, 4),
)(suite_ternary_op)


def suite_three_way_and(outfield: F64, *, a: float, b: float, c: float):
    with computation(PARALLEL), interval(...):
        if a > 0 and b > 0 and c > 0:
            outfield = 1
        else:
            outfield = 0


def suite_three_way_or(outfield: F64, *, a: float, b: float, c: float):
    with computation(PARALLEL), interval(...):
        if a > 0 or b > 0 or c > 0:
            outfield = 1
        else:
            outfield = 0


case("suite_three_way_and", fields={"outfield": fs(4, 4, 3)}, params={"a": 1.0, "b": 2.0, "c": 3.0})(suite_three_way_and)
case("suite_three_way_or", fields={"outfield": fs(4, 4, 3)}, params={"a": -1.0, "b": -2.0, "c": 3.0})(suite_three_way_or)


def optional_field(in_field: F64, out_field: F64, dyn_tend: F64, phys_tend: F64 = None, *, dt: float):
    from __externals__ import PHYS_TEND

    with computation(PARALLEL), interval(...):
        out_field = in_field + dt * dyn_tend
        if __INLINED(PHYS_TEND):
            out_field = out_field + dt * phys_tend


case(
    "optional_field_used",
    fields={"in_field": fs(7, 6, 5), "out_field": fs(7, 6, 5), "dyn_tend": fs(7, 6, 5), "phys_tend": fs(7, 6, 5)},
    params={"dt": 0.5},
    externals={"PHYS_TEND": True},
)(optional_field)
case(
    "optional_field_unused",
    fields={"in_field": fs(7, 6, 5), "out_field": fs(7, 6, 5), "dyn_tend": fs(7, 6, 5), "phys_tend": None},
    params={"dt": 0.5},
    externals={"PHYS_TEND": False},
)(optional_field)


# --------------------------------------------------------------------------------------
# stencil_definitions.py programs
# --------------------------------------------------------------------------------------


def arithmetic_ops(field_a: F64, field_b: F64):
    with computation(PARALLEL), interval(...):
        field_a = (((((field_b + 42.0) - 42.0) * +42.0) / -42.0) % 42.0) ** 2


case("arithmetic_ops", fields={"field_a": fs(6, 5, 4), "field_b": fs(6, 5, 4)})(arithmetic_ops)


def scalar_inputs(field_a: F64, scalar_in: float):
    with computation(PARALLEL), interval(...):
        field_a = field_a * scalar_in


case("scalar_inputs", fields={"field_a": fs(6, 5, 4)}, params={"scalar_in": 1.5})(scalar_inputs)


def unary_operation(field_a: F64, scalar_in: float):
    with computation(PARALLEL), interval(...):
        field_a = -scalar_in


case("unary_operation", fields={"field_a": fs(6, 5, 4)}, params={"scalar_in": 2.75})(unary_operation)


def temporary_stencil(field_a: F64, field_b: F2D, scalar_in: float):
    with computation(PARALLEL), interval(...):
        tmp = field_a * scalar_in

    with computation(FORWARD), interval(0, 1):
        field_b += tmp


case(
    "temporary_stencil",
    fields={"field_a": fs(6, 5, 4), "field_b": fs(6, 5)},
    params={"scalar_in": 3.0},
    features=("2d",),
)(temporary_stencil)


@gtscript.function
def a_gtscript_function(b):
    return sqrt(abs(b[0, 1, 0]))


def native_functions(field_a: F64, field_b: F64):
    with computation(PARALLEL), interval(...):
        abs_res = abs(field_a)
        max_res = max(abs_res, 1.0)
        min_res = min(max_res, 42)
        mod_res = mod(min_res, 37.5)
        sin_res = sin(mod_res)
        asin_res = asin(sin_res)
        cos_res = cos(asin_res)
        acos_res = acos(cos_res)
        tan_res = tan(acos_res)
        atan_res = atan(tan_res)
        sinh_res = sinh(atan_res)
        asinh_res = asinh(sinh_res)
        cosh_res = cosh(asinh_res)
        acosh_res = acosh(cosh_res)
        tanh_res = tanh(acosh_res)
        atanh_res = atanh(tanh_res)
        sqrt_res = a_gtscript_function(atanh_res)
        pow10_res = 10 ** (sqrt_res)
        log10_res = log10(pow10_res)
        exp_res = exp(log10_res)
        log_res = log(exp_res)
        gamma_res = gamma(log_res)
        cbrt_res = cbrt(gamma_res)
        floor_res = floor(cbrt_res)
        ceil_res = ceil(floor_res)
        trunc_res = trunc(ceil_res)
        round_res = round(trunc_res)
        round_afz_res = round_away_from_zero(round_res)
        erf_res = erf(round_afz_res)
        erfc_res = erfc(erf_res)
        field_b = (
            trunc_res
            if isfinite(erfc_res)
            else field_a
            if isinf(erfc_res)
            else field_b
            if isnan(erfc_res)
            else 0.0
        )


case(
    "native_functions",
    fields={"field_a": fs(6, 6, 4), "field_b": fs(6, 5, 4)},
    domain=(6, 5, 4),
    rtol=1e-12,
    atol=1e-12,
)(native_functions)


def math_chain(field_a: F64, field_b: F64):
    with computation(PARALLEL), interval(...):
        field_b = sqrt(abs(field_a)) + exp(field_a * 0.1) - log(abs(field_a) + 1.0) + sin(field_a) * cos(field_a)


case("math_chain", fields={"field_a": fs(8, 6, 4), "field_b": fs(8, 6, 4)}, rtol=1e-13, atol=1e-13)(math_chain)


def while_stencil(field_a: F64, field_b: F64):
    with computation(BACKWARD), interval(...):
        while field_a > 2.0:
            field_b = -1
            field_a = -field_b


case("while_stencil", fields={"field_a": fs(6, 5, 4), "field_b": fs(6, 5, 4)})(while_stencil)


def copy_stencil_plus_one(field_a: F64, field_b: F64):
    with computation(PARALLEL), interval(...):
        field_b = field_a[0, 0, 0] + 1


case("copy_stencil_plus_one", fields={"field_a": fs(6, 5, 4), "field_b": fs(6, 5, 4)})(copy_stencil_plus_one)


def runtime_if(field_a: F64, field_b: F64):
    with computation(BACKWARD), interval(...):
        if field_a > 0.0:
            field_b = -1
            field_a = -field_a
        else:
            field_b = 1
            field_a = field_a


case("runtime_if", fields={"field_a": fs(6, 5, 4), "field_b": fs(6, 5, 4)})(runtime_if)


def simple_horizontal_diffusion(in_field: F64, coeff: F64, out_field: F64):
    with computation(PARALLEL), interval(...):
        lap_field = 4.0 * in_field[0, 0, 0] - (
            in_field[1, 0, 0] + in_field[-1, 0, 0] + in_field[0, 1, 0] + in_field[0, -1, 0]
        )
        flx_field = lap_field[1, 0, 0] - lap_field[0, 0, 0]
        fly_field = lap_field[0, 1, 0] - lap_field[0, 0, 0]
        out_field = in_field[0, 0, 0] - coeff[0, 0, 0] * (
            flx_field[0, 0, 0] - flx_field[-1, 0, 0] + fly_field[0, 0, 0] - fly_field[0, -1, 0]
        )


case(
    "simple_horizontal_diffusion",
    fields={"in_field": fs(16, 14, 5), "coeff": fs(12, 10, 5, init=("u", 0.0, 0.5)), "out_field": fs(12, 10, 5)},
    origin={"in_field": (2, 2, 0), "coeff": (0, 0, 0), "out_field": (0, 0, 0)},
    domain=(12, 10, 5),
)(simple_horizontal_diffusion)


def vertical_advection_dycore(
    utens_stage: F64,
    u_stage: F64,
    wcon: F64,
    u_pos: F64,
    utens: F64,
    *,
    dtr_stage: float,
):
    from __externals__ import BET_M, BET_P

    with computation(FORWARD):
        with interval(0, 1):
            gcv = 0.25 * (wcon[1, 0, 1] + wcon[0, 0, 1])
            cs = gcv * BET_M

            ccol = gcv * BET_P
            bcol = dtr_stage - ccol[0, 0, 0]

            correction_term = -cs * (u_stage[0, 0, 1] - u_stage[0, 0, 0])
            dcol = dtr_stage * u_pos[0, 0, 0] + utens[0, 0, 0] + utens_stage[0, 0, 0] + correction_term

            divided = 1.0 / bcol[0, 0, 0]
            ccol = ccol[0, 0, 0] * divided
            dcol = dcol[0, 0, 0] * divided

        with interval(1, -1):
            gav = -0.25 * (wcon[1, 0, 0] + wcon[0, 0, 0])
            gcv = 0.25 * (wcon[1, 0, 1] + wcon[0, 0, 1])

            as_ = gav * BET_M
            cs = gcv * BET_M

            acol = gav * BET_P
            ccol = gcv * BET_P
            bcol = dtr_stage - acol[0, 0, 0] - ccol[0, 0, 0]

            correction_term = -as_ * (u_stage[0, 0, -1] - u_stage[0, 0, 0]) - cs * (
                u_stage[0, 0, 1] - u_stage[0, 0, 0]
            )
            dcol = dtr_stage * u_pos[0, 0, 0] + utens[0, 0, 0] + utens_stage[0, 0, 0] + correction_term

            divided = 1.0 / (bcol[0, 0, 0] - ccol[0, 0, -1] * acol[0, 0, 0])
            ccol = ccol[0, 0, 0] * divided
            dcol = (dcol[0, 0, 0] - (dcol[0, 0, -1]) * acol[0, 0, 0]) * divided

        with interval(-1, None):
            gav = -0.25 * (wcon[1, 0, 0] + wcon[0, 0, 0])
            as_ = gav * BET_M
            acol = gav * BET_P
            bcol = dtr_stage - acol[0, 0, 0]

            correction_term = -as_ * (u_stage[0, 0, -1] - u_stage[0, 0, 0])
            dcol = dtr_stage * u_pos[0, 0, 0] + utens[0, 0, 0] + utens_stage[0, 0, 0] + correction_term

            divided = 1.0 / (bcol[0, 0, 0] - ccol[0, 0, -1] * acol[0, 0, 0])
            dcol = (dcol[0, 0, 0] - (dcol[0, 0, -1]) * acol[0, 0, 0]) * divided

    with computation(BACKWARD):
        with interval(-1, None):
            datacol = dcol[0, 0, 0]
            utens_stage = dtr_stage * (datacol - u_pos[0, 0, 0])

        with interval(0, -1):
            datacol = dcol[0, 0, 0] - ccol[0, 0, 0] * datacol[0, 0, 1]
            utens_stage = dtr_stage * (datacol - u_pos[0, 0, 0])


case(
    "vertical_advection_dycore",
    fields={
        "utens_stage": fs(8, 7, 10),
        "u_stage": fs(8, 7, 10),
        "wcon": fs(9, 7, 11, init=("u", -1.0, 1.0)),
        "u_pos": fs(8, 7, 10),
        "utens": fs(8, 7, 10),
    },
    params={"dtr_stage": 3.0 / 20.0},
    externals={"BET_M": 0.5, "BET_P": 0.5},
    domain=(8, 7, 10),
)(vertical_advection_dycore)


def large_k_interval(in_field: F64, out_field: F64):
    with computation(PARALLEL):
        with interval(0, 6):
            out_field = in_field
        with interval(6, -10):
            out_field = in_field + 1
        with interval(-10, None):
            out_field = in_field


case("large_k_interval", fields={"in_field": fs(5, 4, 20), "out_field": fs(5, 4, 20)})(large_k_interval)


def single_level_with_offset(in_field: F64, out_field: F64):
    with computation(PARALLEL), interval(1, 2):
        out_field = in_field


case("single_level_with_offset", fields={"in_field": fs(5, 4, 6), "out_field": fs(5, 4, 6)})(single_level_with_offset)


def form_land_mask(in_field: F64, mask: FBool):
    with computation(PARALLEL), interval(...):
        mask = in_field >= 0


case("form_land_mask", fields={"in_field": fs(6, 5, 4), "mask": fs(6, 5, 4, dtype="?", init="bool")})(form_land_mask)


def set_inner_as_kord(a4_1: F64, a4_2: F64, a4_3: F64, extm: FBool):
    with computation(PARALLEL), interval(...):
        diff_23 = 0.0
        if extm and extm[0, 0, -1]:
            a4_2 = a4_1
        elif extm and extm[0, 0, 1]:
            a4_3 = a4_1
        else:
            diff_23 = a4_2 - a4_3


case(
    "set_inner_as_kord",
    fields={"a4_1": fs(6, 5, 8), "a4_2": fs(6, 5, 8), "a4_3": fs(6, 5, 8), "extm": fs(6, 5, 10, dtype="?", init="bool")},
    origin={"a4_1": (0, 0, 0), "a4_2": (0, 0, 0), "a4_3": (0, 0, 0), "extm": (0, 0, 1)},
    domain=(6, 5, 8),
)(set_inner_as_kord)


def local_var_inside_nested_conditional(in_storage: F64, out_storage: F64):
    with computation(PARALLEL), interval(0, 2):
        mid_storage = 2
        if in_storage[0, 0, 0] > 0:
            local_var = 4
            if local_var + in_storage < out_storage:
                mid_storage = 3
            else:
                mid_storage = 4
            out_storage[0, 0, 0] = local_var + mid_storage
    with computation(FORWARD), interval(2, None):
        if in_storage[0, 0, 0] < 0:
            local_var = 6
            out_storage[0, 0, 0] = local_var


case(
    "local_var_inside_nested_conditional",
    fields={"in_storage": fs(6, 5, 6), "out_storage": fs(6, 5, 6)},
)(local_var_inside_nested_conditional)


def multibranch_param_conditional(in_field: F64, out_field: F64, c: float):
    with computation(PARALLEL), interval(...):
        if c > 0.0:
            out_field = in_field + in_field[1, 0, 0]
        elif c < -1.0:
            out_field = in_field - in_field[1, 0, 0]
        else:
            out_field = in_field


for _c, _tag in ((1.0, "pos"), (-2.0, "neg"), (-0.5, "mid")):
    case(
        f"multibranch_param_conditional_{_tag}",
        fields={"in_field": fs(7, 5, 4), "out_field": fs(6, 5, 4)},
        params={"c": _c},
        domain=(6, 5, 4),
    )(multibranch_param_conditional)


def allow_empty_computation(in_field: F64, out_field: F64):
    from __externals__ import DO_SOMETHING

    with computation(FORWARD), interval(...):
        out_field = in_field
    with computation(PARALLEL), interval(...):
        if __INLINED(DO_SOMETHING):
            out_field = abs(in_field)


case(
    "allow_empty_computation",
    fields={"in_field": fs(6, 5, 4), "out_field": fs(6, 5, 4)},
    externals={"DO_SOMETHING": False},
)(allow_empty_computation)


def two_optional_fields(
    in_a: F64,
    in_b: F64,
    out_a: F64,
    out_b: F64,
    dyn_tend_a: F64,
    dyn_tend_b: F64,
    phys_tend_a: F64 = None,
    phys_tend_b: F64 = None,
    *,
    dt: float,
):
    from __externals__ import PHYS_TEND_A, PHYS_TEND_B

    with computation(PARALLEL), interval(...):
        out_a = in_a + dt * dyn_tend_a
        out_b = in_b + dt * dyn_tend_b
        if __INLINED(PHYS_TEND_A):
            out_a = out_a + dt * phys_tend_a
        if __INLINED(PHYS_TEND_B):
            out_b = out_b + dt * phys_tend_b


for _pa, _pb in ((False, False), (False, True), (True, True)):
    case(
        f"two_optional_fields_{int(_pa)}{int(_pb)}",
        fields={
            "in_a": fs(5, 4, 3),
            "in_b": fs(5, 4, 3),
            "out_a": fs(5, 4, 3),
            "out_b": fs(5, 4, 3),
            "dyn_tend_a": fs(5, 4, 3),
            "dyn_tend_b": fs(5, 4, 3),
            "phys_tend_a": fs(5, 4, 3) if _pa else None,
            "phys_tend_b": fs(5, 4, 3) if _pb else None,
        },
        params={"dt": 0.25},
        externals={"PHYS_TEND_A": _pa, "PHYS_TEND_B": _pb},
    )(two_optional_fields)


def horizontal_regions(field_in: F64, field_out: F64):
    with computation(PARALLEL), interval(...):
        with horizontal(region[I[0] : I[0] + 2, J[0] : J[0] + 2], region[I[-1] - 2 : I[-1], J[-1] - 2 : J[-1]]):
            field_out = field_in + 1.0

        with horizontal(region[I[0] : I[0] + 2, J[-1] - 2 : J[-1]], region[I[-1] - 2 : I[-1], J[0] : J[0] + 2]):
            field_out = field_in - 1.0


case(
    "horizontal_regions",
    fields={"field_in": fs(8, 7, 3), "field_out": fs(8, 7, 3)},
    features=("regions",),
)(horizontal_regions)


def mixed_precision(a: F32, b: F64, out32: F32, out64: F64):
    with computation(PARALLEL), interval(...):
        t32 = a + 1
        t64 = a * 2.0 + b
        out32 = t32 * a - b
        out64 = t64 / (a + 3) + t32


def exact_products(a: F32, b: F64, c: F32, n: Field[np.int32], o1: F64, o2: F64, o3: F32, o4: F64):
    """f64 adds and subtractions of exact products -- a power-of-two literal times a value widened
    from f32 or int32 -- which gt:mi355x renders as one fma (codegen/common.py ``exact_fma``), on
    IEEE edge values: signed zeros, denormals, the largest finite values, NaN and infinities."""
    with computation(PARALLEL), interval(...):
        o1 = 4.0 * a - b
        o2 = b - 0.5 * c
        o3 = 2.0 * a + c
        o4 = b + n * 8.0


case(
    "exact_products",
    fields={"a": fs(11, 7, 6, dtype="f4", init=("special", -3.0, 3.0, 0.5)),
            "b": fs(11, 7, 6, init=("special", -3.0, 3.0, 0.5)),
            "c": fs(11, 7, 6, dtype="f4", init=("special", -3.0, 3.0, 0.5)),
            "n": fs(11, 7, 6, dtype="i4", init=("int", -2**31, 2**31 - 1)),
            "o1": fs(11, 7, 6, init="zeros"), "o2": fs(11, 7, 6, init="zeros"),
            "o3": fs(11, 7, 6, dtype="f4", init="zeros"), "o4": fs(11, 7, 6, init="zeros")},
)(exact_products)


case(
    "mixed_precision",
    fields={"a": fs(7, 6, 5, dtype="f4"), "b": fs(7, 6, 5), "out32": fs(7, 6, 5, dtype="f4"), "out64": fs(7, 6, 5)},
)(mixed_precision)


def kcache_forward_backward(a: F64, b: F64, c: F64):
    with computation(FORWARD):
        with interval(0, 1):
            tmp = a
            b = tmp
        with interval(1, None):
            tmp = a + 0.5 * tmp[0, 0, -1]
            b = tmp * b[0, 0, -1]
    with computation(BACKWARD):
        with interval(-1, None):
            c = tmp
        with interval(0, -1):
            c = tmp - 0.25 * c[0, 0, 1] + a[0, 0, 1]


case(
    "kcache_forward_backward",
    fields={"a": fs(6, 5, 9, init=("u", -1.0, 1.0)), "b": fs(6, 5, 9, init=("u", -1.0, 1.0)), "c": fs(6, 5, 9)},
)(kcache_forward_backward)


def parallel_koffsets(a: F64, b: F64):
    with computation(PARALLEL):
        with interval(0, 1):
            b = a[0, 0, 1] - a
        with interval(1, -1):
            b = a[0, 0, 1] - 2.0 * a + a[0, 0, -1]
        with interval(-1, None):
            b = a[0, 0, -1] - a


case("parallel_koffsets", fields={"a": fs(6, 5, 7), "b": fs(6, 5, 7)})(parallel_koffsets)


def multi_stage_temps(a: F64, out: F64, *, alpha: float):
    with computation(PARALLEL), interval(...):
        t1 = a[1, 0, 0] - a[-1, 0, 0]
        t2 = a[0, 1, 0] - a[0, -1, 0]
        t3 = t1[0, 1, 0] + t2[1, 0, 0] + alpha * t1[0, -1, 0] * t2[-1, 0, 0]
        out = t3[1, 1, 0] - t3[-1, -1, 0] + t3


case(
    "multi_stage_temps",
    fields={"a": fs(15, 13, 4), "out": fs(11, 9, 4)},
    params={"alpha": 0.5},
    origin={"a": (2, 2, 0), "out": (0, 0, 0)},
    domain=(11, 9, 4),
)(multi_stage_temps)


# --------------------------------------------------------------------------------------
# Temporaries produced by a column kernel on an IJ halo, lower-dimensional fields
# (test_code_generation.py:171-307, 868-891)
# --------------------------------------------------------------------------------------


def column_temp_halo(a: F64, out: F64):
    with computation(PARALLEL):
        with interval(0, -1):
            tmp = a[0, 0, 1] * 2.0 - a
        with interval(-1, None):
            tmp = a
    with computation(PARALLEL), interval(...):
        out = tmp[1, 0, 0] - tmp[-1, 0, 0] + tmp[0, 1, 0] * tmp[0, -1, 0]


case(
    "column_temp_halo",
    fields={"a": fs(12, 11, 6), "out": fs(10, 9, 6, init="zeros")},
    origin={"a": (1, 1, 0), "out": (0, 0, 0)},
    domain=(10, 9, 6),
)(column_temp_halo)


def forward_temp_halo(a: F64, out: F64):
    with computation(FORWARD):
        with interval(0, 1):
            acc = a
        with interval(1, None):
            acc = acc[0, 0, -1] * 0.5 + a
    with computation(PARALLEL), interval(...):
        out = acc[1, 0, 0] + acc[0, -1, 0] - acc[-1, 1, 0]


case(
    "forward_temp_halo",
    fields={"a": fs(12, 11, 7), "out": fs(10, 9, 7, init="zeros")},
    origin={"a": (1, 1, 0), "out": (0, 0, 0)},
    domain=(10, 9, 7),
)(forward_temp_halo)


F1DK = Field[gtscript.K, np.float64]
F3D = Field[gtscript.IJK, np.float64]


def lowdim_inputs(field_3d: F3D, field_2d: F2D, field_1d: F1DK):
    with computation(PARALLEL):
        with interval(0, -1):
            tmp = field_2d + field_1d[1]
        with interval(-1, None):
            tmp = field_2d + field_1d[0]
    with computation(PARALLEL):
        with interval(0, 1):
            field_3d = tmp[1, 0, 0] + field_1d[1]
        with interval(1, None):
            field_3d[0, 0, 0] = tmp[-1, 0, 0]


case(
    "lowdim_inputs",
    fields={"field_3d": fs(6, 6, 6, init="zeros"), "field_2d": fs(6, 6), "field_1d": fs(6)},
    origin=(1, 1, 0),
    domain=(4, 3, 6),
)(lowdim_inputs)


def lowdim_masked(cond: F3D, inp: F2D, outp: F3D):
    with computation(PARALLEL), interval(...):
        if cond > 0.0:
            outp[0, 0, 0] = inp


case("lowdim_masked", fields={"cond": fs(10, 10, 10), "inp": fs(10, 10), "outp": fs(10, 10, 10)})(lowdim_masked)


def lowdim_masked_forward(cond: F3D, inp: F2D, outp: F3D):
    with computation(FORWARD), interval(...):
        if cond > 0.0:
            outp[0, 0, 0] = inp


case(
    "lowdim_masked_forward", fields={"cond": fs(10, 10, 10), "inp": fs(10, 10), "outp": fs(10, 10, 10)}
)(lowdim_masked_forward)


def k_only_access(in_field: F1DK, out_field: F64):
    with computation(PARALLEL):
        with interval(0, 1):
            out_field[0, 0, 0] = in_field[1]
        with interval(1, None):
            out_field[0, 0, 0] = in_field[-1]


case("k_only_access", fields={"in_field": fs(5), "out_field": fs(4, 4, 5, init="zeros")})(k_only_access)


def lowdim_2d_output(a: F64, colsum: F2D):
    with computation(FORWARD):
        with interval(0, 1):
            colsum = a
        with interval(1, None):
            colsum = colsum + a


case("lowdim_2d_output", fields={"a": fs(7, 6, 5), "colsum": fs(7, 6, init="zeros")})(lowdim_2d_output)


# --------------------------------------------------------------------------------------
# Data dimensions, variable / written K offsets, global tables
# (test_code_generation.py:309-361, 387-427, 463-510, 664-716, 815-1094, 1137-1222, 1604-1619)
# --------------------------------------------------------------------------------------

V2 = (np.float64, (2,))
M22 = (np.float64, (2, 2))
I32V2 = (np.int32, (2,))
V4 = (np.float64, (4,))


def higher_dimensional_fields(field: F64, vec_field: Field[V2], mat_field: Field[M22]):
    with computation(PARALLEL), interval(...):
        tmp = vec_field[0, 0, 0][0] + vec_field[0, 0, 0][1]  # noqa: F841
    with computation(FORWARD):
        with interval(0, 1):
            vec_field[0, 0, 0][0] = field[1, 0, 0]
            vec_field[0, 0, 0][1] = field[0, 1, 0]
        with interval(1, -1):
            vec_field[0, 0, 0][0] = 2 * field[1, 0, -1]
            vec_field[0, 0, 0][1] = 2 * field[0, 1, -1]
        with interval(-1, None):
            vec_field[0, 0, 0][0] = field[1, 0, 0]
            vec_field[0, 0, 0][1] = field[0, 1, 0]
    with computation(PARALLEL), interval(...):
        mat_field[0, 0, 0][0, 0] = vec_field[0, 0, 0][0] + 1.0
        mat_field[0, 0, 0][1, 1] = vec_field[0, 0, 0][1] + 1.0


case(
    "higher_dimensional_fields",
    fields={"field": fs(6, 6, 6), "vec_field": fs(6, 6, 6, 2), "mat_field": fs(6, 6, 6, 2, 2)},
    origin=(1, 1, 0),
    domain=(4, 4, 6),
)(higher_dimensional_fields)


def data_dim_stencil(vec_field: Field[V4], out_field: F64, *, idx: int):
    with computation(PARALLEL), interval(...):
        out_field[0, 0, 0] = vec_field[0, 0, 0][2] * vec_field[1, 0, 0][idx] - vec_field[0, -1, 0][3]


case(
    "data_dim_stencil",
    fields={"vec_field": fs(8, 7, 5, 4), "out_field": fs(8, 7, 5, init="zeros")},
    params={"idx": 1},
    origin={"vec_field": (0, 1, 0, 0), "out_field": (0, 1, 0)},
    domain=(7, 6, 5),
)(data_dim_stencil)


def data_dim_write_index(input_field: Field[gtscript.IJK, np.int32], output_field: Field[gtscript.IJK, I32V2], *, index: int):
    with computation(PARALLEL), interval(...):
        output_field[0, 0, 0][index] = input_field


case(
    "data_dim_write_index",
    fields={"input_field": fs(3, 2, 4, dtype="i4", init=("int", -50, 50)),
            "output_field": fs(3, 2, 4, 2, dtype="i4", init=("int", -5, 5))},
    params={"index": 1},
)(data_dim_write_index)


def data_dim_read_index(input_field: Field[gtscript.IJK, I32V2], output_field: Field[gtscript.IJK, np.int32], *, index: int):
    with computation(PARALLEL), interval(...):
        output_field[0, 0, 0] = input_field[0, 0, 0][index]


case(
    "data_dim_read_index",
    fields={"input_field": fs(3, 2, 4, 2, dtype="i4", init=("int", -50, 50)),
            "output_field": fs(3, 2, 4, dtype="i4", init="zeros")},
    params={"index": 1},
)(data_dim_read_index)


def variable_offsets_ij(in_field: F64, out_field: F64, index_field: Field[gtscript.IJ, np.int64]):
    with computation(FORWARD), interval(...):
        out_field[0, 0, 0] = in_field[0, 0, 1] + in_field[0, 0, index_field + 1]
        index_field = index_field + 1


case(
    "variable_offsets_ij",
    fields={"in_field": fs(5, 4, 12), "out_field": fs(5, 4, 12, init="zeros"),
            "index_field": fs(5, 4, dtype="i8", init=("const", -3))},
    domain=(5, 4, 6),
)(variable_offsets_ij)


def variable_offsets_ijk(in_field: F64, out_field: F64, index_field: Field[np.int64]):
    with computation(PARALLEL), interval(...):
        out_field[0, 0, 0] = in_field[0, 0, 1] + in_field[0, 0, index_field + 1]


case(
    "variable_offsets_ijk",
    fields={"in_field": fs(5, 4, 10), "out_field": fs(5, 4, 10, init="zeros"),
            "index_field": fs(5, 4, 10, dtype="i8", init=("int", -2, 3))},
    origin=(0, 0, 2),
    domain=(5, 4, 5),
)(variable_offsets_ijk)


def variable_offsets_and_while_loop(pe1: F64, pe2: F64, qin: F64, qout: F64, lev: Field[gtscript.IJ, np.int64]):
    with computation(FORWARD), interval(0, -1):
        if pe2[0, 0, 1] <= pe1[0, 0, lev]:
            qout = qin[0, 0, 1]
        else:
            qsum = pe1[0, 0, lev + 1] - pe2[0, 0, lev]
            while pe1[0, 0, lev + 1] < pe2[0, 0, 1]:
                qsum += qin[0, 0, lev] / (pe2[0, 0, 1] - pe1[0, 0, lev])
                lev = lev + 1
            qout[0, 0, 0] = qsum / (pe2[0, 0, 1] - pe2)


case(
    "variable_offsets_and_while_loop",
    fields={"pe1": fs(4, 3, 8, init=("ramp", 0.0, 1.0)), "pe2": fs(4, 3, 8, init=("ramp", 0.05, 0.9)),
            "qin": fs(4, 3, 8), "qout": fs(4, 3, 8, init="zeros"),
            "lev": fs(4, 3, dtype="i8", init=("const", 0))},
)(variable_offsets_and_while_loop)


def variable_k_offset_ij_dropped(in_field: F64, out_field: F64, idx: Field[np.int64]):
    # the reference keeps only the K part of an offset whose K entry is an expression
    # (defir_to_gtir.py:626-639): in_field[1, -1, expr] reads in_field[0, 0, expr]
    with computation(PARALLEL), interval(1, -1):
        out_field[0, 0, 0] = in_field[1, -1, (idx % 3) - 1] + in_field[0, 0, 0]


case(
    "variable_k_offset_ij_dropped",
    fields={"in_field": fs(6, 5, 7), "out_field": fs(6, 5, 7, init="zeros"),
            "idx": fs(6, 5, 7, dtype="i8", init=("int", -4, 5))},
)(variable_k_offset_ij_dropped)


def k_offset_scalar(in_field: F64, out_field: F64, scalar_value: int):
    with computation(PARALLEL), interval(1, None):
        out_field[0, 0, 0] = in_field[0, 0, scalar_value]


case(
    "k_offset_scalar",
    fields={"in_field": fs(4, 4, 4), "out_field": fs(4, 4, 4, init="zeros")},
    params={"scalar_value": -1},
)(k_offset_scalar)


def k_offset_field(in_field: F64, out_field: F64, idx_field: Field[gtscript.IJ, np.int64]):
    with computation(PARALLEL), interval(1, None):
        out_field[0, 0, 0] = in_field[0, 0, idx_field + 1]


case(
    "k_offset_field",
    fields={"in_field": fs(4, 4, 4), "out_field": fs(4, 4, 4, init="zeros"),
            "idx_field": fs(4, 4, dtype="i8", init=("int", -2, 1))},
)(k_offset_field)


def k_offset_write_simple(A: F64, B: F64):
    with computation(FORWARD), interval(...):
        B[0, 0, 1] = A


case("k_offset_write_simple", fields={"A": fs(3, 2, 4), "B": fs(3, 2, 4, init="zeros")}, domain=(3, 2, 3))(
    k_offset_write_simple
)


def k_offset_write_forward(A: F64, B: F64, scalar: np.float64):
    with computation(FORWARD), interval(1, None):
        A[0, 0, -1] = scalar
        B[0, 0, 0] = A


case("k_offset_write_forward", fields={"A": fs(3, 2, 5), "B": fs(3, 2, 5, init="zeros")}, params={"scalar": 2.0})(
    k_offset_write_forward
)


def k_offset_write_backward(A: F64, B: F64, scalar: np.float64):
    with computation(BACKWARD), interval(-1, None):
        A = scalar
    with computation(BACKWARD), interval(1, None):
        A[0, 0, -1] = scalar
        B[0, 0, 0] = A


case("k_offset_write_backward", fields={"A": fs(3, 2, 5), "B": fs(3, 2, 5, init="zeros")}, params={"scalar": 2.0})(
    k_offset_write_backward
)


def k_offset_write_conditional(A: F64, B: F64, scalar: np.float64):
    with computation(BACKWARD), interval(1, -1):
        if A > 0 and B > 0:
            A[0, 0, -1] = scalar
            B[0, 0, 1] = A
        lev = 1
        while A >= 0 and B >= 0:
            A[0, 0, lev] = -1
            B = -1
            lev = lev + 1


case(
    "k_offset_write_conditional",
    fields={"A": fs(3, 2, 4, init=("ramp", 40.0, 44.0)), "B": fs(3, 2, 4, init=("const", 1.0))},
    params={"scalar": 2.0},
)(k_offset_write_conditional)


def cast_in_index(in_field: F64, i32: np.int32, i64: np.int64, out_field: F64):
    with computation(PARALLEL), interval(...):
        out_field[0, 0, 0] = in_field[0, 0, i32 - i64]


case(
    "cast_in_index",
    fields={"in_field": fs(4, 3, 8), "out_field": fs(4, 3, 8, init="zeros")},
    params={"i32": np.int32(3), "i64": np.int64(1)},
    domain=(4, 3, 6),
)(cast_in_index)


def upcasting_k_index_write(in_field: F64, index_field: Field[gtscript.IJ, np.int32], out_field: F64):
    with computation(FORWARD), interval(...):
        out_field[0, 0, index_field - 1] = in_field


case(
    "upcasting_k_index_write",
    fields={"in_field": fs(5, 5, 5), "index_field": fs(5, 5, dtype="i4", init=("const", 1)),
            "out_field": fs(5, 5, 5, init="zeros")},
)(upcasting_k_index_write)


def lagrangian_contributions(q: F64, pe1: F64, pe2: F64, q4_1: F64, q4_2: F64, q4_3: F64, q4_4: F64, dp1: F64,
                             lev: Field[gtscript.IJ, np.int64]):
    with computation(FORWARD), interval(...):
        pl = (pe2 - pe1[0, 0, lev]) / dp1[0, 0, lev]
        if pe2[0, 0, 1] <= pe1[0, 0, lev + 1]:
            pr = (pe2[0, 0, 1] - pe1[0, 0, lev]) / dp1[0, 0, lev]
            q[0, 0, 0] = (
                q4_2[0, 0, lev]
                + 0.5 * (q4_4[0, 0, lev] + q4_3[0, 0, lev] - q4_2[0, 0, lev]) * (pr + pl)
                - q4_4[0, 0, lev] * 1.0 / 3.0 * (pr * (pr + pl) + pl * pl)
            )
        else:
            qsum = (pe1[0, 0, lev + 1] - pe2) * (
                q4_2[0, 0, lev]
                + 0.5 * (q4_4[0, 0, lev] + q4_3[0, 0, lev] - q4_2[0, 0, lev]) * (1.0 + pl)
                - q4_4[0, 0, lev] * 1.0 / 3.0 * (1.0 + pl * (1.0 + pl))
            )
            lev = lev + 1
            while pe1[0, 0, lev + 1] < pe2[0, 0, 1]:
                qsum += dp1[0, 0, lev] * q4_1[0, 0, lev]
                lev = lev + 1
            dp = pe2[0, 0, 1] - pe1[0, 0, lev]
            esl = dp / dp1[0, 0, lev]
            qsum += dp * (
                q4_2[0, 0, lev]
                + 0.5 * esl * (q4_3[0, 0, lev] - q4_2[0, 0, lev] + q4_4[0, 0, lev] * (1.0 - (2.0 / 3.0) * esl))
            )
            q = qsum / (pe2[0, 0, 1] - pe2)
        lev = lev - 1


case(
    "lagrangian_contributions",
    fields={"q": fs(4, 3, 10, init="zeros"), "pe1": fs(4, 3, 10, init=("ramp", 0.0, 1.0)),
            "pe2": fs(4, 3, 10, init=("ramp", 0.0, 0.95)), "q4_1": fs(4, 3, 10), "q4_2": fs(4, 3, 10),
            "q4_3": fs(4, 3, 10), "q4_4": fs(4, 3, 10), "dp1": fs(4, 3, 10, init=("u", 0.5, 1.5)),
            "lev": fs(4, 3, dtype="i8", init=("const", 0))},
    domain=(4, 3, 8),
)(lagrangian_contributions)


def table_access(table_view: gtscript.GlobalTable[(np.float64, (4,))], out_field: F64):
    with computation(PARALLEL):
        with interval(0, 1):
            out_field[0, 0, 0] = table_view.A[1]
        with interval(1, None):
            out_field[0, 0, 0] = table_view.A[2]


case("table_access", fields={"table_view": fs(4), "out_field": fs(4, 4, 4, init="zeros")})(table_access)


def direct_datadims_index(out: F64, inp: gtscript.GlobalTable[(np.float64, (2, 2, 2, 2))]):
    with computation(PARALLEL), interval(...):
        out[0, 0, 0] = inp.A[1, 0, 1, 0] + inp.A[0, 1, 1, 1]


case("direct_datadims_index", fields={"out": fs(2, 2, 2, init="zeros"), "inp": fs(2, 2, 2, 2)})(
    direct_datadims_index
)


# --------------------------------------------------------------------------------------
# Remaining StencilTestSuite definitions (test_suites.py:614-1160): lower-dimensional and
# data-dimension fields, reads outside the K interval, variable K reads, regions, typed and
# vector temporaries, vector/matrix expressions
# --------------------------------------------------------------------------------------


def suite_non3d_fields(
    field_in: Field[gtscript.K, np.float64],
    another_field: Field[gtscript.IJ, (np.float64, (3, 2, 2))],
    field_out: Field[gtscript.IJK, (np.float64, (3, 2))],
):
    with computation(PARALLEL), interval(...):
        field_out[0, 0, 0][0, 0] = field_in[0] + another_field[-1, -1][0, 0, 0] + another_field[-1, -1][0, 0, 1]
        field_out[0, 0, 0][0, 1] = 2 * (
            another_field[-1, -1][1, 0, 0]
            + another_field[-1, -1][1, 0, 1]
            + another_field[-1, -1][1, 1, 0]
            + another_field[-1, -1][1, 1, 1]
        )
        field_out[0, 0, 0][1, 0] = field_in[0] + another_field[1, 1][0, 0, 0] + another_field[1, 1][0, 0, 1]
        field_out[0, 0, 0][1, 1] = 3 * (
            another_field[1, 1][1, 0, 0]
            + another_field[1, 1][1, 0, 1]
            + another_field[1, 1][1, 1, 0]
            + another_field[1, 1][1, 1, 1]
        )
        field_out[0, 0, 0][2, 0] = field_in[0] + another_field[0, 0][0, 0, 0] + another_field[-1, 1][0, 0, 1]
        field_out[0, 0, 0][2, 1] = 4 * (
            another_field[-1, 1][1, 0, 0]
            + another_field[-1, 1][1, 0, 1]
            + another_field[-1, 1][1, 1, 0]
            + another_field[-1, 1][1, 1, 1]
        )


case(
    "suite_non3d_fields",
    fields={"field_in": fs(6), "another_field": fs(9, 7, 3, 2, 2), "field_out": fs(7, 5, 6, 3, 2)},
    origin={"field_in": (0,), "another_field": (1, 1), "field_out": (0, 0, 0)},
    domain=(7, 5, 6),
)(suite_non3d_fields)


def suite_read_outside_k1(field_in: F64, field_out: F64):
    with computation(PARALLEL), interval(...):
        field_out = field_in[0, 0, -1] + field_in[0, 0, 1]


case(
    "suite_read_outside_k1",
    fields={"field_in": fs(4, 4, 6), "field_out": fs(4, 4, 4)},
    origin={"field_in": (0, 0, 1), "field_out": (0, 0, 0)},
    domain=(4, 4, 4),
)(suite_read_outside_k1)


def suite_read_outside_k2(field_in: F64, field_out: F64):
    with computation(PARALLEL), interval(-1, None):
        field_out = field_in[0, 0, 1]


case(
    "suite_read_outside_k2",
    fields={"field_in": fs(4, 4, 5), "field_out": fs(4, 4, 4)},
    domain=(4, 4, 4),
)(suite_read_outside_k2)


def suite_read_outside_k3(field_in: F64, field_out: F64):
    with computation(PARALLEL), interval(0, 1):
        field_out = field_in[0, 0, -1]


case(
    "suite_read_outside_k3",
    fields={"field_in": fs(4, 4, 5), "field_out": fs(4, 4, 4)},
    origin={"field_in": (0, 0, 1), "field_out": (0, 0, 0)},
    domain=(4, 4, 4),
)(suite_read_outside_k3)


def suite_variable_k_read(
    field_in: Field[np.float32], field_out: Field[np.float32], index: Field[gtscript.K, np.int32]
):
    with computation(PARALLEL), interval(1, None):
        field_out = field_in[0, 0, index]


case(
    "suite_variable_k_read",
    fields={"field_in": fs(2, 2, 8, dtype="f4"), "field_out": fs(2, 2, 8, dtype="f4"),
            "index": fs(8, dtype="i4", init=("int", -1, 1))},
)(suite_variable_k_read)


def suite_variable_k_and_read_outside(field_in: F64, field_out: F64, index: Field[gtscript.K, np.int32]):
    with computation(PARALLEL), interval(1, None):
        field_out[0, 0, 0] = field_in[0, 0, index] + field_in[0, 0, -2]


case(
    "suite_variable_k_and_read_outside",
    fields={"field_in": fs(2, 2, 9, init=("u", 0.1, 10.0)), "field_out": fs(2, 2, 8, init=("u", 0.1, 10.0)),
            "index": fs(8, dtype="i4", init=("int", -1, 1))},
    origin={"field_in": (0, 0, 1), "field_out": (0, 0, 0), "index": (0,)},
    domain=(2, 2, 8),
)(suite_variable_k_and_read_outside)


def suite_diagonal_k_offset(field_in: F64, field_out: F64):
    with computation(PARALLEL), interval(...):
        field_out = field_in[0, 0, 1]
    with computation(PARALLEL), interval(0, -1):
        field_out += field_in[0, -1, 1]


case(
    "suite_diagonal_k_offset",
    fields={"field_in": fs(2, 3, 9, init=("u", 0.1, 10.0)), "field_out": fs(2, 2, 8)},
    origin={"field_in": (0, 1, 0), "field_out": (0, 0, 0)},
    domain=(2, 2, 8),
)(suite_diagonal_k_offset)


def suite_horizontal_regions(field_in: Field[np.float32], field_out: Field[np.float32]):
    with computation(PARALLEL), interval(...):
        field_out = field_in
        with horizontal(region[I[0], :], region[I[-1], :]):
            field_out = field_in + 1.0
        with horizontal(region[:, J[0]], region[:, J[-1]]):
            field_out = field_in - 1.0


case("suite_horizontal_regions", fields={"field_in": fs(4, 4, 2, dtype="f4"), "field_out": fs(4, 4, 2, dtype="f4")})(
    suite_horizontal_regions
)


def suite_horizontal_regions_partial(field_in: Field[np.float32], field_out: Field[np.float32]):
    with computation(PARALLEL), interval(...):
        with horizontal(region[I[0], :], region[I[-1], :]):
            field_out = field_in + 1.0
        with horizontal(region[:, J[0]], region[:, J[-1]]):
            field_out = field_in - 1.0


case(
    "suite_horizontal_regions_partial",
    fields={"field_in": fs(4, 4, 2, dtype="f4"), "field_out": fs(4, 4, 2, dtype="f4", init=("const", 42.0))},
)(suite_horizontal_regions_partial)


def suite_horizontal_regions_corners(field_in: Field[np.float32], field_out: Field[np.float32]):
    with computation(PARALLEL), interval(...):
        with horizontal(region[I[0] : I[0] + 2, J[0] : J[0] + 2], region[I[-1] - 2 : I[-1], J[-1] - 2 : J[-1]]):
            field_out = field_in + 1.0
        with horizontal(region[I[0] : I[0] + 2, J[-1] - 2 : J[-1]], region[I[-1] - 2 : I[-1], J[0] : J[0] + 2]):
            field_out = field_in - 1.0


case(
    "suite_horizontal_regions_corners",
    fields={"field_in": fs(6, 5, 2, dtype="f4"), "field_out": fs(6, 5, 2, dtype="f4", init=("const", 42.0))},
)(suite_horizontal_regions_corners)


def suite_typed_temporary(field_in: Field[np.float32], field_out: Field[np.float32]):
    tmp: Field[(np.float32, (2, 2))] = 0
    with computation(PARALLEL):
        with interval(0, -1):
            tmp[0, 0, 0][0, 0] = field_in[0, 0, 0]
            tmp[0, 0, 0][1, 0] = field_in[0, 0, 1]
            tmp[0, 0, 0][0, 1] = -1.0
            tmp[0, 0, 0][1, 1] = -1.0
            field_out = tmp[0, 0, 0][0, 0] + tmp[0, 0, 0][1, 0]
        with interval(-1, None):
            field_out = 0


case(
    "suite_typed_temporary", fields={"field_in": fs(2, 2, 8, dtype="f4"), "field_out": fs(2, 2, 8, dtype="f4")}
)(suite_typed_temporary)


F64V2 = Field[(np.float64, (2,))]
F32V2 = Field[(np.float32, (2,))]


def suite_vector_gen_assignment(field_in: F64V2, field_out: F64V2):
    with computation(PARALLEL), interval(...):
        field_out = 2 * field_in


case("suite_vector_gen_assignment", fields={"field_in": fs(3, 2, 2, 2), "field_out": fs(3, 2, 2, 2)})(
    suite_vector_gen_assignment
)


def suite_matrix_assignment(field_in: Field[(np.float32, (2, 3))], field_out: Field[(np.float32, (2, 3))]):
    with computation(PARALLEL), interval(...):
        field_out = field_in


case(
    "suite_matrix_assignment",
    fields={"field_in": fs(2, 2, 2, 2, 3, dtype="f4"), "field_out": fs(2, 2, 2, 2, 3, dtype="f4")},
)(suite_matrix_assignment)


def suite_vector_vector_op(field_1: F32V2, field_2: F32V2, field_out: F32V2):
    with computation(PARALLEL), interval(...):
        field_out = field_1 + field_2


case(
    "suite_vector_vector_op",
    fields={"field_1": fs(2, 2, 2, 2, dtype="f4"), "field_2": fs(2, 2, 2, 2, dtype="f4"),
            "field_out": fs(2, 2, 2, 2, dtype="f4")},
)(suite_vector_vector_op)


def suite_combined_vector_scalar_op(field_1: F64V2, field_2: F64V2, field_out: F64V2):
    with computation(PARALLEL), interval(...):
        field_out = 3 * (field_1 + field_2 * field_2)


case(
    "suite_combined_vector_scalar_op",
    fields={"field_1": fs(2, 2, 2, 2, init=("u", 1.0, 10.0)), "field_2": fs(2, 2, 2, 2, init=("u", 1.0, 10.0)),
            "field_out": fs(2, 2, 2, 2)},
)(suite_combined_vector_scalar_op)


def suite_vectorized_temporary(field_in: F32V2, field_out: F32V2):
    tmp: Field[(np.float32, (2,))] = 0
    with computation(PARALLEL), interval(...):
        tmp[0, 0, 0][0] = 2
        tmp[0, 0, 0][1] = 3
        field_out = tmp * field_in


case(
    "suite_vectorized_temporary",
    fields={"field_in": fs(2, 2, 2, 2, dtype="f4"), "field_out": fs(2, 2, 2, 2, dtype="f4")},
)(suite_vectorized_temporary)


def suite_matmul(matrix: Field[(np.float64, (4, 6))], field_1: Field[(np.float64, (6,))],
                 field_2: Field[(np.float64, (4,))]):
    with computation(PARALLEL):
        with interval(0, 1):
            field_2 = matrix @ field_1
        with interval(1, 2):
            field_1 = matrix.T @ field_2


case(
    "suite_matmul",
    fields={"matrix": fs(2, 2, 2, 4, 6), "field_1": fs(2, 2, 2, 6), "field_2": fs(2, 2, 2, 4)},
)(suite_matmul)


def suite_masked_matmul(matrix: Field[gtscript.K, (np.float64, (4, 6))], field_1: Field[(np.float64, (6,))],
                        field_2: Field[(np.float64, (4,))]):
    with computation(PARALLEL):
        with interval(0, 1):
            field_2 = matrix @ field_1
        with interval(1, 2):
            field_1 = matrix.T @ field_2


case(
    "suite_masked_matmul",
    fields={"matrix": fs(2, 4, 6), "field_1": fs(2, 2, 2, 6), "field_2": fs(2, 2, 2, 4)},
)(suite_masked_matmul)


# --------------------------------------------------------------------------------------
# Patterns the plane / single-column kernels cannot take directly: the staged lowering
# (phases + scratch temporaries, codegen/lowering.py split_phases)
# --------------------------------------------------------------------------------------


def staged_forward_ij_temp(a: F64, out: F64):
    with computation(FORWARD):
        with interval(0, 1):
            s = a
        with interval(1, None):
            s = s[0, 0, -1] * 0.5 + a
    with computation(FORWARD), interval(...):
        t = s * 2.0 + a
        out = t[1, 0, 0] - t[-1, 0, 0] + t[0, 1, 0] * s


case(
    "staged_forward_ij_temp",
    fields={"a": fs(12, 10, 6), "out": fs(10, 8, 6, init="zeros")},
    origin={"a": (1, 1, 0), "out": (0, 0, 0)},
    domain=(10, 8, 6),
)(staged_forward_ij_temp)


def staged_parallel_k_temp(a: F64, out: F64):
    with computation(PARALLEL), interval(...):
        tmp = a * 2.0 + 1.0
    with computation(PARALLEL), interval(1, -1):
        out = tmp[0, 0, 1] - a + tmp[0, 0, -1]


case(
    "staged_parallel_k_temp",
    fields={"a": fs(7, 6, 8), "out": fs(7, 6, 8, init="zeros")},
)(staged_parallel_k_temp)


def staged_wide_halo(a: F64, out: F64):
    with computation(PARALLEL), interval(...):
        d = a[70, 0, 0] - a[-70, 0, 0]
        out = d[0, 1, 0] + d[0, -1, 0] * 0.25


case(
    "staged_wide_halo",
    fields={"a": fs(150, 7, 3), "out": fs(10, 5, 3, init="zeros")},
    origin={"a": (70, 1, 0), "out": (0, 0, 0)},
    domain=(10, 5, 3),
)(staged_wide_halo)


# --------------------------------------------------------------------------------------
# Iterator access and 2-D temporaries (test_code_generation.py:1350-1383, 1536-1590):
# reference numpy-backend features; gt:mi355x supports iterator access, and raises for 2-D
# temporaries exactly like the reference's gt:* backends
# --------------------------------------------------------------------------------------


def iterator_access(field_A: F64, field_B: F64, offsets: Field[gtscript.K, np.int32]):
    with computation(PARALLEL), interval(...):
        if K == 2:  # noqa: F821
            field_A = 20.20
        field_B = float(K + offsets)  # noqa: F821


case(
    "iterator_access",
    fields={"field_A": fs(3, 4, 5, init="zeros"), "field_B": fs(3, 4, 5, init="zeros"),
            "offsets": fs(5, dtype="i4", init=("int", -3, 3))},
)(iterator_access)


def temporaries_2d(in_field: F64, out_field: F64):
    with computation(FORWARD), interval(0, 1):
        tmp_2D: Field[IJ, np.float64] = 0
    with computation(FORWARD), interval(...):
        tmp_2D = tmp_2D + in_field
    with computation(FORWARD), interval(...):
        out_field = tmp_2D


case(
    "temporaries_2d",
    fields={"in_field": fs(5, 5, 3), "out_field": fs(5, 5, 3, init="zeros")},
    features=("numpy_only",),
)(temporaries_2d)


# --------------------------------------------------------------------------------------
# Absolute K indexing `field.at(K=...)` (test_code_generation.py:1240-1347); fixtures from the
# reference debug backend (its numpy backend raises NotImplementedError for this feature)
# --------------------------------------------------------------------------------------


def abs_k_literal(in_field: F64, out_field: F64):
    with computation(PARALLEL), interval(...):
        out_field = in_field.at(K=2)


case("abs_k_literal", fields={"in_field": fs(5, 4, 6), "out_field": fs(5, 4, 6, init="zeros")},
     features=("golden_debug",))(abs_k_literal)


def abs_k_param(in_field: F64, out_field: F64, idx: int):
    with computation(PARALLEL), interval(...):
        out_field = in_field.at(K=idx) + in_field.at(K=idx - 1)


case("abs_k_param", fields={"in_field": fs(5, 4, 6), "out_field": fs(5, 4, 6, init="zeros")},
     params={"idx": 3}, features=("golden_debug",))(abs_k_param)


def abs_k_field(in_field: F64, index_field: Field[IJ, np.int64], out_field: F64):
    with computation(PARALLEL), interval(...):
        out_field = in_field.at(K=index_field)


case("abs_k_field", fields={"in_field": fs(5, 4, 6), "index_field": fs(5, 4, dtype="i8", init=("int", 0, 6)),
                            "out_field": fs(5, 4, 6, init="zeros")}, features=("golden_debug",))(abs_k_field)


def abs_k_field_computation(in_field: F64, index_field: Field[IJ, np.int32], out_field: F64):
    with computation(FORWARD), interval(...):
        out_field = in_field.at(K=index_field - 1) * 2.0


case("abs_k_field_computation",
     fields={"in_field": fs(5, 4, 6), "index_field": fs(5, 4, dtype="i4", init=("int", 1, 7)),
             "out_field": fs(5, 4, 6, init="zeros")}, features=("golden_debug",))(abs_k_field_computation)


def abs_k_lowdim(k_field: F1DK, out_field: F64):
    with computation(PARALLEL), interval(...):
        out_field = k_field.at(K=2)


case("abs_k_lowdim", fields={"k_field": fs(6), "out_field": fs(5, 4, 6, init="zeros")},
     features=("golden_debug",))(abs_k_lowdim)


def abs_k_conditional(in_field: F64, out_field: F64):
    with computation(PARALLEL), interval(...):
        k_level = 0
        while in_field.at(K=k_level) < 2:
            k_level += 1
        out_field[0, 0, 0] = k_level


case("abs_k_conditional", fields={"in_field": fs(5, 4, 6, init=("ramp", -5.0, 5.0)), "out_field": fs(5, 4, 6, init="zeros")},
     features=("golden_debug",))(abs_k_conditional)


def while_value_condition(a: F64, b: F64, out: F64):
    # a while loop whose condition reads a value its body changes before the counter: per point
    # the counter is incremented with the OLD condition (debug and GridTools backends); the
    # reference numpy backend re-evaluates the condition as the mask of `n = n + 1`
    # (oir_to_npir.py:176-185) and skips the increment once acc has left the range
    with computation(PARALLEL), interval(...):
        n = 0
        acc = a[0, 0, 0]
        while n < 3 and acc < 1.0:
            acc = acc * 0.5 + b[1, 0, 0]
            n = n + 1
        out = acc + n * 10.0


case("while_value_condition", fields={"a": fs(9, 5, 4), "b": fs(9, 5, 4, init=("u", -1.0, 2.0)),
                                      "out": fs(8, 5, 4, init="zeros")},
     origin={"a": (0, 0, 0), "b": (0, 0, 0), "out": (0, 0, 0)}, domain=(8, 5, 4),
     features=("golden_debug",))(while_value_condition)


# --------------------------------------------------------------------------------------
# Remaining stencil_definitions.py programs: every data type, a region with a conditional
# --------------------------------------------------------------------------------------


def data_types(
    bool_field: Field[bool],
    npbool_field: Field[np.bool_],
    int_field: Field[int],
    int8_field: Field[np.int8],
    int16_field: Field[np.int16],
    int32_field: Field[np.int32],
    int64_field: Field[np.int64],
    float_field: Field[float],
    float32_field: Field[np.float32],
    float64_field: Field[np.float64],
):
    with computation(PARALLEL), interval(...):
        bool_field = True
        npbool_field = False
        int_field = 2147483647
        int8_field = 127
        int16_field = 32767
        int32_field = 2147483647
        int64_field = 9223372036854775807
        float_field = 37.5
        float32_field = 37.5
        float64_field = 37.5


case(
    "data_types",
    fields={
        "bool_field": fs(4, 3, 2, dtype="?", init="bool"),
        "npbool_field": fs(4, 3, 2, dtype="?", init="bool"),
        "int_field": fs(4, 3, 2, dtype="i8", init=("int", -9, 9)),
        "int8_field": fs(4, 3, 2, dtype="i1", init=("int", -9, 9)),
        "int16_field": fs(4, 3, 2, dtype="i2", init=("int", -9, 9)),
        "int32_field": fs(4, 3, 2, dtype="i4", init=("int", -9, 9)),
        "int64_field": fs(4, 3, 2, dtype="i8", init=("int", -9, 9)),
        "float_field": fs(4, 3, 2),
        "float32_field": fs(4, 3, 2, dtype="f4"),
        "float64_field": fs(4, 3, 2),
    },
)(data_types)


def horizontal_region_with_conditional(field_in: F64, field_out: F64):
    with computation(PARALLEL), interval(...):
        with horizontal(region[I[0] : I[0] + 2, J[0] : J[0] + 2], region[I[-1] - 2 : I[-1], J[-1] - 2 : J[-1]]):
            if field_in > 0:
                field_out = field_in + 1.0
            else:
                field_out = 0


case(
    "horizontal_region_with_conditional",
    fields={"field_in": fs(7, 6, 3), "field_out": fs(7, 6, 3, init=("const", 42.0))},
)(horizontal_region_with_conditional)


def region_offset_reads(a: F64, b: F64, out: F64):
    """Offset reads inside horizontal regions near the domain edges: the reference clips each
    read's extent by its region's mask (oir_optimizations/utils.py:50-75), so ``b`` needs no
    west halo although it is read at ``[-1, 0, 0]``; overlapping masks of one ``with`` run the
    body once per mask (gtscript_frontend.py:1957-1962): the corner (0, 0) gets +2."""
    with computation(PARALLEL), interval(...):
        out = a
        with horizontal(region[I[-1] - 2 : I[-1], :]):
            out = b[-1, 0, 0] + a[0, 1, 0]
        with horizontal(region[I[0] + 1 : I[0] + 3, J[-1] - 1 : J[-1]]):
            out = out - b[1, 0, 0] * a[-1, 0, 0]
        with horizontal(region[I[0], :], region[:, J[0]]):
            out = out + 1.0


case(
    "region_offset_reads",
    fields={"a": fs(13, 11, 4), "b": fs(13, 11, 4), "out": fs(9, 7, 4, init="zeros")},
    origin={"a": (2, 2, 0), "b": (2, 2, 0), "out": (0, 0, 0)},
    domain=(9, 7, 4),
    features=("regions",),
)(region_offset_reads)


# --------------------------------------------------------------------------------------
# Column-kernel schedule edge cases (gt:mi355x K2: load ring, LDS tail cache, section gaps)
# --------------------------------------------------------------------------------------

case("tridiag_k70", fields=_tridiag_fields(9, 5, 70), features=("hot",))(tridiagonal_solver)  # tail covers 40 of 70 levels
case("tridiag_k161", fields=_tridiag_fields(6, 3, 161), features=("hot",))(tridiagonal_solver)  # ring remainder, long column
case(
    "tridiag_subdomain_k70",
    fields=_tridiag_fields(9, 7, 75),
    origin=(1, 2, 3),
    domain=(7, 4, 70),
    features=("hot",),
)(tridiagonal_solver)

case(
    "vertical_advection_dycore_k80",
    fields={
        "utens_stage": fs(8, 5, 80),
        "u_stage": fs(8, 5, 80),
        "wcon": fs(9, 5, 81, init=("u", -1.0, 1.0)),
        "u_pos": fs(8, 5, 80),
        "utens": fs(8, 5, 80),
    },
    params={"dtr_stage": 3.0 / 20.0},
    externals={"BET_M": 0.5, "BET_P": 0.5},
    domain=(8, 5, 80),
)(vertical_advection_dycore)


case(
    "vertical_advection_dycore_k160",  # long enough for the register band of the column kernel (auto: 96 levels)
    fields={
        "utens_stage": fs(9, 6, 160),
        "u_stage": fs(9, 6, 160),
        "wcon": fs(10, 6, 161, init=("u", -1.0, 1.0)),
        "u_pos": fs(9, 6, 160),
        "utens": fs(9, 6, 160),
    },
    params={"dtr_stage": 3.0 / 20.0},
    externals={"BET_M": 0.5, "BET_P": 0.5},
    domain=(9, 6, 160),
)(vertical_advection_dycore)


def section_gap_register_temp(a: F64, out: F64):
    """A register-only temporary read two levels down across a gap between sections (the gap
    level never runs; the value must survive it)."""
    with computation(FORWARD):
        with interval(0, 1):
            t = a * 2.0
            out = t
        with interval(2, 3):
            out = t[0, 0, -2]


case("section_gap_register_temp", fields={"a": fs(5, 4, 4), "out": fs(5, 4, 4, init="zeros")})(section_gap_register_temp)


def tail_fwd_bwd_offsets(a: F64, b: F64, out: F64):
    """FORWARD writes an API field and a temporary; BACKWARD reads them at two K offsets (fronts
    at different offsets: a band of levels where only some fronts are tail-cached)."""
    with computation(FORWARD):
        with interval(0, 1):
            t = a * 0.5
            b = a + 1.0
        with interval(1, None):
            t = a + t[0, 0, -1] * 0.5
            b = b * 0.75 + b[0, 0, -1] * 0.25
    with computation(BACKWARD):
        with interval(-1, None):
            out = b + t
        with interval(1, -1):
            out = t[0, 0, -1] + b + out[0, 0, 1] * 0.25
        with interval(0, 1):
            out = b + out[0, 0, 1] * 0.25


case(
    "tail_fwd_bwd_offsets",
    fields={"a": fs(7, 5, 75), "b": fs(7, 5, 75), "out": fs(7, 5, 75, init="zeros")},
)(tail_fwd_bwd_offsets)


def tail_bwd_fwd(a: F64, c: F64, out: F64):
    """BACKWARD sweep first, then FORWARD: the tail cache holds the lowest levels."""
    with computation(BACKWARD):
        with interval(-1, None):
            c = a
        with interval(0, -1):
            c = a - 0.5 * c[0, 0, 1]
    with computation(FORWARD):
        with interval(0, 1):
            out = c
        with interval(1, None):
            out = c + 0.25 * out[0, 0, -1] + 0.125 * c[0, 0, -1]


case("tail_bwd_fwd", fields={"a": fs(6, 5, 130), "c": fs(6, 5, 130), "out": fs(6, 5, 130, init="zeros")})(tail_bwd_fwd)
case("tail_bwd_fwd_short", fields={"a": fs(6, 5, 9), "c": fs(6, 5, 9), "out": fs(6, 5, 9, init="zeros")})(tail_bwd_fwd)


def band_ij_accumulator(a: F64, b: F64, out: F64, s: F2D, lev: Field[IJ, np.int32]):
    """A FORWARD sweep producing a tail-cached temporary ``c`` next to an IJ counter ``lev``, then
    a BACKWARD sweep accumulating into the IJ field ``s`` at every level. With nk above the
    register band's minimum (96 levels) both IJ accumulators are read and written inside the band:
    a front of them loaded levels ahead would miss the writes in between."""
    with computation(FORWARD):
        with interval(0, 1):
            c = a
            lev = 0
        with interval(1, None):
            c = a + 0.5 * c[0, 0, -1]
            lev = lev + 1
    with computation(BACKWARD):
        with interval(-1, None):
            s = c * b
            out = s
        with interval(0, -1):
            s = s * 0.5 + c * b
            out = s + lev


def band_ij_accumulator_reader(a: F64, b: F64, out: F64, s: F2D):
    """As ``band_ij_accumulator`` with the IJ accumulator in the reader only, so the writer's last
    band levels prefetch the reader's first ones (the band's prefetch crosses the loop boundary)."""
    with computation(FORWARD):
        with interval(0, 1):
            c = a
        with interval(1, None):
            c = a + 0.5 * c[0, 0, -1]
    with computation(BACKWARD):
        with interval(-1, None):
            s = c * b
            out = s
        with interval(0, -1):
            s = s * 0.5 + c * b
            out = s - a


case("band_ij_accumulator", fields={"a": fs(9, 4, 120), "b": fs(9, 4, 120), "out": fs(9, 4, 120, init="zeros"),
                                    "s": fs(9, 4), "lev": fs(9, 4, dtype="i4", init=("int", 50, 60))})(
    band_ij_accumulator)
case("band_ij_accumulator_reader", fields={"a": fs(9, 4, 131), "b": fs(9, 4, 131),
                                           "out": fs(9, 4, 131, init="zeros"), "s": fs(9, 4)})(
    band_ij_accumulator_reader)


# --------------------------------------------------------------------------------------
# Tile kernels (column kernels in tile mode, codegen/column.py): sequential sweeps that read
# their own products across columns -- the reference's IJ caches
# (gtc/passes/oir_optimizations/caches.py:44-90). Ragged domains leave partial tiles on both
# axes (the default f64 tile is 48 x 6 outputs, f32 112 x 6).
# --------------------------------------------------------------------------------------


def bwd_recurrence_ij_temp(a: F64, b: F64, out: F64):
    with computation(BACKWARD):
        with interval(-1, None):
            s = a
        with interval(0, -1):
            s = s[0, 0, 1] * 0.25 + a - b
    with computation(BACKWARD), interval(...):
        t = s * b
        out = t[0, -1, 0] + t[0, 1, 0] - 2.0 * t[-2, 0, 0] + t[2, 0, 0]


def two_phase_chain(a: F64, c: F64, out: F64):
    with computation(FORWARD), interval(...):
        t1 = a * c + 1.0
        t2 = t1[1, 0, 0] + t1[-1, 0, 0] - t1
        out = t2[0, 1, 0] - t2[0, -1, 0] + c


def tile_with_k_window(a: F64, w: F64, out: F64):
    with computation(FORWARD):
        with interval(0, 1):
            acc = a
        with interval(1, None):
            acc = acc[0, 0, -1] + a * w
    with computation(FORWARD):
        with interval(0, 1):
            t0 = acc * w
            out = t0[1, 0, 0] - t0[0, -1, 0]
        with interval(1, None):
            t1 = acc + w * acc[0, 0, -1]
            out = t1[1, 0, 0] - t1[0, -1, 0] + out[0, 0, -1] * 0.5


def tile_conditional(a: F64, out: F64):
    with computation(FORWARD):
        with interval(0, 1):
            m = a
        with interval(1, None):
            m = m[0, 0, -1] if m[0, 0, -1] > a else a
    with computation(FORWARD), interval(...):
        d = m - a
        if d[1, 0, 0] > d[-1, 0, 0]:
            out = d[1, 0, 0] + d[0, 1, 0]
        else:
            out = d[-1, 0, 0] - d[0, -1, 0]


def tile_f32(a: F32, out: F32):
    with computation(FORWARD):
        with interval(0, 1):
            s = a
        with interval(1, None):
            s = s[0, 0, -1] * 0.5 + a
    with computation(FORWARD), interval(...):
        t = s * 3.0
        out = t[1, 1, 0] - t[-1, -1, 0]



def tile_scratch_product(a: F64, out: F64):
    """A tile-kernel temporary (t2, read across columns through u's LDS plane) that a later
    PARALLEL kernel reads at IJ offsets, so it is stored to a scratch field from the tile kernel:
    only lanes on which t2 is valid may store it (codegen/column.py _tile_local)."""
    with computation(FORWARD):
        with interval(0, 1):
            t1 = a * 0.5
        with interval(1, None):
            t1 = t1[0, 0, -1] * 0.5 + a
    with computation(FORWARD), interval(...):
        u = t1 * 2.0 + a
        t2 = u[1, 0, 0] - u[-1, 0, 0] + u[0, 1, 0]
    with computation(PARALLEL), interval(...):
        out = t2[1, 0, 0] + t2[-1, 0, 0] - t2[0, -1, 0]


# name: (definition, {field: (halo_i_lo, halo_i_hi, halo_j_lo, halo_j_hi)}, dtype)
TILE_PROGRAMS = {
    "fwd_recurrence_ij_temp": (staged_forward_ij_temp, {"a": (1, 1, 0, 1)}, "f8"),
    "bwd_recurrence_ij_temp": (bwd_recurrence_ij_temp, {"a": (2, 2, 1, 1), "b": (2, 2, 1, 1)}, "f8"),
    "two_phase_chain": (two_phase_chain, {"a": (1, 1, 1, 1), "c": (1, 1, 1, 1)}, "f8"),
    "tile_with_k_window": (tile_with_k_window, {"a": (0, 1, 1, 0), "w": (0, 1, 1, 0)}, "f8"),
    "tile_conditional": (tile_conditional, {"a": (1, 1, 1, 1)}, "f8"),
    "tile_f32": (tile_f32, {"a": (1, 1, 1, 1)}, "f4"),
    "tile_scratch_product": (tile_scratch_product, {"a": (2, 2, 1, 1)}, "f8"),
}
TILE_DOMAINS = {"d70": (70, 9, 6), "d131": (131, 23, 13)}
TILE_GOLDEN = []  # golden case names, one per (program, domain)


def _tile_cases():
    for prog, (defn, halos, dt) in TILE_PROGRAMS.items():
        for tag, (ni, nj, nk) in TILE_DOMAINS.items():
            fields, origin = {}, {}
            for f, (ilo, ihi, jlo, jhi) in halos.items():
                fields[f] = fs(ni + ilo + ihi, nj + jlo + jhi, nk, dtype=dt, init=("u", 0.5, 2.0))
                origin[f] = (ilo, jlo, 0)
            fields["out"] = fs(ni, nj, nk, dtype=dt, init="zeros")
            origin["out"] = (0, 0, 0)
            name = f"tile_{prog}_{tag}"
            case(name, fields=fields, origin=origin, domain=(ni, nj, nk), features=("tile",))(defn)
            TILE_GOLDEN.append(name)


_tile_cases()


def tile_kwrite_raw(a: F64, out: F64):
    """A tile sweep whose API output, stored after the LDS barrier one level ahead
    (``out[0, 0, 1]``, a K-offset write: the field bypasses the register window), is read back at
    the next level by the statements before the barrier (``c``). Levels blocked two or four to a
    barrier would run that read before the store and see stale memory, so such a loop keeps one
    level per barrier (codegen/column.py ``_blockable``). The reference numpy backend
    runs the K loop outside the horizontal blocks, as the compiled backends do (its debug backend
    runs each horizontal block over all levels first, so the two disagree on such a program; the
    fixture comes from the numpy backend)."""
    with computation(FORWARD):
        with interval(0, -1):
            c = out
            t1 = a * 0.5 + 1.0
            out[0, 0, 1] = 0.25 * c + t1[1, 0, 0] + t1[0, 1, 0] - t1[0, -1, 0]


def _tile_raw_cases():
    for tag, (ni, nj, nk) in TILE_DOMAINS.items():
        name = f"tile_kwrite_raw_{tag}"
        case(name, fields={"a": fs(ni + 1, nj + 2, nk, init=("u", 0.5, 2.0)), "out": fs(ni, nj, nk, init=("u", -1.0, 1.0))},
             origin={"a": (0, 1, 0), "out": (0, 0, 0)}, domain=(ni, nj, nk), features=("tile",))(tile_kwrite_raw)
        TILE_GOLDEN.append(name)


_tile_raw_cases()


# --------------------------------------------------------------------------------------
# Differential-fuzz programs that take the tile path (tests/fuzz_stencils.py seeds; their
# sources are committed in tests/fuzz_golden_programs.py so the reference frontend can read
# them), pinned to the reference numpy backend at ragged domains
# --------------------------------------------------------------------------------------

import fuzz_golden_programs as _fgp  # noqa: E402

FUZZ_GOLDEN = []


def _fuzz_cases():
    for n, seed in enumerate(_fgp.SEEDS):
        ni, nj, nk = TILE_DOMAINS["d70"]  # 2 x 2 tiles with partial ones (kept small: five random fields)
        fields = {f: fs(ni + 4, nj + 4, nk, init=("u", -4.0, 4.0)) for f in ("a", "b", "c")}
        fields.update({f: fs(ni, nj, nk, init=("u", -1.0, 1.0)) for f in ("out1", "out2")})
        origin = {"a": (2, 2, 0), "b": (2, 2, 0), "c": (2, 2, 0), "out1": (0, 0, 0), "out2": (0, 0, 0)}
        name = f"fuzz_tile_{seed}"
        case(name, fields=fields, params={"s": 0.75}, origin=origin, domain=(ni, nj, nk),
             features=("tile", "fuzz"))(getattr(_fgp, f"fuzz_{seed}"))
        FUZZ_GOLDEN.append(name)


_fuzz_cases()
