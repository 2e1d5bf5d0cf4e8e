"""CPU oracle (TEST INFRASTRUCTURE ONLY) for the hot-path stencils of SURVEY.md §8(a).

This module restates, in plain numpy, what the reference's ``numpy`` backend computes for
the four hot-path stencils. It is the checker for parity tests, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg -- it is never imported by the ``gt4py_amd`` product
path.

Pinning: every function here is checked bit-for-bit against the golden vectors in
``tests/golden/*.npz`` (``tests/test_oracle.py``), which were produced by running the
reference numpy backend itself (``tests/golden/make_golden.py``).

Semantics followed (reference file:line):
- numpy executor: one vectorised expression per statement over ``[i:I, j:J, k:K]``,
  ``src/gt4py/cartesian/gtc/numpy/npir_codegen.py:320-368``; index (i,j,k) maps to
  ``array[origin + (i,j,k) + offset]`` (``src/gt4py/cartesian/utils/field.py:15-74``).
- sequential loops: a Python ``for k_`` loop per interval section,
  ``npir_codegen.py:243-248``.
- casts: ``src/gt4py/cartesian/gtc/passes/gtir_upcaster.py:80-143`` -- 64-bit float
  literals promote f32 operands to f64; the assignment casts to the LHS dtype.
- all arithmetic under ``np.errstate(ignore)`` (``npir_codegen.py:355``).
"""

from __future__ import annotations

import numpy as np

_ERR = dict(divide="ignore", over="ignore", under="ignore", invalid="ignore")


def _view(arr, origin, domain, di=0, dj=0, dk=0, halo=(0, 0)):
    """Slice ``arr`` at logical offset (di,dj,dk), extended by ``halo`` in I/J."""
    oi, oj, ok = origin
    ni, nj, nk = domain
    hi, hj = halo
    return arr[
        oi + di - hi : oi + di + ni + hi,
        oj + dj - hj : oj + dj + nj + hj,
        ok + dk : ok + dk + nk,
    ]


def copy_stencil(field_a, field_b, origin, domain):
    """``out = in[0,0,0]``; ``stencil_definitions.py:73-76``."""
    field_b_v = _view(field_b, origin["field_b"], domain)
    field_b_v[...] = _view(field_a, origin["field_a"], domain)


def lap5(in_field, out_field, origin, domain):
    """``4.0*u - (((u[i+1]+u[i-1])+u[j+1])+u[j-1])``; ``test_suites.py:233-236`` op order."""
    o = origin["in_field"]
    u = lambda di, dj: _view(in_field, o, domain, di, dj)  # noqa: E731
    with np.errstate(**_ERR):
        res = np.float64(4.0) * u(0, 0) - (((u(1, 0) + u(-1, 0)) + u(0, 1)) + u(0, -1))
    _view(out_field, origin["out_field"], domain)[...] = res


def horizontal_diffusion(in_field, out_field, coeff, origin, domain):
    """Limiter horizontal diffusion, ``stencil_definitions.py:316-328``.

    For f32 fields the reference upcasts (gtir_upcaster): ``lap = f64(4.0)*f64(u) -
    f64(f32 neighbour sum)``; ``res``/``flx``/``fly`` are f64; the limiter product casts the
    f32 difference to f64; ``out = f32(f64(u) - f64(coeff)*(...))``.
    """
    dt = in_field.dtype
    o_in = origin["in_field"]
    with np.errstate(**_ERR):

        def u(di, dj, halo=(0, 0)):
            return _view(in_field, o_in, domain, di, dj, halo=halo)

        # lap over domain extended by 1 in I and J
        h = (1, 1)
        lap = np.float64(4.0) * u(0, 0, h).astype(np.float64) - (
            ((u(1, 0, h) + u(-1, 0, h)) + u(0, 1, h)) + u(0, -1, h)
        ).astype(np.float64)
        ni, nj = domain[0], domain[1]
        lap_c = lap[1 : ni + 1, 1 : nj + 1]
        lap_ip = lap[2 : ni + 2, 1 : nj + 1]
        lap_im = lap[0:ni, 1 : nj + 1]
        lap_jp = lap[1 : ni + 1, 2 : nj + 2]
        lap_jm = lap[1 : ni + 1, 0:nj]
        zero = np.float64(np.int64(0))

        def limit(res, du):
            return np.where((res * du.astype(np.float64)) > zero, zero, res)

        flx = limit(lap_ip - lap_c, u(1, 0) - u(0, 0))
        flx_m = limit(lap_c - lap_im, u(0, 0) - u(-1, 0))
        fly = limit(lap_jp - lap_c, u(0, 1) - u(0, 0))
        fly_m = limit(lap_c - lap_jm, u(0, 0) - u(0, -1))
        c = _view(coeff, origin["coeff"], domain).astype(np.float64)
        res = u(0, 0).astype(np.float64) - c * (((flx - flx_m) + fly) - fly_m)
    _view(out_field, origin["out_field"], domain)[...] = res.astype(dt)


def tridiagonal_solver(inf, diag, sup, rhs, out, origin, domain):
    """Thomas algorithm, ``stencil_definitions.py:219-232``; per-level numpy loop."""
    ni, nj, nk = domain
    v = {}
    for name, arr in (("inf", inf), ("diag", diag), ("sup", sup), ("rhs", rhs), ("out", out)):
        oi, oj, ok = origin[name]
        v[name] = arr[oi : oi + ni, oj : oj + nj, ok : ok + nk]
    a, b, c, d, x = v["inf"], v["diag"], v["sup"], v["rhs"], v["out"]
    with np.errstate(**_ERR):
        c[:, :, 0] = c[:, :, 0] / b[:, :, 0]
        d[:, :, 0] = d[:, :, 0] / b[:, :, 0]
        for k in range(1, nk):
            c[:, :, k] = c[:, :, k] / (b[:, :, k] - c[:, :, k - 1] * a[:, :, k])
            d[:, :, k] = (d[:, :, k] - a[:, :, k] * d[:, :, k - 1]) / (b[:, :, k] - c[:, :, k - 1] * a[:, :, k])
        x[:, :, nk - 1] = d[:, :, nk - 1]
        for k in range(nk - 2, -1, -1):
            x[:, :, k] = d[:, :, k] - c[:, :, k] * x[:, :, k + 1]


STENCILS = {
    "copy_stencil": (copy_stencil, ("field_a", "field_b")),
    "lap5": (lap5, ("in_field", "out_field")),
    "horizontal_diffusion": (horizontal_diffusion, ("in_field", "out_field", "coeff")),
    "tridiagonal_solver": (tridiagonal_solver, ("inf", "diag", "sup", "rhs", "out")),
}


def normalize_origin(origin, names):
    if origin is None:
        return {n: (0, 0, 0) for n in names}
    if isinstance(origin, dict):
        allo = origin.get("_all_", (0, 0, 0))
        return {n: tuple(origin.get(n, allo)) for n in names}
    return {n: tuple(origin) for n in names}
