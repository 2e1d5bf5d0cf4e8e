"""The reference's integration suites (``multi_feature_tests/test_suites.py``) run through
``gt4py_amd.testing.StencilTestSuite`` on the ``numpy`` and ``gt:mi355x`` backends.

Each suite restates one reference suite: the same stencil program, the same symbol ranges and
boundaries, and a numpy ``validation`` written here independently of both backends. Hypothesis
draws domain sizes and inputs (``GTMI_SUITE_EXAMPLES`` per test, default 25). Generation tests
(code generation + gfx950 compile for ``gt:mi355x``) run on the CPU; ``gt:mi355x``
implementation tests carry the ``gpu`` marker and compare device results after the call.
"""

import numpy as np

from gt4py_amd import gtscript, testing as gt_testing
from gt4py_amd.gtscript import PARALLEL, Field, I, J, computation, horizontal, interval, region

from stencil_cases import optional_field, two_optional_fields

BACKENDS = ["numpy", "gt:mi355x"]
fld = gt_testing.field
par = gt_testing.parameter
NO_HALO = [(0, 0), (0, 0), (0, 0)]


def _lap(u):
    """5-point Laplacian of the interior of ``u`` (one cell of halo in I and J)."""
    c = u[1:-1, 1:-1]
    return 4.0 * c - (u[2:, 1:-1] + u[:-2, 1:-1] + u[1:-1, 2:] + u[1:-1, :-2])


def _diffused(u, weight):
    """Horizontal diffusion without limiter; ``u`` carries a halo of 2 in I and J."""
    lap = _lap(u)
    fi = lap[1:, 1:-1] - lap[:-1, 1:-1]
    fj = lap[1:-1, 1:] - lap[1:-1, :-1]
    return u[2:-2, 2:-2] - weight * ((fi[1:] - fi[:-1]) + (fj[:, 1:] - fj[:, :-1]))


# ------------------------------------------------------------------------------ basic
class TestIdentity(gt_testing.StencilTestSuite):
    dtypes = {("field_a",): (np.float64, np.float32)}
    domain_range = [(1, 25), (1, 25), (1, 25)]
    backends = BACKENDS
    symbols = dict(field_a=fld(in_range=(-10, 10), boundary=NO_HALO))

    def definition(field_a):
        with computation(PARALLEL), interval(...):
            tmp = field_a
            field_a = tmp

    def validation(field_a, domain=None, origin=None):
        return None


class TestCopy(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 25), (1, 25), (1, 25)]
    backends = BACKENDS
    symbols = dict(src=fld(in_range=(-10, 10), boundary=NO_HALO), dst=fld(in_range=(-10, 10), boundary=NO_HALO))

    def definition(src, dst):
        with computation(PARALLEL), interval(...):
            dst = src

    def validation(src, dst, domain=None, origin=None):
        np.copyto(dst, src)


class TestAugAssign(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 25), (1, 25), (1, 25)]
    backends = BACKENDS
    symbols = dict(a=fld(in_range=(-10, 10), boundary=NO_HALO), b=fld(in_range=(-10, 10), boundary=NO_HALO))

    def definition(a, b):
        with computation(PARALLEL), interval(...):
            a += 1.0
            a *= 2.0
            b -= 1.0
            b /= 2.0

    def validation(a, b, domain=None, origin=None):
        a[...] = 2.0 * (a + 1.0)
        b[...] = (b - 1.0) / 2.0


class TestGlobalScale(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (1, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(
        SCALE_FACTOR=gt_testing.global_name(one_of=(1.0, 1e3, 1e6)),
        a=fld(in_range=(-1, 1), boundary=NO_HALO),
    )

    def definition(a):
        from __externals__ import SCALE_FACTOR

        with computation(PARALLEL), interval(...):
            a = SCALE_FACTOR * a[0, 0, 0]

    def validation(a, domain, origin, **kwargs):
        a *= SCALE_FACTOR  # noqa: F821 (external injected by the suite)


class TestParametricScale(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (1, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(a=fld(in_range=(-10, 10), boundary=NO_HALO), scale=par(in_range=(-100, 100)))

    def definition(a, *, scale):
        with computation(PARALLEL), interval(...):
            a = scale * a

    def validation(a, *, scale, domain, origin, **kwargs):
        a[...] = scale * a


class TestParametricMix(gt_testing.StencilTestSuite):
    dtypes = {
        ("USE_ALPHA",): np.int_,
        ("fa", "fb", "fc"): np.float64,
        ("fout",): np.float32,
        ("weight", "alpha_factor"): np.float64,
    }
    domain_range = [(1, 15), (1, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(
        USE_ALPHA=gt_testing.global_name(one_of=(True, False)),
        fa=fld(in_range=(-10, 10), boundary=NO_HALO),
        fb=fld(in_range=(-10, 10), boundary=NO_HALO),
        fc=fld(in_range=(-10, 10), boundary=NO_HALO),
        fout=fld(in_range=(-10, 10), boundary=NO_HALO),
        weight=par(in_range=(-10, 10)),
        alpha_factor=par(in_range=(-1, 1)),
    )

    def definition(fa, fb, fc, fout, *, weight, alpha_factor):
        from __externals__ import USE_ALPHA
        from __gtscript__ import __INLINED

        with computation(PARALLEL), interval(...):
            if __INLINED(USE_ALPHA):
                factor = alpha_factor
            else:
                factor = 1.0
            fout = factor * fa[0, 0, 0] - (1 - factor) * (fb[0, 0, 0] - weight * fc[0, 0, 0])

    def validation(fa, fb, fc, fout, *, weight, alpha_factor, domain, origin, **kwargs):
        f = alpha_factor if USE_ALPHA else 1.0  # noqa: F821
        fout[...] = f * fa - (1 - f) * (fb - weight * fc)


class TestHeatEquation_FTCS_3D(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (1, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(
        u=fld(in_range=(-10, 10), extent=[(-1, 1), (0, 0), (0, 0)]),
        v=fld(in_range=(-10, 10), extent=[(0, 0), (-1, 1), (0, 0)]),
        u_new=fld(in_range=(-10, 10), extent=[(0, 0), (0, 0), (0, 0)]),
        v_new=fld(in_range=(-10, 10), extent=[(0, 0), (0, 0), (0, 0)]),
        ru=par(in_range=(0, 0.5)),
        rv=par(in_range=(0, 0.5)),
    )

    def definition(u, v, u_new, v_new, *, ru, rv):
        with computation(PARALLEL), interval(...):
            u_new = u[0, 0, 0] + ru * (u[1, 0, 0] - 2 * u[0, 0, 0] + u[-1, 0, 0])
            v_new = v[0, 0, 0] + rv * (v[0, 1, 0] - 2 * v[0, 0, 0] + v[0, -1, 0])

    def validation(u, v, u_new, v_new, *, ru, rv, domain, origin, **kwargs):
        uc, vc = u[1:-1], v[:, 1:-1]
        u_new[...] = uc + ru * (u[2:] - 2 * uc + u[:-2])
        v_new[...] = vc + rv * (v[:, 2:] - 2 * vc + v[:, :-2])


# ------------------------------------------------------------------------------ diffusion
class TestHorizontalDiffusion(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (1, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(
        u=fld(in_range=(-10, 10), boundary=[(2, 2), (2, 2), (0, 0)]),
        diffusion=fld(in_range=(-10, 10), boundary=NO_HALO),
        weight=par(in_range=(0, 0.5)),
    )

    def definition(u, diffusion, *, weight):
        with computation(PARALLEL), interval(...):
            laplacian = 4.0 * u[0, 0, 0] - (u[1, 0, 0] + u[-1, 0, 0] + u[0, 1, 0] + u[0, -1, 0])
            flux_i = laplacian[1, 0, 0] - laplacian[0, 0, 0]
            flux_j = laplacian[0, 1, 0] - laplacian[0, 0, 0]
            diffusion = u[0, 0, 0] - weight * (flux_i[0, 0, 0] - flux_i[-1, 0, 0] + flux_j[0, 0, 0] - flux_j[0, -1, 0])

    def validation(u, diffusion, *, weight, domain, origin, **kwargs):
        diffusion[...] = _diffused(u, weight)


@gtscript.function
def lap_op(u):
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
    return field[1, 0, 0] - field[0, 0, 0]


@gtscript.function
def fwd_diff_op_y(field):
    return field[0, 1, 0] - field[0, 0, 0]


class TestHorizontalDiffusionSubroutines(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (1, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(
        fwd_diff=gt_testing.global_name(singleton=wrap1arg2return),
        u=fld(in_range=(-10, 10), boundary=[(2, 2), (2, 2), (0, 0)]),
        diffusion=fld(in_range=(-10, 10), boundary=NO_HALO),
        weight=par(in_range=(0, 0.5)),
    )

    def definition(u, diffusion, *, weight):
        from __externals__ import fwd_diff

        with computation(PARALLEL), interval(...):
            laplacian = lap_op(u=u)
            flux_i, flux_j = fwd_diff(field=laplacian)
            diffusion = u[0, 0, 0] - weight * (flux_i[0, 0, 0] - flux_i[-1, 0, 0] + flux_j[0, 0, 0] - flux_j[0, -1, 0])

    def validation(u, diffusion, *, weight, domain, origin, **kwargs):
        diffusion[...] = _diffused(u, weight)


class TestHorizontalDiffusionSubroutines2(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (1, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(
        fwd_diff=gt_testing.global_name(singleton=fwd_diff_op_xy),
        BRANCH=gt_testing.global_name(one_of=(True, False)),
        u=fld(in_range=(-10, 10), boundary=[(2, 2), (2, 2), (0, 0)]),
        diffusion=fld(in_range=(-10, 10), boundary=NO_HALO),
        weight=par(in_range=(0, 0.5)),
    )

    def definition(u, diffusion, *, weight):
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

    def validation(u, diffusion, *, weight, domain, origin, **kwargs):
        diffusion[...] = _diffused(u, weight)


# ------------------------------------------------------------------------------ control flow
class TestRuntimeIfFlat(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (1, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(outfield=fld(in_range=(-10, 10), boundary=NO_HALO))

    def definition(outfield):
        with computation(PARALLEL), interval(...):
            if True:
                outfield = 1
            else:
                outfield = 2

    def validation(outfield, *, domain, origin, **kwargs):
        outfield.fill(1)


class TestRuntimeIfNested(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (1, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(outfield=fld(in_range=(-10, 10), boundary=NO_HALO))

    def definition(outfield):
        with computation(PARALLEL), interval(...):
            if (outfield > 0 and outfield > 0) or (not outfield > 0 and not outfield > 0):
                if False:
                    outfield = 1
                else:
                    outfield = 2
            else:
                outfield = 3

    def validation(outfield, *, domain, origin, **kwargs):
        outfield.fill(2)


@gtscript.function
def add_one(field_in):
    return field_in + 1


class Test3FoldNestedIf(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(3, 3), (3, 3), (3, 3)]
    backends = BACKENDS
    symbols = dict(a=fld(in_range=(-1, 1), boundary=NO_HALO))

    def definition(a):
        with computation(PARALLEL), interval(...):
            if a >= 0.0:
                a = 0.0
                if a > 1:
                    a = 1
                    if a > 2:
                        a = 2

    def validation(a, domain, origin):
        # a >= 0 becomes 0; the nested branches can then never fire
        a[a >= 0.0] = 0.0


class TestRuntimeIfNestedDataDependent(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(3, 3), (3, 3), (3, 3)]
    backends = BACKENDS
    symbols = dict(
        factor=par(in_range=(-100, 100)),
        a=fld(in_range=(-1, 1), boundary=NO_HALO),
        b=fld(in_range=(-1, 1), boundary=NO_HALO),
        c=fld(in_range=(-1, 1), boundary=NO_HALO),
    )

    def definition(a, b, c, *, factor):
        with computation(PARALLEL), interval(...):
            if factor > 0:
                if a < 0:
                    b = -a
                else:
                    b = a
            else:
                if a < 0:
                    c = -a
                else:
                    c = a
            a = add_one(a)

    def validation(a, b, c, *, factor, domain, origin, **kwargs):
        (b if factor > 0 else c)[...] = np.abs(a)
        a += 1


class TestRuntimeIfNestedWhile(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (1, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(
        infield=fld(in_range=(-1, 1), boundary=NO_HALO), outfield=fld(in_range=(-10, 10), boundary=NO_HALO)
    )

    def definition(infield, outfield):
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

    def validation(infield, outfield, *, domain, origin, **kwargs):
        outfield.fill(2)  # infield < 1 everywhere


class TestTernaryOp(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (2, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(
        infield=fld(in_range=(-10, 10), boundary=[(0, 0), (0, 1), (0, 0)]),
        outfield=fld(in_range=(-10, 10), boundary=NO_HALO),
    )

    def definition(infield, outfield):
        with computation(PARALLEL), interval(...):
            outfield = infield if infield > 0.0 else -infield[0, 1, 0]

    def validation(infield, outfield, *, domain, origin, **kwargs):
        here, north = infield[:, :-1], infield[:, 1:]
        outfield[...] = np.where(here > 0.0, here, -north)


class TestThreeWayAnd(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (2, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(
        outfield=fld(in_range=(-10, 10), boundary=NO_HALO),
        a=par(in_range=(-100, 100)), b=par(in_range=(-100, 100)), c=par(in_range=(-100, 100)),
    )

    def definition(outfield, *, a, b, c):
        with computation(PARALLEL), interval(...):
            if a > 0 and b > 0 and c > 0:
                outfield = 1
            else:
                outfield = 0

    def validation(outfield, *, a, b, c, domain, origin, **kwargs):
        outfield.fill(float(min(a, b, c) > 0))


class TestThreeWayOr(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 15), (2, 15), (1, 15)]
    backends = BACKENDS
    symbols = dict(
        outfield=fld(in_range=(-10, 10), boundary=NO_HALO),
        a=par(in_range=(-100, 100)), b=par(in_range=(-100, 100)), c=par(in_range=(-100, 100)),
    )

    def definition(outfield, *, a, b, c):
        with computation(PARALLEL), interval(...):
            if a > 0 or b > 0 or c > 0:
                outfield = 1
            else:
                outfield = 0

    def validation(outfield, *, a, b, c, domain, origin, **kwargs):
        outfield.fill(float(max(a, b, c) > 0))


# ------------------------------------------------------------------------------ optional fields
class TestOptionalField(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 32), (1, 32), (1, 32)]
    backends = BACKENDS
    symbols = dict(
        PHYS_TEND=gt_testing.global_name(one_of=(False, True)),
        in_field=fld(in_range=(-10, 10), boundary=NO_HALO),
        out_field=fld(in_range=(-10, 10), boundary=NO_HALO),
        dyn_tend=fld(in_range=(-10, 10), boundary=NO_HALO),
        phys_tend=fld(in_range=(-10, 10), boundary=NO_HALO),
        dt=par(in_range=(0, 100)),
    )
    definition = optional_field

    def validation(in_field, out_field, dyn_tend, phys_tend=None, *, dt, domain, origin, **kwargs):
        res = in_field + dt * dyn_tend
        if PHYS_TEND:  # noqa: F821
            res = res + dt * phys_tend
        out_field[...] = res


class TestNotSpecifiedOptionalField(TestOptionalField):
    backends = BACKENDS
    symbols = dict(TestOptionalField.symbols, PHYS_TEND=gt_testing.global_name(one_of=(False,)),
                   phys_tend=gt_testing.none())


class TestTwoOptionalFields(gt_testing.StencilTestSuite):
    dtypes = (np.float64,)
    domain_range = [(1, 32), (1, 32), (1, 32)]
    backends = BACKENDS
    symbols = dict(
        PHYS_TEND_A=gt_testing.global_name(one_of=(False, True)),
        PHYS_TEND_B=gt_testing.global_name(one_of=(False, True)),
        **{n: fld(in_range=(-10, 10), boundary=NO_HALO)
           for n in ("in_a", "in_b", "out_a", "out_b", "dyn_tend_a", "dyn_tend_b", "phys_tend_a", "phys_tend_b")},
        dt=par(in_range=(0, 100)),
    )
    definition = two_optional_fields

    def validation(in_a, in_b, out_a, out_b, dyn_tend_a, dyn_tend_b, phys_tend_a=None, phys_tend_b=None, *, dt,
                   domain, origin, **kwargs):
        for out, inp, dyn, phys, on in ((out_a, in_a, dyn_tend_a, phys_tend_a, PHYS_TEND_A),  # noqa: F821
                                        (out_b, in_b, dyn_tend_b, phys_tend_b, PHYS_TEND_B)):  # noqa: F821
            res = inp + dt * dyn
            if on:
                res = res + dt * phys
            out[...] = res


class TestNotSpecifiedTwoOptionalFields(TestTwoOptionalFields):
    backends = BACKENDS
    symbols = dict(TestTwoOptionalFields.symbols, PHYS_TEND_A=gt_testing.global_name(one_of=(False,)),
                   phys_tend_a=gt_testing.none())


# ------------------------------------------------------------------------------ non-3-D fields, data dims
class TestNon3DFields(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float64, "another_field": np.float64, "field_out": np.float64}
    domain_range = [(4, 10), (4, 10), (4, 10)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="K", boundary=NO_HALO),
        "another_field": fld(in_range=(-10, 10), axes="IJ", data_dims=(3, 2, 2), boundary=[(1, 1), (1, 1), (0, 0)]),
        "field_out": fld(in_range=(-10, 10), axes="IJK", data_dims=(3, 2), boundary=NO_HALO),
    }

    def definition(field_in, another_field, field_out):
        with computation(PARALLEL), interval(...):
            field_out[0, 0, 0][0, 0] = field_in[0] + another_field[-1, -1][0, 0, 0] + another_field[-1, -1][0, 0, 1]
            field_out[0, 0, 0][0, 1] = 2 * (
                another_field[-1, -1][1, 0, 0] + another_field[-1, -1][1, 0, 1]
                + another_field[-1, -1][1, 1, 0] + another_field[-1, -1][1, 1, 1]
            )
            field_out[0, 0, 0][1, 0] = field_in[0] + another_field[1, 1][0, 0, 0] + another_field[1, 1][0, 0, 1]
            field_out[0, 0, 0][1, 1] = 3 * (
                another_field[1, 1][1, 0, 0] + another_field[1, 1][1, 0, 1]
                + another_field[1, 1][1, 1, 0] + another_field[1, 1][1, 1, 1]
            )
            field_out[0, 0, 0][2, 0] = field_in[0] + another_field[0, 0][0, 0, 0] + another_field[-1, 1][0, 0, 1]
            field_out[0, 0, 0][2, 1] = 4 * (
                another_field[-1, 1][1, 0, 0] + another_field[-1, 1][1, 0, 1]
                + another_field[-1, 1][1, 1, 0] + another_field[-1, 1][1, 1, 1]
            )

    def validation(field_in, another_field, field_out, *, domain, origin):
        ni, nj = field_out.shape[:2]

        def at(di, dj):  # another_field shifted by (di, dj), broadcast over K
            return another_field[1 + di : 1 + di + ni, 1 + dj : 1 + dj + nj, None]

        def quad(a):  # sum of the four [1, x, y] components, left to right
            return ((a[..., 1, 0, 0] + a[..., 1, 0, 1]) + a[..., 1, 1, 0]) + a[..., 1, 1, 1]

        k = field_in[None, None, :]
        field_out[..., 0, 0] = (k + at(-1, -1)[..., 0, 0, 0]) + at(-1, -1)[..., 0, 0, 1]
        field_out[..., 0, 1] = 2 * quad(at(-1, -1))
        field_out[..., 1, 0] = (k + at(1, 1)[..., 0, 0, 0]) + at(1, 1)[..., 0, 0, 1]
        field_out[..., 1, 1] = 3 * quad(at(1, 1))
        field_out[..., 2, 0] = (k + at(0, 0)[..., 0, 0, 0]) + at(-1, 1)[..., 0, 0, 1]
        field_out[..., 2, 1] = 4 * quad(at(-1, 1))


# ------------------------------------------------------------------------------ K offsets
class TestReadOutsideKInterval1(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float64, "field_out": np.float64}
    domain_range = [(4, 4), (4, 4), (4, 4)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=[(0, 0), (0, 0), (1, 1)]),
        "field_out": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
    }

    def definition(field_in, field_out):
        with computation(PARALLEL), interval(...):
            field_out = field_in[0, 0, -1] + field_in[0, 0, 1]

    def validation(field_in, field_out, *, domain, origin):
        field_out[...] = field_in[..., :-2] + field_in[..., 2:]


class TestReadOutsideKInterval2(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float64, "field_out": np.float64}
    domain_range = [(4, 4), (4, 4), (4, 4)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=[(0, 0), (0, 0), (0, 1)]),
        "field_out": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
    }

    def definition(field_in, field_out):
        with computation(PARALLEL), interval(-1, None):
            field_out = field_in[0, 0, 1]

    def validation(field_in, field_out, *, domain, origin):
        field_out[..., domain[2] - 1] = field_in[..., domain[2]]


class TestReadOutsideKInterval3(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float64, "field_out": np.float64}
    domain_range = [(4, 4), (4, 4), (4, 4)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=[(0, 0), (0, 0), (1, 0)]),
        "field_out": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
    }

    def definition(field_in, field_out):
        with computation(PARALLEL), interval(0, 1):
            field_out = field_in[0, 0, -1]

    def validation(field_in, field_out, *, domain, origin):
        field_out[..., 0] = field_in[..., 0]  # field_in starts one level below the domain


class TestVariableKRead(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float32, "field_out": np.float32, "index": np.int32}
    domain_range = [(2, 2), (2, 2), (2, 8)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
        "field_out": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
        "index": fld(in_range=(-1, 0), axes="K", boundary=NO_HALO),
    }

    def definition(field_in, field_out, index):
        with computation(PARALLEL), interval(1, None):
            field_out = field_in[0, 0, index]

    def validation(field_in, field_out, index, *, domain, origin):
        for k in range(1, field_out.shape[2]):
            field_out[:, :, k] = field_in[:, :, k + index[k]]


class TestVariableKAndReadOutside(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float64, "field_out": np.float64, "index": np.int32}
    domain_range = [(2, 2), (2, 2), (2, 8)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(0.1, 10), axes="IJK", boundary=[(0, 0), (0, 0), (1, 0)]),
        "field_out": fld(in_range=(0.1, 10), axes="IJK", boundary=NO_HALO),
        "index": fld(in_range=(-1, 0), axes="K", boundary=NO_HALO),
    }

    def definition(field_in, field_out, index):
        with computation(PARALLEL), interval(1, None):
            field_out[0, 0, 0] = field_in[0, 0, index] + field_in[0, 0, -2]

    def validation(field_in, field_out, index, *, domain, origin):
        for k in range(1, domain[2]):  # field_in level k of the domain is array level k + 1
            field_out[:, :, k] = field_in[:, :, 1 + k + index[k]] + field_in[:, :, k - 1]


class TestDiagonalKOffset(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float64, "field_out": np.float64}
    domain_range = [(2, 2), (2, 2), (2, 8)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(0.1, 10), axes="IJK", boundary=[(0, 0), (1, 0), (0, 1)]),
        "field_out": fld(in_range=(0.1, 10), axes="IJK", boundary=NO_HALO),
    }

    def definition(field_in, field_out):
        with computation(PARALLEL), interval(...):
            field_out = field_in[0, 0, 1]
        with computation(PARALLEL), interval(0, -1):
            field_out += field_in[0, -1, 1]

    def validation(field_in, field_out, *, domain, origin):
        up = field_in[:, 1:, 1:]
        south_up = field_in[:, :-1, 1:]
        field_out[...] = up
        field_out[..., :-1] += south_up[..., :-1]


# ------------------------------------------------------------------------------ horizontal regions
class TestHorizontalRegions(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float32, "field_out": np.float32}
    domain_range = [(4, 4), (4, 4), (2, 2)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
        "field_out": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
    }

    def definition(field_in, field_out):
        with computation(PARALLEL), interval(...):
            field_out = field_in
            with horizontal(region[I[0], :], region[I[-1], :]):
                field_out = field_in + 1.0
            with horizontal(region[:, J[0]], region[:, J[-1]]):
                field_out = field_in - 1.0

    def validation(field_in, field_out, *, domain, origin):
        field_out[...] = field_in
        field_out[[0, -1]] = field_in[[0, -1]] + 1.0
        field_out[:, [0, -1]] = field_in[:, [0, -1]] - 1.0


class TestHorizontalRegionsPartialWrites(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float32, "field_out": np.float32}
    domain_range = [(4, 4), (4, 4), (2, 2)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
        "field_out": fld(in_range=(42, 42), axes="IJK", boundary=NO_HALO),
    }

    def definition(field_in, field_out):
        with computation(PARALLEL), interval(...):
            with horizontal(region[I[0], :], region[I[-1], :]):
                field_out = field_in + 1.0
            with horizontal(region[:, J[0]], region[:, J[-1]]):
                field_out = field_in - 1.0

    def validation(field_in, field_out, *, domain, origin):
        field_out[[0, -1]] = field_in[[0, -1]] + 1.0
        field_out[:, [0, -1]] = field_in[:, [0, -1]] - 1.0


class TestHorizontalRegionsCorners(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float32, "field_out": np.float32}
    domain_range = [(4, 4), (4, 4), (2, 2)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
        "field_out": fld(in_range=(42, 42), axes="IJK", boundary=NO_HALO),
    }

    def definition(field_in, field_out):
        with computation(PARALLEL), interval(...):
            with horizontal(
                region[I[0] : I[0] + 2, J[0] : J[0] + 2], region[I[-1] - 2 : I[-1], J[-1] - 2 : J[-1]]
            ):
                field_out = field_in + 1.0
            with horizontal(
                region[I[0] : I[0] + 2, J[-1] - 2 : J[-1]], region[I[-1] - 2 : I[-1], J[0] : J[0] + 2]
            ):
                field_out = field_in - 1.0

    def validation(field_in, field_out, *, domain, origin):
        n, m = field_out.shape[:2]
        lo_i, hi_i = slice(0, 2), slice(n - 3, n - 1)  # I[-1] is the last index: [I[-1]-2, I[-1])
        lo_j, hi_j = slice(0, 2), slice(m - 3, m - 1)
        for si, sj, d in ((lo_i, lo_j, 1.0), (hi_i, hi_j, 1.0), (lo_i, hi_j, -1.0), (hi_i, lo_j, -1.0)):
            field_out[si, sj] = field_in[si, sj] + d


# ------------------------------------------------------------------------------ typed / vector temporaries
class TestTypedTemporary(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float32, "field_out": np.float32}
    domain_range = [(2, 2), (2, 2), (2, 8)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
        "field_out": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO),
    }

    def definition(field_in, field_out):
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

    def validation(field_in, field_out, *, domain, origin):
        field_out[..., :-1] = field_in[..., :-1] + field_in[..., 1:]
        field_out[..., -1] = 0


class TestVectorGenAssignment(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float64, "field_out": np.float64}
    domain_range = [(2, 2), (2, 2), (2, 2)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(2,)),
        "field_out": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(2,)),
    }

    def definition(field_in, field_out):
        with computation(PARALLEL), interval(...):
            field_out = 2 * field_in

    def validation(field_in, field_out, *, domain, origin):
        np.multiply(field_in, 2, out=field_out)


class TestMatrixAssignment(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float32, "field_out": np.float32}
    domain_range = [(2, 2), (2, 2), (2, 2)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(2, 3)),
        "field_out": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(2, 3)),
    }

    def definition(field_in, field_out):
        with computation(PARALLEL), interval(...):
            field_out = field_in

    def validation(field_in, field_out, *, domain, origin):
        np.copyto(field_out, field_in)


class TestVectorVectorOp(gt_testing.StencilTestSuite):
    dtypes = {"field_1": np.float32, "field_2": np.float32, "field_out": np.float32}
    domain_range = [(2, 2), (2, 2), (2, 2)]
    backends = BACKENDS
    symbols = {n: fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(2,))
               for n in ("field_1", "field_2", "field_out")}

    def definition(field_1, field_2, field_out):
        with computation(PARALLEL), interval(...):
            field_out = field_1 + field_2

    def validation(field_1, field_2, field_out, *, domain, origin):
        np.add(field_1, field_2, out=field_out)


class TestCombinedVectorScalarOp(gt_testing.StencilTestSuite):
    dtypes = {"field_1": np.float64, "field_2": np.float64, "field_out": np.float64}
    domain_range = [(2, 2), (2, 2), (2, 2)]
    backends = BACKENDS
    symbols = {n: fld(in_range=(1, 10), axes="IJK", boundary=NO_HALO, data_dims=(2,))
               for n in ("field_1", "field_2", "field_out")}

    def definition(field_1, field_2, field_out):
        with computation(PARALLEL), interval(...):
            field_out = 3 * (field_1 + field_2 * field_2)

    def validation(field_1, field_2, field_out, *, domain, origin):
        field_out[...] = 3 * (field_1 + np.square(field_2))


class TestVectorizedTemporary(gt_testing.StencilTestSuite):
    dtypes = {"field_in": np.float32, "field_out": np.float32}
    domain_range = [(2, 2), (2, 2), (2, 2)]
    backends = BACKENDS
    symbols = {
        "field_in": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(2,)),
        "field_out": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(2,)),
    }

    def definition(field_in, field_out):
        tmp: Field[(np.float32, (2,))] = 0
        with computation(PARALLEL), interval(...):
            tmp[0, 0, 0][0] = 2
            tmp[0, 0, 0][1] = 3
            field_out = tmp * field_in

    def validation(field_in, field_out, *, domain, origin):
        field_out[...] = field_in * np.array([2, 3], dtype=field_in.dtype)


class TestMatmul(gt_testing.StencilTestSuite):
    dtypes = {"matrix": np.float64, "field_1": np.float64, "field_2": np.float64}
    domain_range = [(2, 2), (2, 2), (2, 2)]
    backends = BACKENDS
    symbols = {
        "matrix": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(4, 6)),
        "field_1": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(6,)),
        "field_2": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(4,)),
    }

    def definition(matrix, field_1, field_2):
        with computation(PARALLEL):
            with interval(0, 1):
                field_2 = matrix @ field_1
            with interval(1, 2):
                field_1 = matrix.T @ field_2

    def validation(matrix, field_1, field_2, *, domain, origin):
        field_2[:, :, 0] = (matrix[:, :, 0] @ field_1[:, :, 0, :, None])[..., 0]
        field_1[:, :, 1] = (np.swapaxes(matrix[:, :, 1], -1, -2) @ field_2[:, :, 1, :, None])[..., 0]


class TestMaskedMatmul(gt_testing.StencilTestSuite):
    dtypes = {"matrix": np.float64, "field_1": np.float64, "field_2": np.float64}
    domain_range = [(2, 2), (2, 2), (2, 2)]
    backends = BACKENDS
    symbols = {
        "matrix": fld(in_range=(-10, 10), axes="K", boundary=NO_HALO, data_dims=(4, 6)),
        "field_1": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(6,)),
        "field_2": fld(in_range=(-10, 10), axes="IJK", boundary=NO_HALO, data_dims=(4,)),
    }

    def definition(matrix, field_1, field_2):
        with computation(PARALLEL):
            with interval(0, 1):
                field_2 = matrix @ field_1
            with interval(1, 2):
                field_1 = matrix.T @ field_2

    def validation(matrix, field_1, field_2, *, domain, origin):
        field_2[:, :, 0] = field_1[:, :, 0] @ matrix[0].T
        field_1[:, :, 1] = field_2[:, :, 1] @ matrix[1]
