"""``StencilTestSuite``: Hypothesis-driven parity suites for GTScript stencils.

User-facing contract of ``gt4py.cartesian.testing.suites`` (``SuiteMeta`` ``suites.py:50-356``,
``StencilTestSuite`` ``:359-624``): a ``Test*`` class declares ``dtypes``, ``domain_range``,
``backends``, ``symbols``, a stencil ``definition`` and a numpy ``validation`` function with the
same signature (plus ``domain`` / ``origin`` keywords). The metaclass expands the class into two
parametrized pytest methods per (backend, dtype combination, external set):

* ``test_generation`` builds the stencil (for ``gt:mi355x``: code generation and the gfx950
  compile, which run on the CPU) and checks its field boundaries against the declared ones;
* ``test_implementation`` draws domains and inputs with Hypothesis, runs the stencil on the
  backend's storages, runs ``validation`` on cropped numpy copies and compares every field
  (``assert_allclose`` with the reference's ``RTOL``/``ATOL``).

MI355X-specific choices: implementation tests of device backends carry the ``gpu`` marker (this
repository's split between the CPU suite and the GPU box) and skip without a ROCm device; an
implementation test builds its stencil itself when the generation test did not run in the same
process (the in-process cache and the content-hashed HIP cache make that a lookup); device
results are copied to the host for the comparison, so every backend's outputs are checked.
"""

from __future__ import annotations

import copy
import inspect
import itertools
import os
import sys
import types
from typing import Any, Dict, List, Sequence, Tuple

import numpy as np

from gt4py_amd.definitions import AccessKind, FieldInfo
from gt4py_amd.testing.symbols import Symbol, SymbolKind

RTOL = 1e-05
ATOL = 1e-08
EQUAL_NAN = False

_REQUIRED = ("domain_range", "symbols", "definition", "validation", "backends", "dtypes")


def _examples() -> int:
    return int(os.environ.get("GTMI_SUITE_EXAMPLES", "25"))


def _settings():
    import hypothesis as hyp

    return hyp.settings(
        max_examples=_examples(),
        deadline=None,
        suppress_health_check=[hyp.HealthCheck.too_slow, hyp.HealthCheck.data_too_large],
        database=None,
    )


def _normalize_dtypes(dtypes, symbol_names) -> Dict[Tuple[str, ...], List[np.dtype]]:
    """``{group of names: [dtypes]}``; a bare sequence applies to every symbol (suites.py:317-319)."""
    if not isinstance(dtypes, dict):
        dtypes = {tuple(symbol_names): dtypes}
    out: Dict[Tuple[str, ...], List[np.dtype]] = {}
    for key, val in dtypes.items():
        names = (key,) if isinstance(key, str) else tuple(key)
        if not all(isinstance(n, str) for n in names):
            raise AssertionError("Invalid key in 'dtypes'.")
        vals = (val,) if isinstance(val, (type, np.dtype)) else tuple(val)
        out[names] = [np.dtype(v) for v in vals]
    seen = [n for names in out for n in names]
    if len(seen) != len(set(seen)):
        raise ValueError("Any field can be in only one group.")
    return out


def _dtype_combinations(groups: Dict[Tuple[str, ...], List[np.dtype]]) -> List[Dict[str, np.dtype]]:
    combos = []
    for choice in itertools.product(*groups.values()):
        combos.append({n: dt for names, dt in zip(groups.keys(), choice) for n in names})
    return combos


def _annotated(definition, annotations: Dict[str, Any]):
    """A copy of ``definition`` whose arguments carry the given type annotations."""
    fn = types.FunctionType(definition.__code__, definition.__globals__, definition.__name__,
                            definition.__defaults__, definition.__closure__)
    fn.__kwdefaults__ = copy.copy(definition.__kwdefaults__)
    fn.__module__ = definition.__module__
    spec = inspect.getfullargspec(fn)
    fn.__annotations__ = {k: annotations[k] for k in list(spec.args) + list(spec.kwonlyargs)}
    return fn


def _backend_name(b) -> str:
    return b if isinstance(b, str) else b.values[0]


def _backend_is_device(name: str) -> bool:
    from gt4py_amd.backend import from_name

    return from_name(name).storage_info["device"] == "gpu"


class _SuiteMeta(type):
    """Expands a ``StencilTestSuite`` subclass into parametrized generation/implementation tests."""

    def __new__(mcs, cls_name, bases, ns):
        if ns.get("_skip_", False):
            return super().__new__(mcs, cls_name, bases, ns)
        for key in _REQUIRED:  # inherited members (e.g. a suite re-run with other backends)
            if key not in ns:
                for b in bases:
                    if hasattr(b, key):
                        ns[key] = getattr(b, key)
                        break
        missing = [k for k in _REQUIRED if k not in ns]
        if missing:
            raise TypeError(f"Missing {set(missing)} required members in '{cls_name}' definition")
        mcs._check(cls_name, ns)
        mcs._analyse(cls_name, ns)
        mcs._expand(cls_name, ns)
        return super().__new__(mcs, cls_name, bases, ns)

    @staticmethod
    def _check(cls_name, ns):
        from gt4py_amd.backend import REGISTRY

        import pytest

        param_type = type(pytest.param())
        dr = ns["domain_range"]
        assert 1 <= len(dr) <= 3 and all(len(d) == 2 for d in dr), "Invalid 'domain_range' definition"
        ns["ndims"] = len(dr)
        if cls_name[-2:] in ("1D", "2D", "3D"):
            assert ns["ndims"] == int(cls_name[-2]), "Suite name does not match the actual 'ndims'"
        if not isinstance(ns["symbols"], dict):
            raise AssertionError("Invalid 'symbols' mapping")
        backends = []
        for b in ns["backends"]:
            if not (isinstance(b, str) or (isinstance(b, param_type) and len(b.values) == 1
                                           and isinstance(b.values[0], str))):
                raise TypeError("'backends' must be a sequence of strings")
            if _backend_name(b) in REGISTRY:
                backends.append(b)
        ns["backends"] = backends
        for attr in ("definition", "validation"):
            if not isinstance(ns[attr], types.FunctionType):
                raise TypeError(f"The '{attr}' attribute must be a "
                                + ("stencil definition function" if attr == "definition" else "validation function"))
        dsig = inspect.signature(ns["definition"]).parameters
        vsig = inspect.signature(ns["validation"]).parameters
        for (dn, dp), (vn, vp) in zip(dsig.items(), vsig.items()):
            if dn != vn or dp.kind != vp.kind:
                raise ValueError("Incompatible signatures for 'definition' and 'validation' functions")
            if dp.kind == inspect.Parameter.KEYWORD_ONLY and dp.default is not inspect.Parameter.empty:
                assert dp.default == vp.default
        run_names = {n for n, p in dsig.items()}
        declared = {n for n, s in ns["symbols"].items()
                    if s.kind in (SymbolKind.FIELD, SymbolKind.PARAMETER, SymbolKind.NONE)}
        assert run_names == declared, f"Missing or invalid keys in 'symbols' mapping (generated: {declared})"
        ns["dtypes"] = _normalize_dtypes(ns["dtypes"], list(ns["symbols"].keys()))

    @staticmethod
    def _analyse(cls_name, ns):
        symbols: Dict[str, Symbol] = ns["symbols"]
        lo = [0, 0, 0]
        hi = [0, 0, 0]
        for s in symbols.values():
            if s.kind == SymbolKind.FIELD:
                for d, (a, b) in enumerate(s.boundary):
                    lo[d], hi[d] = max(lo[d], a), max(hi[d], b)
        ns["max_boundary"] = tuple(zip(lo, hi))
        ns["origin"] = tuple(lo)
        ns["field_params"] = {
            n: (s.axes or "IJK", tuple(s.data_dims)) for n, s in symbols.items() if s.kind == SymbolKind.FIELD
        }
        ns["global_boundaries"] = {n: s.boundary for n, s in symbols.items() if s.kind == SymbolKind.FIELD}
        ns["constants"] = {n: s.values for n, s in symbols.items() if s.kind == SymbolKind.GLOBAL_SET}
        ns["singletons"] = {n: s.values[0] for n, s in symbols.items() if s.kind == SymbolKind.SINGLETON}
        ns["drawn_globals"] = {n: s for n, s in symbols.items() if s.kind == SymbolKind.GLOBAL_STRATEGY}

    @staticmethod
    def _expand(cls_name, ns):
        import pytest

        from gt4py_amd import gtscript

        field_params = ns["field_params"]
        tests = []
        for b in ns["backends"]:
            bname = _backend_name(b)
            for dts in _dtype_combinations(ns["dtypes"]):
                const_names = list(ns["constants"])
                for values in itertools.product(*ns["constants"].values()):
                    consts = {n: dts[n].type(v) if n in dts else v for n, v in zip(const_names, values)}
                    ann = {}
                    for n, dt in dts.items():
                        if n in field_params:
                            axes, ddims = field_params[n]
                            ann[n] = gtscript.Field[getattr(gtscript, axes), (dt.type, ddims)]
                        else:
                            ann[n] = dt.type
                    tid = bname + "".join(f"_{k}_{v}" for k, v in consts.items())
                    tid += "".join(f"_{k}_{v.name}" for k, v in dts.items())
                    marks = [] if isinstance(b, str) else list(b.marks)
                    tests.append(dict(
                        backend=bname, suite=cls_name, constants=consts, dtypes=dts, marks=marks, id=tid,
                        index=len(tests), definition=_annotated(ns["definition"], ann), implementation=None,
                    ))
        ns["tests"] = tests

        gen_params = [pytest.param(t, marks=t["marks"], id=t["id"]) for t in tests]
        impl_params = []
        for t in tests:
            marks = list(t["marks"])
            if _backend_is_device(t["backend"]):
                marks.append(pytest.mark.gpu)
            impl_params.append(pytest.param(t, marks=marks, id=t["id"]))

        def test_generation(self, test):
            type(self)._test_generation(test)

        def test_implementation(self, test):
            type(self)._test_implementation(test)

        ns["test_generation"] = pytest.mark.parametrize("test", gen_params)(test_generation)
        ns["test_implementation"] = pytest.mark.parametrize("test", impl_params)(test_implementation)


class StencilTestSuite(metaclass=_SuiteMeta):
    """Base class of every stencil test suite (see the module docstring for the contract)."""

    _skip_ = True

    # ------------------------------------------------------------------ generation
    @classmethod
    def _externals(cls, test) -> Dict[str, Any]:
        ext = dict(test["constants"])
        ext.update(cls.singletons)
        if cls.drawn_globals:  # one deterministic draw per test (seeded by the test index)
            rng = np.random.default_rng(test["index"])
            for n, s in cls.drawn_globals.items():
                lo, hi = s.value_range
                dt = test["dtypes"].get(n, np.dtype(np.float64))
                v = rng.integers(lo, hi + 1) if dt.kind in "iu" else rng.uniform(lo, hi)
                ext[n] = dt.type(v)
        return ext

    @classmethod
    def _build(cls, test, rebuild: bool):
        from gt4py_amd import gtscript

        slug = "".join(ch for ch in test["backend"] if ch.isalnum())
        ext = cls._externals(test)
        impl = gtscript.stencil(
            backend=test["backend"], definition=test["definition"], externals=ext, rebuild=rebuild,
            name=f"{cls.__module__}.{test['suite']}_{slug}_{test['index']}",
        )
        for k, v in ext.items():
            impl.constants[k] = v
        test["implementation"] = impl
        return impl

    @classmethod
    def _test_generation(cls, test):
        from gt4py_amd.stencil_object import StencilObject

        impl = cls._build(test, rebuild=False)
        assert isinstance(impl, StencilObject)
        assert impl.backend == test["backend"]
        for name, info in impl.field_info.items():
            if info is None or info.access == AccessKind.NONE:
                continue
            declared = cls.global_boundaries[name]
            for d, ax in enumerate("IJ"):
                if ax in info.axes:
                    assert tuple(info.boundary[d]) >= tuple(declared[d]), (
                        f"field '{name}': boundary {info.boundary} smaller than declared {declared}"
                    )

    # ------------------------------------------------------------------ implementation
    @classmethod
    def _input_strategy(cls, test):
        """Hypothesis strategy of one set of run-time inputs (shared domain, per-field halos)."""
        import hypothesis.strategies as st
        from hypothesis.extra import numpy as hnp

        domain_st = st.tuples(*[st.integers(a, b) for a, b in cls.domain_range])
        dts = test["dtypes"]

        @st.composite
        def draw_inputs(draw):
            dom = tuple(draw(domain_st)) + (0,) * (3 - len(cls.domain_range))
            out = {}
            for name, sym in cls.symbols.items():
                if sym.kind == SymbolKind.FIELD:
                    axes, ddims = cls.field_params[name]
                    shape = tuple(dom[d] + lo + hi for d, ((lo, hi), ax) in
                                  enumerate(zip(cls.max_boundary, "IJK")) if ax in axes)
                    shape = shape + tuple(ddims)
                    el = sym.value_strategy(dts[name])
                    out[name] = draw(hnp.arrays(dts[name], shape, elements=el, fill=el))
                elif sym.kind in (SymbolKind.PARAMETER, SymbolKind.NONE):
                    out[name] = draw(sym.value_strategy(dts.get(name, np.dtype(np.float64))))
            return out

        return draw_inputs()

    @classmethod
    def _test_implementation(cls, test):
        from hypothesis import given

        if _backend_is_device(test["backend"]):
            import torch

            if not torch.cuda.is_available():
                import pytest

                pytest.skip(f"{test['backend']} needs a ROCm device")
        impl = test["implementation"] or cls._build(test, rebuild=False)

        @_settings()
        @given(inputs=cls._input_strategy(test))
        def run(inputs):
            cls._run_test_implementation(inputs, impl)

        run()

    @classmethod
    def _run_test_implementation(cls, inputs: Dict[str, Any], impl, exec_info=None):
        from gt4py_amd import storage

        masks = {n: tuple(ax in cls.field_params[n][0] for ax in "IJK") for n, v in inputs.items()
                 if isinstance(v, np.ndarray)}
        # data shape: the smallest extent of every axis over the fields that have it
        data_shape = [sys.maxsize] * 3
        for n, m in masks.items():
            it = iter(inputs[n].shape)
            for d in range(3):
                if m[d]:
                    data_shape[d] = min(data_shape[d], next(it))
        lo = [b[0] for b in cls.max_boundary]
        hi = [b[1] for b in cls.max_boundary]
        domain = tuple(data_shape[d] - lo[d] - hi[d] for d in range(3))

        referenced = {n for n, i in impl.field_info.items() if i is not None}
        referenced |= {n for n, i in impl.parameter_info.items() if i is not None}
        module = sys.modules.get(cls.__module__)
        if module is not None:  # externals are visible to the validation function as globals
            for k, v in impl.constants.items():
                module.__dict__[k] = v

        run_args, expected = {}, {}
        for n, v in inputs.items():
            if n not in referenced:
                run_args[n] = expected[n] = None
            elif isinstance(impl.field_info.get(n), FieldInfo):
                axes, ddims = cls.field_params[n]
                dt = (v.dtype, ddims) if ddims else v.dtype
                run_args[n] = storage.from_array(
                    v, dt, backend=impl.backend, dimensions=tuple(axes),
                    aligned_index=tuple(o for o, m in zip(cls.origin, masks[n]) if m),
                )
                expected[n] = np.array(v)
            else:
                run_args[n] = expected[n] = v

        impl(**run_args, origin=cls.origin, domain=domain, exec_info=exec_info)

        # validation sees each field cropped to the region its own boundary frames
        cropped = {}
        for n, v in expected.items():
            sym = cls.symbols[n]
            if v is None or sym.kind != SymbolKind.FIELD:
                cropped[n] = v
                continue
            sl = []
            for d in range(3):
                if masks[n][d]:
                    a = lo[d] - sym.boundary[d][0]
                    b = data_shape[d] - (hi[d] - sym.boundary[d][1])
                    sl.append(slice(a, b))
            sl += [slice(None)] * len(cls.field_params[n][1])
            cropped[n] = v[tuple(sl)]
        cls.validation(
            **cropped, domain=domain,
            origin={n: i.boundary.lower_indices for n, i in impl.field_info.items() if i is not None},
        )
        for n, v in run_args.items():
            if n in masks and v is not None:
                np.testing.assert_allclose(
                    storage.to_numpy(v), expected[n], rtol=RTOL, atol=ATOL, equal_nan=EQUAL_NAN,
                    err_msg=f"Wrong data in output field '{n}'",
                )
