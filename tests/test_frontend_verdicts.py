"""Accept / reject parity with the reference frontend (CPU): every program of
``tests/frontend_cases.py`` must be accepted by gt4py_amd exactly when the reference accepted it
(``tests/golden/frontend/verdicts.json``, recorded from the reference itself by
``tests/golden/make_frontend_verdicts.py``) and refused with the same exception class (gt4py_amd's
GTScript errors mirror the reference's hierarchy, ``gt4py_amd/frontend.py``). Where the reference
fails with an internal error (a bare KeyError) only the refusal is required.

Every accepted program also runs on the reference's seeded inputs and must give the reference's
results (``tests/golden/frontend/outputs.npz``): bit-exact on the numpy backend, and bit-exact on
gt:mi355x except for the programs in ``LIBM``, whose device sin/cos/asin/pow are compared at
rtol 1e-14 (glibc and the device math library round differently in the last place)."""

import json
import os

import numpy as np
import pytest

import frontend_cases as fc
from gt4py_amd import gtscript

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "frontend", "verdicts.json")) as _f:
    VERDICTS = json.load(_f)

OUTPUTS = np.load(os.path.join(HERE, "golden", "frontend", "outputs.npz"))
DOMAIN = (6, 5, 8)  # make_frontend_verdicts.DOMAIN
ACCEPTED = sorted(n for n, v in VERDICTS.items() if v["accepted"])
LIBM = {"native_offset_arg_ok", "native_nested_ok", "native_in_function_ok", "native_ternary_ok", "power_ok"}
_SPECIFIC = ("GTScriptSyntaxError", "GTScriptSymbolError", "GTScriptDefinitionError", "GTScriptValueError",
             "GTScriptDataTypeError", "GTScriptAssertionError", "ValueError", "TypeError")


def test_every_case_has_a_verdict():
    assert set(VERDICTS) == set(fc.CASES)


@pytest.mark.parametrize("name", sorted(fc.CASES))
def test_same_verdict_as_reference(name):
    defn, externals = fc.CASES[name]
    want = VERDICTS[name]
    try:
        gtscript.stencil(backend="numpy", definition=defn, externals=externals, name=f"verdict.{name}")
    except Exception as e:  # noqa: BLE001
        assert not want["accepted"], f"{name}: accepted by the reference, refused here: {type(e).__name__}: {e}"
        if want["error"] in _SPECIFIC:
            mro = [c.__name__ for c in type(e).__mro__]
            assert want["error"] in mro, (f"{name}: reference raised {want['error']} ({want['message'][:120]}), "
                                          f"gt4py_amd raised {type(e).__name__}: {e}")
        return
    assert want["accepted"], f"{name}: refused by the reference ({want['error']}: {want['message'][:160]}), accepted here"


def case_io(name):
    """(inputs, origin, params, expected) of an accepted case, from the reference's run."""
    ins, org, par, want = {}, {}, {}, {}
    pre = name + "__"
    for k in OUTPUTS.files:
        if not k.startswith(pre):
            continue
        kind, f = k[len(pre):].split("__", 1)
        v = OUTPUTS[k]
        if kind == "in":
            ins[f] = v
        elif kind == "org":
            org[f] = tuple(int(x) for x in v)
        elif kind == "par":
            par[f] = v[()]
        else:
            want[f] = v
    for f, v in ins.items():
        want.setdefault(f, v)  # fields the reference left unchanged
    return ins, org, par, want


def test_every_accepted_case_has_outputs():
    assert ACCEPTED and all(case_io(n)[0] for n in ACCEPTED)


@pytest.mark.parametrize("name", ACCEPTED)
def test_accepted_case_results_numpy(name):
    defn, externals = fc.CASES[name]
    ins, org, par, want = case_io(name)
    st = gtscript.stencil(backend="numpy", definition=defn, externals=externals, name=f"verdict.{name}")
    arrays = {k: v.copy() for k, v in ins.items()}
    st(**arrays, **par, origin=org, domain=DOMAIN)
    for k, v in want.items():
        np.testing.assert_array_equal(arrays[k], v, err_msg=f"{name}:{k}")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ACCEPTED)
def test_accepted_case_results_gpu(name):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import storage

    defn, externals = fc.CASES[name]
    ins, org, par, want = case_io(name)
    st = gtscript.stencil(backend="gt:mi355x", definition=defn, externals=externals, name=f"verdict.gpu.{name}")
    dev = {k: storage.from_array(v, None, backend="gt:mi355x", aligned_index=org[k] + (0,) * (v.ndim - len(org[k])))
           for k, v in ins.items()}
    st(**dev, **par, origin=org, domain=DOMAIN)
    for k, v in want.items():
        got = storage.to_numpy(dev[k])
        if name in LIBM:
            np.testing.assert_allclose(got, v, rtol=1e-14, atol=0, equal_nan=True, err_msg=f"{name}:{k}")
        else:
            np.testing.assert_array_equal(got, v, err_msg=f"{name}:{k}")
