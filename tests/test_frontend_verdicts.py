"""Accept / reject parity with the reference frontend (CPU): every program of
``tests/frontend_cases.py`` must be accepted by gt4py_amd exactly when the reference accepted it
(``tests/golden/frontend_verdicts.json``, recorded from the reference itself by
``tests/golden/make_frontend_verdicts.py``) and refused with the same exception class (gt4py_amd's
GTScript errors mirror the reference's hierarchy, ``gt4py_amd/frontend.py``). Where the reference
fails with an internal error (a bare KeyError) only the refusal is required."""

import json
import os

import pytest

import frontend_cases as fc
from gt4py_amd import gtscript

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "frontend_verdicts.json")) as _f:
    VERDICTS = json.load(_f)

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
