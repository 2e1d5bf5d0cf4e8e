"""Drop-in halos: every field allocated with EXACTLY the boundary the reference reports in
``field_info`` (its ``FieldInfo.boundary``, stored in each golden's metadata by
tests/golden/make_golden.py), no more. A reference user sizes arrays from that boundary, so the
same call must validate and give the golden results here. Horizontal regions make this sharp:
the reference clips a region's reads by the region's mask (``oir_optimizations/utils.py:50-75``),
so e.g. ``b[-1, 0, 0]`` read only in an east-edge region needs no west halo
(``region_offset_reads``). Run on the numpy backend (CPU) and on gt:mi355x (GPU), whose kernels
clamp every load to the array they are given.
"""

import numpy as np
import pytest

import golden_utils as gu
import stencil_cases as sc
from gt4py_amd import gtscript

BK = "gt:mi355x"


def _eligible(name):
    case = sc.CASES[name]
    if not isinstance(case.origin, dict) or case.domain is None or case.externals:
        return False
    _, _, meta = gu.load(name)
    fi = meta["field_info"]
    ins = case.make_inputs()
    return all(v is not None and v.ndim == 3 and n in fi and fi[n]["axes"] == ["I", "J", "K"]
               for n, v in ins.items())


CASES = [n for n in gu.available() if _eligible(n)]
assert "region_offset_reads" in CASES


def tight(name):
    """(inputs, origin, expected outputs) with every field cut to the reference's boundary."""
    case = sc.CASES[name]
    _, outputs, meta = gu.load(name)
    host = case.make_inputs()
    ni, nj, _ = case.domain
    ins, org, want = {}, {}, {}
    for f, arr in host.items():
        (ilo, ihi), (jlo, jhi), _ = meta["field_info"][f]["boundary"]
        oi, oj, ok = case.origin[f]
        sl = (slice(oi - ilo, oi + ni + ihi), slice(oj - jlo, oj + nj + jhi), slice(None))
        ins[f] = np.ascontiguousarray(arr[sl])
        org[f] = (ilo, jlo, ok)
        want[f] = outputs[f][sl]
    return ins, org, want


@pytest.mark.parametrize("name", CASES)
def test_tight_boundary_numpy(name):
    case = sc.CASES[name]
    ins, org, want = tight(name)
    st = gtscript.stencil(backend="numpy", definition=case.definition, name=f"tight.{name}")
    arrays = {k: v.copy() for k, v in ins.items()}
    st(**arrays, **case.params, origin=org, domain=case.domain)
    for k, v in want.items():
        gu.assert_match(arrays[k], v, rtol=case.rtol, atol=case.atol, name=f"{name}:{k}")


def test_region_reads_are_clipped_like_the_reference():
    st = gtscript.stencil(backend="numpy", definition=sc.region_offset_reads, name="tight.region_fi")
    fi = st.field_info
    assert [list(x) for x in fi["b"].boundary] == [[0, 0], [0, 0], [0, 0]]
    assert [list(x) for x in fi["a"].boundary] == [[0, 0], [0, 1], [0, 0]]


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_tight_boundary_gpu(name):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import storage

    case = sc.CASES[name]
    ins, org, want = tight(name)
    st = gtscript.stencil(backend=BK, definition=case.definition, name=f"gpu.{name}")
    # a negative boundary (a field read only at positive offsets) gives a negative origin: the
    # array starts inside the domain, as the reference allows
    dev = {k: storage.from_array(v, None, backend=BK, aligned_index=tuple(max(0, x) for x in org[k]))
           for k, v in ins.items()}
    st(**dev, **case.params, origin=org, domain=case.domain)
    for k, v in want.items():
        gu.assert_match(storage.to_numpy(dev[k]), v, rtol=case.rtol, atol=case.atol, name=f"{name}:{k}")
