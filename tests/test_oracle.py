"""Pin the CPU oracles (numpy + C restatements) against the reference golden vectors."""

import numpy as np
import pytest

import golden_utils as gu
import stencil_cases as sc
from oracle import c_oracle, numpy_oracle

HOT = {
    "copy": "copy_stencil",
    "copy_subdomain": "copy_stencil",
    "lap5": "lap5",
    "hdiff_f64": "horizontal_diffusion",
    "hdiff_f64_demo": "horizontal_diffusion",
    "hdiff_f64_origin": "horizontal_diffusion",
    "hdiff_f64_ties": "horizontal_diffusion",
    "hdiff_f64_nan": "horizontal_diffusion",
    "hdiff_f32": "horizontal_diffusion",
    "hdiff_f32_demo": "horizontal_diffusion",
    "tridiag": "tridiagonal_solver",
    "tridiag_k2": "tridiagonal_solver",
    "tridiag_subdomain": "tridiagonal_solver",
}


def _domain(case, inputs, origin, names):
    if case.domain is not None:
        return case.domain
    return tuple(min(inputs[n].shape[d] - origin[n][d] for n in names) for d in range(3))


@pytest.mark.parametrize("impl", ["numpy", "c"])
@pytest.mark.parametrize("name", sorted(HOT))
def test_oracle_matches_golden(name, impl):
    inputs, outputs, _ = gu.load(name)
    case = sc.CASES[name]
    mod = numpy_oracle if impl == "numpy" else c_oracle
    fn, names = mod.STENCILS[HOT[name]]
    origin = numpy_oracle.normalize_origin(case.origin, names)
    domain = _domain(case, inputs, origin, names)
    arrays = {n: inputs[n].copy() for n in names}
    if impl == "c":
        # exercise I-first (Fortran-order) strides too
        arrays = {n: np.asfortranarray(a) for n, a in arrays.items()}
    fn(*[arrays[n] for n in names], origin=origin, domain=domain)
    for n in names:
        gu.assert_match(arrays[n], outputs[n], name=f"{name}:{n}")


def test_case_inputs_reproducible():
    """The golden inputs are regenerated bit-identically from the case recipes."""
    for name in gu.available():
        inputs, _, _ = gu.load(name)
        regen = sc.CASES[name].make_inputs()
        for k, v in inputs.items():
            gu.assert_match(regen[k], v, name=f"{name}:{k}")
