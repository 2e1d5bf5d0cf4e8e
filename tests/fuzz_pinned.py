"""The differential-fuzz programs pinned to the reference numpy backend
(tests/golden/fuzz_reference.json, made by tests/golden/make_fuzz_golden.py)."""

import fuzz_stencils

# the default fuzz seeds (f64 programs: PARALLEL/FORWARD/BACKWARD, horizontal regions, staged
# sweeps, sweep pairs and tile templates), the mixed-precision, K-offset and
# lower-dimensional-field programs
N_MIXED, N_KOFF, N_LOWDIM = 160, 80, 60
PINNED = list(range(60)) + list(range(1000, 1060)) + list(range(7000, 7024)) + list(
    range(fuzz_stencils.MIXED_BASE, fuzz_stencils.MIXED_BASE + N_MIXED)) + list(
    range(fuzz_stencils.KOFF_BASE, fuzz_stencils.KOFF_BASE + N_KOFF)) + list(
    range(fuzz_stencils.LOWDIM_BASE, fuzz_stencils.LOWDIM_BASE + N_LOWDIM))


def pinned_shape(seed):
    """Small domains: odd seeds a width that is not a multiple of any lane or tile width."""
    return (13, 11, 8) if seed % 2 == 0 else (21, 9, 7)
