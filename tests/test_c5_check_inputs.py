"""The sharded C5 checker's own logic, on the CPU (tests/c5_sharded_check.py): each rank builds its
strip of the global input from global indices, so the strips must be slices of one global field,
and the C oracle on a strip (its halo rows from the same formula) must reproduce the oracle on the
whole domain -- otherwise a bit-exact per-rank comparison would not prove the global result."""

import numpy as np

import c5_sharded_check as c5


def test_strips_are_slices_of_one_global_input():
    ni, nj, nk, h, world = 48, 10, 3, 2, 4
    full = c5.global_in(ni, nj * world, -h, ni + h, -h, nj * world + h, 0, nk)
    cfull = c5.global_coeff(0, ni, 0, nj * world, 0, nk)
    for r in range(world):
        j0 = r * nj
        strip = c5.global_in(ni, nj * world, -h, ni + h, j0 - h, j0 + nj + h, 0, nk)
        np.testing.assert_array_equal(strip, full[:, j0:j0 + nj + 2 * h, :])
        np.testing.assert_array_equal(c5.global_coeff(0, ni, j0, j0 + nj, 0, nk), cfull[:, j0:j0 + nj, :])
    assert full.dtype == np.float32 and np.isfinite(full).all()
    assert 0.025 <= cfull.min() and cfull.max() < 0.125


def test_oracle_on_strips_equals_oracle_on_the_whole_domain():
    from oracle import c_oracle

    ni, nj, nk, h, world = 40, 9, 4, 2, 3
    origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    a = c5.global_in(ni, nj * world, -h, ni + h, -h, nj * world + h, 0, nk)
    c = c5.global_coeff(0, ni, 0, nj * world, 0, nk)
    ref = np.zeros((ni, nj * world, nk), dtype=np.float32, order="F")
    c_oracle.horizontal_diffusion(a, ref, c, origin, (ni, nj * world, nk), nthreads=1)
    for r in range(world):
        j0 = r * nj
        sa = c5.global_in(ni, nj * world, -h, ni + h, j0 - h, j0 + nj + h, 0, nk)
        sc_ = c5.global_coeff(0, ni, j0, j0 + nj, 0, nk)
        out = np.zeros((ni, nj, nk), dtype=np.float32, order="F")
        c_oracle.horizontal_diffusion(sa, out, sc_, origin, (ni, nj, nk), nthreads=1)
        np.testing.assert_array_equal(out, ref[:, j0:j0 + nj, :])
