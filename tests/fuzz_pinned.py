"""The differential-fuzz programs pinned to the reference numpy backend
(tests/golden/fuzz_reference.json, made by tests/golden/make_fuzz_golden.py)."""

import fuzz_stencils

# the default fuzz seeds (f64 programs: PARALLEL/FORWARD/BACKWARD, horizontal regions, staged
# sweeps, sweep pairs and tile templates), the mixed-precision, K-offset,
# lower-dimensional-field, operator,
# while-loop / horizontal-region, mixed tile,
# gtscript-function, run-time K offset,
# interval-partition and absolute-K programs
N_MIXED, N_KOFF, N_LOWDIM, N_OPS, N_CTRL, N_TILE, N_FUNC, N_VK, N_IVL, N_ABSK = 160, 80, 60, 100, 100, 60, 60, 60, 60, 40
# programs the reference refuses: its upcaster raises "Type mismatch in `BinaryOp`. Types are
# FLOAT32, INT64" on a comparison of sqrt(<int64>) (typed float32, as ours types it too) with an
# int64; gt:mi355x accepts them. tests/test_fuzz.py still runs them against our
# numpy backend.
REFERENCE_REFUSED = {9850}
# while loops whose condition reads a value the body changes: the reference's numpy backend masks
# every statement of the body with the condition re-evaluated after the statements before it
# (oir_to_npir.py:176-185, npir_codegen.py:252-267), so `n = n + 1` after `acc = ...` sees the new
# acc; its debug backend and its GridTools backends run the loop per point, as gt:mi355x and our
# numpy backend do (per-point semantics pinned by the debug-backend golden
# `while_value_condition`). These programs are not pinned to the numpy backend.
REFERENCE_DIVERGENT = {s for s in range(fuzz_stencils.CTRL_BASE, fuzz_stencils.CTRL_BASE + 100)
                       if " and acc " in fuzz_stencils.generate(s)[0]}
PINNED = list(range(60)) + list(range(1000, 1060)) + list(range(7000, 7024)) + list(
    range(fuzz_stencils.MIXED_BASE, fuzz_stencils.MIXED_BASE + N_MIXED)) + list(
    range(fuzz_stencils.KOFF_BASE, fuzz_stencils.KOFF_BASE + N_KOFF)) + list(
    range(fuzz_stencils.LOWDIM_BASE, fuzz_stencils.LOWDIM_BASE + N_LOWDIM)) + list(
    range(fuzz_stencils.OPS_BASE, fuzz_stencils.OPS_BASE + N_OPS)) + list(
    range(fuzz_stencils.CTRL_BASE, fuzz_stencils.CTRL_BASE + N_CTRL)) + list(
    range(fuzz_stencils.TILE_BASE, fuzz_stencils.TILE_BASE + N_TILE)) + list(
    range(fuzz_stencils.FUNC_BASE, fuzz_stencils.FUNC_BASE + N_FUNC)) + list(
    range(fuzz_stencils.VK_BASE, fuzz_stencils.VK_BASE + N_VK)) + list(
    range(fuzz_stencils.IVL_BASE, fuzz_stencils.IVL_BASE + N_IVL)) + list(
    range(fuzz_stencils.ABSK_BASE, fuzz_stencils.ABSK_BASE + N_ABSK))
PINNED = [s for s in PINNED if s not in REFERENCE_REFUSED | REFERENCE_DIVERGENT]


# the same programs at >= 98 levels, where the column kernels switch on their register band, LDS
# tail cache and head/tail placement and tile kernels block levels: the sweep templates (sweep
# pairs and tiles, K-offset sweeps) and the first 40 mixed-precision programs
DEEP = [s for s in list(range(7000, 7024)) + list(range(fuzz_stencils.KOFF_BASE, fuzz_stencils.KOFF_BASE + N_KOFF))
        + list(range(fuzz_stencils.MIXED_BASE, fuzz_stencils.MIXED_BASE + 40))
        + list(range(fuzz_stencils.TILE_BASE, fuzz_stencils.TILE_BASE + 30))
        + list(range(fuzz_stencils.VK_BASE, fuzz_stencils.VK_BASE + 30))
        + list(range(fuzz_stencils.IVL_BASE, fuzz_stencils.IVL_BASE + 30)) if s in PINNED]
# golden record keys: "<seed>" at pinned_shape(seed), "<seed>@deep" at deep_shape(seed)
CASES = [(s, False) for s in PINNED] + [(s, True) for s in DEEP]


def pinned_shape(seed):
    """Small domains: odd seeds a width that is not a multiple of any lane or tile width."""
    return (13, 11, 8) if seed % 2 == 0 else (21, 9, 7)


def deep_shape(seed):
    return (13, 11, 120) if seed % 2 == 0 else (21, 9, 121)


def case_key(seed, deep):
    return f"{seed}@deep" if deep else str(seed)


def case_shape(seed, deep):
    return deep_shape(seed) if deep else pinned_shape(seed)
