"""Multi-process J-strip decomposition + halo exchange (gloo on CPU, world sizes 2 and 3).

Each rank owns a J strip whose interior halo rows start as NaN: only a correct exchange fills
them. The distributed result (interior/boundary split with the exchange overlapped) must equal
the single-domain result of the same stencil bit-for-bit (hdiff f64 and the lap5 stencil).
"""

import os
import socket
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, outdir, which):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import stencil_cases as sc
    from gt4py_amd import gtscript
    from gt4py_amd.distributed import HaloStencil, JStrips

    dist.init_process_group("gloo", rank=rank, world_size=world)
    ni, njg, nk, h = 12, 23, 4, (2 if which == "hdiff" else 1)
    rng = np.random.default_rng(11)
    gin = rng.uniform(-10, 10, (ni + 2 * h, njg + 2 * h, nk))
    gco = rng.uniform(0, 0.5, (ni, njg, nk))
    j0, j1 = JStrips(njg, world).bounds(rank)
    nj = j1 - j0
    lin = gin[:, j0 : j1 + 2 * h, :].copy()
    if rank > 0:
        lin[:, :h, :] = np.nan
    if rank < world - 1:
        lin[:, nj + h :, :] = np.nan
    t_in = torch.from_numpy(lin)
    t_out = torch.zeros((ni, nj, nk), dtype=torch.float64)
    if which == "hdiff":
        st = gtscript.stencil(backend="numpy", definition=sc.hdiff_f64, name="dist.hdiff")
        args = {"in_field": t_in, "out_field": t_out, "coeff": torch.from_numpy(gco[:, j0:j1, :].copy())}
        origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    else:
        st = gtscript.stencil(backend="numpy", definition=sc.lap5, name="dist.lap5")
        args = {"in_field": t_in, "out_field": t_out}
        origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0)}
    runner = HaloStencil(st, ["in_field"], nj, h, rank, world)
    runner(args, origin, (ni, nj, nk))
    np.save(os.path.join(outdir, f"out_{rank}.npy"), t_out.numpy())
    # the halos now hold the neighbours' rows
    np.save(os.path.join(outdir, f"in_{rank}.npy"), t_in.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,which", [(2, "hdiff"), (3, "hdiff"), (2, "lap5")])
def test_jstrip_halo_exchange_matches_single_domain(tmp_path, world, which):
    import torch.multiprocessing as mp

    sys.path.insert(0, REPO)
    import stencil_cases as sc
    from gt4py_amd import gtscript
    from gt4py_amd.distributed import JStrips

    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), which), nprocs=world, join=True)
    ni, njg, nk, h = 12, 23, 4, (2 if which == "hdiff" else 1)
    rng = np.random.default_rng(11)
    gin = rng.uniform(-10, 10, (ni + 2 * h, njg + 2 * h, nk))
    gco = rng.uniform(0, 0.5, (ni, njg, nk))
    ref = np.zeros((ni, njg, nk))
    if which == "hdiff":
        st = gtscript.stencil(backend="numpy", definition=sc.hdiff_f64, name="dist.hdiff")
        st(gin.copy(), ref, gco, origin={"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)})
    else:
        st = gtscript.stencil(backend="numpy", definition=sc.lap5, name="dist.lap5")
        st(gin.copy(), ref, origin={"in_field": (h, h, 0), "out_field": (0, 0, 0)})
    parts = [np.load(tmp_path / f"out_{r}.npy") for r in range(world)]
    got = np.concatenate(parts, axis=1)
    assert np.array_equal(got, ref)
    strips = JStrips(njg, world)
    for r in range(world):
        j0, j1 = strips.bounds(r)
        assert np.array_equal(np.load(tmp_path / f"in_{r}.npy"), gin[:, j0 : j1 + 2 * h, :])


def test_jstrips_cover_domain():
    from gt4py_amd.distributed import JStrips

    for n in (1, 7, 64, 2048):
        for w in (1, 2, 3, 8):
            if w > n:
                continue
            s = JStrips(n, w)
            b = [s.bounds(r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            assert max(s.size(r) for r in range(w)) - min(s.size(r) for r in range(w)) <= 1


# ---------------------------------------------------------------------------------------
# 2-D decomposition: corners, batching of several fields, periodic boundaries
# ---------------------------------------------------------------------------------------


def _worker2d(rank, world, port, outdir, pi, pj, periodic, ifirst=True, scheme="two_phase"):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import stencil_cases as sc
    from gt4py_amd import gtscript
    from gt4py_amd.distributed import Decomposition2D, HaloStencil2D

    dist.init_process_group("gloo", rank=rank, world_size=world)
    gin, gco = _global_inputs(periodic)
    h = 2
    nig, njg = gco.shape[:2]
    dec = Decomposition2D(nig, njg, pi, pj, periodic)
    (i0, i1), (j0, j1) = dec.bounds(rank)
    ni, nj = i1 - i0, j1 - j0
    lin = gin[i0 : i1 + 2 * h, j0 : j1 + 2 * h, :].copy()
    ci, cj = dec.coords(rank)
    # halo cells owned by another rank start as NaN: only the exchange may fill them
    if ci > 0 or periodic[0]:
        lin[:h] = np.nan
    if ci < pi - 1 or periodic[0]:
        lin[ni + h :] = np.nan
    if cj > 0 or periodic[1]:
        lin[:, :h] = np.nan
    if cj < pj - 1 or periodic[1]:
        lin[:, nj + h :] = np.nan
    t_in = torch.from_numpy(lin)
    t_in2 = torch.from_numpy(lin.copy() * 2.0)  # a second exchanged field (batched message)
    t_out = torch.zeros((ni, nj, gin.shape[2]), dtype=torch.float64)
    st = gtscript.stencil(backend="numpy", definition=sc.hdiff_f64, name="dist2d.hdiff")
    args = {"in_field": t_in, "out_field": t_out, "coeff": torch.from_numpy(gco[i0:i1, j0:j1, :].copy())}
    origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    runner = HaloStencil2D(st, ["in_field"], dec, rank, (h, h), ifirst=ifirst, scheme=scheme)
    runner(args, origin, (ni, nj, gin.shape[2]))
    runner.ex.exchange([t_in2])
    np.save(os.path.join(outdir, f"out_{rank}.npy"), t_out.numpy())
    np.save(os.path.join(outdir, f"in_{rank}.npy"), t_in.numpy())
    np.save(os.path.join(outdir, f"in2_{rank}.npy"), t_in2.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _global_inputs(periodic):
    rng = np.random.default_rng(5)
    nig, njg, nk, h = 13, 11, 3, 2
    core = rng.uniform(-10, 10, (nig + 2 * h, njg + 2 * h, nk))
    if periodic[0]:
        core[:h] = core[nig : nig + h]
        core[nig + h :] = core[h : 2 * h]
    if periodic[1]:
        core[:, :h] = core[:, njg : njg + h]
        core[:, njg + h :] = core[:, h : 2 * h]
    gco = rng.uniform(0, 0.5, (nig, njg, nk))
    return core, gco


@pytest.mark.parametrize(
    "pi,pj,periodic,ifirst,scheme",
    [(2, 2, (False, False), True, "two_phase"), (3, 2, (False, False), True, "two_phase"),
     (3, 2, (False, False), False, "two_phase"), (2, 2, (True, True), True, "two_phase"),
     (2, 2, (True, True), False, "two_phase"), (1, 2, (True, False), True, "two_phase"),
     (2, 1, (False, True), True, "two_phase"),
     (2, 2, (False, False), True, "diagonal"), (3, 2, (False, False), True, "diagonal"),
     (2, 2, (True, True), True, "diagonal"), (1, 2, (True, False), True, "diagonal"),
     (2, 1, (False, True), True, "diagonal"), (3, 3, (True, False), True, "diagonal")],
)
def test_2d_decomposition_matches_single_domain(tmp_path, pi, pj, periodic, ifirst, scheme):
    """``scheme``: two exchange phases (``ifirst``: I faces before a full-width interior, else
    west/east bands) or one phase with corner messages to the diagonal neighbours."""
    import torch.multiprocessing as mp

    sys.path.insert(0, REPO)
    import stencil_cases as sc
    from gt4py_amd import gtscript
    from gt4py_amd.distributed import Decomposition2D

    world = pi * pj
    port = _free_port()
    mp.spawn(_worker2d, args=(world, port, str(tmp_path), pi, pj, periodic, ifirst, scheme), nprocs=world, join=True)
    gin, gco = _global_inputs(periodic)
    h = 2
    nig, njg, nk = gco.shape
    ref = np.zeros((nig, njg, nk))
    st = gtscript.stencil(backend="numpy", definition=sc.hdiff_f64, name="dist2d.hdiff")
    st(gin.copy(), ref, gco, origin={"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)})
    dec = Decomposition2D(nig, njg, pi, pj, periodic)
    for r in range(world):
        (i0, i1), (j0, j1) = dec.bounds(r)
        assert np.array_equal(np.load(tmp_path / f"out_{r}.npy"), ref[i0:i1, j0:j1]), r
        # halos incl. corners hold the owning ranks' cells (periodic images included)
        assert np.array_equal(np.load(tmp_path / f"in_{r}.npy"), gin[i0 : i1 + 2 * h, j0 : j1 + 2 * h]), r
        assert np.array_equal(np.load(tmp_path / f"in2_{r}.npy"), 2.0 * gin[i0 : i1 + 2 * h, j0 : j1 + 2 * h]), r


def test_balanced_decomposition():
    from gt4py_amd.distributed import Decomposition2D

    d = Decomposition2D.balanced(8192, 8192, 8)
    assert (d.pi, d.pj) in ((2, 4), (4, 2))
    d = Decomposition2D.balanced(8192, 1024, 4)
    assert (d.pi, d.pj) == (4, 1)
    for r in range(d.size):
        assert d.rank_of(*d.coords(r)) == r


def _worker1d_periodic(rank, world, port, outdir):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import stencil_cases as sc
    from gt4py_amd import gtscript
    from gt4py_amd.distributed import HaloStencil, JStrips

    dist.init_process_group("gloo", rank=rank, world_size=world)
    gin, gco = _global_inputs((False, True))
    h = 2
    nig, njg, nk = gco.shape
    j0, j1 = JStrips(njg, world).bounds(rank)
    nj = j1 - j0
    lin = gin[:, j0 : j1 + 2 * h, :].copy()
    lin[:, :h] = np.nan  # every J halo is owned by a (periodic) neighbour
    lin[:, nj + h :] = np.nan
    t_in = torch.from_numpy(lin)
    t_out = torch.zeros((nig, nj, nk), dtype=torch.float64)
    st = gtscript.stencil(backend="numpy", definition=sc.hdiff_f64, name="dist1dp.hdiff")
    args = {"in_field": t_in, "out_field": t_out, "coeff": torch.from_numpy(gco[:, j0:j1, :].copy())}
    origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    HaloStencil(st, ["in_field"], nj, h, rank, world, periodic=True)(args, origin, (nig, nj, nk))
    np.save(os.path.join(outdir, f"out_{rank}.npy"), t_out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_jstrips_periodic(tmp_path, world):
    """Periodic J strips: two ranks are each other's prev and next (message order matters), one
    rank copies its own faces (gloo cannot send to itself; RCCL self-sends: scripts/rccl_halo_selftest.py)."""
    import torch.multiprocessing as mp

    sys.path.insert(0, REPO)
    import stencil_cases as sc
    from gt4py_amd import gtscript

    port = _free_port()
    mp.spawn(_worker1d_periodic, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    gin, gco = _global_inputs((False, True))
    h = 2
    ref = np.zeros(gco.shape)
    st = gtscript.stencil(backend="numpy", definition=sc.hdiff_f64, name="dist1dp.hdiff")
    st(gin.copy(), ref, gco, origin={"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)})
    got = np.concatenate([np.load(tmp_path / f"out_{r}.npy") for r in range(world)], axis=1)
    assert np.array_equal(got, ref)


def test_overlap_off_when_a_halo_field_is_written():
    """A stencil that writes one of its halo fields must not overlap the exchange (the packing of
    that field's edge rows would race with the interior kernel's writes): advisor finding r1."""
    sys.path.insert(0, REPO)
    from gt4py_amd import gtscript
    from gt4py_amd.distributed import Decomposition2D, HaloStencil, HaloStencil2D
    from gt4py_amd.gtscript import PARALLEL, Field, computation, interval

    def smooth(a: Field[np.float64], b: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            b = a[0, 1, 0] + a[0, -1, 0]

    st = gtscript.stencil(backend="numpy", definition=smooth, name="dist.readonly")
    # GTScript forbids reading a written field at IJ offsets, so a written halo field is one the
    # caller lists although the stencil only writes it ("b")
    assert HaloStencil(st, ["a"], 16, 1, 0, 2).overlap
    assert not HaloStencil(st, ["a", "b"], 16, 1, 0, 2).overlap
    dec = Decomposition2D(16, 16, 2, 1)
    assert HaloStencil2D(st, ["a"], dec, 0, (1, 1)).overlap
    assert not HaloStencil2D(st, ["b"], dec, 0, (1, 1)).overlap


def test_gated_strips_run_beside_the_interior_only_without_scratch():
    """GTMI_HALO_GATE: the boundary strips may skip waiting for the interior only when the two
    launches share no scratch temporaries (gt:mi355x plans say; other backends count as sharing)."""
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import stencil_cases as sc

    from gt4py_amd import gtscript
    from gt4py_amd.distributed.halo import _uses_scratch

    assert not _uses_scratch(gtscript.stencil(backend="gt:mi355x", definition=sc.hdiff_f64, name="dist.gate.hdiff"))
    assert _uses_scratch(gtscript.stencil(backend="gt:mi355x", definition=sc.staged_forward_ij_temp,
                                          name="dist.gate.staged", tile=0))
    assert _uses_scratch(gtscript.stencil(backend="numpy", definition=sc.hdiff_f64, name="dist.gate.np"))
