"""The sharded HIP path on one MI355X through RCCL, checked against the C oracle.

A world-size-1 NCCL (= RCCL) process group is created in-process (TCP store on 127.0.0.1, no
torchrun). With ``periodic`` + ``force_comm`` the rank is its own neighbour, so every halo
face goes pack kernel -> RCCL send/recv -> unpack kernel while the interior kernel runs (both
stream orderings: everything on the caller's stream with RCCL on its own, the default; or a
dedicated halo stream) -- the same code the N-GPU bench runs
(``distributed/halo.py`` HaloStencil, ``distributed/decomp2d.py`` HaloStencil2D).
Halos start as NaN; only a correct exchange fills them. Each of 3 iterations feeds the result
back as the next input, and must equal the C oracle's hdiff on the wrap-padded input bit for bit.
"""

import os
import socket

import numpy as np
import pytest

import golden_utils as gu

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def rccl_group():
    import torch
    import torch.distributed as dist

    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    os.environ.setdefault("NCCL_DEBUG", "WARN")
    torch.cuda.set_device(0)
    from gt4py_amd.distributed.halo import rccl_options

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0), pg_options=rccl_options())
    yield dist
    dist.destroy_process_group()


def _hdiff_stencil():
    import stencil_cases as sc
    from gt4py_amd import gtscript

    return gtscript.stencil(backend="gt:mi355x", definition=sc.hdiff_f64, name="gpu.halo.hdiff", device_sync=False)


def _oracle_hdiff(core, coeff, h, wrap_i):
    """One hdiff step of the periodic problem: J always wraps; I wraps when ``wrap_i``, else the
    I halo keeps the fixed boundary values of ``core``'s padded copy."""
    from oracle import c_oracle

    ni, nj, nk = core.shape
    pad_i = (h, h)
    padded = np.pad(core, (pad_i, (h, h), (0, 0)), mode="wrap")
    if not wrap_i:
        padded[:h] = 7.0  # fixed global I boundary (global boundaries are plain input cells)
        padded[-h:] = -3.0
    out = np.zeros((ni, nj, nk), order="F")
    org = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    c_oracle.horizontal_diffusion(np.asfortranarray(padded), out, np.asfortranarray(coeff), org, (ni, nj, nk))
    return out, padded


@pytest.mark.parametrize("stream_mode", ["main", "main_bands", "side", "side_bands_main", "side_unpack_main", "side_split3",
                                         "diag", "side_gate", "side_gate_unpack_main"])
@pytest.mark.parametrize("mode", ["jstrips", "tiles2d", "tiles2d_jperiodic"])
def test_rccl_halo_hdiff_vs_c_oracle(rccl_group, mode, stream_mode):
    import torch

    from gt4py_amd import storage
    from gt4py_amd.distributed import Decomposition2D, HaloStencil, HaloStencil2D

    ni, nj, nk, h = 384, 256, 24, 2
    st = _hdiff_stencil()
    rng = np.random.default_rng(21)
    core = rng.uniform(-10, 10, (ni, nj, nk))
    coeff_h = rng.uniform(0, 0.5, (ni, nj, nk))
    coeff = storage.from_array(coeff_h, backend="gt:mi355x")
    out = storage.zeros((ni, nj, nk), np.float64, backend="gt:mi355x")
    wrap_i = mode == "tiles2d"
    origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    if "gate" in stream_mode and mode != "jstrips":
        pytest.skip("the gated interior (GTMI_HALO_GATE) is a J-strip option")
    if mode == "jstrips":
        if stream_mode == "diag":
            pytest.skip("the diagonal (one-phase) scheme is a 2-D tile exchange")
        run = HaloStencil(st, ["in_field"], nj, h, 0, 1, periodic=True, force_comm=True)
        wrap_i = False
    else:
        dec = Decomposition2D(ni, nj, 1, 1, (wrap_i, True))
        run = HaloStencil2D(st, ["in_field"], dec, 0, (h, h), force_comm=True,
                            scheme="diagonal" if stream_mode == "diag" else "two_phase")
    run.stream_mode = {"diag": "main"}.get(stream_mode, stream_mode.split("_")[0])
    if hasattr(run, "gate"):
        run.gate = "gate" in stream_mode  # interior waits for the pack; strips beside the interior
    if hasattr(run, "bands_on_halo"):
        run.bands_on_halo = not stream_mode.endswith("bands_main")
        run.split = 3 if stream_mode.endswith("split3") else 1
        run.unpack_on_main = stream_mode.endswith("unpack_main")
    if hasattr(run, "ifirst"):  # 2-D: "*bands*" modes run the west/east band variant
        run.ifirst = not (stream_mode.endswith("bands_main") or stream_mode == "main_bands")
    assert run.overlap, "the interior/exchange overlap path must be the one under test"
    for it in range(3):
        ref, padded = _oracle_hdiff(core, coeff_h, h, wrap_i)
        start = padded.copy()
        start[:, :h] = np.nan  # J halos: filled by the exchange only
        start[:, -h:] = np.nan
        if wrap_i:
            start[:h] = np.nan
            start[-h:] = np.nan
        fin = storage.from_array(start, backend="gt:mi355x", aligned_index=(h, h, 0))
        run({"in_field": fin, "out_field": out, "coeff": coeff}, origin, (ni, nj, nk))
        torch.cuda.synchronize()
        gu.assert_match(storage.to_numpy(out), ref, name=f"halo_{mode}_{stream_mode}_it{it}")
        np.testing.assert_array_equal(storage.to_numpy(fin), padded)  # halos hold the neighbours' rows
        core = ref
