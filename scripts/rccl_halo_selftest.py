#!/usr/bin/env python3
"""One-GPU end-to-end check of the RCCL halo path: a 1x1 fully periodic 2-D decomposition whose
exchanges go through RCCL (self send/recv, ``force_comm``) on the halo stream while the interior
kernel runs; the result must equal hdiff on a wrap-padded single domain, bit for bit.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29542 scripts/rccl_halo_selftest.py
"""

import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import torch.distributed as dist

    import bench
    from gt4py_amd import gtscript, storage
    from gt4py_amd.distributed import Decomposition2D, HaloStencil2D, init_process_group

    rank, world = init_process_group("nccl")
    assert world == 1
    ni, nj, nk, h = 512, 384, 32, 2
    st = gtscript.stencil(backend="gt:mi355x", definition=bench.stencil_defs()[("horizontal_diffusion", np.float64)],
                          name="rccl_halo.hdiff", device_sync=False)
    rng = np.random.default_rng(9)
    core = rng.uniform(-10, 10, (ni, nj, nk))
    coeff_h = rng.uniform(0, 0.5, (ni, nj, nk))
    padded = np.pad(core, ((h, h), (h, h), (0, 0)), mode="wrap")
    # reference: the same kernel on the wrap-padded array
    fin_ref = storage.from_array(padded, backend="gt:mi355x", aligned_index=(h, h, 0))
    coeff = storage.from_array(coeff_h, backend="gt:mi355x")
    out_ref = storage.zeros((ni, nj, nk), np.float64, backend="gt:mi355x")
    origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    st(fin_ref, out_ref, coeff, origin=origin, domain=(ni, nj, nk))
    # distributed path: halos start as NaN, RCCL fills them (incl. corners) while the interior runs
    nanpad = padded.copy()
    nanpad[:h] = np.nan
    nanpad[-h:] = np.nan
    nanpad[:, :h] = np.nan
    nanpad[:, -h:] = np.nan
    fin = storage.from_array(nanpad, backend="gt:mi355x", aligned_index=(h, h, 0))
    out = storage.zeros((ni, nj, nk), np.float64, backend="gt:mi355x")
    dec = Decomposition2D(ni, nj, 1, 1, (True, True))
    run = HaloStencil2D(st, ["in_field"], dec, 0, (h, h), force_comm=True)
    ok = True
    for it in range(3):
        run({"in_field": fin, "out_field": out, "coeff": coeff}, origin, (ni, nj, nk))
        torch.cuda.synchronize()
        ok = ok and np.array_equal(storage.to_numpy(out), storage.to_numpy(out_ref))
        ok = ok and np.array_equal(storage.to_numpy(fin), padded)
    # 1-D J strips, periodic, one rank: the bench's default N>1 path through RCCL (force_comm)
    from gt4py_amd.distributed import HaloStencil

    jpad = np.pad(core, ((h, h), (h, h), (0, 0)), mode="wrap")
    jpad[:, :h] = np.nan
    jpad[:, -h:] = np.nan
    fin1 = storage.from_array(jpad, backend="gt:mi355x", aligned_index=(h, h, 0))
    out1 = storage.zeros((ni, nj, nk), np.float64, backend="gt:mi355x")
    run1 = HaloStencil(st, ["in_field"], nj, h, 0, 1, periodic=True, force_comm=True)
    ok1 = True
    for it in range(3):
        run1({"in_field": fin1, "out_field": out1, "coeff": coeff}, origin, (ni, nj, nk))
        torch.cuda.synchronize()
        ok1 = ok1 and np.array_equal(storage.to_numpy(out1), storage.to_numpy(out_ref))
    dist.barrier()
    print(json.dumps({"rccl_halo_2d_periodic_selfcomm": bool(ok), "rccl_halo_jstrips_periodic_selfcomm": bool(ok1)}),
          flush=True)
    ok = ok and ok1
    dist.destroy_process_group()
    if not ok:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
