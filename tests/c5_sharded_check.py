#!/usr/bin/env python3
"""C5 through the sharded path, checked cell by cell: hdiff f32 as J strips of an
NI x (NJ * world) x NK global domain over ``world`` ranks (BASELINE configs[4]: 8192 x 8192 x 160
at 8 ranks of 8192 x 1024 x 160), the J halos exchanged by ``gt4py_amd.distributed.HaloStencil``.

Test infrastructure (tests/): every rank compares its output strip bit-for-bit with the C oracle
(oracle/cpu_stencils.c) on the same global input, and the halo rows the exchange delivered with
the rows its neighbours own. The global input is a deterministic function of the global (i, j, k)
-- the demo analytic field of SURVEY §8(d) C3 plus a K term, and a hashed coefficient -- so each rank
builds its own strip (halos included) without any rank holding the global field.

Launch one process per rank (ranks may share one GPU: RCCL refuses two ranks on a device, so
GTMI_DIST_BACKEND=gloo then moves the halos through host memory)::

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29561 tests/c5_sharded_check.py --ni 8192 --nj 1024 --nk 160

Rank 0 prints one JSON line: the global domain, the transport, mismatches (0 = bit-exact),
and the halo step's time (ranks sharing one GPU: a functional run, not a scaling figure).
"""

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)


def global_in(ni, nj_glob, gi0, gi1, gj0, gj1, k0, k1):
    """in_field over global columns [gi0, gi1) x rows [gj0, gj1) x levels [k0, k1), f32, I-first:
    5 + 8 (2 + cos(pi (x + 1.5 y)) + sin(2 pi (x + 1.5 y))) / 4 + 0.001 k, x = i / NI, y = j / NJ."""
    x = np.arange(gi0, gi1, dtype=np.float64)[:, None] / ni
    y = np.arange(gj0, gj1, dtype=np.float64)[None, :] / nj_glob
    t = x + 1.5 * y
    plane = 5.0 + 8.0 * (2.0 + np.cos(np.pi * t) + np.sin(2.0 * np.pi * t)) / 4.0
    ks = np.arange(k0, k1, dtype=np.float64)[None, None, :] * 1e-3
    return np.asfortranarray((plane[:, :, None] + ks).astype(np.float32))


def global_coeff(gi0, gi1, gj0, gj1, k0, k1):
    """coeff in [0.025, 0.125): a hash of the global position (not smooth, so the limiter's
    branches mix)."""
    i = np.arange(gi0, gi1, dtype=np.float64)[:, None, None]
    j = np.arange(gj0, gj1, dtype=np.float64)[None, :, None]
    k = np.arange(k0, k1, dtype=np.float64)[None, None, :]
    h = np.sin(12.9898 * i + 78.233 * j + 0.37 * k) * 43758.5453
    return np.asfortranarray((0.025 + 0.1 * (h - np.floor(h))).astype(np.float32))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ni", type=int, default=8192)
    ap.add_argument("--nj", type=int, default=1024, help="rows per rank")
    ap.add_argument("--nk", type=int, default=160)
    ap.add_argument("--kchunk", type=int, default=16, help="levels per host chunk (bounds host memory)")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from gt4py_amd import gtscript, storage
    from gt4py_amd.distributed import HaloStencil, init_process_group
    from oracle import c_oracle

    sys.path.insert(0, HERE)
    import stencil_cases as sc

    rank, world = init_process_group()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    ni, nj, nk, h = args.ni, args.nj, args.nk, 2
    nj_glob = nj * world
    j0 = rank * nj  # this rank's first global row
    st = gtscript.stencil(backend="gt:mi355x", definition=sc.hdiff_f32, name="c5.sharded.hdiff_f32",
                          device_sync=False)
    fin = storage.empty((ni + 2 * h, nj + 2 * h, nk), np.float32, backend="gt:mi355x", aligned_index=(h, h, 0))
    coeff = storage.empty((ni, nj, nk), np.float32, backend="gt:mi355x")
    out = storage.zeros((ni, nj, nk), np.float32, backend="gt:mi355x")
    kc = args.kchunk

    def progress(msg):
        if rank == 0:
            print(f"[c5 check] {msg} ({time.time() - t_start:.0f} s)", file=sys.stderr, flush=True)

    t_start = time.time()
    for k0 in range(0, nk, kc):
        k1 = min(nk, k0 + kc)
        progress(f"fill levels {k0}-{k1 - 1}")
        a = global_in(ni, nj_glob, -h, ni + h, j0 - h, j0 + nj + h, k0, k1)
        if rank > 0:
            a[:, :h, :] = np.nan  # filled by the exchange only
        if rank < world - 1:
            a[:, -h:, :] = np.nan
        fin[:, :, k0:k1].copy_(torch.from_numpy(np.ascontiguousarray(a)))
        coeff[:, :, k0:k1].copy_(torch.from_numpy(np.ascontiguousarray(global_coeff(0, ni, j0, j0 + nj, k0, k1))))
    run = HaloStencil(st, ["in_field"], nj, h, rank, world)
    assert run.overlap
    origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    fields = {"in_field": fin, "out_field": out, "coeff": coeff}
    run(fields, origin, (ni, nj, nk))
    torch.cuda.synchronize()
    # check: the oracle on this rank's strip of the global input, chunk by chunk
    bad_out = bad_halo = 0
    threads = max(1, int(os.environ.get("OMP_NUM_THREADS", "16")) // world)
    for k0 in range(0, nk, kc):
        k1 = min(nk, k0 + kc)
        progress(f"check levels {k0}-{k1 - 1}")
        a = global_in(ni, nj_glob, -h, ni + h, j0 - h, j0 + nj + h, k0, k1)
        c = global_coeff(0, ni, j0, j0 + nj, k0, k1)
        ref = np.zeros((ni, nj, k1 - k0), dtype=np.float32, order="F")
        c_oracle.horizontal_diffusion(a, ref, c, origin, (ni, nj, k1 - k0), nthreads=threads)
        got = out[:, :, k0:k1].cpu().numpy()
        bad_out += int((got != ref).sum())
        halo = fin[:, :, k0:k1].cpu().numpy()
        bad_halo += int((halo != a).sum())  # exchanged rows = the neighbours' own rows (no NaN left)
        del a, c, ref, got, halo
    # the halo step's time (ranks sharing one GPU and a host-staged transport: functional only)
    for _ in range(2):
        run(fields, origin, (ni, nj, nk))
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run(fields, origin, (ni, nj, nk))
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    res = torch.tensor([bad_out, bad_halo, el], dtype=torch.float64)
    dist.all_reduce(res[:2], op=dist.ReduceOp.SUM)
    mx = torch.tensor([el], dtype=torch.float64)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({
            "check": "hdiff f32 J strips vs the C oracle on the global input",
            "world_size": world,
            "global_domain": [ni, nj_glob, nk],
            "domain_per_rank": [ni, nj, nk],
            "transport": str(dist.get_backend()),
            "devices": torch.cuda.device_count(),
            "halo_schedule": run.schedule(),
            "mismatched_cells": int(res[0]),
            "mismatched_halo_cells": int(res[1]),
            "cells_checked": ni * nj_glob * nk,
            "ms_per_step": round(float(mx[0]) / args.steps * 1e3, 3),
            "note": "ranks share the box's GPUs; the time is not a scaling figure",
        }), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if int(res[0]) == 0 and int(res[1]) == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
