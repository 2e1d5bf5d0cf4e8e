#!/usr/bin/env python3
"""Kernel time against the J extent of the domain, on fixed buffers: is a kernel paced by bytes
(time grows with nj in proportion) or by rounds of resident workgroups (time grows in steps of
one round of the machine's block slots)?

    python scripts/staircase.py --config staged --variants "tile_by=8;tile_by=16" --nj 64,128,...

One line per (variant, nj): median ms of --reps launches, blocks in the grid, and ms per Mcell.
"""

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from sweep import parse_variants  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="staged")
    ap.add_argument("--variants", default="tile_by=8")
    ap.add_argument("--nj", default="")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    import bench
    from gt4py_amd import gtscript

    sname, dtype, (ni, nj, nk), h, bpc = bench.CONFIGS[args.config]
    if sname != "staged_forward_ij_temp":
        raise SystemExit("staircase.py: only the staged config is wired")
    defn = bench.stencil_defs()[(sname, dtype)]
    variants = parse_variants(args.variants)
    stencils = [gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"stair.{args.config}.{i}",
                                 device_sync=False, **v) for i, v in enumerate(variants)]
    if args.build_only:
        print(f"built {len(stencils)} variants")
        return
    import torch

    from gt4py_amd import storage

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    a = storage.empty((ni + 2 * h, nj + 2 * h, nk), dtype, backend="gt:mi355x", aligned_index=(h, h, 0))
    a.copy_(torch.rand(a.shape, generator=gen, device=dev, dtype=storage.torch_dtype(dtype)) * 2 - 1)
    out = storage.zeros((ni, nj, nk), dtype, backend="gt:mi355x")
    origin = {"a": (h, h, 0), "out": (0, 0, 0)}
    njs = [int(x) for x in args.nj.split(",")] if args.nj else [nj * f // 16 for f in range(1, 17)]
    for v, st in zip(variants, stencils):
        by = int(v.get("tile_by", 8))
        for n in njs:
            dom = (ni, n, nk)
            for _ in range(3):
                st(a, out, origin=origin, domain=dom, validate_args=False)
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    st(a, out, origin=origin, domain=dom, validate_args=False)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / args.reps)
            ms = float(np.median(ts))
            # tile geometry of the staged stencil: I extent +-1, J extent 0..+1
            blocks = -(-ni // 62) * -(-n // (by - 1))
            print(json.dumps({"variant": v, "nj": n, "ms": round(ms, 4), "blocks": blocks,
                              "ms_per_Mcell": round(ms / (ni * n * nk / 1e6), 5)}), flush=True)


if __name__ == "__main__":
    main()
