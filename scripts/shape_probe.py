#!/usr/bin/env python3
"""Launch-size probe: lap5 and copy at K = 80 and K = 160, one process,
interleaved rounds, HIP events on the launch stream, every config on its own fields.

    python scripts/shape_probe.py [--configs lap5,lap5_k160,copy_k80,copy] [--rounds 7 --reps 20]

If lap5 at 1024^2x160 (same cell count as the copy config) reaches copy's fraction of the HBM
roofline, lap5's gap at K = 80 is the launch's fixed ramp/tail, not the kernel. Prints one JSON
line per config with the median kernel time, the fixed cost implied by the two K sizes
(t80 - (t160 - t80)), and the fraction of 8 TB/s.
"""

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="lap5,lap5_k160,copy_k80,copy")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch

    import bench
    from gt4py_amd import gtscript, storage

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    runs = []
    for cfg in args.configs.split(","):
        sname, dtype, (ni, nj, nk), h, bpc = bench.CONFIGS[cfg]
        assert sname in ("lap5", "copy_stencil"), cfg
        st = gtscript.stencil(backend="gt:mi355x", definition=bench.stencil_defs()[(sname, dtype)],
                              name=f"bench.{cfg}", device_sync=False)
        tdt = storage.torch_dtype(dtype)
        fin = storage.empty((ni + 2 * h, nj + 2 * h, nk), dtype, backend="gt:mi355x", aligned_index=(h, h, 0))
        fin.copy_(torch.rand(fin.shape, generator=gen, device=dev, dtype=tdt) * 20 - 10)
        out = storage.zeros((ni, nj, nk), dtype, backend="gt:mi355x")
        if sname == "lap5":
            origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0)}
        else:
            origin = (0, 0, 0)
        st(fin, out, origin=origin, domain=(ni, nj, nk))
        runs.append((cfg, st, (fin, out), origin, (ni, nj, nk), bpc))
    torch.cuda.synchronize()
    times = {r[0]: [] for r in runs}
    for _ in range(args.rounds):
        for cfg, st, a, origin, dom, _bpc in runs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                st(*a, origin=origin, domain=dom, validate_args=False)
            e1.record()
            torch.cuda.synchronize()
            times[cfg].append(e0.elapsed_time(e1) / args.reps)
    med = {c: float(np.median(t)) for c, t in times.items()}
    for cfg, _st, _a, _o, (ni, nj, nk), bpc in runs:
        gbs = ni * nj * nk * bpc / (med[cfg] * 1e-3) / 1e9
        line = {"config": cfg, "domain": [ni, nj, nk], "median_ms": round(med[cfg], 5),
                "min_ms": round(min(times[cfg]), 5), "GBps": round(gbs, 1), "frac": round(gbs / 8000, 4)}
        twin = {"lap5": "lap5_k160", "copy_k80": "copy"}.get(cfg)
        if twin in med:  # linear model t(K) = fixed + K * per_level from the two K sizes
            line["fixed_ms"] = round(2 * med[cfg] - med[twin], 5)
            line["frac_without_fixed"] = round(ni * nj * nk * bpc / ((med[twin] - med[cfg]) * 1e-3) / 1e9 / 8000, 4)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
