#!/usr/bin/env python3
"""Interleaved A/B timing of gt:mi355x codegen variants in ONE process (cdna guide §5.4 rule 24).

    python scripts/sweep.py --config hdiff --variants "vector=1,prefetch=1;vector=2,prefetch=2"
    python scripts/sweep.py --config hdiff --variants "..." --build-only   # prebuild on CPU

Every variant's output is checked bit-for-bit against the first variant's output.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def parse_variants(text):
    out = []
    for part in text.split(";"):
        part = part.strip()
        if not part:
            continue
        d = {}
        for kv in part.split(","):
            k, v = kv.split("=")
            d[k.strip()] = int(v) if v.strip().lstrip("-").isdigit() else v.strip()
        out.append(d)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="hdiff")
    ap.add_argument("--variants", required=True)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    import bench
    from gt4py_amd import gtscript

    sname, dtype, (ni, nj, nk), h, bpc = bench.CONFIGS[args.config]
    defn = bench.stencil_defs()[(sname, dtype)]
    variants = parse_variants(args.variants)
    stencils = []
    for i, v in enumerate(variants):
        stencils.append(
            gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"sweep.{args.config}.{i}", device_sync=False,
                             externals=bench.EXTERNALS.get(sname, {}), **v)
        )
    if args.build_only:
        print(f"built {len(stencils)} variants")
        return
    import torch

    from gt4py_amd import storage

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    tdt = storage.torch_dtype(dtype)

    def uniform(shape, lo, hi, aligned):
        t = storage.empty(shape, dtype, backend="gt:mi355x", aligned_index=aligned)
        t.copy_(torch.rand(shape, generator=gen, device=dev, dtype=tdt) * (hi - lo) + lo)
        return t

    params = {}
    if sname in ("horizontal_diffusion", "lap5"):
        fin = uniform((ni + 2 * h, nj + 2 * h, nk), -10, 10, (h, h, 0))
        shared = storage.zeros((ni, nj, nk), dtype, backend="gt:mi355x")
        outs = [shared for _ in variants]  # one buffer: HBM placement is identical for every variant
        if sname == "horizontal_diffusion":
            coeff = uniform((ni, nj, nk), 0, 0.5, (0, 0, 0))
            argsets = [(fin, o, coeff) for o in outs]
            origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
        else:
            argsets = [(fin, o) for o in outs]
            origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0)}
        check = [o for o in outs]
    elif sname == "tridiagonal_solver":
        # ONE set of buffers for every variant (HBM placement moves column-kernel times by +-8 %);
        # sup/rhs are solved in place, so they are restored before each variant's checked call
        base = [uniform((ni, nj, nk), lo, hi, (0, 0, 0)) for lo, hi in ((-1, 1), (4, 5), (-1, 1), (-10, 10), (0, 0))]
        saved = [base[2].clone(), base[3].clone()]

        def restore():
            base[2].copy_(saved[0])
            base[3].copy_(saved[1])
            base[4].zero_()

        argsets = [tuple(base) for _ in variants]
        check = [base[4] for _ in variants]
        origin = (0, 0, 0)
    elif sname == "vertical_advection_dycore":
        ins = [uniform((ni, nj, nk), -1, 1, (0, 0, 0)) for _ in range(3)]
        wcon = uniform((ni + 1, nj, nk + 1), -1, 1, (0, 0, 0))
        ust = storage.zeros((ni, nj, nk), dtype, backend="gt:mi355x")
        argsets = [(ust, ins[0], wcon, ins[1], ins[2]) for _ in variants]
        check = [ust for _ in variants]
        params = {"dtr_stage": 3.0 / 20.0}
        origin = (0, 0, 0)
    elif sname == "staged_forward_ij_temp":
        a = uniform((ni + 2 * h, nj + 2 * h, nk), -1, 1, (h, h, 0))
        shared = storage.zeros((ni, nj, nk), dtype, backend="gt:mi355x")
        argsets = [(a, shared) for _ in variants]
        check = [shared for _ in variants]
        origin = {"a": (h, h, 0), "out": (0, 0, 0)}
    else:
        a = uniform((ni, nj, nk), -10, 10, (0, 0, 0))
        shared = storage.zeros((ni, nj, nk), dtype, backend="gt:mi355x")
        outs = [shared for _ in variants]
        argsets = [(a, o) for o in outs]
        check = outs
        origin = (0, 0, 0)
    dom = (ni, nj, nk)
    ref = None
    for i, (st, a) in enumerate(zip(stencils, argsets)):
        if sname == "tridiagonal_solver":
            restore()
        elif sname == "vertical_advection_dycore":
            check[i].zero_()  # utens_stage is read and written: identical input for every variant
        st(*a, **params, origin=origin, domain=dom)
        torch.cuda.synchronize()
        if ref is None:  # first call of every variant runs on identical inputs
            ref = check[i].clone()
        elif not torch.equal(check[i], ref):
            print(f"variant {i} {variants[i]} MISMATCH: {int((check[i] != ref).sum())} cells")
    times = [[] for _ in variants]
    for r in range(args.rounds):
        for i, (st, a) in enumerate(zip(stencils, argsets)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                st(*a, **params, origin=origin, domain=dom, validate_args=False)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / args.reps)
    res = []
    for v, t in zip(variants, times):
        med = float(np.median(t))
        gbs = ni * nj * nk * bpc / (med * 1e-3) / 1e9
        res.append({"variant": v, "median_ms": round(med, 4), "min_ms": round(min(t), 4), "GBps": round(gbs, 1),
                    "frac": round(gbs / 8000, 4)})
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
