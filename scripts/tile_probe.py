#!/usr/bin/env python3
"""Tile-kernel geometry probe: every tile program of tests/stencil_cases.py (TILE_PROGRAMS) at a
large domain, codegen variants timed interleaved in ONE process on shared buffers, each variant's
output checked bit-for-bit against the first variant's.

    python scripts/tile_probe.py --variants "tile_by=8;tile_by=16" [--domain 1024,1024,80]
    python scripts/tile_probe.py --variants "..." --build-only     # prebuild on CPU

Prints one JSON line per (program, variant): median kernel time and Mcells/s.
"""

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def parse_variants(text):
    out = []
    for part in filter(None, (p.strip() for p in text.split(";"))):
        d = {}
        for kv in part.split(","):
            k, v = kv.split("=")
            d[k.strip()] = int(v) if v.strip().lstrip("-").isdigit() else v.strip()
        out.append(d)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True)
    ap.add_argument("--programs", default="")
    ap.add_argument("--domain", default="1024,1024,80")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    import stencil_cases as sc

    from gt4py_amd import gtscript

    variants = parse_variants(args.variants)
    progs = [p for p in sc.TILE_PROGRAMS if not args.programs or p in args.programs.split(",")]
    built = {p: [gtscript.stencil(backend="gt:mi355x", definition=sc.TILE_PROGRAMS[p][0], name=f"tile_probe.{p}",
                                  device_sync=False, **v) for v in variants] for p in progs}
    if args.build_only:
        print(f"built {len(progs)} x {len(variants)} variants")
        return
    import torch

    from gt4py_amd import storage

    ni, nj, nk = (int(x) for x in args.domain.split(","))
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    for p in progs:
        defn, halos, dt = sc.TILE_PROGRAMS[p]
        dtype = np.dtype(dt).type
        tdt = storage.torch_dtype(dtype)
        arrays, origin = {}, {}
        for f, (ilo, ihi, jlo, jhi) in halos.items():
            t = storage.empty((ni + ilo + ihi, nj + jlo + jhi, nk), dtype, backend="gt:mi355x", aligned_index=(ilo, jlo, 0))
            t.copy_(torch.rand(t.shape, generator=gen, device=dev, dtype=tdt) * 1.5 + 0.5)
            arrays[f], origin[f] = t, (ilo, jlo, 0)
        arrays["out"] = storage.zeros((ni, nj, nk), dtype, backend="gt:mi355x")
        origin["out"] = (0, 0, 0)
        ref = None
        for i, st in enumerate(built[p]):
            arrays["out"].zero_()
            st(**arrays, origin=origin, domain=(ni, nj, nk))
            torch.cuda.synchronize()
            if ref is None:
                ref = arrays["out"].clone()
            elif not torch.equal(arrays["out"], ref):
                print(f"{p} variant {i} {variants[i]} MISMATCH: {int((arrays['out'] != ref).sum())} cells", flush=True)
        times = [[] for _ in variants]
        for _ in range(args.rounds):
            for i, st in enumerate(built[p]):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    st(**arrays, origin=origin, domain=(ni, nj, nk), validate_args=False)
                e1.record()
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) / args.reps)
        for v, t in zip(variants, times):
            med = float(np.median(t))
            print(json.dumps({"program": p, "dtype": np.dtype(dtype).name, "variant": v, "median_ms": round(med, 4),
                              "Mcells_s": round(ni * nj * nk / (med * 1e-3) / 1e6, 1)}), flush=True)
        del arrays
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
