#!/usr/bin/env python3
"""HBM channel aliasing between a stencil's streams: the same three hdiff buffers, viewed at
different byte offsets inside one over-allocated raw buffer each, so that only the residues of
the field base addresses modulo 8 MiB change (the physical pages stay the same).

    python scripts/placement_residue.py [--config hdiff|tridiag] [--rounds 5]

Prints one JSON line per residue tuple (median kernel ms over interleaved rounds).
"""

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

MIB = 1 << 20
WINDOW = 8 * MIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="hdiff")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--kpad", default="", help="comma list of K-stride paddings in bytes (sweeps them instead of residues)")
    ap.add_argument("--ipad", default="", help="comma list of extra I-pitch elements (sweeps them instead of residues)")
    args = ap.parse_args()
    import torch

    import bench
    from gt4py_amd import gtscript

    sname, dtype, (ni, nj, nk), h, bpc = bench.CONFIGS[args.config]
    st = gtscript.stencil(backend="gt:mi355x", definition=bench.stencil_defs()[(sname, dtype)], name=f"bench.{args.config}",
                          externals=bench.EXTERNALS.get(sname, {}), device_sync=False)
    isz = np.dtype(dtype).itemsize
    if sname == "horizontal_diffusion":
        shapes = [(ni + 2 * h, nj + 2 * h, nk), (ni, nj, nk), (ni, nj, nk)]
        names = ["in_field", "out_field", "coeff"]
        origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
        aligned = [(h, h, 0), (0, 0, 0), (0, 0, 0)]
    elif sname == "lap5":
        shapes = [(ni + 2 * h, nj + 2 * h, nk), (ni, nj, nk)]
        names = ["in_field", "out_field"]
        origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0)}
        aligned = [(h, h, 0), (0, 0, 0)]
    elif sname == "copy_stencil":
        shapes = [(ni, nj, nk)] * 2
        names = ["field_a", "field_b"]
        origin = (0, 0, 0)
        aligned = [(0, 0, 0)] * 2
    else:
        shapes = [(ni, nj, nk)] * 5
        names = ["inf", "diag", "sup", "rhs", "out"]
        origin = (0, 0, 0)
        aligned = [(0, 0, 0)] * 5
    kpads = [int(x) for x in args.kpad.split(",") if x] or [0]
    ipads = [int(x) for x in args.ipad.split(",") if x] or [0]
    maxpad = max(kpads)
    raws, geo = [], []
    for shp in shapes:
        pi = -(-shp[0] // 32) * 32
        strides = (1, pi, pi * shp[1])
        nbytes = ((pi + max(ipads)) * shp[1] * isz + maxpad) * shp[2]
        raws.append(torch.empty(nbytes + 2 * WINDOW, dtype=torch.uint8, device="cuda"))
        geo.append((shp, strides))
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)

    def views(residues, kpad=0, ipad=0):
        out = []
        for (shp, strides), raw, al, res in zip(geo, raws, aligned, residues):
            pitch = strides[1] + ipad
            strides = (strides[0], pitch, pitch * shp[1] + kpad // isz)
            base = raw.data_ptr()
            lead = (al[0] * strides[0] + al[1] * strides[1]) * isz  # the aligned element's byte offset
            off = (res - (base + lead)) % WINDOW
            flat = raw[off:off + (strides[2] * shp[2]) * isz].view(torch.float64 if isz == 8 else torch.float32)
            out.append(torch.as_strided(flat, shp, strides))
        return out

    r = int(MIB)
    tuples = [
        (0, 0, 0), (0, 1 * r, 2 * r), (0, 1 * r, 3 * r), (0, 2 * r, 4 * r), (0, 3 * r, 6 * r), (0, r // 4, r // 2),
        (0, r // 2, r), (0, 3 * r // 2, 3 * r), (0, 5 * r, 2 * r), (0, 0, 0),
    ]
    if len(shapes) == 5:
        tuples = [t + (t[1] + t[2], 2 * t[2]) for t in tuples]
    tuples = [t[:len(shapes)] for t in tuples]
    cases = [(t, 0, 0) for t in tuples]
    odd = tuple((q % 2) * r for q in range(len(shapes)))
    if args.kpad:
        same = tuple(0 for _ in shapes)
        cases = [(res, kp, 0) for kp in kpads for res in (same, odd)]
    if args.ipad:
        cases = [(odd, 0, ip) for ip in ipads] + [(odd, 0, ipads[0])]
    tuples = [c[0] for c in cases]
    sets = []
    for t, kp, ip in cases:
        v = views(t, kp, ip)
        for x in v:
            x.copy_(torch.rand(x.shape, generator=gen, device="cuda", dtype=x.dtype))
        sets.append(v)
    dom = (ni, nj, nk)
    times = [[] for _ in tuples]
    for _ in range(args.rounds):
        for i, v in enumerate(sets):
            kw = dict(zip(names, v))
            st(**kw, origin=origin, domain=dom)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                st(**kw, origin=origin, domain=dom, validate_args=False)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / args.reps)
    for (t, kp, ip), ts in zip(cases, times):
        med = float(np.median(ts))
        print(json.dumps({"config": args.config, "kpad_bytes": kp, "ipad": ip, "residues_MiB": [round(x / MIB, 3) for x in t],
                          "median_ms": round(med, 4),
                          "frac": round(ni * nj * nk * bpc / (med * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
