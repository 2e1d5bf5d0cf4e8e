#!/usr/bin/env python3
"""Does HBM placement (row pitch / plane pitch / buffer identity) change the hdiff kernel time?

One kernel variant, several allocations of the three fields; interleaved rounds in one process.
"""

import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch

    import bench
    from gt4py_amd import gtscript

    opts = dict(prefetch=4, jchunk=32, strip_align=16)
    if len(sys.argv) > 1:
        opts = json.loads(sys.argv[1])
    ni, nj, nk = 2048, 2048, 160
    optsets = opts if isinstance(opts, list) else [opts]
    sts = [gtscript.stencil(backend="gt:mi355x", definition=bench.stencil_defs()[("horizontal_diffusion", np.float64)],
                            name=f"placement.hdiff{i}", device_sync=False, **o) for i, o in enumerate(optsets)]
    if len(sys.argv) > 4:
        print("built"); return
    dev = torch.device("cuda", 0)

    g = torch.Generator(device=dev)
    g.manual_seed(3)
    base_in = torch.rand((ni + 4, nj + 4, nk), generator=g, device=dev, dtype=torch.float64) * 20 - 10
    base_co = torch.rand((ni, nj, nk), generator=g, device=dev, dtype=torch.float64) * 0.5
    pi_in, pi = -(-(ni + 4) // 32) * 32, ni
    n_in, n_f = pi_in * (nj + 4) * nk, pi * nj * nk
    MiB = 1 << 20

    def carve(gap_co, gap_out):
        """in, coeff, out carved from ONE allocation with byte gaps between them."""
        g_co, g_out = gap_co // 8, gap_out // 8
        total = n_in + g_co + n_f + g_out + n_f + 64
        buf = torch.empty(total, dtype=torch.float64, device=dev)
        o_in, o_co = 0, n_in + g_co
        o_out = o_co + n_f + g_out
        fin = torch.as_strided(buf, (ni + 4, nj + 4, nk), (1, pi_in, pi_in * (nj + 4)), o_in)
        co = torch.as_strided(buf, (ni, nj, nk), (1, pi, pi * nj), o_co)
        out = torch.as_strided(buf, (ni, nj, nk), (1, pi, pi * nj), o_out)
        fin.copy_(base_in)
        co.copy_(base_co)
        return fin, out, co

    gaps = [0, 256, 4096, 65536, MiB, 2 * MiB, 2 * MiB + 4096, 8 * MiB + 65536]
    if len(sys.argv) > 2:
        gaps = json.loads(sys.argv[2])
    sets = {}
    for gc in gaps:
        for go in ((gc,) if len(sys.argv) > 3 else (gc, 3 * gc + 4096 if gc else 0)):
            key = f"gap_co={gc},gap_out={go}"
            if key not in sets:
                sets[key] = carve(gc, go)
    origin = {"in_field": (2, 2, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    for a in sets.values():
        for st in sts:
            st(*a, origin=origin, domain=(ni, nj, nk))
    torch.cuda.synchronize()
    ref = next(iter(sets.values()))[1]
    for n, a in sets.items():
        assert torch.equal(a[1], ref), n
    times = {(n, i): [] for n in sets for i in range(len(sts))}
    for r in range(4):
        for (n, i) in times:
            a, st = sets[n], sts[i]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                st(*a, origin=origin, domain=(ni, nj, nk), validate_args=False)
            e1.record()
            torch.cuda.synchronize()
            times[(n, i)].append(e0.elapsed_time(e1) / 10)
    for (n, i), t in times.items():
        med = float(np.median(t))
        print(json.dumps({"alloc": n, "opts": optsets[i], "median_ms": round(med, 4), "min_ms": round(min(t), 4),
                          "GBps": round(ni * nj * nk * 24 / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
