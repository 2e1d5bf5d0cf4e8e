#!/usr/bin/env python3
"""Does the hdiff time of a fresh process depend on what was allocated before its fields?

One process = one allocation history: optionally hold ``--pre-gb`` GB of device memory, then
build the bench workload (in_field, out_field, coeff through gt4py_amd.storage, in bench order)
and time the kernel (HIP events, median of 20). Several processes in a row on one box compare
histories; each prints one JSON line.

    python3 scripts/alloc_probe.py --pre-gb 16 --tag pre16
"""
import argparse
import json
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="hdiff")
    ap.add_argument("--pre-gb", type=float, default=0.0, help="device memory held before the fields")
    ap.add_argument("--post-free", action="store_true", help="free the pre-allocation before timing")
    ap.add_argument("--carve", action="store_true",
                    help="free the pre-allocation BEFORE the fields: torch's caching allocator then carves "
                         "the fields out of that one cached segment")
    ap.add_argument("--warm-s", type=float, default=0.0,
                    help="keep the GPU busy this long before the fields are allocated")
    ap.add_argument("--warm-with", default="copy", help="'copy' (a torch device copy loop) or a bench config")
    ap.add_argument("--pre-chunks", type=int, default=0, help="hold this many --pre-chunk-gb blocks before the fields")
    ap.add_argument("--pre-chunk-gb", type=float, default=1.5)
    ap.add_argument("--empty-cache", action="store_true", help="release torch's cached blocks after the warm-up")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()

    import torch

    import bench

    if args.warm_s > 0:
        import time

        if args.warm_with == "copy":
            a = torch.empty(1 << 30, dtype=torch.float32, device="cuda")
            b = torch.empty_like(a)
            step = lambda: b.copy_(a)  # noqa: E731
        else:
            ns0 = types.SimpleNamespace(decomp="jstrips", jchunk=None, opt=None, fill="bulk", no_overlap=False,
                                        halo_selfcomm=False)
            wl0 = bench.Workload(args.warm_with, ns0, 0, 1, torch.device("cuda", 0), "gt:mi355x")
            step = wl0.plain_step
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.warm_s:
            for _ in range(20):
                step()
            torch.cuda.synchronize()
        del step
        if args.warm_with == "copy":
            del a, b
        else:
            del wl0
        if args.empty_cache:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    held = [torch.empty(int(args.pre_chunk_gb * (1 << 30)), dtype=torch.uint8, device="cuda")
            for _ in range(args.pre_chunks)]
    pre = None
    if args.pre_gb > 0:
        pre = torch.empty(int(args.pre_gb * (1 << 30)), dtype=torch.uint8, device="cuda")
        if args.carve:
            del pre
            pre = None
    ns = types.SimpleNamespace(decomp="jstrips", jchunk=None, opt=None, fill="bulk", no_overlap=False,
                               halo_selfcomm=False)
    wl = bench.Workload(args.config, ns, 0, 1, torch.device("cuda", 0), "gt:mi355x")
    if pre is not None and args.post_free:
        del pre
        pre = None
    torch.cuda.synchronize()
    for _ in range(3):
        wl.plain_step()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for a, b in evs:
        a.record()
        wl.plain_step()
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in evs)
    rec = {"tag": args.tag, "config": args.config, "pre_gb": args.pre_gb, "carve": args.carve, "warm_s": args.warm_s, "warm_with": args.warm_with, "empty_cache": args.empty_cache, "pre_chunks": args.pre_chunks,
           "pre_chunk_gb": args.pre_chunk_gb, "held": len(held), "kernel_ms": round(ms[len(ms) // 2], 4),
           "ptrs": [hex(t.data_ptr()) for t in wl.args if hasattr(t, "data_ptr")]}
    rec["placement_probe"] = (wl.placement or {}).get("candidates_ms")
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
