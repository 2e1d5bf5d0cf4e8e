#!/usr/bin/env python3
"""Does the hdiff kernel time depend on WHERE in device memory its three fields live?

One big pool (``--pool-gb`` of HBM, one allocation) holds every placement; the fields are
strided views into it, laid out exactly as ``gt4py_amd.storage`` lays them out (I pitch padded to
32 elements, the compute origin on a 256-B boundary). The same compiled library runs on each
placement (HIP-event time per launch, median of ``--reps``):

* scan ``packed``: the triplet (in, coeff, out) back to back, its start moved through the pool;
* scan ``out``: in + coeff fixed at the pool start, only ``out`` moved;
* scan ``gap``: in + coeff + out back to back at the pool start, with a gap of g MiB between
  consecutive fields (g sweeps 0..N).

    python3 scripts/placement_scan.py --pool-gb 160 --step-gb 4 > gpurun_out/placement_scan.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool-gb", type=float, default=160.0)
    ap.add_argument("--step-gb", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--scans", default="packed,out,gap,packed")
    ap.add_argument("--gaps-mib", default="0,1,2,4,6,8,16,32,64,128,256,512,1024")
    ap.add_argument("--config", default="hdiff")
    ap.add_argument("--check", action="store_true",
                    help="every variant's output must be bit-identical to the default library's (first placement)")
    ap.add_argument("--probe-strides", default="",
                    help="comma-separated byte strides: per placement, also time a strided sum over the triplet's "
                         "bytes touching one element per stride (a TLB-reach probe: a few MB of traffic, one access "
                         "per page at 4096)")
    ap.add_argument("--rw-probe", action="store_true",
                    help="per placement, also time a plain write (fill_) over out's bytes and a plain read (sum) "
                         "over in's bytes: does the placement effect follow the written or the read stream?")
    ap.add_argument("--variants", default="",
                    help="';'-separated codegen option sets timed on every placement (e.g. 'order=5;order=3'); "
                         "the default library is always first")
    args = ap.parse_args()

    import torch

    import bench
    from gt4py_amd import gtscript

    sname, dtype, (ni, nj, nk), h, bpc = bench.CONFIGS[args.config]
    it = np.dtype(dtype).itemsize
    tdt = {8: torch.float64, 4: torch.float32}[it]
    variants = [("default", {})]
    for v in filter(None, args.variants.split(";")):
        opts = {}
        for kv in v.split(","):
            k, x = kv.split("=")
            opts[k] = int(x)
        variants.append((v, opts))
    stencils = [(vn, gtscript.stencil(backend="gt:mi355x", definition=bench.stencil_defs()[(sname, dtype)],
                                      name=f"bench.{args.config}", device_sync=False, **opts))  # the bench's library
                for vn, opts in variants]
    if os.environ.get("BUILD_ONLY"):
        return
    pool_bytes = int(args.pool_gb * (1 << 30))
    t0 = time.time()
    pool = torch.empty(pool_bytes // it, dtype=tdt, device="cuda")
    chunk = 1 << 28
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1337)
    for s in range(0, pool.numel(), chunk):
        e = min(pool.numel(), s + chunk)
        pool[s:e].uniform_(0.0, 0.5, generator=gen)
    torch.cuda.synchronize()
    base_ptr = pool.data_ptr()
    print(json.dumps({"pool_gb": args.pool_gb, "base": hex(base_ptr), "fill_s": round(time.time() - t0, 2)}), flush=True)

    pad = lambda n: -(-n // 32) * 32  # noqa: E731
    shp_in = (ni + 2 * h, nj + 2 * h, nk)
    shp = (ni, nj, nk)
    str_in = (1, pad(shp_in[0]), pad(shp_in[0]) * shp_in[1])
    str_o = (1, pad(ni), pad(ni) * nj)
    bytes_in = str_in[2] * nk * it
    bytes_o = str_o[2] * nk * it

    def view(byte_off, shape, strides, aligned):
        """Field view whose aligned element sits at the first 256-B boundary >= byte_off."""
        ai = sum(a * s for a, s in zip(aligned, strides)) * it
        addr = base_ptr + byte_off + ai
        addr += (-addr) % 256
        first = (addr - ai - base_ptr) // it
        end = first + sum((n - 1) * s for n, s in zip(shape, strides)) + 1
        assert first >= 0 and end <= pool.numel(), (byte_off, first, end, pool.numel())
        return torch.as_strided(pool, size=shape, stride=strides, storage_offset=first)

    def run(off_in, off_c, off_o):
        fin = view(off_in, shp_in, str_in, (h, h, 0))
        co = view(off_c, shp, str_o, (0, 0, 0))
        out = view(off_o, shp, str_o, (0, 0, 0))
        orig = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
        res = {}
        ref = None
        for vn, st in stencils:
            call = lambda: st(fin, out, co, origin=orig, domain=shp, validate_args=False)  # noqa: E731
            call()
            call()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.reps)]
            for a, b in evs:
                a.record()
                call()
                b.record()
            torch.cuda.synchronize()
            ms = sorted(a.elapsed_time(b) for a, b in evs)
            res[vn] = round(ms[len(ms) // 2], 4)
            if args.check and not checked:
                if ref is None:
                    ref = out.clone()
                else:
                    same = bool(torch.equal(out, ref))
                    print(json.dumps({"check": vn, "bit_identical": same}), flush=True)
                    if not same:
                        raise SystemExit(f"variant {vn} differs from the default library")
                out.fill_(float("nan"))
        if args.check:
            checked.append(True)
        return res

    probe_strides = [int(x) for x in args.probe_strides.split(",") if x]

    def probe(off, nbytes):
        """ms of a strided sum over [off, off + nbytes) of the pool, one element per stride."""
        res = {}
        for sb in probe_strides:
            v = pool[off // it:(off + nbytes) // it:sb // it]
            v.sum()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(5):
                e0.record()
                v.sum()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res[f"probe{sb}"] = round(sorted(ts)[2], 4)
        return res

    checked = []
    def rw_probe(off_in, off_o):
        """GB/s of a plain read of in's bytes and a plain write of out's bytes (median of 5)."""
        res = {}
        for kind, off, nb in (("read", off_in, bytes_in), ("write", off_o, bytes_o)):
            v = pool[off // it:(off + nb) // it]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(6):
                e0.record()
                if kind == "read":
                    v.sum()
                else:
                    v.fill_(0.25)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res[f"{kind}_GBs"] = round(nb / (sorted(ts[1:])[2] * 1e-3) / 1e9, 1)
        return res

    step = int(args.step_gb * (1 << 30))
    triple = bytes_in + 2 * bytes_o + 3 * 256
    for scan in args.scans.split(","):
        if scan == "packed":
            offs = range(0, pool_bytes - triple - 2 * MIB, step)
            for o in offs:
                res = run(o, o + bytes_in + 256, o + bytes_in + bytes_o + 512)
                res.update(probe(o, triple))
                if args.rw_probe:
                    res.update(rw_probe(o, o + bytes_in + bytes_o + 512))
                print(json.dumps({"scan": scan, "off_gb": round(o / (1 << 30), 2), "ms": res}), flush=True)
        elif scan == "out":
            lo = bytes_in + bytes_o + 512
            for o in range(lo, pool_bytes - bytes_o - 2 * MIB, step):
                res = run(0, bytes_in + 256, o)
                res.update(probe(o, bytes_o))
                if args.rw_probe:
                    res.update(rw_probe(0, o))
                print(json.dumps({"scan": scan, "out_gb": round(o / (1 << 30), 2), "ms": res}), flush=True)
        elif scan == "gap":
            for g in (int(x) for x in args.gaps_mib.split(",")):
                gb = g * MIB
                res = run(0, bytes_in + gb, bytes_in + bytes_o + 2 * gb)
                print(json.dumps({"scan": scan, "gap_mib": g, "ms": res}), flush=True)


if __name__ == "__main__":
    main()
