#!/usr/bin/env python3
"""Fast and slow HBM placements of a column kernel's fields, side by side in one process.

The column kernels run in two modes on the same library (tridiag 1024^2x160: ~1.55 ms or
~1.80 ms; a fresh process's first allocation is the slow one, profiles/r05/r05t-r05w). This
probe gives ALL of a config's fields ``--sets`` placements (set 0 = the Workload's first
allocation, the others ``placement.like`` copies of every field, all alive at once), times each
set (one warm launch + ``--reps`` timed launches, in set order) and prints the times and field
addresses. Run it under ``rocprofv3 --pmc <counters>`` and ``--summarize`` groups the column
kernel's per-dispatch counters by set, so a fast and a slow set can be compared counter by counter.

    python3 scripts/column_placement_probe.py --config tridiag --sets 6 > times.jsonl
    rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum -d d1 -o p -- python3 scripts/column_placement_probe.py ...
    python3 scripts/column_placement_probe.py --summarize d1 d2 --sets 6 --reps 6
"""
import argparse
import csv
import glob
import json
import os
import re
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def summarize(dirs, sets, reps):
    out = {}
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path, newline="") as f:
                rows = [r for r in csv.DictReader(f) if re.match(r"^k\d+_(column|plane)", r["Kernel_Name"])]
            per = {}
            for r in rows:
                per.setdefault(r["Counter_Name"], {}).setdefault(int(r["Dispatch_Id"]), 0.0)
                per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            for ctr, byd in per.items():
                vals = [byd[k] for k in sorted(byd)][1:]  # skip the Workload's validating launch
                assert len(vals) == sets * (reps + 1), (path, ctr, len(vals))
                out[ctr] = [sum(vals[s * (reps + 1) + 1:(s + 1) * (reps + 1)]) / reps for s in range(sets)]
    print(json.dumps({"per_dispatch_by_set": out}, indent=1))


def _time(call, reps):
    import torch

    call()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record()
        call()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in evs)
    return round(t[len(t) // 2], 4)


def build_variants(args):
    import bench
    from gt4py_amd import gtscript

    variants = []
    for part in filter(None, (p.strip() for p in args.variants.split(";"))):
        variants.append({k.strip(): int(v) for k, v in (kv.split("=") for kv in part.split(","))} if "=" in part else {})
    sname, dtype = bench.CONFIGS[args.config][:2]
    sts = [gtscript.stencil(backend="gt:mi355x", definition=bench.stencil_defs()[(sname, dtype)],
                            name=f"cpp.{args.config}.{i}", device_sync=False,
                            externals=bench.EXTERNALS.get(sname, {}), **v) for i, v in enumerate(variants)]
    return variants, sts


def variant_matrix(args, wl, sets):
    variants, sts = build_variants(args)
    rows = []
    for si, s in enumerate(sets):
        for st in sts:  # first call: validation on this set
            st(*s, **wl.params, origin=wl.origin, domain=wl.domain)
        ms = [[] for _ in sts]
        for _ in range(args.rounds):
            for i, st in enumerate(sts):
                ms[i].append(_time(lambda st=st, s=s: st(*s, **wl.params, origin=wl.origin, domain=wl.domain,
                                                           validate_args=False), args.reps))
        rows.append({"set": si, "ms": [sorted(m)[len(m) // 2] for m in ms]})
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"config": args.config, "variants": variants, "matrix": [r["ms"] for r in rows]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="tridiag")
    ap.add_argument("--sets", type=int, default=6)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--summarize", nargs="*", default=None)
    ap.add_argument("--variants", default="",
                    help="codegen option sets 'k=v,k=v;k=v' timed on every placement set, interleaved "
                         "(a variant matrix: which schedule wins in which placement mode)")
    ap.add_argument("--build-only", action="store_true", help="compile the --variants libraries (no GPU)")
    args = ap.parse_args()
    if args.summarize is not None:
        return summarize(args.summarize, args.sets, args.reps)
    if args.build_only:
        return print(f"built {len(build_variants(args)[1])} variants")
    import torch

    import bench
    from gt4py_amd.storage.placement import like

    ns = types.SimpleNamespace(decomp="jstrips", jchunk=None, opt=None, fill="bulk", no_overlap=False,
                               halo_selfcomm=False, placement_candidates=0)
    wl = bench.Workload(args.config, ns, 0, 1, torch.device("cuda", 0), "gt:mi355x")
    fields = [a for a in wl.args if hasattr(a, "data_ptr")]
    sets = [list(wl.args)]
    for _ in range(args.sets - 1):
        s = []
        for a in wl.args:
            if hasattr(a, "data_ptr"):
                b = like(a)
                b.copy_(a)
                s.append(b)
            else:
                s.append(a)
        sets.append(s)
    torch.cuda.synchronize()
    if args.variants:
        return variant_matrix(args, wl, sets)
    res = []
    for s in sets:
        call = lambda s=s: wl.stencil(*s, **wl.params, origin=wl.origin, domain=wl.domain,  # noqa: E731
                                      validate_args=False)
        call()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in evs:
            a.record()
            call()
            b.record()
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) for a, b in evs)
        res.append({"ms": round(t[len(t) // 2], 4),
                    "ptrs": [hex(a.data_ptr()) for a in s if hasattr(a, "data_ptr")]})
    print(json.dumps({"config": args.config, "fields": len(fields), "sets": res}), flush=True)


if __name__ == "__main__":
    main()
