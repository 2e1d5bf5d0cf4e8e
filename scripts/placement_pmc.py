#!/usr/bin/env python3
"""Do fast and slow HBM placements move the same bytes? hdiff with its in/coeff fixed and
``out_field`` in ``--sets`` buffers (set 0 = the first allocation), ``--reps`` launches per set in
set order, after the Workload's one validating launch. Run it plain (HIP-event times per set are
printed) and under ``rocprofv3 --pmc FETCH_SIZE`` / ``WRITE_SIZE``; ``--summarize DIR...`` then
groups the per-dispatch counters of the stencil kernel by set.

    python3 scripts/placement_pmc.py --sets 6 > times.jsonl
    rocprofv3 --pmc FETCH_SIZE -d d_fetch -o p -- python3 scripts/placement_pmc.py --sets 6
    python3 scripts/placement_pmc.py --summarize d_fetch d_write --sets 6
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
                rows = [r for r in csv.DictReader(f) if re.match(r"^k\d+_plane", r["Kernel_Name"])]
            rows.sort(key=lambda r: int(r["Dispatch_Id"]))
            ctr = rows[0]["Counter_Name"]
            vals = [float(r["Counter_Value"]) for r in rows][1:]  # skip the validating launch
            assert len(vals) == sets * reps, (path, len(vals))
            out[ctr] = [round(sum(vals[s * reps:(s + 1) * reps]) / reps / 1024, 1) for s in range(sets)]
    print(json.dumps({"MiB_per_dispatch_by_set": out}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=6)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--summarize", nargs="*", default=None)
    args = ap.parse_args()
    if args.summarize is not None:
        return summarize(args.summarize, args.sets, args.reps)
    import torch

    import bench
    from gt4py_amd.storage.placement import like

    ns = types.SimpleNamespace(decomp="jstrips", jchunk=None, opt=None, fill="bulk", no_overlap=False,
                               halo_selfcomm=False, placement_candidates=0)
    wl = bench.Workload("hdiff", ns, 0, 1, torch.device("cuda", 0), "gt:mi355x")
    outs = [wl.named["out_field"]] + [like(wl.named["out_field"]) for _ in range(args.sets - 1)]
    ms = []
    for o in outs:
        call = lambda: wl.stencil(in_field=wl.named["in_field"], out_field=o, coeff=wl.named["coeff"],  # noqa: E731
                                  origin=wl.origin, domain=wl.domain, validate_args=False)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in evs:
            a.record()
            call()
            b.record()
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) for a, b in evs)
        ms.append(round(t[len(t) // 2], 4))
    print(json.dumps({"ms_by_set": ms}), flush=True)


if __name__ == "__main__":
    main()
