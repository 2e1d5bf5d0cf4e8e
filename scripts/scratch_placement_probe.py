#!/usr/bin/env python3
"""Does a column kernel's time depend on where its SCRATCH temporaries live (vadv: ccol/dcol
cross the two sweeps)? The API fields stay where they are; the launcher's
scratch buffers are re-allocated ``--sets`` times (old sets kept alive, so no prepared launch
can point at freed memory) and the same call is timed on each (HIP events, median of 10).

    python3 scripts/scratch_placement_probe.py --config vadv --sets 6
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
    ap.add_argument("--config", default="vadv")
    ap.add_argument("--sets", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import torch

    import bench
    from gt4py_amd.storage.placement import _time_call

    ns = types.SimpleNamespace(decomp="jstrips", jchunk=None, opt=None, fill="bulk", no_overlap=False,
                               halo_selfcomm=False, placement_candidates=0)
    wl = bench.Workload(args.config, ns, 0, 1, torch.device("cuda", 0), "gt:mi355x")
    launcher = wl.stencil._gt_run_impl_.compiled.launcher
    keep, sets = [], []
    for s in range(args.sets):
        if s:
            keep.append(dict(launcher._scratch_cache))
            launcher._scratch_cache.clear()
            launcher._pack_cache.clear()
            wl.stencil.clean_call_args_cache()
        wl.plain_step()
        torch.cuda.synchronize()
        sets.append(dict(launcher._scratch_cache))
    res = []
    for r in range(args.rounds):  # revisit every set: is the time a property of the set?
        row = []
        for s in sets:
            launcher._scratch_cache.clear()
            launcher._scratch_cache.update(s)
            launcher._pack_cache.clear()
            wl.stencil.clean_call_args_cache()
            row.append(round(_time_call(wl.plain_step, 10), 4))
        res.append(row)
        print(json.dumps({"config": args.config, "round": r, "scratch_sets_ms": row,
                          "n_scratch": len(launcher.scratch)}), flush=True)
    del keep


if __name__ == "__main__":
    main()
