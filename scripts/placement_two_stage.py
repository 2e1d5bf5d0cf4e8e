#!/usr/bin/env python3
"""Is placing the READ fields worth a second tuning stage? Written fields first (as bench.py
does), then the read fields with the written ones fixed; both stages' per-set times printed.

    python3 scripts/placement_two_stage.py --config hdiff
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
    ap.add_argument("--candidates", type=int, default=5)
    args = ap.parse_args()
    import torch

    import bench
    from gt4py_amd.storage.placement import tune_fields, written_fields

    ns = types.SimpleNamespace(decomp="jstrips", jchunk=None, opt=None, fill="bulk", no_overlap=False,
                               halo_selfcomm=False, placement_candidates=0)
    wl = bench.Workload(args.config, ns, 0, 1, torch.device("cuda", 0), "gt:mi355x")
    names = list(wl.stencil.field_info.keys())
    arrays = dict(zip(names, wl.args))
    kw = dict(origin=wl.origin, domain=wl.domain, params=wl.params, candidates=args.candidates)
    w = written_fields(wl.stencil)
    arrays, r1 = tune_fields(wl.stencil, arrays, w, **kw)
    r = [n for n in names if n not in w]
    arrays, r2 = tune_fields(wl.stencil, arrays, r, **kw)
    arrays, r3 = tune_fields(wl.stencil, arrays, w, **kw)  # written again, reads now placed
    print(json.dumps({"config": args.config, "written": r1["candidates_ms"], "read": r2["candidates_ms"],
                      "written_again": r3["candidates_ms"], "final_ms": r3["tuned_ms"]}), flush=True)


if __name__ == "__main__":
    main()
