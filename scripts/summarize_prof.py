#!/usr/bin/env python3
"""Summarise rocprofv3 output (kernel-trace stats + FETCH_SIZE/WRITE_SIZE passes) for gt:mi355x
kernels (names k<N>_plane / k<N>_column), writing profiles/<tag>_summary.json and a short
per-config text table. FETCH_SIZE/WRITE_SIZE are in KiB per dispatch (rocprofv3 derived)."""

import csv
import glob
import json
import os
import re
import sys

OURS = re.compile(r"^k\d+_(plane|column)")


def read_csv(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main(prof_dir, tag):
    out = {}
    for bench in sorted(glob.glob(os.path.join(prof_dir, "bench_*.json"))):
        cfg = os.path.basename(bench)[6:-5]
        with open(bench) as f:
            b = json.load(f)
        entry = {"bench": {k: b[k] for k in ("value", "unit", "ms_per_step")}, "roofline": b["roofline"],
                 "workload": b["config"]["workload"]}
        stats = glob.glob(os.path.join(prof_dir, f"kt_{cfg}", "*kernel_stats.csv"))
        if stats:
            rows = [r for r in read_csv(stats[0]) if OURS.match(r["Name"])]
            entry["kernel_stats"] = [
                {"name": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                 "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])} for r in rows
            ]
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            files = glob.glob(os.path.join(prof_dir, f"pmc_{cfg}_{ctr}", "*counter_collection.csv"))
            if not files:
                continue
            vals = [float(r["Counter_Value"]) for r in read_csv(files[0])
                    if OURS.match(r["Kernel_Name"]) and r["Counter_Name"] == ctr]
            if vals:
                entry[ctr + "_KiB_per_dispatch"] = sum(vals) / len(vals)
        out[cfg] = entry
    path = os.path.join("profiles", f"{tag}_summary.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    for cfg, e in out.items():
        ks = e.get("kernel_stats", [])
        avg = ks[0]["avg_ns"] / 1e6 if ks else float("nan")
        print(f"{cfg:10s} {e['bench']['value']:>12.1f} Mcells/s  event {e['roofline']['kernel_ms']:.4f} ms  "
              f"rocprof {avg:.4f} ms  frac {e['roofline']['frac']:.3f}  "
              f"FETCH {e.get('FETCH_SIZE_KiB_per_dispatch', float('nan')) / 1024:.1f} MiB  "
              f"WRITE {e.get('WRITE_SIZE_KiB_per_dispatch', float('nan')) / 1024:.1f} MiB")
        fetch, write = e.get("FETCH_SIZE_KiB_per_dispatch"), e.get("WRITE_SIZE_KiB_per_dispatch")
        if fetch is not None and write is not None:
            # bench.py reads roofline.traffic from here (per-launch HBM bytes, gfx950 correction)
            with open(os.path.join("profiles", f"pmc_{cfg}.json"), "w") as f:
                json.dump({
                    "config": cfg,
                    "workload": e["workload"],
                    # bench.py reports this record's bytes only for the library it was measured on
                    "build_key": e["roofline"].get("library"),
                    "hbm_bytes_per_launch": int(round((2 * fetch + write) * 1024)),
                    "fetch_size_kib": round(fetch, 1),
                    "write_size_kib": round(write, 1),
                    "correction": CORRECTION,
                    "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
                              f"bench.py --config {cfg} (profiles/{tag}_summary.json)",
                }, f, indent=1)
    return path


CORRECTION = ("hbm = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 B: on gfx950 FETCH_SIZE reports half the bytes of a "
              "wide coalesced read (MI355X_MICROARCH.md HBM section); calibrated on the copy stencil "
              "(1280 MiB read -> FETCH 640 MiB, WRITE 1280 MiB exact)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
