#!/usr/bin/env python3
"""Split a rocprofv3 --kernel-trace of ``bench.py`` by code object.

``--stats`` aggregates dispatches by kernel NAME, and every gt:mi355x library names its kernel
``k0_plane_v2`` / ``k0_column`` / ...: one profiled bench run (headline + extra configs) mixes the
hdiff, lap5, copy and hdiff_blocks launches under one ``k0_plane_v2`` line. Each loaded library
has its own ``Kernel_Id``, so grouping the trace by it gives one line per config; the configs
appear in bench.py's order (headline first, then ``extra_configs``), which pairs each line with
the bench line's event-timed ``kernel_ms``.

    python scripts/trace_by_kernel.py gpurun_out/r05o/kt_bench/kt_kernel_trace.csv \
        gpurun_out/r05o/bench.json > profiles/r05/r05o_kernel_trace_by_config.json
"""

import csv
import json
import re
import statistics
import sys

OURS = re.compile(r"^k\d+_(plane|column)")


def main(trace, bench):
    groups = {}
    for r in csv.DictReader(open(trace, newline="")):
        if not OURS.match(r["Kernel_Name"]):
            continue
        g = groups.setdefault(int(r["Kernel_Id"]), {"name": r["Kernel_Name"], "grid_x": int(r["Grid_Size_X"]),
                                                     "vgpr": int(r["VGPR_Count"]), "lds": int(r["LDS_Block_Size"]),
                                                     "ns": []})
        g["ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    b = json.load(open(bench))
    configs = [(b["config"]["workload"], b["roofline"]["kernel_ms"])]
    configs += [(c["workload"], c["kernel_ms"]) for c in b.get("extra_configs", {}).values()]
    out = []
    for (kid, g), cfg in zip(sorted(groups.items()), configs + [(None, None)] * len(groups)):
        ns = g.pop("ns")
        row = {"kernel_id": kid, **g, "dispatches": len(ns), "avg_ms": round(statistics.mean(ns) / 1e6, 4),
               "median_ms": round(statistics.median(ns) / 1e6, 4), "min_ms": round(min(ns) / 1e6, 4),
               "workload": cfg[0], "bench_kernel_ms": cfg[1]}
        if cfg[1]:
            row["median_vs_bench"] = round(row["median_ms"] / cfg[1], 4)
        out.append(row)
    json.dump({"trace": trace, "bench": bench, "note": __doc__.split("\n\n")[0], "kernels": out},
              sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
