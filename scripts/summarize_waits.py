#!/usr/bin/env python3
"""Summarise scripts/pmc_waits.sh: per config, the per-dispatch average of every counter over the
stencil's kernel launches (names containing ``_plane`` or ``_column``), and the wave-cycle split

    parked  = SQ_WAIT_ANY / SQ_WAVE_CYCLES          (s_waitcnt / barrier: waiting for memory)
    stalled = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES     (issue stalls: dependencies, pipes)
    active  = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES   (issuing)

plus the L2 hit rate TCC_HIT / (TCC_HIT + TCC_MISS) and the VALU/VMEM/LDS shares of issue.

    python scripts/summarize_waits.py gpurun_out/waits_r05a vadv copy
"""

import csv
import glob
import json
import sys


def counters(out, cfg):
    vals = {}
    for p in ("A", "B", "C", "D", "E", "F"):
        for f in glob.glob(f"{out}/{cfg}_{p}/**/*counter_collection.csv", recursive=True):
            per = {}
            for r in csv.DictReader(open(f)):
                if "_plane" not in r["Kernel_Name"] and "_column" not in r["Kernel_Name"]:
                    continue
                per.setdefault(r["Counter_Name"], {}).setdefault(r.get("Dispatch_Id", r.get("Correlation_Id")), 0.0)
                per[r["Counter_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id"))] += float(r["Counter_Value"])
            for name, d in per.items():
                vals[name] = sum(d.values()) / len(d)
                vals[name + "__dispatches"] = len(d)
    return vals


def main():
    out = sys.argv[1]
    res = {}
    for cfg in sys.argv[2:]:
        v = counters(out, cfg)
        wc = v.get("SQ_WAVE_CYCLES")
        row = {k: round(x, 1) for k, x in v.items()}
        if wc:
            for key, name in (("parked", "SQ_WAIT_ANY"), ("stalled", "SQ_WAIT_INST_ANY"), ("active", "SQ_ACTIVE_INST_ANY")):
                if name in v:
                    row[key] = round(v[name] / wc, 4)
        if "SQ_ACTIVE_INST_ANY" in v:
            for key in ("VALU", "VMEM", "LDS", "SCA"):
                name = f"SQ_ACTIVE_INST_{key}"
                if name in v and v["SQ_ACTIVE_INST_ANY"]:
                    row[f"issue_share_{key}"] = round(v[name] / v["SQ_ACTIVE_INST_ANY"], 4)
        if v.get("SQ_INSTS_VMEM") and v.get("SQ_INST_LEVEL_VMEM") is not None:
            # Little's law: VMEM instructions in flight (summed per cycle) / issued = mean latency
            row["vmem_latency_quad_cycles"] = round(v["SQ_INST_LEVEL_VMEM"] / v["SQ_INSTS_VMEM"], 1)
        for f in ("SQ_VMEM_TA_ADDR_FIFO_FULL", "SQ_VMEM_TA_CMD_FIFO_FULL", "SQ_VMEM_WR_TA_DATA_FIFO_FULL"):
            if f in v and wc:
                row[f.lower() + "_per_wave_cycle"] = round(v[f] / wc, 5)
        ih, im = v.get("SQC_ICACHE_HITS"), v.get("SQC_ICACHE_MISSES")
        if ih is not None and im is not None and ih + im:
            row["icache_miss_rate"] = round(im / (ih + im), 4)
        if v.get("SQ_IFETCH") and v.get("SQ_IFETCH_LEVEL") is not None:
            row["ifetch_latency_quad_cycles"] = round(v["SQ_IFETCH_LEVEL"] / v["SQ_IFETCH"], 1)
        h, m = v.get("TCC_HIT_sum"), v.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m:
            row["L2_hit"] = round(h / (h + m), 4)
        res[cfg] = row
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
