#!/usr/bin/env python3
"""Timeline of the bench workload's step time next to the GPU's clock / power state.

Runs a bench config (default hdiff 2048x2048x160 f64) back to back for ``--seconds`` and prints,
per ``--window`` seconds, the mean ms/step together with what sysfs says about the card the
process runs on (current sclk / mclk / fclk / socclk DPM level, power, temperature). Used to
find out whether the driver's fresh-lease runs sit in a different clock or power state than
runs that follow other GPU work (VERDICT r02 "next round" item 1).

    python3 scripts/clock_probe.py --seconds 60 --tag first > gpurun_out/probe_first.jsonl
"""
import argparse
import json
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="hdiff")
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--window", type=float, default=0.5)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()

    import torch

    import bench

    t_start = time.time()
    card, ident = bench.box_identity(0)
    snapshot = bench.card_snapshot
    head = {"tag": args.tag, "card": card, "identity": ident, "before": snapshot(card), "pid": os.getpid()}
    print(json.dumps(head), flush=True)
    dev = torch.device("cuda", 0)
    ns = types.SimpleNamespace(decomp="jstrips", jchunk=None, opt=None, fill="bulk", no_overlap=False,
                               halo_selfcomm=False)
    wl = bench.Workload(args.config, ns, 0, 1, dev, "gt:mi355x")
    torch.cuda.synchronize()
    print(json.dumps({"tag": args.tag, "setup_s": round(time.time() - t_start, 2), "after_setup": snapshot(card)}),
          flush=True)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:
        w0 = time.perf_counter()
        n = 0
        while True:
            wl.plain_step()
            n += 1
            if n % 8 == 0:
                torch.cuda.synchronize()
                if time.perf_counter() - w0 >= args.window:
                    break
        dt = time.perf_counter() - w0
        rec = {"t": round(w0 - t0, 2), "steps": n, "ms": round(dt / n * 1e3, 4)}
        rec.update(snapshot(card))
        print(json.dumps(rec), flush=True)
    print(json.dumps({"tag": args.tag, "end": snapshot(card)}), flush=True)


if __name__ == "__main__":
    main()
