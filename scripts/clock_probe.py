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
import glob
import json
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def find_card(pci_bus_id: str):
    """sysfs device directory of the GPU with this PCI bus id (``0000:xx:00.0``)."""
    want = pci_bus_id.lower()
    for d in sorted(glob.glob("/sys/class/drm/card*/device")):
        ue = _read(os.path.join(d, "uevent")) or ""
        for line in ue.splitlines():
            if line.startswith("PCI_SLOT_NAME=") and line.split("=", 1)[1].lower().endswith(want[-7:]):
                return d
    return None


def _cur_level(text):
    if not text:
        return None
    for line in text.splitlines():
        if line.rstrip().endswith("*"):
            return line.split(":", 1)[-1].replace("*", "").strip()
    return None


def snapshot(card):
    """Current DPM levels, power, temperature and busy counters of the card (sysfs)."""
    if card is None:
        return {}
    s = {}
    for clk in ("sclk", "mclk", "fclk", "socclk", "vclk", "dcefclk"):
        s[clk] = _cur_level(_read(os.path.join(card, f"pp_dpm_{clk}")))
    s["perf_level"] = _read(os.path.join(card, "power_dpm_force_performance_level"))
    s["gpu_busy"] = _read(os.path.join(card, "gpu_busy_percent"))
    s["mem_busy"] = _read(os.path.join(card, "mem_busy_percent"))
    hw = sorted(glob.glob(os.path.join(card, "hwmon", "hwmon*")))
    if hw:
        h = hw[0]
        for name in ("power1_average", "power1_input", "power1_cap", "power1_cap_max", "temp1_input",
                     "temp2_input", "temp3_input", "freq1_input", "freq2_input"):
            v = _read(os.path.join(h, name))
            if v is not None:
                s[name] = v
    return s


def static_info(card):
    if card is None:
        return {}
    out = {}
    for name in ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "pp_dpm_socclk", "unique_id", "serial_number",
                 "product_name", "current_link_speed", "current_link_width", "vbios_version",
                 "mem_info_vram_used", "mem_info_vram_total", "pp_power_profile_mode"):
        v = _read(os.path.join(card, name))
        if v is not None:
            out[name] = v
    return out


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
    props = torch.cuda.get_device_properties(0)
    pci = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
    card = find_card(pci)
    head = {"tag": args.tag, "pci": pci, "card": card, "name": props.name, "uuid": str(props.uuid),
            "static": static_info(card), "before": snapshot(card), "pid": os.getpid()}
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
