#!/usr/bin/env python3
"""Benchmark of the gt:mi355x hot path (BASELINE.json metric).

Default workload (``--config hdiff``): ``horizontal_diffusion`` (lap + flux + limiter,
PARALLEL K) at 2048 x 2048 x 160 fp64 per GPU -- BASELINE.json configs[2], the config the
metric "Mcells/s + achieved HBM GB/s, horiz-diffusion 2048x2048x160 fp64, 1/2/4/8 GPU" is
quoted on. ``--gpus N`` (N > 1) without a torchrun environment starts N ranks itself
(``torch.distributed.run`` child, one process per GPU) and relays rank 0's line; under torchrun
each rank owns a 2048 x 2048 x 160 J strip of a 2048 x (2048*N) x 160 global domain (weak
scaling) and every step exchanges the 2-row J halo of ``in_field`` over RCCL while the interior
computes.

One step = one stencil application over the whole (local) domain, inputs resident in HBM.
Timing: W untimed warmups, then K steps bracketed by barrier + synchronize; max over ranks.
``roofline`` = algorithmic bytes (24 B/cell: in + coeff read, out written)
per launch / mean launch time from HIP events on the launch stream; ``traffic`` = rocprofv3
PMC bytes per launch from ``profiles/pmc_<config>.json`` when that record was measured on the
same library (build key), else null. ``sustained`` (N=1): the same step repeated for ~3 s after
the timed K steps (steady-state ms/step; ``--sustain 0`` skips it). ``full_call`` (N=1): K calls
the reference's way (validate_args=True, synchronize after each). ``extra_configs`` (N=1): the
other BASELINE configs timed in the same process. ``cpu_baseline`` = the C restatement (cpu_ifirst-equivalent, OpenMP) on
the full domain, median of 40 after 3 warm-ups, in a child process; lap5 (C2) and tridiag (C4)
carry their own ``extra_configs.<cfg>.cpu_baseline`` (median of 20) next to their GPU figures.
"""



import argparse
import json
import os
import sys
import time

import numpy as np

_START = time.time()
REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (stencil, dtype, (ni, nj, nk), halo, bytes/cell)
    "hdiff": ("horizontal_diffusion", np.float64, (2048, 2048, 160), 2, 24),
    "hdiff_f32": ("horizontal_diffusion", np.float32, (8192, 1024, 160), 2, 12),
    "lap5": ("lap5", np.float64, (1024, 1024, 80), 1, 16),
    "tridiag": ("tridiagonal_solver", np.float64, (1024, 1024, 160), 0, 56),
    "copy": ("copy_stencil", np.float64, (1024, 1024, 160), 0, 16),
    # the canonical production K-sweep (5 fields read, 1 written)
    "vadv": ("vertical_advection_dycore", np.float64, (1024, 1024, 160), 0, 48),
    # hdiff written as three computations (lap / fluxes / update): fused into one launch
    "hdiff_blocks": ("horizontal_diffusion_blocks", np.float64, (2048, 2048, 160), 2, 24),
    # a multi-stage stencil the two skeletons cannot take directly (a FORWARD recurrence feeding
    # a temporary read at IJ offsets in a FORWARD loop): the staged lowering (SURVEY.md §8(f)
    # row 1); algorithmic bytes: `a` read + `out` written
    "staged": ("staged_forward_ij_temp", np.float64, (1024, 1024, 160), 1, 16),
    # shape probes for work-order experiments (scripts/sweep.py; never bench lines)
    "staged_f32": ("staged_forward_ij_temp", np.float32, (2048, 1024, 160), 1, 8),
    "lap5_k160": ("lap5", np.float64, (1024, 1024, 160), 1, 16),
    "lap5_2k": ("lap5", np.float64, (2048, 2048, 80), 1, 16),
    "copy_k80": ("copy_stencil", np.float64, (1024, 1024, 80), 0, 16),
    "hdiff_k80": ("horizontal_diffusion", np.float64, (2048, 2048, 80), 2, 24),
}


EXTERNALS = {"vertical_advection_dycore": {"BET_M": 0.5, "BET_P": 0.5}}


def stencil_defs():
    from gt4py_amd.gtscript import BACKWARD, FORWARD, PARALLEL, Field, computation, interval

    def make_hdiff(dtype):
        FT = Field[dtype]

        def horizontal_diffusion(in_field: FT, out_field: FT, coeff: FT):
            with computation(PARALLEL), interval(...):
                lap_field = 4.0 * in_field[0, 0, 0] - (
                    in_field[1, 0, 0] + in_field[-1, 0, 0] + in_field[0, 1, 0] + in_field[0, -1, 0]
                )
                res = lap_field[1, 0, 0] - lap_field[0, 0, 0]
                flx_field = 0 if (res * (in_field[1, 0, 0] - in_field[0, 0, 0])) > 0 else res
                res = lap_field[0, 1, 0] - lap_field[0, 0, 0]
                fly_field = 0 if (res * (in_field[0, 1, 0] - in_field[0, 0, 0])) > 0 else res
                out_field = in_field[0, 0, 0] - coeff[0, 0, 0] * (
                    flx_field[0, 0, 0] - flx_field[-1, 0, 0] + fly_field[0, 0, 0] - fly_field[0, -1, 0]
                )

        return horizontal_diffusion

    F64 = Field[np.float64]

    def lap5(in_field: F64, out_field: F64):
        with computation(PARALLEL), interval(...):
            out_field = 4.0 * in_field[0, 0, 0] - (
                in_field[1, 0, 0] + in_field[-1, 0, 0] + in_field[0, 1, 0] + in_field[0, -1, 0]
            )

    def copy_stencil(field_a: F64, field_b: F64):
        with computation(PARALLEL), interval(...):
            field_b = field_a[0, 0, 0]

    def tridiagonal_solver(inf: F64, diag: F64, sup: F64, rhs: F64, out: F64):
        with computation(FORWARD):
            with interval(0, 1):
                sup = sup / diag
                rhs = rhs / diag
            with interval(1, None):
                sup = sup / (diag - sup[0, 0, -1] * inf)
                rhs = (rhs - inf * rhs[0, 0, -1]) / (diag - sup[0, 0, -1] * inf)
        with computation(BACKWARD):
            with interval(-1, None):
                out = rhs
            with interval(0, -1):
                out = rhs - sup * out[0, 0, 1]

    def vertical_advection_dycore(utens_stage: F64, u_stage: F64, wcon: F64, u_pos: F64, utens: F64, *,
                                  dtr_stage: float):
        # stencil_definitions.py:236-313 (restated)
        from __externals__ import BET_M, BET_P

        with computation(FORWARD):
            with interval(0, 1):
                gcv = 0.25 * (wcon[1, 0, 1] + wcon[0, 0, 1])
                cs = gcv * BET_M
                ccol = gcv * BET_P
                bcol = dtr_stage - ccol[0, 0, 0]
                correction_term = -cs * (u_stage[0, 0, 1] - u_stage[0, 0, 0])
                dcol = dtr_stage * u_pos[0, 0, 0] + utens[0, 0, 0] + utens_stage[0, 0, 0] + correction_term
                divided = 1.0 / bcol[0, 0, 0]
                ccol = ccol[0, 0, 0] * divided
                dcol = dcol[0, 0, 0] * divided
            with interval(1, -1):
                gav = -0.25 * (wcon[1, 0, 0] + wcon[0, 0, 0])
                gcv = 0.25 * (wcon[1, 0, 1] + wcon[0, 0, 1])
                as_ = gav * BET_M
                cs = gcv * BET_M
                acol = gav * BET_P
                ccol = gcv * BET_P
                bcol = dtr_stage - acol[0, 0, 0] - ccol[0, 0, 0]
                correction_term = -as_ * (u_stage[0, 0, -1] - u_stage[0, 0, 0]) - cs * (
                    u_stage[0, 0, 1] - u_stage[0, 0, 0]
                )
                dcol = dtr_stage * u_pos[0, 0, 0] + utens[0, 0, 0] + utens_stage[0, 0, 0] + correction_term
                divided = 1.0 / (bcol[0, 0, 0] - ccol[0, 0, -1] * acol[0, 0, 0])
                ccol = ccol[0, 0, 0] * divided
                dcol = (dcol[0, 0, 0] - (dcol[0, 0, -1]) * acol[0, 0, 0]) * divided
            with interval(-1, None):
                gav = -0.25 * (wcon[1, 0, 0] + wcon[0, 0, 0])
                as_ = gav * BET_M
                acol = gav * BET_P
                bcol = dtr_stage - acol[0, 0, 0]
                correction_term = -as_ * (u_stage[0, 0, -1] - u_stage[0, 0, 0])
                dcol = dtr_stage * u_pos[0, 0, 0] + utens[0, 0, 0] + utens_stage[0, 0, 0] + correction_term
                divided = 1.0 / (bcol[0, 0, 0] - ccol[0, 0, -1] * acol[0, 0, 0])
                dcol = (dcol[0, 0, 0] - (dcol[0, 0, -1]) * acol[0, 0, 0]) * divided
        with computation(BACKWARD):
            with interval(-1, None):
                datacol = dcol[0, 0, 0]
                utens_stage = dtr_stage * (datacol - u_pos[0, 0, 0])
            with interval(0, -1):
                datacol = dcol[0, 0, 0] - ccol[0, 0, 0] * datacol[0, 0, 1]
                utens_stage = dtr_stage * (datacol - u_pos[0, 0, 0])

    def horizontal_diffusion_blocks(in_field: F64, out_field: F64, coeff: F64):
        with computation(PARALLEL), interval(...):
            lap = 4.0 * in_field[0, 0, 0] - (
                in_field[1, 0, 0] + in_field[-1, 0, 0] + in_field[0, 1, 0] + in_field[0, -1, 0]
            )
        with computation(PARALLEL), interval(...):
            res = lap[1, 0, 0] - lap[0, 0, 0]
            flx = 0 if (res * (in_field[1, 0, 0] - in_field[0, 0, 0])) > 0 else res
            res_j = lap[0, 1, 0] - lap[0, 0, 0]
            fly = 0 if (res_j * (in_field[0, 1, 0] - in_field[0, 0, 0])) > 0 else res_j
        with computation(PARALLEL), interval(...):
            out_field = in_field[0, 0, 0] - coeff[0, 0, 0] * (
                flx[0, 0, 0] - flx[-1, 0, 0] + fly[0, 0, 0] - fly[0, -1, 0]
            )

    def make_staged(dtype):
        FT = Field[dtype]

        def staged_forward_ij_temp(a: FT, out: FT):
            # tests/stencil_cases.py staged_forward_ij_temp (golden-pinned)
            with computation(FORWARD):
                with interval(0, 1):
                    s = a
                with interval(1, None):
                    s = s[0, 0, -1] * 0.5 + a
            with computation(FORWARD), interval(...):
                t = s * 2.0 + a
                out = t[1, 0, 0] - t[-1, 0, 0] + t[0, 1, 0] * s

        return staged_forward_ij_temp

    return {
        ("staged_forward_ij_temp", np.float64): make_staged(np.float64),
        ("staged_forward_ij_temp", np.float32): make_staged(np.float32),
        ("horizontal_diffusion_blocks", np.float64): horizontal_diffusion_blocks,
        ("vertical_advection_dycore", np.float64): vertical_advection_dycore,
        ("horizontal_diffusion", np.float64): make_hdiff(np.float64),
        ("horizontal_diffusion", np.float32): make_hdiff(np.float32),
        ("lap5", np.float64): lap5,
        ("copy_stencil", np.float64): copy_stencil,
        ("tridiagonal_solver", np.float64): tridiagonal_solver,
    }




# ------------------------------------------------------------------------------------------
# CPU baseline (BASELINE.md "CPU-baseline plan"): the C restatement of the stencil
# (cpu_ifirst-equivalent, I-first layout, OpenMP over (K, J) rows) on the full domain of the
# config, median of 20 calls after 3 warm-ups, OMP_PROC_BIND=close / OMP_PLACES=cores. It runs
# in a child process started after the GPU work so that the OpenMP placement variables are in
# its environment before libgomp loads.
# ------------------------------------------------------------------------------------------


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _physical_cores(cpus) -> int:
    """Distinct (package, core) pairs among ``cpus`` (sysfs topology; SMT siblings count once)."""
    seen = set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            with open(base + "physical_package_id") as f:
                pkg = f.read().strip()
            with open(base + "core_id") as f:
                core = f.read().strip()
        except OSError:
            return len(list(cpus))
        seen.add((pkg, core))
    return len(seen)


def _demo_field(ni, nj, nk, dtype):
    """The demo analytic field in=5+8*(2+cos(pi(x+1.5y))+sin(2pi(x+1.5y)))/4,
    constant in K, I-first (Fortran-ordered) host array."""
    x = np.arange(ni, dtype=np.float64)[:, None] / ni
    y = np.arange(nj, dtype=np.float64)[None, :] / nj
    t = x + 1.5 * y
    plane = (5.0 + 8.0 * (2.0 + np.cos(np.pi * t) + np.sin(2 * np.pi * t)) / 4.0).astype(dtype)
    arr = np.empty((ni, nj, nk), dtype=dtype, order="F")
    arr[...] = plane[:, :, None]
    return arr


def cpu_child(cfg_name: str, reps: int, warm: int, domain=None) -> dict:
    """Body of the ``--cpu-child`` process: time the C oracle on the config's full domain
    (``domain`` overrides it only for the CPU rehearsal of the dry run)."""
    from oracle import c_oracle

    sname, dtype, (ni, nj, nk), h, bpc = CONFIGS[cfg_name]
    if domain is not None:
        ni, nj, nk = domain
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    rng = np.random.default_rng(1337)

    def uni(shape, lo, hi):
        a = np.empty(shape, dtype=dtype, order="F")
        for k in range(shape[2]):  # plane by plane: bounded temporaries
            a[:, :, k] = rng.uniform(lo, hi, shape[:2])
        return a

    second = None
    if sname == "horizontal_diffusion":
        # the GPU's field distributions (in U(-10,10), coeff U(0,0.5), bench Workload): the
        # limiter branches are data-dependent, so the headline CPU figure uses the same mix
        a = uni((ni + 2 * h, nj + 2 * h, nk), -10, 10)
        c = uni((ni, nj, nk), 0.0, 0.5)
        o = np.zeros((ni, nj, nk), dtype=dtype, order="F")
        org = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
        fn = lambda: c_oracle.horizontal_diffusion(a, o, c, org, (ni, nj, nk), nthreads=threads)  # noqa: E731
        inputs = "in_field U(-10,10), coeff U(0,0.5), seed 1337 (the GPU's distributions)"
        a_demo = _demo_field(ni + 2 * h, nj + 2 * h, nk, dtype)
        c_demo = np.full((ni, nj, nk), 0.025, dtype=dtype, order="F")
        second = ("demo analytic in_field, coeff 0.025",
                  lambda: c_oracle.horizontal_diffusion(a_demo, o, c_demo, org, (ni, nj, nk), nthreads=threads))
    elif sname == "lap5":
        a = uni((ni + 2, nj + 2, nk), -10, 10)
        o = np.zeros((ni, nj, nk), order="F")
        fn = lambda: c_oracle.lap5(a, o, {"in_field": (1, 1, 0), "out_field": (0, 0, 0)}, (ni, nj, nk), threads)  # noqa: E731
        inputs = "U(-10,10) seed 1337"
    elif sname == "tridiagonal_solver":
        arrs = [uni((ni, nj, nk), lo, hi) for lo, hi in ((-1, 1), (4, 5), (-1, 1), (-10, 10), (0, 0))]
        org = {k: (0, 0, 0) for k in ("inf", "diag", "sup", "rhs", "out")}
        fn = lambda: c_oracle.tridiagonal_solver(*arrs, org, (ni, nj, nk), nthreads=threads)  # noqa: E731
        inputs = "diag 4+U[0,1), inf/sup U[-1,1), rhs U[-10,10), seed 1337"
    elif sname == "copy_stencil":
        a = uni((ni, nj, nk), -10, 10)
        o = np.zeros_like(a, order="F")
        fn = lambda: c_oracle.copy_stencil(a, o, {"field_a": (0, 0, 0), "field_b": (0, 0, 0)}, (ni, nj, nk), threads)  # noqa: E731
        inputs = "U(-10,10) seed 1337"
    else:
        return {}

    spent = [0.0]

    def median_s(f):
        for _ in range(warm):
            f()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t0)
        spent[0] += sum(ts)
        return float(np.median(ts))

    med = median_s(fn)
    timed_s = spent[0]
    cells = ni * nj * nk
    affinity = int(os.environ.get("GTMI_PARENT_AFFINITY", "0")) or None
    rec = {
        "value": round(cells / med / 1e6, 2),
        "unit": "Mcells/s",
        "cores": threads,
        "affinity_cpus": affinity,
        "physical_cores_in_affinity": int(os.environ.get("GTMI_PHYS_CORES", "0")) or None,
        "inherited_OMP_NUM_THREADS": os.environ.get("GTMI_INHERITED_OMP"),
        "threads_policy": "the GPU pool's per-GPU CPU share (inherited OMP_NUM_THREADS; the host is shared by "
                          "8 GPUs' jobs); not every physical core of the host",
        "os_cpu_count": os.cpu_count(),
        "kind": "port",
        "ms_per_call": round(med * 1e3, 3),
        "timed_s": round(timed_s, 2),
        "cpu_model": _cpu_model(),
        "sample": (f"cpu_ifirst-equivalent (own C++/OpenMP restatement, oracle/cpu_stencils.c) on the full "
                   f"{ni}x{nj}x{nk} {np.dtype(dtype).name} domain ({inputs}); median of {reps} calls after {warm} "
                   f"warm-ups; {threads} OpenMP threads on the {affinity} CPUs of the bench process's affinity set, "
                   f"OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND')}, OMP_PLACES={os.environ.get('OMP_PLACES')}"),
    }
    if second is not None:
        med2 = median_s(second[1])
        rec["second_input"] = {"inputs": second[0], "value": round(cells / med2 / 1e6, 2), "unit": "Mcells/s",
                               "ms_per_call": round(med2 * 1e3, 3)}
    if domain is not None:
        rec["dry_run_domain"] = list(domain)
    if sname == "horizontal_diffusion" and threads > 1 and domain is None:
        # thread scaling of the same code on a K-slab sample: the pool's rules
        # cap a one-GPU job at its CPU share, so the all-core figure is not run; the curve up to the
        # share says how the figure grows with cores
        ks = min(nk, 16)
        curve = []
        for t in sorted({1, 2, 4, 8, threads} & set(range(1, threads + 1))):
            f = lambda t=t: c_oracle.horizontal_diffusion(a, o, c, org, (ni, nj, ks), nthreads=t)  # noqa: E731
            for _ in range(1):
                f()
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                f()
                ts.append(time.perf_counter() - t0)
            curve.append({"threads": t, "Mcells_s": round(ni * nj * ks / float(np.median(ts)) / 1e6, 2)})
        rec["thread_scaling"] = {"sample": f"{ni}x{nj}x{ks} slab of the same inputs, median of 5 calls", "curve": curve}
    return rec


def cpu_baseline(cfg_name: str, reps: int = 40, warm: int = 3, timeout_s: float = 240.0, domain=None):
    """Run ``cpu_child`` in a child process (fresh OpenMP runtime with the placement variables)."""
    import subprocess

    env = dict(os.environ)
    # this (unbound) process's CPU set: the child's own affinity is a single core once libgomp has
    # bound its master thread, and more threads than CPUs would only oversubscribe
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cpus = list(range(os.cpu_count() or 1))
    ncpu = len(cpus)
    # Thread count: the CPU share the GPU pool gives one GPU's job (OMP_NUM_THREADS, 16 per GPU on
    # the MI355X boxes, whose hosts are shared by 8 GPUs' jobs; the pool asks GPU jobs to size
    # thread pools to it and not to raise it). SURVEY.md §8(d) would use every physical core of
    # the host; that count is recorded next to the figure, not used.
    inherited = env.get("OMP_NUM_THREADS")
    threads = min(int(inherited or ncpu), ncpu)
    env["OMP_NUM_THREADS"] = str(threads)
    env["GTMI_PARENT_AFFINITY"] = str(ncpu)
    env["GTMI_INHERITED_OMP"] = str(inherited)
    env["GTMI_PHYS_CORES"] = str(_physical_cores(cpus))
    env["OMP_PROC_BIND"] = "close"
    env["OMP_PLACES"] = "cores"
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-child", cfg_name, "--cpu-reps", str(reps),
           "--cpu-warm", str(warm)]
    if domain is not None:
        cmd += ["--cpu-domain", "x".join(str(int(n)) for n in domain)]
    try:
        res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"error": f"cpu baseline timed out after {timeout_s:.0f} s"}
    for line in reversed(res.stdout.splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return {"error": f"cpu baseline child failed (rc {res.returncode}): {res.stderr[-400:]}"}


# ------------------------------------------------------------------------------------------
# Box state (record which state a box is in). sysfs of the card this process uses:
# identity, DPM clock levels, power and its cap, VRAM already in use before our allocations.
# ------------------------------------------------------------------------------------------


def _read_text(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def find_card(pci_bus_id: str):
    """sysfs device directory of the GPU with this PCI bus id (``dddd:bb:dd.f``)."""
    import glob

    want = pci_bus_id.lower()
    for d in sorted(glob.glob("/sys/class/drm/card*/device")):
        for line in (_read_text(os.path.join(d, "uevent")) or "").splitlines():
            if line.startswith("PCI_SLOT_NAME=") and line.split("=", 1)[1].lower() == want:
                return d
    return None


def _dpm_current(text):
    for line in (text or "").splitlines():
        if line.rstrip().endswith("*"):
            return line.split(":", 1)[-1].replace("*", "").strip()
    return None


def card_snapshot(card):
    """Current DPM levels, power, temperatures and busy counters of the card (sysfs)."""
    import glob

    if card is None:
        return {}
    s = {clk: _dpm_current(_read_text(os.path.join(card, f"pp_dpm_{clk}"))) for clk in ("sclk", "mclk", "fclk", "socclk")}
    s["gpu_busy"] = _read_text(os.path.join(card, "gpu_busy_percent"))
    s["vram_used"] = _read_text(os.path.join(card, "mem_info_vram_used"))
    hw = sorted(glob.glob(os.path.join(card, "hwmon", "hwmon*")))
    if hw:
        for name in ("power1_input", "power1_average", "power1_cap", "temp1_input", "temp2_input", "temp3_input"):
            v = _read_text(os.path.join(hw[0], name))
            if v is not None:
                s[name] = v
    return s


def box_identity(dev_index: int = 0):
    """(card sysfs dir, identity dict) of the device this process runs on."""
    import torch

    p = torch.cuda.get_device_properties(dev_index)
    pci = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    card = find_card(pci)
    ident = {"pci": pci, "name": p.name, "uuid": str(p.uuid), "cus": p.multi_processor_count}
    if card is not None:
        for name in ("product_name", "serial_number", "unique_id", "vbios_version"):
            v = _read_text(os.path.join(card, name))
            if v is not None:
                ident[name] = v
        ident["mclk_levels"] = (_read_text(os.path.join(card, "pp_dpm_mclk")) or "").replace("\n", "; ")
    return card, ident


# ------------------------------------------------------------------------------------------
# Workloads
# ------------------------------------------------------------------------------------------


# placement tuning scope per config (--placement-scope auto): the column kernels (one wave per SIMD,
# latency-bound on every stream they read) re-home all their fields, the plane and tile kernels
# the written ones (DESIGN.md §5 "the column kernels have placement modes too")
PLACEMENT_SCOPE = {"tridiag": "all", "vadv": "all"}


def placement_scope(cfg, args) -> str:
    scope = getattr(args, "placement_scope", "auto")
    return PLACEMENT_SCOPE.get(cfg, "written") if scope == "auto" else scope


def hbm_estimate(stencil, args, candidates, scope="written") -> dict:
    """Peak device memory of one rank for this config (bytes, from the allocated fields): the
    fields themselves, and the placement tuner's transient copies of the fields the stencil writes
    (a backup plus ``candidates`` buffer sets, each padded by 2 MiB; the tuner itself caps the sets
    at 80 % of free memory); the halo path's pack buffers are faces, negligible. DESIGN.md §6."""
    from gt4py_amd.storage.placement import scope_fields

    def nbytes(t):
        try:
            return t.untyped_storage().nbytes()
        except AttributeError:  # dry run on host arrays
            return getattr(t, "nbytes", 0)

    names = list(stencil.field_info)
    fields = sum(nbytes(t) for t in args)
    tuned = set(scope_fields(stencil, scope))
    per_set = sum(nbytes(t) + (2 << 20) for n, t in zip(names, args) if n in tuned)
    tuner = (1 + candidates) * per_set if candidates > 0 else 0
    return {"fields_gb": round(fields / 1e9, 6), "tuner_transient_gb": round(tuner / 1e9, 6),
            "peak_gb": round((fields + tuner) / 1e9, 6)}


class Workload:
    """One config's fields, stencil and step function on this rank."""

    def __init__(self, cfg, args, rank, world, dev, backend, dry_run=False):
        import torch

        from gt4py_amd import gtscript, storage
        from gt4py_amd.distributed import Decomposition2D, HaloStencil, HaloStencil2D

        self.cfg = cfg
        self.dev = dev
        sname, dtype, (ni, nj, nk), h, bpc = CONFIGS[cfg]
        if dry_run:  # CPU rehearsal of the launcher / rendezvous / halo path: a small tile per rank
            ni, nj, nk = 64, 32, 8
        self.sname, self.dtype, self.h, self.bpc = sname, dtype, h, bpc
        self.global_ij = (ni, nj * world)  # weak scaling: the per-GPU tile is fixed
        self.dec2d = None
        if world > 1 and args.decomp == "2d":
            # the most square process grid pi x pj (pi <= pj: 1x2, 2x2, 2x4) of whole per-GPU
            # tiles, so the global domain grows along both axes and every rank has four neighbours
            # once pi, pj >= 2 (a J-only growth would make the least-perimeter grid a 1 x N strip)
            pi = max(p for p in range(1, int(world ** 0.5) + 1) if world % p == 0)
            pj = world // pi
            self.global_ij = (ni * pi, nj * pj)
            self.dec2d = Decomposition2D(self.global_ij[0], self.global_ij[1], pi, pj, (False, False))
            ni, nj = self.dec2d.local_shape(rank)
        self.domain = (ni, nj, nk)
        opts = {} if dry_run else {"device_sync": False}
        if args.jchunk and not dry_run:
            opts["jchunk"] = args.jchunk
        if not dry_run:
            for kv in args.opt or []:  # codegen options (A/B in separate processes: identical placement)
                k, v = kv.split("=", 1)
                opts[k] = int(v) if v.lstrip("-").isdigit() else v
        self.stencil = gtscript.stencil(backend=backend, definition=stencil_defs()[(sname, dtype)],
                                        name=f"bench.{cfg}", externals=EXTERNALS.get(sname, {}), **opts)
        tdt = storage.torch_dtype(dtype)
        gen = torch.Generator(device=dev)
        gen.manual_seed(1337 + rank)

        def alloc(shape, aligned):
            if dry_run:  # the numpy backend's own layout, as a torch CPU tensor (the halo path uses torch ops)
                return torch.from_numpy(storage.empty(shape, dtype, backend=backend, aligned_index=aligned))
            return storage.empty(shape, dtype, backend=backend, aligned_index=aligned)

        def uniform(shape, lo, hi, aligned=(0, 0, 0)):
            t = alloc(shape, aligned)
            if getattr(args, "fill", "bulk") == "bulk":
                t.copy_(torch.rand(shape, generator=gen, device=dev, dtype=tdt) * (hi - lo) + lo)
                return t
            # filled one K slab at a time: no field-sized temporaries, so the caching allocator
            # holds only the fields themselves (their HBM placement does not depend on freed
            # temporaries)
            for k0 in range(0, shape[2], 16):
                k1 = min(shape[2], k0 + 16)
                sub = (shape[0], shape[1], k1 - k0)
                t[:, :, k0:k1].copy_(torch.rand(sub, generator=gen, device=dev, dtype=tdt) * (hi - lo) + lo)
            return t

        def zeros(shape):
            t = alloc(shape, (0, 0, 0))
            t.zero_()
            return t

        self.halo = None
        self.named = None
        self.params = {}
        if sname in ("horizontal_diffusion", "horizontal_diffusion_blocks", "lap5"):
            fin = uniform((ni + 2 * h, nj + 2 * h, nk), -10, 10, (h, h, 0))
            out = zeros((ni, nj, nk))
            self.named = {"in_field": fin, "out_field": out}
            self.origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0)}
            if sname != "lap5":
                self.named["coeff"] = uniform((ni, nj, nk), 0.0, 0.5)
                self.origin["coeff"] = (0, 0, 0)
            self.args = tuple(self.named.values())
            overlap = not args.no_overlap
            if self.dec2d is not None:
                # 2-D tile: two-phase (corner-correct) exchange on the halo stream, interior overlapped
                self.halo = HaloStencil2D(self.stencil, ["in_field"], self.dec2d, rank, (h, h), overlap=overlap)
            elif world > 1:
                # J strip of the global domain: the in_field halo moves over RCCL while the interior computes
                self.halo = HaloStencil(self.stencil, ["in_field"], nj, h, rank, world, overlap=overlap)
            elif args.halo_selfcomm and args.decomp == "2d":
                # one 1x1 tile, periodic in I and J: both exchange phases go through RCCL to itself
                dec = Decomposition2D(ni, nj, 1, 1, (True, True))
                self.halo = HaloStencil2D(self.stencil, ["in_field"], dec, 0, (h, h), overlap=overlap,
                                          force_comm=True)
            elif args.halo_selfcomm:
                self.halo = HaloStencil(self.stencil, ["in_field"], nj, h, 0, 1, periodic=True, force_comm=True,
                                        overlap=overlap)
        elif sname == "staged_forward_ij_temp":
            self.args = (uniform((ni + 2 * h, nj + 2 * h, nk), -1, 1, (h, h, 0)), zeros((ni, nj, nk)))
            self.origin = {"a": (h, h, 0), "out": (0, 0, 0)}
        elif sname == "tridiagonal_solver":
            self.args = tuple(uniform((ni, nj, nk), lo, hi) for lo, hi in ((-1, 1), (4, 5), (-1, 1), (-10, 10), (0, 0)))
            self.origin = (0, 0, 0)
        elif sname == "vertical_advection_dycore":
            us, ust, upos, ut = (uniform((ni, nj, nk), -1, 1) for _ in range(4))
            wcon = uniform((ni + 1, nj, nk + 1), -1, 1)
            self.args = (us, ust, wcon, upos, ut)
            self.params = {"dtr_stage": 3.0 / 20.0}
            self.origin = (0, 0, 0)
        else:
            self.args = (uniform((ni, nj, nk), -10, 10), zeros((ni, nj, nk)))
            self.origin = (0, 0, 0)
        # validate once (full argument checks), then every timed call skips validation
        self.stencil(*self.args, **self.params, origin=self.origin, domain=self.domain)
        self.placement = None
        self.untuned = None
        self.hbm_estimate = hbm_estimate(self.stencil, self.args, getattr(args, "placement_candidates", 0),
                                         placement_scope(cfg, args))
        ncand = getattr(args, "placement_candidates", 0)
        if not dry_run and ncand > 0:
            self.tune_placement(ncand, args)

    def tune_placement(self, candidates: int, args):
        """Re-home the fields this stencil writes to the fastest of ``candidates + 1`` buffer sets
        through the drop-in call, ``StencilObject.tune_placement`` (in place: the argument tensors
        stay the same objects; DESIGN.md §5 "HBM placement"): done once, before any timed step, as
        a long-running simulation would after allocating its fields. The first allocation's time is
        measured first exactly as the headline is (K steps, HIP events), so the line carries the
        untuned figure as well."""
        steps, warm = (args.steps, args.warmup) if self.cfg == args.config else (args.extra_steps, 3)
        el, km = time_workload(self, steps, warm, self.dev, None, step=self.plain_step)
        self.untuned = {"ms_per_step": el / steps * 1e3, "kernel_ms": km}
        try:
            self.placement = self.stencil.tune_placement(*self.args, **self.params, origin=self.origin,
                                                         scope=placement_scope(self.cfg, args),
                                                         domain=self.domain, candidates=candidates)
        except (ValueError, RuntimeError, TypeError) as e:
            # a refusal (e.g. a viewed or weakly referenced written field) leaves the first
            # allocation in place: the line then reports the untuned figure as the headline
            import torch

            torch.cuda.synchronize()
            self.placement = {"error": f"{type(e).__name__}: {e}"[:300], "in_place": False}

    def step(self):
        if self.halo is not None:
            self.halo(self.named, self.origin, self.domain)
        else:
            self.plain_step()

    def validated_step(self):
        """The reference's default call: full argument validation (cached per domain/origin
        signature, as the reference's ``_domain_origin_cache``) and synchronisation after the call."""
        self.stencil(*self.args, **self.params, origin=self.origin, domain=self.domain, validate_args=True)
        if self.dev.type == "cuda":
            import torch

            torch.cuda.synchronize()

    def plain_step(self):
        """One launch over the whole local domain, no exchange (the halo path's A/B reference)."""
        self.stencil(*self.args, **self.params, origin=self.origin, domain=self.domain, validate_args=False)

    def library_key(self):
        """Content key of the generated library (``.gt_cache/gt_mi355x/<key>/stencil.so``)."""
        compiled = getattr(getattr(self.stencil, "_gt_run_impl_", None), "compiled", None)
        if compiled is None:
            return None
        return os.path.basename(os.path.dirname(compiled.lib_path))


def time_workload(wl, steps, warmup, dev, dist=None, events=True, step=None):
    """W untimed warm-ups, then K steps bracketed by barrier + synchronize; returns (elapsed s,
    mean per-launch kernel ms from HIP events on the launch stream, or None)."""
    import torch

    cuda = dev.type == "cuda"
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    step = step or wl.step
    for _ in range(warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    evs = None
    if cuda and events:
        # events on torch's current stream: gtmi_stencil_run enqueues on that stream
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for s in range(steps):
        if evs is not None:
            evs[s][0].record()
        step()
        if evs is not None:
            evs[s][1].record()
    wl.enqueue_s = time.perf_counter() - t0  # host time to enqueue the K steps (before the final sync)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in evs])) if evs is not None else None
    return elapsed, kernel_ms


def traffic_for(cfg, key):
    """HBM bytes per launch from ``profiles/pmc_<cfg>.json`` -- only when that measurement was
    taken on the library this run executed (same build key); otherwise null plus the reason."""
    path = os.path.join(REPO, "profiles", f"pmc_{cfg}.json")
    if not os.path.exists(path):
        return None, "no pmc measurement for this config"
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None, "unreadable pmc record"
    if key is None or rec.get("build_key") != key:
        return None, f"pmc record is for library {rec.get('build_key')}, this run executed {key}"
    return rec.get("hbm_bytes_per_launch"), f"profiles/pmc_{cfg}.json (library {key})"


# N=1: configs that also get a cpu_ifirst-equivalent figure of their own in extra_configs
CPU_EXTRA_CONFIGS = ("lap5", "tridiag")
DRY_RUN_CPU_DOMAIN = (64, 32, 8)
EXTRA_CONFIGS = ("lap5", "tridiag", "hdiff_f32", "copy", "vadv", "hdiff_blocks", "staged")
C5_CONFIG = "hdiff_f32"  # BASELINE configs[4]: 8192x1024x160 f32 per GPU, J strips, RCCL halo


def sharded_leg(cfg, args, rank, world, dev, backend, dist) -> dict:
    """One more config through the N-rank path after the headline (same ranks, same process
    group): its own fields, halo exchange and timing (barrier + synchronize around K steps, max
    over ranks). A rank that cannot set the workload up (e.g. out of memory) makes every rank skip
    the leg together -- a flag is all-reduced first -- so no rank waits in a collective alone."""
    import torch

    tdev = dev if str(dist.get_backend()).lower() == "nccl" else "cpu"
    w, err = None, None
    try:
        w = Workload(cfg, args, rank, world, dev, backend, dry_run=args.dry_run)
    except Exception as e:  # noqa: BLE001 - reported in the line, the headline stays valid
        err = f"{type(e).__name__}: {e}"[:300]
    ok = torch.tensor([0 if w is None else 1], device=tdev, dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok[0]) == 0:
        return {"error": err or "the workload failed on another rank"}
    steps = args.extra_steps
    el, km = time_workload(w, steps, 3, dev, dist)
    t = torch.tensor([el, km or 0.0], device=tdev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el, km = float(t[0]), (float(t[1]) if km is not None else None)
    ni, nj, nk = w.domain
    gi, gj = w.global_ij
    rec = {
        "workload": f"{w.sname} {ni}x{nj}x{nk} {np.dtype(w.dtype).name} per GPU, "
                    f"{'J-strips' if w.dec2d is None else f'{w.dec2d.pi}x{w.dec2d.pj} tiles'} of a "
                    f"{gi}x{gj}x{nk} global domain, {halo_transport(dist)} halo {w.h}",
        "n_gpus": world,
        "global_domain": [gi, gj, nk],
        "steps": steps,
        "ms_per_step": round(el / steps * 1e3, 4),
        "step_ms": round(km, 4) if km is not None else None,
        "Mcells_s": round(gi * gj * nk * steps / el / 1e6, 1),
        "scaling": "weak",
        "note": "whole-job cells/s over all ranks (max-over-ranks time); the N=1 line's extra_configs entry "
                "of this config is the single-GPU reference for weak-scaling efficiency",
    }
    if w.placement is not None:
        rec["placement_untuned_ms"] = w.placement.get("untuned_ms")
        rec["placement_tuned_ms"] = w.placement.get("tuned_ms")
    del w
    if dev.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return rec


# ------------------------------------------------------------------------------------------
# Launcher: `bench.py --gpus N` without a torchrun environment starts the N ranks itself
# ------------------------------------------------------------------------------------------


class RankPhase:
    """Bounded set-up of an N-rank run: a daemon thread ends the rank with
    exit status 3 and its last phase on stderr if process-group set-up, the first collectives and
    the link probe have not completed within ``limit_s`` (``GTMI_DIST_SETUP_TIMEOUT``, default
    300 s) -- a rank stuck in a rendezvous or a first RCCL call then fails the launch with a
    reason instead of hanging it. Nothing is re-executed."""

    def __init__(self, rank: int, limit_s: float):
        import threading

        self.rank, self.limit, self.name, self.t0 = rank, limit_s, "start", time.time()
        self.history = []
        self._done = threading.Event()
        threading.Thread(target=self._watch, name="gtmi-rank-phase", daemon=True).start()

    def set(self, name: str) -> None:
        self.history.append((name, round(time.time() - self.t0, 3)))
        self.name = name

    def finish(self) -> None:
        self.set("setup done")
        self._done.set()

    def _watch(self) -> None:
        if not self._done.wait(self.limit):
            sys.stderr.write(f"bench.py rank {self.rank}: no progress past phase '{self.name}' after "
                             f"{self.limit:.0f} s (phases so far: {self.history}); exiting with status 3\n")
            sys.stderr.flush()
            os._exit(3)


def halo_transport(dist) -> str:
    """What moves the halos: RCCL (backend "nccl") or gloo through host memory (CPU rehearsals,
    ranks sharing one GPU)."""
    return "RCCL" if str(dist.get_backend()).lower() == "nccl" else "gloo (host-staged)"


def probe_peers(rank, world, dec2d, selfcomm=False):
    """The ranks this rank exchanges halos with: J-strip neighbours, or the (up to eight) 2-D
    neighbours incl. corners; itself for the one-GPU self-exchange."""
    if selfcomm and world == 1:
        return [0]
    if dec2d is None:
        return sorted({r for r in (rank - 1, rank + 1) if 0 <= r < world})
    ci, cj = dec2d.coords(rank)
    peers = {dec2d.rank_of(ci + di, cj + dj) for di in (-1, 0, 1) for dj in (-1, 0, 1) if (di, dj) != (0, 0)}
    return sorted(p for p in peers if p is not None and p != rank)


def link_probe(dist, dev, rank, peers, nbytes=10_485_760, reps=3) -> dict:
    """One face-sized message (10.5 MB, the C5 f32 tile's 2-row J face: 8192 x 2 x 160 x 4 B) to
    and from every peer in one ``batch_isend_irecv``, timed after a warm-up exchange: per-rank
    milliseconds and GB/s per link and direction, before the headline runs."""
    import torch

    tdev = dev if str(dist.get_backend()).lower() == "nccl" else torch.device("cpu")
    n = nbytes // 4
    send = {p: torch.full((n,), float(rank), dtype=torch.float32, device=tdev) for p in peers}
    recv = {p: torch.empty(n, dtype=torch.float32, device=tdev) for p in peers}

    def once():
        ops = [dist.P2POp(dist.isend, send[p], p) for p in peers] + [dist.P2POp(dist.irecv, recv[p], p) for p in peers]
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        if tdev.type == "cuda":
            torch.cuda.synchronize(tdev)

    once()  # connections and buffers are set up by the first exchange
    ok = all(float(recv[p][0]) == float(p) and float(recv[p][-1]) == float(p) for p in peers)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    sec = (time.perf_counter() - t0) / reps
    return {"rank": rank, "peers": peers, "bytes_per_message": n * 4, "ms": round(sec * 1e3, 4),
            "GBps_per_link_each_way": round(n * 4 / sec / 1e9, 2) if peers else None,
            "GBps_rank_total": round(2 * len(peers) * n * 4 / sec / 1e9, 2) if peers else None,
            "payload_ok": ok}


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args, argv) -> int:
    """Start ``args.gpus`` ranks with torch.distributed.run (one process per GPU) as a CHILD
    process -- this process never touches the GPU, so nothing here initialises HIP before the
    ranks exist -- and relay rank 0's single JSON line. Non-zero exit if any rank fails."""
    import subprocess

    n = args.gpus
    if not args.dry_run:
        import torch  # device_count() does not initialise HIP on this image

        ndev = torch.cuda.device_count()
        if ndev < n:
            print(f"bench.py: --gpus {n} but only {ndev} GPU(s) are visible", file=sys.stderr)
            return 2
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    if args.dry_run:
        env["GTMI_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    res = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith('{"metric"')]
    if res.returncode != 0 or len(lines) != 1:
        sys.stderr.write(res.stdout)
        print(f"bench.py: {n}-rank run failed (rc {res.returncode}, {len(lines)} result lines)", file=sys.stderr)
        return res.returncode or 1
    rec = json.loads(lines[0])
    if rec.get("n_gpus") != n:
        print(f"bench.py: ranks reported n_gpus={rec.get('n_gpus')}, expected {n}", file=sys.stderr)
        return 1
    print(lines[0], flush=True)
    return 0


# ------------------------------------------------------------------------------------------


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="hdiff", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="N=1: skip the extra_configs timings")
    ap.add_argument("--extra-steps", type=int, default=20)
    ap.add_argument("--sustain", type=float, default=3.0,
                    help="N=1: after the timed K steps, run the step for about this many seconds more and report "
                         "the steady-state ms/step as `sustained` (0 = off)")
    ap.add_argument("--jchunk", type=int, default=None)
    ap.add_argument("--placement-candidates", type=int, default=5,
                    help="before timing, place the fields the stencil writes in the fastest of this many other "
                         "buffer sets besides the first allocation (gt4py_amd.storage.placement; 0 = off, the "
                         "first allocation is timed)")
    ap.add_argument("--placement-scope", default="auto", choices=["auto", "written", "all"],
                    help="fields the placement tuner re-homes: auto (all fields for the column-kernel configs "
                         "tridiag and vadv, the written ones otherwise), written, or all")
    ap.add_argument("--opt", action="append", default=None, metavar="KEY=VALUE",
                    help="gt:mi355x codegen option for the headline config (repeatable)")
    ap.add_argument("--fill", default="bulk", choices=["slab", "bulk"],
                    help="synthetic fields filled with field-sized temporaries (default) or per K slab")
    ap.add_argument("--decomp", default="jstrips", choices=["jstrips", "2d"],
                    help="N>1: J strips (default) or a balanced 2-D process grid (corners exchanged)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: exchange first, then one kernel over the whole strip (no interior/boundary split)")
    ap.add_argument("--halo-selfcomm", action="store_true",
                    help="N=1 under torchrun: run the J-strip halo path with the rank as its own periodic "
                         "neighbour through RCCL (measures the per-rank cost of the exchange + split)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal: numpy backend, gloo, a 64x32x8 tile per rank (no GPU)")
    ap.add_argument("--cpu-child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-reps", type=int, default=40, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-warm", type=int, default=3, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-domain", default=None, help=argparse.SUPPRESS)
    argv = sys.argv[1:]
    args = ap.parse_args(argv)

    if args.cpu_child:
        dom = tuple(int(n) for n in args.cpu_domain.split("x")) if args.cpu_domain else None
        print(json.dumps(cpu_child(args.cpu_child, args.cpu_reps, args.cpu_warm, dom)), flush=True)
        return 0
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return launch(args, argv)
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2

    # exactly one JSON line on stdout: native libraries (RCCL's version banner, ...) write to fd 1,
    # so fd 1 is pointed at stderr for the whole run and the result goes to a saved copy of it
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dev = torch.device("cpu")
        backend = "numpy"
    else:
        if not torch.cuda.is_available():
            raise SystemExit("bench.py needs a ROCm GPU (use --dry-run for the CPU rehearsal)")
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local_rank % ndev)
        dev = torch.device("cuda", local_rank % ndev)
        backend = "gt:mi355x"
    dist = None
    probe = None
    if world > 1 or args.halo_selfcomm:
        from gt4py_amd.distributed import init_process_group

        phase = RankPhase(rank, float(os.environ.get("GTMI_DIST_SETUP_TIMEOUT", "300")))
        # nccl (= RCCL over xGMI) on a real node; GTMI_DIST_BACKEND=gloo rehearses N ranks.
        # Keep RCCL's version banner off stdout: rank 0 prints exactly one JSON line there.
        os.environ.setdefault("NCCL_DEBUG", "WARN")
        phase.set("init_process_group")
        init_process_group("gloo" if args.dry_run else os.environ.get("GTMI_DIST_BACKEND", "nccl"))
        import torch.distributed as dist

        assert dist.get_world_size() == world, (dist.get_world_size(), world)
        phase.set("first barrier")
        dist.barrier()
        phase.set("link probe")
        dec = None
        if world > 1 and args.decomp == "2d":
            from gt4py_amd.distributed import Decomposition2D

            pi = max(p for p in range(1, int(world ** 0.5) + 1) if world % p == 0)
            dec = Decomposition2D(pi, world // pi, pi, world // pi, (False, False))
        mine = link_probe(dist, dev, rank, probe_peers(rank, world, dec, args.halo_selfcomm))
        probe = [None] * world
        dist.all_gather_object(probe, mine)
        phase.finish()

    box = None
    if not args.dry_run:
        card, ident = box_identity(torch.cuda.current_device())
        box = {"identity": ident, "before": card_snapshot(card), "pid": os.getpid(),
               "process_uptime_s": round(time.time() - _START, 2)}
    wl = Workload(args.config, args, rank, world, dev, backend, dry_run=args.dry_run)
    elapsed, kernel_ms = time_workload(wl, args.steps, args.warmup, dev, dist)
    elapsed_rank = elapsed
    if dist is not None:
        tdev = dev if str(dist.get_backend()).lower() == "nccl" else "cpu"
        t = torch.tensor([elapsed, kernel_ms or 0.0], device=tdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), (float(t[1]) if kernel_ms is not None else None)
    dist_rec = None
    if dist is not None and world > 1:
        # the same ranks, the same buffers: one plain launch over the whole local tile with no
        # exchange, so the line says what the exchange costs per rank (max over ranks)
        el_p, km_p = time_workload(wl, args.steps, args.warmup, dev, dist, step=wl.plain_step)
        el_h2, _ = time_workload(wl, args.steps, args.warmup, dev, dist)  # halo path again, interleaved
        el_hb = min(elapsed_rank, el_h2)
        tdev = dev if str(dist.get_backend()).lower() == "nccl" else "cpu"
        mine = torch.tensor([el_p, km_p or 0.0, el_hb / el_p - 1.0], device=tdev, dtype=torch.float64)
        dist.all_reduce(mine, op=dist.ReduceOp.MAX)
        ranks = [None] * world
        me = {"rank": rank, "local_rank": local_rank, "host": os.uname().nodename}
        if dev.type == "cuda":
            p = torch.cuda.get_device_properties(dev)
            me.update(device=torch.cuda.current_device(), pci_bus_id=f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:"
                      f"{p.pci_device_id:02x}.0", name=p.name)
        dist.all_gather_object(ranks, me)
        try:
            rccl = ".".join(str(x) for x in torch.cuda.nccl.version()) if tdev is dev else None
        except Exception:  # noqa: BLE001
            rccl = None
        dist_rec = {
            "world_size": dist.get_world_size(),
            "backend": str(dist.get_backend()),
            "rccl_version": rccl,
            "ranks": ranks,
            "step_ms": round(kernel_ms, 4) if kernel_ms is not None else None,
            "plain_ms_per_step": round(float(mine[0]) / args.steps * 1e3, 4),
            "plain_kernel_ms": round(float(mine[1]), 4) if km_p is not None else None,
            "exchange_overhead": round(float(mine[2]), 4),
            "halo_schedule": wl.halo.schedule() if hasattr(getattr(wl, "halo", None), "schedule") else None,
            "note": "plain = one launch over the whole local tile on the same buffers, no exchange; "
                    "exchange_overhead = halo-path time / plain time - 1 per rank, max over ranks",
        }
    halo_ab = None
    if args.halo_selfcomm and world == 1:
        # A/B on the same buffers in the same process: whole-domain launch without exchange,
        # interleaved with a second halo-path measurement
        el_p, km_p = time_workload(wl, args.steps, args.warmup, dev, dist, step=wl.plain_step)
        el_h, _ = time_workload(wl, args.steps, args.warmup, dev, dist)
        enq = wl.enqueue_s
        halo_ab = {"plain_ms_per_step": round(el_p / args.steps * 1e3, 4), "plain_kernel_ms": round(km_p, 4),
                   "halo_host_enqueue_ms_per_step": round(enq / args.steps * 1e3, 4),
                   "halo_ms_per_step": round(min(elapsed, el_h) / args.steps * 1e3, 4),
                   "overhead": round(min(elapsed, el_h) / el_p - 1.0, 4),
                   "halo_schedule": wl.halo.schedule() if hasattr(getattr(wl, "halo", None), "schedule") else None}
    ni, nj, nk = wl.domain
    cells_per_step = ni * nj * nk
    total_cells = wl.global_ij[0] * wl.global_ij[1] * nk * args.steps
    value = total_cells / elapsed / 1e6
    key = None if args.dry_run else wl.library_key()
    if wl.halo is not None:
        # a halo step is interior + boundary strips + pack/unpack + RCCL: the single-launch pmc
        # record of the stencil does not describe it
        traffic, traffic_src = None, ("not measured for the halo step (interior + boundary strips + pack/unpack + "
                                      "RCCL); profiles/pmc_<config>.json describes one plain launch")
    elif args.dry_run:
        traffic, traffic_src = None, "dry run"
    else:
        traffic, traffic_src = traffic_for(args.config, key)
    kms = kernel_ms if kernel_ms else elapsed / args.steps * 1e3
    achieved_gbs = cells_per_step * wl.bpc / (kms * 1e-3) / 1e9
    dec2d = wl.dec2d
    result = {
        "metric": "Mcells/s + achieved HBM GB/s, horiz-diffusion 2048x2048x160 fp64, 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "Mcells/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {np.float64: "f64", np.float32: "f32"}[wl.dtype],
        "data": "synthetic (uniform random fields generated on device)",
        "config": {
            "workload": f"{wl.sname} {ni}x{nj}x{nk} {np.dtype(wl.dtype).name} per GPU"
            + (
                f", {'J-strips' if dec2d is None else f'{dec2d.pi}x{dec2d.pj} tiles'} of a "
                f"{wl.global_ij[0]}x{wl.global_ij[1]}x{nk} global domain, {halo_transport(dist)} halo {wl.h}"
                if world > 1
                else ""
            ),
            "stencil": wl.sname,
            "domain_per_gpu": [ni, nj, nk],
            "global_domain": [wl.global_ij[0], wl.global_ij[1], nk],
            "backend": backend,
            "parallelism": (f"ij-strips{world}" if dec2d is None else f"ij-tiles{dec2d.pi}x{dec2d.pj}")
            if world > 1
            else (f"single+halo-selfcomm{'-2d' if args.decomp == '2d' else ''}" if args.halo_selfcomm else "single"),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            # N=1: mean per-launch kernel time; with a halo path it is the HIP-event span of the
            # whole step (exchange + interior + strips), so it is named step_ms there
            ("kernel_ms" if wl.halo is None else "step_ms"): round(kernel_ms, 4) if kernel_ms is not None else None,
            "algorithmic_bytes_per_cell": wl.bpc,
            "library": key,
        },
    }
    if wl.untuned is not None:
        # the first allocation (what a plain `@gtscript.stencil` + storage allocation gives a
        # drop-in user without the opt-in tuner), timed the same way as the headline, K steps
        u_ms = wl.untuned["kernel_ms"] or wl.untuned["ms_per_step"]
        u_gbs = cells_per_step * wl.bpc / (u_ms * 1e-3) / 1e9
        result["roofline"].update(kernel_ms_untuned=round(u_ms, 4), achieved_untuned=round(u_gbs, 1),
                                  frac_untuned=round(u_gbs / HBM_PEAK_GBS, 4),
                                  untuned_ms_per_step=round(wl.untuned["ms_per_step"], 4),
                                  Mcells_s_untuned=round(cells_per_step / (wl.untuned["ms_per_step"] * 1e-3) / 1e6, 2),
                                  tuned_note="kernel_ms/frac: fields re-homed in place by the opt-in "
                                             "StencilObject.tune_placement (DESIGN.md §5); *_untuned: the first "
                                             "allocation, same K-step measurement")
    result["hbm_estimate"] = dict(wl.hbm_estimate, per_rank=True)
    if dist_rec is not None:
        result["dist"] = dist_rec
    if probe is not None:
        rates = [r["GBps_per_link_each_way"] for r in probe if r["GBps_per_link_each_way"]]
        result.setdefault("dist", {})["link_probe"] = {
            "note": "before the headline: one 10.5 MB message (the C5 f32 J face) to and from each halo peer in "
                    "one batch_isend_irecv, after a warm-up exchange; per rank",
            "ranks": probe, "min_GBps_per_link": min(rates) if rates else None,
            "all_payloads_ok": all(r["payload_ok"] for r in probe)}
    if halo_ab is not None:
        result["halo_ab"] = halo_ab
    if world == 1 and not args.dry_run and not args.halo_selfcomm and args.sustain > 0:
        # steady state over seconds rather than tens of milliseconds (clocks, HBM refresh, the
        # driver's utilisation sampler); the headline `value` stays the K-step measurement
        n_s = max(args.steps, int(args.sustain / max(elapsed / args.steps, 1e-6)))
        el_s, _ = time_workload(wl, n_s, 0, dev, None, events=False)
        ms_s = el_s / n_s * 1e3
        result["sustained"] = {"steps": n_s, "seconds": round(el_s, 2), "ms_per_step": round(ms_s, 4),
                               "Mcells_s": round(cells_per_step / (ms_s * 1e-3) / 1e6, 1),
                               "frac": round(cells_per_step * wl.bpc / (ms_s * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    if world == 1 and not args.dry_run and not args.halo_selfcomm:
        # full-call time: validate_args=True and a synchronize after every call,
        # i.e. host validation + launch + kernel + sync, as a plain reference-style call loop
        el_v, _ = time_workload(wl, args.steps, 1, dev, None, events=False, step=wl.validated_step)
        # overhead against the back-to-back step time measured right before (sustained, else the
        # K-step kernel time): what validation + launch + a synchronize per call add per call
        base_ms = result["sustained"]["ms_per_step"] if "sustained" in result else (kernel_ms or 0.0)
        result["full_call"] = {"validate_args": True, "sync_each_call": True,
                               "ms_per_call": round(el_v / args.steps * 1e3, 4),
                               "host_overhead_ms": round(el_v / args.steps * 1e3 - base_ms, 4),
                               "overhead_vs": "sustained.ms_per_step" if "sustained" in result else "kernel_ms"}
    if wl.placement is not None:
        # the written fields were placed by measurement before the timed steps: every buffer set's
        # kernel time (set 0 = the first allocation, i.e. the untuned time) and the one chosen
        result["placement"] = dict(wl.placement, note="the fields of `scope` (written ones, or all) in the fastest "
                                   "of the measured buffer sets (gt4py_amd.storage.placement, DESIGN.md §5); "
                                   "set 0 is the first allocation")
    if box is not None:
        box["after"] = card_snapshot(find_card(box["identity"]["pci"]))
        # the fields' virtual addresses modulo 2 MiB and 1 GiB (physical addresses are not visible
        # from user space; hipMalloc blocks are 2 MiB aligned)
        box["field_va_residues"] = {
            k: {"mod_2MiB": t.data_ptr() % (2 << 20), "mod_1GiB": t.data_ptr() % (1 << 30)}
            for k, t in (wl.named or {}).items()
        }
        result["box"] = box
    if args.dry_run:
        result["dry_run"] = True
        result["data"] = "synthetic; DRY RUN on CPU (numpy backend, gloo): not a measurement"
    del wl
    if world > 1 and not args.no_extra and args.config != C5_CONFIG:
        # BASELINE configs[4] (C5) at N>1: the f32 tile sharded the same way, in the same ranks
        result["extra_configs"] = {C5_CONFIG: sharded_leg(C5_CONFIG, args, rank, world, dev, backend, dist)}
    if world == 1 and not args.dry_run and not args.no_extra and not args.halo_selfcomm:
        # the other BASELINE configs, timed in the same process after the headline (C2, C4, the C5
        # per-GPU tile, copy, vadv): per-launch kernel time from HIP events, fraction of 8 TB/s
        extra = {}
        for cfg in EXTRA_CONFIGS:
            if cfg == args.config:
                continue
            try:
                w = Workload(cfg, args, 0, 1, dev, backend)
                el, kms_x = time_workload(w, args.extra_steps, 3, dev)
                n_i, n_j, n_k = w.domain
                gbs = n_i * n_j * n_k * w.bpc / (kms_x * 1e-3) / 1e9
                tr, _ = traffic_for(cfg, w.library_key())
                extra[cfg] = {
                    "workload": f"{w.sname} {n_i}x{n_j}x{n_k} {np.dtype(w.dtype).name}",
                    "ms": round(el / args.extra_steps * 1e3, 4),
                    "kernel_ms": round(kms_x, 4),
                    "Mcells_s": round(n_i * n_j * n_k / (kms_x * 1e-3) / 1e6, 1),
                    "achieved_GBs": round(gbs, 1),
                    "frac": round(gbs / HBM_PEAK_GBS, 4),
                    "algorithmic_bytes_per_cell": w.bpc,
                    "traffic": tr,
                    "library": w.library_key(),
                }
                if w.placement is not None:
                    extra[cfg]["placement"] = {k: w.placement.get(k) for k in ("scope", "candidates_ms", "chosen",
                                                                               "untuned_ms", "error") if k in w.placement}
                if w.untuned is not None and w.untuned["kernel_ms"]:
                    u_gbs = n_i * n_j * n_k * w.bpc / (w.untuned["kernel_ms"] * 1e-3) / 1e9
                    extra[cfg]["kernel_ms_untuned"] = round(w.untuned["kernel_ms"], 4)
                    extra[cfg]["frac_untuned"] = round(u_gbs / HBM_PEAK_GBS, 4)
                del w
            except Exception as e:  # noqa: BLE001 - one failing extra config must not hide the headline
                extra[cfg] = {"error": f"{type(e).__name__}: {e}"[:300]}
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        result["extra_configs"] = extra
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.dry_run:
        cb = cpu_baseline(args.config)
        if cb:
            result["cpu_baseline"] = cb
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.no_extra and not args.halo_selfcomm:
        # BASELINE configs[1] reads "1xMI355X vs gt:cpu_ifirst" (C2) and C4 is the hot path's
        # K sweep: the same C restatement, thread policy and input distributions beside their GPU
        # figures (the dry run rehearses the plumbing on a small domain)
        extra = result.setdefault("extra_configs", {})
        for cfg in CPU_EXTRA_CONFIGS:
            if cfg == args.config:
                continue
            if args.dry_run:
                cb = cpu_baseline(cfg, reps=3, warm=1, domain=DRY_RUN_CPU_DOMAIN)
            else:
                cb = cpu_baseline(cfg, reps=20)
            entry = extra.setdefault(cfg, {})
            entry["cpu_baseline"] = cb
            if "kernel_ms" in entry and cb.get("ms_per_call"):
                entry["gpu_vs_cpu"] = round(cb["ms_per_call"] / entry["kernel_ms"], 1)
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
