#!/usr/bin/env python3
"""Benchmark of the gt:mi355x hot path (BASELINE.json metric).

Default workload (``--config hdiff``): ``horizontal_diffusion`` (lap + flux + limiter,
PARALLEL K) at 2048 x 2048 x 160 fp64 per GPU -- BASELINE.json configs[2], the config the
metric "Mcells/s + achieved HBM GB/s, horiz-diffusion 2048x2048x160 fp64, 1/2/4/8 GPU" is
quoted on. With N GPUs (``torch.distributed.run``, one process per GPU) the global domain is
2048 x (2048*N) x 160 cut into J strips (weak scaling); every step exchanges the 2-row J halo
of ``in_field`` with the neighbours over RCCL, then runs the stencil on the local strip.

One step = one stencil application over the whole (local) domain, inputs resident in HBM.
Timing: W untimed warmups, then K steps bracketed by barrier + synchronize; max over ranks.
``roofline`` = algorithmic bytes (24 B/cell: in + coeff read, out written)
per launch / mean launch time from HIP events on the launch stream. ``cpu_baseline`` = the
C oracle (cpu_ifirst-equivalent restatement, OpenMP) on a bounded K-slice of the same domain.
"""



import argparse
import json
import os
import sys
import time

import numpy as np

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

    return {
        ("vertical_advection_dycore", np.float64): vertical_advection_dycore,
        ("horizontal_diffusion", np.float64): make_hdiff(np.float64),
        ("horizontal_diffusion", np.float32): make_hdiff(np.float32),
        ("lap5", np.float64): lap5,
        ("copy_stencil", np.float64): copy_stencil,
        ("tridiagonal_solver", np.float64): tridiagonal_solver,
    }


def cpu_baseline(cfg_name, budget_s=10.0):
    """Time the C oracle (cpu_ifirst-equivalent, OpenMP) on a bounded K-slice sample."""
    from oracle import c_oracle

    sname, dtype, (ni, nj, nk), h, bpc = CONFIGS[cfg_name]
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    nk_s = max(2, min(nk, 16))
    rng = np.random.default_rng(1337)
    if sname == "horizontal_diffusion":
        a = np.asfortranarray(rng.uniform(-10, 10, (ni + 2 * h, nj + 2 * h, nk_s)).astype(dtype))
        c = np.asfortranarray(rng.uniform(0, 0.5, (ni, nj, nk_s)).astype(dtype))
        o = np.zeros((ni, nj, nk_s), dtype=dtype, order="F")
        org = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
        fn = lambda: c_oracle.horizontal_diffusion(a, o, c, org, (ni, nj, nk_s), nthreads=threads)  # noqa: E731
    elif sname == "lap5":
        a = np.asfortranarray(rng.uniform(-10, 10, (ni + 2, nj + 2, nk_s)))
        o = np.zeros((ni, nj, nk_s), order="F")
        fn = lambda: c_oracle.lap5(a, o, {"in_field": (1, 1, 0), "out_field": (0, 0, 0)}, (ni, nj, nk_s), threads)  # noqa: E731
    elif sname == "tridiagonal_solver":
        arrs = [np.asfortranarray(rng.uniform(lo, hi, (ni, nj, nk_s))) for lo, hi in ((-1, 1), (4, 5), (-1, 1), (-10, 10), (0, 0))]
        org = {k: (0, 0, 0) for k in ("inf", "diag", "sup", "rhs", "out")}
        fn = lambda: c_oracle.tridiagonal_solver(*arrs, org, (ni, nj, nk_s), nthreads=threads)  # noqa: E731
    elif sname == "copy_stencil":
        a = np.asfortranarray(rng.uniform(-10, 10, (ni, nj, nk_s)))
        o = np.zeros_like(a, order="F")
        fn = lambda: c_oracle.copy_stencil(a, o, {"field_a": (0, 0, 0), "field_b": (0, 0, 0)}, (ni, nj, nk_s), threads)  # noqa: E731
    else:
        return None  # no CPU restatement of this stencil in oracle/
    fn()  # warm-up
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or reps >= 5000:
            break
    cells = ni * nj * nk_s * reps
    return {
        "value": round(cells / el / 1e6, 2),
        "unit": "Mcells/s",
        "cores": threads,
        "kind": "port",
        "sample": f"C oracle (cpu_ifirst-equivalent, OpenMP) {ni}x{nj}x{nk_s} {np.dtype(dtype).name}, {reps} calls in {el:.1f} s",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="hdiff", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--jchunk", type=int, default=None)
    ap.add_argument("--decomp", default="jstrips", choices=["jstrips", "2d"],
                    help="N>1: J strips (default) or a balanced 2-D process grid (corners exchanged)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: exchange first, then one kernel over the whole strip (no interior/boundary split)")
    ap.add_argument("--halo-selfcomm", action="store_true",
                    help="N=1 under torchrun: run the J-strip halo path with the rank as its own periodic "
                         "neighbour through RCCL (measures the per-rank cost of the exchange + split)")
    args = ap.parse_args()

    # exactly one JSON line on stdout: native libraries (RCCL's version banner, ...) write to fd 1,
    # so fd 1 is pointed at stderr for the whole run and the result goes to a saved copy of it
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a ROCm GPU")
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local_rank % ndev)
    dev = torch.device("cuda", local_rank % ndev)
    dist = None
    if world > 1 or args.halo_selfcomm:
        from gt4py_amd.distributed import init_process_group

        # nccl (= RCCL over xGMI) on a real node; GTMI_DIST_BACKEND=gloo rehearses N ranks on one GPU.
        # Keep RCCL's version banner off stdout: rank 0 prints exactly one JSON line there.
        os.environ.setdefault("NCCL_DEBUG", "WARN")
        init_process_group(os.environ.get("GTMI_DIST_BACKEND", "nccl"))
        import torch.distributed as dist

    from gt4py_amd import gtscript, storage
    from gt4py_amd.distributed import Decomposition2D, HaloStencil, HaloStencil2D

    sname, dtype, (ni, nj, nk), h, bpc = CONFIGS[args.config]
    # weak scaling: the per-GPU tile is fixed, the global domain is ni x (nj * world)
    global_ij = (ni, nj * world)
    dec2d = None
    if world > 1 and args.decomp == "2d":
        dec2d = Decomposition2D.balanced(global_ij[0], global_ij[1], world)
        ni, nj = dec2d.local_shape(rank)
    defs = stencil_defs()
    opts = {"device_sync": False}
    if args.jchunk:
        opts["jchunk"] = args.jchunk
    externals = EXTERNALS.get(sname, {})
    stencil = gtscript.stencil(backend="gt:mi355x", definition=defs[(sname, dtype)], name=f"bench.{args.config}",
                               externals=externals, **opts)

    be = "gt:mi355x"
    tdt = storage.torch_dtype(dtype)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1337 + rank)

    def uniform(shape, lo, hi, aligned):
        t = storage.empty(shape, dtype, backend=be, aligned_index=aligned)
        t.copy_(torch.rand(shape, generator=gen, device=dev, dtype=tdt) * (hi - lo) + lo)
        return t

    halo = None
    call_params = {}
    if sname == "horizontal_diffusion" or sname == "lap5":
        fin = uniform((ni + 2 * h, nj + 2 * h, nk), -10, 10, (h, h, 0))
        out = storage.zeros((ni, nj, nk), dtype, backend=be)
        if sname == "horizontal_diffusion":
            coeff = uniform((ni, nj, nk), 0.0, 0.5, (0, 0, 0))
            call_args = (fin, out, coeff)
            named = {"in_field": fin, "out_field": out, "coeff": coeff}
            origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
        else:
            call_args = (fin, out)
            named = {"in_field": fin, "out_field": out}
            origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0)}
        if dec2d is not None:
            # 2-D tile: two-phase (corner-correct) exchange on the halo stream, interior overlapped
            halo = HaloStencil2D(stencil, ["in_field"], dec2d, rank, (h, h), overlap=not args.no_overlap)
        elif world > 1:
            # J-strip of the global domain: exchange the in_field halo with the neighbours over
            # RCCL while the interior rows compute, then the two boundary strips
            halo = HaloStencil(stencil, ["in_field"], nj, h, rank, world, overlap=not args.no_overlap)
        elif args.halo_selfcomm:
            halo = HaloStencil(stencil, ["in_field"], nj, h, 0, 1, periodic=True, force_comm=True,
                               overlap=not args.no_overlap)
    elif sname == "tridiagonal_solver":
        fields = [uniform((ni, nj, nk), lo, hi, (0, 0, 0)) for lo, hi in ((-1, 1), (4, 5), (-1, 1), (-10, 10), (0, 0))]
        call_args = tuple(fields)
        origin = (0, 0, 0)
    elif sname == "vertical_advection_dycore":
        us, ust, upos, ut = (uniform((ni, nj, nk), -1, 1, (0, 0, 0)) for _ in range(4))
        wcon = uniform((ni + 1, nj, nk + 1), -1, 1, (0, 0, 0))
        call_args = (us, ust, wcon, upos, ut)
        call_params = {"dtr_stage": 3.0 / 20.0}
        origin = (0, 0, 0)
    else:
        a = uniform((ni, nj, nk), -10, 10, (0, 0, 0))
        b = storage.zeros((ni, nj, nk), dtype, backend=be)
        call_args = (a, b)
        origin = (0, 0, 0)
    domain = (ni, nj, nk)

    def step(ev_pair=None):
        if ev_pair is not None:
            ev_pair[0].record()
        if halo is not None:
            halo(named, origin, domain)
        else:
            stencil(*call_args, **call_params, origin=origin, domain=domain, validate_args=False)
        if ev_pair is not None:
            ev_pair[1].record()

    # validate once (full checks), then warm up
    stencil(*call_args, **call_params, origin=origin, domain=domain)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(evs[s])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    if dist is not None:
        tdev = dev if str(dist.get_backend()).lower() == "nccl" else "cpu"
        t = torch.tensor([elapsed, kernel_ms], device=tdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])
    cells_per_step = ni * nj * nk
    total_cells = global_ij[0] * global_ij[1] * nk * args.steps
    value = total_cells / elapsed / 1e6
    achieved_gbs = cells_per_step * bpc / (kernel_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(REPO, "profiles", f"pmc_{args.config}.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
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
        "dtype": {np.float64: "f64", np.float32: "f32"}[dtype],
        "data": "synthetic (uniform random fields generated on device)",
        "config": {
            "workload": f"{sname} {ni}x{nj}x{nk} {np.dtype(dtype).name} per GPU"
            + (
                f", {'J-strips' if dec2d is None else f'{dec2d.pi}x{dec2d.pj} tiles'} of a "
                f"{global_ij[0]}x{global_ij[1]}x{nk} global domain, RCCL halo {h}"
                if world > 1
                else ""
            ),
            "stencil": sname,
            "domain_per_gpu": [ni, nj, nk],
            "global_domain": [global_ij[0], global_ij[1], nk],
            "backend": "gt:mi355x",
            "parallelism": (f"ij-strips{world}" if dec2d is None else f"ij-tiles{dec2d.pi}x{dec2d.pj}")
            if world > 1
            else ("single+halo-selfcomm" if args.halo_selfcomm else "single"),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel_ms": round(kernel_ms, 4),
            "algorithmic_bytes_per_cell": bpc,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(args.config, args.cpu_budget)
        if cb is not None:
            result["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
