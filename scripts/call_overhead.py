#!/usr/bin/env python3
"""Host cost of one gt:mi355x stencil call, layer by layer (tiny domain: launch-bound).

    python scripts/call_overhead.py [--calls 3000]

Prints one JSON line per layer: StencilObject.__call__ with validation, without, FrozenStencil,
the prepared launch they end in (native, and the same calls with the ctypes closure instead),
the launcher alone, and the bare ``gtmi_stencil_run`` ctypes call on pre-packed arguments.
``device_sync=False`` everywhere: the number is host time per enqueued call.
"""

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=3000)
    args = ap.parse_args()
    import torch

    import bench
    from gt4py_amd import gtscript, storage

    defs = bench.stencil_defs()
    st = gtscript.stencil(backend="gt:mi355x", definition=defs[("horizontal_diffusion", np.float64)],
                          name="overhead.hdiff", device_sync=False)
    ni, nj, nk, h = 32, 16, 4, 2
    fin = storage.from_array(np.random.default_rng(0).uniform(-1, 1, (ni + 2 * h, nj + 2 * h, nk)),
                             backend="gt:mi355x", aligned_index=(h, h, 0))
    out = storage.zeros((ni, nj, nk), np.float64, backend="gt:mi355x")
    coeff = storage.full((ni, nj, nk), 0.1, np.float64, backend="gt:mi355x")
    origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    dom = (ni, nj, nk)

    def timeit(fn, n, burst=64):
        # bursts short enough that the GPU queue never fills (a full queue makes the host wait on
        # the device and turns the number into kernel time); the device drains between bursts,
        # outside the clock; median over bursts
        for _ in range(50):
            fn()
        per = []
        for _ in range(max(1, n // burst)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(burst):
                fn()
            per.append((time.perf_counter() - t0) / burst * 1e6)
        torch.cuda.synchronize()
        per.sort()
        return per[len(per) // 2]

    class _Res(dict):
        def __setitem__(self, k, v):
            super().__setitem__(k, v)
            print(json.dumps({"layer": k, "us_per_call": round(v, 2)}), flush=True)

    res = _Res()
    # warm the host path (clocks, caches, the first-call entries) before any layer is timed
    for _ in range(3000):
        st(fin, out, coeff, origin=origin, domain=dom)
    torch.cuda.synchronize()
    res["call_validate"] = timeit(lambda: st(fin, out, coeff, origin=origin, domain=dom), args.calls)
    res["call_no_validate"] = timeit(
        lambda: st(fin, out, coeff, origin=origin, domain=dom, validate_args=False), args.calls)
    frozen = st.freeze(origin=origin, domain=dom)
    res["frozen"] = timeit(lambda: frozen(in_field=fin, out_field=out, coeff=coeff), args.calls)
    ((entry,),) = type(st)._gt_fast_memo_.values()  # one argument tuple, one (domain, origin) signature
    prepared = entry[2]  # what the cached __call__ ends in (native Prepared, or the ctypes closure)
    print(json.dumps({"prepared_kind": type(prepared).__name__}), flush=True)
    res["prepared_only"] = timeit(lambda: prepared((fin, out, coeff), ()), args.calls)
    from gt4py_amd.runtime import fastcall

    native = fastcall.module()
    if native is not None:  # the same layers with the launcher's ctypes closure instead
        fastcall._module = None
        st.clean_call_args_cache()
        res["call_validate_ctypes_closure"] = timeit(lambda: st(fin, out, coeff, origin=origin, domain=dom),
                                                     args.calls)
        frozen_c = st.freeze(origin=origin, domain=dom)
        res["frozen_ctypes_closure"] = timeit(lambda: frozen_c(in_field=fin, out_field=out, coeff=coeff), args.calls)
        fastcall._module = native
        st.clean_call_args_cache()
    comp = [c.cell_contents for c in type(st).run.__closure__][0].compiled
    launcher = comp.launcher
    arrays = {"in_field": fin, "out_field": out, "coeff": coeff}
    res["launcher"] = timeit(lambda: launcher(dom, origin, arrays, {}, device_sync=False), args.calls)
    # bare ctypes call on pre-packed structs
    lib = launcher.lib
    fields, _ = launcher.pack_fields(dom, origin, arrays)
    from gt4py_amd.runtime import ffi

    scal = (ffi.GtmiScalar * 1)()
    d3 = (ctypes.c_int64 * 3)(*dom)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res["ctypes_only"] = timeit(lambda: lib.run(d3, fields, launcher.n_fields, scal, 0, s), args.calls)
    # a captured HIP graph of 10 calls, per call
    from gt4py_amd.runtime.graph import StencilGraph

    def ten():
        for _ in range(10):
            st(fin, out, coeff, origin=origin, domain=dom, validate_args=False)

    g = StencilGraph(ten)
    res["graph_replay_per_call"] = timeit(g.replay, max(1, args.calls // 10), burst=8) / 10
    # GPU time of the tiny kernel itself, for scale
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        lib.run(d3, fields, launcher.n_fields, scal, 0, s)
    e1.record()
    torch.cuda.synchronize()
    res["gpu_us_per_launch_backtoback"] = e0.elapsed_time(e1) / 200 * 1e3

    # round trips (call + synchronize each time, the bench's full_call shape): the bare ctypes
    # launch sets the driver's floor (launch latency + kernel + completion wake-up); the
    # difference to the validated call is what the Python layers add
    def rt_ctypes():
        lib.run(d3, fields, launcher.n_fields, scal, 0, s)
        torch.cuda.synchronize()

    def rt_call():
        st(fin, out, coeff, origin=origin, domain=dom, validate_args=True)
        torch.cuda.synchronize()

    res["roundtrip_ctypes_sync"] = timeit(rt_ctypes, args.calls // 2)
    res["roundtrip_call_validate_sync"] = timeit(rt_call, args.calls // 2)


if __name__ == "__main__":
    main()
