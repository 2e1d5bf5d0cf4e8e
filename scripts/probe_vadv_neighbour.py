#!/usr/bin/env python3
"""Probe: what does vadv's I-neighbour stream (wcon[1, 0, *], an L2 hit, one extra load per
level) cost? Times vadv against the same program with wcon[1, 0, *] replaced by wcon[0, 0, *]
(a different stencil: same loads minus that stream, same arithmetic), interleaved in one process
on shared buffers. Measurement only; the second program's results are not checked.

    python scripts/probe_vadv_neighbour.py [--build-only]
"""
import inspect
import json
import os
import sys
import textwrap

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench
    from gt4py_amd import gtscript

    defn = bench.stencil_defs()[("vertical_advection_dycore", np.float64)]
    src = textwrap.dedent(inspect.getsource(defn)).replace("wcon[1, 0, 1]", "wcon[0, 0, 1]").replace(
        "wcon[1, 0, 0]", "wcon[0, 0, 0]")
    assert "wcon[1" not in src
    # the frontend reads the definition's source: give the variant a module file of its own
    import importlib.util
    import tempfile

    head = ("import numpy as np\nfrom gt4py_amd.gtscript import Field, computation, interval, PARALLEL, FORWARD, "
            "BACKWARD\nF64 = Field[np.float64]\n")
    d = tempfile.mkdtemp(prefix="probe_vadv_")
    path = os.path.join(d, "probe_vadv_variant.py")
    with open(path, "w") as f:
        f.write(head + src)
    spec = importlib.util.spec_from_file_location("probe_vadv_variant", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    nodef = mod.vertical_advection_dycore
    ext = bench.EXTERNALS["vertical_advection_dycore"]
    sts = [gtscript.stencil(backend="gt:mi355x", definition=d, name=f"probe.vadv.{i}", device_sync=False,
                            externals=ext) for i, d in enumerate((defn, nodef, defn, nodef))]
    if "--build-only" in sys.argv:
        print("built")
        return
    import torch

    from gt4py_amd import storage

    ni, nj, nk = 1024, 1024, 160
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)

    def uniform(shape):
        t = storage.empty(shape, np.float64, backend="gt:mi355x", aligned_index=(0, 0, 0))
        t.copy_(torch.rand(shape, generator=gen, device=dev, dtype=torch.float64) * 2 - 1)
        return t

    ins = [uniform((ni, nj, nk)) for _ in range(3)]
    wcon = uniform((ni + 1, nj, nk + 1))
    ust = storage.zeros((ni, nj, nk), np.float64, backend="gt:mi355x")
    args = (ust, ins[0], wcon, ins[1], ins[2])
    for st in sts:
        st(*args, dtr_stage=0.15, origin=(0, 0, 0), domain=(ni, nj, nk))
    torch.cuda.synchronize()
    times = [[] for _ in sts]
    for _ in range(6):
        for i, st in enumerate(sts):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                st(*args, dtr_stage=0.15, origin=(0, 0, 0), domain=(ni, nj, nk), validate_args=False)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / 10)
    for i, t in enumerate(times):
        print(json.dumps({"program": ["vadv", "no_neighbour"][i % 2], "median_ms": round(float(np.median(t)), 4)}))


if __name__ == "__main__":
    main()
