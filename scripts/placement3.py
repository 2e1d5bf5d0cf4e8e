#!/usr/bin/env python3
"""Is the hdiff time bimodality a property of the physical backing of the field buffers?

Allocates several independent (in, out, coeff) sets three ways -- torch caching allocator,
plain hipMalloc, hipExtMallocWithFlags(hipDeviceMallocContiguous) -- keeps them all live and
times the same kernel on each set, interleaved, in one process.
"""

import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


class _DevBuf:
    """A raw device allocation exposed to torch through __cuda_array_interface__."""

    def __init__(self, hip, ptr, shape, strides_b):
        self.hip, self.ptr = hip, ptr
        self.__cuda_array_interface__ = {"shape": shape, "typestr": "<f8", "data": (ptr, False),
                                         "strides": strides_b, "version": 2}


def main():
    import torch

    import bench
    from gt4py_amd import gtscript

    nsets = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ni, nj, nk = 2048, 2048, 160
    st = gtscript.stencil(backend="gt:mi355x", definition=bench.stencil_defs()[("horizontal_diffusion", np.float64)],
                          name="placement3.hdiff", device_sync=False)
    if os.environ.get("BUILD_ONLY"):
        print("built")
        return
    dev = torch.device("cuda", 0)
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already loaded
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    base_in = torch.rand((ni + 4, nj + 4, nk), generator=g, device=dev, dtype=torch.float64) * 20 - 10
    base_co = torch.rand((ni, nj, nk), generator=g, device=dev, dtype=torch.float64) * 0.5
    pi_in = -(-(ni + 4) // 32) * 32
    keep = []

    def raw(kind, shape, pitch):
        n = pitch * shape[1] * shape[2]
        p = ctypes.c_void_p()
        rc = hip.hipMalloc(ctypes.byref(p), n * 8) if kind == "hipMalloc" else \
            hip.hipExtMallocWithFlags(ctypes.byref(p), n * 8, 0x4)
        if rc != 0:
            raise RuntimeError(f"{kind} failed rc={rc}")
        b = _DevBuf(hip, p.value, shape, (8, pitch * 8, pitch * shape[1] * 8))
        keep.append(b)
        return torch.as_tensor(b, device=dev)

    def make(kind):
        if kind == "torch":
            fin = torch.as_strided(torch.empty(pi_in * (nj + 4) * nk, dtype=torch.float64, device=dev),
                                   (ni + 4, nj + 4, nk), (1, pi_in, pi_in * (nj + 4)))
            co, out = (torch.as_strided(torch.empty(ni * nj * nk, dtype=torch.float64, device=dev),
                                        (ni, nj, nk), (1, ni, ni * nj)) for _ in range(2))
        else:
            fin = raw(kind, (ni + 4, nj + 4, nk), pi_in)
            co, out = raw(kind, (ni, nj, nk), ni), raw(kind, (ni, nj, nk), ni)
        fin.copy_(base_in)
        co.copy_(base_co)
        out.zero_()
        return fin, out, co

    sets = {}
    for s in range(nsets):
        for kind in ("torch", "hipMalloc", "contiguous"):
            try:
                sets[f"{kind}#{s}"] = make(kind)
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"alloc": f"{kind}#{s}", "error": str(e)}), flush=True)
    origin = {"in_field": (2, 2, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    for a in sets.values():
        st(*a, origin=origin, domain=(ni, nj, nk))
    torch.cuda.synchronize()
    ref = next(iter(sets.values()))[1]
    for n, a in sets.items():
        assert torch.equal(a[1], ref), n
    times = {n: [] for n in sets}
    for r in range(4):
        for n, a in sets.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                st(*a, origin=origin, domain=(ni, nj, nk), validate_args=False)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 10)
    for n, t in times.items():
        a = sets[n]
        med = float(np.median(t))
        print(json.dumps({"alloc": n, "ptrs": [hex(x.data_ptr()) for x in a], "median_ms": round(med, 4),
                          "min_ms": round(min(t), 4), "GBps": round(ni * nj * nk * 24 / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
