"""HIP-graph capture of stencil call sequences (launch-bound workloads).

A time step of a model is a fixed sequence of stencil calls on fixed storages. Eagerly, every
call costs ~10 µs of host work (argument extraction, the cached validation lookup, one
``gtmi_stencil_run`` enqueue) -- more than the kernels themselves on small domains. Capturing the
sequence once into a HIP graph (``torch.cuda.CUDAGraph`` = ``hipGraph`` on ROCm) makes a replay one
host call for the whole sequence. This is the MI355X-native replacement for a tracing compiler:
nothing is re-generated, the captured kernels are exactly the gt:mi355x kernels.

Rules (as for any stream capture): every stencil in the sequence must be built with
``device_sync=False``; storages, origins, domains and scalar arguments are frozen at capture time
(a replay re-reads the same device memory, so update field contents in place, not the objects);
the first eager call of each stencil (library load, scratch allocation) happens in a warm-up run
before capture.

    graph = StencilGraph(lambda: [hdiff(fin, out, coeff, origin=o, domain=d, validate_args=False)])
    for step in range(n):
        graph.replay()
"""

from __future__ import annotations

from typing import Callable, Optional


class StencilGraph:
    def __init__(self, fn: Callable[[], object], warmup: int = 1, stream=None):
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("StencilGraph needs a ROCm device")
        self.fn = fn
        # warm-up on a side stream: loads libraries, allocates scratch and packs arguments outside
        # the capture (the captured region must not allocate or synchronise)
        self.stream = stream if stream is not None else torch.cuda.Stream()
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            for _ in range(max(1, warmup)):
                fn()
        torch.cuda.current_stream().wait_stream(self.stream)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            fn()
        torch.cuda.synchronize()

    def replay(self, sync: bool = False) -> None:
        """Enqueue the captured sequence on the current stream's device (one host call)."""
        self.graph.replay()
        if sync:
            import torch

            torch.cuda.synchronize()


def capture(fn: Callable[[], object], warmup: int = 1) -> StencilGraph:
    return StencilGraph(fn, warmup=warmup)


__all__ = ["StencilGraph", "capture"]
