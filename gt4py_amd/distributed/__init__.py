"""Multi-GPU execution: J-strip decomposition + RCCL halo exchange (one process per GPU)."""

from gt4py_amd.distributed.halo import HaloStencil, JHaloExchange, JStrips, init_process_group  # noqa: F401
