"""Multi-GPU execution: IJ decomposition (J strips or a 2-D process grid) + RCCL halo exchange,
one process per GPU."""

from gt4py_amd.distributed.decomp2d import Decomposition2D, HaloExchange2D, HaloStencil2D  # noqa: F401
from gt4py_amd.distributed.halo import HaloStencil, JHaloExchange, JStrips, init_process_group  # noqa: F401
