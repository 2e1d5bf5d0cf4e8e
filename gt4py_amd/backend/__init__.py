"""Backend registry (``gt4py.cartesian.backend`` equivalent)."""

from gt4py_amd.backend.base import REGISTRY, Backend, BaseBackend, from_name, register  # noqa: F401
from gt4py_amd.backend import numpy_backend  # noqa: F401  (registers "numpy")
from gt4py_amd.backend import mi355x_backend  # noqa: F401  (registers "gt:mi355x")

__all__ = ["REGISTRY", "Backend", "BaseBackend", "from_name", "register"]
