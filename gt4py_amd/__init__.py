"""gt4py_amd: an MI355X-native stencil execution backend (``gt:mi355x``) for GTScript stencils.

Public surface mirrors ``gt4py.cartesian`` (``gtscript``, ``backend`` registry,
``StencilObject``) and ``gt4py.storage`` (``gt4py_amd.storage``).
"""

__version__ = "0.1.0"

from gt4py_amd import gtscript  # noqa: F401,E402
from gt4py_amd import backend  # noqa: F401,E402  (registers backends)
from gt4py_amd import storage  # noqa: F401,E402
from gt4py_amd.stencil_object import FrozenStencil, StencilObject  # noqa: F401,E402
