#!/usr/bin/env python3
"""Print per-kernel VGPR/SGPR/LDS/occupancy of a bench config's generated library (hipcc remarks).

    python scripts/resource_usage.py hdiff [opt=value ...]
"""

import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench
    from gt4py_amd.runtime import jit

    cfg = sys.argv[1] if len(sys.argv) > 1 else "hdiff"
    opts = {}
    for kv in sys.argv[2:]:
        k, v = kv.split("=")
        opts[k] = int(v)
    sname, dtype, _, _, _ = bench.CONFIGS[cfg]
    from gt4py_amd.backend.base import from_name
    from gt4py_amd.backend.mi355x_backend import generate_source
    from gt4py_amd.definitions import BuildOptions
    from gt4py_amd.loader import StencilBuilder

    b = StencilBuilder(bench.stencil_defs()[(sname, dtype)], from_name("gt:mi355x"),
                       BuildOptions(name=f"resources.{cfg}", module="resources", backend_opts=opts),
                       bench.EXTERNALS.get(sname, {}), {})
    _, source, _ = generate_source(b.analysis, opts)  # the backend's own lowering chain
    lib = jit.compile_source(source)
    src = os.path.join(os.path.dirname(lib), "stencil.hip")
    cmd = [jit.hipcc_path()] + jit.BASE_FLAGS + [f"-I{jit.CSRC_DIR}", f"-I{jit.INCLUDE_DIR}",
                                                 "-Rpass-analysis=kernel-resource-usage", "-o", "/dev/null", src]
    res = subprocess.run(cmd, capture_output=True, text=True)
    cur = None
    for line in res.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            print(f"\n{cur}")
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|TotalSGPRs|ScratchSize|Occupancy|LDS Size)[^:]*:\s*(\S+)", line)
        if m and cur:
            print(f"  {m.group(1)} = {m.group(2)}")


if __name__ == "__main__":
    main()
