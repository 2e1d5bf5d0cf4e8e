#!/usr/bin/env python3
"""Where does gt:mi355x differ from the numpy backend on a fuzz program?

    python scripts/debug_fuzz_seed.py SEED [JSON-OPTS]

Prints, per output field, the number of differing cells, their (i, j, k) ranges and the first
few values (GPU vs numpy)."""
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import test_fuzz  # noqa: E402

from gt4py_amd import gtscript, storage  # noqa: E402

seed = int(sys.argv[1])
opts = json.loads(sys.argv[2]) if len(sys.argv) > 2 else test_fuzz._opts(seed)
defn, src = test_fuzz._load(seed, tempfile.mkdtemp())
print(src)
ref = test_fuzz._run_numpy(defn, seed)
st = gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"fuzz.hip.{seed}", **opts)
ins, outs, origin = test_fuzz._inputs(seed)
dev = {k: storage.from_array(v, dtype=v.dtype, backend="gt:mi355x", aligned_index=(2, 2, 0)) for k, v in ins.items()}
dev.update({k: storage.from_array(v, dtype=v.dtype, backend="gt:mi355x") for k, v in outs.items()})
st(**dev, s=0.75, origin=origin, domain=test_fuzz._shape(seed))
for k in ("out1", "out2"):
    got, exp = storage.to_numpy(dev[k]), ref[k]
    bad = np.argwhere(~((got == exp) | (np.isnan(got) & np.isnan(exp))))
    print(f"{k}: {len(bad)} of {got.size} cells differ (opts {opts})")
    if len(bad):
        print("  i range", bad[:, 0].min(), bad[:, 0].max(), " j range", bad[:, 1].min(), bad[:, 1].max(),
              " k values", sorted(set(bad[:, 2].tolist())))
        for i, j, kk in bad[:8]:
            print(f"  ({i},{j},{kk}) gpu {got[i, j, kk]!r} numpy {exp[i, j, kk]!r} initial {outs[k][i, j, kk]!r}")
