#!/usr/bin/env python3
"""Probe: I-offset reads of narrow (4-byte) fields in a plane kernel whose output is f64."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gt4py_amd import gtscript, storage  # noqa: E402
from gt4py_amd.gtscript import PARALLEL, Field, computation, interval  # noqa: E402


def p_i32_f64(m: Field[np.int32], out: Field[np.float64]):
    with computation(PARALLEL), interval(...):
        out = abs(m[0, 0, 0] - m[1, 0, 0]) + out


def p_i32_f64_noabs(m: Field[np.int32], out: Field[np.float64]):
    with computation(PARALLEL), interval(...):
        out = (m[0, 0, 0] - 2 * m[1, 0, 0]) + out


def p_f32_f64(m: Field[np.float32], out: Field[np.float64]):
    with computation(PARALLEL), interval(...):
        out = (m[0, 0, 0] - 2 * m[1, 0, 0]) + out


def p_i32_i32(m: Field[np.int32], out: Field[np.int32]):
    with computation(PARALLEL), interval(...):
        out = m[0, 0, 0] - 2 * m[1, 0, 0]


def p_i32_f64_jm1(m: Field[np.int32], out: Field[np.float64]):
    with computation(PARALLEL), interval(...):
        out = (m[0, -1, 0] - 2 * m[1, -1, 0]) + out


CASES = [p_i32_f64, p_i32_f64_noabs, p_f32_f64, p_i32_i32, p_i32_f64_jm1]


def build():
    return {f.__name__: (gtscript.stencil(backend="gt:mi355x", definition=f, name=f"probe.{f.__name__}"),
                         gtscript.stencil(backend="numpy", definition=f, name=f"probe.np.{f.__name__}")) for f in CASES}


if __name__ == "__main__":
    sts = build()
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        sys.exit(0)
    rng = np.random.default_rng(3)
    ni, nj, nk = 13, 11, 4
    for name, (g, n) in sts.items():
        mdt = np.float32 if "f32" in name.split("_")[1] else np.int32
        odt = np.int32 if name.endswith("i32_i32") else np.float64
        m = rng.integers(-5, 6, (ni + 4, nj + 4, nk)).astype(mdt)
        out = rng.uniform(-1, 1, (ni, nj, nk)).astype(odt) if odt == np.float64 else np.zeros((ni, nj, nk), odt)
        origin = {"m": (2, 2, 0), "out": (0, 0, 0)}
        ref = {"m": m.copy(), "out": out.copy()}
        n(**ref, origin=origin, domain=(ni, nj, nk))
        dev = {"m": storage.from_array(m, dtype=mdt, backend="gt:mi355x", aligned_index=(2, 2, 0)),
               "out": storage.from_array(out, dtype=odt, backend="gt:mi355x")}
        g(**dev, origin=origin, domain=(ni, nj, nk))
        got = storage.to_numpy(dev["out"])
        bad = np.argwhere(got != ref["out"])
        print(f"{name}: {len(bad)} of {got.size} differ; odd-i share {np.mean(bad[:, 0] % 2) if len(bad) else 0:.2f}")
        for i, j, k in bad[:3]:
            print(f"   ({i},{j},{k}) gpu {got[i, j, k]} numpy {ref['out'][i, j, k]}  m row: {m[i:i + 6, j + 2, k]}")
