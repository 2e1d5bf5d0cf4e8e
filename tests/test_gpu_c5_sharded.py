"""C5's sharded path end to end on one box (tests/c5_sharded_check.py): hdiff f32 J strips over
8 ranks that share the GPU (gloo moves the halos through host memory, as RCCL refuses two ranks on
one device), every rank's output bit-exact vs the C oracle on the same global input and every
exchanged halo row equal to its owner's row. The default size is small; the full C5 size
(8192 x 8192 x 160 over 8 ranks) runs the same script with ``--ni 8192 --nj 1024 --nk 160``
(``scripts/gpu_r06d.sh``, ``profiles/r06/r06d_c5_sharded_check.json``)."""

import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_c5_sharded_eight_ranks_vs_c_oracle():
    import stencil_cases as sc
    import torch

    from gt4py_amd import gtscript

    # the library the ranks load (built here first: the GPU box runs on prebuilt libraries)
    gtscript.stencil(backend="gt:mi355x", definition=sc.hdiff_f32, name="c5.sharded.hdiff_f32", device_sync=False)
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    env = dict(os.environ, GTMI_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "c5_sharded_check.py"),
           "--ni", "1024", "--nj", "96", "--nk", "24", "--kchunk", "8", "--steps", "2"]
    res = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    rec = json.loads([ln for ln in res.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["world_size"] == 8 and rec["global_domain"] == [1024, 768, 24]
    assert rec["mismatched_cells"] == 0 and rec["mismatched_halo_cells"] == 0
    assert rec["cells_checked"] == 1024 * 768 * 24
