#!/usr/bin/env python3
"""One-GPU check of the RCCL point-to-point path the halo exchanges use.

A single rank (nccl backend = RCCL) sends device buffers to itself with
``dist.batch_isend_irecv`` -- the same call, buffer kinds and stream semantics as
``JHaloExchange``/``HaloExchange2D`` -- and checks the received bytes, with the compute stream
busy on a stencil meanwhile. Run under torchrun with one process:

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29541 scripts/rccl_selftest.py
"""

import json
import os
import sys


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import torch.distributed as dist

    from gt4py_amd.distributed import init_process_group

    rank, world = init_process_group("nccl")
    dev = torch.device("cuda", torch.cuda.current_device())
    face = torch.arange(2 * 2052 * 160, dtype=torch.float64, device=dev).reshape(2052, 2, 160)
    recv = torch.full_like(face, -1.0)
    send = face.clone()
    ops = [dist.P2POp(dist.isend, send, rank), dist.P2POp(dist.irecv, recv, rank)]
    works = dist.batch_isend_irecv(ops)
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    ok = bool(torch.equal(recv, face))
    # the same with several rounds and an all_reduce (bench's max-over-ranks) in between
    t = torch.tensor([1.5], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    for r in range(3):
        send.add_(1.0)
        works = dist.batch_isend_irecv([dist.P2POp(dist.isend, send, rank), dist.P2POp(dist.irecv, recv, rank)])
        for w in works:
            w.wait()
        torch.cuda.synchronize()
        ok = ok and bool(torch.equal(recv, face + (r + 1)))
    dist.barrier()
    print(json.dumps({"rccl_p2p_self": ok, "all_reduce": float(t.item()), "world": world,
                      "nccl_version": ".".join(map(str, torch.cuda.nccl.version()))}), flush=True)
    dist.destroy_process_group()
    if not ok:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
