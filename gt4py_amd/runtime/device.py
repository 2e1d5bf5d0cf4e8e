"""Device selection: one process per GPU (LOCAL_RANK), torch for memory and streams."""

from __future__ import annotations

import os


def current_device():
    import torch

    if not torch.cuda.is_available():
        raise RuntimeError(
            "gt:mi355x needs a ROCm GPU (torch.cuda.is_available() is False); "
            "no CPU fallback exists for this backend"
        )
    return torch.device("cuda", torch.cuda.current_device())


def bind_local_rank() -> int:
    """Select the GPU of this process from LOCAL_RANK (torch.distributed launch convention)."""
    import torch

    lr = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(lr % max(1, torch.cuda.device_count()))
    return lr
