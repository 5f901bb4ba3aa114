"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over RCCL.

On ROCm the ``"nccl"`` backend *is* RCCL; its P2P send/recv between adjacent
pipeline stages travels over the direct xGMI link of the fully connected
8xMI355X board.  The CPU fallback for tests and the plumbing config is
``"gloo"`` (same code path, host tensors).

Rendezvous: ``torchrun``-style env (``RANK``/``WORLD_SIZE``/``MASTER_ADDR``/
``MASTER_PORT``) when present; otherwise derived from the pipeline config —
rank = ``part_index``, world = ``num_parts``, master = stage 0's host and its
port + ``PORT_OFFSET`` (the gRPC control plane keeps the configured port).
The reference has no collective runtime at all; its only
"barrier" is ``asyncio.sleep(2)`` (``node.py:203-207``) — process-group init
is a real barrier.
"""
from __future__ import annotations

import datetime
import os
import sys
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

PORT_OFFSET = 1000


@dataclass
class DistInfo:
    rank: int
    world: int
    local_rank: int
    backend: str
    device: torch.device


def env_rank_world():
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        return int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ.get("LOCAL_RANK", 0))
    return None


def pick_backend(device_type: str) -> str:
    return "nccl" if device_type == "cuda" else "gloo"


def init(backend: Optional[str] = None, rank: Optional[int] = None, world: Optional[int] = None,
         master_addr: Optional[str] = None, master_port: Optional[int] = None,
         device_index: Optional[int] = None, timeout_s: float = 300.0) -> DistInfo:
    """Initialise (idempotent) the default process group and bind this process's device."""
    env = env_rank_world()
    if rank is None or world is None:
        if env is None:
            rank, world = 0, 1
        else:
            rank, world = env[0], env[1]
    local_rank = env[2] if env is not None else (device_index if device_index is not None else rank)
    use_gpu = torch.cuda.is_available() and (backend in (None, "nccl"))
    backend = backend or ("nccl" if use_gpu else "gloo")
    if backend == "nccl":
        idx = device_index if device_index is not None else local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    if backend == "nccl":
        # a failed/timed-out RCCL op tears the communicator down instead of hanging
        # (second line of defence behind parallel/watchdog.py)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", master_addr or "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(master_port or 29500))
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return DistInfo(rank=rank, world=world, local_rank=local_rank, backend=backend, device=device)


_BACK_GROUP = None


def back_group():
    """A second communicator over every rank, for the pipeline back-edge
    (predictions / sampled tokens from the last stage to the return stage).

    On RCCL all P2P between one rank pair shares one communicator and one
    stream, so a return rank that posts its receives ahead of its forward
    sends to the same peer (the 2-stage CIFAR stream, the 2-group decode ring)
    would queue them in front of the data they wait for.  On its own
    communicator the back-edge has its own stream and never orders against
    forward traffic.  Collective: every rank calls it (once, right after
    ``init``); later calls return the cached group.  None on one rank."""
    global _BACK_GROUP
    if _BACK_GROUP is None and dist.is_initialized() and dist.get_world_size() > 1:
        _BACK_GROUP = dist.new_group(list(range(dist.get_world_size())))
    return _BACK_GROUP


def barrier(info: DistInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def shutdown() -> None:
    global _BACK_GROUP
    _BACK_GROUP = None
    rccl = sys.modules.get(__package__ + ".rccl")
    if rccl is not None:  # native RCCL channels (parallel/rccl.py) go before the store they were bootstrapped from
        rccl.destroy_all()
    if dist.is_initialized():
        dist.destroy_process_group()
