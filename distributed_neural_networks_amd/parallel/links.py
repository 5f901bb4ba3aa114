"""Stage-to-stage links.

* ``P2PLink`` — point-to-point ``isend``/``irecv`` through ``torch.distributed``:
  RCCL (backend ``"nccl"``) over the direct xGMI link between the two stage
  GPUs, or gloo on CPU.  RCCL runs each peer pair on its own communicator and
  stream, so a middle stage's recv-from-prev and send-to-next never serialise
  against each other or against compute (ProcessGroupNCCL orders the P2P
  stream after the work already queued on the compute stream, and
  ``Work.wait()`` orders the compute stream after the transfer without
  blocking the host).
* the colocated case (all stages on one GPU) needs no link object: the
  pipeline runner chains stage forwards on one stream and captures them in a
  single HIP graph (``runtime/pipeline.py``).
* the gRPC ``SendTensor`` hop of the reference (``node.py:73-89``) lives in
  ``control/service.py`` (CPU plumbing data path, wire-compatible).

Message framing for open-ended streams (the CLI): a fixed 4 x int64 header
``[kind, batch, seq, tag]`` precedes each payload (``KIND_DATA``) or ends the
stream (``KIND_STOP``).  Benchmarks use static schedules without headers.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

KIND_DATA, KIND_STOP = 1, 2


class P2PLink:
    def __init__(self, peer: int, device: torch.device):
        self.peer = peer
        self.device = device

    def isend(self, t: torch.Tensor):
        return dist.isend(t.contiguous(), self.peer)

    def irecv(self, out: torch.Tensor):
        return dist.irecv(out, self.peer)

    def send(self, t: torch.Tensor) -> None:
        dist.send(t.contiguous(), self.peer)

    def recv(self, out: torch.Tensor) -> torch.Tensor:
        dist.recv(out, self.peer)
        return out

    # -- framed messages (header + payload) --------------------------------
    def send_header(self, kind: int, batch: int = 0, seq: int = 0, tag: int = 0) -> None:
        self.send(torch.tensor([kind, batch, seq, tag], dtype=torch.int64, device=self.device))

    def recv_header(self):
        h = torch.empty(4, dtype=torch.int64, device=self.device)
        self.recv(h)
        return [int(v) for v in h.cpu().tolist()]


def wait(work: Optional[object]) -> None:
    if work is not None:
        work.wait()
