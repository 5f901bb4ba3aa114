"""Stage-to-stage links over ``torch.distributed`` point-to-point.

The reference moves every activation GPU -> host -> protobuf -> TCP -> host ->
GPU through a new gRPC channel per request (``node.py:45-55,73-89``).  Here a
``P2PLink`` is one direction-agnostic peer of this rank: RCCL (backend
``"nccl"``) over the direct xGMI link between the two stage GPUs, or gloo on
CPU.  On RCCL:

* device buffers move GPU -> GPU, no host staging and no serialisation;
* ProcessGroupNCCL runs P2P on its own stream per peer pair, ordered after the
  work already queued on the compute stream when the op is posted, and
  ``Work.wait()`` orders the compute stream after the transfer without
  blocking the host — so a stage never waits on the host for a hop;
* ``exchange`` posts a middle stage's send-to-next and receive-from-prev as one
  group (one ``ncclGroupStart/End``, one fused launch) instead of two.

Every link counts messages and bytes (``stats``) for the METRICS line.
Message framing for open-ended streams (the CLI): a 4 x int64 header
``[kind, a, b, tag]`` precedes a request (``KIND_DATA``) or ends the stream
(``KIND_STOP``).  Static schedules (benchmarks, microbatches of one request)
move payloads without headers.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

KIND_DATA, KIND_STOP = 1, 2


class P2PLink:
    def __init__(self, peer: int, device: torch.device, group=None):
        self.peer = int(peer)
        self.device = device
        self.group = group
        self.sent_msgs = self.sent_bytes = self.recv_msgs = self.recv_bytes = 0
        self._hdr = None

    def _count_send(self, t: torch.Tensor):
        self.sent_msgs += 1
        self.sent_bytes += t.numel() * t.element_size()

    def _count_recv(self, t: torch.Tensor):
        self.recv_msgs += 1
        self.recv_bytes += t.numel() * t.element_size()

    def isend(self, t: torch.Tensor):
        if not t.is_contiguous():
            raise ValueError("P2PLink.isend needs a contiguous tensor (a copy would be freed in flight)")
        self._count_send(t)
        return dist.isend(t, self.peer, group=self.group)

    def irecv(self, out: torch.Tensor):
        self._count_recv(out)
        return dist.irecv(out, self.peer, group=self.group)

    def send(self, t: torch.Tensor) -> None:
        self.isend(t.contiguous()).wait()

    def recv(self, out: torch.Tensor) -> torch.Tensor:
        self.irecv(out).wait()
        return out

    # -- framed messages (header + payload) --------------------------------
    def send_header(self, kind: int, a: int = 0, b: int = 0, tag: int = 0) -> None:
        self.send(torch.tensor([kind, a, b, tag], dtype=torch.int64, device=self.device))

    def recv_header(self) -> List[int]:
        if self._hdr is None:
            self._hdr = torch.empty(4, dtype=torch.int64, device=self.device)
        self.recv(self._hdr)
        return [int(v) for v in self._hdr.cpu().tolist()]

    def stats(self) -> dict:
        return {"peer": self.peer, "sent_msgs": self.sent_msgs, "sent_bytes": self.sent_bytes,
                "recv_msgs": self.recv_msgs, "recv_bytes": self.recv_bytes}


def exchange(sends: Sequence[Tuple[P2PLink, torch.Tensor]], recvs: Sequence[Tuple[P2PLink, torch.Tensor]]):
    """Post several sends and receives as one group; returns their works
    (sends first).  RCCL fuses a group into one launch and never deadlocks on
    the order of the ops inside it."""
    ops = []
    for link, t in sends:
        link._count_send(t)
        ops.append(dist.P2POp(dist.isend, t, link.peer, group=link.group))
    for link, t in recvs:
        link._count_recv(t)
        ops.append(dist.P2POp(dist.irecv, t, link.peer, group=link.group))
    if not ops:
        return None
    return GroupWork(dist.batch_isend_irecv(ops))


class GroupWork:
    """The works of one ``exchange`` group (RCCL returns one coalesced work,
    gloo one per op); ``wait`` is idempotent so every slot that depends on the
    group can wait on it."""

    def __init__(self, works):
        self.works = list(works)

    def wait(self):
        while self.works:
            self.works.pop(0).wait()
        return True


def wait(work: Optional[object]) -> None:
    if work is not None:
        work.wait()
