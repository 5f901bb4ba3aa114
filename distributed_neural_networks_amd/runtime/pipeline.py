"""Pipeline schedules (forward-only inference).

Reference: one request is in flight; stage i's handler blocks on the nested
RPC to stage i+1 for the whole downstream latency (``node.py:70-94``), with a
new channel per request.  Here:

* ``ColocatedPipeline`` — every stage on one GPU (the 1-GPU measurement point):
  stage forwards are chained on one stream over preallocated buffers and the
  whole step is captured into one HIP graph.
* ``run_stage_stream`` — one rank of a multi-process pipeline (RCCL over xGMI,
  or gloo on CPU): a GPipe-style forward-only fill/drain over M microbatches
  with ``depth``-deep slot rings.  The irecv for microbatch i+depth is posted
  while microbatch i computes, and the isend of i overlaps the compute of
  i+1, so in steady state every stage computes while its links move data.
  Slot reuse is ordered by the P2P work handles (no host sync on RCCL).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch

from ..parallel.links import P2PLink
from ..utils import trace
from .graph import GraphedStep
from .ordering import SlotOrder
from .stages import StageCompute, StageOutput


class ColocatedPipeline:
    def __init__(self, stages: Sequence[StageCompute], batch: int):
        self.stages = list(stages)
        self.batch = batch
        dev = self.stages[0].device
        shp, dt = self.stages[0].in_spec(batch)
        self.x = torch.zeros(shp, dtype=dt, device=dev)
        self.bufs: List[torch.Tensor] = []
        for s in self.stages:
            oshp, odt = s.out_spec(batch)
            self.bufs.append(torch.empty(oshp, dtype=odt, device=dev))
        self._graph: Optional[GraphedStep] = None

    def _step(self):
        h = self.x
        for s, b in zip(self.stages, self.bufs):
            h = s.forward(h, b)
        return h

    def capture(self) -> None:
        self._graph = GraphedStep(self._step, self.stages[0].device)

    def __call__(self, x: Optional[torch.Tensor] = None) -> StageOutput:
        if x is not None:
            self.x.copy_(x, non_blocking=True)
        with trace.span("pipeline_step", "compute", device=self.x.device, batch=self.batch):
            if self._graph is not None:
                return self._graph()
            return self._step()


def run_stage_stream(stage: StageCompute, M: int, batch: int, prev: Optional[P2PLink], nxt: Optional[P2PLink],
                     source: Optional[Callable[[int], torch.Tensor]] = None,
                     sink: Optional[Callable[[int, object], None]] = None, depth: int = 2) -> None:
    """Stream M microbatches of `batch` through this rank's stage."""
    dev = stage.device
    ishp, idt = stage.in_spec(batch)
    oshp, odt = stage.out_spec(batch)
    depth = max(1, min(depth, M))
    in_slots = [torch.empty(ishp, dtype=idt, device=dev) for _ in range(depth)] if prev else []
    out_slots = [torch.empty(oshp, dtype=odt, device=dev) for _ in range(depth)]
    rwork: List[object] = [None] * depth
    swork: List[object] = [None] * depth
    ins, outs = SlotOrder("in_slots", depth), SlotOrder("out_slots", depth)  # DNN_DEBUG_ORDER=1 checks
    if prev is not None:
        for k in range(depth):
            rwork[k] = prev.irecv(in_slots[k])
            ins.post(k, "recv", k)
    for i in range(M):
        k = i % depth
        if prev is None:
            x = source(i)
        else:
            with trace.span("recv_wait", "p2p", mb=i):
                rwork[k].wait()
            ins.waited(k)
            ins.use(k, "stage input read", i)
            x = in_slots[k]
        if swork[k] is not None:
            with trace.span("slot_reuse_wait", "p2p", mb=i):
                swork[k].wait()
            swork[k] = None
            outs.waited(k)
        outs.use(k, "stage output write", i)
        with trace.span("stage_forward", "compute", device=dev, mb=i):
            y = stage.forward(x, out_slots[k])
        if prev is not None and i + depth < M:
            rwork[k] = prev.irecv(in_slots[k])  # ordered after this slot's compute (see module doc)
            ins.post(k, "recv", i + depth)
        if nxt is not None:
            swork[k] = nxt.isend(y if isinstance(y, torch.Tensor) else y.probs)
            outs.post(k, "send", i)
        if sink is not None:
            sink(i, y)
    for k, w in enumerate(swork):
        if w is not None:
            w.wait()
            outs.waited(k)
    ins.drained()
    outs.drained()
