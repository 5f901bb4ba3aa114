"""Colocated pipeline: every stage on one GPU (the 1-GPU measurement point).

Stage forwards are chained on one stream over preallocated buffers and the
whole step is captured into one HIP graph.  The multi-rank schedules (GPipe
stream, CLI request stream, decode ring) live in ``runtime/scheduler.py``.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from ..utils import trace
from .graph import GraphedStep
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
