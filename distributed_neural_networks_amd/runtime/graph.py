"""HIP-graph capture of a launch sequence over static buffers.

``torch.cuda.CUDAGraph`` on ROCm is a hipGraph; every HIP kernel in this
package launches on torch's current stream, so a stage (or a whole colocated
pipeline step) captured here replays as one ``hipGraphLaunch`` — the launch
overhead of the ~2-40 kernels per step disappears (guide: graph-replay-floor).
Kernels read dynamic scalars (positions, lengths) from device memory, so one
capture serves every decode step.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class GraphedStep:
    def __init__(self, fn: Callable[[], object], device: Optional[torch.device] = None, warmup: int = 2,
                 pool=None, reset: Optional[Callable[[], None]] = None):
        """``reset`` (optional) runs on the capture stream after the warmup
        runs and before the capture: state the warmup advanced (decode
        positions, input ids) is put back, so the captured run starts where
        the caller's state was."""
        self.fn = fn
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.result = fn()
            if reset is not None:
                reset()
            s.synchronize()
            # thread-local capture: ProcessGroupNCCL's watchdog thread keeps
            # polling its events while a multi-GPU rank captures its decode step
            with torch.cuda.graph(self.graph, stream=s, pool=pool, capture_error_mode="thread_local"):
                self.result = fn()
        torch.cuda.current_stream(self.device).wait_stream(s)

    def __call__(self):
        self.graph.replay()
        return self.result
