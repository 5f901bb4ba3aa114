"""Debug-mode stream-ordering checks for slot buffers (race detection).

The streaming schedules (``runtime/pipeline.py``) reuse a ring of activation
slots: a slot may be overwritten only after every asynchronous transfer that
reads or writes it has been waited on (``Work.wait()`` orders the compute
stream after the transfer, so on the device the reuse is then safe).  A
missing wait is a silent data race on the GPU.  ``SlotOrder`` tracks, per
slot, the transfer in flight and raises on an illegal transition; it is a
no-op unless ``DNN_DEBUG_ORDER=1`` (or ``DNN_DEBUG_SYNC=1``) is set, so the
hot path pays one attribute test.
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple


def ordering_checks_enabled() -> bool:
    return bool(os.environ.get("DNN_DEBUG_ORDER") or os.environ.get("DNN_DEBUG_SYNC"))


class SlotOrderError(RuntimeError):
    pass


class SlotOrder:
    def __init__(self, name: str, n: int, enabled: Optional[bool] = None):
        self.name = name
        self.enabled = ordering_checks_enabled() if enabled is None else enabled
        self.pending: List[Optional[Tuple[str, int]]] = [None] * n
        self.events = 0

    def post(self, k: int, kind: str, mb: int = -1) -> None:
        """An async transfer of ``kind`` ('recv' writes, 'send' reads the slot) was issued."""
        if not self.enabled:
            return
        if self.pending[k] is not None:
            pk, pmb = self.pending[k]
            raise SlotOrderError(f"{self.name}[{k}]: {kind} for microbatch {mb} posted while the {pk} of "
                                 f"microbatch {pmb} is still in flight (no wait)")
        self.pending[k] = (kind, mb)
        self.events += 1

    def waited(self, k: int) -> None:
        if self.enabled:
            self.pending[k] = None

    def use(self, k: int, what: str, mb: int = -1) -> None:
        """Compute is about to read or write slot ``k``."""
        if not self.enabled:
            return
        if self.pending[k] is not None:
            pk, pmb = self.pending[k]
            raise SlotOrderError(f"{self.name}[{k}]: {what} of microbatch {mb} while the {pk} of microbatch {pmb} "
                                 f"has not been waited on")
        self.events += 1

    def drained(self) -> None:
        if not self.enabled:
            return
        busy = [(k, p) for k, p in enumerate(self.pending) if p is not None]
        if busy:
            raise SlotOrderError(f"{self.name}: transfers never waited on: {busy}")
