"""Per-stage metrics: counters and latency samples, emitted as one JSON line.

The reference only prints (metrics/logging).  A ``StageMetrics``
object is owned by each stage loop / servicer; ``summary()`` gives requests,
items, throughput and p50/p99 latency, and ``emit()`` prints
``METRICS {...}`` (one line, machine-readable) — enabled by ``--metrics`` or
``DNN_METRICS=1``.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional


def percentile(xs: List[float], q: float) -> Optional[float]:
    if not xs:
        return None
    s = sorted(xs)
    k = min(len(s) - 1, max(0, int(round(q / 100.0 * (len(s) - 1)))))
    return s[k]


class StageMetrics:
    def __init__(self, node_id: str, stage: int):
        self.node_id, self.stage = node_id, stage
        self.t_start = time.perf_counter()
        self.requests = 0
        self.items = 0
        self.latency_s: List[float] = []
        self.counters: Dict[str, float] = {}

    def record(self, seconds: float, items: int = 1) -> None:
        self.requests += 1
        self.items += items
        self.latency_s.append(seconds)

    def add(self, key: str, v: float = 1.0) -> None:
        self.counters[key] = self.counters.get(key, 0.0) + v

    def summary(self) -> dict:
        el = time.perf_counter() - self.t_start
        lat = self.latency_s
        return {"node_id": self.node_id, "stage": self.stage, "requests": self.requests, "items": self.items,
                "elapsed_s": round(el, 6), "items_per_s": round(self.items / el, 3) if el > 0 else None,
                "latency_ms_p50": None if not lat else round(percentile(lat, 50) * 1e3, 4),
                "latency_ms_p99": None if not lat else round(percentile(lat, 99) * 1e3, 4),
                "latency_ms_mean": None if not lat else round(sum(lat) / len(lat) * 1e3, 4),
                **{k: v for k, v in self.counters.items()}}

    def emit(self, force: bool = False) -> None:
        if force or os.environ.get("DNN_METRICS"):
            print("METRICS " + json.dumps(self.summary()), flush=True)
