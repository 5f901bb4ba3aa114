"""Tracing: host spans + device-timed spans -> Chrome trace JSON, plus roctx
ranges so ``rocprofv3 --marker-trace`` timelines show the same phases.

The reference has no tracing.  Enable with ``DNN_TRACE=out.json``
(or ``trace.enable(path)``); every ``span(name)`` then records
``[start, end)`` on the host clock and, when a CUDA/HIP device is given, a
pair of ``hipEvent``s whose device timestamps are resolved at flush (no
synchronisation inside the hot loop).  Disabled tracing costs one attribute
lookup per span.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time
from typing import List, Optional

_state = {"on": False, "path": None, "events": [], "dev": [], "t0": time.perf_counter(), "epoch0": time.time(),
          "pid": os.getpid()}
_lock = threading.Lock()
_roctx = None


def _load_roctx():
    global _roctx
    if _roctx is not None:
        return _roctx or None
    for name in ("librocprofiler-sdk-roctx.so", "libroctx64.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so",
                 "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            return lib
        except OSError:
            continue
    _roctx = False
    return None


def enable(path: Optional[str] = None) -> None:
    _state["on"] = True
    _state["path"] = path or os.environ.get("DNN_TRACE", "trace.json")
    _load_roctx()


def enabled() -> bool:
    return _state["on"]


if os.environ.get("DNN_TRACE"):
    enable(os.environ["DNN_TRACE"])


@contextlib.contextmanager
def span(name: str, cat: str = "host", device=None, **args):
    if not _state["on"]:
        yield
        return
    rx = _load_roctx()
    if rx:
        rx.roctxRangePushA(name.encode())
    ev = None
    if device is not None and getattr(device, "type", None) == "cuda":
        import torch
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    t = time.perf_counter()
    try:
        yield
    finally:
        t1 = time.perf_counter()
        if ev is not None:
            ev[1].record()
        if rx:
            rx.roctxRangePop()
        tid = threading.get_ident() % 100000
        with _lock:
            _state["events"].append({"name": name, "cat": cat, "ph": "X", "pid": _state["pid"], "tid": tid,
                                     "ts": (t - _state["t0"]) * 1e6, "dur": (t1 - t) * 1e6, "args": args})
            if ev is not None:
                _state["dev"].append((name, cat, ev, t, args))


def instant(name: str, **args) -> None:
    if _state["on"]:
        with _lock:
            _state["events"].append({"name": name, "ph": "i", "s": "p", "pid": _state["pid"], "tid": 0,
                                     "ts": (time.perf_counter() - _state["t0"]) * 1e6, "args": args})


def flush(path: Optional[str] = None) -> Optional[str]:
    """Write the Chrome trace (resolving device spans); returns the path."""
    if not _state["on"]:
        return None
    path = path or _state["path"]
    events: List[dict] = list(_state["events"])
    if _state["dev"]:
        import torch
        torch.cuda.synchronize()
        base = None
        for name, cat, (e0, e1), t_host, args in _state["dev"]:
            if base is None:
                base = (e0, t_host)
            off_ms = base[0].elapsed_time(e0)
            events.append({"name": name, "cat": cat + ".gpu", "ph": "X", "pid": _state["pid"], "tid": "gpu",
                           "ts": (base[1] - _state["t0"]) * 1e6 + off_ms * 1e3, "dur": e0.elapsed_time(e1) * 1e3,
                           "args": args})
    # epoch of ts = 0, so traces of several ranks (one file each) can be merged
    # onto one timeline: wall_us = epoch_t0_us + ts
    meta = {"epoch_t0_us": _state["epoch0"] * 1e6, "pid": _state["pid"]}
    with open(path, "w") as f:
        json.dump({"traceEvents": events, "displayTimeUnit": "ms", "otherData": meta}, f)
    return path


def reset() -> None:
    with _lock:
        _state["events"].clear()
        _state["dev"].clear()
        _state["t0"] = time.perf_counter()
        _state["epoch0"] = time.time()
