"""Logging: the reference prints ``[node_id] ...`` lines to stdout
(``node.py:38-39,62,192``) and its output is block-buffered when piped; here
every line is flushed so multi-process runs interleave readably, and the key
reference lines keep their exact text."""
from __future__ import annotations

import sys
import time

_QUIET = False


def set_quiet(q: bool) -> None:
    global _QUIET
    _QUIET = q


def log(msg: str) -> None:
    if not _QUIET:
        print(msg, flush=True)


def err(msg: str) -> None:
    print(msg, file=sys.stderr, flush=True)


def ts() -> float:
    return time.perf_counter()
