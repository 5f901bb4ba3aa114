"""Loader for the in-tree HIP kernel library (``_dnn_hip*.so``).

``import torch`` happens first so the library binds to the HIP runtime torch
already loaded (same ``libamdhip64.so.7`` soname) and shares its streams.
There is no fallback: on a GPU box a missing or stale library raises with the
build command; CPU-only processes never call into it.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the extension: shared HIP runtime)

_lib = None


def lib():
    global _lib
    if _lib is None:
        try:
            _lib = importlib.import_module("distributed_neural_networks_amd._dnn_hip")
        except ImportError as e:
            raise RuntimeError(
                "HIP kernel library _dnn_hip is not built; run "
                "`python -m distributed_neural_networks_amd.ops.build` (hipcc, gfx950)") from e
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except RuntimeError:
        return False


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


DEBUG_SYNC = bool(os.environ.get("DNN_DEBUG_SYNC"))


def check(rc: int, what: str) -> None:
    """Raise on a rejected/failed launch.  With ``DNN_DEBUG_SYNC=1`` every kernel
    is followed by a device sync so an asynchronous fault (bad address, hang)
    is attributed to the launch that caused it (race/fault triage mode; the
    GPU-side sanitizer is not available on this pool)."""
    if rc != 0:
        raise RuntimeError(f"{what}: HIP launch failed with code {rc}")
    if DEBUG_SYNC:
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError(f"{what}: device fault after launch: {e}") from e


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def library_path() -> str:
    return os.path.abspath(lib().__file__)
