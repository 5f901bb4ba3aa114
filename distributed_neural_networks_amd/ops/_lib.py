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


def verify_stamp(path: str) -> dict:
    """Build provenance check: the library must carry a stamp
    (``ops/build.py::write_stamp``) whose library hash matches the file and
    whose source hashes match the sources in this tree.  A stale binary (built
    from other sources) raises instead of silently running old kernels.
    ``DNN_SKIP_STAMP=1`` skips the check (kernel development only)."""
    import hashlib
    import json
    stamp_path = os.path.join(os.path.dirname(path), "_dnn_hip.build.json")
    if os.environ.get("DNN_SKIP_STAMP"):
        return {}
    if not os.path.exists(stamp_path):
        raise RuntimeError(f"{path} has no build stamp ({stamp_path}); rebuild with "
                           "`python -m distributed_neural_networks_amd.ops.build`")
    stamp = json.load(open(stamp_path))
    if hashlib.sha256(open(path, "rb").read()).hexdigest() != stamp.get("library_sha256"):
        raise RuntimeError(f"{path} does not match its build stamp (library replaced after the build); rebuild")
    from .build import source_digest
    now = source_digest()
    stale = sorted(k for k in set(now) | set(stamp.get("sources", {})) if now.get(k) != stamp["sources"].get(k))
    if stale:
        raise RuntimeError(f"{path} was built from different sources ({', '.join(stale[:6])}); rebuild with "
                           "`python -m distributed_neural_networks_amd.ops.build`")
    return stamp


def _load_override(path: str):
    """``DNN_HIP_LIB=/path/_dnn_hip*.so``: load that build instead of the
    in-tree one (A/B of two builds in one session, bench/probes/lib_ab.py;
    no stamp check: the file is named explicitly)."""
    import importlib.util
    import sys
    spec = importlib.util.spec_from_file_location("distributed_neural_networks_amd._dnn_hip", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["distributed_neural_networks_amd._dnn_hip"] = mod
    return mod


def lib():
    global _lib
    if _lib is None and os.environ.get("DNN_HIP_LIB"):
        _lib = _load_override(os.environ["DNN_HIP_LIB"])
    if _lib is None:
        try:
            mod = importlib.import_module("distributed_neural_networks_amd._dnn_hip")
        except ImportError as e:
            raise RuntimeError(
                "HIP kernel library _dnn_hip is not built; run "
                "`python -m distributed_neural_networks_amd.ops.build` (hipcc, gfx950)") from e
        verify_stamp(mod.__file__)
        _lib = mod
    return _lib


def build_stamp() -> dict:
    import json
    p = os.path.join(os.path.dirname(library_path()), "_dnn_hip.build.json")
    return json.load(open(p)) if os.path.exists(p) else {}


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
