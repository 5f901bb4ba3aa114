"""Build the in-tree HIP kernel library ``_dnn_hip`` for gfx950 with hipcc.

No torch cpp_extension (it hipifies sources); plain ``hipcc --offload-arch=gfx950``
per translation unit, incremental on mtimes, then one shared-object link into
the package directory so the built ``.so`` ships with the repo snapshot to the
GPU box.  Usage: ``python -m distributed_neural_networks_amd.ops.build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "distributed_neural_networks_amd")
BUILD = os.path.join(ROOT, "build", "hip")
ARCH = os.environ.get("DNN_OFFLOAD_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
LIB_PATH = os.path.join(PKG, "_dnn_hip" + EXT_SUFFIX)

TRANSFORMER_SRCS = ("norm_embed.hip", "attention.hip", "sampler.hip", "gemm_fp8.hip")
# ReLU/max-pool epilogues: no NaN-canonicalising v_max before every fmaxf of an MFMA result
# No SLP vectoriser where it packs scalar FP32 into cross-half v_pk_*_f32 (op_sel
# reads of a pair's other half) whose low result a 32-bit VALU op reads: under two
# workgroups per CU that read returned the pre-op value in lanes 48-63 (the
# one-shot GEMM's row statistics, csrc/kernels/gemm_oneshot.h "The race of rounds
# 5-6"; 100 -> 0 mismatches in 10000 calls, profiles/r6_oneshot_race_root_cause.md).
# Explicit vector code keeps its packed ops.
NO_SLP = ["-fno-slp-vectorize"]
PER_FILE_FLAGS = {"cifar_fused.hip": ["-ffast-math"],
                  # fp32-accurate split path: keep IEEE rounding, only drop NaN canonicalisation in fmaxf
                  "cifar_x3.hip": ["-fno-honor-nans"],
                  # flash / decode softmax maxima over MFMA results: no v_max canonicalise
                  # per score (52 -> 17 v_max per GPT-2 flash block); -inf masking is kept
                  "attention.hip": ["-fno-honor-nans"] + NO_SLP,
                  "gemm_skinny.hip": NO_SLP,
                  "gemm_bf16.hip": NO_SLP}


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.exists(c) or c == "hipcc"):
            return c
    raise RuntimeError("hipcc not found")


def sources() -> List[str]:
    return (sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))) + sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
            + [os.path.join(CSRC, "bindings.cpp")])


def _flags(src: str) -> List[str]:
    f = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I" + CSRC, "-Wno-unused-result",
         "-Wno-unused-command-line-argument"]
    f += PER_FILE_FLAGS.get(os.path.basename(src), [])
    have_tf = all(os.path.exists(os.path.join(CSRC, "kernels", s)) for s in TRANSFORMER_SRCS)
    if have_tf:
        f.append("-DDNN_HAVE_TRANSFORMER")
    if src.endswith("bindings.cpp"):
        import pybind11
        f += ["-x", "hip", "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]
    return f


def _headers_mtime() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max([os.path.getmtime(h) for h in hs] + [0.0])


def _obj(src: str) -> str:
    import hashlib
    tag = hashlib.sha1(" ".join(_flags(src)).encode()).hexdigest()[:8]
    return os.path.join(BUILD, f"{os.path.basename(src)}.{tag}.o")


def _compile(src: str, force: bool, hm: float) -> str:
    obj = _obj(src)
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hm):
        return obj
    cmd = [_hipcc()] + _flags(src) + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 0, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sources()
    hm = _headers_mtime()
    jobs = jobs or min(len(srcs), int(os.environ.get("MAX_JOBS", "8")), os.cpu_count() or 4, 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, hm), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < newest:
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + ["-o", LIB_PATH]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    write_stamp(srcs)
    if verbose:
        print(f"[build] {LIB_PATH} ({len(objs)} objects, arch {ARCH})")
    return LIB_PATH


STAMP_PATH = os.path.join(PKG, "_dnn_hip.build.json")


def source_digest(srcs: List[str] = None) -> dict:
    """sha256 of every source and header the library is built from."""
    import hashlib
    srcs = srcs or sources()
    files = sorted(set(srcs) | set(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)))
    return {os.path.relpath(f, ROOT): hashlib.sha256(open(f, "rb").read()).hexdigest() for f in files}


def write_stamp(srcs: List[str]) -> None:
    """Build provenance next to the .so: source hashes, per-file flags, the
    compiler, the library's own hash (``_lib.verify_stamp`` checks them at
    load, so a stale or foreign binary fails loudly instead of running)."""
    import hashlib
    import json
    import time
    r = subprocess.run([_hipcc(), "--version"], capture_output=True, text=True)
    stamp = {"arch": ARCH, "built_at": time.strftime("%Y-%m-%dT%H:%M:%S"),
             "hipcc": (r.stdout or r.stderr).strip().splitlines()[:2],
             "flags": {os.path.basename(s): _flags(s) for s in srcs},
             "sources": source_digest(srcs),
             "library_sha256": hashlib.sha256(open(LIB_PATH, "rb").read()).hexdigest()}
    with open(STAMP_PATH, "w") as f:
        json.dump(stamp, f, indent=1)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    build(a.force, a.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
