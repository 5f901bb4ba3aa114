"""Launch every node of a pipeline config on this machine (one process per stage).

The reference is started by hand, one shell per node (``readme.md:80-98``);
this spawns them all, starts stage 0 last with the initiating arguments, and
returns stage 0's exit code.  Downstream nodes are stopped when stage 0 ends
(``--shutdown_pipeline`` over the control plane, then a kill after a grace
period), so a run never leaves orphan servers.

    python -m distributed_neural_networks_amd.tools.launch --config configs/cifar_2gpu_rccl.json \
        [--input_image img.png] [--num_requests N] [--prompt 1,2,3]

With config ``replicas`` = R (rccl / gloo) it starts R copies of every stage
(``--replica r``); copy 0's stage 0 is the process whose exit code is returned,
the other copies' exit codes are checked too.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--input_image", default=None)
    ap.add_argument("--num_requests", type=int, default=1)
    ap.add_argument("--prompt", default=None)
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    cfg = json.load(open(a.config))
    nodes = sorted(cfg["nodes"], key=lambda n: n["part_index"])
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    node_py = os.path.join(ROOT, "node.py")
    common = ["--config", a.config] + (["--quiet"] if a.quiet else [])
    transport = cfg.get("transport", "grpc")
    procs = []
    reps = int(cfg.get("replicas", 1))
    if transport != "colocated":
        for n in nodes[1:]:
            extra = ["--serve_seconds", str(a.timeout)] if transport == "grpc" else []
            procs.append(subprocess.Popen([sys.executable, node_py, "--node_id", n["id"]] + common + extra, env=env))
    first = [sys.executable, node_py, "--node_id", nodes[0]["id"]] + common + ["--num_requests", str(a.num_requests)]
    # data-parallel copies (config "replicas", rccl / gloo): every stage of copies 1..R-1, then copy 0 as below
    for rep in range(1, reps):
        for n in nodes[1:]:
            procs.append(subprocess.Popen([sys.executable, node_py, "--node_id", n["id"], "--replica", str(rep)]
                                          + common, env=env))
        head = [sys.executable, node_py, "--node_id", nodes[0]["id"], "--replica", str(rep)] + common + \
            ["--num_requests", str(a.num_requests)] + (["--input_image", a.input_image] if a.input_image else
                                                      (["--input_image", "__dummy__.png"]
                                                       if cfg.get("model", "cifar10") == "cifar10" else []))
        if a.prompt:
            head += ["--prompt", a.prompt]
        procs.append(subprocess.Popen(head, env=env))
    if a.input_image:
        first += ["--input_image", a.input_image]
    elif cfg.get("model", "cifar10") == "cifar10":
        first += ["--input_image", "__dummy__.png"]  # missing file -> dummy input, like the reference
    if a.prompt:
        first += ["--prompt", a.prompt]
    if transport == "grpc":
        first += ["--shutdown_pipeline"]
    rc = subprocess.call(first, env=env, timeout=a.timeout)
    deadline = time.time() + 30
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    bad = [p.returncode for p in procs if p.returncode not in (0, None, -9)]
    return rc if rc != 0 else (bad[0] if bad else 0)


if __name__ == "__main__":
    sys.exit(main())
