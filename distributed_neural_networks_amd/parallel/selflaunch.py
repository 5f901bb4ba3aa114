"""Self-launch for the multi-GPU benches: ``python bench.py --gpus N`` with no
launcher starts N rank processes of itself.

The driver (and a user) may invoke ``bench.py --gpus 8`` directly instead of
through ``torch.distributed.run``.  Without ``RANK``/``WORLD_SIZE`` in the
environment the process group would come up as world 1 and the run would
silently measure one GPU.  So a parent that finds no launcher env:

* never touches the GPU (no ``torch.cuda`` call, no HIP init: the children
  own the devices, and nothing is exec'd from a process that initialised HIP);
* spawns N children of the same script with ``RANK``/``LOCAL_RANK``/
  ``WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT`` set (127.0.0.1, a free port),
  each in its own process group;
* relays rank 0's stdout to its own stdout (the JSON line), the other ranks'
  stdout to stderr with a rank prefix, and inherits stderr;
* exits with the first non-zero child status, killing the remaining children
  (exact process groups, never by pattern); a wall-clock limit ends a hung
  run with 124.

Under any launcher, :func:`check_world` makes ``--gpus`` and the world size
agree, so a mislaunched run fails loudly instead of printing a wrong
``n_gpus``.  The reference has no launcher at all: every stage is started by
hand in its own shell (``readme.md:80-98``)."""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional


def launcher_env_present() -> bool:
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pump(src, dst, prefix: str) -> None:
    for line in iter(src.readline, ""):
        dst.write(prefix + line if prefix else line)
        dst.flush()
    src.close()


def _kill_group(p: subprocess.Popen, sig: int) -> None:
    try:
        os.killpg(p.pid, sig)  # the child's own session: exactly the processes this launcher started
    except (ProcessLookupError, PermissionError):
        pass


def spawn_ranks(n: int, script: str, argv: List[str], timeout_s: float = 1800.0,
                extra_env: Optional[dict] = None) -> int:
    """Run ``python script *argv`` as ranks 0..n-1 of one job; return the job's exit code."""
    port = free_port()
    procs, pumps = [], []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
                    "DNN_SELF_LAUNCHED": "1"})
        if extra_env:
            env.update(extra_env)
        p = subprocess.Popen([sys.executable, "-u", script, *argv], env=env, stdout=subprocess.PIPE,
                             stdin=subprocess.DEVNULL, text=True, bufsize=1, start_new_session=True)
        procs.append(p)
        t = threading.Thread(target=_pump, args=(p.stdout, sys.stdout if r == 0 else sys.stderr,
                                                 "" if r == 0 else f"[rank {r}] "), daemon=True)
        t.start()
        pumps.append(t)
    deadline = time.monotonic() + timeout_s
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                sys.stderr.write(f"selflaunch: a rank exited with status {rc}; stopping the others\n")
                break
            if all(c == 0 for c in codes):
                break
            if time.monotonic() > deadline:
                rc = 124
                sys.stderr.write(f"selflaunch: job exceeded {timeout_s:.0f} s; stopping every rank\n")
                break
            time.sleep(0.05)
    finally:
        live = [p for p in procs if p.poll() is None]
        for p in live:
            _kill_group(p, signal.SIGTERM)
        t_end = time.monotonic() + 10
        for p in live:
            try:
                p.wait(max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                _kill_group(p, signal.SIGKILL)
                p.wait()
        for t in pumps:
            t.join(5)
    if rc < 0:  # a child killed by a signal: report it as the shell would
        rc = 128 - rc
    return rc


def maybe_self_launch(n: int, script: str, argv: List[str], timeout_s: float = 1800.0) -> Optional[int]:
    """When ``n > 1`` and no launcher env exists, run the job as ``n`` child
    ranks and return its exit code; otherwise return None (this process is a rank)."""
    if n <= 1 or launcher_env_present():
        return None
    return spawn_ranks(n, script, argv, timeout_s)


def check_world(requested: int, world: int) -> None:
    """``--gpus`` must equal the number of ranks actually running."""
    if requested != world:
        raise SystemExit(f"--gpus {requested} but the job has {world} rank(s) (WORLD_SIZE="
                         f"{os.environ.get('WORLD_SIZE', 'unset')}): launch with --gpus equal to the rank count, "
                         f"or without a launcher so --gpus N spawns N ranks itself")
