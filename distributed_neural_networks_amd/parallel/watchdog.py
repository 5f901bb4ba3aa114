"""Pipeline failure detection for the RCCL / gloo transports.

The reference has no failure handling beyond turning a forwarding RPC error
into a status string (``node.py:91-100``); a dead stage hangs every peer.  On
the P2P transports a dead peer is worse: an RCCL receive from a rank that
exited waits until the process-group timeout (minutes).  This watchdog bounds
that:

* every rank runs a daemon thread that bumps a heartbeat counter
  ``dnn_wd/hb/<rank>`` in the rendezvous TCPStore every ``interval_s`` and
  watches every peer's counter; a peer whose counter has not moved for
  ``peer_timeout_s`` (measured on the local clock, so host clock skew does not
  matter) is declared dead;
* any rank that detects a failure (dead peer, store unreachable, a local stall
  longer than ``stall_timeout_s``, or an exception in the schedule) publishes
  ``dnn_wd/abort`` and exits with ``EXIT_ABORT``; every other rank sees the
  key on its next poll and exits too, so the whole pipeline tears down within
  about ``peer_timeout_s`` instead of the 300 s process-group timeout;
* ranks that finish cleanly publish ``dnn_wd/done/<rank>`` first, so a peer
  that has legitimately stopped beating is not mistaken for a crash.

``os._exit`` skips interpreter teardown on purpose: a thread blocked inside an
RCCL wait cannot be interrupted, and the driver reclaims the device queues of
an exited process.  ProcessGroupNCCL's own async error handling
(``TORCH_NCCL_ASYNC_ERROR_HANDLING``) is enabled by ``comm.init`` as the second
line of defence.
"""
from __future__ import annotations

import datetime
import os
import sys
import threading
import time
from typing import Dict, Optional

EXIT_ABORT = 3
PREFIX = "dnn_wd/"


def _log(msg: str) -> None:
    print(msg, flush=True)
    sys.stderr.flush()


class Watchdog:
    def __init__(self, rank: int, world: int, host: Optional[str] = None, port: Optional[int] = None,
                 peer_timeout_s: float = 15.0, stall_timeout_s: Optional[float] = None, interval_s: float = 0.5,
                 tag: str = "", exit_fn=None):
        self.rank, self.world = rank, world
        self.host = host or os.environ.get("MASTER_ADDR", "127.0.0.1")
        self.port = int(port or os.environ.get("MASTER_PORT", 29500))
        self.peer_timeout_s = float(peer_timeout_s)
        self.stall_timeout_s = stall_timeout_s
        self.interval_s = float(interval_s)
        self.tag = tag or f"[rank {rank}]"
        self.exit_fn = exit_fn or os._exit
        self._progress = time.monotonic()
        self._busy = False
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._store = None
        self.aborted: Optional[str] = None
        self._exited = threading.Lock()

    def _exit(self) -> None:
        # abort() from the schedule and the thread's own poll can both fire
        if self._exited.acquire(blocking=False):
            self._stop.set()
            rccl = sys.modules.get(__package__ + ".rccl")
            if rccl is not None:  # native channels: in-flight P2P kernels return before the process goes
                rccl.abort_all()
            self.exit_fn(EXIT_ABORT)

    # -- called from the schedule (cheap) -----------------------------------
    def beat(self) -> None:
        self._progress = time.monotonic()

    def busy(self, on: bool = True) -> None:
        """Mark that this rank is inside work that should keep progressing."""
        self._busy = on
        self._progress = time.monotonic()

    # -- lifecycle -------------------------------------------------------------
    def _connect(self):
        import torch.distributed as dist
        return dist.TCPStore(self.host, self.port, is_master=False, timeout=datetime.timedelta(seconds=10),
                             wait_for_workers=False)

    def start(self) -> "Watchdog":
        if self.world <= 1 or self._thread is not None:
            return self
        self._store = self._connect()
        self._store.add(f"{PREFIX}hb/{self.rank}", 1)
        self._thread = threading.Thread(target=self._loop, name="dnn-watchdog", daemon=True)
        self._thread.start()
        return self

    def done(self) -> None:
        """This rank finished cleanly: peers must not treat its silence as a crash."""
        if self._store is not None:
            try:
                self._store.set(f"{PREFIX}done/{self.rank}", "1")
            except Exception:  # noqa: BLE001
                pass

    def stop(self) -> None:
        """Stop the thread.  Rank 0 usually hosts the store, so it lingers
        (bounded) until every rank has stopped polling, else a peer's last poll
        would see the store vanish and report a false failure."""
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5 * self.interval_s + 5)
            self._thread = None
        if self._store is None:
            return
        try:
            n = self._store.add(f"{PREFIX}stopped", 1)
            t_end = time.monotonic() + 10.0
            while self.rank == 0 and n < self.world and time.monotonic() < t_end:
                time.sleep(0.02)
                n = self._store.add(f"{PREFIX}stopped", 0)
        except Exception:  # noqa: BLE001
            pass

    def abort(self, reason: str) -> None:
        """Publish the failure so every rank exits, then exit this process."""
        self.aborted = reason
        _log(f"!!! {self.tag} pipeline failure: {reason}; aborting (exit {EXIT_ABORT})")
        try:
            if self._store is None:
                self._store = self._connect()
            self._store.set(f"{PREFIX}abort", f"rank {self.rank}: {reason}")
        except Exception:  # noqa: BLE001
            pass
        self._exit()

    # -- the thread --------------------------------------------------------------
    def _loop(self) -> None:
        st = self._store
        peers = [p for p in range(self.world) if p != self.rank]
        seen: Dict[int, int] = {p: -1 for p in peers}
        changed: Dict[int, float] = {p: time.monotonic() for p in peers}
        done: Dict[int, bool] = {p: False for p in peers}
        while not self._stop.wait(self.interval_s):
            now = time.monotonic()
            try:
                st.add(f"{PREFIX}hb/{self.rank}", 1)
                if st.check([f"{PREFIX}abort"]):
                    msg = st.get(f"{PREFIX}abort").decode()
                    _log(f"!!! {self.tag} peer reported a pipeline failure ({msg}); exiting (exit {EXIT_ABORT})")
                    self.aborted = msg
                    self._exit()
                    return
                for p in peers:
                    if done[p]:
                        continue
                    if st.check([f"{PREFIX}done/{p}"]):
                        done[p] = True
                        continue
                    v = int(st.add(f"{PREFIX}hb/{p}", 0))
                    if v != seen[p]:
                        seen[p], changed[p] = v, now
                    elif now - changed[p] > self.peer_timeout_s:
                        self.abort(f"no heartbeat from rank {p} for {now - changed[p]:.1f} s")
                        return
            except Exception as e:  # noqa: BLE001 (store host gone = rank 0 gone)
                if self._stop.is_set():
                    return
                self.abort(f"control store unreachable ({type(e).__name__}: {e})")
                return
            if self.stall_timeout_s and self._busy and now - self._progress > self.stall_timeout_s:
                self.abort(f"no pipeline progress for {now - self._progress:.1f} s")
                return
