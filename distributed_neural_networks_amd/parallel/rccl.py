"""Native RCCL data plane: Python face of ``csrc/comm/p2p.cpp``.

The SURVEY §7.1 data plane: stage hops go straight to RCCL
(``ncclSend``/``ncclRecv``) on channels this package owns, not through
ProcessGroupNCCL's P2P.

* ``Channel``: one RCCL communicator (a peer pair or a 1-rank loopback) with
  its own high-priority transfer stream and a ring of completion events.  The
  lower rank of a pair draws the RCCL unique id and publishes it in the
  process group's TCP store; the higher rank reads it, and both run the
  collective init, on a background thread, so opening a channel never blocks
  and a rank may open its channels in any order, interleaved with collectives
  — ProcessGroupNCCL instead inits a pair's communicator lazily and blocking
  inside the first op, which deadlocks when two stages meet their links in
  different orders.
* ``RcclLink``: the ``P2PLink`` contract (``isend``/``irecv`` -> work with a
  stream-ordered ``wait``) over a pair channel, plus ``send_on_stream`` /
  ``recv_on_stream`` that enqueue the hop as plain stream work (HIP graph
  capture of recv -> stage kernels -> send).
* ``abort_all`` / ``destroy_all``: the watchdog and ``comm.shutdown`` hooks; an
  aborted channel's in-flight RCCL kernels return instead of spinning on a
  dead peer.

One channel per (tag, rank pair): forward traffic uses tag ``"world"``, the
pipeline back-edge tag ``"back"`` (``comm.back_group``), so a return rank's
pre-posted receives never queue in front of its forward sends to the same
peer.  ``DNN_P2P=torch`` switches ``links.make_link`` back to
ProcessGroupNCCL's isend/irecv.

Reference behaviour replaced: the per-request gRPC channel of
``node.py:45-55,73-89`` (device -> host -> protobuf -> TCP -> host -> device).
"""
from __future__ import annotations

import collections
import contextlib
import os
import threading
from typing import Dict, Optional, Sequence, Tuple

import torch

SEND, RECV = 0, 1
INIT_TIMEOUT_S = float(os.environ.get("DNN_RCCL_INIT_TIMEOUT_S", "300"))

_CHANNELS: Dict[Tuple[str, Tuple[int, ...]], "Channel"] = {}
_LOCK = threading.Lock()
_SCOPES: list = []  # open scope() frames, innermost last: keys of the channels each one opened
# opens per (tag, rank pair) in this process.  Both ranks of a pair open (and
# scope-close) its channel the same number of times in the same order, so the
# count names one generation of the pair's unique id in the store: a reopen
# never reads the id of a communicator that has already been destroyed.
_OPENS: Dict[Tuple[str, Tuple[int, ...]], int] = {}


def _lib():
    from ..ops._lib import lib
    return lib()


def available() -> bool:
    """The kernel library is built and librccl resolves in this process."""
    try:
        return bool(_lib().comm_available())
    except RuntimeError:
        return False


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


class Channel:
    """One RCCL communicator with its transfer stream (``csrc/comm/p2p.cpp``).

    Construction never blocks: the unique id fetch (``uid_fn``, the higher rank
    of a pair reads it from the store) and the collective communicator init run
    on a background thread; ``ready()`` joins it.  So no ordering of channel
    creation against collectives or other channels can deadlock."""

    def __init__(self, uid: Optional[bytes], nranks: int, rank: int, device: torch.device, key=None, uid_fn=None):
        if device.type != "cuda":
            raise ValueError("RCCL channels need a GPU device")
        self.nranks, self.rank, self.device, self.key = nranks, rank, device, key
        self.h = None
        self._err: Optional[BaseException] = None
        self._ready = False
        self._keep = collections.deque()  # (token, tensor): buffers alive until their op completed
        self.closed = False
        self._abort_requested = False
        self._hlock = threading.Lock()

        def init():
            try:
                u = uid if uid is not None else bytes(uid_fn())
                # async create: the handle exists before the collective init
                # finishes, so abort() can reach a channel whose peer never comes
                h = _lib().comm_create(u, nranks, rank, device.index, 1)
                with self._hlock:
                    self.h = h
                    if self._abort_requested:
                        _lib().comm_abort(h)
                if _lib().comm_wait_ready(h, -1) != 0:  # the init's verdict (GIL released while waiting)
                    raise RuntimeError(_lib().comm_last_error())
            except BaseException as e:  # noqa: BLE001 — re-raised by ready()
                self._err = e

        self._thread = threading.Thread(target=init, name=f"rccl-init-{key}", daemon=True)
        self._thread.start()

    # -- lifecycle -----------------------------------------------------------------
    def ready(self, timeout_s: float = INIT_TIMEOUT_S) -> "Channel":
        if self._ready:
            return self
        self._thread.join(timeout_s)
        if self._thread.is_alive():
            raise TimeoutError(f"RCCL channel {self.key}: communicator init not finished after {timeout_s:.0f} s "
                               "(peer rank never opened its end?)")
        if self._err is not None:
            raise RuntimeError(f"RCCL channel {self.key}: init failed: {self._err}") from self._err
        self._ready = True
        return self

    def abort(self) -> None:
        """Make in-flight ops return; also reaches a channel whose init is
        still waiting for its peer (the init then fails instead of blocking)."""
        with self._hlock:
            self._abort_requested = True
            h = self.h
        if not self.closed and h is not None:
            _lib().comm_abort(h)

    def destroy(self) -> None:
        if not self.closed:
            self.closed = True
            self._keep.clear()
            if self.h is not None:
                _lib().comm_destroy(self.h)

    # -- ops -------------------------------------------------------------------------
    def _stream(self, stream) -> int:
        return (stream or torch.cuda.current_stream(self.device)).cuda_stream

    def _check(self, rc: int, what: str) -> int:
        if rc < 0:
            raise RuntimeError(f"RCCL channel {self.key}: {what} failed: {_lib().comm_last_error()}")
        return rc

    def _retain(self, tok: int, tensors) -> None:
        keep = self._keep
        while keep and _lib().comm_query(self.h, keep[0][0]) == 1:
            keep.popleft()
        keep.append((tok, tensors))

    def post(self, kind: int, t: torch.Tensor, peer: int, stream=None, on_stream: bool = False) -> int:
        """One send (kind 0) / recv (kind 1) of ``t``'s bytes.  Channel stream:
        ordered after the work queued on ``stream`` (default: current) when
        posted; returns the completion token.  ``on_stream``: enqueued on
        ``stream`` itself (graph capture); returns 0."""
        self.ready()
        if not t.is_contiguous():
            raise ValueError("RCCL ops need contiguous tensors")
        tok = self._check(_lib().comm_post(self.h, kind, t.data_ptr(), _nbytes(t), peer, self._stream(stream),
                                           int(on_stream)), "send" if kind == SEND else "recv")
        if not on_stream:
            self._retain(tok, t)
        return tok

    def group(self, ops: Sequence[Tuple[int, torch.Tensor, int]], stream=None, on_stream: bool = False) -> int:
        """Several (kind, tensor, peer) ops as one RCCL group (they progress
        together; the only legal form of a send to self)."""
        self.ready()
        for _, t, _ in ops:
            if not t.is_contiguous():
                raise ValueError("RCCL ops need contiguous tensors")
        tok = self._check(_lib().comm_group(self.h, [k for k, _, _ in ops], [t.data_ptr() for _, t, _ in ops],
                                            [_nbytes(t) for _, t, _ in ops], [p for _, _, p in ops],
                                            self._stream(stream), int(on_stream)), "group")
        if not on_stream:
            self._retain(tok, [t for _, t, _ in ops])
        return tok

    def wait(self, tok: int, stream=None) -> None:
        """``stream`` (default: current) waits device-side for the op."""
        self._check(_lib().comm_wait(self.h, tok, self._stream(stream)), "wait")

    def query(self, tok: int) -> bool:
        return self._check(_lib().comm_query(self.h, tok), "query") == 1

    def synchronize(self, tok: int, timeout_s: float = 300.0) -> None:
        rc = _lib().comm_sync(self.h, tok, int(timeout_s * 1000))
        if rc == 1:
            raise TimeoutError(f"RCCL channel {self.key}: op {tok} not complete after {timeout_s:.0f} s")
        self._check(rc, "synchronize")

    def stats(self) -> dict:
        so, sb, ro, rb = _lib().comm_stats(self.h)
        return {"sent_msgs": so, "sent_bytes": sb, "recv_msgs": ro, "recv_bytes": rb}


class Work:
    """Completion of one channel op; ``wait`` orders the caller's current
    stream after it (no host block, like ProcessGroupNCCL's ``Work.wait``) and
    is idempotent."""

    def __init__(self, ch: Channel, tok: int):
        self.ch, self.tok, self.done = ch, tok, False

    def wait(self) -> bool:
        if not self.done:
            self.ch.wait(self.tok)
            self.done = True
        return True

    def is_completed(self) -> bool:
        return self.ch.query(self.tok)

    def synchronize(self, timeout_s: float = 300.0) -> None:
        self.ch.synchronize(self.tok, timeout_s)


def _store():
    import torch.distributed as dist
    return dist.distributed_c10d._get_default_store()


def pair_channel(my_rank: int, peer: int, device: torch.device, tag: str = "world", store=None) -> Channel:
    """The channel of (tag, {my_rank, peer}); opened on first use.  Both ranks
    must open it (in any order relative to their other channels)."""
    if peer == my_rank:
        raise ValueError("a pair channel needs two ranks (use loopback() for a self channel)")
    ranks = (min(my_rank, peer), max(my_rank, peer))
    key = (tag, ranks)
    with _LOCK:
        ch = _CHANNELS.get(key)
        if ch is not None and not ch.closed:
            return ch
        st = store or _store()
        gen = _OPENS.get(key, 0) + 1
        _OPENS[key] = gen
        skey = store_key(tag, ranks, gen)
        if my_rank == ranks[0]:
            uid = _lib().comm_unique_id()
            st.set(skey, uid)
            if gen > 1:  # the previous generation's id is never read again
                _delete_key(st, store_key(tag, ranks, gen - 1))
            ch = Channel(uid, 2, 0, device, key=key)
        else:  # the id is read on the init thread: opening a channel never blocks
            ch = Channel(None, 2, 1, device, key=key, uid_fn=lambda: st.get(skey))
        _CHANNELS[key] = ch
        _note_opened(key)
        return ch


def store_key(tag: str, ranks: Tuple[int, ...], gen: int) -> str:
    """Store key of generation ``gen`` (1 = first open) of a pair's unique id."""
    return f"dnn/rccl/{tag}/{ranks[0]}-{ranks[1]}/{gen}"


def _delete_key(st, k: str) -> None:
    try:
        st.delete_key(k)
    except Exception:  # noqa: BLE001 — hygiene only (a store without delete keeps it)
        pass


def _note_opened(key) -> None:
    if _SCOPES:
        _SCOPES[-1].append(key)


def live_channels() -> int:
    """Channels currently open in this process (communicator + stream + event ring each)."""
    with _LOCK:
        return sum(1 for c in _CHANNELS.values() if not c.closed)


@contextlib.contextmanager
def scope(device: Optional[torch.device] = None):
    """Channels first opened inside the block are destroyed when it ends
    (after the device has drained), so one measurement's channel set — a
    placement's pairs, one decode ring's links — does not stay alive through
    the next.  Channels that already existed are left alone.  Nestable."""
    frame: list = []
    _SCOPES.append(frame)
    ok = False
    try:
        yield frame
        ok = True
    finally:
        # by identity: two frames that opened nothing are equal lists, and
        # list.remove would drop the outer one and orphan this one
        popped = _SCOPES.pop()
        assert popped is frame, "rccl.scope frames closed out of order"
        with _LOCK:
            chans = [_CHANNELS.pop(k) for k in frame if k in _CHANNELS]
        if chans and ok:
            dev = device or chans[0].device
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
        for c in chans:
            if not ok:  # an op may be stuck on a peer: make it return instead of draining the device
                c.abort()
            c.destroy()


def loopback(device: torch.device) -> Channel:
    """A 1-rank channel (self send/recv in groups): the single-GPU test of the
    module, and the hop of stages that share a process."""
    key = ("loopback", (device.index,))
    with _LOCK:
        ch = _CHANNELS.get(key)
        if ch is None or ch.closed:
            ch = _CHANNELS[key] = Channel(_lib().comm_unique_id(), 1, 0, device, key=key)
            _note_opened(key)
        return ch


def abort_all() -> None:
    """Watchdog hook: make every channel's in-flight RCCL kernels return."""
    for ch in list(_CHANNELS.values()):
        try:
            ch.abort()
        except Exception:  # noqa: BLE001 — best effort on the way out
            pass


def destroy_all() -> None:
    with _LOCK:
        chans = list(_CHANNELS.values())
        _CHANNELS.clear()
    for ch in chans:
        ch.destroy()


def group_tag(group) -> str:
    from . import comm
    if group is None:
        return "world"
    if group is comm._BACK_GROUP:
        return "back"
    import torch.distributed as dist
    # other groups: named by their ranks (the same on every member; two
    # groups over the same ranks would share channels)
    return "g" + "-".join(str(r) for r in dist.get_process_group_ranks(group))
