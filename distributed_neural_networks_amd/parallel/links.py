"""Stage-to-stage links.

The reference moves every activation GPU -> host -> protobuf -> TCP -> host ->
GPU through a new gRPC channel per request (``node.py:45-55,73-89``).  Here a
link is one direction-agnostic peer of this rank:

* ``RcclLink`` (GPU stages, the default): this package's own RCCL channel per
  rank pair (``parallel/rccl.py`` over ``csrc/comm/p2p.cpp``) — device
  buffers straight over the xGMI link between the two stage GPUs;
* ``P2PLink``: ``torch.distributed`` isend/irecv — gloo on CPU, or
  ProcessGroupNCCL with ``DNN_P2P=torch``;
* ``HostStagedLink``: gloo between ranks that compute on a GPU (``gloo_gpu``).

All share one contract, stated here for RCCL:

* device buffers move GPU -> GPU, no host staging and no serialisation;
* each peer pair's transfers run on their own stream, ordered after the
  work already queued on the compute stream when the op is posted, and
  ``Work.wait()`` orders the compute stream after the transfer without
  blocking the host — so a stage never waits on the host for a hop;
* ``exchange`` posts a middle stage's send-to-next and receive-from-prev
  together; each peer pair keeps its own communicator and stream, so the two
  transfers run concurrently (see ``exchange`` for why no op is batched).

Every link counts messages and bytes (``stats``) for the METRICS line.
Message framing for open-ended streams (the CLI): a 4 x int64 header
``[kind, a, b, tag]`` precedes a request (``KIND_DATA``) or ends the stream
(``KIND_STOP``).  Static schedules (benchmarks, microbatches of one request)
move payloads without headers.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

KIND_DATA, KIND_STOP = 1, 2


class P2PLink:
    def __init__(self, peer: int, device: torch.device, group=None):
        self.peer = int(peer)
        self.device = device
        self.group = group
        self.sent_msgs = self.sent_bytes = self.recv_msgs = self.recv_bytes = 0
        self._hdr = None

    def _count_send(self, t: torch.Tensor):
        self.sent_msgs += 1
        self.sent_bytes += t.numel() * t.element_size()

    def _count_recv(self, t: torch.Tensor):
        self.recv_msgs += 1
        self.recv_bytes += t.numel() * t.element_size()

    def isend(self, t: torch.Tensor):
        if not t.is_contiguous():
            raise ValueError("P2PLink.isend needs a contiguous tensor (a copy would be freed in flight)")
        self._count_send(t)
        return dist.isend(t, self.peer, group=self.group)

    def irecv(self, out: torch.Tensor):
        self._count_recv(out)
        return dist.irecv(out, self.peer, group=self.group)

    def send(self, t: torch.Tensor) -> None:
        self.isend(t.contiguous()).wait()

    def recv(self, out: torch.Tensor) -> torch.Tensor:
        self.irecv(out).wait()
        return out

    # -- framed messages (header + payload) --------------------------------
    def send_header(self, kind: int, a: int = 0, b: int = 0, tag: int = 0) -> None:
        self.send(torch.tensor([kind, a, b, tag], dtype=torch.int64, device=self.device))

    def recv_header(self) -> List[int]:
        if self._hdr is None:
            self._hdr = torch.empty(4, dtype=torch.int64, device=self.device)
        self.recv(self._hdr)
        return [int(v) for v in self._hdr.cpu().tolist()]

    def stats(self) -> dict:
        return {"peer": self.peer, "sent_msgs": self.sent_msgs, "sent_bytes": self.sent_bytes,
                "recv_msgs": self.recv_msgs, "recv_bytes": self.recv_bytes}


def exchange(sends: Sequence[Tuple[P2PLink, torch.Tensor]], recvs: Sequence[Tuple[P2PLink, torch.Tensor]]):
    """Post several sends and receives together; returns one ``GroupWork``.

    Each op is a plain ``isend``/``irecv``, deliberately not
    ``batch_isend_irecv``: ProcessGroupNCCL runs a single P2P op on the
    two-rank communicator of its peer pair, but a *batched* op on the
    group-wide communicator, and a send posted on one is never matched by a
    receive posted on the other.  Every link in this package therefore uses
    single ops only, so every peer pair has one communicator and one stream
    (different pairs — a middle stage's prev and next, a fan-out's receivers
    — progress concurrently on their own streams)."""
    works = [link.isend(t) for link, t in sends] + [link.irecv(t) for link, t in recvs]
    return GroupWork(works) if works else None


class GroupWork:
    """The works of one ``exchange`` group; ``wait`` is idempotent so every
    slot that depends on the group can wait on it."""

    def __init__(self, works):
        self.works = list(works)

    def wait(self):
        while self.works:
            self.works.pop(0).wait()
        return True


class HostStagedLink(P2PLink):
    """A gloo link between ranks whose stages compute on a GPU (transport
    ``gloo_gpu``: several ranks sharing one device — RCCL refuses two ranks on
    one GPU — so the multi-process schedules run with device compute and HIP
    graphs on a 1-GPU box).  Each hop goes device -> pinned host -> gloo ->
    pinned host -> device, ordered with streams and events the way RCCL
    orders its P2P:

    * ``isend(t)`` reads ``t`` after the work queued on the current stream
      when it is posted (a side stream waits on it, copies to pinned memory);
    * ``irecv(out)`` records the current stream when posted; its ``wait()``
      lands the bytes in ``out`` on the side stream *after that event only*
      and makes the current stream wait for the copy — so, exactly as with
      RCCL, the receive may overwrite ``out`` concurrently with compute
      queued after the post, and a schedule that reuses a slot too early races
      here too instead of passing by accident."""

    def __init__(self, peer: int, device: torch.device, group=None):
        super().__init__(peer, device, group)
        self._side = torch.cuda.Stream(device)
        self._sendq = None  # sender thread's queue (started on the first isend)

    @staticmethod
    def _host_like(t: torch.Tensor) -> torch.Tensor:
        return torch.empty(t.numel() * t.element_size(), dtype=torch.uint8, pin_memory=True)

    def _sender(self):
        """One thread per link posts the gloo sends in order, each once its
        device->host copy has landed, so ``isend`` never blocks the host on
        the compute queued before it (as an RCCL send does not).  The thread
        holds the queue, not the link: ``close()`` — or the link being
        garbage-collected — puts the stop sentinel, so rings and links built
        and dropped by a long process do not leave idle threads behind."""
        import queue
        import threading
        import weakref
        q = self._sendq = queue.Queue()
        peer, group = self.peer, self.group

        def run():
            while True:
                item = q.get()
                if item is None:
                    return
                ev, host, box, done = item
                try:
                    ev.synchronize()
                    box.append(dist.isend(host, peer, group=group))
                except BaseException as e:  # noqa: BLE001 — re-raised by the work's wait()
                    box.append(e)
                done.set()
        self._thread = threading.Thread(target=run, name=f"hostlink-send-{peer}", daemon=True)
        self._thread.start()
        self._stop = weakref.finalize(self, q.put, None)
        # not at interpreter exit: waking the thread while the process group
        # and its gloo threads are torn down aborted the non-first ranks of the
        # gloo_gpu ring ("terminate called without an active exception"); a
        # daemon thread blocked in q.get() is simply dropped at exit, as before
        self._stop.atexit = False

    def close(self, timeout_s: float = 30.0) -> None:
        """Stop the sender thread after the sends already queued are posted."""
        if self._sendq is not None:
            self._stop()
            self._thread.join(timeout_s)
            self._sendq = None

    def isend(self, t: torch.Tensor):
        if not t.is_contiguous():
            raise ValueError("HostStagedLink.isend needs a contiguous tensor")
        import threading
        self._count_send(t)
        host = self._host_like(t)
        self._side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self._side):
            host.view(t.dtype).view(t.shape).copy_(t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(self._side)
        if self._sendq is None:
            self._sender()
        box, done = [], threading.Event()
        self._sendq.put((ev, host, box, done))
        return _HostSendWork(box, done, host)

    def irecv(self, out: torch.Tensor):
        if not out.is_contiguous():
            raise ValueError("HostStagedLink.irecv needs a contiguous tensor")
        self._count_recv(out)
        posted = torch.cuda.Event()
        posted.record(torch.cuda.current_stream(self.device))
        host = self._host_like(out)
        return _HostWork(dist.irecv(host, self.peer, group=self.group), host, out, posted, self._side)


class _HostSendWork:
    """A ``HostStagedLink`` send posted by the link's sender thread: ``wait``
    returns once the gloo send has been posted and has completed (the source
    tensor was already copied out, so no device ordering is needed)."""

    def __init__(self, box, done, host):
        self.box, self.done_ev, self.host = box, done, host
        self.done = False

    def wait(self):
        if self.done:
            return True
        self.done_ev.wait()
        w = self.box[0]
        if isinstance(w, BaseException):
            raise w
        w.wait()
        self.done = True
        return True


class _HostWork:
    """Work of a ``HostStagedLink`` op; ``wait`` is idempotent."""

    def __init__(self, work, host, out=None, posted=None, side=None):
        self.work, self.host, self.out, self.posted, self.side = work, host, out, posted, side
        self.done = False

    def wait(self):
        if self.done:
            return True
        self.work.wait()
        if self.out is not None:
            dev = self.out.device
            self.side.wait_event(self.posted)
            with torch.cuda.stream(self.side):
                self.out.copy_(self.host.view(self.out.dtype).view(self.out.shape), non_blocking=True)
            landed = torch.cuda.Event()
            landed.record(self.side)
            torch.cuda.current_stream(dev).wait_event(landed)
        self.done = True
        return True


class RcclLink(P2PLink):
    """A hop over this package's own RCCL channel (``parallel/rccl.py``,
    ``csrc/comm/p2p.cpp``): the default link between GPU stages.  Same
    contract as ``P2PLink`` — ``isend``/``irecv`` are ordered after the work
    queued on the current stream when posted, their ``wait()`` orders the
    current stream after the transfer without blocking the host — plus
    ``send_on_stream``/``recv_on_stream``, which enqueue the hop on the
    current stream itself (a HIP graph can capture it with the stage's
    kernels).  The pair's channel is opened (init started) at construction."""

    def __init__(self, peer: int, device: torch.device, group=None):
        super().__init__(peer, device, group)
        from . import rccl
        me = dist.get_rank()
        self.ch = rccl.pair_channel(me, self.peer, device, rccl.group_tag(group))
        self.pi = 1 if self.peer > me else 0  # the peer's rank inside the pair channel

    def isend(self, t: torch.Tensor):
        from .rccl import SEND, Work
        if not t.is_contiguous():
            raise ValueError("RcclLink.isend needs a contiguous tensor")
        self._count_send(t)
        return Work(self.ch, self.ch.post(SEND, t, self.pi))

    def irecv(self, out: torch.Tensor):
        from .rccl import RECV, Work
        self._count_recv(out)
        return Work(self.ch, self.ch.post(RECV, out, self.pi))

    def send_on_stream(self, t: torch.Tensor) -> None:
        from .rccl import SEND
        self._count_send(t)
        self.ch.post(SEND, t, self.pi, on_stream=True)

    def recv_on_stream(self, out: torch.Tensor) -> None:
        from .rccl import RECV
        self._count_recv(out)
        self.ch.post(RECV, out, self.pi, on_stream=True)


def p2p_mode() -> str:
    """``DNN_P2P``: ``native`` (default: ``RcclLink``) or ``torch``
    (ProcessGroupNCCL isend/irecv) for RCCL stage hops."""
    mode = os.environ.get("DNN_P2P", "native")
    if mode not in ("native", "torch"):
        raise ValueError(f"DNN_P2P must be native or torch, got {mode!r}")
    return mode


def make_link(peer: int, device: torch.device, group=None) -> P2PLink:
    """The link for this process's backend: GPU stages on RCCL use the native
    channel (``RcclLink``; ``DNN_P2P=torch``: ProcessGroupNCCL's P2P), gloo on
    CPU moves the tensor itself (``P2PLink``), gloo with a GPU stage stages
    through pinned host memory (``HostStagedLink``)."""
    if device.type == "cuda" and dist.is_initialized():
        backend = dist.get_backend(group)
        if backend == "gloo":
            return HostStagedLink(peer, device, group)
        if backend == "nccl" and p2p_mode() == "native":
            return RcclLink(peer, device, group)
    return P2PLink(peer, device, group)


_PREFLIGHT_SEQ = [0]


# bulk part of the preflight: PREFLIGHT_MSGS back-to-back messages of this many
# bytes each way per ring pair, every byte checked (the stage hops move MBs per
# microbatch; a 16-byte exchange alone would not exercise chunked transfers)
PREFLIGHT_BYTES = int(os.environ.get("DNN_PREFLIGHT_BYTES", str(4 << 20)))
PREFLIGHT_MSGS = 3


def preflight_pattern(src: int, k: int, numel: int, device) -> torch.Tensor:
    """Message ``k`` of rank ``src``'s bulk preflight: int32 values unique per
    (src, k, position), so a dropped, duplicated, reordered or truncated
    message fails the receiver's comparison."""
    i = torch.arange(numel, dtype=torch.int64, device=device)
    return ((i * 2654435761 + src * 40503 + k * 7919) & 0x7FFFFFFF).to(torch.int32)


def _preflight_bulk(nxt, prv, r: int, n: int, device, timeout_s: float) -> None:
    numel = max(1, PREFLIGHT_BYTES // 4)
    src = (r - 1) % n
    outs = [preflight_pattern(r, k, numel, device) for k in range(PREFLIGHT_MSGS)]
    ins = [torch.full((numel,), -1, dtype=torch.int32, device=device) for _ in range(PREFLIGHT_MSGS)]
    sends = lambda: [nxt.isend(t) for t in outs]  # noqa: E731
    recvs = lambda: [prv.irecv(t) for t in ins]  # noqa: E731
    works = sends() + recvs() if r % 2 == 0 else recvs() + sends()
    for w in works:
        w.synchronize(timeout_s)
    for k, t in enumerate(ins):
        bad = int((t != preflight_pattern(src, k, numel, device)).sum().item())
        if bad:
            raise RuntimeError(f"bulk preflight message {k} from rank {src}: {bad} of {numel} words differ")


def native_preflight(device: torch.device, timeout_s: float = 90.0, store=None) -> str:
    """Check the native RCCL channels before a multi-GPU run and fall back to
    ProcessGroupNCCL P2P when they do not work, so a run still produces its
    numbers: every rank exchanges 16 bytes with both ring neighbours over its
    own pair channels (even ranks send first, odd ranks receive first, so the
    two ops of a 2-rank ring on one channel match), each op bounded by
    ``timeout_s``; on the forward ring it then sends ``PREFLIGHT_MSGS``
    back-to-back messages of ``PREFLIGHT_BYTES`` (4 MiB; ``DNN_PREFLIGHT_BYTES``)
    and the receiver compares every word against the sender's pattern.  The verdict is agreed through the process group's TCP
    store (no collective: it must work when RCCL itself is what failed).  Any
    failure on any rank aborts the native channels and sets
    ``DNN_P2P=torch`` on every rank.  Returns the mode in effect:
    ``"native"``, ``"torch (native preflight failed: ...)"``, or the backend
    name when native channels do not apply (gloo, one rank, CPU)."""
    if not dist.is_initialized() or dist.get_world_size() < 2:
        return "none"
    if dist.get_backend() != "nccl" or device.type != "cuda":
        return dist.get_backend()
    if p2p_mode() != "native":
        return p2p_mode()
    r, n = dist.get_rank(), dist.get_world_size()
    err = ""
    from . import comm, rccl
    try:
        # the forward tag and the back-edge tag (its own communicators); the
        # ring's channels are closed again afterwards (scope), so pairs no
        # pipeline uses do not keep a communicator, stream and event ring
        with rccl.scope(device):
            for tag, grp in (("world", None), ("back", comm.back_group())):
                nxt, prv = make_link((r + 1) % n, device, grp), make_link((r - 1) % n, device, grp)
                for link in (nxt, prv):
                    link.ch.ready(timeout_s)
                a = torch.full((4,), r, dtype=torch.int32, device=device)
                b = torch.full((4,), -1, dtype=torch.int32, device=device)
                works = [nxt.isend(a), prv.irecv(b)] if r % 2 == 0 else [prv.irecv(b), nxt.isend(a)]
                for w in works:
                    w.synchronize(timeout_s)
                got = int(b[0].item())
                if got != (r - 1) % n:
                    raise RuntimeError(f"{tag} ring payload {got}, expected {(r - 1) % n}")
                if tag == "world" and PREFLIGHT_BYTES > 0:
                    _preflight_bulk(nxt, prv, r, n, device, timeout_s)
    except Exception as e:  # noqa: BLE001 — any failure means: fall back
        err = f"rank {r}: {type(e).__name__}: {e}"[:200]
    st = store or rccl._store()
    seq = _PREFLIGHT_SEQ[0]
    _PREFLIGHT_SEQ[0] += 1
    st.set(f"dnn/preflight/{seq}/{r}", err or "ok")
    errs = []
    for q in range(n):
        v = st.get(f"dnn/preflight/{seq}/{q}").decode(errors="replace")
        if v != "ok":
            errs.append(v)
    if not errs:
        return "native"
    rccl.abort_all()
    rccl.destroy_all()
    os.environ["DNN_P2P"] = "torch"
    return f"torch (native preflight failed: {errs[0]})"


class SplitLink:
    """One logical stage hop over several peers: a tensor sent through it is
    cut into ``len(links)`` equal row slices, slice j going to ``links[j]``; a
    receive assembles its rows from the same slices of every peer, slice a
    from ``links[a]``.  Used for the bipartite hop of the multi-GPU CIFAR
    pipeline (every stage-0 GPU feeds every stage-1 GPU, each pair over its
    own xGMI link), so one microbatch's transfer is spread over all links
    instead of queueing on one.  Same ``isend``/``irecv`` contract as
    ``P2PLink``; rows must divide evenly."""

    def __init__(self, links: Sequence[P2PLink]):
        if not links:
            raise ValueError("SplitLink needs at least one link")
        self.links = list(links)
        self.peer = self.links[0].peer if len(self.links) == 1 else tuple(l.peer for l in self.links)

    def _slices(self, t: torch.Tensor):
        n = len(self.links)
        if t.shape[0] % n:
            raise ValueError(f"SplitLink: {t.shape[0]} rows do not split into {n} equal slices")
        if not t.is_contiguous():
            raise ValueError("SplitLink needs a contiguous tensor")
        sl = t.shape[0] // n
        return [t[j * sl:(j + 1) * sl] for j in range(n)]

    def isend(self, t: torch.Tensor):
        return GroupWork([l.isend(p) for l, p in zip(self.links, self._slices(t))])

    def irecv(self, out: torch.Tensor):
        return GroupWork([l.irecv(p) for l, p in zip(self.links, self._slices(out))])

    def send(self, t: torch.Tensor) -> None:
        self.isend(t).wait()

    def recv(self, out: torch.Tensor) -> torch.Tensor:
        self.irecv(out).wait()
        return out

    def stats(self) -> dict:
        return {"peers": [l.stats() for l in self.links]}


def wait(work: Optional[object]) -> None:
    if work is not None:
        work.wait()
