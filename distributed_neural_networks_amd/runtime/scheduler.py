"""Microbatch schedules for one pipeline rank (forward-only inference).

The reference keeps exactly one request in flight: stage i's handler blocks on
the nested RPC to stage i+1 for the whole downstream latency (``node.py:70-94``)
and the driver sends one hard-coded request (``node.py:173``), so with S stages
S-1 devices idle.  This module holds the schedules that keep every stage busy;
the CLI (``node.py``), ``bench.py`` and ``bench/gpt_bench.py`` all run them:

* ``run_gpipe`` — forward-only GPipe fill/drain of M microbatches through this
  rank's stage (CIFAR, prefill-style work).  Receives land in a ``depth``-deep
  slot ring and are posted ``depth`` microbatches ahead; the send of microbatch
  i overlaps the compute of i+1.  Slot reuse is ordered by the P2P work handles.
* ``ForwardPipeline`` — the open-ended request stream of the CLI on top of
  ``run_gpipe``: stage 0 splits each request into ``num_microbatches``
  microbatches of ``micro_batch_size`` rows, a 4-int64 header announces the
  shape to the downstream ranks, and the last stage returns per-row
  predictions over the back-edge to ``return_to_node_id`` (resolved but unused
  in the reference, ``node.py:272-277``).
* ``DecodeRing`` — autoregressive decode with M microbatches circulating
  stage group 0 -> ... -> last -> (sampled token ids over the back-edge) ->
  stage group 0.  With M >= #groups every rank works on a different microbatch
  at any time.  On a GPU each microbatch's decode compute for this rank is one
  HIP graph; the P2P hops stay outside the graph.

Ordering rules (``Link`` = ``parallel/links.py``): an ``isend``'s source buffer
may be overwritten only after the send's work was waited on (on RCCL that makes
the compute stream wait on the transfer, no host block); a receive may target a
buffer the previous microbatch's compute still reads, because RCCL enqueues the
receive behind the work already queued on the compute stream (gloo runs
compute synchronously).  ``DNN_DEBUG_ORDER=1`` checks the slot protocol
(``runtime/ordering.py``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence

import torch

from ..parallel.links import exchange
from ..utils import trace
from .ordering import SlotOrder
from .stages import StageCompute, StageOutput

Progress = Optional[Callable[[], None]]


def _noop():
    return None


# --------------------------------------------------------------------------- stage chains
class StageChain(StageCompute):
    """Several consecutive stages hosted by one rank (or one GPU), chained over
    preallocated intermediate buffers: to the schedule they are one stage."""

    def __init__(self, stages: Sequence[StageCompute]):
        self.stages = list(stages)
        self.first, self.last = self.stages[0].first, self.stages[-1].last
        self.device = self.stages[0].device
        self._mid: Dict[int, List[torch.Tensor]] = {}

    def in_spec(self, batch):
        return self.stages[0].in_spec(batch)

    def out_spec(self, batch):
        return self.stages[-1].out_spec(batch)

    def forward(self, x, out=None):
        B = x.shape[0]
        mids = self._mid.get(B)
        if mids is None:
            mids = []
            for s in self.stages[:-1]:
                shp, dt = s.out_spec(B)
                mids.append(torch.empty(shp, dtype=dt, device=self.device))
            self._mid[B] = mids
        h = x
        for s, buf in zip(self.stages[:-1], mids):
            h = s.forward(h, buf)
        return self.stages[-1].forward(h, out)


def as_stage(stages) -> StageCompute:
    if isinstance(stages, StageCompute) or hasattr(stages, "forward"):
        return stages
    stages = list(stages)
    return stages[0] if len(stages) == 1 else StageChain(stages)


# --------------------------------------------------------------------------- GPipe forward stream
def run_gpipe(stage, M: int, batch: int, prev=None, nxt=None,
              source: Optional[Callable[[int], torch.Tensor]] = None,
              sink: Optional[Callable[[int, object], None]] = None, depth: int = 2,
              progress: Progress = None) -> None:
    """Stream M microbatches of ``batch`` rows through this rank's stage(s).

    ``prev``/``nxt`` are links to the neighbouring ranks (None at the ends);
    the first rank pulls inputs from ``source(i)``, every rank may observe its
    outputs with ``sink(i, y)`` (the last rank gets ``StageOutput``).  ``prev``
    may be a list of links (fan-in from replicated upstream ranks): microbatch i
    then comes from ``prev[i % len(prev)]``, each sender's stream in order."""
    stage = as_stage(stage)
    prevs = list(prev) if isinstance(prev, (list, tuple)) else ([prev] if prev is not None else [])
    prev = prevs[0] if prevs else None

    def src_link(i):
        return prevs[i % len(prevs)]
    progress = progress or _noop
    dev = stage.device
    ishp, idt = stage.in_spec(batch)
    oshp, odt = stage.out_spec(batch)
    depth = max(1, min(depth, M))
    in_slots = [torch.empty(ishp, dtype=idt, device=dev) for _ in range(depth)] if prev is not None else []
    out_slots = [torch.empty(oshp, dtype=odt, device=dev) for _ in range(depth)]
    rwork: List[object] = [None] * depth
    swork: List[object] = [None] * depth
    ins, outs = SlotOrder("in_slots", depth), SlotOrder("out_slots", depth)
    if prev is not None:
        for k in range(depth):
            rwork[k] = src_link(k).irecv(in_slots[k])
            ins.post(k, "recv", k)
    for i in range(M):
        k = i % depth
        if prev is None:
            x = source(i)
        else:
            with trace.span("recv_wait", "p2p", mb=i):
                rwork[k].wait()
            ins.waited(k)
            ins.use(k, "stage input read", i)
            x = in_slots[k]
        if swork[k] is not None:
            with trace.span("slot_reuse_wait", "p2p", mb=i):
                swork[k].wait()
            swork[k] = None
            outs.waited(k)
        outs.use(k, "stage output write", i)
        with trace.span("stage_forward", "compute", device=dev, mb=i):
            y = stage.forward(x, out_slots[k])
        post_recv = prev is not None and i + depth < M
        send_t = (y if isinstance(y, torch.Tensor) else y.probs) if nxt is not None else None
        if post_recv and send_t is not None:
            # middle stage: send(i) -> next and recv(i+depth) <- prev as one group
            w = exchange([(nxt, send_t)], [(src_link(i + depth), in_slots[k])])
            rwork[k] = swork[k] = w
        elif post_recv:
            rwork[k] = src_link(i + depth).irecv(in_slots[k])  # queued behind this slot's compute
        elif send_t is not None:
            swork[k] = nxt.isend(send_t)
        if post_recv:
            ins.post(k, "recv", i + depth)
        if send_t is not None:
            outs.post(k, "send", i)
        if sink is not None:
            sink(i, y)
        progress()
    for k, w in enumerate(swork):
        if w is not None:
            w.wait()
            outs.waited(k)
    ins.drained()
    outs.drained()


# --------------------------------------------------------------------------- CLI forward stream
KIND_DATA, KIND_STOP = 1, 2


@dataclass
class ForwardLinks:
    prev: object = None          # link to part_index - 1
    nxt: object = None           # link to part_index + 1
    ret_out: object = None       # last stage -> return rank (back-edge), None if last == return rank
    ret_in: object = None        # return rank <- last stage


class ForwardPipeline:
    """Request stream of the CLI over ``run_gpipe`` (CIFAR-style stages).

    Each request of ``mbs * M`` rows is announced by a header
    ``[KIND_DATA, mbs, M, tag]`` and streamed as M microbatches; ``stop()``
    sends ``KIND_STOP`` down the chain.  The last stage sends each microbatch's
    per-row predictions (int32) to the return rank over the back-edge.
    ``on_result(role, tag, preds)`` is called with role ``"last"`` on the last
    stage and ``"return"`` on the return rank (host int32 predictions).
    """

    def __init__(self, stage, links: ForwardLinks, is_first: bool, is_last: bool, is_ret: bool,
                 depth: int = 2, progress: Progress = None, on_result: Optional[Callable] = None):
        self.stage = as_stage(stage)
        self.links = links
        self.is_first, self.is_last, self.is_ret = is_first, is_last, is_ret
        self.depth = depth
        self.progress = progress or _noop
        self.on_result = on_result or (lambda role, tag, preds: None)
        self._slots: Dict[tuple, List[torch.Tensor]] = {}

    def _send_header(self, kind, a=0, b=0, tag=0):
        if self.links.nxt is not None:
            self.links.nxt.send_header(kind, a, b, tag)

    def _stream(self, mbs: int, M: int, tag: int, source=None) -> Optional[torch.Tensor]:
        """This rank's part of one request; returns the last stage's predictions.

        The last stage gives every microbatch its own back-edge slot and waits
        on those sends only after the stream: a send that completes only once
        the return rank has posted its receive (gloo) can never stall the
        forward stream, whatever ``M`` is."""
        local: Dict[int, torch.Tensor] = {}
        work: List[object] = []
        sink = None
        if self.is_last:
            slots = self._slots.get((mbs, M))
            if slots is None:
                slots = self._slots[(mbs, M)] = [torch.empty((mbs,), dtype=torch.int32, device=self.stage.device)
                                                 for _ in range(M)]

            def sink(i, y: StageOutput):
                local[i] = y.pred.clone()
                if self.links.ret_out is not None:
                    slots[i].copy_(y.pred)
                    work.append(self.links.ret_out.isend(slots[i]))
        run_gpipe(self.stage, M, mbs, self.links.prev, self.links.nxt, source=source, sink=sink,
                  depth=self.depth, progress=self.progress)
        for w in work:
            w.wait()
        if not self.is_last:
            return None
        preds = torch.cat([local[i] for i in range(M)]).cpu()
        self.on_result("last", tag, preds)
        return preds

    def _post_collect(self, mbs: int, M: int):
        """Return rank: post the receives of all M prediction slots before
        streaming (the back-edge travels on its own communicator,
        ``comm.back_group``, so these never queue ahead of forward traffic)."""
        dev = self.stage.device
        preds = [torch.empty((mbs,), dtype=torch.int32, device=dev) for _ in range(M)]
        return preds, [self.links.ret_in.irecv(p) for p in preds]

    def _request(self, mbs: int, M: int, tag: int, source=None) -> Optional[torch.Tensor]:
        pending = self._post_collect(mbs, M) if (self.is_ret and self.links.ret_in is not None) else None
        own = self._stream(mbs, M, tag, source)
        if not self.is_ret:
            return None
        if pending is None:
            preds = own
        else:
            bufs, works = pending
            for w in works:
                w.wait()
                self.progress()
            preds = torch.cat(bufs).cpu()
        self.on_result("return", tag, preds)
        return preds

    def run_request(self, x: torch.Tensor, mbs: int, M: int, tag: int = 0) -> Optional[torch.Tensor]:
        """Stage 0: stream one request (``x`` has ``mbs * M`` rows, on the
        stage's device).  Returns the per-row predictions when this rank is
        the return rank."""
        if not self.is_first or x.shape[0] != mbs * M:
            raise ValueError(f"run_request: stage 0 needs mbs*M = {mbs * M} rows, got {tuple(x.shape)}")
        self._send_header(KIND_DATA, mbs, M, tag)
        return self._request(mbs, M, tag, source=lambda i: x[i * mbs:(i + 1) * mbs])

    def serve(self) -> int:
        """Ranks > 0: process requests until ``KIND_STOP``; returns the count."""
        n = 0
        while True:
            kind, mbs, M, tag = self.links.prev.recv_header()
            self.progress()
            if kind == KIND_STOP:
                self._send_header(KIND_STOP)
                return n
            self._send_header(KIND_DATA, mbs, M, tag)
            self._request(mbs, M, tag)
            n += 1

    def stop(self):
        self._send_header(KIND_STOP)


# --------------------------------------------------------------------------- decode ring
@dataclass
class RingLinks:
    prev: object = None       # hidden states from the previous group
    nxt: object = None        # hidden states to the next group
    back_out: object = None   # last group: sampled ids -> group 0
    back_in: object = None    # group 0: sampled ids <- last group


def _act_dtype(st) -> torch.dtype:
    return getattr(st, "act_dtype", torch.bfloat16)


class DecodeRing:
    """Microbatched autoregressive decode over a pipeline of stage groups.

    ``stages``: this rank's consecutive transformer stages (``step`` API of
    ``runtime/transformer.py`` / ``TorchStage``).  ``n_groups`` ranks form the
    ring; microbatch m owns KV-cache rows ``[m*B, (m+1)*B)`` on every stage.
    Group 0 holds the token state; it receives every sampled token over the
    back-edge (or, with one group, the graph writes it in place).
    """

    def __init__(self, stages: Sequence, links: RingLinks, n_groups: int, M: int, B: int,
                 use_graphs: bool = True, record: bool = True, progress: Progress = None, lanes: int = 0,
                 multi_step: int = -1):
        """``lanes`` (one group, M > 1, GPU): the M microbatch steps of a round
        replay on this many HIP streams (0 = one stream, -1 = min(M, 4));
        scratch rows follow the KV rows (``TransformerStage.step``), so
        concurrent microbatches share no buffer.  Off by default: measured on
        GPT-2 4-stage (profiles/archive/r2_decode_lanes_gpt2.jsonl) concurrent small
        microbatches beat the same microbatches on one stream (16 x 4: 2.17 ->
        0.88 ms/round) but not one large batch (64 x 1: 0.60 ms).

        ``multi_step`` (one group, GPU, graphs, no lanes): K >= 2 decode rounds
        of all M microbatches are also captured as ONE HIP graph, and
        ``decode_rounds`` replays it while K or more rounds remain (single-step
        graphs for the rest): the graph-to-graph boundary after every step's
        argmax (profiles/r4_gpt2_b64_decode_gaps.md) is paid once per K steps.
        Positions and input ids live on the device; a greedy last stage writes
        each step's token into a device history (``hist``, indexed by
        position) in its argmax launch, so recording costs nothing per step.
        -1 = ``$DNN_DECODE_MULTISTEP`` or 8; 0 / 1 = off."""
        self.stages = list(stages)
        self.links = links
        self.G, self.M, self.B = n_groups, M, B
        self.first, self.last = self.stages[0].first, self.stages[-1].last
        self.dev = self.stages[0].device
        self.progress = progress or _noop
        self.record = record
        st0 = self.stages[0]
        self.d = st0.d if hasattr(st0, "d") else st0.cfg.n_embd
        for s in self.stages:
            mb = getattr(s, "max_batch", None)
            if mb is not None and mb < M * B:
                raise ValueError(f"stage KV cache holds {mb} sequences, the ring needs M*B = {M * B}")
        dev = self.dev
        self.pos = [torch.zeros((B,), dtype=torch.int32, device=dev) for _ in range(M)]
        self.cur = [torch.zeros((B, 1), dtype=torch.int32, device=dev) for _ in range(M)] if self.first else None
        in_dt = _act_dtype(self.stages[0])
        out_dt = _act_dtype(self.stages[-1])
        # one input slot per microbatch: the receive of microbatch m+1 can land
        # while microbatch m's graph still reads its own slot
        self.xin = [torch.empty((B, self.d), dtype=in_dt, device=dev) for _ in range(M)] if not self.first else None
        # pre-posted receive per microbatch: hidden states (non-first ranks) or
        # the sampled token over the back-edge (group 0 with G > 1)
        self.rwork: List[object] = [None] * M
        self.rorder = SlotOrder("ring_in", M)
        self.prepost = True  # False: each input is received just before its use (the A/B baseline)
        if self.last:
            self.out = [torch.empty((B,), dtype=torch.int32, device=dev) for _ in range(M)]
        else:
            self.out = [torch.empty((B, self.d), dtype=out_dt, device=dev) for _ in range(M)]
        self.swork: List[object] = [None] * M
        # group 0 (G > 1): a sampled token of microbatch m is on its way back
        self.pending = [False] * M
        self.sorder = SlotOrder("ring_out", M)
        self.toks: List[List[torch.Tensor]] = [[] for _ in range(M)]
        self.use_graphs = use_graphs and dev.type == "cuda"
        self.graphs: Dict[int, object] = {}
        self.steps_done = 0
        n_lanes = min(M, 4) if lanes < 0 else min(M, lanes)
        self.lanes = ([torch.cuda.Stream(dev) for _ in range(n_lanes)]
                      if n_groups == 1 and n_lanes > 1 and dev.type == "cuda" else [])
        import os
        self.multi_step = int(os.environ.get("DNN_DECODE_MULTISTEP", "8")) if multi_step < 0 else multi_step
        self.graph_k = None  # the K-round graph (capture)
        self.graph_k_steps = 0
        # device token history (one group, greedy fused tail): hist[m][b, p] =
        # the token sampled at position p; tokens() reads it past the prefill
        tail = self.last and getattr(self.stages[-1], "fuses_step_tail", False)
        cap = min((getattr(s, "max_seq", 0) for s in self.stages), default=0)
        self.hist = ([torch.zeros((B, cap), dtype=torch.int32, device=dev) for _ in range(M)]
                     if n_groups == 1 and tail and cap > 0 and dev.type == "cuda" else None)
        self.hist_base = [0] * M  # position of the first decode token of the current generation
        self.hist_n = [0] * M  # decode tokens recorded in hist since then

    # -- one microbatch through this rank's stages --------------------------
    def _run(self, x, m: int, T: int, out=None, advance=None):
        h = x
        n = len(self.stages)
        for j, s in enumerate(self.stages):
            if j == n - 1 and advance is not None:
                h = s.step(h, self.pos[m], self.B, T, b0=m * self.B, out=out, advance=advance)
            else:
                h = s.step(h, self.pos[m], self.B, T, b0=m * self.B, out=out if j == n - 1 else None)
        return h

    def _decode_body(self, m: int):
        x = self.cur[m] if self.first else self.xin[m]
        # greedy last stage: the argmax launch also writes the next input ids
        # (one group) and advances the positions — no separate copy / add kernels
        if self.last and getattr(self.stages[-1], "fuses_step_tail", False):
            ids = self.cur[m].view(self.B) if self.G == 1 else None
            adv = (ids, self.pos[m]) if self.hist is None else (ids, self.pos[m], self.hist[m])
            self._run(x, m, 1, out=self.out[m], advance=adv)
            return None
        self._run(x, m, 1, out=self.out[m])
        self.pos[m].add_(1)
        if self.last and self.G == 1:
            self.cur[m].copy_(self.out[m].view(self.B, 1))
        return None

    def _out_ready(self, m: int):
        if self.swork[m] is not None:
            self.swork[m].wait()
            self.swork[m] = None
            self.sorder.waited(m)
        self.sorder.use(m, "ring output write", m)

    def _send(self, m: int):
        if self.last:
            if self.G > 1:
                self.swork[m] = self.links.back_out.isend(self.out[m])
                self.sorder.post(m, "send", m)
        else:
            self.swork[m] = self.links.nxt.isend(self.out[m])
            self.sorder.post(m, "send", m)

    def _recv_token(self, m: int):
        """Group 0: the token sampled for microbatch m arrives over the back-edge."""
        if self.G > 1:
            if not self.pending[m]:
                return  # already received (drain) — the ring resumes from cur[m]
            with trace.span("token_recv", "p2p", mb=m):
                self._wait_input(m)
            self.pending[m] = False
        if self.record:
            self.toks[m].append(self.cur[m].view(self.B).clone())

    # -- pre-posted receives ----------------------------------------------------
    def _has_input_link(self) -> bool:
        return (not self.first) or self.G > 1

    def _post_input(self, m: int) -> None:
        """Post the receive of microbatch m's next input (hidden states from the
        previous group, or the token over the back-edge).  On RCCL the
        transfer is ordered after the work queued now, so the slot's last
        reader — microbatch m's previous graph — must already be queued."""
        if self.rwork[m] is not None or not self._has_input_link():
            return
        if self.first:
            if not self.pending[m]:
                return  # no token of m in flight (drained, or m not sent yet): nothing to receive
            self.rwork[m] = self.links.back_in.irecv(self.cur[m].view(self.B))
        else:
            self.rwork[m] = self.links.prev.irecv(self.xin[m])
        self.rorder.post(m, "recv", m)

    def _wait_input(self, m: int) -> None:
        self._post_input(m)  # not pre-posted: post it now
        self.rwork[m].wait()  # stream-ordered: no host block on RCCL
        self.rwork[m] = None
        self.rorder.waited(m)

    # -- prefill ----------------------------------------------------------------
    def prefill(self, prompts: Optional[Sequence[torch.Tensor]], T: int, chunk: int = 0) -> None:
        """Run the T-token prompts of all M microbatches (group 0 passes
        ``prompts[m]`` (B, T) int; other groups pass None).  ``chunk`` > 0
        prefills in pieces of that many tokens (chunked prefill: activation
        buffers and stage hops stay bounded for long prompts; each piece
        attends to the cache written by the previous ones).

        Stages with a calibrated fp8 KV cache that is not calibrated yet
        (``needs_kv_calibration``: the same on every rank, it follows the
        config) first run this prefill ``KV_CAL_ROUNDS`` times (a fixed count,
        so every rank runs the same prefills and the ring hops match), setting
        their per-layer scales from the cache's K / V amax after each and
        clearing it; then the prefill runs for real.  Once per stage lifetime."""
        while any(getattr(s, "needs_kv_calibration", False) for s in self.stages):
            self._prefill(prompts, T, chunk)
            self.drain()
            for s in self.stages:
                if getattr(s, "needs_kv_calibration", False):
                    s.calibrate_kv()
        self._prefill(prompts, T, chunk)

    def _prefill(self, prompts, T: int, chunk: int = 0) -> None:
        B, d = self.B, self.d
        C = T if chunk <= 0 else min(chunk, T)
        pieces = [(t0, min(C, T - t0)) for t0 in range(0, T, C)]
        for m in range(self.M):
            self.pos[m].zero_()
            self.toks[m] = []
        in_dt, out_dt = _act_dtype(self.stages[0]), _act_dtype(self.stages[-1])
        xin_pf = torch.empty((B * C, d), dtype=in_dt, device=self.dev) if not self.first else None
        out_pf = None
        pf_work: List[object] = [None, None]
        if not self.last:
            out_pf = [torch.empty((B * C, d), dtype=out_dt, device=self.dev) for _ in range(2)]
        n_sent = 0
        for m in range(self.M):
            if self.first:
                ids = prompts[m].to(device=self.dev, dtype=torch.int32).contiguous()
            self._out_ready(m)
            for t0, Tc in pieces:
                final = t0 + Tc == T
                if self.first:
                    x = ids[:, t0:t0 + Tc].contiguous()
                else:
                    x = xin_pf[:B * Tc]
                    self.links.prev.recv(x)
                k = n_sent % 2
                if not self.last and pf_work[k] is not None:
                    pf_work[k].wait()
                with trace.span("prefill", "compute", mb=m, t0=t0):
                    y = self._run(x, m, Tc, out=(self.out[m] if self.last else out_pf[k][:B * Tc]))
                self.pos[m].add_(Tc)
                if not self.last:
                    pf_work[k] = self.links.nxt.isend(out_pf[k][:B * Tc])
                    n_sent += 1
                elif final:
                    if self.G == 1:
                        self.cur[m].copy_(self.out[m].view(B, 1))
                        if self.record:
                            self.toks[m].append(self.out[m].clone())
                            self.hist_base[m], self.hist_n[m] = T, 0
                    else:
                        self._send(m)
                self.progress()
        for w in pf_work:
            if w is not None:
                w.wait()
        if self.first and self.G > 1:
            self.pending = [True] * self.M  # every prompt's first token comes back over the back-edge
        self.steps_done = 0

    # -- decode -------------------------------------------------------------------
    def capture(self) -> None:
        """One HIP graph per microbatch for this rank's decode compute."""
        if not self.use_graphs or self.graphs:
            return
        from .graph import GraphedStep
        for m in range(self.M):
            snap = self.pos[m].clone()
            cur = self.cur[m].clone() if self.first else None
            self._out_ready(m)
            self.graphs[m] = GraphedStep(lambda m=m: self._decode_body(m), self.dev, warmup=1)
            self.pos[m].copy_(snap)  # the warmup/capture runs advanced the position
            if cur is not None:
                self.cur[m].copy_(cur)
        torch.cuda.synchronize(self.dev)
        self._capture_multi_step()

    def _capture_multi_step(self) -> None:
        K = self.multi_step
        if (K < 2 or self.G != 1 or self.lanes or not self.graphs or (self.record and self.hist is None)):
            return
        # the warmup and the capture each write K positions past the current
        # one into the KV caches: only when they fit
        cap = min(getattr(s, "max_seq", 1 << 30) for s in self.stages)
        if int(max(int(p.max().item()) for p in self.pos)) + K > cap:
            return
        from .graph import GraphedStep
        snap = [p.clone() for p in self.pos]
        cur = [c.clone() for c in self.cur] if self.first else None

        def body():
            for _ in range(K):
                for m in range(self.M):
                    self._decode_body(m)

        def reset():
            for m in range(self.M):
                self.pos[m].copy_(snap[m])
                if cur is not None:
                    self.cur[m].copy_(cur[m])
        self.graph_k = GraphedStep(body, self.dev, warmup=1, reset=reset)
        self.graph_k_steps = K
        reset()  # the capture run advanced them again
        torch.cuda.synchronize(self.dev)

    def decode_round(self, mbs: Optional[Sequence[int]] = None) -> None:
        """Every microbatch (or those in ``mbs``; every rank must pass the same
        list) advances one token on this rank's stages.  ``mbs=[0]`` after a
        ``drain`` lets one microbatch circulate alone: a round is then exactly
        one trip around the ring (per-token latency)."""
        self.decode_rounds(1, mbs)

    def decode_rounds(self, n: int, mbs: Optional[Sequence[int]] = None) -> None:
        """``n`` decode rounds.  The input of the next microbatch in the
        sequence (across round boundaries too, up to the last one of the
        ``n`` rounds) is received into its own slot while this one computes:
        its receive is posted *before* this microbatch's graph is launched
        (``run_gpipe``'s depth-ahead receive), so on RCCL the hop of
        microbatch m+1 overlaps the compute of m instead of being queued
        behind it.  A receive is never posted for a microbatch whose previous
        graph is not queued yet (one microbatch: no pre-post)."""
        if self.lanes and mbs is None:
            for _ in range(n):
                self._decode_round_lanes()
            return
        if self.graph_k is not None and mbs is None:
            K = self.graph_k_steps
            while n >= K and self.multi_step >= K:
                with trace.span("decode", "compute", mb=-1, step=self.steps_done, rounds=K):
                    self.graph_k()
                self.steps_done += K
                for m in range(self.M):
                    self.hist_n[m] += K
                self.progress()
                n -= K
            if n == 0:
                return
        order = list(range(self.M) if mbs is None else mbs)
        seq = [m for _ in range(n) for m in order]
        G = self.G
        for i, m in enumerate(seq):
            if self.first and G > 1:
                self._recv_token(m)
            elif not self.first:
                with trace.span("hidden_recv", "p2p", mb=m):
                    self._wait_input(m)
            self.rorder.use(m, "ring input read", m)
            nxt_m = seq[i + 1] if i + 1 < len(seq) else None
            if self.prepost and nxt_m is not None and nxt_m != m and self._has_input_link():
                self._post_input(nxt_m)  # its slot's last reader was queued in an earlier item
            self._out_ready(m)
            with trace.span("decode", "compute", mb=m, step=self.steps_done):
                if m in self.graphs:
                    self.graphs[m]()
                else:
                    self._decode_body(m)
            self._send(m)
            if self.first and G > 1:
                self.pending[m] = True
            if self.first and G == 1 and self.record:
                self._record_step(m)
            if i + 1 == len(seq) or (i + 1) % len(order) == 0:
                self.steps_done += 1
            self.progress()

    def _decode_round_lanes(self) -> None:
        """One group, M microbatches on ``len(self.lanes)`` streams: the round
        forks from the current stream and joins back into it, so host-visible
        state (recorded tokens, the next prefill) is ordered as on one stream."""
        cur = torch.cuda.current_stream(self.dev)
        for s in self.lanes:
            s.wait_stream(cur)
        for m in range(self.M):
            s = self.lanes[m % len(self.lanes)]
            with torch.cuda.stream(s):
                with trace.span("decode", "compute", mb=m, step=self.steps_done, lane=m % len(self.lanes)):
                    if m in self.graphs:
                        self.graphs[m]()
                    else:
                        self._decode_body(m)
                if self.record:
                    self._record_step(m)
            self.progress()
        for s in self.lanes:
            cur.wait_stream(s)
        self.steps_done += 1

    def drain(self) -> None:
        """End of generation: group 0 receives the last sampled tokens; every
        rank waits for its outstanding sends."""
        if self.first and self.G > 1:
            for m in range(self.M):
                self._recv_token(m)  # only the tokens still in flight
                self.progress()
        for m in range(self.M):
            if self.swork[m] is not None:
                self.swork[m].wait()
                self.swork[m] = None
                self.sorder.waited(m)
        self.sorder.drained()
        self.rorder.drained()  # decode_rounds never leaves a receive posted past its last item

    def generate(self, prompts, T: int, steps: int, chunk: int = 0) -> Optional[torch.Tensor]:
        """Prefill + ``steps - 1`` decode rounds (``steps`` tokens per sequence).
        Group 0 returns (M*B, steps) int32 on the host; other groups None."""
        self.prefill(prompts, T, chunk)
        if steps > 1:
            self.capture()
        if steps > 1:
            self.decode_rounds(steps - 1)
        self.drain()
        return self.tokens() if self.first else None

    def _record_step(self, m: int) -> None:
        """One group: the token of microbatch m's decode step just queued."""
        if self.hist is not None:
            self.hist_n[m] += 1  # written on the device by the argmax launch
        else:
            self.toks[m].append(self.cur[m].view(self.B).clone())

    def tokens(self) -> torch.Tensor:
        rows = []
        for m, t in enumerate(self.toks):
            parts = [torch.stack(t, 1)] if t else []
            if self.hist is not None and self.hist_n[m]:
                b = self.hist_base[m]
                parts.append(self.hist[m][:, b:b + self.hist_n[m]])
            rows.append(torch.cat(parts, 1))
        return torch.cat(rows, 0).cpu()
