"""CLI generation drivers for the transformer families (GPT-2 / Llama-3).

The reference's GPT stages exist only as modules (``partitions/
gpt_model_parts.py:6-50``) that recompute the whole prefix per call; nothing
drives them (``node.py`` registers CIFAR parts only, ``node.py:29-32``).  Here
the config's ``micro_batch_size`` x ``num_microbatches`` sequences are decoded
greedily (or sampled) through the pipeline with the ``DecodeRing`` schedule
(``runtime/scheduler.py``):

* ``run_generate_colocated`` — every stage on one GPU (one ring group, each
  microbatch's decode step one HIP graph);
* ``run_generate_dist`` — one rank per stage over RCCL / gloo, tokens return to
  stage 0 over the back-edge.

Stage 0 prints the reference's ``***** FINAL PREDICTION (Index): k *****`` line
(first generated token of the first sequence), the generated tokens, and one
``METRICS`` JSON line with prefill / decode token rates.
"""
from __future__ import annotations

import json
import time
from typing import List, Optional

import torch

from ..models import model_info
from ..utils.log import log
from .scheduler import DecodeRing, RingLinks


def make_prompts(pipe, prompt: Optional[str], replica: int = 0) -> torch.Tensor:
    """(micro_batch_size * num_microbatches, T) int64 prompt ids: ``--prompt``
    (comma-separated ids, replicated to every sequence) or seeded random ids
    (each data-parallel replica draws its own batch)."""
    info = model_info(pipe.model)
    n = pipe.micro_batch_size * pipe.num_microbatches
    if prompt:
        ids = [int(v) for v in prompt.split(",") if v.strip()]
        return torch.tensor([ids], dtype=torch.int64).repeat(n, 1)
    g = torch.Generator().manual_seed(1234 + 7919 * replica)
    T = pipe.prompt_len or pipe.seq_len
    return torch.randint(0, info.cfg.vocab_size, (n, T), generator=g)


def kv_capacity(pipe, T: int) -> tuple:
    """(sequences, positions) every stage's KV cache must hold."""
    return pipe.micro_batch_size * pipe.num_microbatches, T + max(1, pipe.decode_steps or 1)


def check_capacity(stages, n_seq: int, n_pos: int) -> None:
    for s in stages:
        mb, ms = getattr(s, "max_batch", None), getattr(s, "max_seq", None)
        if mb is not None and mb < n_seq:
            raise ValueError(f"stage KV cache holds {mb} sequences, the run needs {n_seq}")
        if ms is not None and ms < n_pos:
            raise ValueError(f"stage KV cache holds {ms} positions, the run needs {n_pos} (prompt + decode steps)")
        bs = getattr(getattr(s, "cfg", None), "block_size", None)
        if bs is not None and n_pos > bs:
            raise ValueError(f"prompt + decode steps = {n_pos} exceeds the model's block_size {bs}")


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _report(nid: str, toks: torch.Tensor, prefill_s: float, decode_s: float, n_seq: int, T: int, steps: int,
            M: int, groups: int) -> None:
    first = toks[:, 0].tolist()
    log(f"[{nid}] ***** FINAL PREDICTION (Index): {first[0] if len(first) == 1 else first} *****")
    log(f"[{nid}] generated tokens: {json.dumps(toks.tolist())}")
    m = {"node": nid, "sequences": n_seq, "microbatches": M, "ring_groups": groups, "prompt_len": T,
         "decode_steps": steps - 1,
         "prefill_tokens_per_s": round(n_seq * T / prefill_s, 1) if prefill_s > 0 else None,
         "decode_tokens_per_s": round(n_seq * (steps - 1) / decode_s, 1) if steps > 1 and decode_s > 0 else None,
         "decode_ms_per_step": round(decode_s / (steps - 1) * 1e3, 4) if steps > 1 else None}
    log("METRICS " + json.dumps(m))


def _timed_generate(ring: DecodeRing, prompts, T: int, steps: int, dev, chunk: int = 0):
    t0 = time.perf_counter()
    ring.prefill(prompts, T, chunk)
    if steps > 1:
        ring.capture()
    _sync(dev)
    t1 = time.perf_counter()
    if steps > 1:
        ring.decode_rounds(steps - 1)
    ring.drain()
    _sync(dev)
    t2 = time.perf_counter()
    return t1 - t0, t2 - t1


def run_generate_colocated(ctx, args, stages: List, device) -> int:
    pipe = ctx.pipeline
    prompt = make_prompts(pipe, args.prompt)
    n_seq, T = prompt.shape
    steps = max(1, pipe.decode_steps or 1)
    check_capacity(stages, *kv_capacity(pipe, T))
    M, B = pipe.num_microbatches, pipe.micro_batch_size
    ring = DecodeRing(stages, RingLinks(), 1, M, B)
    prompts = [prompt[m * B:(m + 1) * B] for m in range(M)]
    pf, dec = _timed_generate(ring, prompts, T, steps, device, pipe.prefill_chunk)
    _report(ctx.node_id, ring.tokens(), pf, dec, n_seq, T, steps, M, 1)
    return 0


def run_generate_dist(ctx, args, stage, info, progress=None) -> int:
    """One rank per stage; tokens return to stage 0 over the back-edge.  The
    prompt shape travels down the chain in a header from stage 0."""
    from ..parallel import comm
    from ..parallel.links import KIND_DATA, make_link
    pipe = ctx.pipeline
    S, r, dev = pipe.num_parts, ctx.part_index, info.device
    peer = getattr(ctx, "peer", lambda p: p)  # ranks of this replica's stages
    if pipe.return_to_node_id and pipe.by_id(pipe.return_to_node_id) and \
            pipe.by_id(pipe.return_to_node_id).part_index != 0 and r == S - 1:
        log(f"[{ctx.node_id}] note: generated tokens feed the embedding, so they return to stage 0 "
            f"(return_to_node_id '{pipe.return_to_node_id}' is not stage 0)")
    bg = comm.back_group()  # the token back-edge on its own communicator / stream
    links = RingLinks(prev=make_link(peer(r - 1), dev) if r > 0 else None,
                      nxt=make_link(peer(r + 1), dev) if r < S - 1 else None,
                      back_out=make_link(peer(0), dev, bg) if (r == S - 1 and S > 1) else None,
                      back_in=make_link(peer(S - 1), dev, bg) if (r == 0 and S > 1) else None)
    M, B = pipe.num_microbatches, pipe.micro_batch_size
    steps = max(1, pipe.decode_steps or 1)
    prompts = None
    if r == 0:
        prompt = make_prompts(pipe, args.prompt, getattr(ctx, "replica", 0))
        T = prompt.shape[1]
        prompts = [prompt[m * B:(m + 1) * B] for m in range(M)]
    else:
        _, _, T, steps = links.prev.recv_header()
    if links.nxt is not None:
        links.nxt.send_header(KIND_DATA, B, T, steps)
    check_capacity([stage], *kv_capacity(pipe, T))
    ring = DecodeRing([stage], links, S, M, B, progress=progress)
    pf, dec = _timed_generate(ring, prompts, T, steps, dev, pipe.prefill_chunk)
    if r == 0:
        nid = ctx.node_id + (f" replica {ctx.replica}" if getattr(pipe, "replicas", 1) > 1 else "")
        _report(nid, ring.tokens(), pf, dec, B * M, T, steps, M, S)
    return 0
