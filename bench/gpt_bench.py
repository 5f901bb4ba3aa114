"""GPT-2 small 4-stage pipeline: prefill and greedy-decode tokens/s (bf16, or fp8).

Invoked as ``python bench.py --model gpt2 ...`` (or directly).  The model is
split into 4 pipeline stages (``default_ranges``: 3 blocks each, lm_head on
the last).  N GPUs host the stages as a linear pipeline of min(N, 4) GPU
groups (consecutive stages colocated on one GPU when N < 4), replicated
N // 4 times when N > 4.  Per group, stages are chained on one stream; between
groups activations move with RCCL isend/irecv over xGMI.

Decode is microbatched: M microbatches of B sequences each circulate
stage 0 -> ... -> last -> (sampled token ids over the back-edge) -> stage 0, so
with M >= #groups every GPU works on a different microbatch at any time.
Synthetic prompts, random-init weights.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32, help="timed decode steps")
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--stages", type=int, default=4)
    ap.add_argument("--batch", type=int, default=64, help="sequences per microbatch")
    ap.add_argument("--microbatches", type=int, default=0, help="0 = number of GPU groups")
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--prefill_iters", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--no_graph", action="store_true", help="eager decode launches (no HIP graph)")
    return ap.parse_args(argv)


def _build_group(model, ranges, stage_ids, dev, max_batch, max_seq, fp8):
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.runtime.transformer import TransformerStage
    S = len(ranges)
    out = []
    for s in stage_ids:
        a, b = ranges[s]
        sd = ckpt.random_stage_state_dict(model, a, b, s == 0, s == S - 1, 0, device=dev)
        out.append(TransformerStage(model, sd, a, b, s == 0, s == S - 1, dev, max_batch=max_batch,
                                    max_seq=max_seq, fp8=fp8))
        del sd
    return out


def main(args=None):
    if args is None or not hasattr(args, "prompt"):
        base = args
        args = parse([])
        if base is not None:
            for k in ("gpus", "steps", "warmup", "model"):
                if hasattr(base, k):
                    setattr(args, k, getattr(base, k))
    from distributed_neural_networks_amd.models import default_ranges, gpt2, model_info
    from distributed_neural_networks_amd.parallel import comm
    from distributed_neural_networks_amd.parallel.links import P2PLink

    N = args.gpus
    if N > 1 or "WORLD_SIZE" in os.environ:
        info = comm.init("nccl")
    else:
        torch.cuda.set_device(0)
        info = comm.DistInfo(0, 1, 0, "none", torch.device("cuda", 0))
    N, r, dev = info.world, info.rank, info.device
    model = args.model
    S = args.stages
    ranges = default_ranges(model, S)
    groups = min(N, S)
    replicas = max(1, N // groups)
    grp, rep = r % groups, r // groups
    if rep >= replicas:  # leftover ranks idle (N not a multiple of groups)
        grp = -1
    per = S // groups
    stage_ids = list(range(grp * per, (grp + 1) * per)) if grp >= 0 else []
    if grp == groups - 1:
        stage_ids = list(range(grp * per, S))
    M = args.microbatches or groups
    B = args.batch
    T0 = args.prompt
    total_steps = args.warmup + args.steps + 16 + 2  # + the 16 latency steps + graph-capture slack
    max_seq = T0 + total_steps + 1
    fp8 = args.dtype == "fp8"
    stages = _build_group(model, ranges, stage_ids, dev, B * M, max_seq, fp8) if stage_ids else []
    base = rep * groups
    prev = P2PLink(base + grp - 1, dev) if grp > 0 else None
    nxt = P2PLink(base + grp + 1, dev) if 0 <= grp < groups - 1 else None
    back_to0 = P2PLink(base + 0, dev) if (grp == groups - 1 and groups > 1) else None
    back_from = P2PLink(base + groups - 1, dev) if (grp == 0 and groups > 1) else None
    d = model_info(model).cfg.n_embd
    V = model_info(model).cfg.vocab_size

    pos = [torch.zeros((B,), dtype=torch.int32, device=dev) for _ in range(M)]
    ids = [torch.randint(0, V, (B, T0), device=dev, dtype=torch.int32) for _ in range(M)]
    xin = [torch.empty((B * T0, d), dtype=torch.bfloat16, device=dev) for _ in range(M)]
    nid = [torch.empty((B,), dtype=torch.int32, device=dev) for _ in range(M)]

    def run_group(x, m, Tn):
        h = x
        for st in stages:
            h = st.step(h, pos[m], B, Tn, b0=m * B)
        return h

    def sync():
        torch.cuda.synchronize()
        if N > 1:
            import torch.distributed as dist
            dist.barrier(device_ids=[dev.index])
        return time.perf_counter()

    # ---------------- prefill (all microbatches, T0 tokens each) ----------------
    def prefill_round():
        for m in range(M):
            pos[m].zero_()
        for m in range(M):
            if not stages:
                continue
            if grp == 0:
                x = ids[m]
            else:
                x = xin[m][:B * T0]
                prev.recv(x)
            y = run_group(x, m, T0)
            pos[m].add_(T0)
            if nxt is not None:
                nxt.send(y)
            elif stages[-1].last:
                nid[m].copy_(y.pred)
        if back_to0 is not None:
            for m in range(M):
                back_to0.send(nid[m])
        if back_from is not None:
            for m in range(M):
                back_from.recv(nid[m])

    prefill_round()
    t0 = sync()
    for _ in range(args.prefill_iters):
        prefill_round()
    t1 = sync()
    prefill_s = (t1 - t0) / args.prefill_iters
    prefill_tok = B * M * T0 * replicas

    # ---------------- decode (microbatched ring) ----------------
    dec_x = [torch.empty((B, d), dtype=torch.bfloat16, device=dev) for _ in range(M)]
    cur = [n.view(B, 1).clone() for n in nid]
    lat = []

    def decode_round():
        for m in range(M):
            if not stages:
                continue
            ta = time.perf_counter()
            if grp == 0:
                if groups > 1 and back_from is not None and decode_round.started[m]:
                    back_from.recv(nid[m])
                    cur[m].copy_(nid[m].view(B, 1))
                x = cur[m]
            else:
                x = dec_x[m]
                prev.recv(x)
            y = run_group(x, m, 1)
            pos[m].add_(1)
            if nxt is not None:
                nxt.send(y)
            else:
                if groups > 1:
                    back_to0.send(y.pred)
                else:
                    cur[m].copy_(y.pred.view(B, 1))
            decode_round.started[m] = True
            lat.append(time.perf_counter() - ta)

    decode_round.started = [False] * M

    # One HIP graph per microbatch for this group's decode compute (the P2P
    # hops stay outside: blocking RCCL send/recv order the compute stream).
    graphs = {}
    if stages and not args.no_graph:
        from distributed_neural_networks_amd.runtime.graph import GraphedStep
        gout = {}

        def body(m):
            x = cur[m] if grp == 0 else dec_x[m]
            y = run_group(x, m, 1)
            pos[m].add_(1)
            if isinstance(y, torch.Tensor):
                gout[m] = y
            else:
                nid[m].copy_(y.pred)
            return None

        for m in range(M):
            snap = pos[m].clone()
            graphs[m] = GraphedStep(lambda m=m: body(m), dev, warmup=1)
            pos[m].copy_(snap)
        torch.cuda.synchronize()

        class _Out:
            def __init__(self, p):
                self.pred = p

    def group_step(x, m):
        if graphs:
            y = graphs[m]()
            return gout[m] if m in gout else _Out(nid[m])
        y = run_group(x, m, 1)
        pos[m].add_(1)
        return y

    def decode_round():  # noqa: F811 (graph-aware version)
        for m in range(M):
            if not stages:
                continue
            ta = time.perf_counter()
            if grp == 0:
                if groups > 1 and back_from is not None and decode_round.started[m]:
                    back_from.recv(nid[m])
                    cur[m].copy_(nid[m].view(B, 1))
                x = cur[m]
            else:
                x = dec_x[m]
                prev.recv(x)
            y = group_step(x, m)
            if nxt is not None:
                nxt.send(y)
            else:
                if groups > 1:
                    back_to0.send(y.pred)
                else:
                    cur[m].copy_(y.pred.view(B, 1))
            decode_round.started[m] = True
            lat.append(time.perf_counter() - ta)

    decode_round.started = [False] * M
    for _ in range(args.warmup):
        decode_round()
    t0 = sync()
    for _ in range(args.steps):
        decode_round()
    # drain the back-edge
    if back_from is not None:
        for m in range(M):
            back_from.recv(nid[m])
    t1 = sync()
    decode_s = (t1 - t0) / args.steps
    dec_tok = B * M * replicas
    # per-token latency of one decode step (single group only: a synced step)
    tok_lat = []
    if groups == 1 and stages:
        for _ in range(16):
            ta = sync()
            decode_round()
            tok_lat.append(sync() - ta)
    lat[:] = tok_lat

    def mx(v):
        if N == 1:
            return v
        import torch.distributed as dist
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    prefill_s, decode_s = mx(prefill_s), mx(decode_s)
    if r == 0:
        value = dec_tok / decode_s
        out = {
            "metric": f"tokens/sec {model} {S}-stage greedy decode", "value": round(value, 1), "unit": "tokens/s",
            "n_gpus": N, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(decode_s * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": ("fp8-e4m3 weights (decode: W8A16 on bf16 MFMA; prefill: W8A8 on fp8 MFMA), bf16 activations"
                      if fp8 else "bf16"),
            "data": "synthetic prompts, random-init weights",
            "prefill_tokens_per_s": round(prefill_tok / prefill_s, 1),
            "prefill_ms_per_round": round(prefill_s * 1e3, 3),
            "decode_p50_token_latency_ms": round(statistics.median(lat) * 1e3, 4) if lat else None,
            "hip_graph_decode": bool(graphs),
            "config": {"model": model, "stages": S, "gpu_groups": groups, "replicas": replicas,
                       "micro_batch": B, "microbatches": M, "prompt_len": T0, "seq_len": max_seq,
                       "global_batch": B * M * replicas, "parallelism": f"pp{groups}x dp{replicas}"},
        }
        print(json.dumps(out), flush=True)
    if N > 1:
        comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main(parse()))
