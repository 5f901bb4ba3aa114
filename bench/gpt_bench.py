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


LAT_ROUNDS = 16


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32, help="timed decode steps")
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--stages", type=int, default=4)
    ap.add_argument("--batch", type=int, default=64, help="sequences per microbatch")
    ap.add_argument("--microbatches", type=int, default=0, help="0 = number of GPU groups")
    ap.add_argument("--lanes", type=int, default=0,
                    help="one GPU group: HIP streams the microbatches of a decode round run on (0 = one, -1 = min(M, 4))")
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--prefill_iters", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--kv", default="bf16", choices=["bf16", "fp8"], help="KV cache dtype (fp8: OCP e4m3)")
    ap.add_argument("--kv_scale", default="calibrated", choices=["calibrated", "unit"],
                    help="fp8 KV cache scale: per-layer, from the first prefill's amax, or unit")
    ap.add_argument("--fp8_prefill", default="e4m3", choices=["split", "e4m3"],
                    help="fp8 weights: prefill activations as one e4m3 byte with MX block scales (default) or "
                         "split (e4m3 hi + residual, 2x the prefill MFMA work); GPT-2 XL 48 layers vs the fp32 model "
                         "on the unquantised weights: prefill logits 0.115 vs 0.096 (the fp8 weights dominate)")
    ap.add_argument("--no_graph", action="store_true", help="eager decode launches (no HIP graph)")
    ap.add_argument("--cpu", action="store_true", help="schedule test mode: gloo + fp32 golden stages on CPU")
    ap.add_argument("--gloo_gpu", action="store_true",
                    help="every rank on GPU 0 (HIP kernels + graphs), hops staged through host memory over gloo "
                         "(the 1-GPU box's multi-process schedule test; RCCL refuses two ranks on one GPU)")
    ap.add_argument("--verify_steps", type=int, default=-1,
                    help="after the timed run: greedy tokens of this many steps of the distributed ring on fixed "
                         "seeded prompts, against the same stages colocated on rank 0's device "
                         "(-1 = 8 when the ring spans several GPU groups, else 0)")
    ap.add_argument("--lat_rounds", type=int, default=LAT_ROUNDS,
                    help="synced single-round latency samples after the timed rounds (0: none, so a kernel trace "
                         "of the decode region holds only the timed multi-step graphs)")
    ap.add_argument("--verify_prompt", type=int, default=64, help="prompt length of the --verify_steps check")
    ap.add_argument("--prepost_ab", type=int, default=0,
                    help="after the timed run: this many interleaved A/B pairs of decode runs without / with "
                         "the pre-posted next-microbatch receive (DecodeRing.prepost)")
    return ap.parse_args(argv)


def _build_group(model, ranges, stage_ids, dev, max_batch, max_seq, fp8, kv="bf16", kv_scale="calibrated",
                 fp8_prefill="e4m3"):
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.runtime.stages import TorchStage
    from distributed_neural_networks_amd.runtime.transformer import TransformerStage
    S = len(ranges)
    out = []
    for s in stage_ids:
        a, b = ranges[s]
        if dev.type == "cpu":  # schedule-test mode only (never a reported number)
            sd = ckpt.random_stage_state_dict(model, a, b, s == 0, s == S - 1, 0)
            out.append(TorchStage(model, sd, a, b, s == 0, s == S - 1, dev))
            continue
        sd = ckpt.random_stage_state_dict(model, a, b, s == 0, s == S - 1, 0, device=dev)
        out.append(TransformerStage(model, sd, a, b, s == 0, s == S - 1, dev, max_batch=max_batch,
                                    max_seq=max_seq, fp8=fp8, kv_dtype=kv, kv_scale=kv_scale,
                                    fp8_prefill=fp8_prefill))
        del sd
    return out


def verify_ring(args, info, ring, grp, rep, groups, M, B, V, ranges, max_seq, fp8, kv, sync) -> dict:
    """The tokens that crossed the hops, checked: the
    distributed ring generates ``--verify_steps`` greedy tokens for fixed
    seeded prompts (every microbatch, ``--verify_prompt`` tokens each), then
    rank 0 builds every stage of the model on its own device (same weights:
    ``random_stage_state_dict`` is seeded per stage) as a one-group ring and
    generates from the same prompts.  Returns, on rank 0, the fraction of
    (sequence, step) tokens the two agree on and that of the first (prefill)
    token.  Every rank runs the same collectives; idle ranks only join the
    barriers.  Outside every timed region."""
    from distributed_neural_networks_amd.runtime.scheduler import DecodeRing, RingLinks
    steps = args.verify_steps if args.verify_steps > 0 else 8
    Tv = max(1, min(args.verify_prompt, max_seq - steps - 2))
    g = torch.Generator().manual_seed(4242)
    prompts = [torch.randint(0, V, (B, Tv), generator=g, dtype=torch.int32) for _ in range(M)]
    dev = info.device
    sync()
    toks = None
    if ring is not None:
        ring.record = True
        mine = [p.to(dev) for p in prompts] if grp == 0 else None
        if mine is not None and os.environ.get("DNN_TEST_CORRUPT_VERIFY") == "1":  # tests: a wrong ring must show
            mine[0] = (mine[0] + 1) % V
        toks = ring.generate(mine, Tv, steps)
        ring.record = False
    sync()
    res = {}
    if info.rank == 0:
        S = len(ranges)
        stages = _build_group(args.model, ranges, list(range(S)), dev, B * M, max_seq, fp8, kv,
                              getattr(args, "kv_scale", "calibrated"), getattr(args, "fp8_prefill", "e4m3"))
        ref = DecodeRing(stages, RingLinks(), 1, M, B, use_graphs=not args.no_graph, record=True)
        want = ref.generate([p.to(dev) for p in prompts], Tv, steps)
        del ref, stages
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
        got = toks
        ok = (got == want) if got is not None and got.shape == want.shape else torch.zeros_like(want, dtype=torch.bool)
        res = {"dist_token_agreement_vs_colocated": round(float(ok.float().mean().item()), 6),
               "dist_first_token_agreement_vs_colocated": round(float(ok[:, 0].float().mean().item()), 6),
               "dist_verify_tokens": int(want.numel()), "dist_verify_steps": steps, "dist_verify_prompt_len": Tv,
               "dist_verify_path": f"{groups} GPU groups over the hops + token back-edge vs all stages colocated "
                                   f"on rank 0"}
    sync()
    return res


def main(args=None):
    out = run(args)
    if out is not None:
        print(json.dumps(out), flush=True)
    return 0


def run(args=None, shutdown: bool = True):
    """Run the bench on every rank; rank 0 returns the JSON record (others None).
    ``shutdown=False`` keeps the process group for a caller that runs more
    benches in the same processes (bench.py's multi-GPU extras)."""
    if args is None or not hasattr(args, "prompt"):
        base = args
        args = parse([])
        if base is not None:
            for k in ("gpus", "steps", "warmup", "model"):
                if hasattr(base, k):
                    setattr(args, k, getattr(base, k))
    from distributed_neural_networks_amd.models import default_ranges, gpt2, model_info
    from distributed_neural_networks_amd.parallel import comm
    from distributed_neural_networks_amd.parallel.links import make_link

    N = args.gpus
    if getattr(args, "gloo_gpu", False):
        info = comm.init("gloo")
        torch.cuda.set_device(0)
        info = comm.DistInfo(info.rank, info.world, info.local_rank, "gloo", torch.device("cuda", 0))
    elif getattr(args, "cpu", False):
        info = comm.init("gloo")
    elif N > 1 or "WORLD_SIZE" in os.environ:
        info = comm.init("nccl")
        if info.world > 1:  # native RCCL channels checked on a ring; any failure -> ProcessGroupNCCL P2P
            from distributed_neural_networks_amd.parallel.links import native_preflight
            native_preflight(info.device)
    else:
        torch.cuda.set_device(0)
        info = comm.DistInfo(0, 1, 0, "none", torch.device("cuda", 0))
    from distributed_neural_networks_amd.parallel.selflaunch import check_world
    check_world(args.gpus, info.world)
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
    lat_rounds = getattr(args, "lat_rounds", LAT_ROUNDS)
    total_steps = args.warmup + args.steps + lat_rounds + 2  # + the latency rounds + graph-capture slack
    max_seq = T0 + total_steps + 1
    fp8 = args.dtype == "fp8"
    kv = getattr(args, "kv", "bf16")
    stages = (_build_group(model, ranges, stage_ids, dev, B * M, max_seq, fp8, kv, getattr(args, "kv_scale", "calibrated"),
                           getattr(args, "fp8_prefill", "e4m3"))
              if stage_ids else [])
    base = rep * groups
    prev = make_link(base + grp - 1, dev) if grp > 0 else None
    nxt = make_link(base + grp + 1, dev) if 0 <= grp < groups - 1 else None
    bg = comm.back_group() if N > 1 else None  # the token back-edge on its own communicator / stream
    back_to0 = make_link(base + 0, dev, bg) if (grp == groups - 1 and groups > 1) else None
    back_from = make_link(base + groups - 1, dev, bg) if (grp == 0 and groups > 1) else None
    d = model_info(model).cfg.n_embd
    V = model_info(model).cfg.vocab_size

    from distributed_neural_networks_amd.runtime.scheduler import DecodeRing, RingLinks
    links = RingLinks(prev=prev, nxt=nxt, back_out=back_to0, back_in=back_from)
    ring = (DecodeRing(stages, links, groups, M, B, use_graphs=not args.no_graph, record=False,
                      lanes=getattr(args, "lanes", 0)) if stages else None)
    prompts = [torch.randint(0, V, (B, T0), device=dev, dtype=torch.int32) for _ in range(M)] if grp == 0 else None

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier(info)
        return time.perf_counter()

    # ---------------- prefill (all microbatches, T0 tokens each) ----------------
    def prefill_round():
        if ring is not None:
            ring.prefill(prompts, T0)

    def finish_prefill():  # the prefill's sampled tokens still travel the back-edge
        if ring is not None:
            ring.drain()

    prefill_round()
    finish_prefill()
    t0 = sync()
    for _ in range(args.prefill_iters):
        prefill_round()
        finish_prefill()
    t1 = sync()
    prefill_s = (t1 - t0) / args.prefill_iters
    prefill_tok = B * M * T0 * replicas

    # ---------------- decode (microbatched ring, one HIP graph per microbatch) ----------------
    prefill_round()
    if ring is not None:
        ring.capture()
    if ring is not None and args.warmup:
        ring.decode_rounds(args.warmup)
    t0 = sync()
    if ring is not None:
        ring.decode_rounds(args.steps)  # next microbatch's input received while this one computes
    if ring is not None:
        ring.drain()
    t1 = sync()
    decode_s = (t1 - t0) / args.steps
    dec_tok = B * M * replicas
    # per-token latency.  One group: a synced decode round.  Several groups:
    # microbatch 0 circulates alone (ring.decode_round([0]) on every rank), so
    # a round is one trip stage 0 -> ... -> last -> back-edge -> stage 0; the
    # time between group 0's consecutive post-round syncs is one token.
    lat = []
    if groups == 1 and ring is not None:
        for _ in range(lat_rounds):
            ta = sync()
            ring.decode_round()
            lat.append(sync() - ta)
    elif ring is not None:
        comm.barrier(info)
        stamps = []
        for _ in range(lat_rounds):
            ring.decode_round([0])
            if grp == 0:
                if dev.type == "cuda":
                    torch.cuda.synchronize(dev)
                stamps.append(time.perf_counter())
        ring.drain()
        lat = [b - a for a, b in zip(stamps, stamps[1:])]
    sync()
    graphs = ring is not None and bool(ring.graphs)

    def mx(v):
        if N == 1:
            return v
        import torch.distributed as dist
        t = torch.tensor([v], dtype=torch.float64, device=dev if info.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    vsteps = getattr(args, "verify_steps", -1)
    if vsteps < 0:
        vsteps = 8 if groups > 1 else 0
    ver = verify_ring(args, info, ring, grp, rep, groups, M, B, V, ranges, max_seq, fp8, kv, sync) if vsteps else {}

    ab = {}
    if getattr(args, "prepost_ab", 0) and ring is not None:
        # interleaved A/B of the decode schedule: each input received just before
        # its use vs the next microbatch's receive posted before this one computes
        k = max(2, args.steps // 2)
        times = {False: [], True: []}
        for _ in range(args.prepost_ab):
            for pp in (False, True):
                ring.prepost = pp
                ta = sync()
                ring.decode_rounds(k)
                ring.drain()
                times[pp].append(mx(sync() - ta) / k)
        ring.prepost = True
        ab = {"ab_rounds_per_arm": k, "ab_no_prepost_ms_per_step": [round(t * 1e3, 4) for t in times[False]],
              "ab_prepost_ms_per_step": [round(t * 1e3, 4) for t in times[True]]}
    elif getattr(args, "prepost_ab", 0):
        for _ in range(args.prepost_ab * 2):
            sync()
            sync()
            mx(0.0)

    prefill_s, decode_s = mx(prefill_s), mx(decode_s)
    out = None
    if r == 0:
        value = dec_tok / decode_s
        out = {
            "metric": f"tokens/sec {model} {S}-stage greedy decode", "value": round(value, 1), "unit": "tokens/s",
            "n_gpus": N, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(decode_s * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": (("fp8-e4m3 weights (decode: W8A16 on bf16 MFMA; prefill: fp8 MFMA on split activations, "
                       "e4m3 hi + e4m3 residual), bf16 activations") if fp8 and args.fp8_prefill == "split" else
                      "fp8-e4m3 weights (decode: W8A16 on bf16 MFMA; prefill: W8A8 on fp8 MFMA), bf16 activations"
                      if fp8 else "bf16") + ("; fp8-e4m3 KV cache" if kv == "fp8" else ""),
            "data": "synthetic prompts, random-init weights",
            "prefill_tokens_per_s": round(prefill_tok / prefill_s, 1),
            "prefill_ms_per_round": round(prefill_s * 1e3, 3),
            "decode_p50_token_latency_ms": round(statistics.median(lat) * 1e3, 4) if lat else None,
            "hip_graph_decode": bool(graphs),
            "config": {"model": model, "stages": S, "gpu_groups": groups, "replicas": replicas,
                       "micro_batch": B, "microbatches": M, "prompt_len": T0, "seq_len": max_seq,
                       "decode_lanes": len(ring.lanes) if ring is not None and ring.lanes else 1,
                       "global_batch": B * M * replicas, "parallelism": f"pp{groups}x dp{replicas}"},
        }
        out.update(ab)
        out.update(ver)
    if N > 1 and shutdown:
        comm.shutdown()
    return out if r == 0 else None


if __name__ == "__main__":
    _args = parse()
    from distributed_neural_networks_amd.parallel.selflaunch import maybe_self_launch
    _rc = maybe_self_launch(_args.gpus, os.path.abspath(__file__), sys.argv[1:])
    sys.exit(_rc if _rc is not None else main(_args))
