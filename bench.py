#!/usr/bin/env python3
"""Flagship benchmark: CIFAR-10 ConvNet 2-stage pipeline inference, images/s.

Metric/config from BASELINE.json (the reference's only measured headline:
CIFAR-10 2-stage images/s; 3.40-4.15 k img/s on CPU over localhost gRPC,
BASELINE.md).  Synthetic fp32 images, random-init weights of the reference
architecture, computed at the reference's precision (fp32: every product as
three bf16 MFMA terms, ops/cifar.py); ``--precision bf16`` is the reduced-
precision variant and is reported as extra keys.  Every timed step runs the
complete forward of both stages (conv stage + fc/softmax/argmax stage) on
fresh launches; nothing is cached across steps.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...

Placements:
* N = 1: both stages colocated on the GPU, one HIP graph per step; extra keys:
  the bf16 pipeline, the GPT-2 small 4-stage pipeline (decode / prefill
  tokens/s, p50 per-token latency; bench/gpt_bench.py) and BASELINE configs 4
  and 5 colocated (Llama-3 8B bf16 8-stage B=32, GPT-2 XL fp8 8-stage B=64).
* N > 1 (one process per GPU, RCCL): ``linear`` (default) — the reference
  topology, one stage per GPU, isend/irecv over the direct xGMI links; the
  bottleneck stage is replicated (``parallel/partition.py::linear_plan``: n0
  stage-0 GPUs feed n1 stage-1 GPUs, each sender on its own link), the K steps
  stream as one fill/drain.  ``interleaved`` (opt-in) — every GPU hosts stage
  0 of its pipeline and stage 1 of the others; the hop is an all-to-all.
Scaling is weak: each stage-0 GPU sources ``--batch`` images per step.

``--model gpt2`` runs the GPT-2 4-stage token throughput bench instead
(bench/gpt_bench.py).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

BASELINE_IMG_S = 4150.0  # reference CIFAR-10 2-stage, best batch (255), CPU gRPC
METRIC = "images/sec CIFAR-10 2-stage"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=65536, help="images sourced per GPU per step")
    ap.add_argument("--no_fill", action="store_true",
                    help="linear N>1: stage-1 GPUs only serve received microbatches (no own images)")
    ap.add_argument("--fill_rows", type=int, default=-1, help="linear N>1: own images per round on a stage-1 GPU "
                                                               "(-1 = sized from timing, see receiver_fill_rows)")
    ap.add_argument("--microbatches", type=int, default=2,
                    help="microbatches per step on N>1 (2 x 32768 rows fill the fc1 GEMM's 256 tiles)")
    ap.add_argument("--placement", default="linear", choices=["linear", "interleaved"],
                    help="N>1: linear = the reference topology (one stage per GPU, RCCL send/recv); "
                         "interleaved = opt-in all-to-all variant")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                    help="compute precision of the headline (fp32 = the reference's)")
    ap.add_argument("--no_extra", action="store_true", help="skip the extra bf16 / GPT-2 keys")
    ap.add_argument("--no_big", action="store_true",
                    help="skip the Llama-3 8B / GPT-2 XL extra keys (BASELINE configs 4 and 5)")
    ap.add_argument("--model", default="cifar10")
    ap.add_argument("--latency_iters", type=int, default=200)
    ap.add_argument("--cpu", action="store_true", help="schedule test mode: gloo + fp32 golden stages on CPU")
    ap.add_argument("--s0_spare_cus", type=int, default=-1,
                    help="CUs left free of the persistent stage-0 kernel for the RCCL hop kernels to run "
                         "concurrently (-1 = auto: 0 on 1 GPU, 16 on N > 1)")
    ap.add_argument("--cut", default="auto", choices=["auto", "1", "2"],
                    help="stage boundary: 1 = after conv2/pool (reference), 2 = after fc1; auto = cost model")
    return ap.parse_args()


def dist_setup(n, cpu=False):
    from distributed_neural_networks_amd.parallel import comm
    if cpu:
        return comm.init("gloo")
    if n > 1 or "WORLD_SIZE" in os.environ:
        info = comm.init("nccl")
    else:
        torch.cuda.set_device(0)
        info = comm.DistInfo(0, 1, 0, "none", torch.device("cuda", 0))
    return info


def stages_for(device, cut: int = 1, precision: str = "fp32"):
    """The two pipeline stages: units [0..cut] and [cut+1..3] (cut 1 = the reference's conv|fc split)."""
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.runtime.stages import CifarHipStage, TorchStage
    sd0 = ckpt.random_stage_state_dict("cifar10", 0, cut, True, False, 0)
    sd1 = ckpt.random_stage_state_dict("cifar10", cut + 1, 3, False, True, 0)
    if device.type == "cpu":  # schedule-test mode only (never used for a reported number)
        return (TorchStage("cifar10", sd0, 0, cut, True, False, device),
                TorchStage("cifar10", sd1, cut + 1, 3, False, True, device))
    return CifarHipStage(sd0, 0, cut, device, precision), CifarHipStage(sd1, cut + 1, 3, device, precision)


def pick_cut(args, info) -> int:
    from distributed_neural_networks_amd.parallel.partition import cifar_cut
    if args.cut != "auto":
        return int(args.cut)
    if info.world == 1:
        return 1  # colocated: no hop; keep the reference split
    return cifar_cut(args.placement, info.world, precision=args.precision)


def dsync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def sync_time(info):
    import torch.distributed as dist
    dsync(info.device)
    if info.world > 1:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()
        dsync(info.device)
    return time.perf_counter()


def max_over_ranks(info, v):
    import torch.distributed as dist
    if info.world == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=info.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bench_colocated(args, info):
    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    dev = info.device
    s0, s1 = stages_for(dev, 1, args.precision)
    g = torch.Generator(device=dev).manual_seed(0)
    pipe = ColocatedPipeline([s0, s1], args.batch)
    pipe.x.copy_(torch.randn(pipe.x.shape, device=dev, generator=g))
    pipe.capture()
    for _ in range(args.warmup):
        pipe()
    t0 = sync_time(info)
    for _ in range(args.steps):
        pipe()
    t1 = sync_time(info)
    # p50 single-image pipeline latency (both stages, one graph replay)
    lat = ColocatedPipeline([s0, s1], 1)
    lat.x.copy_(torch.randn(lat.x.shape, device=dev, generator=g))
    lat.capture()
    ts = []
    for _ in range(args.latency_iters):
        torch.cuda.synchronize()
        a = time.perf_counter()
        lat()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    return t1 - t0, args.batch, statistics.median(ts) * 1e3, "pp2-colocated"


def bench_interleaved(args, info):
    import torch.distributed as dist
    dev, N, r = info.device, info.world, info.rank
    s0, s1 = stages_for(dev, args._cut, args.precision)
    M = max(1, args.microbatches)
    mb = args.batch // M
    per_peer = mb // (N - 1)
    mb = per_peer * (N - 1)
    g = torch.Generator(device=dev).manual_seed(1 + r)
    xs = [torch.randn((mb, 3, 32, 32), device=dev, generator=g) for _ in range(M)]
    bdt = s0.out_spec(1)[1]
    bw = s0.out_spec(1)[0][1]  # boundary width: 4096 (cut 1) or 512 (cut 2)
    y0 = [torch.empty((mb, bw), dtype=bdt, device=dev) for _ in range(M)]
    rx = [torch.empty((mb, bw), dtype=bdt, device=dev) for _ in range(M)]
    probs = [torch.empty((mb, 10), device=dev) for _ in range(M)]
    splits = [0 if p == r else per_peer for p in range(N)]

    # Steady-state streaming: the hop of the last microbatch of step k is
    # drained after stage 0 of step k+1's first microbatch has been issued, so
    # no hop is exposed between steps.  Buffer reuse is ordered by the work
    # handles: a2a(i) is waited on before stage 1 of microbatch i, which precedes
    # (in stream order) stage 0 of microbatch i of the next step.
    pending = []

    def drain():
        while pending:
            w, i = pending.pop(0)
            w.wait()
            s1.forward(rx[i], probs[i])

    def step():
        for i in range(M):
            s0.forward(xs[i], y0[i])
            w = dist.all_to_all_single(rx[i], y0[i], splits, splits, async_op=True)
            drain()  # stage 1 of the previous microbatch (possibly of the previous step)
            pending.append((w, i))

    for _ in range(args.warmup):
        step()
    drain()
    t0 = sync_time(info)
    for _ in range(args.steps):
        step()
    drain()
    t1 = sync_time(info)
    # latency: one image per peer through stage0 -> all-to-all -> stage1
    lx = torch.randn((N - 1, 3, 32, 32), device=dev, generator=g)
    ly = torch.empty((N - 1, bw), dtype=bdt, device=dev)
    lr = torch.empty_like(ly)
    lp = torch.empty((N - 1, 10), device=dev)
    one = [0 if p == r else 1 for p in range(N)]
    ts = []
    for _ in range(min(args.latency_iters, 100)):
        sync_time(info)
        a = time.perf_counter()
        s0.forward(lx, ly)
        dist.all_to_all_single(lr, ly, one, one)
        s1.forward(lr, lp)
        dsync(dev)
        ts.append(time.perf_counter() - a)
    return t1 - t0, mb * M, statistics.median(ts) * 1e3, f"pp2-interleaved-a2a-x{N}"


def bench_linear(args, info):
    """Linear 2-stage pipeline, one stage per GPU, RCCL isend/irecv over the
    direct xGMI links (``parallel/partition.py::linear_plan``): n0 stage-0 GPUs
    each source ``--batch`` images per step and stream them to one of n1
    stage-1 GPUs.  The K timed steps run as ONE stream of K x M microbatches
    (fill and drain once, not per step).  A stage-1 GPU spends ~2 % of a
    round on fc2, so it also runs its own images through both stages between
    rounds (``receiver_fill_rows``; measured on one MI355X at 32768-row
    microbatches: stage 0 1.245 ms, stage 1 0.023 ms -> 27648 / 24576 / 19456
    own rows per round at N = 2 / 4 / 8, i.e. 1.84 / 3.75 / 7.59 GPUs of work
    instead of 1 / 3 / 7)."""
    from distributed_neural_networks_amd.parallel.links import P2PLink
    from distributed_neural_networks_amd.parallel.partition import linear_plan, linear_role
    from distributed_neural_networks_amd.runtime.scheduler import run_gpipe
    dev, N, r = info.device, info.world, info.rank
    plan = linear_plan(N, args.precision)
    if args.cut != "auto":
        plan = dict(plan, cut=args._cut)
    args._cut = plan["cut"]
    role = linear_role(r, plan)
    s0, s1 = stages_for(dev, args._cut, args.precision)
    M = max(1, args.microbatches)
    mb = args.batch // M
    g = torch.Generator(device=dev).manual_seed(1 + r)
    if role["stage"] == 0:
        xs = [torch.randn((mb, 3, 32, 32), device=dev, generator=g) for _ in range(M)]
        nxt = P2PLink(role["send_to"], dev)

        def stream(steps):
            run_gpipe(s0, steps * M, mb, None, nxt, source=lambda i: xs[i % M], depth=2)
    else:
        prevs = [P2PLink(p, dev) for p in role["recv_from"]]
        # receiver fill: a stage-1 GPU is mostly idle (fc2 is ~1 % of the model),
        # so between rounds of received microbatches it runs its own images
        # through both stages, sized so a round still fits in a sender's period
        fill = 0 if args.no_fill else (args.fill_rows if args.fill_rows >= 0 else
                                       receiver_fill_rows(s0, s1, mb, len(prevs), dev))
        if fill:
            xl = torch.randn((fill, 3, 32, 32), device=dev, generator=g)
            sh0, dt0 = s0.out_spec(fill)
            sh1, dt1 = s1.out_spec(fill)
            yl0 = torch.empty(sh0, dtype=dt0, device=dev)
            yl1 = torch.empty(sh1, dtype=dt1, device=dev)
        count = [0]

        def local_fill():
            count[0] += 1
            if fill and count[0] % len(prevs) == 0:
                s1.forward(s0.forward(xl, yl0), yl1)

        def stream(steps):
            run_gpipe(s1, steps * M * len(prevs), mb, prevs, None, depth=2 * len(prevs), progress=local_fill)

    stream(args.warmup)
    t0 = sync_time(info)
    stream(args.steps)
    t1 = sync_time(info)
    # images completed per step, job-wide: every sender's stream plus the receivers' own
    local = torch.tensor([0.0 if role["stage"] == 0 else float(fill * M)], dtype=torch.float64,
                         device=dev)
    import torch.distributed as dist
    dist.all_reduce(local)
    imgs_total_per_step = plan["n0"] * mb * M + float(local.item())
    args._fill_rows = float(local.item())
    par = f"pp2-linear-{plan['n0']}x{plan['n1']}" + ("+fill" if local.item() > 0 else "")
    return t1 - t0, imgs_total_per_step / N, float("nan"), par


RECV_ITEM_OVERHEAD_S = 30e-6  # host wait + launch per received microbatch (assumed, not measured here)


def receiver_fill_rows(s0, s1, mb: int, n_prev: int, dev) -> int:
    """Rows of its own images a stage-1 GPU can push through both stages per
    round of ``n_prev`` received microbatches without slowing the senders:
    (t_stage0 - n_prev (t_stage1 + overhead)) / t_both, 10 % margin, whole 1024-row
    blocks (8-row blocks for the small CPU test batches).  Timed on this GPU before the stream (the senders run the same
    stage-0 kernel on the same hardware)."""
    x = torch.randn((mb, 3, 32, 32), device=dev)
    sh0, dt0 = s0.out_spec(mb)
    sh1, dt1 = s1.out_spec(mb)
    y0 = torch.empty(sh0, dtype=dt0, device=dev)
    y1 = torch.empty(sh1, dtype=dt1, device=dev)

    def timed(fn, reps=3):
        fn()
        dsync(dev)
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        dsync(dev)
        return (time.perf_counter() - t) / reps

    t_s0 = timed(lambda: s0.forward(x, y0))
    t_s1 = timed(lambda: s1.forward(y0, y1))
    budget = t_s0 - n_prev * (t_s1 + RECV_ITEM_OVERHEAD_S)
    frac = max(0.0, budget / (t_s0 + t_s1)) * 0.9
    gran = 1024 if mb >= 8192 else 8
    return int(mb * frac) // gran * gran


def extra_keys(args, info):
    """Secondary numbers on the same GPU, same timing discipline: the CIFAR
    pipeline at reduced (bf16) precision when the headline is fp32."""
    out = {}
    if getattr(args, "gpt", True):
        # GPT-2 small 4-stage pipeline (BASELINE.json metric, second half): all
        # 4 stages on this GPU, bf16, B=64 sequences x 512-token prompts,
        # microbatched decode ring with one HIP graph per microbatch
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench"))
        import gpt_bench
        ga = gpt_bench.parse(["--gpus", "1", "--steps", "32", "--warmup", "4", "--batch", "64", "--prompt", "512",
                              "--stages", "4", "--dtype", "bf16"])
        g = gpt_bench.run(ga)
        out["gpt2_4stage_decode_tok_s"] = g["value"]
        out["gpt2_4stage_decode_ms_per_step"] = g["ms_per_step"]
        out["gpt2_4stage_p50_token_ms"] = g["decode_p50_token_latency_ms"]
        out["gpt2_4stage_prefill_tok_s"] = g["prefill_tokens_per_s"]
        out["gpt2_4stage_config"] = {"model": "gpt2 (124M, random init)", "stages": 4, "dtype": "bf16",
                                     "micro_batch": 64, "microbatches": g["config"]["microbatches"],
                                     "prompt_len": 512, "decode_steps_timed": 32,
                                     "placement": "4 stages colocated on 1 GPU"}
        # throughput point: 256 sequences per decode step (medium-M skinny GEMMs)
        ga = gpt_bench.parse(["--gpus", "1", "--steps", "32", "--warmup", "4", "--batch", "256", "--prompt", "512",
                              "--stages", "4", "--dtype", "bf16", "--prefill_iters", "2"])
        g = gpt_bench.run(ga)
        out["gpt2_4stage_b256_decode_tok_s"] = g["value"]
        out["gpt2_4stage_b256_decode_ms_per_step"] = g["ms_per_step"]
        # fp8 (OCP e4m3) KV cache, reduced KV precision (weights/activations bf16):
        # the decode K/V bytes halve (kv_cache_dtype "fp8")
        for key, b in (("gpt2_4stage_kv8", "64"), ("gpt2_4stage_b256_kv8", "256")):
            ga = gpt_bench.parse(["--gpus", "1", "--steps", "32", "--warmup", "4", "--batch", b, "--prompt", "512",
                                  "--stages", "4", "--dtype", "bf16", "--kv", "fp8", "--prefill_iters", "1"])
            g = gpt_bench.run(ga)
            out[key + "_decode_tok_s"] = g["value"]
            out[key + "_decode_ms_per_step"] = g["ms_per_step"]
        out["gpt2_4stage_kv8_dtype"] = "bf16 weights/activations, fp8-e4m3 KV cache"
    if getattr(args, "gpt", True) and not args.no_big:
        # BASELINE.json configs 4 and 5 on this GPU (all stages colocated): Llama-3
        # 8B bf16 8-stage microbatched decode and GPT-2 XL 8-stage with fp8
        # weights; a failure only drops these keys
        for key, argv, cfg in (
                ("llama3_8b_8stage_b32", ["--model", "llama3-8b", "--stages", "8", "--batch", "32", "--prompt", "512",
                                          "--dtype", "bf16"],
                 {"model": "llama3-8b (random init)", "stages": 8, "dtype": "bf16", "micro_batch": 32,
                  "prompt_len": 512}),
                ("gpt2xl_fp8_8stage_b64", ["--model", "gpt2-xl", "--stages", "8", "--batch", "64", "--prompt", "512",
                                           "--dtype", "fp8"],
                 {"model": "gpt2-xl (random init)", "stages": 8,
                  "dtype": "fp8-e4m3 weights (W8A16 decode, W8A8 prefill), bf16 activations", "micro_batch": 64,
                  "prompt_len": 512}),
                ("gpt2xl_fp8_8stage_b64_kv8", ["--model", "gpt2-xl", "--stages", "8", "--batch", "64", "--prompt",
                                               "512", "--dtype", "fp8", "--kv", "fp8"],
                 {"model": "gpt2-xl (random init)", "stages": 8,
                  "dtype": "fp8-e4m3 weights (W8A16 decode, W8A8 prefill), bf16 activations, fp8-e4m3 KV cache",
                  "micro_batch": 64, "prompt_len": 512})):
            try:
                g = gpt_bench.run(gpt_bench.parse(["--gpus", "1", "--steps", "16", "--warmup", "2",
                                                   "--prefill_iters", "1"] + argv))
                out[key + "_decode_tok_s"] = g["value"]
                out[key + "_decode_ms_per_step"] = g["ms_per_step"]
                out[key + "_prefill_tok_s"] = g["prefill_tokens_per_s"]
                out[key + "_config"] = dict(cfg, decode_steps_timed=16, placement="8 stages colocated on 1 GPU")
            except Exception as e:  # noqa: BLE001
                out[key + "_error"] = f"{type(e).__name__}: {e}"[:200]
            torch.cuda.empty_cache()
    if args.precision == "fp32":
        import copy
        a = copy.copy(args)
        a.precision, a.latency_iters = "bf16", 50
        el, imgs, p50, _ = bench_colocated(a, info)
        out["bf16_images_per_s"] = round(imgs * args.steps / el, 1)
        out["bf16_ms_per_step"] = round(el / args.steps * 1e3, 4)
        out["bf16_p50_latency_ms"] = round(p50, 4)
    return out


def main():
    args = parse()
    if args.model != "cifar10":
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench"))
        import gpt_bench
        return gpt_bench.main(args)
    info = dist_setup(args.gpus, args.cpu)
    N = info.world
    args._cut = pick_cut(args, info)
    spare = args.s0_spare_cus if args.s0_spare_cus >= 0 else (16 if N > 1 else 0)
    if spare and info.device.type == "cuda":
        # the stage-0 kernel holds every VGPR of the CUs it runs on, so without
        # spare CUs the all-to-all / isend kernels only start between stage-0
        # launches and each hop is exposed; 16 of 256 CUs (2 per XCD) stay free
        from distributed_neural_networks_amd.ops import cifar as cops
        n_cu = torch.cuda.get_device_properties(info.device).multi_processor_count
        cops.set_stage0_grid(max(1, n_cu - spare))
    if N == 1:
        el, imgs_per_gpu, p50, par = bench_colocated(args, info)
    elif args.placement == "interleaved":
        el, imgs_per_gpu, p50, par = bench_interleaved(args, info)
    else:
        el, imgs_per_gpu, p50, par = bench_linear(args, info)
    el = max_over_ranks(info, el)
    total = imgs_per_gpu * N * args.steps
    value = total / el
    extra = {}
    if N == 1 and not args.no_extra and info.device.type == "cuda":
        extra = extra_keys(args, info)
    hop_kib = 4 * (4 if args.precision == "fp32" else 2)
    if info.rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": N,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": round(value / BASELINE_IMG_S, 2),
            "dtype": args.precision, "data": "synthetic (random fp32 images, random-init weights)",
            "p50_latency_ms": None if p50 != p50 else round(p50, 4),
            "config": {"model": "cifar10-convnet (cifar_model_parts.py NeuralNetwork)",
                       "global_batch": int(round(imgs_per_gpu * N)), "seq_len": None, "parallelism": par,
                       "stages": 2, "microbatches": args.microbatches if N > 1 else 1,
                       "receiver_fill_images_per_step": getattr(args, "_fill_rows", 0),
                       "stage0_spare_cus": spare,
                       "stage_cut": {1: f"conv|fc (reference split, {hop_kib} KiB/img hop)",
                                     2: f"conv+fc1|fc2 ({hop_kib // 8} KiB/img hop)"}[args._cut]},
        }
        out.update(extra)
    if N > 1 and not args.no_extra:
        # GPT-2 small 4-stage decode ring across the GPUs (BASELINE config 3 at
        # N = 4: one stage per GPU, tokens back to stage 0 over RCCL).  Guarded:
        # a failure or hang here only drops these keys, never the headline line.
        g = guarded_multi_gpu_gpt(args, info, out if info.rank == 0 else None)
        if info.rank == 0 and g:
            out.update(g)
    if info.rank == 0:
        print(json.dumps(out), flush=True)
    if N > 1:
        from distributed_neural_networks_amd.parallel import comm
        comm.shutdown()
    return 0


def guarded_multi_gpu_gpt(args, info, line, limit_s: float = 150.0):
    """Run bench/gpt_bench.py's decode ring on all ranks under a timer: on a
    hang every rank exits 0 after ``limit_s`` (rank 0 first prints the CIFAR
    line it already has), on an exception the keys are skipped."""
    import threading
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench"))
    import gpt_bench

    def bail():
        if line is not None:
            line["gpt2_4stage_error"] = f"decode ring exceeded {limit_s:.0f} s; skipped"
            print(json.dumps(line), flush=True)
        os._exit(0)
    timer = threading.Timer(limit_s, bail)
    timer.daemon = True
    timer.start()
    try:
        if info.device.type == "cuda":
            ga = gpt_bench.parse(["--gpus", str(info.world), "--steps", "32", "--warmup", "4", "--batch", "64",
                                  "--prompt", "512", "--stages", "4", "--dtype", "bf16", "--prefill_iters", "3"])
        else:  # schedule-test mode (gloo): the same ring on the tiny model
            ga = gpt_bench.parse(["--gpus", str(info.world), "--cpu", "--model", "gpt2-tiny", "--steps", "3",
                                  "--warmup", "1", "--batch", "2", "--prompt", "8", "--stages", "4",
                                  "--prefill_iters", "1"])
        g = gpt_bench.run(ga)
    except Exception as e:  # noqa: BLE001
        g = None
        if line is not None:
            line["gpt2_4stage_error"] = f"{type(e).__name__}: {e}"[:200]
    finally:
        timer.cancel()
    if g is None:
        return {}
    return {"gpt2_4stage_decode_tok_s": g["value"], "gpt2_4stage_decode_ms_per_step": g["ms_per_step"],
            "gpt2_4stage_prefill_tok_s": g["prefill_tokens_per_s"],
            "gpt2_4stage_config": dict(g["config"], dtype="bf16" if info.device.type == "cuda" else "fp32",
                                       model=("gpt2 (124M, random init)" if info.device.type == "cuda"
                                              else "gpt2-tiny (schedule test)"),
                                       placement=f"{g['config']['gpu_groups']} GPU groups x "
                                                 f"{g['config']['replicas']} replicas, decode ring over RCCL")}


if __name__ == "__main__":
    sys.exit(main())
