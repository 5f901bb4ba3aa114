#!/usr/bin/env python3
"""Flagship benchmark: CIFAR-10 ConvNet 2-stage pipeline inference, images/s.

Metric/config from BASELINE.json (the reference's only measured headline:
CIFAR-10 2-stage images/s; 3.40-4.15 k img/s on CPU over localhost gRPC,
BASELINE.md).  Synthetic fp32 images, random-init weights of the reference
architecture.  Precision: the reference's fp32 contract, computed as **fp32
(bf16x3 split emulation, ~2^-16 relative per product, fp32 accumulation)**:
every product is three bf16 MFMA terms (ops/cifar.py); the line reports the
measured max|dprob| against fp32 torch on 4096 images (outside the timed
region).  ``--precision bf16`` is the reduced-precision variant (extra keys).
Every timed step runs the complete forward of both stages (conv stage +
fc/softmax/argmax stage) on fresh launches; nothing is cached across steps.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...

Placements (the stage cut is the reference's at every N: conv | fc1+fc2+softmax,
``cifar_model_parts.py:29-58``, an fp32 16 KiB/img hop):
* N = 1: both stages colocated on the GPU, one HIP graph per step; extra keys:
  the bf16 pipeline, the GPT-2 small 4-stage pipeline (decode / prefill
  tokens/s, p50 per-token latency; bench/gpt_bench.py) and BASELINE configs 4
  and 5 colocated (Llama-3 8B bf16 8-stage B=32, GPT-2 XL fp8 8-stage B=64).
* N > 1 (one process per GPU, RCCL; ``--placement pp2``, the headline): one
  pipeline stage per GPU — N/2 GPUs run stage 0, N/2 run stage 1.  The hop is
  bipartite: each stage-0 GPU cuts every microbatch into N/2 row slices and
  sends slice j to stage-1 GPU j, so a transfer uses N/2 direct xGMI links at
  once (``parallel/links.py SplitLink``; at N = 2 it is the single pair).
  The K steps stream as one fill/drain.  p50 latency = one image through stage
  0 -> RCCL hop -> stage 1 -> prediction back to stage 0 over the back-edge
  (the reference's request path, ``node.py:137-200``).  Extra keys: the
  fc1-cut plan (``--placement fc1cut``: conv+fc1 | fc2, replicated stage 0,
  receivers fill), and the GPT-2 4-stage, Llama-3 8B 8-stage and GPT-2 XL fp8
  8-stage decode rings across min(N, stages) GPU groups with per-token p50.
  ``--placement interleaved`` (opt-in): every GPU hosts stage 0 of its
  pipeline and stage 1 of the others; the hop is an all-to-all.
Scaling is weak: each stage-0 GPU sources ``--batch`` images per step.

``--model gpt2`` runs the GPT-2 4-stage token throughput bench instead
(bench/gpt_bench.py).
"""
from __future__ import annotations

import time

_T0 = time.perf_counter()  # process start, before torch loads: the --time_budget_s clock

import argparse
import json
import os
import statistics
import sys

import torch

BASELINE_IMG_S = 4150.0  # reference CIFAR-10 2-stage, best batch (255), CPU gRPC
METRIC = "images/sec CIFAR-10 2-stage"
DTYPE_LABEL = {"fp32": "fp32 (bf16x3 split emulation, ~2^-16 per product)", "bf16": "bf16"}
CPU_DTYPE_LABEL = "fp32 (torch CPU golden stages over gloo: schedule test, not a measurement)"
FP8_LABEL = ("fp8-e4m3 weights (W8A16 decode; prefill W8A8 on the scaled fp8 MFMA, e4m3 activations with "
             "MX e8m0 block scales per row x 128 columns), "
             "bf16 activations between kernels")


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
    ap.add_argument("--microbatches", type=int, default=8,
                    help="microbatches per step on N>1 (the hop of one overlaps the stage-0 compute of the next)")
    ap.add_argument("--placement", default="pp2", choices=["pp2", "fc1cut", "interleaved"],
                    help="N>1: pp2 = the reference topology and cut (one stage per GPU, RCCL send/recv, headline); "
                         "fc1cut = conv+fc1 | fc2 with replicated stage 0; interleaved = all-to-all variant")
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
                    help="stage boundary: 1 = after conv2/pool (reference), 2 = after fc1; auto = per placement")
    ap.add_argument("--verify_images", type=int, default=-1,
                    help="N>1 pp2: images each stage-0 GPU pushes through the distributed pipeline and checks "
                         "against fp32 torch after the timed run (0 = off, -1 = 4096 on GPUs, 256 with --cpu)")
    ap.add_argument("--extra_budget_s", type=float, default=420.0,
                    help="N>1: wall-clock cap of the extra keys (a hang only drops keys)")
    ap.add_argument("--time_budget_s", type=float, default=480.0,
                    help="whole-run wall-clock budget per rank, from process start: the N>1 extras get what "
                         "the headline left (minus a margin) and are skipped or cut when it runs out")
    ap.add_argument("--launch_timeout", type=float, default=-1.0,
                    help="N>1 without a launcher: wall-clock limit of the self-launched job "
                         "(-1 = --time_budget_s + 240 s)")
    a = ap.parse_args()
    if a.verify_images < 0:
        a.verify_images = 256 if a.cpu else VERIFY_IMAGES
    if a.launch_timeout < 0:
        a.launch_timeout = a.time_budget_s + 240.0
    return a


EXTRAS_MARGIN_S = 20.0  # kept back from the budget for the line itself and shutdown
FIDELITY_LAYERS = 48  # GPT-2 XL blocks in the fp8-vs-unquantised fidelity key (the whole model)


def elapsed_s() -> float:
    return time.perf_counter() - _T0


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
    # plain fp32 boundary: the blocked hi/lo encoding (ops/cifar.py) measured
    # neutral end to end (profiles/r3_boundary_ab.jsonl: fc1 -0.08 ms, the
    # stage-0 epilogue +0.09 ms)
    return CifarHipStage(sd0, 0, cut, device, precision), CifarHipStage(sd1, cut + 1, 3, device, precision)


def pick_cut(args, info) -> int:
    from distributed_neural_networks_amd.parallel.partition import cifar_cut
    if args.cut != "auto":
        return int(args.cut)
    if info.world == 1 or args.placement == "pp2":
        return 1  # the reference split (conv | fc)
    return cifar_cut("linear" if args.placement == "fc1cut" else args.placement, info.world,
                     precision=args.precision)


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


def bench_pp2(args, info):
    """BASELINE config 2 on N GPUs: the reference's 2-stage pipeline with its
    cut (conv | fc1+fc2+softmax, ``cifar_model_parts.py:29-58``), one stage per
    GPU.  Rank 2p runs stage 0 and rank 2p+1 stage 1 (pipeline p of N/2).
    The fp32 boundary (16 KiB/img) crosses a bipartite hop: every stage-0 GPU
    splits each microbatch into N/2 row slices, slice j to stage-1 GPU j,
    each pair on its own direct xGMI link (``SplitLink``; N = 2: one pair).
    No receiver fill: a stage-1 GPU runs only stage 1 on what it receives."""
    from distributed_neural_networks_amd.parallel import comm
    from distributed_neural_networks_amd.parallel.links import SplitLink, make_link
    from distributed_neural_networks_amd.runtime.scheduler import run_gpipe
    dev, N, r = info.device, info.world, info.rank
    if N % 2:
        raise ValueError(f"the 2-stage pipeline needs an even GPU count, got {N}")
    n = N // 2
    stage = r % 2
    s0, s1 = stages_for(dev, 1, args.precision)
    args._stages = (s0, s1)  # for the distributed correctness check (pp2_verify)
    M = max(1, args.microbatches)
    mb = (args.batch // M) // n * n  # rows per microbatch, split evenly over the N/2 receivers
    if mb < n:
        raise ValueError(f"--batch {args.batch} / {M} microbatches is too small to split over {n} receivers")
    g = torch.Generator(device=dev).manual_seed(1 + r)
    back = comm.back_group()
    if stage == 0:
        xs = [torch.randn((mb, 3, 32, 32), device=dev, generator=g) for _ in range(M)]
        nxt = SplitLink([make_link(2 * j + 1, dev) for j in range(n)])

        def stream(steps):
            run_gpipe(s0, steps * M, mb, None, nxt, source=lambda i: xs[i % M], depth=2)
    else:
        prev = SplitLink([make_link(2 * a, dev) for a in range(n)])

        def stream(steps):
            run_gpipe(s1, steps * M, mb, prev, None, depth=2)

    stream(args.warmup)
    t0 = sync_time(info)
    stream(args.steps)
    t1 = sync_time(info)
    p50 = pp2_latency(args, info, s0, s1, back)
    fabric = "rccl" if dev.type == "cuda" else "gloo-cpu"
    return t1 - t0, n * mb * M / N, p50, f"pp2-{fabric}-{n}x{n}" + ("-bipartite" if n > 1 else "")


def _settle(work, timeout_s: float) -> None:
    """Complete one link op on the host, bounded where the link allows it."""
    if hasattr(work, "ch"):  # native RCCL work: a bounded host wait
        work.synchronize(timeout_s)
    else:
        work.wait()


def agree(info, tag: str, err: str, store=None) -> str:
    """Every rank publishes its local verdict (``err``: "" = ok) through the
    process group's TCP store and reads everyone's: returns the first failure
    of any rank, or "".  No collective, so it holds when the failure is in the
    communicator itself — the ranks then skip the same section together
    instead of some of them blocking in a barrier the others never reach."""
    if info.world == 1:
        return err
    import torch.distributed as dist
    st = store or dist.distributed_c10d._get_default_store()
    seq = _AGREE_SEQ[0]
    _AGREE_SEQ[0] += 1
    st.set(f"dnn/agree/{tag}/{seq}/{info.rank}", err or "ok")
    for q in range(info.world):
        v = st.get(f"dnn/agree/{tag}/{seq}/{q}").decode(errors="replace")
        if v != "ok":
            return v
    return ""


_AGREE_SEQ = [0]


def hop_bandwidth(info, nbytes: int, reps: int = 4, timeout_s: float = 60.0) -> float:
    """GB/s of one stage hop, measured on its own: rank 2p sends ``nbytes``
    ``reps`` times to rank 2p+1 over the same link type as the pp2 hop (native
    RCCL channel, or ProcessGroupNCCL / gloo), every pair at once; the slowest
    pair's rate.  Reported next to the pp2 headline: the reference cut moves
    16 KiB per image, so at N >= 2 the headline is bounded by pairs x this
    rate / 16 KiB, whatever the stage kernels do.

    The link setup and a warm transfer (bounded by ``timeout_s``) run first
    and the ranks agree on their outcome through the store before any
    collective: one rank's failure skips the measurement on every rank
    (raising the same error everywhere) instead of leaving the others in the
    timing barrier."""
    from distributed_neural_networks_amd.parallel.links import make_link
    from distributed_neural_networks_amd.parallel import rccl
    r, N, dev = info.rank, info.world, info.device
    peer = r ^ 1
    el = 0.0
    with rccl.scope(dev):
        err = ""
        try:
            if peer < N:
                link = make_link(peer, dev)
                if hasattr(link, "ch"):
                    link.ch.ready(timeout_s)
                buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
                post = link.isend if r % 2 == 0 else link.irecv
                _settle(post(buf), timeout_s)  # warm: channel / communicator setup outside the timing
                op = link.send if r % 2 == 0 else link.recv
        except Exception as e:  # noqa: BLE001 — agreed below, raised on every rank
            err = f"rank {r}: {type(e).__name__}: {e}"[:200]
        bad = agree(info, "hop", err)
        if bad:
            raise RuntimeError(f"hop setup failed: {bad}")
        t0 = sync_time(info)
        if peer < N:
            for _ in range(reps):
                op(buf)
        el = sync_time(info) - t0
    el = max_over_ranks(info, el)
    return nbytes * reps / el / 1e9 if el > 0 else float("nan")


DEADLINE_RC = 3  # exit status of a run a Deadline cut short (its line is printed first)


class Deadline:
    """A wall-clock backstop for a multi-rank section: if the block is still
    running after ``seconds``, rank 0 prints the line it has (noting what was
    cut) and every rank exits with ``DEADLINE_RC``: a hang drops keys, never
    the headline, and still shows in the job's exit status."""

    def __init__(self, seconds: float, line, what: str):
        import threading
        self.what = what

        def bail():
            if line is not None:
                line["extras_error"] = f"{self.what} exceeded its {seconds:.0f} s budget; skipped"
                print(json.dumps(line), flush=True)
            else:
                time.sleep(3.0)  # rank 0 prints first: a launcher stops the job at the first exit
            sys.stdout.flush()
            os._exit(DEADLINE_RC)
        self.timer = threading.Timer(max(1.0, seconds), bail)
        self.timer.daemon = True

    def __enter__(self):
        self.timer.start()
        return self

    def __exit__(self, *exc):
        self.timer.cancel()
        return False


def pp2_latency(args, info, s0, s1, back) -> float:
    """p50 of one image through the pipeline as the reference serves a
    request (``node.py:137-200``): rank 0 runs stage 0, the 16 KiB boundary
    crosses to rank 1 over RCCL, rank 1 runs stage 1 and returns the
    prediction to rank 0 (``return_to_node_id``) over the back-edge.  Timed
    on rank 0 from the input on the device to the prediction back on it."""
    from distributed_neural_networks_amd.parallel.links import make_link
    dev, r = info.device, info.rank
    iters = max(3, min(args.latency_iters, 200))
    ts = []
    sync_time(info)
    if r == 0:
        x = torch.randn((1, 3, 32, 32), device=dev)
        y = torch.empty(s0.out_spec(1)[0], dtype=s0.out_spec(1)[1], device=dev)
        pred = torch.empty((1,), dtype=torch.int32, device=dev)
        fwd, ret = make_link(1, dev), make_link(1, dev, back)
        for _ in range(iters):
            dsync(dev)
            a = time.perf_counter()
            s0.forward(x, y)
            w = fwd.isend(y)
            ret.recv(pred)
            w.wait()
            dsync(dev)
            ts.append(time.perf_counter() - a)
    elif r == 1:
        y = torch.empty(s1.in_spec(1)[0], dtype=s1.in_spec(1)[1], device=dev)
        probs = torch.empty((1, 10), device=dev)
        fwd, ret = make_link(0, dev), make_link(0, dev, back)
        for _ in range(iters):
            fwd.recv(y)
            out = s1.forward(y, probs)
            ret.send(out.pred)
        dsync(dev)
    sync_time(info)
    return statistics.median(ts) * 1e3 if ts else float("nan")


VERIFY_IMAGES = 4096  # images each stage-0 GPU pushes through the distributed correctness check


def golden_probs(dev, x: torch.Tensor) -> torch.Tensor:
    """fp32 torch probabilities of the benchmarked weights (TF32 off): the oracle
    of ``precision_check`` and of the distributed check."""
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork
    ref = NeuralNetwork().to(dev).eval()
    ref.load_state_dict(ckpt.random_stage_state_dict("cifar10", 0, 3, True, True, 0))
    tf32 = torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32
    torch.backends.cudnn.allow_tf32 = torch.backends.cuda.matmul.allow_tf32 = False
    try:
        with torch.no_grad():
            return ref(x)
    finally:
        torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32 = tf32


def pp2_verify(info, s0, s1, n_img: int = VERIFY_IMAGES) -> dict:
    """The answer that crossed the hops, checked (the
    reference's one check is the prediction that comes back over the hop,
    ``node.py:58-68``, ``node.py:184-192``).  Every stage-0 GPU pushes a fixed
    seeded set of ``n_img`` images through the *distributed* pipeline the
    headline measured: its stage-0 kernel, the bipartite ``SplitLink`` hop to
    every stage-1 GPU, their stage-1 kernels; each stage-1 GPU returns the
    probabilities and its per-row predictions of every slice to the stage-0
    GPU the slice came from, over the back-edge communicator
    (``return_to_node_id``).  The stage-0 GPU compares what came back with the
    fp32 torch model on the same images.  Job-wide: argmax agreement (sum of
    matches over every stage-0 GPU's images), max |dprob| (max over them), and
    whether the returned predictions are the argmax of the returned
    probabilities.  Outside every timed region."""
    import torch.distributed as dist
    from distributed_neural_networks_amd.parallel import comm
    from distributed_neural_networks_amd.parallel.links import SplitLink, make_link
    dev, N, r = info.device, info.world, info.rank
    n = N // 2
    back = comm.back_group()
    vmb = max(n, (1024 if dev.type == "cuda" else 32) // n * n)  # rows per microbatch, split over n receivers
    V = max(vmb, n_img // vmb * vmb)
    stats = torch.zeros(4, dtype=torch.float64, device=dev)  # matches, images, max|dp|, pred==argmax(probs)
    if r % 2 == 0:
        g = torch.Generator(device=dev).manual_seed(7000 + r)
        x = torch.randn((V, 3, 32, 32), device=dev, generator=g)
        fwd = SplitLink([make_link(2 * j + 1, dev) for j in range(n)])
        ret = SplitLink([make_link(2 * j + 1, dev, back) for j in range(n)])
        sh, dt = s0.out_spec(vmb)
        y = torch.empty(sh, dtype=dt, device=dev)
        probs = torch.full((V, 10), float("nan"), device=dev)
        pred = torch.full((V,), -1, dtype=torch.int32, device=dev)
        for i in range(V // vmb):
            s0.forward(x[i * vmb:(i + 1) * vmb], y)
            w = fwd.isend(y)
            rp = ret.irecv(probs[i * vmb:(i + 1) * vmb])
            rq = ret.irecv(pred[i * vmb:(i + 1) * vmb])
            for wk in (w, rp, rq):
                wk.wait()
        dsync(dev)
        p = golden_probs(dev, x)
        stats[0] = float((pred.long() == p.argmax(1)).sum().item())
        stats[1] = float(V)
        stats[2] = float((probs - p).abs().max().item()) if bool(torch.isfinite(probs).all()) else float("inf")
        stats[3] = float((pred.long() == probs.argmax(1)).sum().item())
    else:
        prev = SplitLink([make_link(2 * a, dev) for a in range(n)])
        ret = SplitLink([make_link(2 * a, dev, back) for a in range(n)])
        sh, dt = s1.in_spec(vmb)
        yin = torch.empty(sh, dtype=dt, device=dev)
        pbuf = torch.empty((vmb, 10), device=dev)
        corrupt = os.environ.get("DNN_TEST_CORRUPT_VERIFY") == "1"  # tests: the check must see a bad hop
        for _ in range(V // vmb):
            prev.recv(yin)
            if corrupt:
                yin[::7].mul_(-1.0)
            out = s1.forward(yin, pbuf)
            ret.send(out.probs.contiguous())
            ret.send(out.pred.contiguous())
        dsync(dev)
    mx = torch.tensor([stats[2].item()], dtype=torch.float64, device=dev)
    sm = stats[[0, 1, 3]].clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm)
    matches, imgs, self_ok = (float(v) for v in sm.tolist())
    return {"dist_argmax_agreement_vs_fp32_torch": round(matches / imgs, 6) if imgs else None,
            "dist_max_abs_dprob": float(mx.item()),
            "dist_pred_is_argmax_of_returned_probs": round(self_ok / imgs, 6) if imgs else None,
            "dist_verify_images": int(imgs),
            "dist_verify_path": f"stage 0 x{n} -> bipartite hop -> stage 1 x{n} -> probs + preds back over the "
                                f"back-edge, vs fp32 torch"}


def bench_fc1cut(args, info):
    """Extra key (not the headline): the 2-stage pipeline cut after fc1
    (conv+fc1 | fc2+softmax, a 2 KiB/img hop), one stage per GPU, RCCL
    isend/irecv over the direct xGMI links (``parallel/partition.py::linear_plan``): n0 stage-0 GPUs
    each source ``--batch`` images per step and stream them to one of n1
    stage-1 GPUs.  The K timed steps run as ONE stream of K x M microbatches
    (fill and drain once, not per step).  A stage-1 GPU spends ~2 % of a
    round on fc2, so it also runs its own images through both stages between
    rounds (``receiver_fill_rows``; measured on one MI355X at 32768-row
    microbatches: stage 0 1.245 ms, stage 1 0.023 ms -> 27648 / 24576 / 19456
    own rows per round at N = 2 / 4 / 8, i.e. 1.84 / 3.75 / 7.59 GPUs of work
    instead of 1 / 3 / 7)."""
    from distributed_neural_networks_amd.parallel.links import make_link
    from distributed_neural_networks_amd.parallel.partition import linear_plan, linear_role
    from distributed_neural_networks_amd.runtime.scheduler import run_gpipe
    dev, N, r = info.device, info.world, info.rank
    plan = linear_plan(N, args.precision, cuts=(2,))
    cut = plan["cut"]
    role = linear_role(r, plan)
    s0, s1 = stages_for(dev, cut, args.precision)
    M = max(1, args.microbatches)
    mb = args.batch // M
    g = torch.Generator(device=dev).manual_seed(1 + r)
    if role["stage"] == 0:
        xs = [torch.randn((mb, 3, 32, 32), device=dev, generator=g) for _ in range(M)]
        nxt = make_link(role["send_to"], dev)

        def stream(steps):
            run_gpipe(s0, steps * M, mb, None, nxt, source=lambda i: xs[i % M], depth=2)
    else:
        prevs = [make_link(p, dev) for p in role["recv_from"]]
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
    par = f"pp2-fc1cut-{plan['n0']}x{plan['n1']}" + ("+fill" if local.item() > 0 else "")
    return t1 - t0, imgs_total_per_step / N, float(local.item()), par


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
                  "dtype": FP8_LABEL, "micro_batch": 64,
                  "prompt_len": 512}),
                ("gpt2xl_fp8_8stage_b64_kv8", ["--model", "gpt2-xl", "--stages", "8", "--batch", "64", "--prompt",
                                               "512", "--dtype", "fp8", "--kv", "fp8"],
                 {"model": "gpt2-xl (random init)", "stages": 8,
                  "dtype": FP8_LABEL + ", fp8-e4m3 KV cache",
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
        # the bf16 comparator of config 5's prefill: the same
        # GPT-2 XL 8-stage B=64 x 512 prefill with bf16 weights
        try:
            g = gpt_bench.run(gpt_bench.parse(["--gpus", "1", "--steps", "2", "--warmup", "1", "--prefill_iters", "1",
                                               "--model", "gpt2-xl", "--stages", "8", "--batch", "64", "--prompt",
                                               "512", "--dtype", "bf16"]))
            out["gpt2xl_bf16_8stage_b64_prefill_tok_s"] = g["prefill_tokens_per_s"]
        except Exception as e:  # noqa: BLE001
            out["gpt2xl_bf16_8stage_b64_prefill_error"] = f"{type(e).__name__}: {e}"[:200]
        torch.cuda.empty_cache()
        # what fp8 weights cost at the model level: the XL
        # stage against the fp32 golden on the ORIGINAL unquantised weights,
        # logits error and greedy-token agreement over 8 decode steps
        try:
            from distributed_neural_networks_amd.tools.fp8_fidelity import measure
            out["gpt2xl_fp8_vs_unquantised_fp32"] = dict(
                measure("gpt2-xl", FIDELITY_LAYERS, 64, 512, 8), layers=FIDELITY_LAYERS, batch=64, prompt=512,
                decode_steps=8)
        except Exception as e:  # noqa: BLE001
            out["gpt2xl_fp8_vs_unquantised_fp32_error"] = f"{type(e).__name__}: {e}"[:200]
        torch.cuda.empty_cache()
        # config 5's prefill on split activations (e4m3 hi + residual planes,
        # bf16-equivalent MFMA work; the former default, kept as a key)
        try:
            g = gpt_bench.run(gpt_bench.parse(["--gpus", "1", "--steps", "4", "--warmup", "1", "--prefill_iters", "1",
                                               "--model", "gpt2-xl", "--stages", "8", "--batch", "64", "--prompt",
                                               "512", "--dtype", "fp8", "--fp8_prefill", "split"]))
            out["gpt2xl_fp8_8stage_b64_prefill_split_tok_s"] = g["prefill_tokens_per_s"]
        except Exception as e:  # noqa: BLE001
            out["gpt2xl_fp8_8stage_b64_prefill_split_error"] = f"{type(e).__name__}: {e}"[:200]
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


def precision_check(dev, precision: str, n_img: int = 4096) -> dict:
    """max|dprob| and argmax agreement of the HIP pipeline (the benchmarked
    stages and weights) against the fp32 torch model (TF32 off), on n_img
    random images.  Outside every timed region."""
    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    s0, s1 = stages_for(dev, 1, precision)
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn((n_img, 3, 32, 32), device=dev, generator=g)
    out = ColocatedPipeline([s0, s1], n_img)(x)
    p = golden_probs(dev, x)
    dsync(dev)
    return {"max_abs_dprob_vs_fp32_torch": float((out.probs - p).abs().max().item()),
            "argmax_agreement_vs_fp32_torch": round(float((out.pred.long() == p.argmax(1)).float().mean().item()), 6),
            "precision_check_images": n_img}


def main():
    args = parse()
    from distributed_neural_networks_amd.parallel import selflaunch
    # `python bench.py --gpus N` with no launcher: spawn the N ranks here (the
    # parent never touches the GPU) and relay rank 0's line
    rc = selflaunch.maybe_self_launch(args.gpus, os.path.abspath(__file__), sys.argv[1:], args.launch_timeout)
    if rc is not None:
        return rc
    if args.model != "cifar10":
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench"))
        import gpt_bench
        return gpt_bench.main(args)
    phases = {"startup_s": round(elapsed_s(), 2)}
    tp = time.perf_counter()
    info = dist_setup(args.gpus, args.cpu)
    selflaunch.check_world(args.gpus, info.world)
    N = info.world
    p2p = "none"
    if N > 1:
        from distributed_neural_networks_amd.parallel import comm
        from distributed_neural_networks_amd.parallel.links import native_preflight
        comm.back_group()  # collective: the back-edge communicator (latency path, decode rings)
        # native RCCL channels checked on a ring first; any failure -> ProcessGroupNCCL P2P
        p2p = native_preflight(info.device)
    args._cut = pick_cut(args, info)
    spare = args.s0_spare_cus if args.s0_spare_cus >= 0 else (16 if N > 1 else 0)
    if info.device.type != "cuda":
        spare = 0
    if spare and info.device.type == "cuda":
        # the stage-0 kernel holds every VGPR of the CUs it runs on, so without
        # spare CUs the RCCL send kernels only start between stage-0 launches
        # and each hop is exposed; 16 of 256 CUs (2 per XCD) stay free
        from distributed_neural_networks_amd.ops import cifar as cops
        n_cu = torch.cuda.get_device_properties(info.device).multi_processor_count
        cops.set_stage0_grid(max(1, n_cu - spare))
    fill = 0.0
    phases["init_s"] = round(time.perf_counter() - tp, 2)
    tp = time.perf_counter()
    from distributed_neural_networks_amd.parallel import rccl
    with rccl.scope(info.device):  # this placement's native channels close when it is measured
        if N == 1:
            el, imgs_per_gpu, p50, par = bench_colocated(args, info)
        elif args.placement == "interleaved":
            el, imgs_per_gpu, p50, par = bench_interleaved(args, info)
        elif args.placement == "fc1cut":
            el, imgs_per_gpu, fill, par = bench_fc1cut(args, info)
            p50 = float("nan")
        else:
            el, imgs_per_gpu, p50, par = bench_pp2(args, info)
    el = max_over_ranks(info, el)
    total = imgs_per_gpu * N * args.steps
    value = total / el
    extra = {}
    phases["headline_s"] = round(time.perf_counter() - tp, 2)
    if N == 1 and not args.no_extra and info.device.type == "cuda":
        tp = time.perf_counter()
        extra = extra_keys(args, info)
        phases["extras_s"] = round(time.perf_counter() - tp, 2)
    hop_kib = 4 * (4 if args.precision == "fp32" else 2)
    out = None
    if info.rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": N,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": round(value / BASELINE_IMG_S, 2),
            "dtype": DTYPE_LABEL[args.precision] if info.device.type == "cuda" else CPU_DTYPE_LABEL,
            "data": "synthetic (random fp32 images, random-init weights)",
            "p50_latency_ms": None if p50 != p50 else round(p50, 4),
            "config": {"model": "cifar10-convnet (cifar_model_parts.py NeuralNetwork)",
                       "global_batch": int(round(imgs_per_gpu * N)), "seq_len": None, "parallelism": par,
                       "stages": 2, "microbatches": args.microbatches if N > 1 else 1,
                       "receiver_fill_images_per_step": fill,
                       "stage0_spare_cus": spare, "p2p": p2p,
                       "stage_cut": {1: f"conv|fc (reference split, {hop_kib} KiB/img hop)",
                                     2: f"conv+fc1|fc2 ({hop_kib // 8} KiB/img hop)"}[args._cut]},
        }
        if info.device.type == "cuda" and args.precision == "fp32":
            tp = time.perf_counter()
            out.update(precision_check(info.device, args.precision, 16384))
            phases["precision_check_s"] = round(time.perf_counter() - tp, 2)
        out.update(extra)
    if N > 1 and args.placement == "pp2" and args.verify_images > 0:
        # the answer that crossed the hops, against fp32 torch (pp2_verify)
        tp = time.perf_counter()
        try:
            with Deadline(min(120.0, max(10.0, args.time_budget_s - elapsed_s() - EXTRAS_MARGIN_S)), out,
                          "distributed correctness check"):
                with rccl.scope(info.device):
                    ver = pp2_verify(info, *args._stages, n_img=args.verify_images)
            if out is not None:
                out.update(ver)
        except Exception as e:  # noqa: BLE001 — reported in the line, never silently dropped
            if out is not None:
                out["dist_verify_error"] = f"{type(e).__name__}: {e}"[:200]
        phases["dist_verify_s"] = round(time.perf_counter() - tp, 2)
    if N > 1 and args.placement == "pp2":
        tp = time.perf_counter()
        try:
            with Deadline(min(120.0, max(10.0, args.time_budget_s - elapsed_s() - EXTRAS_MARGIN_S)), out, "hop"):
                bw = hop_bandwidth(info, (4 << 20) if info.device.type != "cuda" else (256 << 20))
            if out is not None:
                pairs = N // 2
                out["hop_GBps_per_pair"] = round(bw, 2)
                out["hop_bound_images_per_s"] = round(pairs * bw * 1e9 / (hop_kib * 1024), 1)
        except Exception as e:  # noqa: BLE001 — a diagnostic: never costs the headline
            if out is not None:
                out["hop_GBps_error"] = f"{type(e).__name__}: {e}"[:200]
        phases["hop_s"] = round(time.perf_counter() - tp, 2)
    if N > 1 and not args.no_extra:
        multi_gpu_extras(args, info, out, phases)
    if out is not None:
        phases["total_s"] = round(elapsed_s(), 2)
        out["phase_s"] = phases
        out["time_budget_s"] = args.time_budget_s
    if info.rank == 0:
        print(json.dumps(out), flush=True)
    if N > 1:
        from distributed_neural_networks_amd.parallel import comm
        comm.shutdown()
    return 0


# extra decode rings at N > 1: (key, GPU argv, schedule-test argv on gloo CPU, config label)
RINGS = (
    ("gpt2_4stage", ["--model", "gpt2", "--stages", "4", "--batch", "64", "--prompt", "512", "--dtype", "bf16",
                     "--steps", "32", "--warmup", "4", "--prefill_iters", "3"],
     ["--model", "gpt2-tiny", "--stages", "4"], "gpt2 (124M, random init), bf16"),
    ("llama3_8b_8stage_b32", ["--model", "llama3-8b", "--stages", "8", "--batch", "32", "--prompt", "512",
                              "--dtype", "bf16", "--steps", "16", "--warmup", "2", "--prefill_iters", "1"],
     ["--model", "llama3-tiny", "--stages", "4"], "llama3-8b (random init), bf16"),
    ("gpt2xl_fp8_8stage_b64", ["--model", "gpt2-xl", "--stages", "8", "--batch", "64", "--prompt", "512",
                               "--dtype", "fp8", "--steps", "16", "--warmup", "2", "--prefill_iters", "1"],
     ["--model", "gpt2-tiny", "--stages", "4", "--dtype", "fp8"],
     "gpt2-xl (random init), " + FP8_LABEL),
)


def multi_gpu_extras(args, info, line, phases):
    """Extra keys at N > 1, on every rank, inside the run's time budget: the
    fc1-cut CIFAR plan, then the GPT-2 4-stage, Llama-3 8B 8-stage and GPT-2 XL
    fp8 8-stage decode rings across min(N, stages) GPU groups (tokens back to
    group 0 over RCCL) with per-token p50.  The extras get what the headline
    left of ``--time_budget_s`` (at most ``--extra_budget_s``); the ranks agree
    on the remaining time (the slowest rank's clock) before each section and
    skip the rest together when it is short.  A failure drops that key; a hang
    past the budget makes every rank exit 0 (rank 0 first prints the line it
    has), so the headline is never lost.  Each section's seconds go into
    ``phase_s``."""
    import copy
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench"))
    import gpt_bench
    from distributed_neural_networks_amd.parallel import comm, rccl

    def remaining() -> float:  # agreed: every rank runs the same collective here
        return args.time_budget_s - EXTRAS_MARGIN_S - max_over_ranks(info, elapsed_s())

    budget = min(args.extra_budget_s, remaining())
    if budget < 15.0:
        if line is not None:
            line["extras_skipped"] = f"time budget: {budget:.0f} s left of {args.time_budget_s:.0f} s"
        return
    t_end = time.perf_counter() + budget
    cuda = info.device.type == "cuda"
    # minimum seconds a section needs to be worth starting (setup + a few steps)
    need = {"fc1cut": 10.0, "gpt2_4stage": 20.0, "llama3_8b_8stage_b32": 45.0, "gpt2xl_fp8_8stage_b64": 45.0}
    with Deadline(budget, line, "extras") as dl:
        tp = time.perf_counter()
        dl.what = "fc1cut"
        try:
            a = copy.copy(args)
            a.latency_iters = 3
            with rccl.scope(info.device):
                el, imgs, fill, par = bench_fc1cut(a, info)
            el = max_over_ranks(info, el)
            if line is not None:
                line["fc1cut_images_per_s"] = round(imgs * info.world * args.steps / el, 1)
                line["fc1cut_ms_per_step"] = round(el / args.steps * 1e3, 4)
                line["fc1cut_config"] = {"parallelism": par, "receiver_fill_images_per_step": fill,
                                         "stage_cut": "conv+fc1|fc2 (2 KiB/img fp32 hop)"}
        except Exception as e:  # noqa: BLE001
            if line is not None:
                line["fc1cut_error"] = f"{type(e).__name__}: {e}"[:200]
        phases["fc1cut_s"] = round(time.perf_counter() - tp, 2)
        for key, argv_gpu, argv_cpu, label in RINGS:
            dl.what = key
            if cuda:
                torch.cuda.empty_cache()
            comm.barrier(info)
            left = max_over_ranks(info, t_end - time.perf_counter())
            if cuda and left < need[key]:
                if line is not None:
                    line[key + "_skipped"] = f"time budget: {left:.0f} s left"
                continue
            tp = time.perf_counter()
            argv = ["--gpus", str(info.world)] + (argv_gpu if cuda else
                                                  ["--cpu", "--steps", "3", "--warmup", "1", "--batch", "2",
                                                   "--prompt", "8", "--prefill_iters", "1"] + argv_cpu)
            try:
                with rccl.scope(info.device):  # each ring's channels close when the ring is measured
                    g = gpt_bench.run(gpt_bench.parse(argv), shutdown=False)
            except Exception as e:  # noqa: BLE001
                if line is not None:
                    line[key + "_error"] = f"{type(e).__name__}: {e}"[:200]
                g = None
            phases[key + "_s"] = round(time.perf_counter() - tp, 2)
            if line is not None and g is not None:
                c = g["config"]
                line[key + "_decode_tok_s"] = g["value"]
                line[key + "_decode_ms_per_step"] = g["ms_per_step"]
                line[key + "_prefill_tok_s"] = g["prefill_tokens_per_s"]
                line[key + "_p50_token_ms"] = g["decode_p50_token_latency_ms"]
                for k in ("dist_token_agreement_vs_colocated", "dist_first_token_agreement_vs_colocated",
                          "dist_verify_tokens", "dist_verify_steps"):
                    if k in g:
                        line[key + "_" + k] = g[k]
                line[key + "_config"] = dict(
                    c, model=label if cuda else f"{c['model']} (gloo schedule test)",
                    placement=f"{c['gpu_groups']} GPU groups x {c['replicas']} replicas, decode ring over "
                              + ("RCCL" if cuda else "gloo (CPU)"))


if __name__ == "__main__":
    sys.exit(main())
