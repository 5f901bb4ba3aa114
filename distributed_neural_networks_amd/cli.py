"""``node.py`` entry point: one pipeline stage per process (reference CLI).

``python node.py --node_id ID --config PATH [--input_image PATH]`` behaves like
the reference (``node.py:210-364``): banner, per-stage weight load, gRPC
server, and stage 0 initiates inference and prints
``[id] ***** FINAL PREDICTION (Index): k *****``.  Additive flags only.

Transports (config ``transport``):

* ``grpc`` (default, the reference's): nested ``SendTensor`` RPC chain, CPU or
  GPU compute per node; reference peers interoperate.
* ``colocated``: the process of the node given by ``--node_id`` hosts every
  stage on one GPU (HIP graph per step); other nodes have nothing to run.
* ``rccl`` / ``gloo``: one rank per stage (rank = ``part_index``), activations
  move with ``torch.distributed`` P2P (RCCL over xGMI on MI355X, gloo on CPU);
  the last stage returns predictions over the back-edge to
  ``return_to_node_id`` (resolved but unused in the reference, ``node.py:272-277``).
  With config ``replicas`` = R the pipeline runs as R data-parallel copies
  (``--replica r``, rank = r * num_parts + part_index, one GPU each): copy r
  serves requests r, r+R, ... (CIFAR) or its own batch of sequences (GPT/Llama).
* ``gloo_gpu``: the ``gloo`` schedules with the stages on the GPU (node
  ``device``, default 0; several ranks may share one device, which RCCL
  refuses) and every hop staged through pinned host memory with RCCL-like
  stream ordering (``parallel/links.py HostStagedLink``): the multi-process
  schedules run with device compute and HIP graphs on a 1-GPU box.
"""
from __future__ import annotations

import argparse
import asyncio
import os
import sys
import time
import traceback
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import checkpoint as ckpt
from .config import ConfigError, NodeContext, banner, load_node
from .models import cifar, default_ranges, model_info
from .utils.log import log, set_quiet


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X pipeline-parallel inference node")
    p.add_argument("--node_id", required=True, help="Unique ID for this node (e.g., node1)")
    p.add_argument("--config", required=True, help="Path to the JSON configuration file")
    p.add_argument("--input_image", help="Path to input image (only used by node with part_index 0)")
    # additive
    p.add_argument("--num_requests", type=int, default=1, help="requests stage 0 sends (default 1)")
    p.add_argument("--prompt", default=None, help="GPT/Llama: comma-separated token ids (default: random)")
    p.add_argument("--shutdown_pipeline", action="store_true",
                   help="stage 0 asks all peers to exit after its requests complete")
    p.add_argument("--serve_seconds", type=float, default=None, help="non-initiating nodes exit after this long")
    p.add_argument("--device", default=None, help="override device: cpu | cuda | cuda:N")
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--trace", default=None, help="write a Chrome trace (host + device spans) to this path")
    p.add_argument("--metrics", action="store_true", help="print one METRICS json line per stage at exit")
    p.add_argument("--replica", type=int, default=None,
                   help="data-parallel copy of the pipeline this process serves (config 'replicas'; "
                        "default: $DNN_REPLICA, else RANK // num_parts under torchrun, else 0)")
    p.add_argument("--dump_result", default=None,
                   help="stage 0 (grpc): save the final result tensor of the last request as .npy")
    return p


# --------------------------------------------------------------------------- input
def load_image(path: Optional[str], nid: str) -> torch.Tensor:
    """Resize(32,32) + ToTensor + Normalize(0.5,0.5) without torchvision
    (reference transform, ``node.py:142-144``); dummy ``randn`` on failure (``:149-154``)."""
    try:
        from PIL import Image
        img = Image.open(path).convert("RGB").resize((32, 32), Image.BILINEAR)
        a = np.asarray(img, dtype=np.float32) / 255.0
        t = torch.from_numpy(a).permute(2, 0, 1).contiguous()
        t = (t - 0.5) / 0.5
        t = t.unsqueeze(0)
        log(f"[{nid}] Loaded input image '{path}', shape: {t.shape}")
        return t
    except FileNotFoundError:
        log(f"[{nid}] Input image '{path}' not found. Using dummy data.")
    except Exception as e:  # noqa: BLE001
        log(f"[{nid}] Error loading image: {e}. Using dummy data.")
    return torch.randn(1, 3, 32, 32)


def make_prompt(ctx: NodeContext, prompt: Optional[str]) -> torch.Tensor:
    from .runtime.generate import make_prompts
    return make_prompts(ctx.pipeline, prompt)


def kv_needs(ctx: NodeContext, args) -> Tuple[int, int]:
    """(sequences, positions) the transformer KV caches are sized for, from the
    config (``micro_batch_size`` x ``num_microbatches``; prompt + decode steps)."""
    pipe = ctx.pipeline
    T = pipe.prompt_len or pipe.seq_len
    if getattr(args, "prompt", None):
        T = len([v for v in args.prompt.split(",") if v.strip()])
    return pipe.micro_batch_size * pipe.num_microbatches, T + max(1, pipe.decode_steps or 1)


def check_config_capacity(ctx: NodeContext, args) -> None:
    """Reject, before any weight is loaded, a run whose prompt + decode steps
    overflow the model's position table / block size."""
    info = model_info(ctx.pipeline.model)
    if info.family == "cifar":
        return
    _, n_pos = kv_needs(ctx, args)
    limit = getattr(info.cfg, "block_size", None) or getattr(info.cfg, "max_seq", None)
    if limit is not None and n_pos > limit:
        raise ConfigError(f"ERROR: prompt + decode_steps = {n_pos} positions exceeds the model's limit {limit}")


# --------------------------------------------------------------------------- stages
def stage_ranges(ctx: NodeContext) -> List[Tuple[int, int]]:
    from .parallel.partition import resolve_ranges
    pipe = ctx.pipeline
    info = model_info(pipe.model)
    given = [n.layers for n in pipe.stages]
    if all(g is None for g in given):
        return default_ranges(pipe.model, pipe.num_parts)
    return resolve_ranges(info.num_layers, pipe.num_parts, given)


def rccl_device_index(ctx: NodeContext, n_dev: int) -> int:
    """GPU of this rank on the rccl transport: the node's ``device`` (default
    its ``part_index``) plus ``replica * num_parts``.  Every (node, replica)
    of the config must map to its own visible GPU; RCCL would otherwise fail
    late with a duplicate-GPU error, so overlaps are a ConfigError up front."""
    pipe = ctx.pipeline

    def idx(node, rep):
        base = node.device if node.device is not None else node.part_index
        return base + rep * ctx.num_parts
    owner = {}
    for rep in range(pipe.replicas):
        for n in pipe.stages:
            i = idx(n, rep)
            if i >= n_dev:
                raise ConfigError(f"ERROR: node '{n.id}' replica {rep} needs GPU {i}, "
                                  f"but only {n_dev} are visible")
            if i in owner:
                raise ConfigError(f"ERROR: node '{n.id}' replica {rep} and node '{owner[i][0]}' replica "
                                  f"{owner[i][1]} both map to GPU {i} (rccl needs one GPU per rank)")
            owner[i] = (n.id, rep)
    return idx(ctx.node, ctx.replica)


def pick_device(ctx: NodeContext, override: Optional[str]) -> torch.device:
    if override:
        return torch.device(override)
    if torch.cuda.is_available() and ctx.pipeline.transport != "gloo":
        idx = ctx.node.device if ctx.node.device is not None else 0
        if ctx.pipeline.transport == "rccl":
            # one GPU per rank; replica r of a stage pinned to device d runs on d + r * num_parts
            idx = rccl_device_index(ctx, torch.cuda.device_count())
        return torch.device("cuda", idx)
    return torch.device("cpu")


def load_stage_weights(ctx: NodeContext, part: int, ranges, full_sd=None, device=None):
    """Per-stage weights; prints the reference's load messages (``node.py:294-317``)."""
    pipe = ctx.pipeline
    a, b = ranges[part]
    first, last = part == 0, part == pipe.num_parts - 1
    if ckpt.is_synthetic(pipe.model_weights):
        log(f"[{ctx.node_id}] Using synthetic random-init weights (seed {ckpt.synthetic_seed(pipe.model_weights)})")
        gen_dev = device if (device is not None and device.type == "cuda" and model_info(pipe.model).family != "cifar") else None
        return ckpt.random_stage_state_dict(pipe.model, a, b, first, last, ckpt.synthetic_seed(pipe.model_weights),
                                            device=gen_dev), full_sd
    if full_sd is None:
        log(f"[{ctx.node_id}] Loading full state dict...")
        full_sd = ckpt.load_full_state_dict(pipe.model_weights)
    log(f"[{ctx.node_id}] Loading model part {part}...")
    sd = ckpt.stage_state_dict(pipe.model, full_sd, a, b, first, last)
    unexpected = ckpt.unexpected_keys(pipe.model, full_sd, a, b, first, last)
    if pipe.model == "cifar10" and pipe.num_parts == 2:
        log(f"[{ctx.node_id}] Expect warnings for {'fc1, fc2' if part == 0 else 'conv1, conv2'} weights "
            f"(loaded by Node {1 - part})")
    if unexpected:
        log(f"[{ctx.node_id}] WARNING: Unexpected keys loading state dict: {unexpected}")
    return sd, full_sd


def build_stage(ctx: NodeContext, part: int, ranges, device: torch.device, full_sd=None, args=None):
    from .runtime.stages import CifarHipStage, TorchStage
    pipe = ctx.pipeline
    a, b = ranges[part]
    first, last = part == 0, part == pipe.num_parts - 1
    sd, full_sd = load_stage_weights(ctx, part, ranges, full_sd, device)
    fam = model_info(pipe.model).family
    if device.type == "cuda":
        if fam == "cifar":
            st = CifarHipStage(sd, a, b, device)
        else:
            from .runtime.transformer import build_device_stage
            n_seq, n_pos = kv_needs(ctx, args) if args is not None else (8, 1024)
            # activation buffers hold the largest single stage call: a whole
            # request over gRPC, else one microbatch x (prefill chunk | prompt)
            if pipe.transport == "grpc":
                ntok = n_seq * n_pos
            else:
                ntok = pipe.micro_batch_size * (min(pipe.prefill_chunk, n_pos) if pipe.prefill_chunk > 0 else n_pos)
            st = build_device_stage(pipe.model, sd, a, b, first, last, device, dtype=pipe.dtype,
                                    max_batch=n_seq, max_seq=n_pos, max_tokens=ntok,
                                    temperature=pipe.temperature, top_k=pipe.top_k, seed=pipe.seed,
                                    kv_dtype=pipe.kv_cache_dtype, kv_scale=pipe.kv_cache_scale,
                                    fp8_prefill=pipe.fp8_prefill)
    else:
        st = TorchStage(pipe.model, sd, a, b, first, last, device,
                        sampling=(pipe.temperature, pipe.top_k, pipe.seed))
    log(f"[{ctx.node_id}] Successfully loaded weights into stage {part} (layers [{a},{b}]) on {device}.")
    return st, full_sd


def _forward_fn(stage, fam: str):
    """(tensor) -> (output tensor, per-row prediction or None)."""
    from .runtime.stages import StageOutput

    def fwd(x):
        x = x.to(stage.device)
        y = stage.forward(x)
        if isinstance(y, StageOutput):
            if stage.device.type == "cuda":
                torch.cuda.synchronize(stage.device)
            return y.probs, y.pred.cpu()
        return y, None
    return fwd


# --------------------------------------------------------------------------- transports
async def run_grpc(ctx: NodeContext, args, stage) -> int:
    from .control.service import NodeClient, NodeServicer, decode_prediction, start_server, SHUTDOWN_MSG
    from .wire import codec, proto
    nid = ctx.node_id
    fam = model_info(ctx.pipeline.model).family
    fwd = _forward_fn(stage, fam)
    servicer = NodeServicer(nid, fwd, ctx.is_last, ctx.next_address, rpc_timeout_s=ctx.pipeline.rpc_timeout_s,
                            stage=ctx.part_index)
    args._servicer = servicer
    listen = f"[::]:{ctx.port}"
    try:
        server = await start_server(servicer, ctx.port)
        log(f"[{nid}] Starting gRPC server listening on {listen}")
        log(f"[{nid}] Server started successfully.")
    except RuntimeError as e:
        log(f"!!! [{nid}] CRITICAL ERROR: Failed to bind server to {listen}: {e}")
        log(f"!!! Check if port {ctx.port} is in use or network issues.")
        return 1
    rc = 0
    try:
        if ctx.part_index == 0 and (args.input_image or fam != "cifar"):
            rc = await initiate(ctx, args, stage, fwd, fam)
            if args.shutdown_pipeline:
                for n in ctx.pipeline.nodes:
                    if n.id != nid:
                        c = NodeClient(n.address)
                        try:
                            await c.message(proto.MessageRequest(sender_id=nid, message_text=SHUTDOWN_MSG), timeout=5)
                        except Exception:  # noqa: BLE001
                            pass
                        await c.close()
            return rc
        if ctx.part_index == 0:
            log("WARNING: Node 0 needs --input_image to start inference. Server will run, but no inference initiated.")
        log(f"[{nid}] Running event loop...")
        waiter = asyncio.ensure_future(servicer.shutdown_event.wait())
        await asyncio.wait([waiter], timeout=args.serve_seconds)
        return 0
    finally:
        log(f"[{nid}] Attempting server shutdown...")
        await servicer.close()
        await server.stop(grace=1)
        log(f"[{nid}] Server shutdown complete.")


async def initiate(ctx: NodeContext, args, stage, fwd, fam) -> int:
    """Stage-0 driver (reference ``initiate_inference``, ``node.py:137-200``)."""
    from .control.service import NodeClient, decode_prediction
    from .wire import codec, proto
    nid = ctx.node_id
    log(f"\n[{nid}] Initiating inference...")
    if ctx.num_parts > 1 and not ctx.next_address:
        log(f"[{nid}] ERROR: Cannot initiate inference, NEXT_NODE_ADDRESS is not set.")
        return 1
    client = NodeClient(ctx.next_address) if ctx.num_parts > 1 else None
    # readiness barrier over every downstream stage (replaces the reference's sleep(2))
    for n in ctx.pipeline.stages[1:]:
        c = client if n.address == ctx.next_address else NodeClient(n.address)
        ok = await c.wait_ready(ctx.pipeline.health_timeout_s)
        if c is not client:
            await c.close()
        if not ok:
            log(f"!!! [{nid}] node {n.id} ({n.address}) did not become healthy")
            if client is not None:
                await client.close()
            return 1
    rc = 0
    # a CIFAR request is micro_batch_size x num_microbatches images (1 by default:
    # the reference's single image); with --metrics, stage 0 records every
    # request's end-to-end latency (forward, hop(s), result back) — the number
    # BASELINE.md's survey measured for the reference
    rows = ctx.pipeline.micro_batch_size * ctx.pipeline.num_microbatches if fam == "cifar" else 1
    met = getattr(getattr(args, "_servicer", None), "metrics", None)
    for r in range(args.num_requests):
        x = cifar_request(args, nid, rows, r) if fam == "cifar" else make_prompt(ctx, args.prompt)
        t_req = time.perf_counter()
        log(f"[{nid}] Running model part {ctx.part_index}...")
        loop = asyncio.get_running_loop()
        if fam == "cifar" and client is not None and ctx.pipeline.num_microbatches > 1:
            # microbatches streamed down the pipeline: microbatch k's hop and the
            # downstream stages run while this stage computes k + 1 (the
            # servicers serialise their compute, not their transfers)
            ok = await _initiate_microbatches(ctx, args, client, fwd, x, r, t_req, met)
            rc = rc if ok else 1
            continue
        out, pred = await loop.run_in_executor(None, fwd, x)
        if client is None:  # single-stage pipeline
            p = pred.tolist()
            log(f"[{nid}] ***** FINAL PREDICTION (Index): {p[0] if len(p) == 1 else p} *****")
            continue
        out = out.detach().cpu()
        if out.is_floating_point():
            out = out.float()
        log(f"[{nid}] Computed intermediate output shape: {tuple(out.shape)}")
        log(f"[{nid}] Sending intermediate tensor to {ctx.next_address}...")
        req = proto.TensorRequest(request_id=f"{ctx.pipeline.model}_pipe_{ctx.num_parts}node_{r:03d}",
                                  tensor=codec.encode(out))
        try:
            import grpc
            resp = await client.send_tensor(req)
            log(f"[{nid}] Received final status from pipeline: {resp.status}")
            pred = decode_prediction(resp)
            if pred is not None and args.dump_result:
                np.save(args.dump_result, codec.decode_numpy(resp.result_tensor))
            if pred is None:
                log(f"[{nid}] Final result status received, but tensor not included in response.")
                rc = 1
            else:
                if met is not None:
                    met.record(time.perf_counter() - t_req, rows)
                p = pred.tolist()
                log(f"[{nid}] ***** FINAL PREDICTION (Index): {p[0] if len(p) == 1 else p} *****")
        except Exception as e:  # noqa: BLE001
            log(f"!!! [{nid}] SendTensor RPC failed during initiation: {e}")
            rc = 1
    await client.close() if client is not None else None
    return rc


async def _initiate_microbatches(ctx: NodeContext, args, client, fwd, x, r: int, t_req: float, met) -> bool:
    """One CIFAR request as ``num_microbatches`` SendTensor calls in flight at
    once (``initiate``): per-row predictions concatenated in microbatch order."""
    from .control.service import decode_prediction
    from .wire import codec, proto
    import grpc
    nid, mbs = ctx.node_id, ctx.pipeline.micro_batch_size
    loop = asyncio.get_running_loop()
    sends = []
    for k in range((x.shape[0] + mbs - 1) // mbs):
        out, _ = await loop.run_in_executor(None, fwd, x[k * mbs:(k + 1) * mbs])
        out = out.detach().cpu()
        if out.is_floating_point():
            out = out.float()
        req = proto.TensorRequest(request_id=f"{ctx.pipeline.model}_pipe_{ctx.num_parts}node_{r:03d}_mb{k}",
                                  tensor=codec.encode(out))
        sends.append(asyncio.ensure_future(client.send_tensor(req)))
    try:
        resps = await asyncio.gather(*sends)
    except grpc.aio.AioRpcError as e:
        log(f"!!! [{nid}] SendTensor RPC failed during initiation: {e}")
        return False
    preds = [decode_prediction(rp) for rp in resps]
    if any(p is None for p in preds):
        log(f"[{nid}] Final result status received, but tensor not included in response.")
        return False
    if met is not None:
        met.record(time.perf_counter() - t_req, int(x.shape[0]))
    p = np.concatenate(preds).tolist()
    log(f"[{nid}] ***** FINAL PREDICTION (Index): {p} *****")
    return True


def cifar_request(args, nid: str, rows: int, tag: int) -> torch.Tensor:
    """One CIFAR request of ``rows`` images: row 0 is ``--input_image`` (reference
    transform, or the reference's random dummy), rows 1.. are seeded synthetic
    images (``micro_batch_size`` x ``num_microbatches`` > 1 runs)."""
    x = load_image(args.input_image, nid)
    if rows > 1:
        g = torch.Generator().manual_seed(1000 + tag)
        x = torch.cat([x, torch.randn((rows - 1, 3, 32, 32), generator=g)])
    return x


def _fmt(preds) -> str:
    p = preds.tolist() if hasattr(preds, "tolist") else list(preds)
    return str(p[0] if len(p) == 1 else p)


def run_colocated(ctx: NodeContext, args, device) -> int:
    """All stages on one GPU in this process; every request of
    ``micro_batch_size * num_microbatches`` rows runs microbatch by microbatch
    through one captured HIP graph (CIFAR) or the decode ring (transformers)."""
    from .runtime.pipeline import ColocatedPipeline
    nid = ctx.node_id
    pipe = ctx.pipeline
    if ctx.part_index != 0:
        log(f"[{nid}] colocated transport: all stages run in the part-0 process; nothing to do here.")
        return 0
    ranges = stage_ranges(ctx)
    fam = model_info(pipe.model).family
    full = None
    stages = []
    for p in range(ctx.num_parts):
        st, full = build_stage(ctx, p, ranges, device, full, args)
        stages.append(st)
    if fam != "cifar":
        from .runtime.generate import run_generate_colocated
        return run_generate_colocated(ctx, args, stages, device)
    mbs, M = pipe.micro_batch_size, pipe.num_microbatches
    cp = ColocatedPipeline(stages, mbs)
    if device.type == "cuda":
        cp.capture()
    for r in range(args.num_requests):
        x = cifar_request(args, nid, mbs * M, r).to(device)
        preds = []
        for i in range(M):
            preds.append(cp(x[i * mbs:(i + 1) * mbs]).pred.clone())
        log(f"[{nid}] ***** FINAL PREDICTION (Index): {_fmt(torch.cat(preds).cpu())} *****")
    return 0


def run_dist(ctx: NodeContext, args, device) -> int:
    """One rank per stage over torch.distributed P2P (RCCL over xGMI / gloo),
    microbatched (``runtime/scheduler.py``), with the failure watchdog."""
    from .parallel import comm
    from .parallel.watchdog import Watchdog
    nid = ctx.node_id
    pipe = ctx.pipeline
    backend = "nccl" if pipe.transport == "rccl" else "gloo"
    if pipe.transport == "gloo_gpu" and device.type != "cuda":
        log(f"[{nid}] ERROR: transport 'gloo_gpu' needs a GPU")
        return 1
    if backend == "nccl" and device.type != "cuda":
        log(f"[{nid}] ERROR: transport 'rccl' needs a GPU")
        return 1
    if pipe.transport == "gloo":
        device = torch.device("cpu")
    s0 = pipe.stage(0)
    info = comm.init(backend, rank=ctx.rank, world=ctx.world, master_addr=s0.host,
                     timeout_s=pipe.comm_timeout_s, master_port=s0.port + comm.PORT_OFFSET, device_index=device.index)
    if pipe.transport == "gloo_gpu":
        # gloo process group, stages on the GPU: hops stage through pinned host
        # memory (parallel/links.py HostStagedLink); ranks may share a device
        import dataclasses
        torch.cuda.set_device(device)
        info = dataclasses.replace(info, device=device)
    comm.back_group()  # collective: the back-edge's own communicator
    if pipe.transport == "rccl":
        from .parallel.links import native_preflight
        mode = native_preflight(info.device)
        if mode != "native":
            log(f"[{nid}] stage hops: {mode}")
    fam = model_info(pipe.model).family
    # the watchdog runs from here on, so a rank that fails while loading its
    # weights takes the pipeline down within heartbeat_timeout_s instead of
    # leaving its peers in the first barrier for comm_timeout_s
    wd = Watchdog(info.rank, info.world, peer_timeout_s=pipe.heartbeat_timeout_s,
                  stall_timeout_s=pipe.stall_timeout_s, tag=f"[{nid}]")
    wd.start()
    try:
        ranges = stage_ranges(ctx)
        stage, _ = build_stage(ctx, ctx.part_index, ranges, info.device, None, args)
    except FileNotFoundError:
        log(f"[{nid}] ERROR: Weights file not found at '{ctx.model_weights}'")
        wd.abort("weights file not found")
        return 1
    except Exception as e:  # noqa: BLE001
        log(f"[{nid}] ERROR loading model/weights: {e}")
        traceback.print_exc()
        wd.abort(f"stage build failed: {type(e).__name__}: {e}")
        return 1  # only reached when exit_fn does not exit (tests)
    comm.barrier(info)
    rep = f", replica {ctx.replica}" if pipe.replicas > 1 else ""
    log(f"[{nid}] rank {info.rank}/{info.world} ready on {info.device} (backend {backend}{rep})")
    rc = 0
    try:
        wd.busy(True)
        if fam != "cifar":
            from .runtime.generate import run_generate_dist
            rc = run_generate_dist(ctx, args, stage, info, progress=wd.beat)
        else:
            rc = _cifar_stream(ctx, args, stage, info, wd)
        wd.busy(False)
    except Exception as e:  # noqa: BLE001 — a failed rank takes the pipeline down
        log(f"!!! [{nid}] pipeline error: {e}")
        traceback.print_exc()
        wd.abort(f"{type(e).__name__}: {e}")
        return 1  # only reached when exit_fn does not exit (tests)
    wd.done()
    comm.barrier(info)
    wd.stop()
    comm.shutdown()
    return rc


def _cifar_stream(ctx: NodeContext, args, stage, info, wd) -> int:
    from .parallel import comm
    from .parallel.links import make_link
    from .runtime.scheduler import ForwardLinks, ForwardPipeline
    nid, pipe, dev = ctx.node_id, ctx.pipeline, info.device
    r, S = ctx.part_index, ctx.num_parts
    ret = pipe.by_id(pipe.return_to_node_id) if pipe.return_to_node_id else None
    ret_part = ret.part_index if ret is not None else 0
    last = r == S - 1
    peer = ctx.peer  # ranks of this replica's stages
    bg = comm.back_group()
    links = ForwardLinks(prev=make_link(peer(r - 1), dev) if r > 0 else None,
                         nxt=make_link(peer(r + 1), dev) if not last else None,
                         ret_out=make_link(peer(ret_part), dev, bg) if (last and ret_part != r) else None,
                         ret_in=make_link(peer(S - 1), dev, bg) if (r == ret_part and not last) else None)
    rep = f" (replica {ctx.replica})" if pipe.replicas > 1 else ""

    def on_result(role, tag, preds):
        if role == "last":
            log(f"[{nid}]{rep} Final Prediction Index: {_fmt(preds)}")
        else:
            log(f"[{nid}]{rep} ***** FINAL PREDICTION (Index): {_fmt(preds)} *****")

    fp = ForwardPipeline(stage, links, r == 0, last, r == ret_part, depth=2, progress=wd.beat, on_result=on_result)
    mbs, M = pipe.micro_batch_size, pipe.num_microbatches
    if r == 0:
        # data parallel: replica k serves requests k, k+R, k+2R, ... (the tag keeps the global number)
        for req in range(ctx.replica, args.num_requests, pipe.replicas):
            x = cifar_request(args, nid, mbs * M, req).to(dev)
            fp.run_request(x, mbs, M, tag=req)
        fp.stop()
    else:
        fp.serve()
    return 0


def _finish(args) -> None:
    from .utils import trace
    sv = getattr(args, "_servicer", None)
    if sv is not None and args.metrics:
        sv.metrics.emit(force=True)
    p = trace.flush()
    if p:
        log(f"[{args.node_id}] trace written to {p}")


def _replica_arg(args) -> int:
    """--replica, else $DNN_REPLICA, else (under torchrun) RANK // num_parts of the config, else 0."""
    if args.replica is not None:
        return args.replica
    if os.environ.get("DNN_REPLICA"):
        return int(os.environ["DNN_REPLICA"])
    if "RANK" in os.environ:
        try:
            import json
            n = int(json.load(open(args.config)).get("num_parts", 1))
            return int(os.environ["RANK"]) // max(1, n)
        except (OSError, ValueError):
            return 0
    return 0


def main(argv=None) -> int:
    log("Script started...")
    args = build_parser().parse_args(argv)
    set_quiet(args.quiet)
    if args.trace:
        from .utils import trace
        trace.enable(args.trace)
    nid = args.node_id
    log(f"Parsed Node ID: {nid}")
    try:
        ctx = load_node(args.config, nid, _replica_arg(args))
        log(f"Loaded configuration from {args.config}")
        check_config_capacity(ctx, args)
        device = pick_device(ctx, args.device)
    except ConfigError as e:
        print(str(e), flush=True)
        return 1
    log(banner(ctx, str(device)))
    try:
        transport = ctx.pipeline.transport
        if transport == "colocated":
            return run_colocated(ctx, args, device)
        if transport in ("rccl", "gloo", "gloo_gpu"):
            return run_dist(ctx, args, device)
        ranges = stage_ranges(ctx)
        stage, _ = build_stage(ctx, ctx.part_index, ranges, device, None, args)
    except FileNotFoundError:
        log(f"[{nid}] ERROR: Weights file not found at '{ctx.model_weights}'")
        return 1
    except Exception as e:  # noqa: BLE001
        log(f"[{nid}] ERROR loading model/weights: {e}")
        traceback.print_exc()
        return 1
    try:
        return asyncio.run(run_grpc(ctx, args, stage))
    except KeyboardInterrupt:
        log(f"\n[{nid}] KeyboardInterrupt received, shutting down...")
        return 0
    finally:
        log(f"[{nid}] Event loop closed. Exiting.")
        _finish(args)
