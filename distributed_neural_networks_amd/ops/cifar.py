"""CIFAR-10 ConvNet on the fused gfx950 kernels.

Two precisions, packed once at load (reference ``node.py:305-306`` only moves
fp32 modules to the device):

* ``fp32`` (the reference's precision, default): ``csrc/kernels/cifar_x3.hip``.
  Every fp32 operand is split into bf16 hi + lo and each product is three bf16
  MFMAs (hi*hi + hi*lo + lo*hi) accumulated in fp32.  Stage boundary tensor
  ``(B,4096)`` fp32 exactly as the reference ships it (``node.py:45-48``).
  fc1 at large batch is ``cifar_fc1_x3``: the fp32 boundary rows are split in
  registers while staged to LDS (A read once as fp32, no split copy); at small
  batch (too few 256-row tiles to fill the chip) it runs as ONE skinny/128^2
  bf16 GEMM over K' = 3*4096 on ``[A_hi | A_hi | A_lo]`` x ``[W_hi | W_lo | W_hi]``.
  Optional boundary encoding ``boundary="split"`` (fp32 only, both ends of
  the hop must be these kernels): the same 16 KiB/img, each row as 32-k blocks
  of 32 bf16 hi then 32 bf16 lo — the very hi/lo operands the x3 MFMAs consume
  (hi + lo = the fp32 value to ~2^-17) — written by the stage-0 epilogue and
  staged into LDS by DMA in fc1 (no register split pass): fc1 0.710 -> 0.632
  ms at B=65536 with bit-identical outputs (profiles/r3_fc1_split_ab.jsonl),
  but the split stores cost the stage-0 epilogue as much, so the 2-stage step
  is unchanged (2.541 vs 2.548 ms, profiles/r3_boundary_ab.jsonl) and the
  pipelines keep plain fp32 (also the wire format a reference peer expects).
  ``decode_boundary`` / ``encode_boundary`` convert.
* ``bf16``: ``csrc/kernels/cifar_fused.hip`` (v4 persistent kernel), bf16
  boundary, an explicitly reduced-precision mode.

Weight layouts:

* conv1 ``(32,3,3,3)`` -> ``[32][48]`` with ``k = ky*16 + kx*4 + c`` (kx<3, c<3 real);
* conv2 ``(64,32,3,3)`` -> ``[64][288]`` with ``k = (ky*3+kx)*32 + c`` (HWC activation image);
* fc1 ``[512][4096]`` (K-contiguous for the GEMM), fc2 ``(10,512)`` -> ``[16][512]``
  zero-padded to one MFMA N-tile.  Biases are fp32.
The flatten order is the reference's NCHW ``c*64 + h*8 + w`` (``cifar_model_parts.py:41``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

from ._lib import check, lib, ptr, stream_ptr
from .gemm import ACT_RELU, linear

PRECISIONS = ("fp32", "bf16")


def split_bf16(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 -> (hi, lo) bf16 with hi + lo == w to ~2^-17 relative."""
    w = w.float()
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    return hi, lo


def _conv1_k48(sd) -> torch.Tensor:
    w = torch.zeros(32, 3, 4, 4)  # (oc, ky, kx, c) zero-padded kx=3, c=3
    w[:, :, :3, :3] = sd["conv1.weight"].float().permute(0, 2, 3, 1)
    return w.reshape(32, 48)


def _conv2_k288(sd) -> torch.Tensor:
    return sd["conv2.weight"].float().permute(0, 2, 3, 1).reshape(64, 288)  # (oc, ky, kx, c)


def _fc2_pad(sd) -> torch.Tensor:
    w = torch.zeros(16, 512)
    w[:10] = sd["fc2.weight"].float()
    return w


@dataclass
class CifarStage0Weights:
    precision: str
    b1: torch.Tensor
    b2: torch.Tensor
    w1: torch.Tensor = None    # bf16: [32][48]
    w2: torch.Tensor = None    # bf16: [64][288]
    w1h: torch.Tensor = None   # fp32 path: split conv weights
    w1l: torch.Tensor = None
    w2h: torch.Tensor = None
    w2l: torch.Tensor = None


@dataclass
class CifarHeadWeights:
    precision: str
    w_fc1: torch.Tensor = None   # bf16: [512][4096]; fp32: [512][3*4096] = [hi | lo | hi] (small batch)
    w_fc1h: torch.Tensor = None  # fp32 path, large batch: W hi / lo [512][4096] each (cifar_fc1_x3)
    w_fc1l: torch.Tensor = None
    b_fc1: torch.Tensor = None
    w_fc2: torch.Tensor = None   # bf16: [16][512]
    w_fc2h: torch.Tensor = None  # fp32 path: split fc2
    w_fc2l: torch.Tensor = None
    b_fc2: torch.Tensor = None


def _check_precision(p: str) -> str:
    if p not in PRECISIONS:
        raise ValueError(f"CIFAR precision must be one of {PRECISIONS}, got {p!r}")
    return p


def pack_stage0(sd: Dict[str, torch.Tensor], device, precision: str = "fp32") -> CifarStage0Weights:
    _check_precision(precision)
    b1 = sd["conv1.bias"].float().to(device).contiguous()
    b2 = sd["conv2.bias"].float().to(device).contiguous()
    w1, w2 = _conv1_k48(sd), _conv2_k288(sd)
    if precision == "bf16":
        return CifarStage0Weights("bf16", b1, b2,
                                  w1=w1.to(device=device, dtype=torch.bfloat16).contiguous(),
                                  w2=w2.to(device=device, dtype=torch.bfloat16).contiguous())
    (w1h, w1l), (w2h, w2l) = split_bf16(w1), split_bf16(w2)
    dv = lambda t: t.to(device).contiguous()  # noqa: E731
    return CifarStage0Weights("fp32", b1, b2, w1h=dv(w1h), w1l=dv(w1l), w2h=dv(w2h), w2l=dv(w2l))


def pack_head(sd: Dict[str, torch.Tensor], device, fc1: bool = True, fc2: bool = True,
              precision: str = "fp32") -> CifarHeadWeights:
    _check_precision(precision)
    w = CifarHeadWeights(precision)
    if fc1:
        f = sd["fc1.weight"].float()
        if precision == "bf16":
            w.w_fc1 = f.to(device=device, dtype=torch.bfloat16).contiguous()
        else:
            hi, lo = split_bf16(f)
            w.w_fc1 = torch.cat([hi, lo, hi], dim=1).to(device).contiguous()
            w.w_fc1h, w.w_fc1l = hi.to(device).contiguous(), lo.to(device).contiguous()
        w.b_fc1 = sd["fc1.bias"].float().to(device).contiguous()
    if fc2:
        f2 = _fc2_pad(sd)
        if precision == "bf16":
            w.w_fc2 = f2.to(device=device, dtype=torch.bfloat16).contiguous()
        else:
            hi, lo = split_bf16(f2)
            w.w_fc2h, w.w_fc2l = hi.to(device).contiguous(), lo.to(device).contiguous()
        w.b_fc2 = sd["fc2.bias"].float().to(device).contiguous()
    return w


def act_dtype(precision: str) -> torch.dtype:
    """dtype of the stage-boundary activations (flattened conv map, fc1 hidden)."""
    return torch.float32 if _check_precision(precision) == "fp32" else torch.bfloat16


STAGE0_GRID = 0  # persistent stage-0 workgroups; 0 = one per CU (256)
# fused fp32 fc1 from this batch on: 2 x B/256 tiles of 128 k32 steps each need
# >= 128 tiles to occupy the chip; below, split3 + the K-concat GEMM is faster
FC1_X3_MIN_ROWS = 16384


def set_stage0_grid(grid: int = 0) -> None:
    """Persistent stage-0 grid size (0 = one workgroup per CU).  With fewer
    workgroups than CUs the spare CUs stay free for concurrent kernels (an RCCL
    hop kernel cannot start a workgroup on a CU the stage-0 kernel holds)."""
    global STAGE0_GRID
    STAGE0_GRID = int(grid)


def _check_act(t: torch.Tensor, shape, dtype, what: str) -> None:
    if t.dtype != dtype or tuple(t.shape[1:]) != tuple(shape) or not t.is_contiguous():
        raise ValueError(f"{what}: expected contiguous {dtype} (B,{','.join(map(str, shape))}), "
                         f"got {t.dtype} {tuple(t.shape)}")


BOUNDARIES = ("fp32", "split")


def _split_boundary(boundary: str, precision: str) -> int:
    if boundary not in BOUNDARIES:
        raise ValueError(f"boundary must be one of {BOUNDARIES}, got {boundary!r}")
    if boundary == "split" and precision != "fp32":
        raise ValueError("the split boundary encoding exists for the fp32 precision only")
    return int(boundary == "split")


def encode_boundary(h: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 (B,K) -> the blocked hi/lo boundary encoding (same shape and dtype)."""
    out = torch.empty_like(h) if out is None else out
    check(lib().cifar_split_blocked(ptr(h), ptr(out), h.shape[0], h.shape[1], 0, stream_ptr()), "encode_boundary")
    return out


def decode_boundary(h: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Blocked hi/lo boundary encoding -> fp32 values (hi + lo)."""
    out = torch.empty_like(h) if out is None else out
    check(lib().cifar_split_blocked(ptr(h), ptr(out), h.shape[0], h.shape[1], 1, stream_ptr()), "decode_boundary")
    return out


def stage0_forward(x: torch.Tensor, w: CifarStage0Weights, out: Optional[torch.Tensor] = None,
                   grid: int = 0, boundary: str = "fp32") -> torch.Tensor:
    """Units 0-1: x (B,3,32,32) fp32 contiguous -> (B,4096) fp32 (or bf16 in bf16 mode;
    ``boundary="split"``: the blocked hi/lo encoding in the fp32 tensor)."""
    split = _split_boundary(boundary, w.precision)
    grid = grid or STAGE0_GRID
    _check_act(x, (3, 32, 32), torch.float32, "stage0 input")
    B = x.shape[0]
    dt = act_dtype(w.precision)
    if out is None:
        out = torch.empty((B, 4096), dtype=dt, device=x.device)
    if tuple(out.shape) != (B, 4096) or out.dtype != dt or not out.is_contiguous():
        raise ValueError("stage0: bad output buffer")
    if w.precision == "fp32":
        check(lib().cifar_stage0_x3(ptr(x), ptr(out), ptr(w.w1h), ptr(w.w1l), ptr(w.b1), ptr(w.w2h), ptr(w.w2l),
                                    ptr(w.b2), B, grid, stream_ptr(), split), "cifar_stage0_x3")
    else:
        check(lib().cifar_stage0_v4(ptr(x), ptr(out), ptr(w.w1), ptr(w.b1), ptr(w.w2), ptr(w.b2), B, grid,
                                    stream_ptr()), "cifar_stage0_v4")
    return out


def fc1_forward(h: torch.Tensor, w: CifarHeadWeights, out: Optional[torch.Tensor] = None,
                scratch: Optional[torch.Tensor] = None, boundary: str = "fp32") -> torch.Tensor:
    """Unit 2: (B,4096) -> relu(fc1) (B,512) on the MFMA GEMM (fp32: split operand,
    ``scratch`` = (>=B, 12288) bf16 for the [hi | hi | lo] rows; ``boundary``:
    the encoding of ``h``)."""
    split = _split_boundary(boundary, w.precision)
    dt = act_dtype(w.precision)
    _check_act(h, (4096,), dt, "fc1 input")
    B = h.shape[0]
    if w.precision == "bf16":
        return linear(h, w.w_fc1, w.b_fc1, act=ACT_RELU, out=out)
    if B >= FC1_X3_MIN_ROWS:
        if out is None:
            out = torch.empty((B, 512), dtype=torch.float32, device=h.device)
        check(lib().cifar_fc1_x3(ptr(h), 4096, ptr(w.w_fc1h), ptr(w.w_fc1l), 4096, ptr(w.b_fc1), ptr(out), 512,
                                 B, 512, 4096, stream_ptr(), split), "cifar_fc1_x3")
        return out
    if scratch is None or scratch.shape[0] < B or tuple(scratch.shape[1:]) != (3 * 4096,):
        scratch = torch.empty((B, 3 * 4096), dtype=torch.bfloat16, device=h.device)
    a3 = scratch[:B]
    check(lib().cifar_split3(ptr(h), 4096, ptr(a3), 3 * 4096, B, 4096, stream_ptr(), split), "cifar_split3")
    if out is None:
        out = torch.empty((B, 512), dtype=torch.float32, device=h.device)
    return linear(a3, w.w_fc1, w.b_fc1, act=ACT_RELU, out=out)


def head_tail(hid: torch.Tensor, w: CifarHeadWeights, probs: Optional[torch.Tensor] = None,
              pred: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Unit 3: (B,512) -> fc2 + softmax (B,10) fp32 + per-row argmax (B,) int32."""
    _check_act(hid, (512,), act_dtype(w.precision), "head_tail input")
    B = hid.shape[0]
    probs = probs if probs is not None else torch.empty((B, 10), dtype=torch.float32, device=hid.device)
    pred = pred if pred is not None else torch.empty((B,), dtype=torch.int32, device=hid.device)
    if w.precision == "fp32":
        check(lib().cifar_head_tail_x3(ptr(hid), ptr(w.w_fc2h), ptr(w.w_fc2l), ptr(w.b_fc2), ptr(probs), ptr(pred),
                                       B, stream_ptr()), "cifar_head_tail_x3")
    else:
        check(lib().cifar_head_tail(ptr(hid), ptr(w.w_fc2), ptr(w.b_fc2), ptr(probs), ptr(pred), B, stream_ptr()),
              "cifar_head_tail")
    return probs, pred


def head_forward(h: torch.Tensor, w: CifarHeadWeights, hid: Optional[torch.Tensor] = None,
                 probs: Optional[torch.Tensor] = None, pred: Optional[torch.Tensor] = None,
                 boundary: str = "fp32") -> Tuple[torch.Tensor, torch.Tensor]:
    """Units 2-3: h (B,4096) -> (probs (B,10) fp32, pred (B,) int32)."""
    hid = fc1_forward(h, w, out=hid, boundary=boundary)
    return head_tail(hid, w, probs, pred)
