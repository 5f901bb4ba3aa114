"""CIFAR-10 ConvNet on the fused gfx950 kernels (``csrc/kernels/cifar_fused.hip``).

Weight packing happens once at load (reference ``node.py:305-306`` only moves
fp32 modules to the device):

* conv1 ``(32,3,3,3)`` -> ``w1p [32][32]`` bf16, im2col column ``k = c*9+ky*3+kx``
  (27 real, 5 zero) = the MFMA B-operand rows;
* conv2 ``(64,32,3,3)`` -> ``w2p [64][288]`` bf16 with ``k = (ky*3+kx)*32 + c``
  to match the HWC activation image in LDS;
* fc1 stays ``[512][4096]`` bf16 (already K-contiguous for the GEMM);
* fc2 ``(10,512)`` -> ``[16][512]`` bf16 zero-padded to one MFMA N-tile.
Biases are fp32.  The stage-boundary tensor is ``(B,4096)`` bf16 in the
reference's NCHW flatten order, so the split matches ``cifar_model_parts.py:41``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

from ._lib import check, lib, ptr, stream_ptr
from .gemm import ACT_RELU, linear


@dataclass
class CifarStage0Weights:
    w1p: torch.Tensor      # v1: [32][32], k = c*9+ky*3+kx
    b1: torch.Tensor
    w2p: torch.Tensor
    b2: torch.Tensor
    w1p2: torch.Tensor = None  # v2: [32][48], k = ky*16 + kx*4 + c (kx<3, c<3 real)


STAGE0_VARIANT = 4  # v4: single-barrier pipeline (csrc/kernels/cifar_fused.hip); 1-3 kept for A/B


@dataclass
class CifarHeadWeights:
    w_fc1: torch.Tensor
    b_fc1: torch.Tensor
    w_fc2p: torch.Tensor
    b_fc2: torch.Tensor


def pack_stage0(sd: Dict[str, torch.Tensor], device) -> CifarStage0Weights:
    w1 = sd["conv1.weight"].float().reshape(32, 27)
    w1p = torch.zeros(32, 32)
    w1p[:, :27] = w1
    w2 = sd["conv2.weight"].float().permute(0, 2, 3, 1).reshape(64, 288)  # (oc, ky, kx, c)
    w1p2 = torch.zeros(32, 3, 4, 4)  # (oc, ky, kx, c) zero-padded kx=3, c=3
    w1p2[:, :, :3, :3] = sd["conv1.weight"].float().permute(0, 2, 3, 1)
    return CifarStage0Weights(
        w1p=w1p.to(device=device, dtype=torch.bfloat16).contiguous(),
        b1=sd["conv1.bias"].float().to(device).contiguous(),
        w2p=w2.to(device=device, dtype=torch.bfloat16).contiguous(),
        b2=sd["conv2.bias"].float().to(device).contiguous(),
        w1p2=w1p2.reshape(32, 48).to(device=device, dtype=torch.bfloat16).contiguous())


def pack_head(sd: Dict[str, torch.Tensor], device, fc1: bool = True, fc2: bool = True) -> CifarHeadWeights:
    w_fc1 = b_fc1 = w2p = b_fc2 = None
    if fc1:
        w_fc1 = sd["fc1.weight"].to(device=device, dtype=torch.bfloat16).contiguous()
        b_fc1 = sd["fc1.bias"].float().to(device).contiguous()
    if fc2:
        w2 = torch.zeros(16, 512)
        w2[:10] = sd["fc2.weight"].float()
        w2p = w2.to(device=device, dtype=torch.bfloat16).contiguous()
        b_fc2 = sd["fc2.bias"].float().to(device).contiguous()
    return CifarHeadWeights(w_fc1=w_fc1, b_fc1=b_fc1, w_fc2p=w2p, b_fc2=b_fc2)


def fc1_forward(h: torch.Tensor, w: CifarHeadWeights, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Unit 2: (B,4096) bf16 -> relu(fc1) (B,512) bf16 on the MFMA GEMM."""
    if h.dtype != torch.bfloat16 or tuple(h.shape[1:]) != (4096,):
        raise ValueError(f"fc1: expected bf16 (B,4096), got {h.dtype} {tuple(h.shape)}")
    return linear(h, w.w_fc1, w.b_fc1, act=ACT_RELU, out=out)


def head_tail(hid: torch.Tensor, w: CifarHeadWeights, probs: Optional[torch.Tensor] = None,
              pred: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Unit 3: (B,512) bf16 -> fc2 + softmax (B,10) fp32 + per-row argmax (B,) int32."""
    if hid.dtype != torch.bfloat16 or tuple(hid.shape[1:]) != (512,) or not hid.is_contiguous():
        raise ValueError(f"head_tail: expected contiguous bf16 (B,512), got {hid.dtype} {tuple(hid.shape)}")
    B = hid.shape[0]
    probs = probs if probs is not None else torch.empty((B, 10), dtype=torch.float32, device=hid.device)
    pred = pred if pred is not None else torch.empty((B,), dtype=torch.int32, device=hid.device)
    check(lib().cifar_head_tail(ptr(hid), ptr(w.w_fc2p), ptr(w.b_fc2), ptr(probs), ptr(pred), B, stream_ptr()),
          "cifar_head_tail")
    return probs, pred


STAGE0_GRID = 0  # persistent stage-0 workgroups; 0 = one per CU (256)


def set_stage0_grid(grid: int = 0) -> None:
    """Persistent stage-0 grid size (0 = one workgroup per CU).  With fewer
    workgroups than CUs the spare CUs stay free for concurrent kernels — the
    RCCL all-to-all of the multi-GPU placements cannot start a workgroup on a
    CU the stage-0 kernel holds (its 2 waves/SIMD fill every VGPR)."""
    global STAGE0_GRID
    STAGE0_GRID = int(grid)


def stage0_forward(x: torch.Tensor, w: CifarStage0Weights, out: Optional[torch.Tensor] = None,
                   grid: int = 0, variant: Optional[int] = None) -> torch.Tensor:
    """x: (B,3,32,32) fp32 contiguous -> (B,4096) bf16."""
    grid = grid or STAGE0_GRID
    if x.dtype != torch.float32 or not x.is_contiguous() or tuple(x.shape[1:]) != (3, 32, 32):
        raise ValueError(f"stage0: expected contiguous fp32 (B,3,32,32), got {x.dtype} {tuple(x.shape)}")
    B = x.shape[0]
    if out is None:
        out = torch.empty((B, 4096), dtype=torch.bfloat16, device=x.device)
    if tuple(out.shape) != (B, 4096) or out.dtype != torch.bfloat16 or not out.is_contiguous():
        raise ValueError("stage0: bad output buffer")
    v = variant or STAGE0_VARIANT
    if v == 4:
        check(lib().cifar_stage0_v4(ptr(x), ptr(out), ptr(w.w1p2), ptr(w.b1), ptr(w.w2p), ptr(w.b2), B, grid,
                                    stream_ptr()), "cifar_stage0_v4")
    elif v == 3:
        check(lib().cifar_stage0_v3(ptr(x), ptr(out), ptr(w.w1p2), ptr(w.b1), ptr(w.w2p), ptr(w.b2), B, grid,
                                    stream_ptr()), "cifar_stage0_v3")
    elif v == 2:
        check(lib().cifar_stage0_v2(ptr(x), ptr(out), ptr(w.w1p2), ptr(w.b1), ptr(w.w2p), ptr(w.b2), B, grid,
                                    stream_ptr()), "cifar_stage0_v2")
    else:
        check(lib().cifar_stage0(ptr(x), ptr(out), ptr(w.w1p), ptr(w.b1), ptr(w.w2p), ptr(w.b2), B, grid,
                                 stream_ptr()), "cifar_stage0")
    return out


def head_forward(h: torch.Tensor, w: CifarHeadWeights, hid: Optional[torch.Tensor] = None,
                 probs: Optional[torch.Tensor] = None, pred: Optional[torch.Tensor] = None
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
    """h: (B,4096) bf16 -> (probs (B,10) fp32, pred (B,) int32)."""
    if h.dtype != torch.bfloat16 or tuple(h.shape[1:]) != (4096,) or not h.is_contiguous():
        raise ValueError(f"head: expected contiguous bf16 (B,4096), got {h.dtype} {tuple(h.shape)}")
    B = h.shape[0]
    dev = h.device
    hid = hid if hid is not None else torch.empty((B, 512), dtype=torch.bfloat16, device=dev)
    probs = probs if probs is not None else torch.empty((B, 10), dtype=torch.float32, device=dev)
    pred = pred if pred is not None else torch.empty((B,), dtype=torch.int32, device=dev)
    linear(h, w.w_fc1, w.b_fc1, act=ACT_RELU, out=hid)
    check(lib().cifar_head_tail(ptr(hid), ptr(w.w_fc2p), ptr(w.b_fc2), ptr(probs), ptr(pred), B, stream_ptr()),
          "cifar_head_tail")
    return probs, pred
