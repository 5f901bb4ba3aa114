"""FP8 (OCP e4m3fn) weight quantisation and the scaled-MFMA GEMM.

Weights: per-output-channel absmax scale, quantised once at load on the host
(``torch.float8_e4m3fn`` is OCP e4m3 — the gfx950 format, not MI300's fnuz).
Activations: per-token absmax scale, quantised on device by
``quant_fp8_rows`` right before each GEMM (fused into the GEMM's producer is a
later optimisation).  ``linear_fp8`` = ``quant -> gemm_fp8`` with the bf16
epilogue (bias / act / residual) of the bf16 GEMM.

Decode-sized M (<= 64) is weight-bandwidth bound, so there the activations
stay bf16 (``linear_w8``: W8A16): the skinny kernel converts the streamed
e4m3 weights to bf16 in registers (exact) and applies the channel scales in
its epilogue — half the bytes of bf16 weights, no activation-quantise launch,
and the fused pre-norm of the bf16 path (ops/gemm.py ``linear_norm``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ._lib import check, lib, ptr, stream_ptr

FP8_MAX = 448.0


@dataclass
class Fp8Weight:
    q: torch.Tensor      # (N, Kpad) float8_e4m3fn, K zero-padded to a multiple of 128
    scale: torch.Tensor  # (N,) fp32
    k: int = 0           # logical K
    shuf: Optional[torch.Tensor] = None  # decode copy in skinny fragment order (gemm.shuffle_weight), or None
    q2: Optional[torch.Tensor] = None    # (N, 2 Kpad) [q | q / 16]: prefill with split activations (attach_split)

    @property
    def shape(self):
        return self.q.shape


def kpad_of(k: int) -> int:
    return -(-k // 128) * 128


def quantize_weight(w: torch.Tensor, device) -> Fp8Weight:
    wf = w.to(device).float()  # quantise where the weight will live (fast on the GPU)
    N, K = wf.shape
    amax = wf.abs().amax(dim=1).clamp_min(1e-12)
    s = amax / FP8_MAX
    q = torch.zeros((N, kpad_of(K)), dtype=torch.float8_e4m3fn, device=wf.device)
    q[:, :K] = (wf / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return Fp8Weight(q.contiguous(), s.to(dtype=torch.float32).contiguous(), K)


def attach_split(w: Fp8Weight) -> Fp8Weight:
    """Prefill weights for split activations: ``q2 = [q | q / 16]`` along K
    (e4m3; q / 16 is exact down to e4m3's subnormals).  The W8A8 prefill then
    feeds ``[hi | lo]`` activation planes (``quant_rows(split=True)``,
    ``layernorm_q8(split=True)``: hi = e4m3(y), lo = e4m3((y - hi) * 16)) and
    one fp8 GEMM over 2 Kpad sums hi.W + lo.W/16 — the activation keeps ~8
    mantissa bits instead of e4m3's 4 (GPT-2 XL logits 5.7 % -> ~0.1 % from
    the fp32 golden).  Twice the prefill weight bytes and MFMA work of plain
    W8A8, i.e. the bf16 prefill's MFMA time with half its weight bytes."""
    if w.q2 is None:
        w.q2 = torch.cat([w.q, (w.q.float() / 16.0).to(torch.float8_e4m3fn)], dim=1).contiguous()
    return w


def quant_rows(x: torch.Tensor, q_out: torch.Tensor, s_out: torch.Tensor, rows: Optional[int] = None,
               split: bool = False):
    """Per-row e4m3 quantisation; q_out rows are zero-padded to kpad_of(K)
    (``split``: rows of 2 kpad bytes, the residual plane after the hi bytes)."""
    M = rows if rows is not None else x.shape[0]
    K = x.shape[-1]
    kp = kpad_of(K)
    if q_out.dtype not in (torch.uint8, torch.float8_e4m3fn) or q_out.numel() < M * kp * (2 if split else 1):
        raise ValueError("quant_rows: bad output buffer")
    check(lib().quant_fp8_rows(ptr(x), x.stride(0), ptr(q_out), ptr(s_out), M, K, kp, stream_ptr(), int(split)),
          "quant_fp8_rows")


MX_PREFILL = True  # e4m3 prefill activations with MX e8m0 block scales (A/B switch)


def mx_mpad(M: int) -> int:
    return -(-M // 64) * 64


def mx_scale_bytes(M: int, kpad: int) -> int:
    """Bytes of the MX scales of M rows x kpad columns: one e8m0 per (row, 128
    columns), rows padded to 64 (csrc/kernels/common.h mx_index)."""
    return mx_mpad(M) * (kpad // 128)


def mx_ok(M: int, N: int, w: Fp8Weight) -> bool:
    """The MX W8A8 path applies: the 256^2 fp8 kernel's shapes, one e4m3 byte
    per activation (no split planes)."""
    return MX_PREFILL and M >= 256 and N >= 256 and w.q2 is None


def quant_rows_mx(x: torch.Tensor, q_out: torch.Tensor, sx_out: torch.Tensor, rows: Optional[int] = None) -> None:
    """MX e4m3 quantisation: q_out (M, kpad) bytes, one e8m0 scale per (row,
    128 columns) in sx_out (``mx_scale_bytes``); K padding zeroed."""
    M = rows if rows is not None else x.shape[0]
    K = x.shape[-1]
    kp = kpad_of(K)
    if q_out.numel() * q_out.element_size() < M * kp or sx_out.numel() * sx_out.element_size() < mx_scale_bytes(M, kp):
        raise ValueError("quant_rows_mx: bad output buffer")
    check(lib().quant_fp8_mx(ptr(x), x.stride(0), ptr(q_out), kp, ptr(sx_out), M, K, kp, stream_ptr()),
          "quant_fp8_mx")


def linear_fp8(x: torch.Tensor, w: Fp8Weight, bias: Optional[torch.Tensor] = None, act: int = 0,
               residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
               qbuf: Optional[torch.Tensor] = None, sbuf: Optional[torch.Tensor] = None,
               prequantized: bool = False, sx: Optional[torch.Tensor] = None,
               q_out: Optional[tuple] = None) -> torch.Tensor:
    """W8A8 GEMM.  ``prequantized``: ``qbuf``/``sbuf`` already hold the e4m3
    rows and scales of x (``transformer_ops.layernorm_q8``); x only gives M, K.
    Prefill rows with ``w.q2`` (``attach_split``) run on split activations
    (2 Kpad bytes per row; a prequantized buffer must be split too).

    ``sx`` (a byte buffer of ``mx_scale_bytes``): where ``mx_ok``, the
    activations carry MX e8m0 scales per (row, 128 columns) applied by the
    scaled MFMA (``quant_rows_mx`` / ``layernorm_q8_mx`` write them; with
    ``prequantized`` they are already in ``qbuf`` / ``sx``).  ``q_out`` =
    (bytes, scales) with act GELU: the epilogue quantises its output for the
    next GEMM (MX) and ``out`` is not written — the c_fc of the MX prefill."""
    x2 = x.reshape(-1, x.shape[-1])
    M, K = x2.shape
    N, kp = w.q.shape
    if kp != kpad_of(K) or (w.k and w.k != K):
        raise ValueError(f"linear_fp8: x K={K} vs weight K={w.k} (padded {kp})")
    if sx is not None and mx_ok(M, N, w):
        if not prequantized:
            if qbuf is None or qbuf.numel() * qbuf.element_size() < M * kp:
                raise ValueError("linear_fp8: MX needs a qbuf of M x kpad bytes")
            quant_rows_mx(x2, qbuf, sx, M)
        qo, sxo, kpo = (None, None, 0)
        if q_out is not None:
            qo, sxo = q_out
            kpo = kpad_of(N)
            if act != 2 or qo.numel() * qo.element_size() < M * kpo or \
                    sxo.numel() * sxo.element_size() < mx_scale_bytes(M, kpo):
                raise ValueError("linear_fp8: q_out needs act GELU and M x kpad(N) bytes + scales")
        elif out is None:
            out = torch.empty((M, N // 2 if act == 3 else N), dtype=torch.bfloat16, device=x.device)
        o2 = out.reshape(-1, out.shape[-1]) if out is not None else None
        r2 = residual.reshape(-1, residual.shape[-1]) if residual is not None else None
        check(lib().gemm_fp8_mx(ptr(qbuf), ptr(sx), ptr(w.q), ptr(w.scale), ptr(o2),
                                0 if o2 is None else o2.stride(0), ptr(bias), ptr(r2),
                                0 if r2 is None else r2.stride(0), M, N, kp, act, ptr(qo), kpo, ptr(sxo), kpo,
                                stream_ptr()), "gemm_fp8_mx")
        return out
    if q_out is not None or (prequantized and sx is not None):
        raise ValueError("linear_fp8: q_out / MX-prequantized input off the MX path (mx_ok)")
    split = w.q2 is not None and M > 64
    kq = 2 * kp if split else kp
    if prequantized:
        if qbuf is None or sbuf is None:
            raise ValueError("linear_fp8: prequantized needs qbuf and sbuf")
        if qbuf.numel() * qbuf.element_size() < M * kq:
            raise ValueError("linear_fp8: prequantized buffer too small for the activation layout")
    else:
        qbuf = qbuf if qbuf is not None else torch.empty((M, kq), dtype=torch.uint8, device=x.device)
        sbuf = sbuf if sbuf is not None else torch.empty((M,), dtype=torch.float32, device=x.device)
        quant_rows(x2, qbuf, sbuf, M, split=split)
    if out is None:
        out = torch.empty((M, N // 2 if act == 3 else N), dtype=torch.bfloat16, device=x.device)
    o2 = out.reshape(-1, out.shape[-1])
    r2 = residual.reshape(-1, residual.shape[-1]) if residual is not None else None
    if M <= 64:  # decode: fp8 weight streaming (half the bytes of bf16)
        check(lib().gemm_skinny(ptr(qbuf), kp, ptr(sbuf), ptr(w.q), kp, ptr(w.scale), ptr(o2), o2.stride(0),
                                ptr(bias), ptr(r2), 0 if r2 is None else r2.stride(0), M, N, kp, act, 0, 1,
                                stream_ptr()), "gemm_skinny_fp8")
        return out
    check(lib().gemm_fp8(ptr(qbuf), ptr(sbuf), ptr(w.q2 if split else w.q), ptr(w.scale), ptr(o2), o2.stride(0),
                         ptr(bias), ptr(r2), 0 if r2 is None else r2.stride(0), M, N, kq, act, stream_ptr()), "gemm_fp8")
    return out


def set_fp8_tile(tile: int = 0) -> None:
    """Force the fp8 GEMM tile (128 or 256) or restore the auto choice (0)."""
    check(lib().gemm_fp8_set_tile(int(tile)), "gemm_fp8_set_tile")


def linear_w8(x: torch.Tensor, w: Fp8Weight, bias: Optional[torch.Tensor] = None, act: int = 0,
              residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, norm: int = 0,
              colsum: Optional[torch.Tensor] = None, eps: float = 0.0,
              ws: Optional[torch.Tensor] = None, rs_out: Optional[torch.Tensor] = None,
              rs_in: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Weight-only fp8 GEMM for decode-sized M (<= 256): bf16 x (M, K) times e4m3 w, bf16 out.
    ``norm`` (1 RMS / 2 LN, with ``colsum`` for LN) fuses a folded pre-norm.
    ``ws``: ``gemm.decode_workspace`` (split-K partials of the decode stream GEMM).
    ``rs_out`` / ``rs_in``: producer-side row statistics (``gemm.linear``,
    ``gemm.linear_norm``)."""
    M, K = x.shape
    N, kp = w.q.shape
    if M > 256 or (w.k and w.k != K) or kp < K or K % 64:
        raise ValueError(f"linear_w8: x {tuple(x.shape)} vs weight {tuple(w.q.shape)} (k={w.k})")
    if x.dtype != torch.bfloat16 or x.stride(1) != 1:
        raise TypeError("linear_w8: bf16 activations with a contiguous last dim")
    Nout = N // 2 if act == 3 else N
    if out is None:
        out = torch.empty((M, Nout), dtype=torch.bfloat16, device=x.device)
    if out.dtype != torch.bfloat16 or out.stride(1) != 1 or out.shape[0] < M or out.shape[1] < Nout:
        raise ValueError("linear_w8: bad output buffer")
    if w.shuf is not None and w.shuf.numel() != -(-N // 16) * 16 * K:
        raise ValueError("linear_w8: shuf is not shuffle_weight(w.q[:, :K])")
    wsp, wsb = (0, 0) if ws is None else (ws.data_ptr(), ws.numel() * ws.element_size())
    from .gemm import _LAST_RS, _RowStats
    rs = _RowStats(rs_out, rs_in, M)
    try:
        check(lib().gemm_skinny_w8(ptr(x), x.stride(0), ptr(w.q), kp, ptr(w.scale), ptr(out), out.stride(0),
                                   ptr(bias), ptr(residual), 0 if residual is None else residual.stride(0), M, N, K,
                                   act, norm, ptr(colsum), eps, stream_ptr(), ptr(w.shuf), wsp, wsb), "gemm_skinny_w8")
    finally:  # a rejected call must not leave the request armed for the next GEMM
        _LAST_RS[0] = rs.done()
    return out
