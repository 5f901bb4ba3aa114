"""bf16 MFMA GEMM with fused epilogues (``csrc/kernels/gemm_bf16.hip``).

``linear(x, w)`` computes ``x @ w.T (+bias) -> act (+residual)`` with ``w`` in
``nn.Linear`` layout ``[out, in]``; rows of ``x`` may be strided (``x.stride(0)``),
the last dim must be contiguous and K a multiple of 64.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._lib import check, lib, ptr, stream_ptr

ACT_NONE, ACT_RELU, ACT_GELU, ACT_SILU_MUL = 0, 1, 2, 3
SKINNY_MAX_M = 256


SKINNY_ALWAYS_M = 64  # bf16: rows up to which the skinny kernels always run (gemm_bf16.hip g_skinny_max_m)


def skinny_rows(M: int, N: int, w8: bool = False) -> bool:
    """Decode-sized GEMM -> the weight-streaming skinny kernels: M <= 64 (always
    for fp8 weights: W8A16 keeps bf16 activations in decode; bf16 per
    ``set_skinny_max_m``), or medium M (<= 256, M split into 16-row tiles) while
    128^2 tiles would not fill 3/4 of the CUs (same rule as gemm_bf16.hip
    launch_gemm)."""
    always = 64 if w8 else SKINNY_ALWAYS_M
    return M <= always or (M <= SKINNY_MAX_M and -(-M // 128) * -(-N // 128) < 192)


def set_skinny_max_m(m: int = 64) -> None:
    """bf16 rows up to which every GEMM streams weights on the skinny kernels
    (default 64, the maximum); lower values are A/B probes (bench/probes/decode_ab.py)."""
    global SKINNY_ALWAYS_M
    check(lib().gemm_set_skinny_max_m(int(m)), "gemm_set_skinny_max_m")
    SKINNY_ALWAYS_M = int(m)
_ACTS = {None: ACT_NONE, "none": ACT_NONE, "relu": ACT_RELU, "gelu": ACT_GELU, "silu_mul": ACT_SILU_MUL}

DECODE_WS_BYTES = 16 << 20
_decode_ws = {}


def decode_workspace(device, slot: int = 0) -> torch.Tensor:
    """Split-K workspace of the decode stream GEMM (``csrc/kernels/gemm_stream.h``):
    fp32 partial slabs of one projection at a time.  One per (device, slot):
    GEMMs on one stream reuse it in stream order; concurrent microbatches
    (``DecodeRing`` lanes) pass their own slot.  Allocated on first use (a
    graph's warm-up run, never inside a capture)."""
    key = (str(device), slot)
    t = _decode_ws.get(key)
    if t is None:
        # zeroed: its last 4 KiB are the stream kernel's split-K tickets, which
        # every launch leaves at zero again (gemm_stream.h, in-launch combine)
        t = _decode_ws[key] = torch.zeros(DECODE_WS_BYTES, dtype=torch.uint8, device=device)
    return t


def set_stream_gemm(on: int = 1, min_bytes: int = 0, fold: int = -1) -> None:
    """Decode stream GEMM: 0 off, 1 on where it measured faster (default), 2
    forced on every eligible shape (tests); ``min_bytes`` = weight-byte
    threshold (0 keeps it); ``fold`` = split-K combine inside the launch by
    the last-arriving workgroup of a tile (1) or as a separate reduce launch
    (0, default: the fold measured 4.08 -> 4.20 ms/step on Llama-3 8B B=32,
    profiles/r3_fold_decode_ab.jsonl — one workgroup per tile serialises the
    combine that the reduce launch spreads over the chip), -1 keeps it."""
    check(lib().gemm_set_stream(int(on), int(min_bytes), int(fold)), "gemm_set_stream")


def set_oneshot_gemm(on: int = 1, mt: int = 0, ntw: int = 0, steps: int = 0, splitk: int = 0) -> None:
    """One-shot decode GEMM (``csrc/kernels/gemm_oneshot.h``, 17..64 rows,
    fragment-order weights): 0 off, 1 on the shapes its plan covers (default),
    2 every eligible shape (tests); a non-zero ``mt``/``ntw``/``steps``/``splitk``
    pins that configuration for every eligible call (A/B probes)."""
    check(lib().gemm_set_oneshot(int(on), int(mt), int(ntw), int(steps), int(splitk)), "gemm_set_oneshot")


ROWSTATS = True  # producer-side decode row statistics (A/B switch; runtime/transformer.py)


def rowstats_buffer(rows: int, width: int, device) -> torch.Tensor:
    """Row-statistics partials of ``rows`` activation rows of ``width``
    columns: one {mean, M2} float2 per 16-column tile (gemm_epilogue.h
    epi_rowstat16), as fp32 (rows, 2 ceil(width / 16))."""
    return torch.zeros((rows, 2 * -(-width // 16)), dtype=torch.float32, device=device)


class _RowStats:
    """Arms the next decode GEMM call with row-statistics buffers
    (gemm_skinny.hip ``dnn_gemm_rowstats``): ``out`` receives the partials of
    the call's output rows, ``inp`` holds those of its input rows (merged
    instead of re-deriving a folded pre-norm's statistics).  ``written`` after
    the call: whether its kernel wrote ``out``."""

    def __init__(self, out: Optional[torch.Tensor], inp: Optional[torch.Tensor], M: int):
        for t, nm in ((out, "rs_out"), (inp, "rs_in")):
            if t is not None and (t.dtype != torch.float32 or t.dim() != 2 or t.shape[0] < M or t.stride(1) != 1
                                  or t.stride(0) % 2):
                raise ValueError(f"{nm}: fp32 (>= {M}, 2P) row-statistics buffer expected")
        self.active = out is not None or inp is not None
        self.written = False
        if self.active:
            lib().gemm_rowstats(ptr(out), 0 if out is None else out.stride(0) // 2, ptr(inp),
                                0 if inp is None else inp.stride(0) // 2)

    def done(self) -> bool:
        if self.active:
            self.written = bool(lib().gemm_rowstats_written())
        return self.written


_LAST_RS = [False]


def rowstats_written() -> bool:
    """Whether the last ``rs_out=`` call's kernel wrote the row statistics."""
    return _LAST_RS[0]


def _ws_args(ws: Optional[torch.Tensor]):
    return (0, 0) if ws is None else (ws.data_ptr(), ws.numel() * ws.element_size())


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act=None,
           residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
           out_dtype: torch.dtype = torch.bfloat16, w_shuf: Optional[torch.Tensor] = None,
           rowstat: Optional[torch.Tensor] = None, colsum: Optional[torch.Tensor] = None,
           ws: Optional[torch.Tensor] = None, rs_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``w_shuf``: ``shuffle_weight(w)``, streamed instead of ``w`` on the skinny path (``skinny_rows``).
    ``rs_out`` (decode): row-statistics partials of the output (``rowstats_buffer``);
    ``rowstats_written()`` tells whether the kernel that ran wrote them.
    ``ws``: ``decode_workspace`` for the decode stream GEMM's split-K partials.
    ``rowstat`` ((M, 2) fp32 from ``transformer_ops.row_stats``) / ``colsum``: a
    folded pre-norm applied in the epilogue, ``rstd (x W^T) - mean rstd colsum``
    (MFMA tile kernels only)."""
    a = _ACTS[act] if not isinstance(act, int) else act
    x2 = x.reshape(-1, x.shape[-1]) if x.dim() != 2 else x
    M, K = x2.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"linear: x {tuple(x2.shape)} vs w {tuple(w.shape)}")
    if K % 64:
        raise ValueError(f"linear: K={K} must be a multiple of 64")
    if x2.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        raise TypeError("linear: bf16 operands required")
    if x2.stride(1) != 1 or w.stride(1) != 1:
        raise ValueError("linear: inner dims must be contiguous")
    Nout = N // 2 if a == ACT_SILU_MUL else N
    if out is None:
        out = torch.empty((M, Nout), dtype=out_dtype, device=x.device)
    o2 = out.reshape(-1, out.shape[-1]) if out.dim() != 2 else out
    if bias is not None and bias.dtype != torch.float32:
        raise TypeError("linear: bias must be fp32")
    r2 = None
    if residual is not None:
        r2 = residual.reshape(-1, residual.shape[-1]) if residual.dim() != 2 else residual
    if w_shuf is not None and w_shuf.numel() * w_shuf.element_size() != -(-N // 16) * 16 * K * 2:
        raise ValueError("linear: w_shuf is not shuffle_weight(w)")
    if rowstat is not None and (rowstat.dtype != torch.float32 or rowstat.numel() < 2 * M
                                or not rowstat.is_contiguous()):
        raise ValueError("linear: rowstat must be contiguous fp32 (M, 2)")
    if colsum is not None and (rowstat is None or colsum.dtype != torch.float32 or colsum.numel() < N):
        raise ValueError("linear: colsum needs rowstat and N fp32 entries")
    wsp, wsb = _ws_args(ws)
    rs = _RowStats(rs_out, None, M)
    try:
        check(lib().gemm_bf16(ptr(x2), x2.stride(0), ptr(w), w.stride(0), ptr(o2), o2.stride(0), ptr(bias),
                              ptr(r2), 0 if r2 is None else r2.stride(0), M, N, K, a,
                              1 if o2.dtype == torch.float32 else 0, stream_ptr(), ptr(w_shuf), ptr(rowstat),
                              ptr(colsum), wsp, wsb), "gemm_bf16")
    finally:  # a rejected call must not leave the request armed for the next GEMM
        _LAST_RS[0] = rs.done()
    return out


def set_gemm_tile(tile: int = 0) -> None:
    """Force the large-GEMM tile (128, 256, or 255 = 256x128) or restore the auto choice (0)."""
    check(lib().gemm_set_tile(int(tile)), "gemm_set_tile")


def set_gemm_split_tail(on=True) -> None:
    """A/B switch of the prefill tail split (gemm_bf16.hip tail_split_cols): a
    256^2 grid of full rounds plus one column of tiles runs that column as
    256x128 tiles in a second launch (GPT-2 O / c_proj / c_attn at M = 32768).
    ``on``: True = the default (bf16 kernel only), False = off, or an int
    bit mask (1 bf16, 2 fp8)."""
    mask = (1 if on else 0) if isinstance(on, bool) else int(on)
    check(lib().gemm_set_split_tail(mask), "gemm_set_split_tail")


def set_gemm_half_cost(c: float = 1e9) -> None:
    """Auto tile rule: the time of a 256x128 tile relative to a 256x256 tile
    (256x128 is picked when its rounds x ``c`` beat the 256^2 rounds; the
    default never picks it: measured slower, csrc/kernels/gemm_bf16.hip)."""
    check(lib().gemm_set_half_cost(float(c)), "gemm_set_half_cost")


def pack_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """Interleave gate/up rows in 8-row groups: [g0..g7, u0..u7, g8..g15, ...]
    so every 16-column MFMA tile holds 8 gate and the 8 matching up columns
    (lane groups 0-1 vs 2-3 of the transposed accumulator): the ACT_SILU_MUL
    epilogue pairs them with one cross-half lane shuffle, at any tile width."""
    F, K = gate.shape
    if F % 8:
        raise ValueError("ffn dim must be a multiple of 8")
    g = gate.reshape(F // 8, 8, K)
    u = up.reshape(F // 8, 8, K)
    return torch.stack([g, u], dim=1).reshape(2 * F, K).contiguous()


NORM_RMS, NORM_LN = 1, 2
FOLD_NORM_PREFILL = True  # prefill (non-skinny) folded norms: row statistics + GEMM epilogue (A/B switch)


class FoldedLinear:
    """A linear layer with the preceding LayerNorm/RMSNorm folded in
    (``fold_norm``): ``w`` = W diag(gamma) (bf16), ``bias`` = W beta + b
    (fp32 or None), ``colsum`` = row sums of the bf16 ``w`` (LayerNorm only)."""

    __slots__ = ("w", "bias", "colsum", "norm", "eps", "ws")

    def __init__(self, w, bias, colsum, norm, eps):
        self.w, self.bias, self.colsum, self.norm, self.eps = w, bias, colsum, norm, eps
        self.ws = None  # bf16 decode copy in skinny fragment order (shuffle_weight)


def fold_norm(w: torch.Tensor, gamma: torch.Tensor, beta: Optional[torch.Tensor], bias: Optional[torch.Tensor],
              rms: bool, eps: float, device, fp8: bool = False) -> FoldedLinear:
    """Fold ``norm(x) @ w.T + bias`` into ``rstd * (x @ w'.T - mean * colsum) + bias'``.

    norm(x) = (x - mean) * rstd * gamma + beta (LayerNorm; RMSNorm: mean = 0,
    no beta), so  norm(x) @ w.T = rstd * (x @ (w * gamma).T - mean * sum_k
    (w * gamma)[n, k]) + w @ beta.  Exact in real arithmetic; colsum is taken
    from the rounded folded weight actually used by the kernel (bf16, or the
    dequantised e4m3 weight with ``fp8=True``)."""
    w32 = w.to(device=device, dtype=torch.float32)
    wf32 = w32 * gamma.to(device=device, dtype=torch.float32)[None, :]
    if fp8:
        from .fp8 import quantize_weight
        wf = quantize_weight(wf32, device)
        wdq = wf.q[:, :wf32.shape[1]].float() * wf.scale[:, None]
    else:
        wf = wf32.to(torch.bfloat16).contiguous()
        wdq = wf.float()
    del wf32
    b = None
    if beta is not None and not rms:
        b = w32 @ beta.to(device=device, dtype=torch.float32)
    if bias is not None:
        b = bias.to(device=device, dtype=torch.float32) if b is None else b + bias.to(device=device,
                                                                                        dtype=torch.float32)
    colsum = None if rms else wdq.sum(dim=1).contiguous()
    return FoldedLinear(wf, None if b is None else b.contiguous(), colsum, NORM_RMS if rms else NORM_LN, float(eps))


def linear_norm(x: torch.Tensor, f: FoldedLinear, act=None, residual: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, std_buf: Optional[torch.Tensor] = None,
                ones: Optional[torch.Tensor] = None, q8: Optional[torch.Tensor] = None,
                s8: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
                rs_in: Optional[torch.Tensor] = None, sx: Optional[torch.Tensor] = None,
                q_out: Optional[tuple] = None) -> torch.Tensor:
    """``linear(norm(x), W, b)`` for a ``FoldedLinear``.  ``rs_in`` (decode):
    the row-statistics partials of ``x`` written by its producer (``linear(...,
    rs_out=)``), merged instead of deriving the statistics from ``x``.  Decode-sized M (<= 64):
    one skinny-GEMM launch that accumulates the row statistics from the A
    fragments it streams (bf16 weights, or e4m3 weights converted in registers).
    Larger M: the norm kernel standardises x into ``std_buf`` (gamma = ``ones``,
    no beta), then the plain GEMM with the folded weight and bias (bf16, or the
    W8A8 fp8 GEMM with the ``q8``/``s8`` activation-quantisation buffers)."""
    from .fp8 import Fp8Weight, linear_fp8, linear_w8
    from .fp8 import mx_ok as fp8_mx_ok
    a = _ACTS[act] if not isinstance(act, int) else act
    M, K = x.shape
    w8 = isinstance(f.w, Fp8Weight)
    N = f.w.shape[0]
    if (not w8 and f.w.shape[1] != K) or x.dtype != torch.bfloat16 or x.stride(1) != 1:
        raise ValueError(f"linear_norm: x {tuple(x.shape)} {x.dtype} vs w {tuple(f.w.shape)}")
    if not skinny_rows(M, N, w8):
        from .transformer_ops import layernorm, layernorm_q8
        if std_buf is None or ones is None:
            raise ValueError("linear_norm: large M needs std_buf and ones")
        if w8 and q8 is not None and sx is not None and fp8_mx_ok(M, N, f.w):
            # standardise + MX-quantise in one pass (e8m0 per 128 columns); the
            # scaled MFMA applies the scales
            from .transformer_ops import layernorm_q8_mx
            kp = f.w.q.shape[1]
            layernorm_q8_mx(x, ones, None, q8, sx, kp, f.eps, f.norm == NORM_RMS, rows=M, ldx=x.stride(0))
            return linear_fp8(x, f.w, f.bias, a, residual, out, q8, None, prequantized=True, sx=sx, q_out=q_out)
        if q_out is not None:
            raise ValueError("linear_norm: q_out needs the MX fp8 prefill path")
        if w8 and q8 is not None and s8 is not None:
            # standardise + quantise in one pass: the e4m3 rows feed the W8A8 GEMM directly
            kp = f.w.q.shape[1]
            layernorm_q8(x, ones, None, q8, s8, kp, f.eps, f.norm == NORM_RMS, rows=M, ldx=x.stride(0),
                         split=f.w.q2 is not None)
            return linear_fp8(x, f.w, f.bias, a, residual, out, q8, s8, prequantized=True)
        if w8:
            xs = layernorm(x, ones, None, std_buf[:M], f.eps, f.norm == NORM_RMS, rows=M, ldx=x.stride(0))
            return linear_fp8(xs[:M], f.w, f.bias, a, residual, out, q8, s8)
        if FOLD_NORM_PREFILL:
            # statistics only (8 B per row, carved from the front of std_buf), the
            # norm applied in the GEMM epilogue on the raw activations: no
            # normalised copy written and re-read (profiles/archive/r2_prefill_fold_norm_ab.jsonl)
            from .transformer_ops import row_stats
            st = std_buf.reshape(-1)[:4 * M].view(torch.float32).view(M, 2)
            row_stats(x, st, f.eps, f.norm == NORM_RMS, rows=M, ldx=x.stride(0))
            return linear(x, f.w, f.bias, a, residual, out, rowstat=st, colsum=f.colsum)
        xs = layernorm(x, ones, None, std_buf[:M], f.eps, f.norm == NORM_RMS, rows=M, ldx=x.stride(0))
        return linear(xs[:M], f.w, f.bias, a, residual, out)
    if w8:
        return linear_w8(x, f.w, f.bias, a, residual, out, f.norm, f.colsum, f.eps, ws=ws, rs_in=rs_in)
    if K % 32:
        raise ValueError(f"linear_norm: K={K} must be a multiple of 32")
    Nout = N // 2 if a == ACT_SILU_MUL else N
    if out is None:
        out = torch.empty((M, Nout), dtype=torch.bfloat16, device=x.device)
    if out.dtype != torch.bfloat16 or out.stride(1) != 1 or out.shape[0] < M or out.shape[1] < Nout:
        raise ValueError("linear_norm: bad output buffer")
    if residual is not None and (residual.shape[0] < M or residual.stride(1) != 1):
        raise ValueError("linear_norm: bad residual")
    if f.ws is not None and f.ws.numel() != -(-N // 16) * 16 * K * 2:
        raise ValueError("linear_norm: ws is not shuffle_weight(w)")
    wsp, wsb = _ws_args(ws)
    rs = _RowStats(None, rs_in, M)
    try:
        check(lib().gemm_skinny_norm(ptr(x), x.stride(0), ptr(f.w), f.w.stride(0), ptr(out), out.stride(0),
                                     ptr(f.bias), ptr(residual), 0 if residual is None else residual.stride(0), M, N,
                                     K, a, f.norm, ptr(f.colsum), f.eps, stream_ptr(), ptr(f.ws), wsp, wsb),
              "gemm_skinny_norm")
    finally:
        rs.done()
    return out

QKV_SCATTER = True  # prefill c_attn writes q / K / V head-major (A/B switch)


def qkv_scatter_norm(x: torch.Tensor, f: FoldedLinear, std_buf: torch.Tensor, q: torch.Tensor, kc: torch.Tensor,
                     vc: torch.Tensor, pos: torch.Tensor, B: int, T: int, H: int, Hkv: int, hd: int,
                     ones: Optional[torch.Tensor] = None, q8: Optional[torch.Tensor] = None,
                     s8: Optional[torch.Tensor] = None, sx: Optional[torch.Tensor] = None) -> bool:
    """Prefill c_attn (folded pre-norm, no RoPE) with the QKV scatter epilogue
    (gemm_bf16.hip ``dnn_gemm_bf16_qkv_scatter``): q lands in ``q`` as (B, H, T,
    hd) and K / V straight in the bf16 caches at rows ``pos[b] + t``, so the head-
    major flash prefill follows without a qkv_split or an in-kernel cache copy.
    fp8 weights (W8A8): the standardise + quantise pass (``ones`` / ``q8`` /
    ``s8`` buffers, as ``linear_norm``) feeds the fp8 256^2 kernel's scatter
    variant.  Returns False (nothing launched) where it does not apply: an fp8
    cache, decode-sized M, or a shape off the 256^2 tile path."""
    from .fp8 import Fp8Weight
    w8 = isinstance(f.w, Fp8Weight)
    if not (QKV_SCATTER and FOLD_NORM_PREFILL) or kc.dtype != torch.bfloat16:
        return False
    M, K = x.shape
    N = f.w.shape[0]
    if M != B * T or N != (H + 2 * Hkv) * hd or skinny_rows(M, N, w8) or x.stride(1) != 1:
        return False
    if not (kc.is_contiguous() and vc.is_contiguous()) or q.numel() < M * H * hd or pos.dtype != torch.int32:
        return False
    if w8 and sx is not None and q8 is not None and ones is not None and N % 32 == 0:
        from .fp8 import mx_ok
        if mx_ok(M, N, f.w):  # MX-scaled activations (e8m0 per 128 columns) on the scaled MFMA
            from .transformer_ops import layernorm_q8_mx
            kp = f.w.q.shape[1]
            layernorm_q8_mx(x, ones, None, q8, sx, kp, f.eps, f.norm == NORM_RMS, rows=M, ldx=x.stride(0))
            check(lib().gemm_fp8_qkv_scatter_mx(ptr(q8), ptr(sx), ptr(f.w.q), ptr(f.w.scale), ptr(f.bias), ptr(q),
                                                ptr(kc), ptr(vc), ptr(pos), B, T, H, Hkv, hd, kc.shape[2], kp,
                                                stream_ptr()), "gemm_fp8_qkv_scatter_mx")
            return True
    if w8:
        if ones is None or q8 is None or s8 is None or N % 32 or M < 256:
            return False
        from .transformer_ops import layernorm_q8
        kp = f.w.q.shape[1]
        split = f.w.q2 is not None  # split activations: [hi | lo] planes against [W | W/16]
        layernorm_q8(x, ones, None, q8, s8, kp, f.eps, f.norm == NORM_RMS, rows=M, ldx=x.stride(0), split=split)
        check(lib().gemm_fp8_qkv_scatter(ptr(q8), ptr(s8), ptr(f.w.q2 if split else f.w.q), ptr(f.w.scale),
                                         ptr(f.bias), ptr(q), ptr(kc), ptr(vc), ptr(pos), B, T, H, Hkv, hd,
                                         kc.shape[2], 2 * kp if split else kp, stream_ptr()),
              "gemm_fp8_qkv_scatter")
        return True
    from .transformer_ops import row_stats
    st = std_buf.reshape(-1)[:4 * M].view(torch.float32).view(M, 2)
    row_stats(x, st, f.eps, f.norm == NORM_RMS, rows=M, ldx=x.stride(0))
    rc = lib().gemm_bf16_qkv_scatter(ptr(x), x.stride(0), ptr(f.w), f.w.stride(0), ptr(f.bias), ptr(st), ptr(f.colsum),
                                     ptr(q), ptr(kc), ptr(vc), ptr(pos), B, T, H, Hkv, hd, kc.shape[2], K, stream_ptr())
    if rc == -3:  # off the 256^2 path: the caller runs the qkv-row GEMM instead (st is recomputed there)
        return False
    check(rc, "gemm_bf16_qkv_scatter")
    return True


FUSED_HEAD = True  # decode head + argmax partials in one launch (A/B switch: set_fused_head)
HEAD_PART_PER_ROW = 256  # int2 partials per row the fused head may write (one per workgroup, <= CUs)


def set_fused_head(on: bool = True) -> None:
    """A/B switch of the fused decode head (``head_argmax``)."""
    global FUSED_HEAD
    FUSED_HEAD = bool(on)
    check(lib().gemm_set_head(1 if on else 0), "gemm_set_head")


def head_argmax(x: torch.Tensor, f: FoldedLinear, logits: torch.Tensor, part: torch.Tensor, out: torch.Tensor,
                also: Optional[torch.Tensor] = None, advance: Optional[torch.Tensor] = None,
                hist: Optional[torch.Tensor] = None) -> bool:
    """Greedy decode head (gemm_head.h): ``logits = linear(norm(x), W)`` for a
    folded-norm head with a fragment-order copy (bf16 or W8A16), and the
    argmax of every row in the same pass — each workgroup writes its winner
    per row to ``part``, a merge launch (``argmax_final``) writes ``out`` and
    the decode step tail (``also`` = copy of the ids, ``hist[row, advance]``
    = the id, ``advance += 1``).
    Returns False with nothing launched where it does not apply (more than 64
    rows, a width without an instantiated config, a vocabulary over two
    column tiles per wave): the caller then runs the GEMM and argmax_rows."""
    from .fp8 import Fp8Weight
    if not FUSED_HEAD or not isinstance(f, FoldedLinear):
        return False
    M, K = x.shape
    w8 = isinstance(f.w, Fp8Weight)
    wsh = f.w.shuf if w8 else f.ws
    if wsh is None or M > 64 or x.dtype != torch.bfloat16 or x.stride(1) != 1:
        return False
    N = f.w.shape[0]
    if logits.dtype != torch.bfloat16 or logits.stride(1) != 1 or logits.shape[0] < M or logits.shape[1] < N:
        raise ValueError("head_argmax: bad logits buffer")
    if part.dtype != torch.int32 or not part.is_contiguous() or part.numel() < 2 * HEAD_PART_PER_ROW * M:
        raise ValueError(f"head_argmax: part must be contiguous int32 with >= {2 * HEAD_PART_PER_ROW * M} entries")
    for t, nm in ((out, "out"), (also, "also"), (advance, "advance")):
        if t is not None and (t.dtype != torch.int32 or t.numel() < M or not t.is_contiguous()):
            raise ValueError(f"head_argmax: {nm} must be contiguous int32 with >= {M} entries")
    from .transformer_ops import check_hist
    hist_ld = check_hist(hist, advance, M, "head_argmax")
    S = lib().gemm_head(ptr(x), x.stride(0), ptr(wsh), ptr(f.w.scale) if w8 else 0, ptr(f.colsum), ptr(f.bias),
                        f.eps, f.norm, ptr(logits), logits.stride(0), M, N, K, 1 if w8 else 0, ptr(part),
                        HEAD_PART_PER_ROW, stream_ptr())
    if S == -1:
        return False
    if S <= 0:
        raise RuntimeError(f"gemm_head failed ({S})")
    check(lib().argmax_final(ptr(part), S, M, ptr(out), ptr(also), ptr(advance), stream_ptr(), ptr(hist), hist_ld),
          "argmax_final")
    return True


def shuffle_weight(w: torch.Tensor) -> torch.Tensor:
    """Pre-shuffle a decode weight [N, K] (bf16, or e4m3 bytes) into the skinny
    GEMM's MFMA fragment order: for column tile t (16 rows) and 64-B chunk c,
    the 16 rows x 64 B form one contiguous 1 KiB block with lane l = 16 g + r
    holding row r, bytes 16 g..16 g+15 of the chunk; blocks of one tile are
    consecutive along K.  N is zero-padded to a multiple of 16.  Returns a flat
    uint8 tensor (the kernel addresses it by bytes)."""
    N = w.shape[0]
    b = w.contiguous().view(torch.uint8).reshape(N, -1)
    kb = b.shape[1]
    if kb % 64:
        raise ValueError(f"shuffle_weight: row bytes {kb} must be a multiple of 64")
    Np = -(-N // 16) * 16
    if Np != N:
        b = torch.cat([b, b.new_zeros(Np - N, kb)])
    return b.view(Np // 16, 16, kb // 64, 4, 16).permute(0, 2, 3, 1, 4).contiguous().view(-1)


def attach_shuffled(w):
    """Give a decode weight its fragment-order copy: a ``FoldedLinear`` gets
    ``.ws`` (bf16) or its ``Fp8Weight`` ``.shuf``; an ``Fp8Weight`` gets
    ``.shuf``; a bf16 tensor returns its shuffled copy (the caller keeps it and
    passes it as ``linear(..., w_shuf=)``).  The row-major weight stays for
    prefill (M > 64), so decode weights take twice their bytes in HBM."""
    from .fp8 import Fp8Weight
    if isinstance(w, FoldedLinear):
        if isinstance(w.w, Fp8Weight):
            attach_shuffled(w.w)
        else:
            w.ws = shuffle_weight(w.w)
        return w
    if isinstance(w, Fp8Weight):
        w.shuf = shuffle_weight(w.q[:, :w.k or w.q.shape[1]])
        return w
    return shuffle_weight(w)
