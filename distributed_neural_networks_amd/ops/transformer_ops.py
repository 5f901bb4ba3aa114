"""Thin wrappers over the transformer kernels (norms, embedding, attention,
sampler, fp8).  Shapes are validated on the host before launch — a kernel is
only ever launched with the operand shapes its grid assumes."""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from ._lib import check, lib, ptr, stream_ptr


def _bf16_2d(x: torch.Tensor, name: str) -> None:
    if x.dtype != torch.bfloat16 or x.stride(-1) != 1:
        raise ValueError(f"{name}: expected bf16 with contiguous last dim, got {x.dtype} strides {x.stride()}")


def layernorm(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], out: torch.Tensor, eps: float = 1e-5,
              rms: bool = False, rows: Optional[int] = None, ldx: Optional[int] = None) -> torch.Tensor:
    """Row-wise LayerNorm (rms=False, with bias) or RMSNorm over the last dim.
    ``rows``/``ldx`` allow normalising a strided subset of rows (e.g. the last
    position of every sequence: ldx = T*d, x pointing at row T-1)."""
    _bf16_2d(x, "layernorm")
    N = x.shape[-1]
    M = rows if rows is not None else x.numel() // N
    ldx = ldx if ldx is not None else N
    if w.dtype != torch.float32 or (b is not None and b.dtype != torch.float32):
        raise TypeError("layernorm: fp32 weight/bias expected")
    if N % 8 or N > 8192:
        raise ValueError(f"layernorm: unsupported width {N}")
    if out.numel() < M * N:
        raise ValueError("layernorm: output too small")
    check(lib().layernorm(ptr(x), ldx, ptr(w), ptr(b), ptr(out), N, M, N, eps, 1 if rms else 0, stream_ptr()),
          "layernorm")
    return out


def row_stats(x: torch.Tensor, stats: torch.Tensor, eps: float = 1e-5, rms: bool = False, rows: Optional[int] = None,
              ldx: Optional[int] = None) -> torch.Tensor:
    """Per-row {rstd, -mean * rstd} (fp32 (M, 2); RMSNorm: {rstd, 0}) of a bf16
    (M, N) activation: the statistics a folded-norm GEMM applies in its epilogue."""
    _bf16_2d(x, "row_stats")
    N = x.shape[-1]
    M = rows if rows is not None else x.numel() // N
    ldx = ldx if ldx is not None else N
    if stats.dtype != torch.float32 or stats.numel() < 2 * M or not stats.is_contiguous():
        raise ValueError("row_stats: stats must be contiguous fp32 with 2 * M entries")
    if N % 8 or N > 8192:
        raise ValueError(f"row_stats: unsupported width {N}")
    check(lib().row_stats(ptr(x), ldx, ptr(stats), M, N, eps, 1 if rms else 0, stream_ptr()), "row_stats")
    return stats


def layernorm_q8(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], q_out: torch.Tensor,
                 s_out: torch.Tensor, kpad: int, eps: float = 1e-5, rms: bool = False, rows: Optional[int] = None,
                 ldx: Optional[int] = None, split: bool = False) -> torch.Tensor:
    """Normalise rows and quantise them to e4m3 with per-row scales in one pass
    (the ``quant_rows`` layout: q_out (M, kpad) bytes, K padding zeroed; s_out (M,);
    ``split``: (M, 2 kpad), the residual plane after the hi bytes, ``fp8.attach_split``)."""
    _bf16_2d(x, "layernorm_q8")
    N = x.shape[-1]
    M = rows if rows is not None else x.numel() // N
    ldx = ldx if ldx is not None else N
    if w.dtype != torch.float32 or (b is not None and b.dtype != torch.float32):
        raise TypeError("layernorm_q8: fp32 weight/bias expected")
    if N % 8 or N > 8192 or kpad < N or kpad % 8:
        raise ValueError(f"layernorm_q8: unsupported width {N} / kpad {kpad}")
    ldq = kpad * (2 if split else 1)
    if q_out.numel() * q_out.element_size() < M * ldq or s_out.numel() < M:
        raise ValueError("layernorm_q8: output too small")
    check(lib().layernorm_q8(ptr(x), ldx, ptr(w), ptr(b), ptr(q_out), ldq, ptr(s_out), M, N, kpad, eps,
                             1 if rms else 0, stream_ptr(), int(split)), "layernorm_q8")
    return q_out


def layernorm_q8_mx(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], q_out: torch.Tensor,
                    sx_out: torch.Tensor, kpad: int, eps: float = 1e-5, rms: bool = False,
                    rows: Optional[int] = None, ldx: Optional[int] = None) -> torch.Tensor:
    """``layernorm_q8`` with MX scales: one e8m0 byte per (row, 128 columns)
    in ``sx_out`` (``fp8.mx_scale_bytes``; csrc/kernels/common.h mx_index)
    instead of a per-row fp32 scale — the input layout of ``fp8.linear_fp8(...,
    sx=)``."""
    from .fp8 import mx_scale_bytes
    _bf16_2d(x, "layernorm_q8_mx")
    N = x.shape[-1]
    M = rows if rows is not None else x.numel() // N
    ldx = ldx if ldx is not None else N
    if w.dtype != torch.float32 or (b is not None and b.dtype != torch.float32):
        raise TypeError("layernorm_q8_mx: fp32 weight/bias expected")
    if N % 8 or N > 8192 or kpad < N or kpad % 128:
        raise ValueError(f"layernorm_q8_mx: unsupported width {N} / kpad {kpad}")
    if q_out.numel() * q_out.element_size() < M * kpad or sx_out.numel() * sx_out.element_size() < mx_scale_bytes(M, kpad):
        raise ValueError("layernorm_q8_mx: output too small")
    check(lib().layernorm_q8_mx(ptr(x), ldx, ptr(w), ptr(b), ptr(q_out), kpad, ptr(sx_out), M, N, kpad, eps,
                                1 if rms else 0, stream_ptr()), "layernorm_q8_mx")
    return q_out


def embed(idx: torch.Tensor, wte: torch.Tensor, wpe: Optional[torch.Tensor], out: torch.Tensor,
          pos: Optional[torch.Tensor]) -> torch.Tensor:
    """out[b*T+t] = wte[idx[b,t]] (+ wpe[pos[b]+t]). idx int32 (B,T)."""
    if idx.dtype != torch.int32 or idx.dim() != 2:
        raise ValueError("embed: idx must be int32 (B,T)")
    B, T = idx.shape
    d = wte.shape[1]
    if out.numel() < B * T * d:
        raise ValueError("embed: output too small")
    check(lib().embed_gpt2(ptr(idx), ptr(wte), ptr(wpe), ptr(out), B, T, d, ptr(pos), wte.shape[0],
                           0 if wpe is None else wpe.shape[0], stream_ptr()), "embed")
    return out


KV8_DTYPES = (torch.float8_e4m3fn, torch.uint8)  # e4m3 KV cache storage (unit scale)


def _kv8(kc: torch.Tensor, vc: torch.Tensor) -> int:
    """1 for an OCP e4m3 KV cache (decode attention / QKV-mode prefill read and
    write it as bytes, attention.hip KV8), 0 for bf16."""
    k8, v8 = kc.dtype in KV8_DTYPES, vc.dtype in KV8_DTYPES
    if k8 != v8:
        raise TypeError("K and V caches must share a dtype")
    if not k8 and kc.dtype != torch.bfloat16:
        raise TypeError(f"KV cache dtype {kc.dtype}: bf16 or float8_e4m3fn")
    return 1 if k8 else 0


def qkv_split(qkv: torch.Tensor, q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, B: int, T: int, H: int,
              Hkv: int, hd: int, pos: torch.Tensor, cos: Optional[torch.Tensor] = None,
              sin: Optional[torch.Tensor] = None) -> None:
    S = kc.shape[2]
    if kc.shape[:2] != (B, Hkv) or kc.shape[3] != hd or vc.shape != kc.shape:
        raise ValueError(f"qkv_split: cache {tuple(kc.shape)} does not match B={B} Hkv={Hkv} hd={hd}")
    if qkv.numel() < B * T * (H + 2 * Hkv) * hd or q.numel() < B * T * H * hd:
        raise ValueError("qkv_split: buffers too small")
    rope = cos is not None
    check(lib().qkv_split(ptr(qkv), ptr(q), ptr(kc), ptr(vc), B, T, H, Hkv, hd, S, ptr(pos), ptr(cos), ptr(sin),
                          1 if rope else 0, stream_ptr(), kv8=_kv8(kc, vc)), "qkv_split")


def flash_attn(q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, out: torch.Tensor, B: int, T: int, H: int,
               Hkv: int, hd: int, pos: torch.Tensor, scale: Optional[float] = None) -> torch.Tensor:
    """Causal attention of T new queries per sequence against the cache
    (positions 0..pos[b]+T-1). q (B,H,T,hd); out (B*T, H*hd)."""
    if hd not in (64, 128):
        raise ValueError(f"flash_attn: head_dim {hd} unsupported (64/128)")
    S = kc.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(hd)
    check(lib().flash_attn(ptr(q), ptr(kc), ptr(vc), ptr(out), B, T, H, Hkv, hd, S, ptr(pos), scale, stream_ptr(),
                           kv8=_kv8(kc, vc)), "flash_attn")
    return out


def flash_attn_qkv(qkv: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, out: torch.Tensor, B: int, T: int, H: int,
                   Hkv: int, hd: int, pos: torch.Tensor, scale: Optional[float] = None) -> torch.Tensor:
    """Causal prefill straight from the c_attn output (no RoPE): qkv (B*T, ld)
    rows [q | k | v]; the new keys/values are written into the cache rows
    pos[b].. as a side effect (what qkv_split would have done)."""
    if hd not in (64, 128):
        raise ValueError(f"flash_attn_qkv: head_dim {hd} unsupported (64/128)")
    S = kc.shape[2]
    if kc.shape[:2] != (B, Hkv) or kc.shape[3] != hd or vc.shape != kc.shape:
        raise ValueError(f"flash_attn_qkv: cache {tuple(kc.shape)} does not match B={B} Hkv={Hkv} hd={hd}")
    if qkv.dim() != 2 or qkv.shape[0] < B * T or qkv.shape[1] < (H + 2 * Hkv) * hd or qkv.stride(1) != 1:
        raise ValueError(f"flash_attn_qkv: qkv {tuple(qkv.shape)} too small")
    if not (kc.is_contiguous() and vc.is_contiguous()):
        raise ValueError("flash_attn_qkv: cache slices must be contiguous")
    scale = scale if scale is not None else 1.0 / math.sqrt(hd)
    check(lib().flash_attn_qkv(ptr(qkv), qkv.stride(0), ptr(kc), ptr(vc), ptr(out), B, T, H, Hkv, hd, S, ptr(pos),
                               scale, stream_ptr(), kv8=_kv8(kc, vc)), "flash_attn_qkv")
    return out


DEC_LDS_SCORES = 160 * 1024 // 4  # fp32 scores one decode-attention workgroup can hold in LDS


def decode_splits(S: int, B: int, Hkv: int, G: int = 1) -> int:
    """Split-K factor for decode attention: one split once B*Hkv alone gives 2
    workgroups per CU; else enough workgroups for ~4 per CU (1024), at most one
    split per 256 keys of cache capacity.  Each split takes
    ``ceil(len/splits)`` of the *runtime* length, so short contexts stay
    balanced; with one split the kernel writes the output itself (no combine).
    Long contexts: a split keeps its G x chunk scores in LDS (160 KiB), so the
    split count never drops below ceil(S / floor(40960 / G)) (14 for a 128 K-token
    Llama-3 cache, G = 4), whatever the batch."""
    lds_min = max(1, -(-S // (DEC_LDS_SCORES // max(1, G))))  # ceil(S/splits) * G <= 40960
    if os.environ.get("DNN_DECODE_SPLITS"):  # A/B override
        return max(lds_min, int(os.environ["DNN_DECODE_SPLITS"]))
    if B * Hkv >= 512:  # >= 2 workgroups per CU already: the combine pass costs more than it hides
        return lds_min    # (GPT-2 B=64: 0.754 -> 0.703 ms/step, profiles/archive/r1_decode_benches_v6.jsonl)
    want = max(1, -(-1024 // max(1, B * Hkv)))
    return max(lds_min, min(want, -(-S // 256)))  # >= 256 keys per split: short contexts skip the combine


def attn_decode(q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, out: torch.Tensor, B: int, H: int, Hkv: int,
                hd: int, lens: torch.Tensor, ws: torch.Tensor, splits: int, scale: Optional[float] = None):
    S = kc.shape[2]
    G = H // Hkv
    need = B * Hkv * splits * G * (hd + 2)
    if ws.numel() < need or ws.dtype != torch.float32:
        raise ValueError(f"attn_decode: workspace needs {need} fp32")
    scale = scale if scale is not None else 1.0 / math.sqrt(hd)
    check(lib().attn_decode(ptr(q), ptr(kc), ptr(vc), ptr(out), B, H, Hkv, hd, S, ptr(lens), scale, splits, ptr(ws),
                            stream_ptr(), kv8=_kv8(kc, vc)), "attn_decode")
    return out


def attn_decode_qkv(qkv: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, out: torch.Tensor, B: int, H: int,
                    Hkv: int, hd: int, pos: torch.Tensor, ws: torch.Tensor, splits: int,
                    cos: Optional[torch.Tensor] = None, sin: Optional[torch.Tensor] = None,
                    scale: Optional[float] = None) -> torch.Tensor:
    """One decode step straight from the QKV projection rows (B, (H+2Hkv)*hd):
    RoPE (when cos/sin), the new k/v written into the cache at ``pos[b]`` and
    attention over ``pos[b]+1`` keys, in one launch (no qkv_split)."""
    S = kc.shape[2]
    if kc.shape[:2] != (B, Hkv) or kc.shape[3] != hd or vc.shape != kc.shape:
        raise ValueError(f"attn_decode_qkv: cache {tuple(kc.shape)} does not match B={B} Hkv={Hkv} hd={hd}")
    if qkv.dim() != 2 or qkv.shape[0] < B or qkv.shape[1] < (H + 2 * Hkv) * hd or qkv.stride(1) != 1:
        raise ValueError(f"attn_decode_qkv: qkv {tuple(qkv.shape)} too small")
    if out.numel() < B * H * hd or pos.numel() < B or pos.dtype != torch.int32:
        raise ValueError("attn_decode_qkv: bad out/pos")
    if cos is not None and (cos.shape[0] < S or cos.shape[1] != hd // 2):
        raise ValueError("attn_decode_qkv: RoPE table does not cover the cache")
    G = H // Hkv
    need = B * Hkv * splits * G * (hd + 2)
    if ws.numel() < need or ws.dtype != torch.float32:
        raise ValueError(f"attn_decode_qkv: workspace needs {need} fp32")
    scale = scale if scale is not None else 1.0 / math.sqrt(hd)
    check(lib().attn_decode_qkv(ptr(qkv), qkv.stride(0), ptr(kc), ptr(vc), ptr(out), B, H, Hkv, hd, S, ptr(pos),
                                ptr(cos), ptr(sin), scale, splits, ptr(ws), stream_ptr(), kv8=_kv8(kc, vc)),
          "attn_decode_qkv")
    return out


ARGMAX_PART_PER_ROW = 64  # int2 partials per row of the row-split argmax workspace
ARGMAX_SPLIT = True  # use the workspace when one is given (A/B switch, bench/probes/decode_ab.py)


def check_hist(hist: Optional[torch.Tensor], advance: Optional[torch.Tensor], M: int, who: str) -> int:
    """Token-history buffer of the decode step tail: (>= M, L) int32, rows
    contiguous; needs ``advance`` (the positions it is indexed by).  Returns L."""
    if hist is None:
        return 0
    if advance is None:
        raise ValueError(f"{who}: hist needs advance (the positions)")
    if hist.dtype != torch.int32 or hist.dim() != 2 or hist.shape[0] < M or hist.stride(1) != 1:
        raise ValueError(f"{who}: hist must be int32 (>= {M}, L) with contiguous rows")
    return hist.stride(0)


def argmax_rows(x: torch.Tensor, out: torch.Tensor, n: Optional[int] = None, also: Optional[torch.Tensor] = None,
                advance: Optional[torch.Tensor] = None, part: Optional[torch.Tensor] = None,
                hist: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-row argmax (ties -> smallest index) into ``out`` (int32).  Decode
    step tail in the same launch: ``also`` receives a copy of the ids,
    ``hist[row, advance[row]]`` the id (token history of a multi-step decode
    graph) and ``advance[row] += 1`` (int32 positions).  ``part`` (int32, >=
    128 M entries): workspace that lets small batches split each row over
    many workgroups (a partial and a merge launch, sampler.hip)."""
    M = x.shape[0]
    N = n if n is not None else x.shape[1]
    for t, nm in ((out, "out"), (also, "also"), (advance, "advance")):
        if t is not None and (t.dtype != torch.int32 or t.numel() < M or not t.is_contiguous()):
            raise ValueError(f"argmax_rows: {nm} must be contiguous int32 with >= {M} entries")
    hist_ld = check_hist(hist, advance, M, "argmax_rows")
    if part is not None and (part.dtype != torch.int32 or part.numel() < 2 * ARGMAX_PART_PER_ROW * M
                             or not part.is_contiguous()):
        raise ValueError(f"argmax_rows: part must be contiguous int32 with >= {2 * ARGMAX_PART_PER_ROW * M} entries")
    check(lib().argmax_rows(ptr(x), x.stride(0), M, N, ptr(out), 1 if x.dtype == torch.float32 else 0,
                            stream_ptr(), ptr(also), ptr(advance), ptr(part if ARGMAX_SPLIT else None), ptr(hist),
                            hist_ld), "argmax_rows")
    return out


def sample_topk(logits: torch.Tensor, out: torch.Tensor, n: int, temperature: float, top_k: int = 0, seed: int = 0,
                step: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Temperature / top-k sampling per row (Gumbel-max over the k largest
    logits), bf16 logits only.  ``step`` (device int32 per row, e.g. the
    sequence position) decorrelates successive decode steps inside one graph."""
    if logits.dtype != torch.bfloat16:
        raise TypeError("sample_topk: bf16 logits expected")
    if not temperature > 0:
        raise ValueError("sample_topk: temperature must be > 0 (use argmax_rows for greedy)")
    M = logits.shape[0]
    check(lib().sample_topk(ptr(logits), logits.stride(0), M, n, ptr(out), float(temperature), int(top_k),
                            int(seed) & 0xFFFFFFFF, ptr(step), stream_ptr()), "sample_topk")
    return out
