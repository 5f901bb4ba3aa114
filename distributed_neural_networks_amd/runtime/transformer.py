"""GPT-2 / Llama-3 pipeline stages on the gfx950 kernels, with a KV cache.

Reference semantics (``partitions/gpt_model_parts.py``): first stage =
``wte(idx) + wpe(arange(T))`` + blocks, middle = blocks, last = blocks +
``ln_f`` + ``lm_head``.  The reference recomputes the whole prefix for every
token and returns full-T fp32 logits over gRPC; here each stage keeps a bf16
KV cache ``[B][Hkv][S][hd]`` per layer (sized up front; 288 GB HBM per GPU),
prefill runs flash attention over the new tokens, decode runs split-K decode
attention, and the last stage applies ``ln_f`` + ``lm_head`` to the last
position only and samples greedily on device (``last_only=False`` gives the
reference's all-position logits).

Per layer (GPT-2): LN -> QKV GEMM(+bias) -> split(+cache write) -> attention ->
O-proj GEMM(+bias, +residual in the epilogue) -> LN -> FC GEMM(+bias, GELU in
the epilogue) -> proj GEMM(+bias, +residual).  In bf16 the LNs (ln_1, ln_2,
ln_f) are folded into the following projection (ops/gemm.py fold_norm): at
decode sizes the skinny GEMM computes the row statistics itself, so a layer
is five launches (QKV, attention, O, FC, proj).  Llama: RMSNorm, RoPE in the
split kernel, GQA, gate|up packed so SiLU(g)*u happens in the GEMM epilogue.
With ``fp8=True`` every projection uses e4m3 weights (per-channel scales): in
prefill with per-token-quantised activations on the scaled fp8 MFMA (W8A8), in
decode as weight-only fp8 (W8A16, the weight bytes halve and the fused
pre-norm stays) — GPT-2 XL config, and Llama-3 8B with ``dtype: fp8``.
All positions/lengths live in device memory so a decode step is one graph.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from ..models import model_info
from ..models.llama3 import rope_tables
from ..ops import gemm as G_
from ..ops.fp8 import mx_ok as fp8_mx_ok
from ..ops import transformer_ops as T_
from ..ops.gemm import (ACT_GELU, ACT_NONE, ACT_SILU_MUL, HEAD_PART_PER_ROW, decode_workspace, fold_norm, head_argmax,
                        linear, linear_norm,
                        pack_gate_up, qkv_scatter_norm, skinny_rows)
from .stages import StageCompute, StageOutput


def _advance3(advance):
    """``step(advance=...)``: (ids, positions) or (ids, positions, token history)."""
    if advance is None:
        return None, None, None
    if len(advance) == 2:
        return advance[0], advance[1], None
    return advance[0], advance[1], advance[2]


def _bf(t, dev):
    return t.to(device=dev, dtype=torch.bfloat16).contiguous()


def _f32(t, dev):
    return t.to(device=dev, dtype=torch.float32).contiguous()


@dataclass
class LayerW:
    ln1_w: torch.Tensor
    ln1_b: Optional[torch.Tensor]
    w_qkv: object
    b_qkv: Optional[torch.Tensor]
    w_o: object
    b_o: Optional[torch.Tensor]
    ln2_w: torch.Tensor
    ln2_b: Optional[torch.Tensor]
    w_up: object          # gpt2: c_fc; llama: packed gate|up
    b_up: Optional[torch.Tensor]
    w_down: object
    b_down: Optional[torch.Tensor]
    w_o_s: Optional[torch.Tensor] = None     # bf16 decode copies in skinny fragment order (shuffle_weight)
    w_down_s: Optional[torch.Tensor] = None


class TransformerStage(StageCompute):
    def __init__(self, model: str, sd: Dict[str, torch.Tensor], start: int, end: int, first: bool, last: bool,
                 device, max_batch: int = 8, max_seq: int = 1024, max_tokens: Optional[int] = None,
                 fp8: bool = False, temperature: float = 0.0, top_k: int = 0, seed: int = 0,
                 kv_dtype: str = "bf16", kv_scale: str = "calibrated", fp8_prefill: str = "e4m3"):
        info = model_info(model)
        # fp8 weights, prefill (W8A8) activations: "e4m3" (default) = one e4m3
        # byte per activation, per-row scale, at the fp8 MFMA rate; "split" =
        # e4m3 hi + e4m3 residual planes against [W | W/16] (ops/fp8.py
        # attach_split: bf16-equivalent MFMA work).  Against the fp32 model on
        # the UNQUANTISED weights the e4m3 weights themselves dominate: GPT-2
        # XL logits 9.6 % (split) vs 11.4 % (e4m3) from the golden, the same
        # 81 % greedy agreement, at 268 k vs 378 k prefill tok/s (bf16 weights:
        # 1.6 %, 330 k; profiles/r5_fp8_fidelity_gpt2xl_48layers.json,
        # profiles/r5b_bench_n1.json), so the byte path is the default; decode
        # is W8A16 either way
        if fp8_prefill not in ("split", "e4m3"):
            raise ValueError(f"fp8_prefill {fp8_prefill!r}: split or e4m3")
        self.fp8_prefill = fp8_prefill
        # sampling (last stage): temperature 0 = greedy argmax; otherwise
        # Gumbel-max over the top_k logits (0 = all), seeded per (row, position)
        self.temperature, self.top_k, self.seed = float(temperature), int(top_k), int(seed)
        self.model, self.family, self.cfg = model, info.family, info.cfg
        self.start, self.end, self.first, self.last = start, end, first, last
        self.device = dev = torch.device(device)
        self.fp8 = fp8
        self.fuse_norm = True  # fold pre-norms into the projections (ops/gemm.py fold_norm)
        c = self.cfg
        self.d = c.n_embd
        self.H = c.n_head
        self.Hkv = getattr(c, "n_kv_head", c.n_head)
        self.hd = c.n_embd // c.n_head
        self.V = c.vocab_size
        self.Vpad = -(-self.V // 64) * 64
        self.eps = 1e-5 if self.family == "gpt2" else c.norm_eps
        self.rms = self.family == "llama3"
        self.max_batch, self.max_seq = max_batch, max_seq
        self.max_tokens = max_tokens or max_batch * max_seq
        # activation rows: a prefill chunk uses rows [0, B*T), a decode step of
        # microbatch m rows [m*B, (m+1)*B) (they follow the KV rows), so the
        # buffers hold max(max_tokens, max_batch) rows
        self.buf_rows = max(self.max_tokens, max_batch)
        self.ones = torch.ones((self.d,), dtype=torch.float32, device=dev)
        self.layers: List[LayerW] = [self._pack_layer(sd, j) for j in range(end - start + 1)]
        if first:
            if self.family == "gpt2":
                self.wte, self.wpe = _bf(sd["wte.weight"], dev), _bf(sd["wpe.weight"], dev)
            else:
                self.wte, self.wpe = _bf(sd["embed_tokens.weight"], dev), None
        if last:
            if self.family == "gpt2":
                self.lnf_w, self.lnf_b = _f32(sd["ln_f.weight"], dev), _f32(sd["ln_f.bias"], dev)
            else:
                self.lnf_w, self.lnf_b = _f32(sd["norm.weight"], dev), None
            if self.fuse_norm:
                self.w_head = fold_norm(sd["lm_head.weight"], self.lnf_w, self.lnf_b, None, self.rms, self.eps, dev,
                                        self.fp8)
            else:
                self.w_head = self._w(sd["lm_head.weight"])
        # decode copies of every projection in the skinny GEMM's fragment order
        # (contiguous 1 KiB per wave load; DNN_SHUF_WEIGHTS=0 disables): twice
        # the weight bytes in HBM, -9..-19 % per decode projection at M = 32
        if os.environ.get("DNN_SHUF_WEIGHTS", "1") != "0":
            self._attach_decode_copies()
        if self.fp8 and self.fp8_prefill == "split":
            self._attach_split_prefill()
        # RoPE tables (Llama)
        self.cos = self.sin = None
        if self.family == "llama3":
            cos, sin = rope_tables(c, max_seq)
            self.cos, self.sin = _f32(cos, dev), _f32(sin, dev)
        # KV cache: [layer] -> (B, Hkv, S, hd)
        L = len(self.layers)
        # KV cache: bf16, or OCP e4m3 ("fp8": half the bytes every decode step
        # streams; attention.hip KV8: MHA, or GQA at head dim 128)
        if kv_dtype not in ("bf16", "fp8"):
            raise ValueError(f"kv_dtype {kv_dtype!r}: bf16 or fp8")
        if kv_dtype == "fp8" and self.Hkv != self.H and (self.hd != 128 or self.H // self.Hkv not in (2, 4)):
            raise ValueError("fp8 KV cache: MHA, or GQA with head dim 128 and 2 or 4 query heads per kv head")
        self.kv_dtype = kv_dtype
        # fp8 cache scale per layer (powers of two): "unit", or "calibrated" =
        # set from the K / V amax of the first prefill (DecodeRing.prefill runs
        # it, then calibrate_kv(), then the real prefill); see set_kv_scales
        if kv_scale not in ("unit", "calibrated"):
            raise ValueError(f"kv_scale {kv_scale!r}: unit or calibrated")
        self.kv_scale_mode = kv_scale
        self.kv_scales = [(1.0, 1.0)] * (end - start + 1)
        self.kv_calibrated = False
        kvt = torch.float8_e4m3fn if kv_dtype == "fp8" else torch.bfloat16
        self.kc = torch.zeros((L, max_batch, self.Hkv, max_seq, self.hd), dtype=kvt, device=dev)
        self.vc = torch.zeros_like(self.kc)
        self._alloc(self.buf_rows)

    # ------------------------------------------------------------------ weights
    def _attach_decode_copies(self):
        from ..ops.gemm import attach_shuffled
        for L in self.layers:
            for name in ("w_qkv", "w_up"):
                w = getattr(L, name)
                if not isinstance(w, torch.Tensor):  # FoldedLinear / Fp8Weight: the copy rides on the object
                    attach_shuffled(w)
            for name in ("w_o", "w_down"):
                w = getattr(L, name)
                if isinstance(w, torch.Tensor):
                    setattr(L, name + "_s", attach_shuffled(w))
                else:
                    attach_shuffled(w)
        if self.last and not isinstance(self.w_head, torch.Tensor):
            attach_shuffled(self.w_head)

    def _attach_split_prefill(self):
        """[W | W/16] prefill copies of every block projection (split activations)."""
        from ..ops.fp8 import Fp8Weight, attach_split
        for L in self.layers:
            for w in (L.w_qkv, L.w_o, L.w_up, L.w_down):
                w = getattr(w, "w", w)  # FoldedLinear -> its Fp8Weight
                if isinstance(w, Fp8Weight):
                    attach_split(w)

    # ------------------------------------------------------------------ fp8 KV scale
    @property
    def needs_kv_calibration(self) -> bool:
        return self.kv_dtype == "fp8" and self.kv_scale_mode == "calibrated" and not self.kv_calibrated

    KV_TARGET = 224.0  # calibrated |K|, |V| max maps to <= 224 (half the e4m3 range: headroom for later tokens)
    E4M3_MAX = 448.0
    KV_CAL_ROUNDS = 2  # calibration prefills per stage lifetime: the same count on every rank (ring hops match)
    KV_SAT_JUMP = 512.0  # a saturated first round retries at 512x the scale (|K| up to ~229 k measured exactly)

    def calibrate_kv(self) -> List[tuple]:
        """Per-tensor fp8 K / V scales from what the cache holds now (after a
        prefill at the current scales): s = 2^ceil(log2(amax / KV_TARGET)) per
        layer, so the values use the e4m3 normal range instead of its
        subnormals.  The KV store clamps to +-448 before converting, so a
        cache amax of 448 means the true amax is unknown (larger): that layer
        retries at ``KV_SAT_JUMP`` x its scale in the next round instead of
        trusting the clamped value.  Always ``KV_CAL_ROUNDS`` rounds (a fixed
        count, so every rank of a ring runs the same prefills); a layer still
        saturated after the last one keeps its largest scale and is reported in
        ``kv_saturated_layers``.  Clears the cache: the caller re-runs the
        prefill at the new scales."""
        scales = []
        self._kv_round = getattr(self, "_kv_round", 0) + 1
        sat = []
        for li in range(len(self.layers)):
            sk0, sv0 = self.kv_scales[li]
            new = []
            for t, s0 in ((self.kc[li], sk0), (self.vc[li], sv0)):
                a = _e4m3_amax(t)
                if a >= self.E4M3_MAX:  # clamped: the real amax is above what the cache can show
                    new.append(s0 * self.KV_SAT_JUMP)
                    sat.append(li)
                else:
                    new.append(2.0 ** math.ceil(math.log2(max(a * s0, 1e-30) / self.KV_TARGET)))
            scales.append(tuple(new))
        last = self._kv_round >= self.KV_CAL_ROUNDS
        if last and sat:  # still clamping after the retry: keep the previous (largest measured-safe) scales
            import warnings
            warnings.warn(f"fp8 KV calibration: layers {sorted(set(sat))} still saturate e4m3 after "
                          f"{self._kv_round} rounds; their K/V clamp at +-448 x scale")
            scales = [self.kv_scales[li] if li in sat else sc for li, sc in enumerate(scales)]
        self.kv_saturated_layers = sorted(set(sat)) if last else []
        self.set_kv_scales(scales)
        self.kv_calibrated = last
        self.reset()
        return scales

    def set_kv_scales(self, scales: List[tuple]) -> None:
        """Store layer li's K as K / s_k and V as V / s_v in the fp8 cache, with
        no kernel change: the scales fold into the weights.  The q rows of
        the QKV projection are multiplied by s_k and the k rows divided by it
        (q.k unchanged; RoPE is linear); the v rows are divided by s_v and the
        output projection multiplied by s_v (P.V is linear).  Powers of two
        keep every bf16 weight exact; e4m3 weights only change their channel
        scales.  Relative to the scales already applied."""
        from ..ops.fp8 import Fp8Weight
        from ..ops.gemm import FoldedLinear, attach_shuffled
        qn, kn = self.H * self.hd, self.Hkv * self.hd
        for li, (L, (sk, sv)) in enumerate(zip(self.layers, scales)):
            ok, ov = self.kv_scales[li]
            rk, rv = sk / ok, sv / ov
            if rk == 1.0 and rv == 1.0:
                continue
            r = torch.ones(qn + 2 * kn, dtype=torch.float32, device=self.device)
            r[:qn], r[qn:qn + kn], r[qn + kn:] = rk, 1.0 / rk, 1.0 / rv
            w = L.w_qkv
            if isinstance(w, FoldedLinear):
                if w.bias is not None:
                    w.bias.mul_(r)
                if w.colsum is not None:
                    w.colsum.mul_(r)
                w = w.w
            elif L.b_qkv is not None:
                L.b_qkv.mul_(r)
            if isinstance(w, Fp8Weight):
                w.scale.mul_(r)
            else:
                w.mul_(r.to(w.dtype)[:, None])
                if isinstance(L.w_qkv, FoldedLinear) and L.w_qkv.ws is not None:
                    attach_shuffled(L.w_qkv)
            if isinstance(L.w_o, Fp8Weight):
                L.w_o.scale.mul_(rv)
            else:
                L.w_o.mul_(rv)
                if L.w_o_s is not None:
                    L.w_o_s = attach_shuffled(L.w_o)
            self.kv_scales[li] = (sk, sv)

    def _w(self, w):
        if self.fp8:
            from ..ops.fp8 import quantize_weight
            return quantize_weight(w, self.device)
        return _bf(w, self.device)

    def _pack_layer(self, sd, j) -> LayerW:
        dev = self.device
        if self.family == "gpt2":
            p = f"h.{j}."
            ln1_w, ln1_b = _f32(sd[p + "ln_1.weight"], dev), _f32(sd[p + "ln_1.bias"], dev)
            ln2_w, ln2_b = _f32(sd[p + "ln_2.weight"], dev), _f32(sd[p + "ln_2.bias"], dev)
            w_qkv, b_qkv = sd[p + "attn.c_attn.weight"], sd[p + "attn.c_attn.bias"]
            w_up, b_up = sd[p + "mlp.c_fc.weight"], sd[p + "mlp.c_fc.bias"]
            if self.fuse_norm:
                qkv_f = fold_norm(w_qkv, ln1_w, ln1_b, b_qkv, False, self.eps, dev, self.fp8)
                up_f = fold_norm(w_up, ln2_w, ln2_b, b_up, False, self.eps, dev, self.fp8)
                return LayerW(None, None, qkv_f, None,
                              self._w(sd[p + "attn.c_proj.weight"]), _f32(sd[p + "attn.c_proj.bias"], dev),
                              None, None, up_f, None,
                              self._w(sd[p + "mlp.c_proj.weight"]), _f32(sd[p + "mlp.c_proj.bias"], dev))
            return LayerW(ln1_w, ln1_b, self._w(w_qkv), _f32(b_qkv, dev),
                          self._w(sd[p + "attn.c_proj.weight"]), _f32(sd[p + "attn.c_proj.bias"], dev),
                          ln2_w, ln2_b, self._w(w_up), _f32(b_up, dev),
                          self._w(sd[p + "mlp.c_proj.weight"]), _f32(sd[p + "mlp.c_proj.bias"], dev))
        p = f"layers.{j}."
        qkv = torch.cat([sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.k_proj.weight"],
                         sd[p + "self_attn.v_proj.weight"]], dim=0)
        gu = pack_gate_up(sd[p + "mlp.gate_proj.weight"].float(), sd[p + "mlp.up_proj.weight"].float())
        ln1_w = _f32(sd[p + "input_layernorm.weight"], dev)
        ln2_w = _f32(sd[p + "post_attention_layernorm.weight"], dev)
        if self.fuse_norm:
            return LayerW(None, None, fold_norm(qkv, ln1_w, None, None, True, self.eps, dev, self.fp8), None,
                          self._w(sd[p + "self_attn.o_proj.weight"]), None, None, None,
                          fold_norm(gu, ln2_w, None, None, True, self.eps, dev, self.fp8), None,
                          self._w(sd[p + "mlp.down_proj.weight"]), None)
        return LayerW(ln1_w, None, self._w(qkv), None, self._w(sd[p + "self_attn.o_proj.weight"]), None,
                      ln2_w, None, self._w(gu), None, self._w(sd[p + "mlp.down_proj.weight"]), None)

    def _alloc(self, ntok: int):
        dev, c = self.device, self.cfg
        d, H, Hkv, hd = self.d, self.H, self.Hkv, self.hd
        ffn = 4 * d if self.family == "gpt2" else c.ffn_dim
        bf = torch.bfloat16
        self.buf_h = torch.empty((ntok, d), dtype=bf, device=dev)
        self.buf_a = torch.empty((ntok, d), dtype=bf, device=dev)
        self.buf_qkv = torch.empty((ntok, (H + 2 * Hkv) * hd), dtype=bf, device=dev)
        self.buf_q = torch.empty((ntok * H * hd,), dtype=bf, device=dev)
        self.buf_att = torch.empty((ntok, H * hd), dtype=bf, device=dev)
        self.buf_f = torch.empty((ntok, ffn), dtype=bf, device=dev)
        self.lens = torch.zeros((self.max_batch,), dtype=torch.int32, device=dev)
        self.splits = T_.decode_splits(self.max_seq, self.max_batch, Hkv, H // Hkv)
        G = H // Hkv
        self.ws_per_seq = Hkv * self.splits * G * (hd + 2)  # decode-attention partials of one sequence
        self.ws = torch.empty((self.max_batch * self.ws_per_seq,), dtype=torch.float32, device=dev)
        # row-split argmax partials (last stage; rows offset by the microbatch like the logits)
        self.amx_part = torch.empty((self.max_batch * 2 * T_.ARGMAX_PART_PER_ROW,),
                                    dtype=torch.int32, device=dev)
        # fused decode head's per-workgroup argmax partials (ops/gemm.py head_argmax)
        self.head_part = (torch.empty((self.max_batch * 2 * HEAD_PART_PER_ROW,), dtype=torch.int32, device=dev)
                          if self.last else None)
        self.rowstat = G_.rowstats_buffer(self.max_batch, d, dev)  # decode rows only
        self.q8 = self.s8 = None
        self.sx8 = self.q8b = self.sx8b = None
        if self.fp8:
            from ..ops.fp8 import kpad_of, mx_scale_bytes
            kmax = max(kpad_of(d), kpad_of(ffn)) * (2 if self.fp8_prefill == "split" else 1)
            self.q8 = torch.empty((ntok * kmax,), dtype=torch.uint8, device=dev)
            self.s8 = torch.empty((ntok,), dtype=torch.float32, device=dev)
            if self.fp8_prefill == "e4m3":
                # MX prefill (ops/fp8.py linear_fp8 sx=): the e8m0 scales of the
                # projection inputs, and the c_fc output quantised by its own
                # epilogue for c_proj (bytes + scales)
                self.sx8 = torch.empty((mx_scale_bytes(ntok, kmax),), dtype=torch.uint8, device=dev)
                self.q8b = torch.empty((ntok * kpad_of(ffn),), dtype=torch.uint8, device=dev)
                self.sx8b = torch.empty((mx_scale_bytes(ntok, kpad_of(ffn)),), dtype=torch.uint8, device=dev)
        if self.last:
            self.buf_lnf = torch.empty((ntok, d), dtype=bf, device=dev)
            self.logits = torch.empty((ntok, self.Vpad), dtype=bf, device=dev)
            self.next_ids = torch.empty((ntok,), dtype=torch.int32, device=dev)

    def _lin(self, x, w, b, act=ACT_NONE, residual=None, out=None, ncols=None, w_shuf=None, ws=None, rs_out=None,
             mx_in=None):
        """``rs_out``: decode row-statistics partials of the output (see ``step``);
        ``mx_in`` (fp8 prefill): (bytes, scales) of x already MX-quantised by its
        producer.  Returns (out, whether the row statistics were written)."""
        from ..ops.gemm import rowstats_written
        if self.fp8:
            from ..ops.fp8 import linear_fp8, linear_w8
            if skinny_rows(x.shape[0], w.q.shape[0], w8=True):  # decode: weight-only fp8 (bf16 activations)
                y = linear_w8(x, w, b, act, residual, out, ws=ws, rs_out=rs_out)
                return y, rs_out is not None and rowstats_written()
            if mx_in is not None:
                return linear_fp8(x, w, b, act, residual, out, mx_in[0], None, prequantized=True, sx=mx_in[1]), False
            return linear_fp8(x, w, b, act, residual, out, self.q8, self.s8, sx=self.sx8), False
        y = linear(x, w, b, act, residual, out, w_shuf=w_shuf, ws=ws, rs_out=rs_out)
        return y, rs_out is not None and rowstats_written()

    # ------------------------------------------------------------------ specs
    act_dtype = torch.bfloat16  # stage-boundary hidden states

    def in_spec(self, batch: int, T: int = 1):
        if self.first:
            return (batch, T), torch.int32
        return (batch * T, self.d), torch.bfloat16

    def out_spec(self, batch: int, T: int = 1):
        if self.last:
            return (batch,), torch.int32
        return (batch * T, self.d), torch.bfloat16

    # ------------------------------------------------------------------ forward
    @property
    def fuses_step_tail(self) -> bool:
        """Greedy last stage: ``step(advance=...)`` folds the decode step's tail
        (input-id copy, position update) into the argmax launch."""
        return self.last and not self.temperature > 0

    def step(self, x: torch.Tensor, pos: torch.Tensor, B: int, T: int, b0: int = 0, out: Optional[torch.Tensor] = None,
             last_only: bool = True, advance=None):
        """Run this stage for B sequences x T new tokens at cache rows
        [b0, b0+B) and positions ``pos`` (device int32 (B,), tokens already
        cached).  Returns hidden (B*T, d) bf16, or StageOutput for the last stage.
        ``advance`` = (ids or None, positions[, token history]): greedy last stage only
        (``fuses_step_tail``): the sampled ids are also written to ``ids`` and
        ``positions += 1``, in the argmax launch."""
        if advance is not None and not (self.fuses_step_tail and last_only):
            raise ValueError("step(advance=...) needs a greedy last stage with last_only")
        ntok = B * T
        if ntok > self.buf_h.shape[0]:
            raise ValueError(f"stage buffers hold {self.buf_h.shape[0]} tokens, got {ntok}")
        if b0 + B > self.max_batch:
            raise ValueError("batch slice exceeds the KV cache")
        d = self.d
        # decode scratch rows follow the KV rows (r0 = b0): microbatches on
        # different cache rows share no buffer, so their steps may run
        # concurrently on separate streams (DecodeRing lanes); prefill (T > 1)
        # uses the rows from 0 and stays one-at-a-time
        r0 = b0 if T == 1 else 0
        r1 = r0 + ntok
        if r1 > self.buf_h.shape[0]:
            raise ValueError(f"stage buffers hold {self.buf_h.shape[0]} rows, step needs rows [{r0}, {r1})")
        if self.first:
            if x.dtype != torch.int32 or tuple(x.shape) != (B, T):
                raise ValueError(f"first stage expects int32 ids (B,T)=({B},{T}), got {x.dtype} {tuple(x.shape)}")
            T_.embed(x, self.wte, self.wpe, self.buf_h[r0:r1], pos)
            h_in = self.buf_h[r0:r1]
        else:
            h_in = x.reshape(ntok, d)
        h = self.buf_h[r0:r1]
        a = self.buf_a[r0:r1]
        q8, s8 = self.q8, self.s8
        if self.fp8 and T == 1:
            q8 = self.q8[r0 * (self.q8.numel() // self.buf_rows):]
            s8 = self.s8[r0:]
        ws = self.ws[r0 * self.ws_per_seq:] if T == 1 else self.ws
        # decode stream-GEMM split-K workspace: one per concurrent microbatch slot
        gws = decode_workspace(self.device, b0 // B) if T == 1 else None
        # decode row statistics produced by the residual-writing projections
        # (O, c_proj: per-16-column {mean, M2} partials of h) and merged by the
        # next folded pre-norm projection (c_fc, the next layer's QKV) instead
        # of every column-tile workgroup re-deriving them
        rs = self.rowstat[r0:r1] if (T == 1 and self.fuse_norm and G_.ROWSTATS) else None
        have_rs = False
        for li, L in enumerate(self.layers):
            kc, vc = self.kc[li, b0:b0 + B], self.vc[li, b0:b0 + B]
            att = self.buf_att[r0:r1]
            scattered = (T > 1 and self.cos is None and self.fuse_norm and
                         qkv_scatter_norm(h_in, L.w_qkv, a, self.buf_q, kc, vc, pos, B, T, self.H, self.Hkv,
                                          self.hd, ones=self.ones, q8=q8, s8=s8, sx=self.sx8 if T > 1 else None))
            if scattered:
                pass  # prefill (no RoPE): c_attn wrote q head-major and K / V straight into the caches
            elif self.fuse_norm:
                qkv = linear_norm(h_in, L.w_qkv, out=self.buf_qkv[r0:r1], std_buf=a, ones=self.ones, q8=q8,
                                  s8=s8, ws=gws, rs_in=rs if have_rs else None)
            else:
                T_.layernorm(h_in, L.ln1_w, L.ln1_b, a, self.eps, self.rms, rows=ntok)
                qkv, _ = self._lin(a, L.w_qkv, L.b_qkv, out=self.buf_qkv[r0:r1])
            if scattered:
                T_.flash_attn(self.buf_q, kc, vc, att, B, T, self.H, self.Hkv, self.hd, pos)
            elif T == 1:  # decode: split/RoPE/cache write fused into the attention launch
                T_.attn_decode_qkv(qkv, kc, vc, att, B, self.H, self.Hkv, self.hd, pos, ws, self.splits,
                                   self.cos, self.sin)
            elif self.cos is None:  # no RoPE (GPT-2): attention reads the c_attn output directly
                T_.flash_attn_qkv(qkv, kc, vc, att, B, T, self.H, self.Hkv, self.hd, pos)
            else:
                T_.qkv_split(qkv, self.buf_q, kc, vc, B, T, self.H, self.Hkv, self.hd, pos, self.cos, self.sin)
                T_.flash_attn(self.buf_q, kc, vc, att, B, T, self.H, self.Hkv, self.hd, pos)
            _, have_rs = self._lin(att, L.w_o, L.b_o, residual=h_in, out=h, w_shuf=L.w_o_s, ws=gws, rs_out=rs)
            up_act = ACT_GELU if self.family == "gpt2" else ACT_SILU_MUL
            mx_f = None
            if self.fuse_norm:
                # fp8 MX prefill: the GELU c_fc quantises its own output for c_proj
                if (self.q8b is not None and T > 1 and up_act == ACT_GELU
                        and fp8_mx_ok(ntok, L.w_up.w.shape[0], L.w_up.w)):
                    mx_f = (self.q8b, self.sx8b)
                f = linear_norm(h, L.w_up, act=up_act, out=self.buf_f[r0:r1], std_buf=a, ones=self.ones, q8=q8,
                                s8=s8, ws=gws, rs_in=rs if have_rs else None,
                                sx=self.sx8 if T > 1 else None, q_out=mx_f)
                if mx_f is not None:
                    f = self.buf_f[r0:r1]  # shape only: c_proj reads the e4m3 bytes in mx_f
            else:
                T_.layernorm(h, L.ln2_w, L.ln2_b, a, self.eps, self.rms, rows=ntok)
                f, _ = self._lin(a, L.w_up, L.b_up, act=up_act, out=self.buf_f[r0:r1])
            _, have_rs = self._lin(f, L.w_down, L.b_down, residual=h, out=h, w_shuf=L.w_down_s, ws=gws, rs_out=rs,
                                   mx_in=mx_f)
            h_in = h
        if not self.last:
            if out is not None:
                out.view(ntok, d).copy_(h)
                return out
            return h
        if last_only:
            rows, src, ldx = B, h[T - 1:], T * d
        else:
            rows, src, ldx = ntok, h, d
        logits = self.logits[r0:r0 + rows]
        if self.fuse_norm and last_only and not self.temperature > 0:
            # greedy: the head writes the logits and each workgroup's argmax
            # partials; one merge launch takes the ids and the step tail
            x_last = torch.as_strided(src, (rows, d), (ldx, 1))
            dst = out if out is not None else self.next_ids[r0:r0 + rows]
            also, adv, hist = _advance3(advance)
            if head_argmax(x_last, self.w_head, logits[:, :self.V], self.head_part[r0 * 2 * HEAD_PART_PER_ROW:], dst,
                           also, adv, hist):
                return StageOutput(logits[:, :self.V], dst)
        if self.fuse_norm:
            x_last = torch.as_strided(src, (rows, d), (ldx, 1))
            linear_norm(x_last, self.w_head, out=logits[:, :self.V], std_buf=self.buf_lnf[r0:], ones=self.ones,
                        q8=q8, s8=s8, ws=gws)
        else:
            lnf = self.buf_lnf[r0:r0 + rows]
            T_.layernorm(src, self.lnf_w, self.lnf_b, lnf, self.eps, self.rms, rows=rows, ldx=ldx)
            if self.fp8:
                self._head_fp8(lnf, logits)
            else:
                linear(lnf, self.w_head, None, out=logits[:, :self.V])
        nxt = self.next_ids[r0:r0 + rows]
        if self.temperature > 0 and last_only:
            T_.sample_topk(logits, nxt, self.V, self.temperature, self.top_k, self.seed, step=pos)
            if out is not None:
                out.copy_(nxt)
            return StageOutput(logits[:, :self.V], nxt)
        dst = out if (last_only and out is not None) else nxt
        also, adv, hist = _advance3(advance)
        part = self.amx_part[r0 * 2 * T_.ARGMAX_PART_PER_ROW:] if last_only else None
        T_.argmax_rows(logits, dst, n=self.V, also=also, advance=adv, part=part, hist=hist)
        return StageOutput(logits[:, :self.V], dst)

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None):
        """Full-prefix forward of one request (the reference stage call,
        ``partitions/gpt_model_parts.py:13-22,31-34,44-50``; gRPC data path).

        x = token ids (B, T) on the first stage, else hidden states (B, T, d).
        Returns hidden states (B, T, d) bf16, or on the last stage a
        ``StageOutput`` with the all-position logits (B, T, V) as the reference
        returns them and the greedy next token of every sequence.  Each call is
        an independent request: it runs as a prefill at positions 0..T-1 in KV
        rows [0, B) (the reference keeps no cache and recomputes the prefix)."""
        if self.first:
            B, T = x.shape
            h = x.to(device=self.device, dtype=torch.int32).contiguous()
        else:
            B, T = x.shape[0], x.shape[1]
            h = x.to(device=self.device, dtype=torch.bfloat16).reshape(B * T, self.d).contiguous()
        if B > self.max_batch or T > self.max_seq:
            raise ValueError(f"request (B={B}, T={T}) exceeds the stage KV cache "
                             f"(max_batch={self.max_batch}, max_seq={self.max_seq})")
        pos = torch.zeros((B,), dtype=torch.int32, device=self.device)
        y = self.step(h, pos, B, T, last_only=not self.last)
        if not self.last:
            return y.view(B, T, self.d)
        logits = y.probs.reshape(B, T, self.V)
        return StageOutput(logits, y.pred.view(B, T)[:, -1].contiguous())

    def _head_fp8(self, lnf, logits):
        from ..ops.fp8 import linear_fp8
        linear_fp8(lnf, self.w_head, None, 0, None, logits[:, :self.V], self.q8, self.s8)

    def reset(self):
        self.kc.zero_()
        self.vc.zero_()


def _e4m3_amax(t: torch.Tensor) -> float:
    """max |x| of an e4m3fn tensor without widening it: with the sign bit
    cleared the bytes order like the magnitudes (0x7f, NaN, never stored)."""
    b = torch.bitwise_and(t.view(torch.uint8), 0x7F).amax()
    return float(b.view(1).view(torch.float8_e4m3fn).float().item())


def build_device_stage(model: str, sd, start: int, end: int, first: bool, last: bool, device, dtype=None,
                       max_batch: int = 8, max_seq: int = 1024, max_tokens: Optional[int] = None,
                       temperature: float = 0.0, top_k: int = 0, seed: int = 0, kv_dtype: str = "bf16",
                       kv_scale: str = "calibrated", fp8_prefill: str = "e4m3"):
    fp8 = dtype in ("fp8", "float8_e4m3fn", "fp8_e4m3")
    info = model_info(model)
    max_seq = min(max_seq, getattr(info.cfg, "block_size", getattr(info.cfg, "max_seq", max_seq)))
    return TransformerStage(model, sd, start, end, first, last, device, max_batch, max_seq, max_tokens, fp8,
                            temperature, top_k, seed, kv_dtype=kv_dtype, kv_scale=kv_scale, fp8_prefill=fp8_prefill)


# ---------------------------------------------------------------------- smoke / golden check
def smoke(dev) -> None:
    """GPT-2-tiny and Llama-tiny, 2 stages each on the decode ring, vs the fp32
    torch golden: prefill logits within 2e-2 relative, the first generated
    token exact, and the greedy continuation equal to the golden's until the
    golden's top-2 logits come within bf16 resolution of each other."""
    from .. import checkpoint as ckpt
    from ..models import build_golden_stage
    from .scheduler import DecodeRing, RingLinks
    for model in ("gpt2-tiny", "llama3-tiny"):
        n = model_info(model).num_layers
        ranges = [(0, n // 2 - 1), (n // 2, n - 1)]
        sds = [ckpt.random_stage_state_dict(model, a, b, i == 0, i == 1, 7, nontrivial=True)
               for i, (a, b) in enumerate(ranges)]
        stages = [TransformerStage(model, sds[i], a, b, i == 0, i == 1, dev, max_batch=2, max_seq=64)
                  for i, (a, b) in enumerate(ranges)]
        golden = []
        for i, (a, b) in enumerate(ranges):
            g = build_golden_stage(model, a, b, i == 0, i == 1)
            g.load_state_dict(sds[i])
            golden.append(g.eval())
        g = torch.Generator().manual_seed(3)
        prompt = torch.randint(0, model_info(model).cfg.vocab_size, (2, 16), generator=g)
        # prefill logits of the device stages (all positions) vs golden
        h = prompt
        for st in stages:
            h = st.forward(h)
        with torch.no_grad():
            ref_logits = prompt
            for gs in golden:
                ref_logits = gs(ref_logits)
        dev_logits = h.probs.float().cpu()
        rel = ((dev_logits - ref_logits).norm() / ref_logits.norm()).item()
        if rel > 2e-2:
            raise AssertionError(f"smoke {model}: prefill logits rel err {rel:.3e}")
        ring = DecodeRing(stages, RingLinks(), 1, 1, 2)
        toks = ring.generate([prompt], 16, 4)
        torch.cuda.synchronize(dev)
        seq = prompt.clone()
        with torch.no_grad():
            for t in range(4):
                hh = seq
                for gs in golden:
                    hh = gs(hh)
                last = hh[:, -1]
                top2 = last.topk(2, dim=-1).values
                nid = last.argmax(-1)
                for b in range(2):
                    if int(toks[b, t]) != int(nid[b]):
                        tie = (top2[b, 0] - top2[b, 1]).item() <= 2e-2 * top2[b, 0].abs().item()
                        if t == 0 or not tie:
                            raise AssertionError(f"smoke {model}: token {t} of row {b}: {toks[b].tolist()} vs "
                                                 f"golden {int(nid[b])}")
                seq = torch.cat([seq, toks[:, t:t + 1].long()], 1)  # follow the device's sequence
