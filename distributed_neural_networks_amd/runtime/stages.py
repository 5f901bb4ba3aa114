"""Stage compute objects: one pipeline stage's forward over preallocated buffers.

``StageCompute`` is what a pipeline rank runs per microbatch.  Two families:

* ``CifarHipStage`` — the MI355X path: fused gfx950 kernels over weights
  packed once at load (``ops/cifar.py``; fp32 by default, the reference's
  precision, or bf16); no torch op runs in ``forward``.
* ``TorchStage`` — the golden torch module on CPU (fp32): the data path of the
  reference's CPU/gRPC configuration (``BASELINE.json`` configs[0]) and the
  oracle in tests.  It is never used on a GPU device.

The GPT-2 / Llama stages live in ``runtime/transformer.py`` (same interface).
Reference: the stage forward is ``my_model_part(input_torch)`` in
``node.py:52-53``; the result argmax is ``node.py:61`` (there over the flattened
batch; here per row).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

from ..models import cifar, model_info

Spec = Tuple[Tuple[int, ...], torch.dtype]


@dataclass
class StageOutput:
    """Last-stage result: probabilities/logits and per-row predictions."""
    probs: torch.Tensor
    pred: torch.Tensor


class StageCompute:
    first: bool
    last: bool
    device: torch.device

    def in_spec(self, batch: int) -> Spec:
        raise NotImplementedError

    def out_spec(self, batch: int) -> Spec:
        raise NotImplementedError

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None):
        raise NotImplementedError


class CifarHipStage(StageCompute):
    """CIFAR units [start, end] on the fused HIP kernels.

    Units 0-1 always run together (the fused conv1/pool/conv2/pool kernel), so
    the supported ranges are (0,1) = reference part 0, (2,3) = reference part 1,
    (0,3) = whole model, (2,2) = fc1 alone (3-stage pipelines), and the fc1 cut (0,2) | (3,3) whose stage boundary is
    the 512-wide hidden (2 KiB/img in fp32 instead of 16 KiB: what the
    multi-GPU placement uses when the xGMI hop, not compute, would bound the
    pipeline, parallel/partition.py ``cifar_cut``).

    ``precision`` "fp32" (default, the reference's: fp32 in, fp32 boundary,
    3-term bf16 split products accumulated in fp32) or "bf16".

    ``boundary`` (fp32, the conv|fc cut): "fp32" values on the 16 KiB/img
    boundary (default; what a reference peer expects over gRPC), or "split" —
    the blocked hi/lo encoding of the same 16 KiB (``ops/cifar.py``;
    bit-identical results, measured neutral end to end).  Both stages of a hop
    must agree."""

    SUPPORTED = {(0, 1), (2, 3), (0, 3), (0, 2), (2, 2), (3, 3)}

    def __init__(self, sd: Dict[str, torch.Tensor], start: int, end: int, device: torch.device,
                 precision: str = "fp32", boundary: str = "fp32"):
        from ..ops import cifar as cops
        if (start, end) not in self.SUPPORTED:
            raise ValueError(f"HIP CIFAR backend supports unit ranges {sorted(self.SUPPORTED)}, got ({start},{end})")
        self.start, self.end, self.device = start, end, torch.device(device)
        self.first, self.last = start == 0, end == cifar.NUM_UNITS - 1
        self.precision = precision
        if boundary not in cops.BOUNDARIES:
            raise ValueError(f"boundary must be one of {cops.BOUNDARIES}")
        # the encoding only exists on the 4096-wide conv|fc boundary of the fp32 path
        self.boundary = boundary if precision == "fp32" else "fp32"
        self._cops = cops
        self.adt = cops.act_dtype(precision)
        self.w0 = cops.pack_stage0(sd, self.device, precision) if start == 0 else None
        self.wh = cops.pack_head(sd, self.device, fc1=start <= 2 <= end, fc2=end == 3, precision=precision)
        self._scratch: Dict[int, Dict[str, torch.Tensor]] = {}

    def _boundary(self, unit: int):
        return ((cifar.FLAT_DIM if unit == 1 else 512), self.adt)

    def in_spec(self, batch):
        if self.first:
            return (batch, 3, 32, 32), torch.float32
        w, dt = self._boundary(self.start - 1)
        return (batch, w), dt

    def out_spec(self, batch):
        if self.last:
            return (batch, 10), torch.float32
        w, dt = self._boundary(self.end)
        return (batch, w), dt

    def _buf(self, batch):
        b = self._scratch.get(batch)
        if b is None:
            d = self.device
            b = {}
            if self.first and self.end >= 2:
                b["mid"] = torch.empty((batch, 4096), dtype=self.adt, device=d)
            if self.start <= 2 <= self.end and self.precision == "fp32" and batch < self._cops.FC1_X3_MIN_ROWS:
                b["split"] = torch.empty((batch, 3 * 4096), dtype=torch.bfloat16, device=d)
            if self.last:
                b["hid"] = torch.empty((batch, 512), dtype=self.adt, device=d)
                b["pred"] = torch.empty((batch,), dtype=torch.int32, device=d)
            self._scratch[batch] = b
        return b

    def forward(self, x, out=None):
        B = x.shape[0]
        buf = self._buf(B)
        h = x
        if self.first:
            if h.dtype != torch.float32:
                h = h.float()
            h = self._cops.stage0_forward(h.contiguous(), self.w0, buf["mid"] if self.end >= 2 else out,
                                          boundary=self.boundary)
            if self.end == 1:
                return h
        elif h.dtype != self.adt:
            h = h.to(self.adt)
        if self.start <= 2 <= self.end:
            h = self._cops.fc1_forward(h.contiguous(), self.wh, out if self.end == 2 else buf["hid"],
                                       scratch=buf.get("split"), boundary=self.boundary)
            if self.end == 2:
                return h
        probs, pred = self._cops.head_tail(h.contiguous(), self.wh, out, buf["pred"])
        return StageOutput(probs, pred)


class TorchStage(StageCompute):
    """Golden torch module as a stage (CPU fp32 plumbing path / tests)."""

    def __init__(self, model: str, sd: Dict[str, torch.Tensor], start: int, end: int, first: bool, last: bool,
                 device="cpu", dtype=torch.float32, sampling=(0.0, 0, 0)):
        from ..models import build_golden_stage
        self.temperature, self.top_k, self.seed = float(sampling[0]), int(sampling[1]), int(sampling[2])
        self.model, self.start, self.end, self.first, self.last = model, start, end, first, last
        self.device = torch.device(device)
        self.family = model_info(model).family
        self.module = build_golden_stage(model, start, end, first, last)
        missing, unexpected = self.module.load_state_dict(sd, strict=False)
        if missing:
            raise KeyError(f"stage [{start},{end}] missing weights: {missing[:8]}")
        self.module = self.module.to(device=self.device, dtype=dtype).eval()
        # CPU CIFAR convolutions in NHWC (oneDNN's preferred layout): stage 0
        # at B = 255 on 4 threads 56 -> 29 ms; the flatten to the (B, 4096)
        # boundary still follows the reference's NCHW order (a logical reshape).
        # GPU golden stages keep NCHW (the fp32 oracle of the HIP kernels).
        self.nhwc = self.family == "cifar" and self.device.type == "cpu"
        if self.nhwc:
            self.module = self.module.to(memory_format=torch.channels_last)
        self.dtype = dtype

    def in_spec(self, batch, seq: int = 0):
        if self.family == "cifar":
            return cifar.input_shape(self.start, batch), self.dtype
        info = model_info(self.model)
        if self.first:
            return (batch, seq), torch.int64
        return (batch, seq, info.cfg.n_embd), self.dtype

    def out_spec(self, batch, seq: int = 0):
        if self.family == "cifar":
            return cifar.output_shape(self.end, batch), self.dtype
        info = model_info(self.model)
        if self.last:
            return (batch, seq, info.cfg.vocab_size), self.dtype
        return (batch, seq, info.cfg.n_embd), self.dtype

    @property
    def d(self) -> int:
        return model_info(self.model).cfg.n_embd

    @property
    def act_dtype(self) -> torch.dtype:
        return self.dtype

    @torch.no_grad()
    def step(self, x, pos, B: int, T: int, b0: int = 0, out=None, last_only: bool = True):
        """KV-cached transformer step (CPU golden path; same contract as
        ``TransformerStage.step``): x = ids (B,T) on the first stage, else
        hidden (B*T, d); ``pos`` = tokens already cached (uniform per batch);
        rows ``[b0, b0+B)`` of the cache (one KV cache per microbatch offset)."""
        cfg = model_info(self.model).cfg
        p = int(pos[0]) if isinstance(pos, torch.Tensor) else int(pos)
        caches = getattr(self, "_kv", None)
        if caches is None:
            caches = self._kv = {}
        kv = caches.get(b0)
        if kv is None or kv[0][0].shape[0] != B:
            S = getattr(cfg, "block_size", getattr(cfg, "max_seq", 1024))
            hkv = getattr(cfg, "n_kv_head", cfg.n_head)
            hd = cfg.n_embd // cfg.n_head
            n = len(self.module.h if self.family == "gpt2" else self.module.layers)
            kv = caches[b0] = [(torch.zeros(B, hkv, S, hd, dtype=self.dtype), torch.zeros(B, hkv, S, hd, dtype=self.dtype))
                               for _ in range(n)]
        if self.first:
            h = x.to(torch.int64).view(B, T)
        else:
            h = x.view(B, T, cfg.n_embd).to(self.dtype)
        y = self.module(h, kv, p, last_only=last_only)
        if self.last:
            from .sampling import pick
            logits = y[:, -1, :] if last_only else y.reshape(B * T, -1)
            step = pos if isinstance(pos, torch.Tensor) else torch.full((B,), p, dtype=torch.int32)
            pred = pick(y[:, -1, :], self.temperature, self.top_k, self.seed, step).to(torch.int32)
            if out is not None and last_only:
                out.copy_(pred)
                pred = out
            return StageOutput(logits, pred)
        y = y.reshape(B * T, cfg.n_embd)
        if out is not None:
            out.view(B * T, cfg.n_embd).copy_(y)
            return out
        return y

    @torch.no_grad()
    def forward(self, x, out=None):
        x = x.to(self.device)
        with torch.no_grad():  # no autograd graph: a third of the CPU conv stage's time
            if self.nhwc and x.dim() == 4:
                x = x.contiguous(memory_format=torch.channels_last)
            y = self.module(x)
            if y.dim() == 4:
                y = y.contiguous()  # a 4-D boundary crosses the wire in NCHW order
        if self.last:
            if self.family == "cifar":
                return StageOutput(y, y.argmax(dim=1).to(torch.int32))
            return StageOutput(y, y[:, -1, :].argmax(dim=-1).to(torch.int32))
        if out is not None:
            out.copy_(y)
            return out
        return y
