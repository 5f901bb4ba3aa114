"""Tensor <-> ``node_service.Tensor`` codec.

Reference encoding (inline in ``node.py:45-48,64-68,76-81,174-178,186-189``):
``tensor_data = ndarray.tobytes()`` (C order, native little-endian),
``shape = list(shape)``, ``dtype = str(ndarray.dtype)`` (a numpy dtype name such
as ``"float32"``/``"int64"``).  Decoding is ``np.frombuffer(...).reshape(shape)``.

Kept identical for numpy dtypes.  Extension: dtypes numpy cannot express are
sent as raw little-endian bytes under their torch names — ``"bfloat16"``,
``"float8_e4m3fn"``, ``"float8_e5m2"`` — so a bf16 activation crosses the CPU
wire without an fp32 round trip.  The GPU data plane never uses this (RCCL
moves device buffers).
"""
from __future__ import annotations

from typing import Union

import numpy as np
import torch

from . import proto

_TORCH_ONLY = {
    "bfloat16": torch.bfloat16,
    "float8_e4m3fn": torch.float8_e4m3fn,
    "float8_e5m2": torch.float8_e5m2,
}
_TORCH_ONLY_INV = {v: k for k, v in _TORCH_ONLY.items()}


def encode(t: Union[torch.Tensor, np.ndarray]) -> "proto.Tensor":
    if isinstance(t, torch.Tensor):
        t = t.detach()
        if t.device.type != "cpu":
            t = t.cpu()
        if t.dtype in _TORCH_ONLY_INV:
            name = _TORCH_ONLY_INV[t.dtype]
            raw = t.contiguous().view(torch.uint8).numpy().tobytes()
            return proto.Tensor(tensor_data=raw, shape=list(t.shape), dtype=name)
        t = t.contiguous().numpy()
    a = np.ascontiguousarray(t)
    return proto.Tensor(tensor_data=a.tobytes(), shape=list(a.shape), dtype=str(a.dtype))


def decode(msg: "proto.Tensor", device: Union[str, torch.device, None] = None) -> torch.Tensor:
    shape = tuple(msg.shape)
    if msg.dtype in _TORCH_ONLY:
        u8 = torch.frombuffer(bytearray(msg.tensor_data), dtype=torch.uint8)
        t = u8.view(_TORCH_ONLY[msg.dtype]).reshape(shape)
    else:
        a = np.frombuffer(msg.tensor_data, dtype=np.dtype(msg.dtype)).reshape(shape)
        t = torch.from_numpy(a.copy())
    return t.to(device) if device is not None else t


def decode_numpy(msg: "proto.Tensor") -> np.ndarray:
    if msg.dtype in _TORCH_ONLY:
        return decode(msg).float().numpy()
    return np.frombuffer(msg.tensor_data, dtype=np.dtype(msg.dtype)).reshape(tuple(msg.shape))
