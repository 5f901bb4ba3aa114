"""CIFAR-10 ConvNet: torch golden model + pipeline stage modules.

Architecture and state-dict keys follow the reference (``cifar_model_parts.py:7-26``):
conv1 3->32 k3 p1, 2x2 max-pool, conv2 32->64 k3 p1, pool, flatten (NCHW order),
fc1 4096->512, fc2 512->10, softmax(dim=1) inside the model.  Keys:
``conv1.{weight,bias}`` (32,3,3,3), ``conv2.*`` (64,32,3,3), ``fc1.*`` (512,4096),
``fc2.*`` (10,512) so reference ``.pth`` files load unchanged.

The model is expressed as four *layer units* so any contiguous split can be a
pipeline stage (the reference hard-wires the 2-stage split after the conv
blocks, ``cifar_model_parts.py:29-58``; that split is the default here):

    unit 0: conv1 + ReLU + pool        (B,3,32,32)  -> (B,32,16,16)
    unit 1: conv2 + ReLU + pool + flat (B,32,16,16) -> (B,4096)
    unit 2: fc1 + ReLU                 (B,4096)     -> (B,512)
    unit 3: fc2 + softmax              (B,512)      -> (B,10)

These modules are the fp32 golden oracle and the CPU (gRPC plumbing) compute
path.  The MI355X path uses the fused HIP kernels in ``ops/cifar.py``.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

NUM_UNITS = 4
DEFAULT_SPLIT_2 = [(0, 1), (2, 3)]
FLAT_DIM = 64 * 8 * 8
NUM_CLASSES = 10
UNIT_KEYS = {0: ("conv1",), 1: ("conv2",), 2: ("fc1",), 3: ("fc2",)}


class NeuralNetwork(nn.Module):
    """Full CIFAR-10 ConvNet (golden). Parameter names match the reference checkpoint."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3, 1, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1, 1)
        self.fc1 = nn.Linear(FLAT_DIM, 512)
        self.fc2 = nn.Linear(512, NUM_CLASSES)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        for u in range(NUM_UNITS):
            x = run_unit(self, u, x)
        return x


def run_unit(m: nn.Module, unit: int, x: torch.Tensor) -> torch.Tensor:
    if unit == 0:
        return F.max_pool2d(F.relu(m.conv1(x)), 2, 2)
    if unit == 1:
        return F.max_pool2d(F.relu(m.conv2(x)), 2, 2).reshape(-1, FLAT_DIM)
    if unit == 2:
        return F.relu(m.fc1(x))
    if unit == 3:
        return F.softmax(m.fc2(x), dim=1)
    raise ValueError(f"CIFAR ConvNet has units 0..3, got {unit}")


class CifarStage(nn.Module):
    """Units ``[start, end]`` (inclusive) of the ConvNet as one pipeline stage.

    Owns only its own parameters (under their full-model names), so
    ``load_state_dict(full_sd, strict=False)`` picks exactly this stage's
    weights — the same mechanism as the reference's part classes
    (``node.py:305-306``), but checked: ``checkpoint.load_stage`` verifies no
    stage key is missing.
    """

    def __init__(self, start: int, end: int):
        super().__init__()
        if not (0 <= start <= end < NUM_UNITS):
            raise ValueError(f"invalid CIFAR unit range [{start}, {end}]")
        self.start, self.end = start, end
        full = NeuralNetwork()
        for u in range(start, end + 1):
            for name in UNIT_KEYS[u]:
                setattr(self, name, getattr(full, name))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        for u in range(self.start, self.end + 1):
            x = run_unit(self, u, x)
        return x

    def expected_keys(self) -> List[str]:
        return list(self.state_dict().keys())


def stage_ranges(num_parts: int) -> List[Tuple[int, int]]:
    """Default unit ranges per stage. 2 stages = the reference split."""
    if num_parts == 2:
        return list(DEFAULT_SPLIT_2)
    if num_parts == 1:
        return [(0, NUM_UNITS - 1)]
    if num_parts == 4:
        return [(i, i) for i in range(4)]
    if num_parts == 3:
        return [(0, 0), (1, 1), (2, 3)]
    raise ValueError(f"CIFAR ConvNet supports 1..4 stages, got {num_parts}")


def input_shape(unit: int, batch: int) -> Tuple[int, ...]:
    return {0: (batch, 3, 32, 32), 1: (batch, 32, 16, 16), 2: (batch, FLAT_DIM), 3: (batch, 512)}[unit]


def output_shape(unit: int, batch: int) -> Tuple[int, ...]:
    return {0: (batch, 32, 16, 16), 1: (batch, FLAT_DIM), 2: (batch, 512), 3: (batch, NUM_CLASSES)}[unit]


def flops_per_image() -> Dict[str, float]:
    c1 = 2 * 32 * 32 * 32 * 27
    c2 = 2 * 16 * 16 * 64 * 288
    f1 = 2 * 4096 * 512
    f2 = 2 * 512 * 10
    return {"conv1": c1, "conv2": c2, "fc1": f1, "fc2": f2, "total": c1 + c2 + f1 + f2}


def random_state_dict(seed: int = 0) -> Dict[str, torch.Tensor]:
    torch.manual_seed(seed)
    return NeuralNetwork().state_dict()
