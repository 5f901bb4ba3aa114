"""Layer-range partitioning for pipeline stages.

The reference splits layers by hand-written part classes (CIFAR,
``cifar_model_parts.py:29-58``) or by explicit ``(start_layer, end_layer)``
inclusive ranges (GPT, ``partitions/gpt_model_parts.py:7-12``) that nothing ever
computes.  Here ranges are either given per node (``layers: [start, end]`` in the
config) or computed by a cost-balanced split that accounts for the extra work of
the first stage (embedding) and the last stage (``ln_f`` + ``lm_head``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

Range = Tuple[int, int]


def even_ranges(num_layers: int, num_stages: int) -> List[Range]:
    """Contiguous inclusive ranges, sizes differing by at most one (earlier stages larger)."""
    if num_stages < 1 or num_layers < num_stages:
        raise ValueError(f"cannot split {num_layers} layers into {num_stages} stages")
    base, rem = divmod(num_layers, num_stages)
    out, s = [], 0
    for i in range(num_stages):
        n = base + (1 if i < rem else 0)
        out.append((s, s + n - 1))
        s += n
    return out


def balanced_ranges(num_layers: int, num_stages: int, first_extra: float = 0.0,
                    last_extra: float = 0.0) -> List[Range]:
    """Minimise the max stage cost where each layer costs 1, the first stage
    carries ``first_extra`` and the last ``last_extra`` layer-equivalents.
    Exact DP over split points (L, S are small)."""
    if num_stages < 1 or num_layers < num_stages:
        raise ValueError(f"cannot split {num_layers} layers into {num_stages} stages")
    L, S = num_layers, num_stages
    INF = float("inf")

    def cost(stage: int, a: int, b: int) -> float:  # layers a..b-1
        c = float(b - a)
        if stage == 0:
            c += first_extra
        if stage == S - 1:
            c += last_extra
        return c

    # best[s][i] = min max-cost placing first i layers into s stages
    best = [[INF] * (L + 1) for _ in range(S + 1)]
    arg = [[-1] * (L + 1) for _ in range(S + 1)]
    best[0][0] = 0.0
    for s in range(1, S + 1):
        for i in range(s, L + 1):
            for j in range(s - 1, i):
                if best[s - 1][j] == INF:
                    continue
                v = max(best[s - 1][j], cost(s - 1, j, i))
                # tie-break: prefer earlier stages larger (stable, matches even_ranges)
                if v < best[s][i] - 1e-12:
                    best[s][i], arg[s][i] = v, j
    out: List[Range] = []
    i = L
    for s in range(S, 0, -1):
        j = arg[s][i]
        out.append((j, i - 1))
        i = j
    return out[::-1]


def validate_ranges(ranges: Sequence[Range], num_layers: int) -> None:
    s = 0
    for a, b in ranges:
        if a != s or b < a:
            raise ValueError(f"layer ranges {list(ranges)} are not a contiguous cover of 0..{num_layers - 1}")
        s = b + 1
    if s != num_layers:
        raise ValueError(f"layer ranges {list(ranges)} do not cover 0..{num_layers - 1}")


def resolve_ranges(num_layers: int, num_stages: int, given: Sequence[Optional[Range]],
                   first_extra: float = 0.0, last_extra: float = 0.0) -> List[Range]:
    """Use per-node ``layers`` if every node gives one, else compute a balanced split."""
    if given and all(g is not None for g in given):
        r = [tuple(g) for g in given]  # type: ignore[arg-type]
        validate_ranges(r, num_layers)
        return r  # type: ignore[return-value]
    if any(g is not None for g in given):
        raise ValueError("either every node or no node may specify 'layers'")
    return balanced_ranges(num_layers, num_stages, first_extra, last_extra)
