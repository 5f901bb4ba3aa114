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


def choose_cut(unit_ns: Sequence[float], boundary_bytes: Sequence[int], cuts: Sequence[int], placement: str,
               world: int, link_gbs: float) -> int:
    """Pick the 2-stage cut (stage 0 = units [0..c], stage 1 = [c+1..]) that
    minimises the per-item pipeline period under a compute + link cost model.

    * ``linear`` (one stage per GPU): period = max(t_stage0, t_stage1, hop)
      with the hop on ONE xGMI link;
    * ``interleaved`` (every GPU hosts stage 0 of one pipeline and stage 1 of
      the others, hop = all-to-all): compute is balanced by construction and
      the hop is spread over the ``world-1`` links of the fully connected
      board, overlapped with compute: period = max(sum(t), hop / (world-1)).
    ``unit_ns`` = per-item compute of each unit; ``boundary_bytes[c]`` = bytes
    per item crossing a cut after unit c; ``link_gbs`` = usable GB/s per link.
    """
    best, best_t = None, float("inf")
    for c in cuts:
        t0, t1 = sum(unit_ns[:c + 1]), sum(unit_ns[c + 1:])
        hop = boundary_bytes[c] / link_gbs  # bytes / (GB/s) = ns
        if placement == "linear":
            t = max(t0, t1, hop)
        else:
            t = max(t0 + t1, hop / max(1, world - 1))
        if t < best_t - 1e-9:
            best, best_t = c, t
    return best


# Measured on 1x MI355X: per-image ns of the CIFAR units with the fused kernels
# (conv stage = units 0-1 together) and the boundary bytes per image, per
# precision (bf16: profiles/archive/r1_*; fp32: profiles/archive/r2_cifar_fc1_fused_ab.jsonl,
# profiles/archive/r2_bench_cifar_fp32_n1_kernels.md at B = 65536).
CIFAR_UNIT_NS = {"bf16": (0.0, 10.8, 5.3, 0.3), "fp32": (0.0, 27.0, 11.7, 0.5)}
CIFAR_BOUNDARY_BYTES = {"bf16": (32 * 16 * 16 * 2, 4096 * 2, 512 * 2, 10 * 4),
                        "fp32": (32 * 16 * 16 * 4, 4096 * 4, 512 * 4, 10 * 4)}
XGMI_LINK_GBS = 50.0  # conservative usable P2P GB/s per direction per link (7 links x ~153 GB/s aggregate spec)


def cifar_cut(placement: str, world: int, link_gbs: float = XGMI_LINK_GBS, precision: str = "fp32") -> int:
    """Cut for the CIFAR 2-stage pipeline on MI355X: 1 (reference conv|fc) or 2 (after fc1)."""
    if placement == "linear":
        return linear_plan(world, precision, link_gbs)["cut"]
    return choose_cut(CIFAR_UNIT_NS[precision], CIFAR_BOUNDARY_BYTES[precision], (1, 2), placement, world, link_gbs)


def linear_plan(world: int, precision: str = "fp32", link_gbs: float = XGMI_LINK_GBS,
                unit_ns: Optional[Sequence[float]] = None, boundary_bytes: Optional[Sequence[int]] = None,
                cuts: Sequence[int] = (1, 2)) -> dict:
    """Linear 2-stage pipeline on ``world`` GPUs, one stage per GPU: ``n0``
    GPUs run stage 0 (units [0..cut]) and each sends its activations over its
    own direct xGMI link to one of ``n1`` stage-1 GPUs (sender s -> receiver
    n0 + s % n1).  The bottleneck stage is replicated instead of left idle:
    with stage 0 at ~99 % of the compute after the fc1 cut, 7 stage-0 GPUs feed
    1 stage-1 GPU on 8 GPUs (every sender on a link of its own on the fully
    connected board).  Chooses (cut, n0, n1) maximising items per ns:
    min(n0 / t0, n1 / t1, n0 / hop) (a hop overlaps the next microbatch)."""
    unit_ns = unit_ns or CIFAR_UNIT_NS[precision]
    boundary_bytes = boundary_bytes or CIFAR_BOUNDARY_BYTES[precision]
    if world < 2:
        raise ValueError("a linear pipeline needs >= 2 GPUs")
    best, best_rate = None, -1.0
    for c in cuts:
        t0, t1 = sum(unit_ns[:c + 1]), sum(unit_ns[c + 1:])
        hop = boundary_bytes[c] / link_gbs
        for n1 in range(1, world):
            n0 = world - n1
            rate = min(n0 / t0, n1 / max(t1, 1e-9), n0 / hop)
            if rate > best_rate + 1e-12:
                best, best_rate = {"cut": c, "n0": n0, "n1": n1}, rate
    best["items_per_ns"] = best_rate
    return best


def linear_role(rank: int, plan: dict) -> dict:
    """This rank's role in ``linear_plan``: stage, its peer(s)."""
    n0, n1 = plan["n0"], plan["n1"]
    if rank < n0:
        return {"stage": 0, "send_to": n0 + rank % n1}
    return {"stage": 1, "recv_from": [s for s in range(n0) if n0 + s % n1 == rank]}


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
