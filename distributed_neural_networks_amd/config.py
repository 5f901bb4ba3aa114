"""Config loading and validation for the reference ``config.json`` schema.

Behavioural contract (reference ``node.py:222-290``, ``config.json:1-18``):

* ``nodes[{id, address, part_index}]``, ``model_weights``, ``num_parts`` and the
  optional ``return_to_node_id`` keep their meaning and the reference's error
  strings (``node.py:227,230,236,251,257,266,270``).
* The reference hard-rejects ``num_parts != 2`` (``node.py:246-248``).  Here any
  ``num_parts >= 1`` is accepted as long as the ``part_index`` values are a
  permutation of ``0..num_parts-1`` — the only way a pipeline of more than two
  stages (GPT-2 4-stage, Llama-3 8-stage) can be described with this schema.
* Additive optional fields (absent in the reference file, so it still loads):
  top level ``model``, ``dtype``, ``transport``, ``micro_batch_size``,
  ``num_microbatches``, ``seq_len``, ``decode_steps``, ``prompt_len``, ``temperature``, ``top_k``,
  ``seed``, ``heartbeat_timeout_s``, ``stall_timeout_s``, ``prefill_chunk``, ``replicas``,
  ``kv_cache_dtype``, ``kv_cache_scale``, ``fp8_prefill``; per node
  ``layers: [start, end]`` (inclusive, as in
  ``partitions/gpt_model_parts.py:12``) and ``device``.

Nothing here touches torch, so it is cheap to import from the CLI and tests.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

TRANSPORTS = ("grpc", "colocated", "rccl", "gloo", "gloo_gpu")
DIST_TRANSPORTS = ("rccl", "gloo", "gloo_gpu")  # one rank per stage (and replica)
MODELS = ("cifar10", "gpt2", "gpt2-medium", "gpt2-large", "gpt2-xl", "gpt2-tiny",
          "llama3-8b", "llama3-tiny")


class ConfigError(Exception):
    """A config problem the CLI reports as ``print(msg); exit(1)`` (reference style)."""


@dataclass
class NodeSpec:
    id: str
    address: str
    part_index: int
    layers: Optional[Tuple[int, int]] = None
    device: Optional[int] = None

    @property
    def host(self) -> str:
        return self.address.rsplit(":", 1)[0]

    @property
    def port(self) -> int:
        return int(self.address.rsplit(":", 1)[-1])


@dataclass
class PipelineConfig:
    """The whole topology: every stage, in stage order."""

    nodes: List[NodeSpec]
    model_weights: str
    num_parts: int
    return_to_node_id: Optional[str] = None
    model: str = "cifar10"
    dtype: Optional[str] = None
    kv_cache_dtype: str = "bf16"              # "fp8": OCP e4m3 KV cache (half the decode K/V bytes)
    kv_cache_scale: str = "calibrated"        # fp8 cache: per-layer scale from the first prefill's amax, or "unit"
    fp8_prefill: str = "e4m3"                 # dtype fp8: prefill activations "e4m3" (one byte, per-row scale) or "split" (e4m3 hi + residual)
    transport: str = "grpc"
    micro_batch_size: int = 1
    num_microbatches: int = 1
    seq_len: int = 64
    prompt_len: Optional[int] = None
    decode_steps: int = 0
    prefill_chunk: int = 0                    # > 0: chunked prefill, this many prompt tokens per stage call
    temperature: float = 0.0                  # 0 = greedy; > 0 = sampling (last stage)
    top_k: int = 0                            # 0 = whole vocabulary
    seed: int = 0                             # sampling seed (counter-based RNG, reproducible)
    rpc_timeout_s: Optional[float] = None     # per-hop SendTensor deadline (reference: none)
    health_timeout_s: float = 120.0           # readiness barrier before stage 0 sends
    comm_timeout_s: float = 300.0             # process-group (RCCL/gloo) op timeout
    heartbeat_timeout_s: float = 15.0         # parallel/watchdog.py: peer declared dead after this
    stall_timeout_s: Optional[float] = None   # parallel/watchdog.py: abort when this rank stops progressing
    replicas: int = 1                         # data-parallel copies of the whole pipeline (rccl / gloo)
    raw: Dict[str, Any] = field(default_factory=dict)

    def stage(self, part_index: int) -> NodeSpec:
        for n in self.nodes:
            if n.part_index == part_index:
                return n
        raise ConfigError(f"ERROR: Could not find node config for next part index {part_index}")

    def by_id(self, node_id: str) -> Optional[NodeSpec]:
        return next((n for n in self.nodes if n.id == node_id), None)

    @property
    def stages(self) -> List[NodeSpec]:
        return sorted(self.nodes, key=lambda n: n.part_index)


@dataclass
class NodeContext:
    """Per-process view of the config (replaces the reference's module globals,
    ``node.py:17-26``)."""

    node_id: str
    address: str
    port: int
    part_index: int
    num_parts: int
    model_weights: str
    is_last: bool
    next_address: Optional[str]
    return_address: Optional[str]
    pipeline: PipelineConfig
    replica: int = 0  # which data-parallel copy of the pipeline this process serves

    @property
    def node(self) -> NodeSpec:
        return self.pipeline.stage(self.part_index)

    @property
    def rank(self) -> int:
        """Process-group rank: replica-major, ``replica * num_parts + part_index``."""
        return self.replica * self.num_parts + self.part_index

    @property
    def world(self) -> int:
        return self.pipeline.replicas * self.num_parts

    def peer(self, part_index: int) -> int:
        """Rank of stage ``part_index`` of this process's own replica."""
        return self.replica * self.num_parts + part_index


def load_json(path: str) -> Dict[str, Any]:
    """``node.py:222-231``: file-not-found and bad-JSON errors, same wording."""
    try:
        with open(path, "r") as f:
            return json.load(f)
    except FileNotFoundError:
        raise ConfigError(f"ERROR: Config file not found at '{path}'")
    except json.JSONDecodeError as e:
        raise ConfigError(f"ERROR: Invalid JSON in config file '{path}': {e}")


def _parse_layers(v: Any) -> Optional[Tuple[int, int]]:
    if v is None:
        return None
    if not (isinstance(v, (list, tuple)) and len(v) == 2 and all(isinstance(i, int) for i in v)):
        raise ConfigError(f"ERROR: 'layers' must be [start, end] (inclusive), got {v!r}")
    if v[0] > v[1] or v[0] < 0:
        raise ConfigError(f"ERROR: invalid layer range {v!r}")
    return (int(v[0]), int(v[1]))


def parse_pipeline(cfg: Dict[str, Any], path: str = "<config>") -> PipelineConfig:
    raw_nodes = cfg.get("nodes", [])
    num_parts = cfg.get("num_parts")
    weights = cfg.get("model_weights")
    nodes: List[NodeSpec] = []
    for n in raw_nodes:
        if n.get("address") is None or n.get("part_index") is None:
            raise ConfigError("ERROR: Config file is missing required fields (address, part_index, model_weights, num_parts)")
        address = n["address"]
        try:
            int(str(address).split(":")[-1])
        except (ValueError, IndexError):
            raise ConfigError(f"ERROR: Invalid format for MY_ADDRESS '{address}'. Expected IP:Port.")
        nodes.append(NodeSpec(id=str(n.get("id")), address=str(address), part_index=int(n["part_index"]),
                              layers=_parse_layers(n.get("layers")), device=n.get("device")))
    if None in [weights, num_parts]:
        raise ConfigError("ERROR: Config file is missing required fields (address, part_index, model_weights, num_parts)")
    if not isinstance(num_parts, int) or num_parts < 1:
        raise ConfigError(f"ERROR: Configuration file specifies num_parts={num_parts}, but this script expects a positive integer.")
    idx = sorted(n.part_index for n in nodes)
    if idx != list(range(num_parts)):
        raise ConfigError(f"ERROR: Configuration file specifies num_parts={num_parts}, but part_index values are {idx}; "
                          f"expected a permutation of 0..{num_parts - 1}.")
    transport = cfg.get("transport", "grpc")
    if transport not in TRANSPORTS:
        raise ConfigError(f"ERROR: unknown transport '{transport}', expected one of {TRANSPORTS}")
    model = cfg.get("model", "cifar10")
    if model not in MODELS:
        raise ConfigError(f"ERROR: unknown model '{model}', expected one of {MODELS}")
    for key in ("micro_batch_size", "num_microbatches"):
        v = cfg.get(key, 1)
        if not isinstance(v, int) or v < 1:
            raise ConfigError(f"ERROR: '{key}' must be a positive integer, got {v!r}")
    for key in ("prefill_chunk", "decode_steps", "top_k", "seed"):
        v = cfg.get(key, 0)
        if not isinstance(v, int) or isinstance(v, bool) or v < 0:
            raise ConfigError(f"ERROR: '{key}' must be a non-negative integer, got {v!r}")
    for key in ("heartbeat_timeout_s", "stall_timeout_s", "health_timeout_s", "comm_timeout_s", "rpc_timeout_s"):
        v = cfg.get(key)
        if v is not None and (not isinstance(v, (int, float)) or isinstance(v, bool) or v <= 0):
            raise ConfigError(f"ERROR: '{key}' must be a positive number of seconds, got {v!r}")
    reps = cfg.get("replicas", 1)
    if not isinstance(reps, int) or isinstance(reps, bool) or reps < 1:
        raise ConfigError(f"ERROR: 'replicas' must be a positive integer, got {reps!r}")
    if reps > 1 and transport not in DIST_TRANSPORTS:
        raise ConfigError(f"ERROR: 'replicas' > 1 needs transport 'rccl', 'gloo' or 'gloo_gpu' (one rank per stage and replica), "
                          f"got '{transport}'")
    kvd = cfg.get("kv_cache_dtype", "bf16")
    if kvd not in ("bf16", "fp8"):
        raise ConfigError(f"ERROR: 'kv_cache_dtype' must be 'bf16' or 'fp8', got {kvd!r}")
    fpp = cfg.get("fp8_prefill", "e4m3")
    if fpp not in ("split", "e4m3"):
        raise ConfigError(f"ERROR: 'fp8_prefill' must be 'split' or 'e4m3', got {fpp!r}")
    kvs = cfg.get("kv_cache_scale", "calibrated")
    if kvs not in ("calibrated", "unit"):
        raise ConfigError(f"ERROR: 'kv_cache_scale' must be 'calibrated' or 'unit', got {kvs!r}")
    t = cfg.get("temperature", 0.0)
    if not isinstance(t, (int, float)) or t < 0:
        raise ConfigError(f"ERROR: 'temperature' must be >= 0, got {t!r}")
    ret = cfg.get("return_to_node_id")
    if ret is not None and transport in DIST_TRANSPORTS:
        rn = next((n for n in nodes if n.id == ret), None)
        if rn is None:
            raise ConfigError(f"ERROR: return_to_node_id '{ret}' is not a node of this config")
    return PipelineConfig(
        nodes=nodes, model_weights=str(weights), num_parts=num_parts,
        return_to_node_id=cfg.get("return_to_node_id"), model=model, dtype=cfg.get("dtype"), kv_cache_dtype=kvd,
        kv_cache_scale=kvs, fp8_prefill=fpp,
        transport=transport, micro_batch_size=int(cfg.get("micro_batch_size", 1)),
        num_microbatches=int(cfg.get("num_microbatches", 1)), seq_len=int(cfg.get("seq_len", 64)),
        prompt_len=cfg.get("prompt_len"), decode_steps=int(cfg.get("decode_steps", 0)),
        prefill_chunk=int(cfg.get("prefill_chunk", 0)),
        temperature=float(cfg.get("temperature", 0.0)), top_k=int(cfg.get("top_k", 0)), seed=int(cfg.get("seed", 0)),
        rpc_timeout_s=cfg.get("rpc_timeout_s"), health_timeout_s=float(cfg.get("health_timeout_s", 120.0)),
        comm_timeout_s=float(cfg.get("comm_timeout_s", 300.0)),
        heartbeat_timeout_s=float(cfg.get("heartbeat_timeout_s", 15.0)),
        stall_timeout_s=(None if cfg.get("stall_timeout_s") is None else float(cfg["stall_timeout_s"])),
        replicas=int(reps), raw=cfg)


def resolve_node(cfg: Dict[str, Any], node_id: str, path: str = "<config>", replica: int = 0) -> NodeContext:
    """Own-node lookup + topology (``node.py:234-278``); ``replica`` selects the
    data-parallel copy of the pipeline (config ``replicas``)."""
    mine = next((n for n in cfg.get("nodes", []) if n.get("id") == node_id), None)
    if not mine:
        raise ConfigError(f"ERROR: Node ID '{node_id}' not found in config file '{path}'")
    address, part_index = mine.get("address"), mine.get("part_index")
    if None in [address, part_index, cfg.get("model_weights"), cfg.get("num_parts")]:
        raise ConfigError("ERROR: Config file is missing required fields (address, part_index, model_weights, num_parts)")
    try:
        port = int(str(address).split(":")[-1])
    except (ValueError, IndexError):
        raise ConfigError(f"ERROR: Invalid format for MY_ADDRESS '{address}'. Expected IP:Port.")
    pipe = parse_pipeline(cfg, path)
    is_last = part_index == pipe.num_parts - 1
    next_address = None
    return_address = None
    if not is_last:
        nxt = next((n for n in pipe.nodes if n.part_index == part_index + 1), None)
        if nxt is None:
            raise ConfigError(f"ERROR: Could not find node config for next part index {part_index + 1}")
        if not nxt.address:
            raise ConfigError(f"ERROR: Next node (index {part_index + 1}) is missing address in config")
        next_address = nxt.address
    else:
        # The reference resolves this and never uses it (node.py:272-277); here it is
        # the ring back-edge: where the last stage sends results / sampled tokens.
        if pipe.return_to_node_id:
            ret = pipe.by_id(pipe.return_to_node_id)
            if ret is not None:
                return_address = ret.address
    if not (isinstance(replica, int) and 0 <= replica < pipe.replicas):
        raise ConfigError(f"ERROR: replica {replica!r} out of range: the config has {pipe.replicas} replica(s)")
    return NodeContext(node_id=node_id, address=str(address), port=port, part_index=int(part_index),
                       num_parts=pipe.num_parts, model_weights=pipe.model_weights, is_last=is_last,
                       next_address=next_address, return_address=return_address, pipeline=pipe, replica=replica)


def load_node(path: str, node_id: str, replica: int = 0) -> NodeContext:
    return resolve_node(load_json(path), node_id, path, replica)


def banner(ctx: NodeContext, device: str) -> str:
    """Config banner (``node.py:280-290``), same lines."""
    return "\n".join([
        "--- Node Configuration ---",
        f"  ID: {ctx.node_id}",
        f"  Full Address (for clients): {ctx.address}",
        f"  Server Listening Port: {ctx.port}",
        f"  Part Index: {ctx.part_index} / {ctx.num_parts - 1}",
        f"  Is Last: {ctx.is_last}",
        f"  Next Node Address: {ctx.next_address}",
        f"  Return Node Addr: {ctx.return_address}",
        f"  Weights: {ctx.model_weights}",
        f"  Device: {device}",
        f"  Model: {ctx.pipeline.model}  Transport: {ctx.pipeline.transport}"
        + (f"  Replica: {ctx.replica} / {ctx.pipeline.replicas - 1}" if ctx.pipeline.replicas > 1 else ""),
        "-------------------------",
    ])
