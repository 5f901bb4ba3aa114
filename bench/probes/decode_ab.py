"""Interleaved in-process A/B of a decode-path switch (box-to-box clock
differences cancel): bench/gpt_bench.py runs alternately with each variant's
setting applied before the stages are built and captured.

    python bench/probes/decode_ab.py --switch skinny_max_m --values 32,64 [gpt_bench args...]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))


def apply(switch: str, v: int) -> None:
    from distributed_neural_networks_amd.ops import gemm
    from distributed_neural_networks_amd.ops._lib import lib
    if switch == "skinny_max_m":
        gemm.set_skinny_max_m(v)
    elif switch == "res_prefetch":
        lib().gemm_set_res_prefetch(v)
    elif switch == "fold_norm":
        gemm.FOLD_NORM_PREFILL = bool(v)
    elif switch == "kv8_u":  # fp8-KV decode attention rows in flight per thread (attention.hip KV8U)
        os.environ["DNN_KV8_U"] = str(v)
    elif switch == "qkv_scatter":  # prefill c_attn straight into q / the KV caches (ops/gemm.py QKV_SCATTER)
        gemm.QKV_SCATTER = bool(v)
    elif switch == "decode_splits":  # decode-attention split count (0 = the heuristic), read at stage build
        if v:
            os.environ["DNN_DECODE_SPLITS"] = str(v)
        else:
            os.environ.pop("DNN_DECODE_SPLITS", None)
    elif switch == "stream_fold":  # stream GEMM split-K combine: 1 in the launch, 0 separate reduce launch
        gemm.set_stream_gemm(1, 0, v)
    elif switch == "stream":  # decode stream GEMM: 0 off, 1 where it measured faster, 2 forced (gemm_stream.h)
        gemm.set_stream_gemm(v)
    elif switch == "decode_1p":  # one-pass decode attention: 0 batched kernel, 1 default, 2 forced (attention.hip)
        os.environ["DNN_DECODE_1P"] = str(v)
    elif switch == "decode_1p_kf":  # one-pass decode attention: K/V loads issued before q (attention.hip KF)
        os.environ["DNN_DECODE_1P_KF"] = str(v)
    elif switch == "flash_db":  # flash prefill with double-buffered K/V LDS (attention.hip DNN_FLASH_DB)
        os.environ["DNN_FLASH_DB"] = str(v)
    elif switch == "epi_pre":  # decode GEMM epilogue operands issued with the first loads (gemm_oneshot.h / skinny)
        lib().gemm_set_epi_prefetch(v)
    elif switch == "os_lds_floor":  # one-shot launch LDS floor in bytes (gemm_skinny.hip g_os_lds_floor; 0 = own size)
        lib().gemm_set_oneshot_lds_floor(v)
    elif switch == "flash_pipe":  # hd-64 flash prefill software pipeline (attention.hip DNN_FLASH_PIPE)
        os.environ["DNN_FLASH_PIPE"] = str(v)
    elif switch == "rowstats_r":  # prefill row statistics rows per wave (norm_embed.hip dnn_row_stats)
        os.environ["DNN_ROWSTATS_R"] = str(v)
    elif switch == "oneshot":  # one-shot decode GEMM: 0 off, 1 planned shapes, 2 every eligible shape
        gemm.set_oneshot_gemm(v)
    elif switch == "gemm_tile":  # prefill GEMM tile: 0 auto, 256, 255 (= 256x128), 128
        gemm.set_gemm_tile(v)
    elif switch == "half_cost":  # auto 256x128 rule: relative tile cost x 100
        gemm.set_gemm_half_cost(v / 100.0)
    elif switch == "decode_1p_ns":  # one-pass decode attention: at least v key splits (attention.hip)
        os.environ["DNN_DECODE_1P_NS"] = str(v)
    elif switch == "split_tail":  # prefill 256^2 + 256x128 tail split (gemm_bf16.hip): mask 1 bf16, 2 fp8
        gemm.set_gemm_split_tail(int(v))
    elif switch == "fused_head":  # decode head + argmax partials in one launch (gemm_head.h)
        gemm.set_fused_head(bool(v))
    elif switch == "mx_prefill":  # MX-scaled e4m3 prefill activations (ops/fp8.py MX_PREFILL)
        from distributed_neural_networks_amd.ops import fp8
        fp8.MX_PREFILL = bool(v)
    elif switch == "rowstats":  # producer-side decode row statistics (ops/gemm.py ROWSTATS)
        gemm.ROWSTATS = bool(v)
    elif switch == "multistep":  # K decode rounds per HIP graph (runtime/scheduler.py DecodeRing multi_step)
        os.environ["DNN_DECODE_MULTISTEP"] = str(v)
    elif switch == "skinny_pin":  # M 17..64 skinny config: v = id*1000 + ks*100 + shape (gemm_skinny.hip SkinnyPin)
        # shapes (N, K): 1 Llama-3 8B QKV, 2 its O projection, 3 its down projection (bypasses the stream plan),
        # 4 GPT-2 c_proj
        n, k = {0: (0, 0), 1: (6144, 4096), 2: (4096, 4096), 3: (4096, 14336), 4: (768, 3072)}[v % 100]
        assert lib().gemm_set_skinny_pin(v // 1000, (v // 100) % 10 or 4, n, k) == 0
    elif switch == "argmax_split":
        from distributed_neural_networks_amd.ops import transformer_ops
        transformer_ops.ARGMAX_SPLIT = bool(v)
    else:
        raise SystemExit(f"unknown switch {switch}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--switch", required=True)
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--rounds", type=int, default=2)
    a, rest = ap.parse_known_args()
    import gpt_bench
    vals = [int(v) for v in a.values.split(",")]
    res = {v: [] for v in vals}
    for _ in range(a.rounds):
        for v in vals:
            apply(a.switch, v)
            g = gpt_bench.run(gpt_bench.parse(rest))
            res[v].append((g["ms_per_step"], g["prefill_tokens_per_s"]))
            torch.cuda.empty_cache()
    out = {"switch": a.switch, "args": " ".join(rest)}
    for v in vals:
        out[f"{v}_decode_ms"] = min(r[0] for r in res[v])
        out[f"{v}_prefill_tok_s"] = max(r[1] for r in res[v])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
