"""Golden models, stage splits, checkpoint slicing/remap, partition math (CPU)."""
import os

import pytest
import torch
from hypothesis import given, settings, strategies as st

from distributed_neural_networks_amd import checkpoint as ckpt
from distributed_neural_networks_amd.models import build_golden_stage, cifar, default_ranges, gpt2, llama3, model_info
from distributed_neural_networks_amd.parallel.partition import balanced_ranges, even_ranges, resolve_ranges, validate_ranges


def test_cifar_split_equals_full():
    # reference property: ModelPart1(ModelPart0(x)) == NeuralNetwork(x)
    torch.manual_seed(0)
    full = cifar.NeuralNetwork().eval()
    sd = full.state_dict()
    x = torch.randn(5, 3, 32, 32)
    parts = []
    for a, b in cifar.stage_ranges(2):
        p = cifar.CifarStage(a, b).eval()
        missing, unexpected = p.load_state_dict(sd, strict=False)
        assert not missing
        parts.append(p)
    with torch.no_grad():
        assert torch.allclose(parts[1](parts[0](x)), full(x))
        for n in (1, 3, 4):
            h = x
            for a, b in cifar.stage_ranges(n):
                s = cifar.CifarStage(a, b)
                s.load_state_dict(sd, strict=False)
                h = s(h)
            assert torch.allclose(h, full(x), atol=1e-6)


def test_cifar_keys_match_reference_layout():
    sd = cifar.NeuralNetwork().state_dict()
    assert {k: tuple(v.shape) for k, v in sd.items()} == {
        "conv1.weight": (32, 3, 3, 3), "conv1.bias": (32,), "conv2.weight": (64, 32, 3, 3), "conv2.bias": (64,),
        "fc1.weight": (512, 4096), "fc1.bias": (512,), "fc2.weight": (10, 512), "fc2.bias": (10,)}
    assert sum(v.numel() for v in sd.values()) == 2122186


def _gpt_full_sd(name, seed=0):
    torch.manual_seed(seed)
    m = gpt2.GPT(gpt2.GPT_CONFIGS[name]).eval()
    return m, m.state_dict()


def test_gpt2_stages_equal_full_model():
    m, sd = _gpt_full_sd("gpt2-tiny")
    ids = torch.randint(0, 512, (2, 20))
    ranges = default_ranges("gpt2-tiny", 3)
    validate_ranges(ranges, 4)
    with torch.no_grad():
        h = ids
        for i, (a, b) in enumerate(ranges):
            ssd = ckpt.stage_state_dict("gpt2-tiny", sd, a, b, i == 0, i == len(ranges) - 1)
            s = build_golden_stage("gpt2-tiny", a, b, i == 0, i == len(ranges) - 1)
            s.load_state_dict(ssd)
            h = s(h)
        assert torch.allclose(h, m(ids), atol=1e-5)


def test_gpt2_hf_conv1d_layout_and_tying(tmp_path):
    m, sd = _gpt_full_sd("gpt2-tiny", 1)
    hf = {}
    for k, v in sd.items():
        if k == "lm_head.weight":
            continue  # HF GPT2Model checkpoints omit the tied head
        k2 = k.replace("transformer.", "")
        if any(k.endswith(s) for s in ("c_attn.weight", "c_proj.weight", "c_fc.weight")):
            v = v.t().contiguous()  # Conv1D stores (in, out)
        hf[k2] = v
    p = tmp_path / "hf.pth"
    torch.save(hf, p)
    full = ckpt.load_full_state_dict(str(p))
    ssd = ckpt.stage_state_dict("gpt2-tiny", full, 0, 3, True, True)
    s = build_golden_stage("gpt2-tiny", 0, 3, True, True)
    s.load_state_dict(ssd)
    ids = torch.randint(0, 512, (1, 9))
    with torch.no_grad():
        assert torch.allclose(s(ids), m(ids), atol=1e-5)


def test_nanogpt_ckpt_dict_and_orig_mod(tmp_path):
    m, sd = _gpt_full_sd("gpt2-tiny", 2)
    p = tmp_path / "ckpt.pt"
    torch.save({"model": {"_orig_mod." + k: v for k, v in sd.items()}, "iter_num": 5}, p)
    full = ckpt.load_full_state_dict(str(p))
    assert "transformer.wte.weight" in full


def test_missing_key_fails_loudly():
    _, sd = _gpt_full_sd("gpt2-tiny", 3)
    del sd["transformer.h.2.mlp.c_fc.weight"]
    with pytest.raises(ckpt.CheckpointError, match="transformer.h.2.mlp.c_fc.weight"):
        ckpt.stage_state_dict("gpt2-tiny", sd, 2, 3, False, True)


def test_gpt2_kv_cache_matches_recompute():
    m, sd = _gpt_full_sd("gpt2-tiny", 4)
    s = build_golden_stage("gpt2-tiny", 0, 3, True, True)
    s.load_state_dict(ckpt.stage_state_dict("gpt2-tiny", sd, 0, 3, True, True))
    ids = torch.randint(0, 512, (2, 12))
    cfg = gpt2.GPT_CONFIGS["gpt2-tiny"]
    kv = [(torch.zeros(2, cfg.n_head, 32, cfg.head_dim), torch.zeros(2, cfg.n_head, 32, cfg.head_dim)) for _ in range(4)]
    with torch.no_grad():
        out1 = s(ids[:, :8], kv, 0)
        out2 = s(ids[:, 8:], kv, 8)
        ref = m(ids)
    assert torch.allclose(torch.cat([out1, out2], 1), ref, atol=1e-4)


def test_llama_stages_and_cache():
    name = "llama3-tiny"
    n = model_info(name).num_layers
    sd_full = {}
    for i, (a, b) in enumerate([(0, n - 1)]):
        sd_full = ckpt.random_stage_state_dict(name, a, b, True, True, 9)
    whole = build_golden_stage(name, 0, n - 1, True, True)
    whole.load_state_dict(sd_full)
    km = llama3.stage_key_map(llama3.LLAMA_CONFIGS[name], 0, n - 1, True, True)
    full = {km[k]: v for k, v in sd_full.items()}
    ids = torch.randint(0, 512, (2, 10))
    with torch.no_grad():
        ref = whole(ids)
        h = ids
        for i, (a, b) in enumerate(default_ranges(name, 2)):
            s = build_golden_stage(name, a, b, i == 0, i == 1)
            s.load_state_dict(ckpt.stage_state_dict(name, full, a, b, i == 0, i == 1))
            h = s(h)
        assert torch.allclose(h, ref, atol=1e-4)
        cfg = llama3.LLAMA_CONFIGS[name]
        kv = [(torch.zeros(2, cfg.n_kv_head, 16, cfg.head_dim), torch.zeros(2, cfg.n_kv_head, 16, cfg.head_dim))
              for _ in range(n)]
        o1 = whole(ids[:, :6], kv, 0)
        o2 = whole(ids[:, 6:], kv, 6)
        assert torch.allclose(torch.cat([o1, o2], 1), ref, atol=1e-4)


def test_random_stage_weights_consistent_across_splits():
    # slicing a random model per stage == the same layers generated for a different split
    a = ckpt.random_stage_state_dict("gpt2-tiny", 0, 1, True, False, 5)
    b = ckpt.random_stage_state_dict("gpt2-tiny", 1, 3, False, True, 5)
    assert torch.equal(a["h.1.attn.c_attn.weight"], b["h.0.attn.c_attn.weight"])
    full = ckpt.random_stage_state_dict("gpt2-tiny", 0, 3, True, True, 5)
    assert torch.equal(full["lm_head.weight"], full["wte.weight"])
    assert torch.equal(b["lm_head.weight"], a["wte.weight"])


def test_make_checkpoint_roundtrip(tmp_path):
    p = tmp_path / "c.pth"
    ckpt.make_full_checkpoint("cifar10", str(p), 0)
    sd = ckpt.load_full_state_dict(str(p))
    assert set(sd) == set(cifar.NeuralNetwork().state_dict())
    p2 = tmp_path / "g.pth"
    ckpt.make_full_checkpoint("gpt2-tiny", str(p2), 0)
    sd2 = ckpt.load_full_state_dict(str(p2))
    assert "transformer.h.3.mlp.c_proj.weight" in sd2 and "lm_head.weight" in sd2


def test_safetensors_lazy(tmp_path):
    from safetensors.torch import save_file
    sd = ckpt.random_stage_state_dict("llama3-tiny", 0, 3, True, True, 1)
    km = llama3.stage_key_map(llama3.LLAMA_CONFIGS["llama3-tiny"], 0, 3, True, True)
    save_file({km[k]: v.contiguous() for k, v in sd.items()}, str(tmp_path / "model.safetensors"))
    full = ckpt.load_full_state_dict(str(tmp_path))
    st2 = ckpt.stage_state_dict("llama3-tiny", full, 2, 3, False, True)
    assert torch.equal(st2["layers.0.mlp.up_proj.weight"], sd["layers.2.mlp.up_proj.weight"])


@settings(max_examples=60, deadline=None)
@given(L=st.integers(1, 64), S=st.integers(1, 16), fe=st.floats(0, 3), le=st.floats(0, 3))
def test_partition_properties(L, S, fe, le):
    if S > L:
        with pytest.raises(ValueError):
            balanced_ranges(L, S)
        return
    r = balanced_ranges(L, S, fe, le)
    validate_ranges(r, L)
    e = even_ranges(L, S)
    validate_ranges(e, L)
    cost = lambda rr: max((b - a + 1) + (fe if i == 0 else 0) + (le if i == S - 1 else 0) for i, (a, b) in enumerate(rr))
    assert cost(r) <= cost(e) + 1e-9


def test_resolve_ranges_given():
    assert resolve_ranges(12, 3, [(0, 3), (4, 7), (8, 11)]) == [(0, 3), (4, 7), (8, 11)]
    with pytest.raises(ValueError):
        resolve_ranges(12, 3, [(0, 3), (5, 7), (8, 11)])
    with pytest.raises(ValueError):
        resolve_ranges(12, 3, [(0, 3), None, (8, 11)])


def test_default_ranges_gpt2_head_balancing():
    r = default_ranges("gpt2", 4)
    validate_ranges(r, 12)
    assert r[-1][1] - r[-1][0] + 1 <= r[0][1] - r[0][0] + 1  # last stage (lm_head) gets no more layers
