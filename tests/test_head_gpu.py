"""Fused decode head (csrc/kernels/gemm_head.h, ops/gemm.py head_argmax):
logits of the folded-norm vocabulary projection plus the greedy argmax from
per-workgroup partials, against an fp32 torch golden of the same op and
against the unfused path (linear_norm + argmax_rows)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _setup(M, K, N, w8, rms=False, seed=0):
    from distributed_neural_networks_amd.ops.gemm import attach_shuffled, fold_norm
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = (3.0 + torch.randn(M, K, device=DEV, generator=g)).bfloat16()  # mean offset: the shifted statistics
    gamma = 1 + 0.1 * torch.randn(K, device=DEV, generator=g)
    beta = None if rms else 0.1 * torch.randn(K, device=DEV, generator=g)
    w = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    f = attach_shuffled(fold_norm(w, gamma, beta, None, rms, 1e-5, DEV, fp8=w8))
    xf = x.float()
    if rms:
        xn = xf * torch.rsqrt(xf.pow(2).mean(1, keepdim=True) + 1e-5) * gamma
    else:
        xn = torch.nn.functional.layer_norm(xf, (K,), gamma, beta, 1e-5)
    ref = xn @ w.t()
    return x, f, ref


@pytest.mark.parametrize("M,K,N,w8,rms", [
    (64, 768, 50257, False, False),   # GPT-2 head at the bench batch
    (1, 768, 50257, False, False),
    (17, 768, 50257, False, True),
    (64, 1600, 50257, True, False),   # GPT-2 XL fp8 head (two K passes)
    (33, 256, 512, False, False),     # gpt2-tiny
    (8, 256, 512, True, False),
    (64, 1280, 5000, False, False),   # two K passes, bf16
    (48, 1280, 4000, True, False),
    (16, 1024, 3000, False, False),   # every instantiated width: gpt2-medium / gpt2-xl bf16 / gpt2 fp8 / medium fp8
    (40, 1600, 3000, False, False),
    (24, 768, 3000, True, False),
    (64, 1024, 3000, True, True),
])
def test_head_matches_golden_and_unfused(M, K, N, w8, rms):
    from distributed_neural_networks_amd.ops import transformer_ops as T_
    from distributed_neural_networks_amd.ops.gemm import HEAD_PART_PER_ROW, head_argmax, linear_norm
    x, f, ref = _setup(M, K, N, w8, rms)
    ldc = (N + 7) // 8 * 8 + 8  # argmax_rows reads 16-B rows
    logits = torch.full((M, ldc), float("nan"), device=DEV, dtype=torch.bfloat16)
    part = torch.empty(2 * HEAD_PART_PER_ROW * M, dtype=torch.int32, device=DEV)
    out = torch.full((M,), -1, dtype=torch.int32, device=DEV)
    also = torch.full((M,), -1, dtype=torch.int32, device=DEV)
    adv = torch.arange(M, dtype=torch.int32, device=DEV)
    assert head_argmax(x, f, logits[:, :N], part, out, also, adv)
    torch.cuda.synchronize()
    lg = logits[:, :N].float()
    assert torch.isfinite(lg).all()
    assert torch.isnan(logits[:, N:].float()).all()  # nothing written past N
    err = ((lg - ref).norm() / ref.norm()).item()
    assert err < (3e-2 if w8 else 1e-2), err
    # the unfused path on the same weights
    l2 = torch.empty((M, N), device=DEV, dtype=torch.bfloat16)
    std = torch.empty((M, K), device=DEV, dtype=torch.bfloat16)
    ones = torch.ones(K, device=DEV)
    linear_norm(x, f, out=l2, std_buf=std, ones=ones)
    torch.cuda.synchronize()
    e2 = ((lg - l2.float()).norm() / l2.float().norm()).item()
    assert e2 < 5e-3, e2
    # argmax of the kernel's own rounded logits, ties -> first index; step tail
    want = lg.argmax(1).to(torch.int32)
    assert torch.equal(out, want)
    assert torch.equal(also, want)
    assert torch.equal(adv, torch.arange(M, dtype=torch.int32, device=DEV) + 1)
    # and argmax_rows over the same logits agrees
    o2 = torch.empty(M, dtype=torch.int32, device=DEV)
    T_.argmax_rows(logits[:, :N], o2, n=N)
    torch.cuda.synchronize()
    assert torch.equal(o2, out)


def test_head_ties_take_smallest_index():
    """Identical columns make exact ties across workgroups: the merge keeps the
    smallest index, as argmax_rows / numpy."""
    from distributed_neural_networks_amd.ops.gemm import HEAD_PART_PER_ROW, attach_shuffled, fold_norm, head_argmax
    M, K, N = 16, 768, 8192
    g = torch.Generator(device=DEV).manual_seed(3)
    w = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    best = torch.randn(1, K, device=DEV, generator=g)
    w[[7000, 123, 4096]] = best * 4  # the same (largest-norm) row three times
    f = attach_shuffled(fold_norm(w, torch.ones(K, device=DEV), torch.zeros(K, device=DEV), None, False, 1e-5, DEV))
    x = best.expand(M, K).contiguous().bfloat16()
    logits = torch.empty((M, N), device=DEV, dtype=torch.bfloat16)
    part = torch.empty(2 * HEAD_PART_PER_ROW * M, dtype=torch.int32, device=DEV)
    out = torch.empty(M, dtype=torch.int32, device=DEV)
    assert head_argmax(x, f, logits, part, out)
    torch.cuda.synchronize()
    assert (out == 123).all(), out


def test_head_declines_uncovered_shapes():
    """Shapes outside the instantiated set return False without launching."""
    from distributed_neural_networks_amd.ops.gemm import HEAD_PART_PER_ROW, head_argmax
    part = torch.empty(2 * HEAD_PART_PER_ROW * 65, dtype=torch.int32, device=DEV)
    out = torch.empty(65, dtype=torch.int32, device=DEV)
    x, f, _ = _setup(65, 768, 1024, False)  # 65 rows
    assert not head_argmax(x, f, torch.empty((65, 1024), device=DEV, dtype=torch.bfloat16), part, out)
    x, f, _ = _setup(8, 4096, 1024, False, rms=True, seed=1)  # Llama width: no config
    assert not head_argmax(x, f, torch.empty((8, 1024), device=DEV, dtype=torch.bfloat16), part, out)


def test_head_switch_matches_decode_tokens():
    """GPT-2 tiny, 2 stages on the decode ring (HIP graphs), greedy
    generation: the fused head and the unfused head give the same tokens."""
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.models import model_info
    from distributed_neural_networks_amd.ops import gemm
    from distributed_neural_networks_amd.runtime.scheduler import DecodeRing, RingLinks
    from distributed_neural_networks_amd.runtime.transformer import TransformerStage
    model = "gpt2-tiny"
    n = model_info(model).num_layers
    ranges = [(0, n // 2 - 1), (n // 2, n - 1)]
    sds = [ckpt.random_stage_state_dict(model, a, b, i == 0, i == 1, 7, nontrivial=True)
           for i, (a, b) in enumerate(ranges)]
    prompt = torch.randint(0, model_info(model).cfg.vocab_size, (8, 12), generator=torch.Generator().manual_seed(5))
    toks = {}
    try:
        for on in (True, False):
            gemm.set_fused_head(on)
            stages = [TransformerStage(model, sds[i], a, b, i == 0, i == 1, DEV, max_batch=8, max_seq=32)
                      for i, (a, b) in enumerate(ranges)]
            toks[on] = DecodeRing(stages, RingLinks(), 1, 1, 8).generate([prompt], 12, 8)
            torch.cuda.synchronize()
    finally:
        gemm.set_fused_head(True)
    assert torch.equal(toks[True], toks[False]), (toks[True], toks[False])
