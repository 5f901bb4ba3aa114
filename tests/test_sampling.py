"""Sampler (temperature + top-k Gumbel-max): CPU mirror properties, and the
device kernel against the mirror (GPU)."""
import pytest
import torch

from distributed_neural_networks_amd.runtime.sampling import pick, sample_topk_ref


def test_topk1_and_cold_temperature_are_greedy():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(64, 1000, generator=g).bfloat16()
    greedy = x.float().argmax(1).to(torch.int32)
    assert torch.equal(sample_topk_ref(x, 1.0, top_k=1, seed=5), greedy)
    assert torch.equal(sample_topk_ref(x, 1e-4, top_k=0, seed=5), greedy)
    assert torch.equal(pick(x.float(), 0.0), greedy)


def test_topk_support():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(256, 500, generator=g).bfloat16()
    k = 7
    ids = sample_topk_ref(x, 2.0, top_k=k, seed=3, step=torch.arange(256, dtype=torch.int32))
    kth = x.float().topk(k, dim=1).values[:, -1]  # ties at the k-th value are all eligible
    assert bool((x.float().gather(1, ids[:, None].long())[:, 0] >= kth).all())


def test_frequencies_follow_softmax():
    """Many independent draws (distinct steps) of one row reproduce softmax(x/T)."""
    x = torch.tensor([[2.0, 1.0, 0.5, 0.0, -1.0, -3.0]]).bfloat16()
    n = 20000
    rows = x.repeat(n, 1)
    ids = sample_topk_ref(rows, 0.8, top_k=0, seed=11, step=torch.arange(n, dtype=torch.int32))
    freq = torch.bincount(ids.long(), minlength=6).float() / n
    p = torch.softmax(x.float()[0] / 0.8, 0)
    assert (freq - p).abs().max().item() < 0.015
    # top-k renormalises over the k largest
    ids3 = sample_topk_ref(rows, 0.8, top_k=3, seed=11, step=torch.arange(n, dtype=torch.int32))
    f3 = torch.bincount(ids3.long(), minlength=6).float() / n
    p3 = torch.softmax(x.float()[0, :3] / 0.8, 0)
    assert (f3[:3] - p3).abs().max().item() < 0.015 and f3[3:].sum().item() == 0


def test_reproducible_and_step_dependent():
    x = torch.randn(8, 300).bfloat16()
    a = sample_topk_ref(x, 1.0, 50, seed=9, step=torch.zeros(8, dtype=torch.int32))
    b = sample_topk_ref(x, 1.0, 50, seed=9, step=torch.zeros(8, dtype=torch.int32))
    c = sample_topk_ref(x, 1.0, 50, seed=9, step=torch.ones(8, dtype=torch.int32))
    assert torch.equal(a, b)
    assert not torch.equal(a, c) or True  # may coincide; only reproducibility is a hard contract


@pytest.mark.gpu
@pytest.mark.parametrize("N,k,T", [(50257, 0, 1.0), (50257, 40, 0.7), (128256, 50, 1.3), (512, 8, 1.0),
                                   (128256, 0, 0.5)])
def test_device_sampler_matches_mirror(N, k, T):
    from distributed_neural_networks_amd.ops import transformer_ops as Tops
    torch.manual_seed(3)
    M = 48
    ld = -(-N // 64) * 64
    logits = (torch.randn(M, ld, device="cuda") * 3).bfloat16()
    step = torch.arange(M, device="cuda", dtype=torch.int32) * 7
    out = torch.empty(M, device="cuda", dtype=torch.int32)
    Tops.sample_topk(logits, out, N, T, k, seed=1234, step=step)
    ref = sample_topk_ref(logits[:, :N].float(), T, k, 1234, step)
    agree = (out.cpu() == ref).float().mean().item()
    assert agree >= 0.95, agree  # __logf vs log: rare near-ties may flip
    if k:
        lf = logits[:, :N].float().cpu()
        kth = lf.topk(k, dim=1).values[:, -1]
        assert bool((lf.gather(1, out.cpu()[:, None].long())[:, 0] >= kth).all())


@pytest.mark.gpu
def test_device_sampler_topk1_is_argmax():
    from distributed_neural_networks_amd.ops import transformer_ops as Tops
    x = torch.randn(16, 50304, device="cuda").bfloat16()
    out = torch.empty(16, device="cuda", dtype=torch.int32)
    Tops.sample_topk(x, out, 50257, 1.0, 1, seed=1)
    xf = x[:, :50257].float().cpu()
    # bf16 ties at the maximum are all eligible: the pick must be a maximiser
    assert torch.equal(xf.gather(1, out.cpu()[:, None].long())[:, 0], xf.max(1).values)
