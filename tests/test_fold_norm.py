"""CPU check of the norm-folding algebra used by the fused pre-norm GEMMs
(ops/gemm.py fold_norm): rstd * (x W'^T - mean colsum) + bias' must equal
linear(norm(x)) for LayerNorm and RMSNorm."""
import torch
import torch.nn.functional as F

from distributed_neural_networks_amd.ops.gemm import NORM_LN, NORM_RMS, fold_norm


def _apply(x, f):
    xf = x.double()
    K = xf.shape[1]
    if f.norm == NORM_LN:
        mean = xf.mean(1, keepdim=True)
        rstd = torch.rsqrt(xf.pow(2).mean(1, keepdim=True) - mean ** 2 + f.eps)
        y = rstd * (xf @ f.w.double().t() - mean * f.colsum.double()[None, :])
    else:
        rstd = torch.rsqrt(xf.pow(2).mean(1, keepdim=True) + f.eps)
        y = rstd * (xf @ f.w.double().t())
    if f.bias is not None:
        y = y + f.bias.double()
    assert K == f.w.shape[1]
    return y


def test_fold_layernorm():
    torch.manual_seed(0)
    K, N = 96, 40
    x = torch.randn(5, K) * 3 + 1
    g, b = torch.rand(K) + 0.5, torch.randn(K)
    W, bias = torch.randn(N, K) / 10, torch.randn(N)
    f = fold_norm(W, g, b, bias, False, 1e-5, "cpu")
    assert f.norm == NORM_LN and f.colsum is not None
    ref = F.layer_norm(x.double(), (K,), g.double(), b.double(), 1e-5) @ W.double().t() + bias.double()
    assert torch.allclose(_apply(x, f), ref, rtol=2e-2, atol=2e-2)  # bf16 folded weight


def test_fold_rmsnorm():
    torch.manual_seed(1)
    K, N = 64, 48
    x = torch.randn(3, K)
    g = torch.rand(K) + 0.5
    W = torch.randn(N, K) / 8
    f = fold_norm(W, g, None, None, True, 1e-6, "cpu")
    assert f.norm == NORM_RMS and f.colsum is None and f.bias is None
    xd = x.double()
    ref = (xd * torch.rsqrt(xd.pow(2).mean(1, keepdim=True) + 1e-6) * g.double()) @ W.double().t()
    assert torch.allclose(_apply(x, f), ref, rtol=2e-2, atol=2e-2)
