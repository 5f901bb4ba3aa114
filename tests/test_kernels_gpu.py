"""HIP kernel numerics vs plain PyTorch fp32 references (MI355X only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 768), (77, 200, 128), (4096, 512, 4096),
                                   (1, 768, 768), (7, 3072, 768), (16, 50257, 768), (300, 2304, 768),
                                   (32, 4096, 14336), (64, 2304, 768), (40, 100, 128), (2, 28672, 4096)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_gemm_bf16(M, N, K, act):
    from distributed_neural_networks_amd.ops.gemm import linear
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    b = torch.randn(N, device=DEV)
    r = torch.randn(M, N, device=DEV).bfloat16()
    y = linear(x, w, b, act=act, residual=r)
    ref = x.float() @ w.float().t() + b
    if act == 1:
        ref = torch.relu(ref)
    elif act == 2:
        ref = torch.nn.functional.gelu(ref)
    ref = ref + r.float()
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 512, 4096), (300, 2304, 768), (1000, 520, 192),
                                   (2048, 768, 3072), (65, 300, 128)])
@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_gemm_bf16_256_tile(M, N, K, act):
    """The 256x256 4-phase GEMM (forced), including edge tiles and odd K-tile counts."""
    from distributed_neural_networks_amd.ops.gemm import linear, set_gemm_tile
    if act == 3 and N % 16:
        pytest.skip("packed gate|up needs N % 16 == 0")
    torch.manual_seed(2)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    b = torch.randn(N, device=DEV)
    set_gemm_tile(256)
    try:
        if act == 3:
            y = linear(x, w, act="silu_mul")
        else:
            r = torch.randn(M, N, device=DEV).bfloat16()
            y = linear(x, w, b, act=act, residual=r)
        torch.cuda.synchronize()
    finally:
        set_gemm_tile(0)
    ref = x.float() @ w.float().t()
    if act == 3:
        g = ref.view(M, N // 16, 2, 8)
        ref = (torch.nn.functional.silu(g[:, :, 0]) * g[:, :, 1]).reshape(M, N // 2)
    else:
        ref = ref + b
        ref = torch.relu(ref) if act == 1 else torch.nn.functional.gelu(ref) if act == 2 else ref
        ref = ref + r.float()
    assert _rel(y, ref) < 1e-2


def test_gemm_256_asymmetric_layout():
    from distributed_neural_networks_amd.ops.gemm import linear, set_gemm_tile
    n = 512
    x = torch.eye(n, device=DEV).bfloat16()
    w = torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n).remainder(97).bfloat16()
    set_gemm_tile(256)
    try:
        y = linear(x, w, out_dtype=torch.float32)
        torch.cuda.synchronize()
    finally:
        set_gemm_tile(0)
    assert torch.equal(y, w.float().t())


def test_gemm_asymmetric_layout():
    """A = I with an asymmetric W catches a transposed C write (guide §3)."""
    from distributed_neural_networks_amd.ops.gemm import linear
    n = 128
    x = torch.eye(n, device=DEV).bfloat16()
    w = torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n).remainder(97).bfloat16()
    y = linear(x, w, out_dtype=torch.float32)
    assert torch.equal(y, w.float().t())


@pytest.mark.parametrize("tile", [128, 256])
@pytest.mark.parametrize("n", [512, 520])
def test_gemm_asymmetric_layout_bf16(tile, n):
    """bf16 output takes the widened (permlane16-swapped, 16-B) store path; an
    identity A with an asymmetric W pins every column of the swapped layout,
    and n = 520 leaves a 32-column group that falls back to 8-B stores."""
    from distributed_neural_networks_amd.ops.gemm import linear, set_gemm_tile
    k = 512
    x = torch.eye(k, device=DEV).bfloat16()
    w = torch.arange(n * k, device=DEV, dtype=torch.float32).reshape(n, k).remainder(97).bfloat16()
    set_gemm_tile(tile)
    try:
        y = linear(x, w)
        torch.cuda.synchronize()
    finally:
        set_gemm_tile(0)
    assert y.dtype == torch.bfloat16
    assert torch.equal(y, w.t())


def test_gemm_gelu_erf_accuracy():
    """The branch-free erf GELU epilogue vs torch's exact-erf GELU, element-wise
    (identity A, fp32 out): |error| must stay far below one bf16 ulp."""
    from distributed_neural_networks_amd.ops.gemm import linear
    n = 256
    x = torch.eye(n, device=DEV).bfloat16()
    w = torch.linspace(-12, 12, n * n, device=DEV).reshape(n, n).bfloat16()
    y = linear(x, w, act=2, out_dtype=torch.float32)
    ref = torch.nn.functional.gelu(w.float().t())
    assert (y - ref).abs().max().item() < 2e-6 * 12


def test_gemm_silu_mul():
    from distributed_neural_networks_amd.ops.gemm import linear, pack_gate_up
    torch.manual_seed(1)
    for M in (1, 5, 31, 64, 65, 200):
        x = torch.randn(M, 256, device=DEV).bfloat16()
        g = (torch.randn(512, 256, device=DEV) * 0.05).bfloat16()
        u = (torch.randn(512, 256, device=DEV) * 0.05).bfloat16()
        y = linear(x, pack_gate_up(g, u), act="silu_mul")
        ref = torch.nn.functional.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
        assert y.shape == (M, 512)
        assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("B", [1, 3, 64, 1000])
def test_cifar_stage0_and_head(B):
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork, CifarStage
    from distributed_neural_networks_amd.ops import cifar as cops
    torch.manual_seed(0)
    model = NeuralNetwork().eval()
    sd = model.state_dict()
    x = torch.randn(B, 3, 32, 32)
    with torch.no_grad():
        ref_mid = CifarStage(0, 1).eval()
        ref_mid.load_state_dict(sd, strict=False)
        mid = ref_mid(x)
        ref_out = model(x)
    w0 = cops.pack_stage0(sd, DEV)
    wh = cops.pack_head(sd, DEV)
    h = cops.stage0_forward(x.to(DEV), w0)
    torch.cuda.synchronize()
    assert _rel(h.cpu(), mid) < 1e-2
    probs, pred = cops.head_forward(h, wh)
    torch.cuda.synchronize()
    assert (probs.cpu() - ref_out).abs().max().item() < 2e-2
    agree = (pred.cpu().long() == ref_out.argmax(1)).float().mean().item()
    assert agree > 0.9
    # argmax must be consistent with our own probabilities
    assert torch.equal(pred.cpu().long(), probs.cpu().argmax(1))


@pytest.mark.parametrize("variant", [1, 2, 3, 4])
def test_cifar_stage0_variants_agree(variant):
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork, CifarStage
    from distributed_neural_networks_amd.ops import cifar as cops
    torch.manual_seed(4)
    sd = NeuralNetwork().state_dict()
    w0 = cops.pack_stage0(sd, DEV)
    for B in (1, 5, 300, 4099):
        x = torch.randn(B, 3, 32, 32)
        ref = CifarStage(0, 1)
        ref.load_state_dict(sd, strict=False)
        with torch.no_grad():
            r = ref(x)
        h = cops.stage0_forward(x.to(DEV), w0, variant=variant)
        assert _rel(h.cpu(), r) < 1e-2, (variant, B)


@pytest.mark.parametrize("cut", [1, 2])
def test_cifar_stage_cuts(cut):
    """Both 2-stage cuts (reference conv|fc and the fc1 cut) reproduce the full model."""
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork
    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    from distributed_neural_networks_amd.runtime.stages import CifarHipStage
    torch.manual_seed(5)
    m = NeuralNetwork().eval()
    sd = m.state_dict()
    st = [CifarHipStage(sd, 0, cut, DEV), CifarHipStage(sd, cut + 1, 3, DEV)]
    x = torch.randn(64, 3, 32, 32)
    out = ColocatedPipeline(st, 64)(x.to(DEV))
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = m(x)
    assert (out.probs.cpu() - ref).abs().max().item() < 2e-2
    assert st[0].out_spec(8)[0] == (8, 4096 if cut == 1 else 512)
