"""HIP kernel numerics vs plain PyTorch fp32 references (MI355X only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 768), (77, 200, 128), (4096, 512, 4096),
                                   (1, 768, 768), (7, 3072, 768), (16, 50257, 768), (300, 2304, 768),
                                   (32, 4096, 14336), (64, 2304, 768), (40, 100, 128), (2, 28672, 4096),
                                   (128, 768, 768), (200, 2304, 768), (256, 3072, 768), (97, 768, 3072)])
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
@pytest.mark.parametrize("tile", [256, 255])
def test_gemm_bf16_256_tile(M, N, K, act, tile):
    """The 256x256 4-phase GEMM and its 256x128 2-phase variant (tile 255),
    forced, including edge tiles and odd K-tile counts."""
    from distributed_neural_networks_amd.ops.gemm import linear, set_gemm_tile
    if act == 3 and N % 16:
        pytest.skip("packed gate|up needs N % 16 == 0")
    torch.manual_seed(2)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    b = torch.randn(N, device=DEV)
    set_gemm_tile(tile)
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


@pytest.mark.parametrize("M,N,K", [(4400, 4208, 192), (4352, 4352, 768), (8192, 768, 768)])
@pytest.mark.parametrize("epi", ["res", "gelu", "silu_mul", "norm"])
@pytest.mark.parametrize("tile", [256, 255])
def test_gemm_bf16_256_many_tiles(M, N, K, epi, tile):
    """More 256^2 tiles than CUs (several waves of workgroups, edge tiles, odd
    K-tile counts) with every prefill epilogue, incl. the folded pre-norm, vs fp32."""
    from distributed_neural_networks_amd.ops.gemm import linear, set_gemm_tile
    torch.manual_seed(3)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    b = torch.randn(N, device=DEV)
    r = torch.randn(M, N, device=DEV).bfloat16()
    rowstat = colsum = None
    if epi == "norm":  # folded pre-norm epilogue: v = rstd acc - mean rstd colsum
        mean, rstd = torch.randn(M, device=DEV), torch.rand(M, device=DEV) + 0.5
        rowstat = torch.stack([rstd, -mean * rstd], 1).contiguous()
        colsum = torch.randn(N, device=DEV)
    set_gemm_tile(tile)
    try:
        if epi == "silu_mul":
            y = linear(x, w, act="silu_mul")
        elif epi == "gelu":
            y = linear(x, w, b, act="gelu")
        elif epi == "res":
            y = linear(x, w, b, residual=r)
        else:
            y = linear(x, w, b, rowstat=rowstat, colsum=colsum)
        torch.cuda.synchronize()
    finally:
        set_gemm_tile(0)
    ref = x.float() @ w.float().t()
    if epi == "silu_mul":
        g = ref.view(M, N // 16, 2, 8)
        ref = (torch.nn.functional.silu(g[:, :, 0]) * g[:, :, 1]).reshape(M, N // 2)
    elif epi == "gelu":
        ref = torch.nn.functional.gelu(ref + b)
    elif epi == "res":
        ref = ref + b + r.float()
    else:
        ref = ref * rowstat[:, :1] + rowstat[:, 1:] * colsum + b
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(4400, 1536, 192), (300, 768, 768), (513, 2304, 3072)])
@pytest.mark.parametrize("dtype", ["bf16", "fp8mx"])
@pytest.mark.parametrize("tile", [256, 255])
def test_gemm_256_residual_tile_dma_bit_identical(M, N, K, dtype, tile):
    """The 256^2 / 256x128 residual epilogue with its residual tile moved by
    LDS-DMA (gemm_epilogue.h res_tile_dma, the default) writes exactly what the
    per-lane residual gathers wrote (anatomy bit 4), incl. partial M tiles."""
    from distributed_neural_networks_amd.ops._lib import lib, ptr, stream_ptr
    from distributed_neural_networks_amd.ops.gemm import linear, set_gemm_tile
    from distributed_neural_networks_amd.ops.fp8 import kpad_of, mx_scale_bytes, quant_rows_mx, quantize_weight
    torch.manual_seed(9)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    b = torch.randn(N, device=DEV)
    r = torch.randn(M, N, device=DEV).bfloat16()
    L = lib()
    if dtype == "fp8mx":
        if M < 256 or tile != 256:
            pytest.skip("the MX path: 256^2 tiles, M >= 256")
        wq = quantize_weight(w.float(), torch.device(DEV))
        kp = kpad_of(K)
        qb = torch.empty(M, kp, dtype=torch.uint8, device=DEV)
        sx = torch.empty(mx_scale_bytes(M, kp), dtype=torch.uint8, device=DEV)
        quant_rows_mx(x, qb, sx)

        def run():
            o = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            assert L.gemm_fp8_mx(ptr(qb), ptr(sx), ptr(wq.q), ptr(wq.scale), ptr(o), N, ptr(b), ptr(r), N, M, N, kp,
                                 0, 0, 0, 0, 0, stream_ptr()) == 0
            return o
    else:
        def run():
            return linear(x, w, b, residual=r)
    set_gemm_tile(tile)
    try:
        outs = []
        for bits in (4, 0):
            assert L.gemm_set_anatomy(bits) == 0
            outs.append(run())
            torch.cuda.synchronize()
    finally:
        L.gemm_set_anatomy(0)
        set_gemm_tile(0)
    assert torch.equal(outs[0], outs[1])
    ref = x.float() @ w.float().t() + b + r.float()
    assert _rel(outs[1], ref) < (5e-2 if dtype == "fp8mx" else 1e-2)


@pytest.mark.parametrize("tile", [256, 255])
def test_gemm_256_asymmetric_layout(tile):
    from distributed_neural_networks_amd.ops.gemm import linear, set_gemm_tile
    n = 512
    x = torch.eye(n, device=DEV).bfloat16()
    w = torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n).remainder(97).bfloat16()
    set_gemm_tile(tile)
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


@pytest.mark.parametrize("tile", [128, 256])
@pytest.mark.parametrize("M,N,K", [(300, 2048, 768), (1000, 528, 256), (4096, 1024, 512)])
def test_gemm_silu_mul_tiles(tile, M, N, K):
    """SwiGLU epilogue of the tiled GEMMs (paired-tile permlane32 exchange),
    forced 128^2 and 256^2, partial tiles included."""
    from distributed_neural_networks_amd.ops.gemm import linear, pack_gate_up, set_gemm_tile
    torch.manual_seed(5)
    x = torch.randn(M, K, device=DEV).bfloat16()
    g = (torch.randn(N // 2, K, device=DEV) * 0.05).bfloat16()
    u = (torch.randn(N // 2, K, device=DEV) * 0.05).bfloat16()
    set_gemm_tile(tile)
    try:
        y = linear(x, pack_gate_up(g, u), act="silu_mul")
        torch.cuda.synchronize()
    finally:
        set_gemm_tile(0)
    ref = torch.nn.functional.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
    assert y.shape == (M, N // 2)
    assert _rel(y, ref) < 1e-2


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


def _cifar_golden(seed, B):
    from distributed_neural_networks_amd.models.cifar import CifarStage, NeuralNetwork
    torch.manual_seed(seed)
    model = NeuralNetwork().eval()
    sd = model.state_dict()
    x = torch.randn(B, 3, 32, 32)
    with torch.no_grad():
        part0 = CifarStage(0, 1).eval()
        part0.load_state_dict(sd, strict=False)
        mid = part0(x)
        ref = model(x)
    return sd, x, mid, ref


@pytest.mark.parametrize("B", [1, 3, 64, 1000])
def test_cifar_stage0_and_head_bf16(B):
    from distributed_neural_networks_amd.ops import cifar as cops
    sd, x, mid, ref_out = _cifar_golden(0, B)
    w0 = cops.pack_stage0(sd, DEV, "bf16")
    wh = cops.pack_head(sd, DEV, precision="bf16")
    h = cops.stage0_forward(x.to(DEV), w0)
    torch.cuda.synchronize()
    assert h.dtype == torch.bfloat16
    assert _rel(h.cpu(), mid) < 1e-2
    probs, pred = cops.head_forward(h, wh)
    torch.cuda.synchronize()
    assert (probs.cpu() - ref_out).abs().max().item() < 2e-2
    assert (pred.cpu().long() == ref_out.argmax(1)).float().mean().item() > 0.9
    assert torch.equal(pred.cpu().long(), probs.cpu().argmax(1))


@pytest.mark.parametrize("B", [1, 3, 257, 1000])
def test_cifar_fp32_stage0_and_head(B):
    """fp32 path (3-term bf16 split on MFMA) against the fp32 torch stages."""
    from distributed_neural_networks_amd.ops import cifar as cops
    sd, x, mid, ref_out = _cifar_golden(1, B)
    w0 = cops.pack_stage0(sd, DEV)
    wh = cops.pack_head(sd, DEV)
    h = cops.stage0_forward(x.to(DEV), w0)
    torch.cuda.synchronize()
    assert h.dtype == torch.float32
    err = (h.cpu() - mid).abs().max().item()
    assert err <= 2e-5 * max(1.0, mid.abs().max().item()), err
    probs, pred = cops.head_forward(h, wh)
    torch.cuda.synchronize()
    assert (probs.cpu() - ref_out).abs().max().item() <= 1e-5
    assert torch.equal(pred.cpu().long(), probs.cpu().argmax(1))


@pytest.mark.parametrize("boundary", ["fp32", "split"])
def test_cifar_fp32_pipeline_4096_images_matches_reference(boundary):
    """Acceptance: the 2-stage pipeline at the reference's
    precision on 4096 images: max |dprob| <= 1e-5 vs fp32 torch
    (cifar_model_parts.py:7-26) and 100 % argmax agreement (rows whose golden
    top-2 probabilities tie within 1e-6 are excluded as numerically undecidable)."""
    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    from distributed_neural_networks_amd.runtime.stages import CifarHipStage
    sd, x, _, ref = _cifar_golden(2, 4096)
    st = [CifarHipStage(sd, 0, 1, DEV, boundary=boundary), CifarHipStage(sd, 2, 3, DEV, boundary=boundary)]
    assert st[0].out_spec(4) == ((4, 4096), torch.float32)
    out = ColocatedPipeline(st, 4096)(x.to(DEV))
    torch.cuda.synchronize()
    dp = (out.probs.cpu() - ref).abs().max().item()
    assert dp <= 1e-5, dp
    top2 = ref.topk(2, dim=1).values
    decidable = (top2[:, 0] - top2[:, 1]) > 1e-6
    agree = out.pred.cpu().long() == ref.argmax(1)
    assert bool(agree[decidable].all()), int((~agree[decidable]).sum())


@pytest.mark.parametrize("cut,precision", [(1, "fp32"), (2, "fp32"), (1, "bf16"), (2, "bf16")])
def test_cifar_stage_cuts(cut, precision):
    """Both 2-stage cuts (reference conv|fc and the fc1 cut) reproduce the full model."""
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork
    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    from distributed_neural_networks_amd.runtime.stages import CifarHipStage
    torch.manual_seed(5)
    m = NeuralNetwork().eval()
    sd = m.state_dict()
    st = [CifarHipStage(sd, 0, cut, DEV, precision), CifarHipStage(sd, cut + 1, 3, DEV, precision)]
    x = torch.randn(64, 3, 32, 32)
    out = ColocatedPipeline(st, 64)(x.to(DEV))
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = m(x)
    tol = 1e-5 if precision == "fp32" else 2e-2
    assert (out.probs.cpu() - ref).abs().max().item() < tol
    dt = torch.float32 if precision == "fp32" else torch.bfloat16
    assert st[0].out_spec(8) == ((8, 4096 if cut == 1 else 512), dt)


@pytest.mark.parametrize("split_in", [0, 1])
@pytest.mark.parametrize("M,N,K", [(300, 256, 64), (1000, 512, 4096), (16384 + 77, 512, 4096)])
def test_cifar_fc1_x3_kernel(M, N, K, split_in):
    """Fused fp32 fc1 (A split in registers while staging, or A in the blocked
    hi/lo encoding staged by DMA): relu(A W^T + b) vs fp32 torch, relative
    error at the ~2^-16 level of the 3-term split."""
    from distributed_neural_networks_amd.ops import _lib
    from distributed_neural_networks_amd.ops.cifar import encode_boundary, split_bf16
    torch.manual_seed(M)
    a = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) / K ** 0.5
    b = torch.randn(N, device=DEV) * 0.1
    wh, wl = split_bf16(w)
    out = torch.empty(M, N, device=DEV)
    a_in = encode_boundary(a) if split_in else a
    rc = _lib.lib().cifar_fc1_x3(a_in.data_ptr(), K, wh.data_ptr(), wl.data_ptr(), K, b.data_ptr(), out.data_ptr(),
                                 N, M, N, K, torch.cuda.current_stream().cuda_stream, split_in)
    assert rc == 0
    torch.cuda.synchronize()
    ref = torch.relu(a.double() @ w.double().t() + b.double())
    err = (out.double() - ref).abs().max().item()
    assert err <= 2e-5 * ref.abs().max().item(), err


@pytest.mark.parametrize("boundary", ["fp32", "split"])
def test_cifar_fp32_pipeline_large_batch_fused_fc1(boundary):
    """The large-batch fp32 head (fused fc1) on 20000 images: max |dprob| <= 1e-5
    vs the fp32 torch model and argmax agreement on every decidable row."""
    from distributed_neural_networks_amd.ops import cifar as cops
    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    from distributed_neural_networks_amd.runtime.stages import CifarHipStage
    B = 20000
    assert B >= cops.FC1_X3_MIN_ROWS
    sd, x, _, ref = _cifar_golden(3, B)
    st = [CifarHipStage(sd, 0, 1, DEV, boundary=boundary), CifarHipStage(sd, 2, 3, DEV, boundary=boundary)]
    out = ColocatedPipeline(st, B)(x.to(DEV))
    torch.cuda.synchronize()
    dp = (out.probs.cpu() - ref).abs().max().item()
    assert dp <= 1e-5, dp
    top2 = ref.topk(2, dim=1).values
    decidable = (top2[:, 0] - top2[:, 1]) > 1e-6
    agree = out.pred.cpu().long() == ref.argmax(1)
    assert bool(agree[decidable].all()), int((~agree[decidable]).sum())


@pytest.mark.parametrize("B", [1, 300, 16384 + 77])
def test_cifar_split_boundary_bit_identical(B):
    """The blocked hi/lo boundary encoding is exactly the split of the fp32
    boundary (stage-0 epilogue == encode of the fp32 output, bitwise), decodes
    to it within 2^-16, and the pipeline's probabilities and predictions are
    bitwise those of the fp32 boundary (small-batch split3 path and the fused
    fc1 path)."""
    from distributed_neural_networks_amd.ops import cifar as cops
    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    from distributed_neural_networks_amd.runtime.stages import CifarHipStage
    torch.manual_seed(B)
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork
    sd = NeuralNetwork().state_dict()
    x = torch.randn(B, 3, 32, 32, device=DEV)
    w0 = cops.pack_stage0(sd, DEV, "fp32")
    h32 = cops.stage0_forward(x, w0, boundary="fp32")
    hsp = cops.stage0_forward(x, w0, boundary="split")
    assert torch.equal(cops.encode_boundary(h32).view(torch.int32), hsp.view(torch.int32))
    back = cops.decode_boundary(hsp)
    assert ((back - h32).abs() <= h32.abs() * 2 ** -16).all()
    outs = {}
    for bd in ("fp32", "split"):
        st = [CifarHipStage(sd, 0, 1, DEV, boundary=bd), CifarHipStage(sd, 2, 3, DEV, boundary=bd)]
        o = ColocatedPipeline(st, B)(x)
        outs[bd] = (o.probs.clone(), o.pred.clone())
    torch.cuda.synchronize()
    assert torch.equal(outs["fp32"][0], outs["split"][0])
    assert torch.equal(outs["fp32"][1], outs["split"][1])


@pytest.mark.parametrize("K,act,res,fold", [(768, None, True, False), (3072, None, True, False),
                                            (768, "gelu", False, False), (768, None, False, True)])
def test_gemm_tail_split_matches_single_grid(K, act, res, fold):
    """GPT-2's 768-wide prefill projections at M = 32768 run as 256^2 tiles on
    the first 512 columns plus 256x128 tiles on the last 256 (two launches,
    disjoint columns): identical to the single 256^2 grid (same per-output
    MFMA order), with bias, residual, activation and the folded-norm epilogue,
    and close to fp32."""
    from distributed_neural_networks_amd.ops import transformer_ops as T
    from distributed_neural_networks_amd.ops.gemm import linear, set_gemm_split_tail, set_gemm_tile
    M, N = 32768, 768
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    w = (torch.randn(N, K, device=DEV, generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=DEV, generator=g) * 0.1
    r = torch.randn(M, N, device=DEV, generator=g).bfloat16() if res else None
    kw = {}
    if fold:
        st = torch.empty((M, 2), device=DEV, dtype=torch.float32)
        T.row_stats(x, st, 1e-5, False, rows=M, ldx=K)
        kw = dict(rowstat=st, colsum=w.float().sum(1).contiguous())
    outs = []
    try:
        for tile, split in ((0, True), (256, False)):
            set_gemm_tile(tile)
            set_gemm_split_tail(split)
            outs.append(linear(x, w, b, act, r, **kw))
            torch.cuda.synchronize()
    finally:
        set_gemm_tile(0)
        set_gemm_split_tail(True)
    assert torch.equal(outs[0], outs[1])
    xf = x.float()
    if fold:
        xf = torch.nn.functional.layer_norm(xf, (K,), eps=1e-5)
    ref = xf @ w.float().t() + b
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    if res:
        ref = ref + r.float()
    err = ((outs[0].float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("N,K,split,act,res", [(1600, 1600, True, 0, True), (6400, 1600, True, 2, False),
                                               (1600, 6400, False, 0, True), (4800, 1600, True, 0, False)])
def test_fp8_gemm_tail_split_matches_single_grid(N, K, split, act, res):
    """GPT-2 XL prefill shapes on the fp8 256^2 kernel at M = 32768: the grid's
    last column of tiles (64 / 256 / 192 wide) as 256x128 tiles in a second
    launch gives the single grid's bits (split activations or not, GELU,
    residual)."""
    from distributed_neural_networks_amd.ops.fp8 import attach_split, linear_fp8, quantize_weight
    from distributed_neural_networks_amd.ops.gemm import set_gemm_split_tail
    M = 32768
    g = torch.Generator(device=DEV).manual_seed(6)
    x = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    w = quantize_weight(torch.randn(N, K, device=DEV, generator=g) / K ** 0.5, DEV)
    if split:
        attach_split(w)
    b = torch.randn(N, device=DEV, generator=g) * 0.1
    r = torch.randn(M, N, device=DEV, generator=g).bfloat16() if res else None
    outs = []
    try:
        for mask in (3, 0):  # fp8 split on (off by default) / off
            set_gemm_split_tail(mask)
            outs.append(linear_fp8(x, w, b, act, r))
            torch.cuda.synchronize()
    finally:
        set_gemm_split_tail(True)
    assert torch.equal(outs[0], outs[1])
    ref = x.float() @ (w.q[:, :K].float() * w.scale[:, None]).t() + b
    if act == 2:
        ref = torch.nn.functional.gelu(ref)
    if res:
        ref = ref + r.float()
    err = ((outs[0].float() - ref).norm() / ref.norm()).item()
    assert err < (3e-2 if split else 8e-2), err
