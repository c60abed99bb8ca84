"""The 256x256 LDS-DMA GEMM (gemm256.hip) pinned with nrse_gemm_select(3): every operand layout,
ragged M/N/K tails, z-batching, K segments + split-K atomics and each fused epilogue, against a
float64 reference of the bf16-rounded operands (and, for the hashed dropout, against the 128x128
kernel, whose mask is the same function of the output offset)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.double(); b = b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(params=[256, 224], ids=["gen3_bm256", "gen3_bm224"])
def gen3(nrse_device, request):
    """The 256-column kernel generation (gemm256.hip) at each tile height."""
    from nrse_amd import kernels as K
    old = K.gemm_select(3)
    old_rows = K.gemm_tile_rows(request.param)
    K.current_gen = 3
    yield K
    K.gemm_select(old)
    K.gemm_tile_rows(old_rows)


def bf(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("akc", [True, False])
@pytest.mark.parametrize("bkc", [True, False])
@pytest.mark.parametrize("shape", [(304, 264, 200), (520, 1000, 1032), (256, 256, 64), (1304, 136, 520),
                                   (672, 264, 136), (232, 520, 96)])
def test_layouts_and_tails(gen3, nrse_device, akc, bkc, shape):
    K = gen3
    M, N, Kd = shape
    dev = nrse_device
    a, b = bf(M, Kd, dev=dev), bf(N, Kd, dev=dev)
    A = K.Operand(a, True, Kd) if akc else K.Operand(a.t().contiguous(), False, M)
    B = K.Operand(b, True, Kd) if bkc else K.Operand(b.t().contiguous(), False, N)
    c = torch.full((M, N), 7.0, device=dev)
    K.gemm(A, B, c, M, N, Kd, ldc=N)
    assert rel(c, a.double() @ b.double().t()) < 1e-5


def test_epilogue_bias_gelu_resid_bf16_out(gen3, nrse_device):
    K = gen3
    from nrse_amd import _lib
    dev = nrse_device
    M, N, Kd = 700, 520, 384
    x, w = bf(M, Kd, dev=dev), bf(N, Kd, dev=dev, scale=0.05)
    bias = torch.randn(N, device=dev)
    r = bf(M, N, dev=dev)
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.linear_fwd(x, w, out, bias=bias, flags=_lib.EPI_GELU | _lib.EPI_RESID, aux=pre, ldaux=N, resid=r, ldr=N)
    ref_pre = x.double() @ w.double().t() + bias.double()
    assert rel(pre, ref_pre) < 4e-3
    assert rel(out, F.gelu(ref_pre) + r.double()) < 4e-3


def test_epilogue_gelu_bwd_accum(gen3, nrse_device):
    K = gen3
    from nrse_amd import _lib
    dev = nrse_device
    M, N, Kd = 600, 264, 512
    dy, w = bf(M, Kd, dev=dev), bf(N, Kd, dev=dev)
    pre = bf(M, N, dev=dev)
    c0 = torch.randn(M, N, device=dev)
    c = c0.clone()
    K.gemm(K.Operand(dy, True, Kd), K.Operand(w, True, Kd), c, M, N, Kd, ldc=N,
           flags=_lib.EPI_GELU_BWD | _lib.EPI_ACCUM, aux=pre, ldaux=N)
    p = pre.double()
    gp = 0.5 * (1 + torch.erf(p / 2 ** 0.5)) + p * torch.exp(-0.5 * p * p) / (2 * torch.pi) ** 0.5
    assert rel(c, c0.double() + (dy.double() @ w.double().t()) * gp) < 1e-5


@pytest.mark.parametrize("after", [False, True])
def test_epilogue_dropout_matches_128_kernel(gen3, nrse_device, after):
    K = gen3
    from nrse_amd import _lib
    dev = nrse_device
    M, N, Kd = 640, 512, 256
    x, w = bf(M, Kd, dev=dev), bf(N, Kd, dev=dev)
    r = torch.randn(M, N, device=dev)
    flags = _lib.EPI_RESID | (_lib.EPI_DROP_AFTER if after else 0)
    outs = []
    for g in (K.current_gen, 2):
        K.gemm_select(g)
        c = torch.empty(M, N, device=dev)
        K.gemm(K.Operand(x, True, Kd), K.Operand(w, True, Kd), c, M, N, Kd, ldc=N, flags=flags, resid=r, ldr=N,
               dropout_p=0.2, seed=1234)
        outs.append(c)
    K.gemm_select(K.current_gen)
    assert torch.equal(outs[0] == 0, outs[1] == 0)
    assert rel(outs[0], outs[1]) < 1e-6
    dropped = (outs[0] == 0) if after else (outs[0] - r == 0)
    assert 0.17 < float(dropped.float().mean()) < 0.23


def test_epilogue_colsum(gen3, nrse_device):
    K = gen3
    dev = nrse_device
    M, N, Kd = 900, 328, 200
    x, w = bf(M, Kd, dev=dev), bf(N, Kd, dev=dev)
    c = torch.empty(M, N, device=dev)
    cs = torch.zeros(N, device=dev)
    K.gemm(K.Operand(x, True, Kd), K.Operand(w, True, Kd), c, M, N, Kd, ldc=N, colsum=cs)
    ref = x.double() @ w.double().t()
    assert rel(c, ref) < 1e-5
    assert rel(cs, ref.sum(0)) < 1e-5


@pytest.mark.parametrize("bkc", [True, False])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_epilogue_gelu_bwd_dropout_colsum(gen3, nrse_device, out_dtype, bkc):
    """The FFN output-dense dgrad epilogue of the step (GELU' from the bf16 pre-activation, the
    activation-dropout mask, the intermediate bias gradient as column sums), against the 128x128
    kernel on the same operands: same dropped elements, same values, same column sums (the
    256-column register epilogue sums the values as stored, so bf16-rounded for bf16 output)."""
    K = gen3
    from nrse_amd import _lib
    dev = nrse_device
    M, N, Kd = 700, 520, 384
    dy, w = bf(M, Kd, dev=dev), bf(N, Kd, dev=dev)
    pre = bf(M, N, dev=dev)
    outs, sums = [], []
    for g in (K.current_gen, 2):
        K.gemm_select(g)
        c = torch.empty(M, N, device=dev, dtype=out_dtype)
        cs = torch.zeros(N, device=dev)
        B = K.Operand(w, True, Kd) if bkc else K.Operand(w.t().contiguous(), False, N)
        K.gemm(K.Operand(dy, True, Kd), B, c, M, N, Kd, ldc=N, flags=_lib.EPI_GELU_BWD,
               aux=pre, ldaux=N, dropout_p=0.1, seed=77, colsum=cs)
        outs.append(c)
        sums.append(cs)
    K.gemm_select(K.current_gen)
    assert torch.equal(outs[0] == 0, outs[1] == 0)
    tol = 1e-5 if out_dtype == torch.float32 else 4e-3
    assert rel(outs[0], outs[1]) < tol
    assert rel(sums[0], sums[1]) < tol
    assert rel(sums[0], outs[0].double().sum(0)) < tol


@pytest.mark.parametrize("splits", [1, 3])
def test_wgrad_segments_split_atomic(gen3, nrse_device, splits):
    """dW[out, in] = dY^T X over a token axis cut into segments, split-K with atomics."""
    K = gen3
    from nrse_amd import _lib
    dev = nrse_device
    R, Nout, Kin = 3 * 1040, 520, 264
    dy, x = bf(R, Nout, dev=dev), bf(R, Kin, dev=dev)
    nseg = 2
    seg_rows = R // (splits * nseg)
    dw = torch.zeros(Nout, Kin, device=dev)
    K.gemm(K.Operand(dy, False, Nout, seg_stride=seg_rows * Nout), K.Operand(x, False, Kin, seg_stride=seg_rows * Kin),
           dw, Nout, Kin, seg_rows, ldc=Kin, nseg=nseg, splits=splits, flags=_lib.EPI_ATOMIC)
    assert rel(dw, dy.double().t() @ x.double()) < 1e-5


def test_conv_implicit_batched(gen3, nrse_device):
    K = gen3
    dev = nrse_device
    B, Tin, C, k, s = 3, 601, 256, 3, 2
    Tout = (Tin - k) // s + 1
    x = bf(B, Tin, C, dev=dev)
    w = bf(C, C, k, dev=dev, scale=0.1)
    wr = w.permute(0, 2, 1).contiguous()
    y = torch.empty(B, Tout, C, device=dev)
    K.gemm(K.Operand(x, True, s * C, z1=Tin * C), K.Operand(wr, True, k * C), y, Tout, C, k * C,
           ldc=C, batch=B, c_z1=Tout * C)
    ref = F.conv1d(x.double().transpose(1, 2), w.double(), stride=s).transpose(1, 2)
    assert rel(y, ref) < 1e-5


def test_step_shapes_agree_with_128_kernel(gen3, nrse_device):
    """The WavLM-Large FFN shape, both kernels, same operands."""
    K = gen3
    dev = nrse_device
    M, N, Kd = 12768, 4096, 1024
    x, w = bf(M, Kd, dev=dev), bf(N, Kd, dev=dev, scale=0.03)
    outs = []
    for g in (K.current_gen, 2):
        K.gemm_select(g)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        K.gemm(K.Operand(x, True, Kd), K.Operand(w, True, Kd), c, M, N, Kd, ldc=N)
        outs.append(c.float())
    K.gemm_select(K.current_gen)
    assert rel(outs[0], outs[1]) < 5e-3
    idx = torch.randint(0, M, (64,), device=dev)
    assert rel(outs[0][idx], x[idx].double() @ w.double().t()) < 4e-3


def test_many_tiles_per_workgroup_tails_batched(gen3, nrse_device):
    """More tiles than CUs (several waves of workgroups), ragged M / N / K, a z-batch and the bias +
    GELU + residual epilogue."""
    K = gen3
    from nrse_amd import _lib
    dev = nrse_device
    Z, M, N, Kd = 2, 2100, 4104, 200
    x = bf(Z, M, Kd, dev=dev)
    w = bf(Z, N, Kd, dev=dev, scale=0.1)
    bias = torch.randn(N, device=dev)
    r = torch.randn(Z, M, N, device=dev)
    pre = torch.empty(Z, M, N, device=dev, dtype=torch.bfloat16)
    c = torch.empty(Z, M, N, device=dev)
    K.gemm(K.Operand(x, True, Kd, z1=M * Kd), K.Operand(w, True, Kd, z1=N * Kd), c, M, N, Kd, ldc=N, batch=Z,
           c_z1=M * N, bias=bias, flags=_lib.EPI_GELU, aux=pre, ldaux=N, aux_z1=M * N, resid=r, ldr=N, r_z1=M * N)
    ref_pre = torch.einsum("zmk,znk->zmn", x.double(), w.double()) + bias.double()
    assert rel(pre, ref_pre) < 4e-3
    assert rel(c, F.gelu(ref_pre) + r.double()) < 1e-5
