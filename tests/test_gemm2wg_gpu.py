"""The two-workgroups-per-CU GEMM (gemm2wg.hip) pinned with nrse_gemm_select(5): k-contiguous
operands, ragged M / N / K tails at both tile heights (112 and 128 rows), z-batching, K segments
and each epilogue it instantiates, against a float64 reference of the bf16-rounded operands and,
for the hashed dropout, against the 128x128 kernel (the mask is a function of the output offset)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.double(); b = b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture
def gen5(nrse_device):
    from nrse_amd import kernels as K
    old = K.gemm_select(5)
    yield K
    K.gemm_select(old)


def bf(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("shape", [(304, 264, 200), (520, 1000, 1032), (256, 256, 64), (1304, 256, 520),
                                   (672, 264, 136), (128, 520, 96), (12768, 1024, 96), (4000, 4096, 40)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_tails(gen5, nrse_device, shape, out_dtype):
    K = gen5
    M, N, Kd = shape
    dev = nrse_device
    a, b = bf(M, Kd, dev=dev), bf(N, Kd, dev=dev)
    c = torch.full((M, N), 7.0, device=dev, dtype=out_dtype)
    K.gemm(K.Operand(a, True, Kd), K.Operand(b, True, Kd), c, M, N, Kd, ldc=N)
    assert rel(c, a.double() @ b.double().t()) < (1e-5 if out_dtype == torch.float32 else 4e-3)


def test_bias_gelu_aux(gen5, nrse_device):
    K = gen5
    from nrse_amd import _lib
    dev = nrse_device
    M, N, Kd = 1700, 776, 384
    x, w = bf(M, Kd, dev=dev), bf(N, Kd, dev=dev, scale=0.05)
    bias = torch.randn(N, device=dev)
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.linear_fwd(x, w, out, bias=bias, flags=_lib.EPI_GELU, aux=pre, ldaux=N)
    ref_pre = x.double() @ w.double().t() + bias.double()
    assert rel(pre, ref_pre) < 4e-3
    assert rel(out, F.gelu(ref_pre)) < 4e-3


@pytest.mark.parametrize("flags_name", ["resid", "resid_after", "gelu"])
def test_dropout_matches_128_kernel(gen5, nrse_device, flags_name):
    K = gen5
    from nrse_amd import _lib
    dev = nrse_device
    M, N, Kd = 900, 512, 256
    x, w = bf(M, Kd, dev=dev), bf(N, Kd, dev=dev)
    bias = torch.randn(N, device=dev)
    r = torch.randn(M, N, device=dev)
    outs = []
    for g in (5, 2):
        K.gemm_select(g)
        if flags_name == "gelu":
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            K.linear_fwd(x, w, c, bias=bias, flags=_lib.EPI_GELU, aux=pre, ldaux=N, dropout_p=0.2, seed=99)
        else:
            flags = _lib.EPI_RESID | (_lib.EPI_DROP_AFTER if flags_name == "resid_after" else 0)
            c = torch.empty(M, N, device=dev)
            K.linear_fwd(x, w, c, bias=bias, flags=flags, resid=r, ldr=N, dropout_p=0.2, seed=1234)
        outs.append(c.float())
    K.gemm_select(5)
    assert torch.equal(outs[0] == 0, outs[1] == 0)
    assert rel(outs[0], outs[1]) < (4e-3 if flags_name == "gelu" else 1e-6)


def test_batched_segments(gen5, nrse_device):
    """z-batch with a K axis cut into two segments (nseg), bias + residual epilogue."""
    K = gen5
    from nrse_amd import _lib
    dev = nrse_device
    Z, M, N, Kh = 2, 1000, 520, 160
    x = bf(Z, M, 2 * Kh, dev=dev)
    w = bf(Z, N, 2 * Kh, dev=dev, scale=0.1)
    bias = torch.randn(N, device=dev)
    r = torch.randn(Z, M, N, device=dev)
    c = torch.empty(Z, M, N, device=dev)
    K.gemm(K.Operand(x, True, 2 * Kh, z1=M * 2 * Kh, seg_stride=Kh), K.Operand(w, True, 2 * Kh, z1=N * 2 * Kh, seg_stride=Kh),
           c, M, N, Kh, ldc=N, batch=Z, c_z1=M * N, nseg=2, bias=bias, flags=_lib.EPI_RESID, resid=r, ldr=N, r_z1=M * N)
    ref = torch.einsum("zmk,znk->zmn", x.double(), w.double()) + bias.double() + r.double()
    assert rel(c, ref) < 1e-5


def test_unsupported_problems_fall_back(gen5, nrse_device):
    """Layouts and epilogues the kernel does not take (m-contiguous B, GELU', column sums) still
    run, through the other generations."""
    K = gen5
    dev = nrse_device
    M, N, Kd = 600, 264, 512
    dy, w = bf(M, Kd, dev=dev), bf(Kd, N, dev=dev)
    c = torch.empty(M, N, device=dev)
    cs = torch.zeros(N, device=dev)
    K.gemm(K.Operand(dy, True, Kd), K.Operand(w, False, N), c, M, N, Kd, ldc=N, colsum=cs)
    ref = dy.double() @ w.double()
    assert rel(c, ref) < 1e-5 and rel(cs, ref.sum(0)) < 1e-5
