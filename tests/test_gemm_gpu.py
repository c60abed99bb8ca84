"""nrse_gemm vs a float64 torch reference of the same contraction (all layout variants)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.double(); b = b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("akc", [True, False])
@pytest.mark.parametrize("bkc", [True, False])
@pytest.mark.parametrize("shape", [(200, 136, 72), (128, 256, 512), (88, 40, 1000)])
def test_gemm_layouts(nrse_device, dtype, akc, bkc, shape):
    from nrse_amd import kernels as K
    M, N, Kd = shape
    dev = nrse_device
    a = torch.randn(M, Kd, device=dev).to(dtype)
    b = torch.randn(N, Kd, device=dev).to(dtype)
    A = K.Operand(a, True, Kd) if akc else K.Operand(a.t().contiguous(), False, M)
    B = K.Operand(b, True, Kd) if bkc else K.Operand(b.t().contiguous(), False, N)
    c = torch.zeros(M, N, device=dev, dtype=torch.float32)
    K.gemm(A, B, c, M, N, Kd, ldc=N)
    ref = a.double() @ b.double().t()
    tol = 1e-6 if dtype == torch.float32 else 1e-5
    assert rel(c, ref) < tol


def test_gemm_epilogue_bias_gelu_resid(nrse_device):
    from nrse_amd import kernels as K, _lib
    dev = nrse_device
    M, N, Kd = 300, 192, 256
    x = torch.randn(M, Kd, device=dev)
    w = torch.randn(N, Kd, device=dev) * 0.05
    bias = torch.randn(N, device=dev)
    r = torch.randn(M, N, device=dev)
    pre = torch.empty(M, N, device=dev)
    out = torch.empty(M, N, device=dev)
    K.linear_fwd(x, w, out, bias=bias, flags=_lib.EPI_GELU | _lib.EPI_RESID, aux=pre, ldaux=N, resid=r, ldr=N)
    ref_pre = x.double() @ w.double().t() + bias.double()
    ref = torch.nn.functional.gelu(ref_pre) + r.double()
    assert rel(pre, ref_pre) < 1e-6
    assert rel(out, ref) < 1e-6


def test_gemm_segments_and_splits(nrse_device):
    """wgrad form: reduce over a segmented token axis with split-K atomics."""
    from nrse_amd import kernels as K
    dev = nrse_device
    M, N, Kd = 1024, 96, 64
    dy = torch.randn(M, N, device=dev)
    x = torch.randn(M, Kd, device=dev)
    dw = torch.zeros(N, Kd, device=dev)
    K.linear_wgrad(dy, x, dw, splits=4)
    ref = dy.double().t() @ x.double()
    assert rel(dw, ref) < 1e-6


def test_gemm_conv_implicit(nrse_device):
    """Strided Conv1d (k=3, s=2) on channels-last data as an implicit GEMM."""
    from nrse_amd import kernels as K
    dev = nrse_device
    B, Tin, C, k, s = 3, 101, 64, 3, 2
    Tout = (Tin - k) // s + 1
    x = torch.randn(B, Tin, C, device=dev)
    w = torch.randn(C, C, k, device=dev) * 0.1
    wr = w.permute(0, 2, 1).contiguous()  # [co][j][ci]
    y = torch.empty(B, Tout, C, device=dev)
    K.gemm(K.Operand(x, True, s * C, z1=Tin * C), K.Operand(wr, True, k * C), y, Tout, C, k * C,
           ldc=C, batch=B, c_z1=Tout * C)
    ref = torch.nn.functional.conv1d(x.double().transpose(1, 2), w.double(), stride=s).transpose(1, 2)
    assert rel(y, ref) < 1e-6


@pytest.mark.parametrize("shape", [(12768, 3072, 1024), (12768, 1024, 1024), (4096, 520, 264)])
def test_linear_wgrad_slab_splitk(nrse_device, shape):
    """linear_wgrad's split-K slab path (f32 partial slabs + nrse_splitk_reduce, accumulating into
    an existing gradient) against float64, and identical to itself run to run (deterministic)."""
    from nrse_amd import kernels as K
    M, N, Kin = shape
    dev = nrse_device
    dy = (torch.randn(M, N, device=dev) * 0.1).to(torch.bfloat16)
    x = torch.randn(M, Kin, device=dev).to(torch.bfloat16)
    g0 = torch.randn(N, Kin, device=dev)
    S = K._slab_splits(M, N, Kin)
    dw = g0.clone()
    K.linear_wgrad(dy, x, dw)
    ref = g0.double() + dy.double().t() @ x.double()
    assert rel(dw, ref) < 1e-5, (S, rel(dw, ref))
    dw2 = g0.clone()
    K.linear_wgrad(dy, x, dw2)
    if S:
        assert torch.equal(dw, dw2)


def test_splitk_reduce(nrse_device):
    from nrse_amd import kernels as K, _lib
    dev = nrse_device
    for n, S in ((4096, 3), (1000, 1), (12, 5), (8192, 8), (4100, 2)):
        slabs = torch.randn(S, n, device=dev)
        dst = torch.randn(n, device=dev)
        ref = dst.double() + slabs.double().sum(0)
        _lib.call("nrse_splitk_reduce", K.ptr(dst), K.ptr(slabs), S, n, 1, K.stream_ptr())
        assert rel(dst, ref) < 1e-6
        _lib.call("nrse_splitk_reduce", K.ptr(dst), K.ptr(slabs), S, n, 0, K.stream_ptr())
        assert rel(dst, slabs.double().sum(0)) < 1e-6


def _posconv_call(K, _lib, hpad, wf, out, T, H, G, pk, *, fwd, bias=None, pre=None, resid=None, p=0.0, seed=0):
    cpg = H // G
    cs = cpg.bit_length() - 1
    B = hpad.shape[0]
    A = K.Operand(hpad, True, H, chunk_shift=cs, ld_chunk=H, z1=(T + pk) * H, z2=cpg)
    Bw = K.Operand(wf, True, pk * cpg, z2=cpg * pk * cpg)
    if fwd:
        K.gemm(A, Bw, out, T, cpg, pk * cpg, ldc=H, batch=B * G, zdiv=G, c_z1=T * H, c_z2=cpg, bias=bias,
               bias_z2=cpg, flags=_lib.EPI_GELU | _lib.EPI_DROP_AFTER, aux=pre, ldaux=H, aux_z1=T * H, aux_z2=cpg,
               resid=resid, ldr=H, r_z1=T * H, r_z2=cpg, dropout_p=p, seed=seed)
    else:
        K.gemm(A, Bw, out, T, cpg, pk * cpg, ldc=H, batch=B * G, zdiv=G, c_z1=T * H, c_z2=cpg,
               flags=_lib.EPI_ACCUM)


@pytest.mark.parametrize("T", [399, 100, 600])
def test_posconv_sliding_window(nrse_device, T):
    """The grouped pos-conv (H = 1024, 16 groups of 64, 128 taps) routed to the sliding-window
    kernel (csrc/posconv.hip): forward with the fused bias + GELU (+ pre-activation) + residual +
    dropout epilogue, and the dgrad form accumulating into C, against float64 torch conv1d and
    against the generic LDS-DMA GEMM on the same call (same dropout mask)."""
    from nrse_amd import kernels as K, _lib
    dev = nrse_device
    B, H, G, pk = 3, 1024, 16, 128
    cpg = H // G
    g = torch.Generator(device=dev).manual_seed(T)
    x = torch.randn(B, T, H, device=dev, generator=g)
    hpad = torch.zeros(B, T + pk, H, device=dev, dtype=torch.bfloat16)
    hpad[:, pk // 2:pk // 2 + T] = x.to(torch.bfloat16)
    wf = (torch.randn(G, cpg, pk * cpg, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    bias = torch.randn(H, device=dev, generator=g) * 0.1
    resid = torch.randn(B * T, H, device=dev, generator=g)
    # float64 reference: conv1d with W[g*cpg + o, i, tap] = wf[g, o, tap*cpg + i]
    W = wf.double().view(G, cpg, pk, cpg).permute(0, 1, 3, 2).reshape(H, cpg, pk)
    conv = torch.nn.functional.conv1d(hpad.double().transpose(1, 2), W, groups=G)[:, :, :T].transpose(1, 2)
    ref_pre = conv.reshape(B * T, H) + bias.double()
    ref = torch.nn.functional.gelu(ref_pre) + resid.double()
    out = torch.empty(B * T, H, device=dev)
    pre = torch.empty(B * T, H, device=dev, dtype=torch.bfloat16)
    _posconv_call(K, _lib, hpad, wf, out, T, H, G, pk, fwd=True, bias=bias, pre=pre, resid=resid)
    assert rel(out, ref) < 1e-5
    assert rel(pre.float(), ref_pre) < 5e-3
    # dropout after the residual: the same mask and values as the generic kernel
    o1 = torch.empty(B * T, H, device=dev)
    o2 = torch.empty(B * T, H, device=dev)
    _posconv_call(K, _lib, hpad, wf, o1, T, H, G, pk, fwd=True, bias=bias, pre=pre, resid=resid, p=0.1, seed=7)
    prev = K.gemm_select(2)
    try:
        _posconv_call(K, _lib, hpad, wf, o2, T, H, G, pk, fwd=True, bias=bias, pre=pre, resid=resid, p=0.1, seed=7)
    finally:
        K.gemm_select(prev)
    assert torch.equal(o1 == 0, o2 == 0)
    assert rel(o1, o2) < 1e-6
    # dgrad form: C += conv (EPI_ACCUM)
    c0 = torch.randn(B * T, H, device=dev, generator=g)
    c = c0.clone()
    _posconv_call(K, _lib, hpad, wf, c, T, H, G, pk, fwd=False)
    assert rel(c, c0.double() + conv.reshape(B * T, H)) < 1e-5


@pytest.mark.parametrize("T,nseg,splits", [(399, 1, 3), (100, 3, 1), (600, 1, 3)])
def test_posconv_wgrad_sliding_window(nrse_device, T, nseg, splits):
    """The pos-conv weight gradient as the engine poses it (engine.py encoder_backward: A = dy
    rows of the padded dypad, B = the chunked Xp, M = 64, N = 128 taps x 64, K = T per utterance
    segment, f32 atomics into a zeroed dWf) routed to csrc/posconv.hip's posconv_wgrad_kernel:
    against a float64 einsum over the unfolded windows and against the generic 128x128 kernel."""
    from nrse_amd import kernels as K, _lib
    dev = nrse_device
    B, H, G, pk = nseg * splits, 1024, 16, 128
    cpg = H // G
    cs = cpg.bit_length() - 1
    g = torch.Generator(device=dev).manual_seed(T + 1)
    hpad = torch.zeros(B, T + pk, H, device=dev, dtype=torch.bfloat16)
    hpad[:, pk // 2:pk // 2 + T] = torch.randn(B, T, H, device=dev, generator=g).to(torch.bfloat16)
    lead = pk // 2 - 1
    dypad = torch.zeros(B, T + pk, H, device=dev, dtype=torch.bfloat16)
    dypad[:, lead:lead + T] = torch.randn(B, T, H, device=dev, generator=g).to(torch.bfloat16)

    def run():
        dWf = torch.zeros(G, cpg, pk * cpg, device=dev)
        K.gemm(K.Operand(dypad, False, H, offset=lead * H, seg_stride=(T + pk) * H, z1=cpg),
               K.Operand(hpad, False, H, chunk_shift=cs, ld_chunk=H, seg_stride=(T + pk) * H, z1=cpg),
               dWf, cpg, pk * cpg, T, ldc=pk * cpg, nseg=nseg, splits=splits, batch=G, c_z1=cpg * pk * cpg,
               flags=_lib.EPI_ATOMIC)
        return dWf

    got = run()
    again = run()
    assert torch.equal(got, again)  # two partial sums per element onto zeros: order-independent
    prev = K.gemm_select(2)
    try:
        generic = run()
    finally:
        K.gemm_select(prev)
    dy = dypad[:, lead:lead + T].double()
    win = hpad.double().unfold(1, pk, 1)[:, :T]  # [B, T, H, pk]: rows t .. t + pk - 1
    for gi in range(G):
        sl = slice(gi * cpg, (gi + 1) * cpg)
        ref = torch.einsum("bto,btip->opi", dy[..., sl], win[:, :, sl]).reshape(cpg, pk * cpg)
        assert rel(got[gi], ref) < 1e-5, gi
    assert rel(got, generic) < 1e-5


@pytest.mark.parametrize("T,nseg", [(399, 2), (100, 1)])
def test_posconv_wgrad_slabs(nrse_device, T, nseg):
    """The engine's form of the pos-conv weight gradient (engine.py encoder_backward): splits = 2
    with per-split f32 slabs stored whole by posconv_wgrad_kernel, then summed in slab order by
    nrse_splitk_reduce. Bit-identical to the two-share atomic form (two partial sums onto zeros),
    and within f32 accumulation of a float64 einsum."""
    from nrse_amd import kernels as K, _lib
    dev = nrse_device
    B, H, G, pk = 2 * nseg, 1024, 16, 128
    cpg = H // G
    cs = cpg.bit_length() - 1
    g = torch.Generator(device=dev).manual_seed(T + 7)
    hpad = torch.zeros(B, T + pk, H, device=dev, dtype=torch.bfloat16)
    hpad[:, pk // 2:pk // 2 + T] = torch.randn(B, T, H, device=dev, generator=g).to(torch.bfloat16)
    lead = pk // 2 - 1
    dypad = torch.zeros(B, T + pk, H, device=dev, dtype=torch.bfloat16)
    dypad[:, lead:lead + T] = torch.randn(B, T, H, device=dev, generator=g).to(torch.bfloat16)
    A_op = K.Operand(dypad, False, H, offset=lead * H, seg_stride=(T + pk) * H, z1=cpg)
    B_op = K.Operand(hpad, False, H, chunk_shift=cs, ld_chunk=H, seg_stride=(T + pk) * H, z1=cpg)
    n = G * cpg * pk * cpg
    slab = torch.full((2, n), float("nan"), device=dev)
    K.gemm(A_op, B_op, slab, cpg, pk * cpg, T, ldc=pk * cpg, nseg=nseg, splits=2, batch=G,
           c_z1=cpg * pk * cpg, c_split=n)
    got = torch.empty(n, device=dev)
    K.splitk_reduce(got, slab, 2, accumulate=False)
    atom = torch.zeros(n, device=dev)
    K.gemm(A_op, B_op, atom, cpg, pk * cpg, T, ldc=pk * cpg, nseg=nseg, splits=2, batch=G,
           c_z1=cpg * pk * cpg, flags=_lib.EPI_ATOMIC)
    assert torch.equal(got, atom)
    dy = dypad[:, lead:lead + T].double()
    win = hpad.double().unfold(1, pk, 1)[:, :T]
    got = got.view(G, cpg, pk * cpg)
    for gi in (0, G - 1):
        sl = slice(gi * cpg, (gi + 1) * cpg)
        ref = torch.einsum("bto,btip->opi", dy[..., sl], win[:, :, sl]).reshape(cpg, pk * cpg)
        assert rel(got[gi], ref) < 1e-5, gi


def _split(w):
    from nrse_amd import kernels as K
    w2 = torch.empty((2,) + tuple(w.shape), device=w.device, dtype=torch.bfloat16)
    K.split_bf16(w.contiguous(), w2[0], w2[1])
    return w2


@pytest.mark.parametrize("shape", [(12768, 1024, 1024), (300, 192, 256), (4000, 3072, 1024)])
def test_linear_fwd_split_weights(nrse_device, shape):
    """Split-weight mode: x @ (w_hi + w_lo)^T as two K segments of one launch
    (A read twice, B's lo plane seg_stride further on) carries the f32 weight: the product
    matches x_bf16 @ w_f32 to f32-accumulation level, and the bf16-weight product misses it by
    the weight rounding."""
    from nrse_amd import kernels as K, _lib
    M, N, Kd = shape
    dev = nrse_device
    x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w = torch.randn(N, Kd, device=dev) * 0.05
    bias = torch.randn(N, device=dev)
    w2 = _split(w)
    hi_err = ((w2[0].double() - w.double()).abs() / w.double().abs().clamp_min(1e-30)).max().item()
    assert hi_err <= 2 ** -8
    assert rel(w2[0].double() + w2[1].double(), w) < 3e-5    # hi + lo: ~2^-17 relative per element
    out = torch.empty(M, N, device=dev)
    K.linear_fwd(x, w2[0], out, bias=bias, w_lo=w2[0].numel())
    ref = x.double() @ w.double().t() + bias.double()
    e_split = rel(out, ref)
    out1 = torch.empty(M, N, device=dev)
    K.linear_fwd(x, w2[0], out1, bias=bias)
    e_hi = rel(out1, ref)
    assert e_split < 2e-5, (e_split, e_hi)
    assert e_hi > 10 * e_split, (e_split, e_hi)
    # bf16 output + GELU epilogue (the FFN-up form)
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    g = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.linear_fwd(x, w2[0], g, bias=bias, flags=_lib.EPI_GELU, aux=pre, ldaux=N, w_lo=w2[0].numel())
    assert rel(pre.float(), ref) < 5e-3
    assert rel(g.float(), torch.nn.functional.gelu(ref)) < 5e-3


@pytest.mark.parametrize("T", [399, 100])
def test_posconv_split_weights(nrse_device, T):
    """The pos-conv sliding-window kernel with two weight planes (nseg = 2, the split-weight
    mode's hi + lo): conv of the bf16 input with the f32 weights."""
    from nrse_amd import kernels as K, _lib
    dev = nrse_device
    B, H, G, pk = 2, 1024, 16, 128
    cpg = H // G
    g = torch.Generator(device=dev).manual_seed(T + 1)
    x = torch.randn(B, T, H, device=dev, generator=g)
    hpad = torch.zeros(B, T + pk, H, device=dev, dtype=torch.bfloat16)
    hpad[:, pk // 2:pk // 2 + T] = x.to(torch.bfloat16)
    wf32 = torch.randn(G, cpg, pk * cpg, device=dev, generator=g) * 0.02
    wf2 = _split(wf32)
    bias = torch.randn(H, device=dev, generator=g) * 0.1
    resid = torch.randn(B * T, H, device=dev, generator=g)
    W = wf32.double().view(G, cpg, pk, cpg).permute(0, 1, 3, 2).reshape(H, cpg, pk)
    conv = torch.nn.functional.conv1d(hpad.double().transpose(1, 2), W, groups=G)[:, :, :T].transpose(1, 2)
    ref_pre = conv.reshape(B * T, H) + bias.double()
    ref = torch.nn.functional.gelu(ref_pre) + resid.double()
    out = torch.empty(B * T, H, device=dev)
    pre = torch.empty(B * T, H, device=dev, dtype=torch.bfloat16)
    A = K.Operand(hpad, True, H, chunk_shift=cpg.bit_length() - 1, ld_chunk=H, z1=(T + pk) * H, z2=cpg)
    Bw = K.Operand(wf2[0], True, pk * cpg, z2=cpg * pk * cpg, seg_stride=wf32.numel())
    K.gemm(A, Bw, out, T, cpg, pk * cpg, ldc=H, batch=B * G, zdiv=G, nseg=2, c_z1=T * H, c_z2=cpg, bias=bias,
           bias_z2=cpg, flags=_lib.EPI_GELU | _lib.EPI_DROP_AFTER, aux=pre, ldaux=H, aux_z1=T * H, aux_z2=cpg,
           resid=resid, ldr=H, r_z1=T * H, r_z2=cpg)
    assert rel(out, ref) < 5e-6       # f32 accumulation over 2 x 8192 terms + the GELU's erf approximation
    # the hi plane alone misses the f32 weights by their bf16 rounding
    o1 = torch.empty(B * T, H, device=dev)
    K.gemm(A, K.Operand(wf2[0], True, pk * cpg, z2=cpg * pk * cpg), o1, T, cpg, pk * cpg, ldc=H, batch=B * G, zdiv=G,
           c_z1=T * H, c_z2=cpg, bias=bias, bias_z2=cpg, flags=_lib.EPI_GELU | _lib.EPI_DROP_AFTER, aux=pre, ldaux=H,
           aux_z1=T * H, aux_z2=cpg, resid=resid, ldr=H, r_z1=T * H, r_z2=cpg)
    assert rel(o1, ref) > 10 * rel(out, ref)
    # the same call on the generic LDS-DMA kernel agrees
    o2 = torch.empty(B * T, H, device=dev)
    prev = K.gemm_select(2)
    try:
        K.gemm(A, Bw, o2, T, cpg, pk * cpg, ldc=H, batch=B * G, zdiv=G, nseg=2, c_z1=T * H, c_z2=cpg, bias=bias,
               bias_z2=cpg, flags=_lib.EPI_GELU | _lib.EPI_DROP_AFTER, aux=pre, ldaux=H, aux_z1=T * H,
               aux_z2=cpg, resid=resid, ldr=H, r_z1=T * H, r_z2=cpg)
    finally:
        K.gemm_select(prev)
    assert rel(o2, ref) < 5e-6


def test_conv_gemm_split_activations(nrse_device):
    """The split-weight mode's conv GEMM: activations as NRSE_BF16X3 planes [hi | lo | hi] against
    weight planes [hi | hi | lo], three K segments of one launch: the f32 conv to ~2^-16."""
    from nrse_amd import kernels as K
    dev = nrse_device
    B, Tin, C, k, s = 4, 801, 512, 3, 2
    Tout = (Tin - k) // s + 1
    x = torch.randn(B, Tin, C, device=dev)
    w = torch.randn(C, C, k, device=dev) * 0.05
    wr = w.permute(0, 2, 1).contiguous()
    x3 = torch.empty(3, B * Tin * C, device=dev, dtype=torch.bfloat16)
    K.split_bf16(x.reshape(-1), x3[0], x3[1])
    x3[2].copy_(x3[0])
    w3 = torch.empty(3, C * k * C, device=dev, dtype=torch.bfloat16)
    K.split_bf16(wr.reshape(-1), w3[0], w3[2])
    w3[1].copy_(w3[0])
    y = torch.empty(B * Tout, C, device=dev)
    K.gemm(K.Operand(x3[0], True, s * C, z1=Tin * C, seg_stride=B * Tin * C),
           K.Operand(w3[0], True, k * C, seg_stride=C * k * C), y, Tout, C, k * C, ldc=C, batch=B, c_z1=Tout * C,
           nseg=3)
    ref = torch.nn.functional.conv1d(x.double().transpose(1, 2), w.double(), stride=s).transpose(1, 2).reshape(-1, C)
    assert rel(y, ref) < 2e-5


@pytest.mark.parametrize("shape", [(12768, 4096, 1024), (300, 256, 128)])
def test_gelu_without_preactivation_matches(nrse_device, shape):
    """The FFN-up epilogue without a pre-activation output (the target view keeps no tape) gives
    the same bf16 output as the taped form, bit for bit, and the taped pre-activation matches
    float64."""
    from nrse_amd import kernels as K, _lib
    M, N, Kd = shape
    dev = nrse_device
    x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    y1 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    y2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.linear_fwd(x, w, y1, bias=b, flags=_lib.EPI_GELU, aux=pre, ldaux=N)
    K.linear_fwd(x, w, y2, bias=b, flags=_lib.EPI_GELU)
    assert torch.equal(y1, y2)
    ref_pre = x.double() @ w.double().t() + b.double()
    assert rel(pre, ref_pre) < 5e-3
    assert rel(y2, torch.nn.functional.gelu(ref_pre)) < 5e-3


def test_bias_dropout_f32_matches_residual_form(nrse_device):
    """bias + dropout with an f32 output (the feature projection) equals the bias + dropout +
    residual form with a zero residual, bit for bit (same keep mask, same rounding)."""
    from nrse_amd import kernels as K
    M, N, Kd = 12768, 1024, 512
    dev = nrse_device
    x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    zero = torch.zeros(M, N, device=dev)
    y1 = torch.empty(M, N, device=dev)
    y2 = torch.empty(M, N, device=dev)
    K.linear_fwd(x, w, y1, bias=b, dropout_p=0.1, seed=7)
    K.linear_fwd(x, w, y2, bias=b, resid=zero, ldr=N, dropout_p=0.1, seed=7)
    assert torch.equal(y1, y2)
    kept = (y1 != 0).float().mean().item()
    assert abs(kept - 0.9) < 0.01
