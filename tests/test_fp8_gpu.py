"""The split-weight mode's fp8 form (ABI 6) piece by piece:

* the fp8 conversions (nrse_cast_fp8, nrse_split_lo8) against torch's float8_e4m3fn (OCP e4m3fn,
  round to nearest even) of the clamped values: bit-exact, saturating at +-448;
* the 256x256 GEMM's fp8 correction segment (MX-scaled v_mfma_scale_f32_16x16x128_f8f6f4) against a
  float64 product of the same bf16 / fp8 operands, every tile height, ragged M, both epilogue
  families of the step (bias + GELU + pre-activation + fp8 output copy; bias + dropout + f32
  residual), and the split weight it restores (x @ (w_hi + 2^-e lo8) vs the exact f32 weight);
* the fp8 copies written beside their bf16 outputs (LayerNorm y8, GEMM c8): bit-exact;
* the AdamW pass's fp8 planes (online and fused EMA target) and its gradient zeroing.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
E4M3 = torch.float8_e4m3fn


def rel(a, b):
    a = a.double(); b = b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def fp8_ref(x: torch.Tensor) -> torch.Tensor:
    """torch's e4m3fn of x clamped to the finite range (the kernels saturate; torch gives NaN)."""
    return x.detach().float().cpu().clamp(-448.0, 448.0).to(E4M3)


def d(t: torch.Tensor) -> torch.Tensor:
    """float64 on the device (fp8 widened on the host first)."""
    return t.detach().cpu().double().cuda()


def bits(t: torch.Tensor) -> torch.Tensor:
    return t.detach().cpu().view(torch.uint8)


def lo_ref(w: torch.Tensor, e: int) -> torch.Tensor:
    """fp8((w - bf16(w)) 2^e) in f32 arithmetic (the subtraction is exact)."""
    w = w.detach().float().cpu()
    return fp8_ref((w - w.to(torch.bfloat16).float()) * 2.0 ** e)


@pytest.fixture(params=[256, 224], ids=["bm256", "bm224"])
def gen3(nrse_device, request):
    from nrse_amd import kernels as K
    old = K.gemm_select(3)
    old_rows = K.gemm_tile_rows(request.param)
    yield K
    K.gemm_select(old)
    K.gemm_tile_rows(old_rows)


def test_cast_fp8_matches_torch(nrse_device):
    from nrse_amd import kernels as K
    g = torch.Generator(device="cpu").manual_seed(3)
    parts = [torch.randn(4096, generator=g) * s for s in (1e-4, 1e-2, 1.0, 30.0, 600.0)]
    x = torch.cat(parts + [torch.tensor([0.0, -0.0, 448.0, -448.0, 464.0, 1e6, -1e6, 2.0 ** -10, 2.0 ** -9])])
    for src in (x.cuda(), x.to(torch.bfloat16).cuda()):
        y = torch.empty(x.numel(), device="cuda", dtype=E4M3)
        K.cast_fp8(src, y)
        torch.cuda.synchronize()
        assert torch.equal(bits(y), bits(fp8_ref(src.float()))), "fp8 conversion differs from torch e4m3fn"


@pytest.mark.parametrize("n", [4099, 65536])
def test_split_lo8_matches_torch(nrse_device, n):
    from nrse_amd import kernels as K
    w = torch.randn(n, device="cuda") * 0.03
    w[:7] = torch.tensor([1.0, 3.75, -0.5, 1e-6, 0.0, 2.0 ** -20, 100.0])
    for e in (8, 19):
        lo = torch.empty(n, device="cuda", dtype=E4M3)
        K.split_lo8(w, lo, e)
        torch.cuda.synchronize()
        assert torch.equal(bits(lo), bits(lo_ref(w, e)))


@pytest.mark.parametrize("shape", [(700, 512, 384), (1304, 1024, 1024), (520, 3072, 1024), (12768, 1024, 1024)])
def test_gemm_fp8_correction_segment(gen3, nrse_device, shape):
    K = gen3
    M, N, Kd = shape
    x = (torch.randn(M, Kd, device="cuda")).to(torch.bfloat16)
    w = torch.randn(N, Kd, device="cuda") * 0.03
    bias = torch.randn(N, device="cuda")
    e = 19
    w_hi = w.to(torch.bfloat16)
    w8 = torch.empty(N, Kd, device="cuda", dtype=E4M3)
    K.split_lo8(w, w8, e)
    x8 = torch.empty(M, Kd, device="cuda", dtype=E4M3)
    K.cast_fp8(x, x8)
    out = torch.empty(M, N, device="cuda")
    K.linear_fwd(x, w_hi, out, bias=bias, x8=x8, w8=w8, lo8_exp=e)
    torch.cuda.synchronize()
    xd = d(x)
    ref = xd @ d(w_hi).t() + 2.0 ** -e * (d(x8) @ d(w8).t()) + d(bias)
    assert rel(out, ref) < 2e-6, rel(out, ref)
    # the split weight: against the exact f32 weight, ~2^-13 instead of bf16's ~2^-9
    exact = xd @ d(w).t() + d(bias)
    hi_only = xd @ d(w_hi).t() + d(bias)
    assert rel(out, exact) < rel(hi_only, exact) / 6, (rel(out, exact), rel(hi_only, exact))


@pytest.mark.parametrize("aux", [True, False], ids=["aux", "noaux"])
def test_gemm_fp8_gelu_epilogue_with_fp8_copy(gen3, nrse_device, aux):
    """The FFN-up form: bias + GELU (+ bf16 pre-activation), bf16 output and its fp8 copy c8."""
    K = gen3
    from nrse_amd import _lib
    M, N, Kd = 1000, 1024, 512
    x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, Kd, device="cuda") * 0.05
    bias = torch.randn(N, device="cuda") * 0.1
    e = 17
    w_hi = w.to(torch.bfloat16)
    w8 = torch.empty(N, Kd, device="cuda", dtype=E4M3)
    K.split_lo8(w, w8, e)
    x8 = torch.empty(M, Kd, device="cuda", dtype=E4M3)
    K.cast_fp8(x, x8)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if aux else None
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    out8 = torch.empty(M, N, device="cuda", dtype=E4M3)
    K.linear_fwd(x, w_hi, out, bias=bias, flags=_lib.EPI_GELU, aux=pre, ldaux=N if aux else 0, x8=x8, w8=w8,
                 lo8_exp=e, out8=out8)
    torch.cuda.synchronize()
    ref_pre = d(x) @ d(w_hi).t() + 2.0 ** -e * (d(x8) @ d(w8).t()) + d(bias)
    if aux:
        assert rel(pre, ref_pre) < 4e-3
    assert rel(out, F.gelu(ref_pre)) < 4e-3
    assert torch.equal(bits(out8), bits(fp8_ref(out.float())))


def test_gemm_fp8_resid_dropout_epilogue(gen3, nrse_device):
    """The FFN-down / out-proj form: bias + dropout + f32 residual, f32 output; the fp8 segment
    must not change the dropout mask (a function of the output offset)."""
    K = gen3
    M, N, Kd = 900, 1024, 4096
    x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, Kd, device="cuda") * 0.02
    bias = torch.randn(N, device="cuda") * 0.1
    r = torch.randn(M, N, device="cuda")
    e = 20
    w_hi = w.to(torch.bfloat16)
    w8 = torch.empty(N, Kd, device="cuda", dtype=E4M3)
    K.split_lo8(w, w8, e)
    x8 = torch.empty(M, Kd, device="cuda", dtype=E4M3)
    K.cast_fp8(x, x8)
    out = torch.empty(M, N, device="cuda")
    K.linear_fwd(x, w_hi, out, bias=bias, resid=r, ldr=N, dropout_p=0.1, seed=99, x8=x8, w8=w8, lo8_exp=e)
    plain = torch.empty(M, N, device="cuda")
    K.linear_fwd(x, w_hi, plain, bias=bias, resid=r, ldr=N, dropout_p=0.1, seed=99)
    torch.cuda.synchronize()
    kept = (plain - r) != 0
    assert torch.equal(kept, (out - r) != 0)
    corr = 2.0 ** -e * (d(x8) @ d(w8).t())
    ref = (d(x) @ d(w_hi).t() + corr + d(bias)) * kept.double() / 0.9 + d(r)
    assert rel(out, ref) < 2e-6


def test_gemm_fp8_refuses_unsupported(nrse_device):
    from nrse_amd import kernels as K, _lib
    x = torch.randn(512, 320, device="cuda").to(torch.bfloat16)   # K % 128 != 0
    w = torch.randn(512, 320, device="cuda").to(torch.bfloat16)
    x8 = torch.empty(512, 320, device="cuda", dtype=E4M3)
    w8 = torch.empty(512, 320, device="cuda", dtype=E4M3)
    out = torch.empty(512, 512, device="cuda")
    with pytest.raises(_lib.NrseError):
        K.linear_fwd(x, w, out, x8=x8, w8=w8, lo8_exp=10)


def test_layernorm_fp8_copy(nrse_device):
    from nrse_amd import kernels as K
    rows, C = 1333, 1024
    x = torch.randn(rows, C, device="cuda") * 3
    g, b = torch.randn(C, device="cuda"), torch.randn(C, device="cuda")
    y = torch.empty(rows, C, device="cuda", dtype=torch.bfloat16)
    y8 = torch.empty(rows, C, device="cuda", dtype=E4M3)
    mean, rstd = torch.empty(rows, device="cuda"), torch.empty(rows, device="cuda")
    K.ln_fwd(x, g, b, y, mean, rstd, 1e-5, y8=y8)
    torch.cuda.synchronize()
    assert rel(y, F.layer_norm(x.double(), (C,), g.double(), b.double(), 1e-5)) < 4e-3
    assert torch.equal(bits(y8), bits(fp8_ref(y.float())))


@pytest.mark.parametrize("n,ne", [(40003, 30001), (65536, 65536)])
def test_adamw_fp8_planes_and_zero_grad(nrse_device, n, ne):
    from nrse_amd import kernels as K
    dev = "cuda"
    p0 = torch.randn(n, device=dev) * 0.05
    g0 = torch.randn(n, device=dev) * 1e-3
    m0, v0 = torch.randn(n, device=dev) * 1e-4, torch.rand(n, device=dev) * 1e-7
    t0 = p0[:ne] + torch.randn(ne, device=dev) * 1e-4
    sumsq = torch.tensor([float((g0.double() ** 2).sum())], device=dev, dtype=torch.float64)
    e = 19
    outs = []
    for fused in (False, True):
        p, g, m, v, t = p0.clone(), g0.clone(), m0.clone(), v0.clone(), t0.clone()
        sh, lo = torch.empty(n, device=dev, dtype=torch.bfloat16), torch.empty(n, device=dev, dtype=torch.bfloat16)
        tsh, tlo = torch.empty(ne, device=dev, dtype=torch.bfloat16), torch.empty(ne, device=dev, dtype=torch.bfloat16)
        lo8 = torch.empty(n, device=dev, dtype=E4M3) if fused else None
        tlo8 = torch.empty(ne, device=dev, dtype=E4M3) if fused else None
        K.adamw(p, g, m, v, sh, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-5, step=3, max_norm=1.0,
                sumsq_buf=sumsq, shadow_lo=lo, ema_t=t, ema_shadow=tsh, ema_shadow_lo=tlo, ema_decay=0.997,
                shadow_lo8=lo8, ema_shadow_lo8=tlo8, lo8_exp=e, zero_grad=fused)
        torch.cuda.synchronize()
        outs.append((p, g, m, v, t, sh, lo, tsh, tlo, lo8, tlo8))
    a, b = outs
    for i in (0, 2, 3, 4, 5, 6, 7, 8):   # identical update with the new outputs switched on
        assert torch.equal(a[i], b[i]), i
    assert torch.equal(a[1], g0) and float(b[1].abs().max()) == 0.0   # zero_grad
    assert torch.equal(bits(b[9]), bits(lo_ref(b[0], e)))
    assert torch.equal(bits(b[10]), bits(lo_ref(b[4], e)))


def test_attention_fp8_context_copy(nrse_device):
    """The attention forward's ctx8 (ABI 6): fp8 of the stored bf16 context, bit-exact, and the
    context itself unchanged by it."""
    from nrse_amd import kernels as K
    B, T, H = 2, 150, 4
    qkv = (torch.randn(B * T, 3 * H * 64, device="cuda")).to(torch.bfloat16)
    gate = torch.rand(B, H, T, device="cuda") + 0.5
    vec = torch.randn(H, 2 * T - 1, device="cuda") * 0.1
    outs = []
    for with8 in (False, True):
        ctx = torch.empty(B * T, H * 64, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B, H, T, device="cuda")
        c8 = torch.empty(B * T, H * 64, device="cuda", dtype=E4M3) if with8 else None
        K.attn_fwd(qkv, gate, None, ctx, lse, B, T, H, 0.1, 42, bias_vec=vec, ctx8=c8)
        torch.cuda.synchronize()
        outs.append((ctx, c8))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(bits(outs[1][1]), bits(fp8_ref(outs[1][0].float())))


# ---------------------------------------------------------------- the conv stack's fp8 form (ABI 7)
def _split_check(hi, lo8, e, ref):
    """hi + 2^-e lo8 restores the exact ref to ~2^-13 (hi alone: ~2^-9)."""
    got = d(hi) + 2.0 ** -e * d(lo8)
    r_hi = rel(hi, ref)
    assert rel(got, ref) < 1e-4 and rel(got, ref) < r_hi / 8, (rel(got, ref), r_hi)


@pytest.mark.parametrize("C", [512, 256])
def test_conv0_fp8_planes(nrse_device, C):
    """conv0 (matrix-core form) with y8 (ABI 7): out = bf16(o) as the split-planes form stores it,
    y8 = [fp8((o - hi) 2^e) | fp8(hi)]: the hi plane bit-exact, hi + lo restoring the float64 conv."""
    from nrse_amd import kernels as K
    dev = nrse_device
    B, L, k, s, e = 3, 8001, 10, 5, 11
    T0 = (L - k) // s + 1
    rows = B * T0
    wav = torch.randn(B, L, device=dev) * 0.2
    w = torch.randn(C, 1, k, device=dev) * 0.3
    g = torch.randn(C, device=dev) * 0.1 + 1; b = torch.randn(C, device=dev) * 0.1
    out3 = torch.empty(3, rows, C, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    K.conv0_fwd(wav, w.view(C, k), g, b, out3, mean, rstd, T0, k, s, 1e-5, split3=True)
    out = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
    y8 = torch.empty(2, rows, C, device=dev, dtype=E4M3)
    mean2, rstd2 = torch.empty_like(mean), torch.empty_like(rstd)
    K.conv0_fwd(wav, w.view(C, k), g, b, out, mean2, rstd2, T0, k, s, 1e-5, y8=y8, y8_exp=e)
    torch.cuda.synchronize()
    assert torch.equal(out, out3[0]) and torch.equal(mean, mean2) and torch.equal(rstd, rstd2)
    assert torch.equal(bits(y8[1]), bits(fp8_ref(out.float())))
    y = F.conv1d(wav.double()[:, None], w.double(), stride=s).transpose(1, 2).reshape(rows, C)
    mu = y.mean(1); var = y.var(1, unbiased=False)
    ref = F.gelu((y - mu[:, None]) / torch.sqrt(var[:, None] + 1e-5) * g.double() + b.double())
    _split_check(out, y8[0], e, ref)


def test_layernorm_fp8_split_planes(nrse_device):
    """LN + GELU with y8_split (the conv stack's form): y = bf16(o), y8 = [fp8((o - y) 2^e) | fp8(y)]."""
    from nrse_amd import kernels as K
    rows, C, e = 2053, 512, 11
    x = torch.randn(rows, C, device="cuda") * 3
    g, b = torch.randn(C, device="cuda") * 0.2 + 1, torch.randn(C, device="cuda") * 0.1
    y = torch.empty(rows, C, device="cuda", dtype=torch.bfloat16)
    y8 = torch.empty(2, rows, C, device="cuda", dtype=E4M3)
    mean, rstd = torch.empty(rows, device="cuda"), torch.empty(rows, device="cuda")
    K.ln_fwd(x, g, b, y, mean, rstd, 1e-5, gelu=True, y8=y8, y8_exp=e)
    torch.cuda.synchronize()
    ref = F.gelu(F.layer_norm(x.double(), (C,), g.double(), b.double(), 1e-5))
    assert torch.equal(bits(y8[1]), bits(fp8_ref(y.float())))
    _split_check(y, y8[0], e, ref)
    # the plain copy form is unchanged by the new fields
    y8c = torch.empty(rows, C, device="cuda", dtype=E4M3)
    K.ln_fwd(x, g, b, y, mean, rstd, 1e-5, gelu=True, y8=y8c)
    torch.cuda.synchronize()
    assert torch.equal(bits(y8c), bits(y8[1]))


@pytest.mark.parametrize("k,s,Tin", [(3, 2, 301), (2, 2, 300)])
def test_gemm_fp8_conv_segments(gen3, nrse_device, k, s, Tin):
    """The conv stack's GEMM in the fp8 split form, as encoder_forward issues it: overlapping rows
    (ld = s Cin), batch z1 strides, one bf16 segment + two fp8 segments [x_lo8 | x_hi8] x [w_hi8 |
    w_lo8] scaled by 2^-e, f32 output; against float64 of the same operands, and the exact conv."""
    K = gen3
    B, Cin, C, e = 3, 512, 512, 11
    Tout = (Tin - k) // s + 1
    x = F.gelu(torch.randn(B, Tin, Cin, device="cuda"))
    w = torch.randn(C, Cin, k, device="cuda") * 0.03
    x_hi = x.to(torch.bfloat16)
    x8 = torch.stack([fp8_ref((x - x_hi.float()) * 2.0 ** e), fp8_ref(x_hi.float())]).cuda()
    r = w.permute(0, 2, 1).reshape(C, k * Cin).contiguous()   # [co][k][ci]
    r_hi = r.to(torch.bfloat16)
    w8 = torch.stack([fp8_ref(r_hi.float()), lo_ref(r, e)]).cuda()
    out = torch.empty(B * Tout, C, device="cuda")
    K.gemm(K.Operand(x_hi, True, s * Cin, z1=Tin * Cin), K.Operand(r_hi, True, k * Cin), out, Tout, C, k * Cin,
           ldc=C, batch=B, c_z1=Tout * C,
           a8=K.Operand(x8, True, s * Cin, z1=Tin * Cin, seg_stride=B * Tin * Cin),
           b8=K.Operand(w8, True, k * Cin, seg_stride=C * k * Cin), nseg8=2, b8_exp=e)
    torch.cuda.synchronize()

    def conv(a, ww):   # a [B, Tin, Cin], ww [C, k*Cin] (tap-major) -> [B*Tout, C]
        wk = d(ww).view(C, k, Cin).permute(0, 2, 1)
        return F.conv1d(d(a).permute(0, 2, 1), wk, stride=s).permute(0, 2, 1).reshape(B * Tout, C)

    ref = conv(x_hi, r_hi) + 2.0 ** -e * (conv(x8[0], w8[0]) + conv(x8[1], w8[1]))
    assert rel(out, ref) < 2e-6, rel(out, ref)
    exact = conv(x, r)
    assert rel(out, exact) < rel(conv(x_hi, r_hi), exact) / 8, (rel(out, exact), rel(conv(x_hi, r_hi), exact))


def test_conv0_and_ln_fp8_planes_refused(nrse_device):
    from nrse_amd import kernels as K, _lib
    dev = nrse_device
    B, L, k, s, C = 1, 2001, 10, 5, 512
    T0 = (L - k) // s + 1
    wav = torch.randn(B, L, device=dev)
    w = torch.randn(C, k, device=dev); g = torch.ones(C, device=dev); b = torch.zeros(C, device=dev)
    mean, rstd = torch.empty(T0, device=dev), torch.empty(T0, device=dev)
    y8 = torch.empty(2, T0, C, device=dev, dtype=E4M3)
    out32 = torch.empty(T0, C, device=dev)
    with pytest.raises(_lib.NrseError):   # f32 out: the VALU kernel has no fp8 planes
        K.conv0_fwd(wav, w, g, b, out32, mean, rstd, T0, k, s, 1e-5, y8=y8, y8_exp=11)
    x = torch.randn(T0, C, device=dev)
    y = torch.empty(T0, C, device=dev, dtype=torch.bfloat16)
    with pytest.raises(_lib.NrseError):   # exponent out of range
        K.ln_fwd(x, g, b, y, mean, rstd, 1e-5, y8=y8, y8_exp=99)
    # fp8 segments at M < 128 (a short utterance's last conv layers): refused, never dropped --
    # the engine keeps the three bf16 planes there
    Tin, Cin, kk, ss = 160, 512, 2, 2
    xa = torch.randn(2, Tin, Cin, device=dev).to(torch.bfloat16)
    x8 = torch.zeros(2, 2, Tin, Cin, device=dev, dtype=E4M3)
    r = torch.randn(C, kk * Cin, device=dev).to(torch.bfloat16)
    w8 = torch.zeros(2, C, kk * Cin, device=dev, dtype=E4M3)
    o = torch.empty(2 * 80, C, device=dev)
    with pytest.raises(_lib.NrseError):
        K.gemm(K.Operand(xa, True, ss * Cin, z1=Tin * Cin), K.Operand(r, True, kk * Cin), o, 80, C, kk * Cin, ldc=C,
               batch=2, c_z1=80 * C, a8=K.Operand(x8, True, ss * Cin, z1=Tin * Cin, seg_stride=2 * Tin * Cin),
               b8=K.Operand(w8, True, kk * Cin, seg_stride=C * kk * Cin), nseg8=2, b8_exp=11)
