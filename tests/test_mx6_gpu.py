"""The split-weight mode's MXFP6 form (ABI 8, NRSE_MX6) piece by piece, against the
CPU restatement of the format (oracle/mx6.py):

* the MXFP6 producers write exactly the oracle's bytes for the values they store: nrse_cast_mx6 /
  nrse_split_lo_mx6, the LayerNorm y8 copy, the conv0 and conv-stack LayerNorm split planes (hi
  plane bit-exact; the lo plane restores the exact output to ~2^-13), the FFN-up GEMM epilogue's c8,
  the attention forward's ctx8, and the AdamW pass's weight / EMA-target planes;
* the 256x256 GEMM's MXFP6 correction segments (v_mfma_scale_f32_16x16x128_f8f6f4, e2m3 with the
  blocks' own E8M0 scales) against a float64 product of the decoded operands, for the layer form
  (one segment) and the conv-stack form (overlapping rows, batch strides, two segments), and the
  split weight they restore against the exact f32 weight.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import mx6 as MX

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def enc(t: torch.Tensor) -> np.ndarray:
    """oracle bytes of the values t holds (f32 view)."""
    return MX.encode(t.detach().float().cpu().numpy())


def dec(t8: torch.Tensor) -> torch.Tensor:
    return torch.from_numpy(MX.decode(t8.detach().cpu().numpy()))


def same(t8: torch.Tensor, ref: np.ndarray):
    got = t8.detach().cpu().numpy()
    bad = np.argwhere(got != ref)
    assert bad.size == 0, f"{len(bad)} bytes differ, first at {bad[:4].tolist()}"


@pytest.fixture(params=[256, 224], ids=["bm256", "bm224"])
def gen3(nrse_device, request):
    from nrse_amd import kernels as K
    old = K.gemm_select(3)
    old_rows = K.gemm_tile_rows(request.param)
    yield K
    K.gemm_select(old)
    K.gemm_tile_rows(old_rows)


def test_cast_and_split_match_oracle(nrse_device):
    from nrse_amd import kernels as K
    g = torch.Generator(device="cpu").manual_seed(7)
    parts = [torch.randn(4096, generator=g) * s for s in (1e-30, 1e-6, 1e-2, 1.0, 300.0, 1e30)]
    special = torch.zeros(64)
    special[32:] = torch.tensor([7.5, -7.5, 0.0625, 0.1875, -0.0, 1.0, 3.75, 3.76] * 4)
    x = torch.cat(parts + [special])
    for src in (x.cuda(), x.to(torch.bfloat16).cuda()):
        y = torch.empty(x.numel(), device="cuda", dtype=K.MX6)
        K.cast_fp8(src, y)
        torch.cuda.synchronize()
        same(y, enc(src))
    w = (torch.randn(3 * 4096, generator=g) * 0.05).cuda()
    lo = torch.empty(w.numel(), device="cuda", dtype=K.MX6)
    K.split_lo8(w, lo)
    torch.cuda.synchronize()
    same(lo, enc(w - w.to(torch.bfloat16).float()))


@pytest.mark.parametrize("shape", [(700, 512, 384), (1304, 1024, 1024), (520, 3072, 1024), (12768, 1024, 4096)])
def test_gemm_mx6_correction_segment(gen3, nrse_device, shape):
    K = gen3
    M, N, Kd = shape
    x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, Kd, device="cuda") * 0.03
    bias = torch.randn(N, device="cuda")
    w_hi = w.to(torch.bfloat16)
    w8 = torch.empty(N, Kd, device="cuda", dtype=K.MX6)
    K.split_lo8(w, w8)
    x8 = torch.empty(M, Kd, device="cuda", dtype=K.MX6)
    K.cast_fp8(x, x8)
    out = torch.empty(M, N, device="cuda")
    K.linear_fwd(x, w_hi, out, bias=bias, x8=x8, w8=w8)
    torch.cuda.synchronize()
    xd, bd = x.double().cpu(), bias.double().cpu()
    ref = xd @ w_hi.double().cpu().t() + dec(x8) @ dec(w8).t() + bd
    assert rel(out, ref) < 2e-6, rel(out, ref)
    exact = xd @ w.double().cpu().t() + bd
    hi_only = xd @ w_hi.double().cpu().t() + bd
    assert rel(out, exact) < rel(hi_only, exact) / 6, (rel(out, exact), rel(hi_only, exact))


def test_gemm_mx6_gelu_epilogue_copy(gen3, nrse_device):
    """FFN-up form: bias + GELU + bf16 pre-activation, with the MXFP6 c8 of the stored output."""
    K = gen3
    M, N, Kd = 1304, 4096, 1024
    x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, Kd, device="cuda") * 0.03
    w_hi = w.to(torch.bfloat16)
    w8 = torch.empty(N, Kd, device="cuda", dtype=K.MX6); K.split_lo8(w, w8)
    x8 = torch.empty(M, Kd, device="cuda", dtype=K.MX6); K.cast_fp8(x, x8)
    bias = torch.randn(N, device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    c8 = torch.empty(M, N, device="cuda", dtype=K.MX6)
    K.linear_fwd(x, w_hi, out, bias=bias, flags=K._lib.EPI_GELU, aux=pre, ldaux=N, x8=x8, w8=w8, out8=c8)
    torch.cuda.synchronize()
    same(c8, enc(out))
    ref = F.gelu(x.double().cpu() @ w_hi.double().cpu().t() + dec(x8) @ dec(w8).t() + bias.double().cpu())
    assert rel(out, ref) < 4e-3


def test_gemm_mx6_c8_refused_outside_register_epilogue(nrse_device):
    from nrse_amd import kernels as K, _lib
    x = torch.randn(512, 512, device="cuda").to(torch.bfloat16)
    w = torch.randn(512, 512, device="cuda").to(torch.bfloat16)
    out = torch.empty(512, 512, device="cuda", dtype=torch.bfloat16)
    c8 = torch.empty(512, 512, device="cuda", dtype=K.MX6)
    with pytest.raises(_lib.NrseError):   # accumulate: the general epilogue
        K.linear_fwd(x, w, out, flags=_lib.EPI_ACCUM, out8=c8)


@pytest.mark.parametrize("split", [False, True])
def test_layernorm_mx6(nrse_device, split):
    from nrse_amd import kernels as K
    rows, C = 2053, 1024 if not split else 512
    x = torch.randn(rows, C, device="cuda") * 3
    g, b = torch.randn(C, device="cuda") * 0.2 + 1, torch.randn(C, device="cuda") * 0.1
    y = torch.empty(rows, C, device="cuda", dtype=torch.bfloat16)
    y8 = torch.empty((2, rows, C) if split else (rows, C), device="cuda", dtype=K.MX6)
    mean, rstd = torch.empty(rows, device="cuda"), torch.empty(rows, device="cuda")
    K.ln_fwd(x, g, b, y, mean, rstd, 1e-5, gelu=split, y8=y8, y8_exp=0 if split else None)
    torch.cuda.synchronize()
    ref = F.layer_norm(x.double(), (C,), g.double(), b.double(), 1e-5)
    if not split:
        same(y8, enc(y))
        return
    ref = F.gelu(ref).cpu()
    same(y8[1], enc(y))
    got = y.double().cpu() + dec(y8[0])
    assert rel(got, ref) < 1e-4 and rel(got, ref) < rel(y, ref) / 8, (rel(got, ref), rel(y, ref))


@pytest.mark.parametrize("C", [512, 256])
def test_conv0_mx6_planes(nrse_device, C):
    from nrse_amd import kernels as K
    dev = nrse_device
    B, L, k, s = 3, 8001, 10, 5
    T0 = (L - k) // s + 1
    rows = B * T0
    wav = torch.randn(B, L, device=dev) * 0.2
    w = torch.randn(C, 1, k, device=dev) * 0.3
    g = torch.randn(C, device=dev) * 0.1 + 1; b = torch.randn(C, device=dev) * 0.1
    out = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
    y8 = torch.empty(2, rows, C, device=dev, dtype=K.MX6)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    K.conv0_fwd(wav, w.view(C, k), g, b, out, mean, rstd, T0, k, s, 1e-5, y8=y8)
    torch.cuda.synchronize()
    same(y8[1], enc(out))
    y = F.conv1d(wav.double()[:, None], w.double(), stride=s).transpose(1, 2).reshape(rows, C)
    mu = y.mean(1); var = y.var(1, unbiased=False)
    ref = F.gelu((y - mu[:, None]) / torch.sqrt(var[:, None] + 1e-5) * g.double() + b.double()).cpu()
    got = out.double().cpu() + dec(y8[0])
    assert rel(got, ref) < 1e-4 and rel(got, ref) < rel(out, ref) / 8, (rel(got, ref), rel(out, ref))


@pytest.mark.parametrize("k,s,Tin", [(3, 2, 301), (2, 2, 300)])
def test_gemm_mx6_conv_segments(gen3, nrse_device, k, s, Tin):
    K = gen3
    B, Cin, C = 3, 512, 512
    Tout = (Tin - k) // s + 1
    x = F.gelu(torch.randn(B, Tin, Cin, device="cuda"))
    w = torch.randn(C, Cin, k, device="cuda") * 0.03
    x_hi = x.to(torch.bfloat16)
    x8 = torch.empty(2, B, Tin, Cin, device="cuda", dtype=K.MX6)
    K.cast_fp8(x - x_hi.float(), x8[0])
    K.cast_fp8(x_hi, x8[1])
    r = w.permute(0, 2, 1).reshape(C, k * Cin).contiguous()
    r_hi = r.to(torch.bfloat16)
    w8 = torch.empty(2, C, k * Cin, device="cuda", dtype=K.MX6)
    K.cast_fp8(r_hi, w8[0])
    K.split_lo8(r, w8[1])
    out = torch.empty(B * Tout, C, device="cuda")
    K.gemm(K.Operand(x_hi, True, s * Cin, z1=Tin * Cin), K.Operand(r_hi, True, k * Cin), out, Tout, C, k * Cin,
           ldc=C, batch=B, c_z1=Tout * C,
           a8=K.Operand(x8, True, s * Cin, z1=Tin * Cin, seg_stride=B * Tin * Cin),
           b8=K.Operand(w8, True, k * Cin, seg_stride=C * k * Cin), nseg8=2)
    torch.cuda.synchronize()

    def conv(a, ww):   # a [B, Tin, Cin], ww [C, k*Cin] (tap-major) -> [B*Tout, C], float64 CPU
        wk = torch.as_tensor(ww).double().cpu().view(C, k, Cin).permute(0, 2, 1)
        return F.conv1d(torch.as_tensor(a).double().cpu().permute(0, 2, 1), wk, stride=s).permute(0, 2, 1) \
            .reshape(B * Tout, C)

    ref = conv(x_hi, r_hi) + conv(dec(x8[0]), dec(w8[0])) + conv(dec(x8[1]), dec(w8[1]))
    assert rel(out, ref) < 2e-6, rel(out, ref)
    exact = conv(x, r)
    assert rel(out, exact) < rel(conv(x_hi, r_hi), exact) / 8, (rel(out, exact), rel(conv(x_hi, r_hi), exact))


def test_attention_mx6_context(nrse_device):
    from nrse_amd import kernels as K
    B, T, H = 2, 150, 4
    qkv = torch.randn(B * T, 3 * H * 64, device="cuda").to(torch.bfloat16)
    gate = torch.rand(B, H, T, device="cuda") + 0.5
    vec = torch.randn(H, 2 * T - 1, device="cuda") * 0.1
    ctx = torch.empty(B * T, H * 64, device="cuda", dtype=torch.bfloat16)
    ref_ctx = torch.empty_like(ctx)
    lse = torch.empty(B, H, T, device="cuda")
    c8 = torch.empty(B * T, H * 64, device="cuda", dtype=K.MX6)
    K.attn_fwd(qkv, gate, None, ref_ctx, lse, B, T, H, 0.1, 42, bias_vec=vec)
    K.attn_fwd(qkv, gate, None, ctx, lse, B, T, H, 0.1, 42, bias_vec=vec, ctx8=c8)
    torch.cuda.synchronize()
    assert torch.equal(ctx, ref_ctx)
    same(c8, enc(ctx))


def test_adamw_mx6_planes(nrse_device):
    from nrse_amd import kernels as K
    dev = "cuda"
    n, ne = 65536 + 4096, 40960
    p = torch.randn(n, device=dev) * 0.05
    g = torch.randn(n, device=dev) * 1e-3
    m, v = torch.randn(n, device=dev) * 1e-4, torch.rand(n, device=dev) * 1e-7
    t = p[:ne] + torch.randn(ne, device=dev) * 1e-4
    sumsq = torch.tensor([float((g.double() ** 2).sum())], device=dev, dtype=torch.float64)
    sh, lo = torch.empty(n, device=dev, dtype=torch.bfloat16), torch.empty(n, device=dev, dtype=torch.bfloat16)
    tsh, tlo = torch.empty(ne, device=dev, dtype=torch.bfloat16), torch.empty(ne, device=dev, dtype=torch.bfloat16)
    lo8 = torch.empty(n, device=dev, dtype=K.MX6)
    tlo8 = torch.empty(ne, device=dev, dtype=K.MX6)
    K.adamw(p, g, m, v, sh, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-5, step=3, max_norm=1.0,
            sumsq_buf=sumsq, shadow_lo=lo, ema_t=t, ema_shadow=tsh, ema_shadow_lo=tlo, ema_decay=0.997,
            shadow_lo8=lo8, ema_shadow_lo8=tlo8, zero_grad=True)
    torch.cuda.synchronize()
    same(lo8, enc(p - p.to(torch.bfloat16).float()))
    same(tlo8, enc(t - t.to(torch.bfloat16).float()))
