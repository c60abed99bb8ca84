"""Gated rel-pos attention kernels (MFMA bf16 and exact-f32 paths) vs a float64 PyTorch
reference of the same op ([TF]modeling_wavlm.py:164-184 + SDPA), forward and backward,
including attention dropout with the counter-hash masks (oracle/masks.py)."""
import numpy as np
import pytest
import torch

from oracle import masks as MK

pytestmark = pytest.mark.gpu


def reference(qkv, gate, bias, B, T, H, p, seed):
    """float64 autograd reference -> (ctx, lse, grads dict) for a random upstream dctx."""
    D = 64
    x = qkv.double().clone().requires_grad_(True)
    g = gate.double().clone().requires_grad_(True)
    bt = bias[:, :, :T].double().clone().requires_grad_(True)
    q = x[:, :H * D].view(B, T, H, D).transpose(1, 2)
    k = x[:, H * D:2 * H * D].view(B, T, H, D).transpose(1, 2)
    v = x[:, 2 * H * D:].view(B, T, H, D).transpose(1, 2)
    s = q @ k.transpose(-1, -2) / 8.0 + g[..., None] * bt[None]
    lse = torch.logsumexp(s, -1)
    pr = torch.softmax(s, -1)
    if p > 0:
        m = torch.from_numpy(MK.attn_dropout_mask(seed, p, (B, H, T, T))).double().to(qkv.device)
        pr = pr * m
    ctx = (pr @ v).transpose(1, 2).reshape(B * T, H * D)
    return x, g, bt, ctx, lse


def toeplitz_bias(H, T, dev):
    """The rel-pos bias depends on j - i only: a random vec [H, 2T-1] (the bf16 kernels' input)
    and the [H, T, Tb] table built from it (the f32 kernels' input)."""
    from nrse_amd import kernels as K
    vec = torch.randn(H, 2 * T - 1, device=dev)
    ii = torch.arange(T, device=dev)[:, None]
    jj = torch.arange(T, device=dev)[None, :]
    bias = torch.zeros(H, T, K.bias_ld(T), device=dev)
    bias[:, :, :T] = vec[:, jj - ii + T - 1]
    return vec, bias


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("T", [49, 130, 399, 599, 1001])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_fwd_bwd(nrse_device, dtype, T, p):
    from nrse_amd import kernels as K
    dev = nrse_device
    B, H = 2, 4
    torch.manual_seed(T)
    qkv = (torch.randn(B * T, 3 * H * 64, device=dev) * 0.5).to(dtype)
    gate = torch.rand(B, H, T, device=dev) + 1.0
    vec, bias = toeplitz_bias(H, T, dev)
    bv = vec if dtype == torch.bfloat16 else None
    seed = 77
    ctx = torch.empty(B * T, H * 64, device=dev, dtype=dtype)
    lse = torch.empty(B, H, T, device=dev)
    K.attn_fwd(qkv, gate, bias, ctx, lse, B, T, H, p, seed, bias_vec=bv)
    x, g, bt, rctx, rlse = reference(qkv, gate, bias, B, T, H, p, seed)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    e = ((ctx.double() - rctx).norm() / rctx.norm()).item()
    assert e < tol, e
    assert ((lse.double() - rlse).abs().max()).item() < 10 * tol
    # backward
    dctx = (torch.randn(B * T, H * 64, device=dev) * 0.5).to(dtype)
    rctx.backward(dctx.double())
    dqkv = torch.empty_like(qkv)
    dgate = torch.empty(B, H, T, device=dev)
    diag = torch.zeros(H, 2 * T - 1, device=dev)
    delta = torch.empty(B, H, T, device=dev)
    K.attn_bwd(qkv, gate, bias, ctx, dctx, lse, delta, dqkv, dgate, diag, B, T, H, p, seed, bias_vec=bv)
    for name, got, ref in (("dq", dqkv[:, :H * 64], x.grad[:, :H * 64]),
                           ("dk", dqkv[:, H * 64:2 * H * 64], x.grad[:, H * 64:2 * H * 64]),
                           ("dv", dqkv[:, 2 * H * 64:], x.grad[:, 2 * H * 64:]),
                           ("dgate", dgate, g.grad)):
        e = ((got.double() - ref).norm() / ref.norm()).item()
        assert e < 3 * tol, (name, e)
    # diag: sum over b, i of gate * dS along j - i  == d(bias)[h, i, j] summed per diagonal
    dbias = bt.grad  # [H, T, T]
    ref_diag = torch.zeros(H, 2 * T - 1, device=dev, dtype=torch.float64)
    ii = torch.arange(T, device=dev)[:, None]
    jj = torch.arange(T, device=dev)[None, :]
    idx = (jj - ii + T - 1).expand(T, T).reshape(-1)
    for h in range(H):
        ref_diag[h].index_add_(0, idx, dbias[h].reshape(-1))
    e = ((diag.double() - ref_diag).norm() / ref_diag.norm()).item()
    assert e < 3 * tol, ("diag", e)


@pytest.mark.parametrize("T", [49, 399, 599])
def test_attention_recorded_dropout_mask(nrse_device, T):
    """The forward records the probability-dropout keep bits (drop_mask, [B*H][key tile][4][Tp]
    u16) and the backward reads them instead of re-hashing: the bits are the counter hash's
    (oracle/masks.py attn_keep_mask), and the mask-reading backward equals the re-hashing one
    bit for bit."""
    from nrse_amd import kernels as K
    dev = nrse_device
    B, H, p, seed = 2, 4, 0.1, 123
    torch.manual_seed(T + 5)
    qkv = (torch.randn(B * T, 3 * H * 64, device=dev) * 0.5).to(torch.bfloat16)
    gate = torch.rand(B, H, T, device=dev) + 1.0
    vec, bias = toeplitz_bias(H, T, dev)
    ctx = torch.empty(B * T, H * 64, device=dev, dtype=torch.bfloat16)
    ctx2 = torch.empty_like(ctx)
    lse = torch.empty(B, H, T, device=dev)
    mask = torch.zeros(K.attn_mask_elems(B, T, H), device=dev, dtype=torch.int16)
    K.attn_fwd(qkv, gate, None, ctx, lse, B, T, H, p, seed, bias_vec=vec, drop_mask=mask)
    K.attn_fwd(qkv, gate, None, ctx2, lse, B, T, H, p, seed, bias_vec=vec)
    assert torch.equal(ctx, ctx2)
    # decode: word (bh, kt, g, q) bit 4t + r <-> key 64 kt + 16 t + 4 g + r
    nt = (T + 63) // 64
    Tp = nt * 64
    w = mask.view(B * H, nt, 4, Tp).to(torch.int32).cpu() & 0xFFFF
    bits = torch.stack([(w >> b) & 1 for b in range(16)], -1)          # [bh, kt, g, q, 4t + r]
    bits = bits.view(B * H, nt, 4, Tp, 4, 4).permute(0, 3, 1, 4, 2, 5)  # [bh, q, kt, t, g, r]
    keep = bits.reshape(B * H, Tp, nt * 64)[:, :T, :T].bool().numpy()
    ref = MK.attn_dropout_mask(seed, p, (B, H, T, T)).reshape(B * H, T, T) > 0
    assert (keep == ref).all()
    dctx = (torch.randn(B * T, H * 64, device=dev) * 0.5).to(torch.bfloat16)
    outs = []
    for m in (None, mask):
        dqkv = torch.empty_like(qkv)
        dgate = torch.empty(B, H, T, device=dev)
        diag = torch.zeros(H, 2 * T - 1, device=dev)
        delta = torch.empty(B, H, T, device=dev)
        K.attn_bwd(qkv, gate, None, ctx, dctx, lse, delta, dqkv, dgate, diag, B, T, H, p, seed, bias_vec=vec,
                   drop_mask=m)
        outs.append((dqkv, dgate, diag))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("T", [49, 399, 599])
def test_attention_precomputed_dropout_mask(nrse_device, T):
    """nrse_attn_dropout_mask writes exactly the keep bits the forward records (every word of a
    valid query), and the forward that reads them (mask_in) gives the hashing forward's ctx and
    lse bit for bit."""
    from nrse_amd import kernels as K
    dev = nrse_device
    B, H, p, seed = 2, 4, 0.1, 77
    torch.manual_seed(T + 9)
    qkv = (torch.randn(B * T, 3 * H * 64, device=dev) * 0.5).to(torch.bfloat16)
    gate = torch.rand(B, H, T, device=dev) + 1.0
    vec, _ = toeplitz_bias(H, T, dev)
    ctx1 = torch.empty(B * T, H * 64, device=dev, dtype=torch.bfloat16)
    ctx2 = torch.empty_like(ctx1)
    lse1 = torch.empty(B, H, T, device=dev)
    lse2 = torch.empty_like(lse1)
    rec = torch.zeros(K.attn_mask_elems(B, T, H), device=dev, dtype=torch.int16)
    K.attn_fwd(qkv, gate, None, ctx1, lse1, B, T, H, p, seed, bias_vec=vec, drop_mask=rec)
    pre = torch.full_like(rec, -1)
    K.attn_dropout_mask(pre, B, T, H, p, seed)
    nt = (T + 63) // 64
    Tp = nt * 64
    valid = (torch.arange(Tp, device=dev) < T).view(1, 1, 1, Tp).expand(B * H, nt, 4, Tp).reshape(-1)
    assert torch.equal(pre[valid], rec[valid])
    assert (pre[~valid] == 0).all()
    K.attn_fwd(qkv, gate, None, ctx2, lse2, B, T, H, p, seed, bias_vec=vec, drop_mask=pre, mask_in=True)
    assert torch.equal(ctx1, ctx2) and torch.equal(lse1, lse2)
