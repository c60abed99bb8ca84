"""Per-kernel parity on the GPU: each HIP kernel vs a float64 PyTorch reference of the same op
(floating-point kernels) or vs the committed golden fixtures (SNR mix)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a = a.double(); b = b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("C", [256, 512, 1024])
@pytest.mark.parametrize("xdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("gelu", [False, True])
def test_layernorm_fwd_bwd(nrse_device, C, xdt, gelu):
    from nrse_amd import kernels as K
    dev = nrse_device
    rows = 333
    x = (torch.randn(rows, C, device=dev) * 2 + 0.5).to(xdt)
    g = torch.randn(C, device=dev) * 0.1 + 1
    b = torch.randn(C, device=dev) * 0.1
    y = torch.empty(rows, C, device=dev)
    mean = torch.empty(rows, device=dev); rstd = torch.empty(rows, device=dev)
    K.ln_fwd(x, g, b, y, mean, rstd, 1e-5, gelu=gelu)
    xr = x.double().requires_grad_(True)
    gr, br = g.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = F.layer_norm(xr, (C,), gr, br, 1e-5)
    if gelu:
        ref = F.gelu(ref)
    assert rel(y, ref) < 1e-5
    dy = torch.randn(rows, C, device=dev)
    resid = torch.randn(rows, C, device=dev)
    dx = torch.empty(rows, C, device=dev)
    dg = torch.zeros(C, device=dev); db = torch.zeros(C, device=dev)
    K.ln_bwd(dy, x, g, mean, rstd, dx, beta=b, gelu=gelu, resid=resid, dgamma=dg, dbeta=db)
    ref.backward(dy.double())
    assert rel(dx, xr.grad + resid.double()) < 1e-5
    assert rel(dg, gr.grad) < 1e-5 and rel(db, br.grad) < 1e-5


@pytest.mark.parametrize("rows", [1, 3, 7, 9, 17, 4099])
@pytest.mark.parametrize("ydt", [torch.float32, torch.bfloat16])
def test_layernorm_fwd_f32_tail_rows(nrse_device, rows, ydt):
    """The f32-input forward (one row per wave, 4 per workgroup) at row counts that leave a
    workgroup's last waves idle: matches torch, and nothing past the last row is written."""
    from nrse_amd import kernels as K
    dev = nrse_device
    C = 1024
    x = torch.randn(rows, C, device=dev) * 3 - 0.25
    g = torch.randn(C, device=dev) * 0.1 + 1
    b = torch.randn(C, device=dev) * 0.1
    y = torch.full((rows + 1, C), 7.0, device=dev, dtype=ydt)   # one guard row past the end
    mean = torch.full((rows + 1,), 7.0, device=dev); rstd = torch.full((rows + 1,), 7.0, device=dev)
    K.ln_fwd(x, g, b, y[:rows], mean[:rows], rstd[:rows], 1e-5)
    ref = F.layer_norm(x.double(), (C,), g.double(), b.double(), 1e-5)
    assert rel(y[:rows].float(), ref) < (1e-5 if ydt == torch.float32 else 4e-3)
    assert torch.equal(y[rows].float(), torch.full((C,), 7.0, device=dev))
    assert mean[rows].item() == 7.0 and rstd[rows].item() == 7.0
    assert rel(mean[:rows], x.double().mean(1)) < 1e-6


@pytest.mark.parametrize("rows", [12768, 333, 5])
@pytest.mark.parametrize("dvdt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_layernorm_bwd_fused_dropout_colsum(nrse_device, rows, dvdt, p):
    """The LN backward's fused consumer equals the separate dropout_cast_colsum pass over dx
    (same mask, same cast, same column sums), and dx / dgamma / dbeta are unchanged by it."""
    from nrse_amd import kernels as K
    dev = nrse_device
    C = 1024
    x = torch.randn(rows, C, device=dev) * 2 + 0.5
    g = torch.randn(C, device=dev) * 0.1 + 1
    b = torch.randn(C, device=dev) * 0.1
    y = torch.empty(rows, C, device=dev)
    mean = torch.empty(rows, device=dev); rstd = torch.empty(rows, device=dev)
    K.ln_fwd(x, g, b, y, mean, rstd, 1e-5)
    dy = torch.randn(rows, C, device=dev)
    resid = torch.randn(rows, C, device=dev)
    outs = []
    for fused in (False, True):
        dx = torch.empty(rows, C, device=dev)
        dg = torch.zeros(C, device=dev); db = torch.zeros(C, device=dev)
        dv = torch.empty(rows, C, device=dev, dtype=dvdt); cs = torch.zeros(C, device=dev)
        if fused:
            K.ln_bwd(dy, x, g, mean, rstd, dx, resid=resid, dgamma=dg, dbeta=db, dv=dv, dv_colsum=cs, dv_p=p,
                     dv_seed=4321)
        else:
            K.ln_bwd(dy, x, g, mean, rstd, dx, resid=resid, dgamma=dg, dbeta=db)
            K.dropout_cast_colsum(dx, dv, cs, p, 4321)
        outs.append((dx, dg, db, dv, cs))
    (dx0, dg0, db0, dv0, cs0), (dx1, dg1, db1, dv1, cs1) = outs
    assert torch.equal(dx0, dx1) and torch.equal(dv0, dv1)
    assert rel(dg1, dg0) < 1e-6 and rel(db1, db0) < 1e-6 and rel(cs1, cs0) < 1e-6
    if p > 0:
        frac = float((dv1 == 0).float().mean())
        assert abs(frac - p) < (0.01 if rows > 1000 else 0.05)


@pytest.mark.parametrize("C,k,s", [(256, 3, 2), (512, 2, 2), (256, 5, 2), (512, 3, 1)])
def test_layernorm_bwd_col2im_and_bcast(nrse_device, C, k, s):
    """col2im dy: the two-tap path (k <= 2s: every feature-encoder conv) and the generic tap loop."""
    from nrse_amd import kernels as K, _lib
    dev = nrse_device
    B, Tin = 3, 52
    Tout = (Tin - k) // s + 1
    x = torch.randn(B * Tin, C, device=dev)
    g = torch.ones(C, device=dev); b = torch.zeros(C, device=dev)
    y = torch.empty_like(x); mean = torch.empty(B * Tin, device=dev); rstd = torch.empty_like(mean)
    K.ln_fwd(x, g, b, y, mean, rstd, 1e-5)
    G = torch.randn(B * Tout, k * C, device=dev)
    dy = torch.zeros(B, Tin, C, device=dev, dtype=torch.float64)
    Gv = G.double().view(B, Tout, k, C)
    for j in range(k):
        dy[:, j:j + s * (Tout - 1) + 1:s] += Gv[:, :, j]
    dx = torch.empty_like(x)
    K.ln_bwd(G, x, g, mean, rstd, dx, mode=_lib.DY_COL2IM, col=(k, s, Tout, Tin), rows=B * Tin)
    xr = x.double().requires_grad_(True)
    F.layer_norm(xr, (C,), None, None, 1e-5).backward(dy.view(B * Tin, C))
    assert rel(dx, xr.grad) < 1e-6
    # broadcast (time-mean) mode
    demb = torch.randn(B, C, device=dev)
    K.ln_bwd(demb, x, g, mean, rstd, dx, mode=_lib.DY_BCAST, bcast_t=Tin, dy_scale=1.0 / Tin, rows=B * Tin)
    xr.grad = None
    F.layer_norm(xr, (C,), None, None, 1e-5).view(B, Tin, C).mean(1).backward(demb.double())
    assert rel(dx, xr.grad) < 1e-6


@pytest.mark.parametrize("C,k,s", [(512, 3, 2), (512, 2, 2), (256, 3, 2)])
def test_layernorm_bwd_col2im_f32x_bf16dy(nrse_device, C, k, s):
    """The split-weight conv stack's LN + GELU backward: f32 pre-activation x, bf16 two-tap col2im
    dy (the XF form, raw-word loads), against float64 autograd of the same bf16 dy values."""
    from nrse_amd import kernels as K, _lib
    dev = nrse_device
    B, Tin = 3, 52
    Tout = (Tin - k) // s + 1
    x = torch.randn(B * Tin, C, device=dev)
    g = 1 + 0.1 * torch.randn(C, device=dev); b = 0.1 * torch.randn(C, device=dev)
    y = torch.empty_like(x); mean = torch.empty(B * Tin, device=dev); rstd = torch.empty_like(mean)
    K.ln_fwd(x, g, b, y, mean, rstd, 1e-5)
    G = torch.randn(B * Tout, k * C, device=dev).to(torch.bfloat16)
    dy = torch.zeros(B, Tin, C, device=dev, dtype=torch.float64)
    Gv = G.double().view(B, Tout, k, C)
    for j in range(k):
        dy[:, j:j + s * (Tout - 1) + 1:s] += Gv[:, :, j]
    dx = torch.empty(B * Tin, C, device=dev, dtype=torch.bfloat16)
    dg = torch.zeros(C, device=dev); db = torch.zeros(C, device=dev)
    K.ln_bwd(G, x, g, mean, rstd, dx, mode=_lib.DY_COL2IM, col=(k, s, Tout, Tin), rows=B * Tin,
             dgamma=dg, dbeta=db, gelu=True, beta=b)
    xr = x.double().requires_grad_(True)
    gr, br = g.double().requires_grad_(True), b.double().requires_grad_(True)
    F.gelu(F.layer_norm(xr, (C,), gr, br, 1e-5)).backward(dy.view(B * Tin, C))
    assert rel(dx, xr.grad) < 1e-2   # bf16 output
    assert rel(dg, gr.grad) < 1e-5 and rel(db, br.grad) < 1e-5


@pytest.mark.parametrize("C,k", [(256, 10), (512, 10), (512, 8)])
def test_conv0_fwd_bwd(nrse_device, C, k):
    """conv0 + LN + GELU forward / backward against float64 autograd: the model's k = 10 (the
    compile-time-geometry kernels) and k = 8 (the runtime-k form)."""
    from nrse_amd import kernels as K
    dev = nrse_device
    B, L, s = 2, 4001, 5
    T0 = (L - k) // s + 1
    wav = torch.randn(B, L, device=dev)
    w = torch.randn(C, 1, k, device=dev) * 0.3
    g = torch.randn(C, device=dev) * 0.1 + 1; b = torch.randn(C, device=dev) * 0.1
    out = torch.empty(B * T0, C, device=dev)
    mean = torch.empty(B * T0, device=dev); rstd = torch.empty_like(mean)
    K.conv0_fwd(wav, w.view(C, k), g, b, out, mean, rstd, T0, k, s, 1e-5)
    wr = w.double().requires_grad_(True); gr = g.double().requires_grad_(True); br = b.double().requires_grad_(True)
    ref = F.conv1d(wav.double()[:, None], wr, stride=s)
    ref = F.gelu(F.layer_norm(ref.transpose(1, 2), (C,), gr, br, 1e-5)).reshape(B * T0, C)
    assert rel(out, ref) < 1e-5
    dy = torch.randn(B * T0, C, device=dev)
    dw = torch.zeros(C, k, device=dev); dg = torch.zeros(C, device=dev); db = torch.zeros(C, device=dev)
    K.conv0_bwd(wav, w.view(C, k), g, b, mean, rstd, dy, dw, dg, db, T0, k, s, None)
    ref.backward(dy.double())
    assert rel(dw, wr.grad.view(C, k)) < 1e-4
    assert rel(dg, gr.grad) < 1e-5 and rel(db, br.grad) < 1e-5


@pytest.mark.parametrize("C", [512, 256])
@pytest.mark.parametrize("split3", [False, True])
def test_conv0_fwd_mfma_bf16_outputs(nrse_device, C, split3):
    """conv0 forward with bf16 / split-bf16 outputs (the matrix-core kernel: split-bf16 operands,
    transposed product) against float64: the output within its storage precision, mean / rstd
    within the split contraction's ~2^-16."""
    from nrse_amd import kernels as K
    dev = nrse_device
    B, L, k, s = 3, 8001, 10, 5
    T0 = (L - k) // s + 1  # 1599 rows per utterance: the last 16-row block is partial
    wav = torch.randn(B, L, device=dev) * 0.2
    w = torch.randn(C, 1, k, device=dev) * 0.3
    g = torch.randn(C, device=dev) * 0.1 + 1; b = torch.randn(C, device=dev) * 0.1
    rows = B * T0
    out = torch.empty((3, rows, C) if split3 else (rows, C), device=dev, dtype=torch.bfloat16)
    mean = torch.empty(rows, device=dev); rstd = torch.empty_like(mean)
    K.conv0_fwd(wav, w.view(C, k), g, b, out, mean, rstd, T0, k, s, 1e-5, split3=split3)
    y = F.conv1d(wav.double()[:, None], w.double(), stride=s).transpose(1, 2).reshape(rows, C)
    mu = y.mean(1); var = y.var(1, unbiased=False)
    ref = F.gelu((y - mu[:, None]) / torch.sqrt(var[:, None] + 1e-5) * g.double() + b.double())
    assert rel(mean, mu) < 1e-5
    assert rel(rstd, 1 / torch.sqrt(var + 1e-5)) < 1e-5
    if split3:
        assert torch.equal(out[0], out[2])
        got = out[0].double() + out[1].double()
        assert rel(got, ref) < 5e-5
    else:
        assert rel(out, ref) < 4e-3


@pytest.mark.parametrize("C,ck,cs,dt", [(512, 3, 2, torch.bfloat16), (512, 2, 2, torch.float32),
                                         (256, 3, 2, torch.float32), (512, 4, 1, torch.float32)])
def test_conv0_bwd_col2im(nrse_device, C, ck, cs, dt):
    """conv0 backward with dy as the col2im fold of the next conv's dgrad output [B, Tout, ck*C]
    (the engine's form): two-tap path (ck <= 2cs) and the generic tap loop (ck = 4, cs = 1)."""
    from nrse_amd import kernels as K
    dev = nrse_device
    B, L, k, s = 3, 3001, 10, 5
    T0 = (L - k) // s + 1
    Tout = (T0 - ck) // cs + 1
    wav = torch.randn(B, L, device=dev)
    w = torch.randn(C, 1, k, device=dev) * 0.3
    g = torch.randn(C, device=dev) * 0.1 + 1; b = torch.randn(C, device=dev) * 0.1
    out = torch.empty(B * T0, C, device=dev)
    mean = torch.empty(B * T0, device=dev); rstd = torch.empty_like(mean)
    K.conv0_fwd(wav, w.view(C, k), g, b, out, mean, rstd, T0, k, s, 1e-5)
    col = (torch.randn(B * Tout, ck * C, device=dev)).to(dt)
    dyf = torch.zeros(B, T0, C, device=dev, dtype=torch.float64)
    cv = col.double().view(B, Tout, ck, C)
    for j in range(ck):
        dyf[:, j:j + cs * (Tout - 1) + 1:cs] += cv[:, :, j]
    wr = w.double().requires_grad_(True); gr = g.double().requires_grad_(True); br = b.double().requires_grad_(True)
    ref = F.conv1d(wav.double()[:, None], wr, stride=s)
    ref = F.gelu(F.layer_norm(ref.transpose(1, 2), (C,), gr, br, 1e-5))
    ref.backward(dyf)
    dw = torch.zeros(C, k, device=dev); dg = torch.zeros(C, device=dev); db = torch.zeros(C, device=dev)
    K.conv0_bwd(wav, w.view(C, k), g, b, mean, rstd, col, dw, dg, db, T0, k, s, (ck, cs, Tout))
    assert rel(dw, wr.grad.view(C, k)) < 1e-4
    assert rel(dg, gr.grad) < 1e-5 and rel(db, br.grad) < 1e-5


@pytest.mark.parametrize("C,mode", [(512, "col"), (256, "col"), (512, "direct")])
def test_conv0_bwd_bf16_matrix_core(nrse_device, C, mode):
    """The bf16 step's conv0 backward (matrix-core kernel: the conv recomputed by MFMA as the
    forward computes it, dW as split-bf16 MFMAs over 16-row chunks, LN sums across 4 waves) against
    float64 autograd, with the MFMA forward's mean / rstd as the step has them; a ragged last chunk."""
    from nrse_amd import kernels as K
    dev = nrse_device
    B, L, k, s = 3, 4003, 10, 5
    T0 = (L - k) // s + 1      # 799 rows per utterance: 2397 rows, the last 16-row chunk partial
    wav = torch.randn(B, L, device=dev) * 0.3
    w = torch.randn(C, 1, k, device=dev) * 0.3
    g = torch.randn(C, device=dev) * 0.1 + 1; b = torch.randn(C, device=dev) * 0.1
    out = torch.empty(B * T0, C, device=dev, dtype=torch.bfloat16)
    mean = torch.empty(B * T0, device=dev); rstd = torch.empty_like(mean)
    K.conv0_fwd(wav, w.view(C, k), g, b, out, mean, rstd, T0, k, s, 1e-5)
    if mode == "col":
        ck, cs = 3, 2
        Tout = (T0 - ck) // cs + 1
        dy = torch.randn(B * Tout, ck * C, device=dev).to(torch.bfloat16)
        dyf = torch.zeros(B, T0, C, device=dev, dtype=torch.float64)
        cv = dy.double().view(B, Tout, ck, C)
        for j in range(ck):
            dyf[:, j:j + cs * (Tout - 1) + 1:cs] += cv[:, :, j]
        colspec = (ck, cs, Tout)
    else:
        dy = torch.randn(B * T0, C, device=dev).to(torch.bfloat16)
        dyf = dy.double().view(B, T0, C)
        colspec = None
    wr = w.double().requires_grad_(True); gr = g.double().requires_grad_(True); br = b.double().requires_grad_(True)
    ref = F.conv1d(wav.double()[:, None], wr, stride=s)
    ref = F.gelu(F.layer_norm(ref.transpose(1, 2), (C,), gr, br, 1e-5))
    ref.backward(dyf)
    dw = torch.zeros(C, k, device=dev); dg = torch.zeros(C, device=dev); db = torch.zeros(C, device=dev)
    K.conv0_bwd(wav, w.view(C, k), g, b, mean, rstd, dy, dw, dg, db, T0, k, s, colspec)
    torch.cuda.synchronize()
    assert rel(dw, wr.grad.view(C, k)) < 1e-4, rel(dw, wr.grad.view(C, k))
    assert rel(dg, gr.grad) < 2e-5 and rel(db, br.grad) < 2e-5, (rel(dg, gr.grad), rel(db, br.grad))


def test_weight_norm_fwd_bwd(nrse_device):
    from nrse_amd import kernels as K
    dev = nrse_device
    H, G, Kk = 256, 16, 128
    cpg = H // G
    v = torch.randn(H, cpg, Kk, device=dev)
    gg = torch.rand(1, 1, Kk, device=dev) + 0.5
    wf = torch.empty(G, cpg, Kk * cpg, device=dev); wd = torch.empty_like(wf)
    norms = torch.empty(Kk, device=dev)
    K.weight_norm_fwd(gg, v, wf, wd, norms, H, cpg, Kk)
    vr = v.double().requires_grad_(True); gr = gg.double().requires_grad_(True)
    w = vr * (gr / vr.pow(2).sum(dim=(0, 1), keepdim=True).sqrt())       # [H, cpg, K]
    ref_wf = w.view(G, cpg, cpg, Kk).permute(0, 1, 3, 2).reshape(G, cpg, Kk * cpg)
    ref_wd = w.view(G, cpg, cpg, Kk).flip(-1).permute(0, 2, 3, 1).reshape(G, cpg, Kk * cpg)
    assert rel(wf, ref_wf) < 1e-6 and rel(wd, ref_wd) < 1e-6
    dWf = torch.randn_like(wf)
    dg = torch.zeros(1, 1, Kk, device=dev); dv = torch.zeros_like(v)
    K.weight_norm_bwd(dWf, gg, v, norms, dg, dv, torch.empty(Kk, device=dev), H, cpg, Kk)
    ref_wf.backward(dWf.double())
    assert rel(dv, vr.grad) < 1e-5 and rel(dg, gr.grad) < 1e-5


def test_batchnorm_relu_and_loss(nrse_device):
    from nrse_amd import kernels as K
    dev = nrse_device
    x = torch.randn(32, 300, device=dev) * 3 + 1
    w = torch.randn(300, device=dev); b = torch.randn(300, device=dev)
    rm = torch.zeros(300, device=dev); rv = torch.ones(300, device=dev)
    y = torch.empty_like(x); sm = torch.empty(300, device=dev); si = torch.empty(300, device=dev)
    K.bn_fwd(x, w, b, y, rm, rv, sm, si, True, True)
    xr = x.double().requires_grad_(True); wr = w.double().requires_grad_(True); br = b.double().requires_grad_(True)
    rm2 = torch.zeros(300, device=dev, dtype=torch.float64); rv2 = torch.ones_like(rm2)
    ref = torch.relu(F.batch_norm(xr, rm2, rv2, wr, br, training=True, momentum=0.1, eps=1e-5))
    assert rel(y, ref) < 1e-6 and rel(rm, rm2) < 1e-6 and rel(rv, rv2) < 1e-6
    dy = torch.randn_like(x)
    dx = torch.empty_like(x); dw = torch.zeros(300, device=dev); db = torch.zeros(300, device=dev)
    K.bn_bwd(dy, x, y, w, sm, si, dx, dw, db, True)
    ref.backward(dy.double())
    assert rel(dx, xr.grad) < 1e-5 and rel(dw, wr.grad) < 1e-5 and rel(db, br.grad) < 1e-5
    # BYOL loss fwd + bwd (src/models/byol.py:104-128)
    p = torch.randn(32, 1024, device=dev); z = torch.randn(32, 1024, device=dev)
    loss = torch.zeros(1, device=dev); dp = torch.empty_like(p); stats = torch.zeros(2, device=dev)
    K.byol_loss(p, z, loss, dp, stats)
    pr = p.double().requires_grad_(True)
    pn = F.normalize(pr + 1e-10, dim=1, eps=1e-10); zn = F.normalize(z.double() + 1e-10, dim=1, eps=1e-10)
    rl = 2 - 2 * torch.clamp((pn * zn).sum(1), -1, 1).mean()
    rl.backward()
    assert abs(float(loss) - float(rl)) < 1e-6 and rel(dp, pr.grad) < 1e-5


def test_adamw_clip_ema(nrse_device):
    from nrse_amd import kernels as K
    dev = nrse_device
    n = 100_003
    p = torch.randn(n, device=dev); g = torch.randn(n, device=dev) * 3
    m = torch.zeros(n, device=dev); v = torch.zeros(n, device=dev)
    sh = torch.empty(n, device=dev, dtype=torch.bfloat16)
    ss = torch.zeros(1, device=dev, dtype=torch.float64)
    K.sumsq(g, ss)
    assert abs(float(ss.sqrt()) - float(g.double().norm())) / float(g.double().norm()) < 1e-12
    pt = torch.nn.Parameter(p.clone())
    opt = torch.optim.AdamW([pt], lr=1e-3, weight_decay=1e-2)
    pt.grad = g.clone()
    torch.nn.utils.clip_grad_norm_([pt], max_norm=1.0)
    opt.step()
    K.adamw(p, g, m, v, sh, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, step=1, max_norm=1.0,
            sumsq_buf=ss)
    assert rel(p, pt.detach()) < 1e-6
    assert rel(sh.float(), p) < 1e-2
    t = torch.randn(n, device=dev)
    t_ref = 0.997 * t + 0.003 * p
    K.ema(t, p, None, 0.997)
    assert rel(t, t_ref) < 1e-6
    # split-weight mode: the AdamW / EMA kernels also write the lo plane bf16(x - hi), bit-equal to
    # nrse_split_bf16 of the updated f32 values
    for shadow_len in (n, 4096):
        p2, m2, v2 = p.clone()[:shadow_len], torch.zeros(shadow_len, device=dev), torch.zeros(shadow_len, device=dev)
        hi = torch.empty(shadow_len, device=dev, dtype=torch.bfloat16)
        lo = torch.empty_like(hi)
        K.adamw(p2, g[:shadow_len], m2, v2, hi, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2,
                step=1, max_norm=1.0, sumsq_buf=ss, shadow_lo=lo)
        h2, l2 = torch.empty_like(hi), torch.empty_like(hi)
        K.split_bf16(p2, h2, l2)
        assert torch.equal(hi, h2) and torch.equal(lo, l2)
        assert torch.equal(hi, p2.to(torch.bfloat16))
        assert rel(hi.double() + lo.double(), p2) < 3e-5 < rel(hi.float(), p2)
        t2 = torch.randn(shadow_len, device=dev)
        K.ema(t2, p2, hi, 0.997, shadow_lo=lo)
        K.split_bf16(t2, h2, l2)
        assert torch.equal(hi, h2) and torch.equal(lo, l2)


def test_adamw_fused_ema_matches_two_passes(nrse_device):
    """The target EMA fused into the AdamW pass (nrse_adamw_params.ema_t) equals nrse_adamw followed
    by nrse_ema on the updated weights, bit for bit, with the EMA range ending inside a float4 quad,
    on a quad boundary, in the scalar tail and shorter than one quad; shadows (bf16 and split-plane) included."""
    from nrse_amd import kernels as K
    dev = nrse_device
    n = 100_003
    g = torch.randn(n, device=dev) * 3
    ss = torch.zeros(1, device=dev, dtype=torch.float64)
    K.sumsq(g, ss)
    kw = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, step=3, max_norm=1.0, sumsq_buf=ss)
    base = torch.randn(n, device=dev)
    m0, v0 = torch.randn(n, device=dev) * 0.1, torch.rand(n, device=dev) * 0.01
    t0 = torch.randn(n, device=dev)
    for ne, split in ((n, False), (n - 1, True), (4 * 11111, False), (4 * 11111 + 3, True), (4 * 25000 + 2, False),
                      (3, False), (4, True)):
        outs = []
        for fused in (False, True):
            p, m, v, t = base.clone(), m0.clone(), v0.clone(), t0[:ne].clone()
            sh = torch.empty(n, device=dev, dtype=torch.bfloat16)
            tsh = torch.empty(ne, device=dev, dtype=torch.bfloat16)
            lo = torch.empty_like(sh) if split else None
            tlo = torch.empty_like(tsh) if split else None
            if fused:
                K.adamw(p, g, m, v, sh, shadow_lo=lo, ema_t=t, ema_shadow=tsh, ema_shadow_lo=tlo, ema_decay=0.997,
                        **kw)
            else:
                K.adamw(p, g, m, v, sh, shadow_lo=lo, **kw)
                K.ema(t, p[:ne], tsh, 0.997, shadow_lo=tlo)
            outs.append((p, m, v, t, sh, tsh) + ((lo, tlo) if split else ()))
        for a, b in zip(*outs):
            assert torch.equal(a, b), (ne, split)


def test_snr_mix_matches_reference_fixture(nrse_device):
    from nrse_amd import kernels as K
    z = np.load(os.path.join(GOLD, "snr_mix.npz"))
    dev = nrse_device
    for i in range(int(z["n_cases"])):
        s = torch.from_numpy(z[f"c{i}_speech"]).to(dev)[None]
        n = torch.from_numpy(z[f"c{i}_noise"]).to(dev)[None]
        snr = torch.tensor([float(z[f"c{i}_snr"])], device=dev)
        nlen = torch.tensor([n.shape[1]], device=dev, dtype=torch.int32)
        c_out = torch.empty_like(s); n_out = torch.empty_like(s)
        st = torch.empty(1, device=dev, dtype=torch.int32); ks = torch.empty(1, device=dev)
        K.snr_mix(s, n, nlen, snr, c_out, n_out, st, ks, K.SNR_PEAK_ZMUV)
        ok = int(z[f"c{i}_ok"]) == 1
        assert (int(st) == 0) == ok, (i, int(st))
        if ok:
            assert rel(c_out[0], torch.from_numpy(z[f"c{i}_clean_iv"]).to(dev)) < 1e-5
            assert rel(n_out[0], torch.from_numpy(z[f"c{i}_noisy_iv"]).to(dev)) < 1e-5
            K.snr_mix(s, n, nlen, snr, c_out, n_out, st, ks, K.SNR_RAW)
            assert rel(n_out[0], torch.from_numpy(z[f"c{i}_noisy_raw"]).to(dev)) < 1e-6


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_snr_mix_chunked_matches_single_workgroup(nrse_device, mode):
    """The chunked SNR mix (16 workgroups per pair, scratch partials) against the one-workgroup-
    per-pair form on a batch with tiled short noise, longer noise, a NaN speech pair, a silent
    noise pair and a silent speech pair: same status codes, same outputs (f64 sums reordered)."""
    from nrse_amd import kernels as K, _lib
    dev = nrse_device
    B, L, NS = 6, 48000, 60000
    g = torch.Generator(device=dev).manual_seed(4)
    s = torch.randn(B, L, device=dev, generator=g) * 0.1
    n = torch.randn(B, NS, device=dev, generator=g)
    nlen = torch.tensor([NS, 7001, 48000, 20000, 100, 33333], device=dev, dtype=torch.int32)
    s[2, 1234] = float("nan")
    n[3] = 0.0
    s[4] = 0.0
    snr = torch.tensor([4.0, 8.0, 0.0, 12.0, 4.0, -2.0], device=dev)
    outs = []
    for scratch in (torch.empty(B * K.SNR_SCRATCH_PER_PAIR, device=dev, dtype=torch.float64), None):
        c_out = torch.full_like(s, 7.0); n_out = torch.full_like(s, 7.0)
        st = torch.full((B,), -1, device=dev, dtype=torch.int32); ks = torch.empty(B, device=dev)
        _lib.call("nrse_snr_mix", K.ptr(s), K.ptr(n), K.ptr(nlen), n.stride(0), K.ptr(snr), K.ptr(c_out),
                  K.ptr(n_out), K.ptr(st), K.ptr(ks), K.ptr(scratch), B, L, mode, K.stream_ptr())
        outs.append((c_out, n_out, st, ks))
    (c1, n1, s1, k1), (c2, n2, s2, k2) = outs
    assert torch.equal(s1, s2), (s1, s2)
    assert int(s1[2]) == 1 and int(s1[4]) == 3 and int(s1[3]) == 4
    ok = s1 == 0
    assert rel(c1[ok], c2[ok]) < 1e-6 and rel(n1[ok], n2[ok]) < 1e-6 and rel(k1[ok], k2[ok]) < 1e-6
    assert float(c1[~ok].abs().max()) == 0.0 and float(n1[~ok].abs().max()) == 0.0


def test_health_flags(nrse_device):
    from nrse_amd import kernels as K
    x = torch.randn(10000, device=nrse_device)
    x[5] = float("nan"); x[7] = float("inf")
    st = torch.zeros(4, device=nrse_device)
    K.health(x, st)
    assert st[0] == 1 and st[1] == 1
    y = x.clone(); y[5] = 0; y[7] = 0
    assert abs(float(st[2]) - float(y.abs().sum())) / float(y.abs().sum()) < 1e-5
    assert float(st[3]) == float(y.abs().max())


def _gate_reference(x1, W, b, c, B, T, H):
    """WavLMAttention gate, [TF]modeling_wavlm.py:168-176 (float64)."""
    xh = x1.double().view(B, T, H, 64).permute(0, 2, 1, 3)                     # [B, H, T, 64]
    pr = F.linear(xh, W, b).view(B, H, T, 2, 4).sum(-1)
    ga, gb = torch.sigmoid(pr).chunk(2, dim=-1)
    return (ga * (gb * c.view(1, H, 1, 1) - 1.0) + 2.0).squeeze(-1)            # [B, H, T]


@pytest.mark.parametrize("xdt", [torch.float32, torch.bfloat16])
def test_gate_fwd_bwd(nrse_device, xdt):
    from nrse_amd import kernels as K
    dev = nrse_device
    B, T, H = 3, 77, 16
    x1 = torch.randn(B * T, H * 64, device=dev).to(xdt)
    W = torch.randn(8, 64, device=dev) * 0.2
    bv = torch.randn(8, device=dev) * 0.2
    c = torch.randn(H, device=dev)
    gate = torch.empty(B, H, T, device=dev)
    K.gate_fwd(x1, W, bv, c, gate, B, T, H)
    Wr, br, cr = (t.double().requires_grad_(True) for t in (W, bv, c))
    xr = x1.double().requires_grad_(True)
    ref = _gate_reference(xr, Wr, br, cr.view(1, H, 1, 1), B, T, H)
    assert rel(gate, ref) < 1e-6
    dgate = torch.randn(B, H, T, device=dev)
    dx1 = torch.randn(B * T, H * 64, device=dev)
    dx1_0 = dx1.clone()
    dW = torch.zeros(8, 64, device=dev); db = torch.zeros(8, device=dev); dc = torch.zeros(1, H, 1, 1, device=dev)
    K.gate_bwd(x1, W, bv, c.view(1, H, 1, 1), dgate, dx1, dW, db, dc, B, T, H)
    ref.backward(dgate.double())
    assert rel(dx1 - dx1_0, xr.grad) < 1e-5
    assert rel(dW, Wr.grad) < 1e-5 and rel(db, br.grad) < 1e-5 and rel(dc.view(-1), cr.grad) < 1e-5


@pytest.mark.parametrize("xdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,T,H", [(3, 77, 16), (4, 399, 16), (2, 50, 4)])
def test_gate_bwd_into_layernorm_bwd(nrse_device, xdt, B, T, H):
    """The step's form of the gate backward: nrse_gate_bwd_dp's per-(row, head) (dpa, dpb) added
    by the encoder LayerNorm backward as it reads dx1 gives the LN backward of the gate_bwd
    read-modify-write form (dx, dgamma, dbeta, the fused dropout consumer), and the same
    parameter gradients."""
    from nrse_amd import kernels as K
    dev = nrse_device
    C = H * 64
    rows = B * T
    x1 = torch.randn(rows, C, device=dev).to(xdt)
    W = torch.randn(8, 64, device=dev) * 0.2
    bv = torch.randn(8, device=dev) * 0.2
    c = torch.randn(H, device=dev)
    dgate = torch.randn(B, H, T, device=dev)
    dx1 = torch.randn(rows, C, device=dev)
    h = torch.randn(rows, C, device=dev)
    g = torch.randn(C, device=dev) * 0.1 + 1
    mean = h.mean(1); rstd = 1 / torch.sqrt(h.var(1, unbiased=False) + 1e-5)
    resid = torch.randn(rows, C, device=dev)
    outs = []
    for fused in (False, True):
        dW = torch.zeros(8, 64, device=dev); db = torch.zeros(8, device=dev); dc = torch.zeros(H, device=dev)
        dy = dx1.clone()
        kw = {}
        if fused:
            dp = torch.empty(rows, H, 2, device=dev)
            K.gate_bwd_dp(x1, W, bv, c, dgate, dp, dW, db, dc, B, T, H)
            kw = dict(gate_dp=dp, gate_w=W)
        else:
            K.gate_bwd(x1, W, bv, c, dgate, dy, dW, db, dc, B, T, H)
        dx = torch.empty(rows, C, device=dev)
        dv = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
        dg = torch.zeros(C, device=dev); dbe = torch.zeros(C, device=dev); dvc = torch.zeros(C, device=dev)
        K.ln_bwd(dy, h, g, mean, rstd, dx, resid=resid, dgamma=dg, dbeta=dbe, dv=dv, dv_colsum=dvc, dv_p=0.1,
                 dv_seed=3, **kw)
        outs.append((dx, dv.float(), dg, dbe, dvc, dW, db, dc))
    # (dv is bf16: a last-bit difference of dx may flip its rounding; the gate parameter gradients
    # dW / db / dc (5..7) are summed over rows by two different kernels, in different orders)
    for i, (a, b) in enumerate(zip(*outs)):
        assert rel(a, b) < (1e-4 if i == 1 else (1e-5 if i >= 5 else 1e-6)), (i, rel(a, b))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,C", [(12768, 1024), (333, 3072), (1000, 8), (77, 520)])
def test_colsum(nrse_device, dt, rows, C):
    from nrse_amd import kernels as K
    x = torch.randn(rows, C, device=nrse_device).to(dt)
    out = torch.full((C,), 0.5, device=nrse_device)
    K.colsum(x, out)
    assert rel(out, x.double().sum(0) + 0.5) < 1e-5


@pytest.mark.parametrize("M,N,Kd", [(32, 1024, 1024), (32, 2048, 2048), (32, 1024, 2048), (5, 256, 512)])
def test_small_m_split_k_linears(nrse_device, M, N, Kd):
    from nrse_amd import kernels as K
    dev = nrse_device
    x = torch.randn(M, Kd, device=dev); w = torch.randn(N, Kd, device=dev); b = torch.randn(N, device=dev)
    y = torch.full((M, N), 7.0, device=dev)
    K.linear_fwd_small(x, w, y, bias=b)
    assert rel(y, x.double() @ w.double().t() + b.double()) < 1e-5
    dy = torch.randn(M, N, device=dev)
    dx = torch.full((M, Kd), 7.0, device=dev)
    K.linear_dgrad_small(dy, w, dx)
    assert rel(dx, dy.double() @ w.double()) < 1e-5


@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_dropout_cast_colsum(nrse_device, odt, p):
    from nrse_amd import kernels as K
    dev = nrse_device
    x = torch.randn(1000, 1024, device=dev)
    ref = torch.empty(1000, 1024, device=dev, dtype=odt)
    K.dropout_cast(x, ref, p, 1234)                      # the standalone kernel defines the mask
    out = torch.empty_like(ref)
    cs = torch.zeros(1024, device=dev)
    K.dropout_cast_colsum(x, out, cs, p, 1234)
    assert torch.equal(out, ref)
    keep = (ref != 0) | (x == 0)
    exact = torch.where(keep, x.double() / (1 - p), torch.zeros_like(x, dtype=torch.float64))
    assert rel(cs, exact.sum(0)) < 1e-5


def test_split3_outputs(nrse_device):
    """NRSE_BF16X3 outputs of the LN forward and conv0 (the split-weight mode's conv stack):
    planes [hi | lo | hi] with hi = bf16(y), lo = bf16(y - hi), equal to the f32 output split."""
    from nrse_amd import kernels as K
    dev = nrse_device
    for xdt in (torch.float32, torch.bfloat16):
        rows, C = 1001, 512
        x = (torch.randn(rows, C, device=dev) * 2).to(xdt)
        g = torch.randn(C, device=dev) * 0.1 + 1
        b = torch.randn(C, device=dev) * 0.1
        y32 = torch.empty(rows, C, device=dev)
        m = torch.empty(rows, device=dev); r = torch.empty(rows, device=dev)
        K.ln_fwd(x, g, b, y32, m, r, 1e-5, gelu=True)
        y3 = torch.empty(3, rows, C, device=dev, dtype=torch.bfloat16)
        K.ln_fwd(x, g, b, y3, m, r, 1e-5, gelu=True, split3=True)
        hi, lo = torch.empty(rows, C, device=dev, dtype=torch.bfloat16), torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
        K.split_bf16(y32, hi, lo)
        assert torch.equal(y3[0], hi) and torch.equal(y3[1], lo) and torch.equal(y3[2], hi)
    B, L, k, s = 3, 16000, 10, 5
    T0 = (L - k) // s + 1
    wav = torch.randn(B, L, device=dev) * 0.1
    w = torch.randn(512, k, device=dev) * 0.3
    g = torch.randn(512, device=dev) * 0.1 + 1
    b = torch.randn(512, device=dev) * 0.1
    o32 = torch.empty(B * T0, 512, device=dev)
    m = torch.empty(B * T0, device=dev); r = torch.empty(B * T0, device=dev)
    K.conv0_fwd(wav, w, g, b, o32, m, r, T0, k, s, 1e-5)
    o3 = torch.empty(3, B * T0, 512, device=dev, dtype=torch.bfloat16)
    K.conv0_fwd(wav, w, g, b, o3, m, r, T0, k, s, 1e-5, split3=True)
    # conv0's split output comes from the matrix-core kernel (split-operand contraction), the f32
    # output from the exact VALU kernel: the planes carry the f32 result to ~2^-16
    assert torch.equal(o3[0], o3[2])
    assert rel(o3[0].double() + o3[1].double(), o32) < 3e-5
    assert (o3[1].float().abs() <= o3[0].float().abs() * 2 ** -8 + 1e-30).all()


@pytest.mark.parametrize("S,n,batch,acc", [(512, 3072, 1, False), (512, 3072, 1, True), (64, 4096, 1, False),
                                           (224, 796, 16, False), (130, 520, 2, True)])
def test_rows_reduce(nrse_device, S, n, batch, acc):
    """nrse_rows_reduce against float64 in both workgroup shapes (256-column groups; 64-column
    groups when the grid is small), into three destinations, accumulating or not, and the same
    bits on a second run."""
    from nrse_amd import kernels as K
    dev = nrse_device
    slab = torch.randn(batch, S, n, device=dev)
    n0, n1 = n // 2, n // 4
    n2 = n - n0 - n1
    base = [torch.randn(batch, m, device=dev) if acc else torch.zeros(batch, m, device=dev) for m in (n0, n1, n2)]
    outs = []
    for _ in range(2):
        d = [x.clone() for x in base]
        K.rows_reduce(slab, S, *d, batch=batch, accumulate=acc)
        outs.append(torch.cat(d, 1))
    ref = slab.double().sum(1) + torch.cat(base, 1).double()
    assert rel(outs[0], ref) < 1e-6
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("T,B", [(49, 4), (149, 32), (399, 32), (599, 7)])
def test_specaug_mask_device_matches_oracle(nrse_device, T, B):
    """ABI 10: the SpecAugment time masks drawn on the device (nrse_specaug_mask) equal the oracle's
    restatement (oracle/masks.py specaug_mask) bit for bit, for several seeds and the step's lengths;
    mask_prob 0 gives zeros."""
    from nrse_amd import kernels as K
    from oracle import masks as MK
    for seed in (1, 77, 0xDEADBEEF):
        m = torch.empty(B, T, device="cuda", dtype=torch.uint8)
        K.specaug_mask(m, 0.075, 10, 2, seed)
        torch.cuda.synchronize()
        ref = MK.specaug_mask(seed, B, T, 0.075, 10, 2)
        assert np.array_equal(m.cpu().numpy().astype(bool), ref), (T, seed)
        assert ref.any()
    m.fill_(7)
    K.specaug_mask(m, 0.0, 10, 2, 5)
    torch.cuda.synchronize()
    assert int(m.sum()) == 0


@pytest.mark.parametrize("T,prob,L,min_masks", [(10, 0.65, 10, 2), (12, 0.05, 5, 2), (37, 1.0, 10, 2), (23, 0.3, 1, 0)])
def test_specaug_mask_edge_cases_match_oracle(nrse_device, T, prob, L, min_masks):
    """The span count's clamps ([TF]modeling_wavlm.py _compute_mask_indices): one start only (T = L),
    min_masks forcing more spans than fit (n = T // L), mask_prob 1 (n capped at T // L), spans of
    length 1; and mask_length > T raises like the reference's ValueError."""
    from nrse_amd import kernels as K, _lib
    from oracle import masks as MK
    B = 5
    for seed in (3, 1234):
        m = torch.empty(B, T, device="cuda", dtype=torch.uint8)
        K.specaug_mask(m, prob, L, min_masks, seed)
        torch.cuda.synchronize()
        ref = MK.specaug_mask(seed, B, T, prob, L, min_masks)
        assert np.array_equal(m.cpu().numpy().astype(bool), ref), (T, prob, L, seed)
    with pytest.raises(_lib.NrseError, match="mask_length"):
        K.specaug_mask(torch.empty(B, 8, device="cuda", dtype=torch.uint8), 0.5, 10, 2, 1)
    with pytest.raises(ValueError):
        MK.specaug_mask(1, B, 8, 0.5, 10, 2)
