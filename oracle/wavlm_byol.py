"""ORACLE (test infrastructure only — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; never by the product path, which must run on libnrse_hip.so or fail).

fp32 PyTorch-eager CPU restatement of the reference BYOL-on-WavLM training step, written
fresh from the reference's algorithm (no transformers import). Pinned against golden
fixtures produced by the reference itself (tests/golden/make_golden.py) in
tests/test_oracle_golden.py.

Followed line by line:
  conv feature encoder      [TF]modeling_wavlm.py:712-720, 773-783
  feature projection        [TF]modeling_wavlm.py:93-105
  SpecAugment (time masks)  [TF]modeling_wavlm.py:985-1011 (mask indices are inputs here)
  positional conv           [TF]modeling_wavlm.py:48-90 (weight_norm dim=2)
  stable-LN encoder         [TF]modeling_wavlm.py:465-513 (LayerDrop decisions are inputs)
  layer                     [TF]modeling_wavlm.py:355-373
  gated rel-pos attention   [TF]modeling_wavlm.py:147-271, [TORCH]functional.py:6206 (SDPA)
  FFN                       [TF]modeling_wavlm.py:274-295
  time-mean shim            SURVEY.md §0.2 (documented deviation)
  heads                     src/models/multi_layer_heads.py:4-48
  BYOL forward / EMA        src/models/byol.py:62-97
  loss                      src/models/byol.py:104-128
  step                      train_byol.py:56-74 (zero_grad, backward, clip 1.0, AdamW, EMA)

Dropout masks: the counter hash of oracle/masks.py (identical to the HIP kernels) driven by
nrse_amd.rng site seeds; with every probability at 0 (the "det" arch) it is exactly the
reference's train-mode computation.
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "noise-robust-speech-embedding_amd"))
from nrse_amd import rng  # noqa: E402  (seed derivation only; no compute)

from . import masks  # noqa: E402


# ------------------------------------------------------------------------- relative buckets
def rel_bucket(rel: np.ndarray, num_buckets: int = 320, max_distance: int = 800) -> np.ndarray:
    """[TF]modeling_wavlm.py:253-271 in numpy; float32 log like torch's `.float()` path."""
    nb = num_buckets // 2
    out = (rel > 0).astype(np.int64) * nb
    rp = np.abs(rel)
    max_exact = nb // 2
    is_small = rp < max_exact
    with np.errstate(divide="ignore"):
        lg = np.log(rp.astype(np.float32) / np.float32(max_exact)).astype(np.float32)
    lg = (lg / np.float32(math.log(max_distance / max_exact))).astype(np.float32)
    lg = (lg * np.float32(nb - max_exact)).astype(np.float32)
    large = (np.float32(max_exact) + lg)
    large = np.where(np.isfinite(large), large, 0).astype(np.int64)
    large = np.minimum(large, nb - 1)
    return out + np.where(is_small, rp, large)


def bucket_vector(T: int, num_buckets: int = 320, max_distance: int = 800) -> np.ndarray:
    """bucket(j - i) for d = j - i in [-(T-1), T-1], index d + T - 1."""
    d = np.arange(-(T - 1), T, dtype=np.int64)
    return rel_bucket(d, num_buckets, max_distance)


def position_bias(E: torch.Tensor, T: int, nb: int, md: int) -> torch.Tensor:
    """compute_bias ([TF]modeling_wavlm.py:243-251): [H, T, T] from rel_attn_embed [nb, H]."""
    i = np.arange(T)[:, None]
    j = np.arange(T)[None, :]
    b = torch.from_numpy(rel_bucket(j - i, nb, md))
    return E[b].permute(2, 0, 1)


# ------------------------------------------------------------------------- operand rounding
# bf16-operand mode (set_operand_dtype(torch.bfloat16)) restates the numerics of the engine's bf16
# mode (nrse_amd/engine.py): GEMM / attention operands and the activations the engine stores in
# bf16 are rounded to bf16 (round-to-nearest-even), arithmetic and accumulation stay f32, the
# residual stream, master weights, norms and softmax statistics stay f32. Two rounding points:
#   _rf(x)  rounds in the forward pass (straight-through in backward): a bf16-stored activation or
#           GEMM operand whose gradient the engine keeps in f32;
#   _rg(x)  rounds the gradient in the backward pass: a tensor whose gradient the engine stores in
#           bf16 as the dY operand of the dgrad / wgrad GEMMs (dv, df1, dqkv, dctx, dS, dpre ...).
# Rounding sites (set_operand_dtype(dtype, sites=...) rounds only those; None = every site):
#   conv     conv1-6 implicit-GEMM operands and stored outputs
#   proj     feature-projection LN output and GEMM
#   posconv  pos-conv operands
#   qkv      the QKV GEMM (LN output, weights, stored q / k / v)
#   attn     the attention core (P for P V, stored context)
#   oproj    the out-proj GEMM
#   ffn_up   the FFN-up GEMM (LN output, weights, stored pre-activation and GELU output)
#   ffn_down the FFN-down GEMM weights
SITES = ("conv", "proj", "posconv", "qkv", "attn", "oproj", "ffn_up", "ffn_down")
# the engine's split-weight mode (bf16sw): every weight exact (the forward GEMMs multiply by the
# weights' hi + lo bf16 pair), the conv stack's activations exact too (split bf16 planes and f32
# pre-activations), every other activation operand rounded
SPLIT_WEIGHT_SITES = tuple(f"{s}:a" for s in SITES if s not in ("attn", "conv")) + ("attn",)
# the split-weight mode's fp8 form (the engine's default bf16sw, ABI 6): at these GEMM sites the
# weight correction x (w - w_hi) runs as fp8(x) times the fp8 plane fp8((w - w_hi) 2^e), scaled
# by 2^-e (nrse_gemm's a8 / b8 segment); at "conv" (ABI 7, conv1-6 over exact activations) both
# corrections: x_hi w_hi + 2^-c (fp8((x - x_hi) 2^c) fp8(w_hi) + fp8(x_hi) fp8((w - w_hi) 2^c)), c
# the engine's conv_lo8_exp (conv_lo8_exponent; 11 at the seeded init); set_split8(sites, e, c) switches it on
SPLIT8_SITES = ("qkv", "oproj", "ffn_up", "ffn_down", "conv")
CONV_LO8_EXP = 11   # nrse_amd/engine.py CONV_LO8_EXP: conv_lo8_exponent at gamma = 1, beta = 0
_OPERAND_DTYPE = None
_SITES = None
_SPLIT8 = None   # (frozenset of sites, exponent e, conv exponent c) or None


def set_operand_dtype(dtype, sites=None) -> None:
    global _OPERAND_DTYPE, _SITES
    _OPERAND_DTYPE = None if dtype in (None, torch.float32) else dtype
    _SITES = None if sites is None else frozenset(sites)
    if _SITES is not None and not {x.split(":")[0] for x in _SITES} <= set(SITES):
        raise ValueError(f"unknown rounding sites {sorted(_SITES)}")


def _site_on(site, kind=None) -> bool:
    """Rounding on at `site`; a sites entry "name:w" / "name:a" selects only that site's weight /
    activation operands (kind "w" / "a")."""
    if _OPERAND_DTYPE is None:
        return False
    if _SITES is None or site is None or site in _SITES:
        return True
    if kind == "p":   # a stored pre-activation: an activation ("a") unless selected on its own
        return f"{site}:a" in _SITES or f"{site}:p" in _SITES
    return kind is not None and f"{site}:{kind}" in _SITES


def operand_dtype():
    return _OPERAND_DTYPE


def set_split8(sites=None, exponent: int = 0, conv_exponent: int = CONV_LO8_EXP) -> None:
    """The fp8 correction form of the split-weight mode at `sites` (None: off), lo8_exp = exponent
    (engine: ByolEngine._set_lo8_planes), the conv stack's exponent conv_exponent."""
    global _SPLIT8
    _SPLIT8 = None if sites is None else (frozenset(sites), int(exponent), int(conv_exponent))


def _q8(t: torch.Tensor, e: int) -> torch.Tensor:
    """A correction operand as the engine stores it, scaled back: fp8(t 2^e) 2^-e."""
    return fp8_e4m3(t * 2.0 ** e) * 2.0 ** -e


def _conv_split8(x: torch.Tensor, w: torch.Tensor, stride: int, c: int) -> torch.Tensor:
    """The engine's conv1-6 GEMM in the fp8 split form (one bf16 K segment + two fp8 segments over
    the activations' planes [fp8((x - x_hi) 2^c) | fp8(x_hi)] and the weights' [fp8(w_hi) |
    fp8((w - w_hi) 2^c)], scaled by 2^-c)."""
    bf = torch.bfloat16
    x_hi, w_hi = x.to(bf).to(x.dtype), w.to(bf).to(w.dtype)
    corr = (F.conv1d(fp8_e4m3((x - x_hi) * 2.0 ** c), fp8_e4m3(w_hi), stride=stride) +
            F.conv1d(fp8_e4m3(x_hi), fp8_e4m3((w - w_hi) * 2.0 ** c), stride=stride))
    return F.conv1d(x_hi, w_hi, stride=stride) + corr * 2.0 ** -c


def fp8_e4m3(x: torch.Tensor) -> torch.Tensor:
    """OCP e4m3fn rounding (nearest even) of x saturated at +-448, as nrse_cast_fp8 / the kernels'
    fp8x4 (torch's own cast gives NaN beyond the range), back in x's dtype."""
    return x.clamp(-448.0, 448.0).to(torch.float8_e4m3fn).to(x.dtype)


def lo8_exponent(weights) -> int:
    """The engine's lo8_exp: floor(log2(224 / (2^-8 max|w|))) over the fp8-corrected weights."""
    W = max(float(w.detach().abs().max()) for w in weights)
    return max(-60, min(60, int(math.floor(math.log2(224.0 * 256.0 / W))))) if W > 0 else 0


def conv_lo8_exponent(P: dict, a) -> int:
    """The engine's conv-stack exponent (ABI 10, ByolEngine._conv_plane_bound): the conv planes carry
    residuals of the activations feeding conv 1..n-1 -- GELU(LayerNorm_C) outputs, bounded by
    sqrt(C) max|gamma| + max|beta| -- and of the conv weights; e = floor(log2(224 / (2^-8 bound)))."""
    B = 0.0
    for i in range(len(a.conv_dim) - 1):
        pre = f"feature_extractor.conv_layers.{i}.layer_norm."
        B = max(B, math.sqrt(a.conv_dim[i]) * float(P[pre + "weight"].detach().abs().max())
                + float(P[pre + "bias"].detach().abs().max()))
    for i in range(1, len(a.conv_dim)):
        B = max(B, float(P[f"feature_extractor.conv_layers.{i}.conv.weight"].detach().abs().max()))
    return max(-60, min(60, int(math.floor(math.log2(224.0 * 256.0 / B))))) if B > 0 else 0


class _RoundFwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dt):
        return x.to(dt).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _RoundGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dt):
        ctx.dt = dt
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dt).to(g.dtype), None


def _rf(x: torch.Tensor, site=None, kind="a") -> torch.Tensor:
    return _RoundFwd.apply(x, _OPERAND_DTYPE) if _site_on(site, kind) else x


def _rg(x: torch.Tensor, site=None) -> torch.Tensor:
    return _RoundGrad.apply(x, _OPERAND_DTYPE) if _site_on(site, "a") else x


def _lin(x, w, b=None, *, store=False, site=None):
    """Linear on the GEMM path: rounded operands, f32 accumulate + bias epilogue, the output's
    gradient rounded (it is the dY operand of this GEMM's dgrad / wgrad); store=True when the
    engine also stores the output itself in bf16 (QKV, FFN-up pre-activation). Under set_split8,
    at its sites: x_b w_hi + 2^-e fp8(x_b) fp8((w - w_hi) 2^e), the correction outside autograd
    (the engine's backward uses w_hi alone, as the straight-through w_hi here does)."""
    y = _rg(_linear_core(_rf(x, site), w, b, site), site)
    return _rf(y, site) if store else y


def _linear_core(xr, w, b, site):
    """xr (rounded operand) @ w^T + b at `site`: the weight rounded as the mode says, or under
    set_split8 the fp8 correction form x_b w_hi + 2^-e fp8(x_b) fp8((w - w_hi) 2^e)."""
    if _SPLIT8 is not None and site in _SPLIT8[0]:
        e = _SPLIT8[1]
        with torch.no_grad():
            w_hi = w.to(torch.bfloat16).to(w.dtype)
            corr = F.linear(_q8(xr.detach(), 0), _q8(w - w_hi, e))
        return F.linear(xr, _RoundFwd.apply(w, torch.bfloat16), b) + corr
    return F.linear(xr, _rf(w, site, "w"), b)


# ------------------------------------------------------------------------- pieces
def _drop(x: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    if p <= 0:
        return x
    m = torch.from_numpy(masks.dropout_mask(seed, p, tuple(x.shape)))
    return x * m


def conv_stack(P: dict, a, wav: torch.Tensor) -> torch.Tensor:
    """wav [B, L] -> extract_features [B, T, C]."""
    x = wav[:, None]
    for i, (k, s) in enumerate(zip(a.conv_kernel, a.conv_stride)):
        pre = f"feature_extractor.conv_layers.{i}."
        if i == 0:   # direct conv from the f32 waveform (engine: conv0 kernel, f32 weights)
            x = F.conv1d(x, P[pre + "conv.weight"], stride=s)
        else:        # implicit GEMM, bf16 operands, pre-LN output stored in the compute dtype
            xin, w = _rf(x, "conv"), _rf(P[pre + "conv.weight"], "conv", "w")
            y = F.conv1d(xin, w, stride=s)
            if _SPLIT8 is not None and "conv" in _SPLIT8[0]:   # forward value only (gradient as before)
                with torch.no_grad():
                    d = _conv_split8(xin, w, s, _SPLIT8[2]) - y
                y = y + d
            x = _rf(_rg(y, "conv"), "conv", "p")
        x = F.layer_norm(x.transpose(1, 2), (x.shape[1],), P[pre + "layer_norm.weight"], P[pre + "layer_norm.bias"],
                         a.eps).transpose(1, 2)
        x = _rg(_rf(F.gelu(x), "conv"), "conv")
    return x.transpose(1, 2)


def weight_norm_w(g: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """torch.nn.utils.parametrizations.weight_norm(dim=2): w = g * v / ||v|| (norm over 0,1)."""
    return v * (g / v.pow(2).sum(dim=(0, 1), keepdim=True).sqrt())


def gate(P: dict, pre: str, x1: torch.Tensor, heads: int) -> torch.Tensor:
    """[TF]modeling_wavlm.py:164-176: gate [B, H, T]."""
    B, T, H = x1.shape
    gh = x1.view(B, T, heads, -1).permute(0, 2, 1, 3)
    proj = F.linear(gh, P[pre + "gru_rel_pos_linear.weight"], P[pre + "gru_rel_pos_linear.bias"])
    proj = proj.view(B, heads, T, 2, 4).sum(-1)
    ga, gb = torch.sigmoid(proj).chunk(2, dim=-1)
    c = P[pre + "gru_rel_pos_const"].view(1, heads, 1, 1)
    return (ga * (gb * c - 1.0) + 2.0).squeeze(-1)


class _FlashBf16(torch.autograd.Function):
    """Gated rel-pos attention core in the engine's bf16 numerics (attention_mfma.hip): q, k, v
    bf16; S = q k^T / 8 + gate * bias and the softmax in f32; P rounded for P V; the context stored
    in bf16 and its incoming gradient dO in bf16. Backward as the flash kernels compute it:
    delta = rowsum(dO * O) from the bf16-stored O, dS = P (dP - delta) in f32, dV = P_bf16^T dO,
    dQ / dK from bf16 dS, the gate and rel-pos bias gradients from the f32 dS."""

    @staticmethod
    def forward(ctx, q, k, v, g, pbias, dt):
        hd = q.shape[-1]
        s = (q @ k.transpose(-1, -2)) / math.sqrt(hd) + g[..., None] * pbias[None]
        p = torch.softmax(s, dim=-1)
        o = (p.to(dt).float() @ v).to(dt).float()
        ctx.save_for_backward(q, k, v, g, pbias, p, o)
        ctx.dt = dt
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, g, pbias, p, o = ctx.saved_tensors
        dt = ctx.dt
        hd = q.shape[-1]
        do = do.to(dt).float()
        dp = do @ v.transpose(-1, -2)
        delta = (do * o).sum(-1, keepdim=True)
        ds = p * (dp - delta)
        dv = p.to(dt).float().transpose(-1, -2) @ do
        ds16 = ds.to(dt).float()
        dq = ds16 @ k / math.sqrt(hd)
        dk = ds16.transpose(-1, -2) @ q / math.sqrt(hd)
        dg = (ds * pbias[None]).sum(-1)
        dbias = (ds * g[..., None]).sum(0)
        return dq, dk, dv, dg, dbias, None


def attention(P: dict, a, li: int, x1: torch.Tensor, pbias: torch.Tensor, fseed: int, train: bool):
    B, T, H = x1.shape
    nh, hd = a.heads, a.head_dim
    pre = f"encoder.layers.{li}.attention."
    q = _lin(x1, P[pre + "q_proj.weight"], P[pre + "q_proj.bias"], store=True, site="qkv")
    k = _lin(x1, P[pre + "k_proj.weight"], P[pre + "k_proj.bias"], store=True, site="qkv")
    v = _lin(x1, P[pre + "v_proj.weight"], P[pre + "v_proj.bias"], store=True, site="qkv")
    q = q.view(B, T, nh, hd).transpose(1, 2)
    k = k.view(B, T, nh, hd).transpose(1, 2)
    v = v.view(B, T, nh, hd).transpose(1, 2)
    g = gate(P, pre, x1, nh)                               # [B, nh, T]
    if _site_on("attn") and not (train and a.attention_dropout > 0):
        ctx = _FlashBf16.apply(q, k, v, g, pbias, _OPERAND_DTYPE).transpose(1, 2).reshape(B, T, H)
        return _lin(ctx, P[pre + "out_proj.weight"], P[pre + "out_proj.bias"], site="oproj")
    s = (q @ k.transpose(-1, -2)) / math.sqrt(hd) + g[..., None] * pbias[None]
    p = torch.softmax(s, dim=-1)
    if train:
        if a.attention_dropout > 0:  # the pair-hash mask of the attention kernels (masks.attn_keep_mask)
            p = p * torch.from_numpy(masks.attn_dropout_mask(rng.site_seed(fseed, rng.site_attn_probs(li)),
                                                             a.attention_dropout, tuple(p.shape)))
    ctx = (p @ v).transpose(1, 2).reshape(B, T, H)
    return _lin(ctx, P[pre + "out_proj.weight"], P[pre + "out_proj.bias"], site="oproj")


def encoder_forward(P: dict, a, wav: torch.Tensor, *, train: bool = False, fseed: int = 0,
                    layer_skip=None, mask_time=None) -> torch.Tensor:
    """WavLMModel.forward ([TF]modeling_wavlm.py:1032-1096) -> last_hidden_state [B, T, H]."""
    feats = conv_stack(P, a, wav)
    B, T, C = feats.shape
    xn = _rf(F.layer_norm(feats, (C,), P["feature_projection.layer_norm.weight"],
                          P["feature_projection.layer_norm.bias"], a.eps), "proj")
    h = _lin(xn, P["feature_projection.projection.weight"], P["feature_projection.projection.bias"], site="proj")
    if train:
        h = _drop(h, a.feat_proj_dropout, rng.site_seed(fseed, rng.SITE_FEAT_PROJ))
    if train and mask_time is not None:
        m = torch.as_tensor(mask_time, dtype=torch.bool)
        h = torch.where(m[..., None], P["masked_spec_embed"].view(1, 1, -1), h)
    pre = "encoder.pos_conv_embed.conv."
    w = weight_norm_w(P[pre + "parametrizations.weight.original0"], P[pre + "parametrizations.weight.original1"])
    pc = _rg(F.conv1d(_rf(h, "posconv").transpose(1, 2), _rf(w, "posconv", "w"), P[pre + "bias"],
                      padding=a.pos_kernel // 2, groups=a.pos_groups), "posconv")
    if a.pos_kernel % 2 == 0:
        pc = pc[:, :, :-1]
    h = h + F.gelu(pc).transpose(1, 2)
    if train:
        h = _drop(h, a.hidden_dropout, rng.site_seed(fseed, rng.SITE_POS))
    pbias = position_bias(P["encoder.layers.0.attention.rel_attn_embed.weight"], T, a.num_buckets, a.max_distance)
    for li in range(a.layers):
        if train and layer_skip is not None and layer_skip[li]:
            continue
        pre = f"encoder.layers.{li}."
        x1 = _rf(F.layer_norm(h, (h.shape[-1],), P[pre + "layer_norm.weight"], P[pre + "layer_norm.bias"], a.eps),
                 "qkv")
        att = attention(P, a, li, x1, pbias, fseed, train)
        if train:
            att = _drop(att, a.hidden_dropout, rng.site_seed(fseed, rng.site_attn_out(li)))
        h = h + att
        x2 = _rf(F.layer_norm(h, (h.shape[-1],), P[pre + "final_layer_norm.weight"],
                              P[pre + "final_layer_norm.bias"], a.eps), "ffn_up")
        f = _rf(F.gelu(_rg(_linear_core(x2, P[pre + "feed_forward.intermediate_dense.weight"],
                                        P[pre + "feed_forward.intermediate_dense.bias"], "ffn_up"), "ffn_up")), "ffn_up")
        if train:
            f = _drop(f, a.activation_dropout, rng.site_seed(fseed, rng.site_act(li)))
        f = _lin(f, P[pre + "feed_forward.output_dense.weight"], P[pre + "feed_forward.output_dense.bias"], site="ffn_down")
        if train:
            f = _drop(f, a.hidden_dropout, rng.site_seed(fseed, rng.site_ffn_out(li)))
        h = h + f
    return F.layer_norm(h, (h.shape[-1],), P["encoder.layer_norm.weight"], P["encoder.layer_norm.bias"], a.eps)


def bn_train(x, w, b, run_mean, run_var, momentum=0.1, eps=1e-5, train=True):
    """nn.BatchNorm1d: batch stats (biased var) in train mode, running stats updated with the
    unbiased var; running stats in eval mode."""
    return F.batch_norm(x, run_mean, run_var, w, b, training=train, momentum=momentum, eps=eps)


def projector(P: dict, x, buf: dict, train=True):
    x = F.linear(x, P["layers.0.weight"], P["layers.0.bias"])
    x = torch.relu(bn_train(x, P["layers.1.weight"], P["layers.1.bias"], buf["layers.1.running_mean"],
                            buf["layers.1.running_var"], train=train))
    x = F.linear(x, P["layers.3.weight"], P["layers.3.bias"])
    return bn_train(x, P["layers.4.weight"], P["layers.4.bias"], buf["layers.4.running_mean"],
                    buf["layers.4.running_var"], train=train)


def predictor(P: dict, x, buf: dict, train=True):
    x = F.linear(x, P["layers.0.weight"], P["layers.0.bias"])
    x = torch.relu(bn_train(x, P["layers.1.weight"], P["layers.1.bias"], buf["layers.1.running_mean"],
                            buf["layers.1.running_var"], train=train))
    x = F.linear(x, P["layers.3.weight"], P["layers.3.bias"])
    x = torch.relu(bn_train(x, P["layers.4.weight"], P["layers.4.bias"], buf["layers.4.running_mean"],
                            buf["layers.4.running_var"], train=train))
    return F.linear(x, P["layers.6.weight"], P["layers.6.bias"])


def byol_loss(p: torch.Tensor, z: torch.Tensor) -> torch.Tensor:
    """src/models/byol.py:104-128."""
    p = F.normalize(p + 1e-10, dim=1, eps=1e-10)
    z = F.normalize(z + 1e-10, dim=1, eps=1e-10)
    s = torch.clamp((p * z).sum(1), -1.0, 1.0)
    return 2 - 2 * s.mean()


def _flat_key(gname: str, name: str) -> str:
    return {"encoder": "online_encoder.model.", "projector": "online_projector.",
            "predictor": "online_predictor."}[gname] + name


def split_flat(layout, flat: torch.Tensor, target: bool = False, leaves: bool = False) -> dict:
    """{'encoder': {...}, 'projector': {...}, 'predictor': {...}} of module-relative views.
    leaves=True: each view becomes its own autograd leaf (a module's parameters), so backward
    accumulates per-tensor gradients instead of one flat-sized gradient per slice."""
    out = {"encoder": {}, "projector": {}, "predictor": {}}
    for gname, s in layout.specs:
        if target and gname == "predictor":
            continue
        off, n, shp = layout.offsets[_flat_key(gname, s.name)]
        v = flat[off:off + n].view(shp)
        out[gname][s.name] = v.detach().requires_grad_(True) if leaves else v
    return out


def gather_grad(layout, params: dict) -> torch.Tensor:
    """Flat gradient in the parameter layout from a split_flat(..., leaves=True) dict."""
    g = torch.zeros(layout.numel)
    for gname, d in params.items():
        for name, t in d.items():
            off, n, _ = layout.offsets[_flat_key(gname, name)]
            if t.grad is not None:
                g[off:off + n] = t.grad.reshape(-1)
    return g


def head_buffers(proj_dim: int, pred_dim: int) -> dict:
    def bn(c):
        return {"running_mean": torch.zeros(c), "running_var": torch.ones(c)}
    return {
        "online_projector": {f"layers.{i}.{k}": v for i in (1, 4) for k, v in bn(proj_dim).items()},
        "target_projector": {f"layers.{i}.{k}": v for i in (1, 4) for k, v in bn(proj_dim).items()},
        "online_predictor": {**{f"layers.1.{k}": v for k, v in bn(pred_dim).items()},
                             **{f"layers.4.{k}": v for k, v in bn(pred_dim).items()}},
    }


class OracleState:
    """Full training state of the oracle: flat online / target params + AdamW moments."""

    def __init__(self, layout, flat: torch.Tensor):
        self.layout = layout
        self.online = flat.clone()
        self.target = flat[:layout.ema_numel].clone()
        self.m = torch.zeros_like(self.online)
        self.v = torch.zeros_like(self.online)
        self.step = 0
        self.buffers = head_buffers(layout.proj_dim, layout.pred_dim)


def forward(state: OracleState, clean, noisy, *, train: bool, step_seed: int = 0, online_flat=None,
            layer_skip=(None, None), mask_time=(None, None), time_mean: bool = True, online_params=None):
    """BYOLSpeechModel.forward (src/models/byol.py:75-97) -> (online_pred, target_proj, emb)."""
    a = state.layout.arch
    on = online_params if online_params is not None else \
        split_flat(state.layout, state.online if online_flat is None else online_flat)
    tg = split_flat(state.layout, state.target, target=True)
    h = encoder_forward(on["encoder"], a, clean, train=train, fseed=rng.forward_seed(step_seed, 0),
                        layer_skip=layer_skip[0], mask_time=mask_time[0])
    emb = h.mean(1) if time_mean else h
    proj = projector(on["projector"], emb, state.buffers["online_projector"], train)
    pred = predictor(on["predictor"], proj, state.buffers["online_predictor"], train)
    with torch.no_grad():
        ht = encoder_forward(tg["encoder"], a, noisy, train=train, fseed=rng.forward_seed(step_seed, 1),
                             layer_skip=layer_skip[1], mask_time=mask_time[1])
        tproj = projector(tg["projector"], ht.mean(1), state.buffers["target_projector"], train)
    return pred, tproj, emb


def train_step(state: OracleState, clean, noisy, *, lr: float, weight_decay: float, ema_decay: float,
               max_norm: float = 1.0, step_seed: int = 0, layer_skip=(None, None), mask_time=(None, None)):
    """One iteration of train_byol.py:56-74; returns dict of diagnostics."""
    params = split_flat(state.layout, state.online, leaves=True)
    pred, tproj, emb = forward(state, clean, noisy, train=True, step_seed=step_seed, online_params=params,
                               layer_skip=layer_skip, mask_time=mask_time)
    loss = byol_loss(pred, tproj)
    loss.backward()
    g = gather_grad(state.layout, params)
    # clip_grad_norm_: norm of the per-parameter norms ([TORCH]nn/utils/clip_grad.py); a single
    # fp32 norm over the 3e8-element flat vector loses the small entries.
    per = [g[off:off + n].norm() for (off, n, _) in state.layout.offsets.values()]
    total_norm = torch.stack(per).norm()
    coef = min(1.0, max_norm / (float(total_norm) + 1e-6))
    g = g * coef
    # torch.optim.AdamW (decoupled wd, bias-corrected, eps outside sqrt)
    state.step += 1
    b1, b2, eps = 0.9, 0.999, 1e-8
    w = state.online * (1 - lr * weight_decay)
    state.m.mul_(b1).add_(g, alpha=1 - b1)
    state.v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** state.step
    bc2 = 1 - b2 ** state.step
    denom = state.v.sqrt() / math.sqrt(bc2) + eps
    state.online = w - (lr / bc1) * state.m / denom
    # EMA of encoder + projector parameters (src/models/byol.py:62-73)
    state.target = ema_decay * state.target + (1 - ema_decay) * state.online[:state.layout.ema_numel]
    return {"loss": float(loss.detach()), "grad_norm": float(total_norm), "pred": pred.detach(), "tproj": tproj.detach(),
            "emb": emb.detach(), "grad": g / coef}
