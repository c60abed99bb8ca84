"""BYOL parameter inventory, portable seeded initialisation and the flat HBM layout.

Names follow the reference state_dict exactly: the encoder part is the
transformers WavLMModel naming under `online_encoder.model.` (src/models/encoder.py:14), the
heads are `online_projector.layers.{0,1,3,4}` / `online_predictor.layers.{0,1,3,4,6}`
(src/models/multi_layer_heads.py:16-20, 39-45), the target mirrors encoder + projector
(src/models/byol.py:40-49).

Initialisation is a portable, seeded function of (seed, parameter name) built on torch's CPU
generator, so the GPU box regenerates bit-identical weights without shipping checkpoints
(pretrained hub weights are unavailable offline).
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass

import torch

from .arch import WavLMArch

ALIGN = 64  # elements; keeps every parameter 256-byte aligned in the flat f32 buffer


@dataclass(frozen=True)
class PSpec:
    name: str          # module-relative name (WavLMModel / Sequential naming)
    shape: tuple
    init: str          # init recipe key
    scale: float = 0.0


def encoder_specs(a: WavLMArch) -> list[PSpec]:
    """WavLMModel parameters in our flat order (forward order, q/k/v adjacent so the fused
    QKV weight [3H, H] and bias [3H] are contiguous views)."""
    S: list[PSpec] = []
    H = a.hidden
    if a.mask_time_prob > 0:
        S.append(PSpec("masked_spec_embed", (H,), "uniform01"))
    cin = 1
    for i, (c, k) in enumerate(zip(a.conv_dim, a.conv_kernel)):
        p = f"feature_extractor.conv_layers.{i}."
        S.append(PSpec(p + "conv.weight", (c, cin, k), "kaiming", math.sqrt(2.0 / (cin * k))))
        S.append(PSpec(p + "layer_norm.weight", (c,), "ln_w"))
        S.append(PSpec(p + "layer_norm.bias", (c,), "ln_b"))
        cin = c
    S.append(PSpec("feature_projection.layer_norm.weight", (cin,), "ln_w"))
    S.append(PSpec("feature_projection.layer_norm.bias", (cin,), "ln_b"))
    k = 1.0 / math.sqrt(cin)
    S.append(PSpec("feature_projection.projection.weight", (H, cin), "uniform", k))
    S.append(PSpec("feature_projection.projection.bias", (H,), "uniform", k))
    pk, G = a.pos_kernel, a.pos_groups
    S.append(PSpec("encoder.pos_conv_embed.conv.bias", (H,), "uniform", math.sqrt(G / (H * pk))))
    S.append(PSpec("encoder.pos_conv_embed.conv.parametrizations.weight.original0", (1, 1, pk), "wn_g"))
    S.append(PSpec("encoder.pos_conv_embed.conv.parametrizations.weight.original1", (H, H // G, pk), "normal",
                   2.0 * math.sqrt(1.0 / (pk * H))))
    for li in range(a.layers):
        p = f"encoder.layers.{li}."
        at = p + "attention."
        for nm in ("q_proj", "k_proj", "v_proj"):
            S.append(PSpec(at + nm + ".weight", (H, H), "normal", 0.02))
        for nm in ("q_proj", "k_proj", "v_proj"):
            S.append(PSpec(at + nm + ".bias", (H,), "normal", 0.02))
        S.append(PSpec(at + "out_proj.weight", (H, H), "normal", 0.02))
        S.append(PSpec(at + "out_proj.bias", (H,), "normal", 0.02))
        S.append(PSpec(at + "gru_rel_pos_const", (1, a.heads, 1, 1), "gru_const"))
        S.append(PSpec(at + "gru_rel_pos_linear.weight", (8, a.head_dim), "normal", 0.2))
        S.append(PSpec(at + "gru_rel_pos_linear.bias", (8,), "normal", 0.2))
        if li == 0:
            S.append(PSpec(at + "rel_attn_embed.weight", (a.num_buckets, a.heads), "normal", 1.0))
        S.append(PSpec(p + "layer_norm.weight", (H,), "ln_w"))
        S.append(PSpec(p + "layer_norm.bias", (H,), "ln_b"))
        S.append(PSpec(p + "feed_forward.intermediate_dense.weight", (a.ffn, H), "normal", 0.02))
        S.append(PSpec(p + "feed_forward.intermediate_dense.bias", (a.ffn,), "normal", 0.02))
        S.append(PSpec(p + "feed_forward.output_dense.weight", (H, a.ffn), "normal", 0.02))
        S.append(PSpec(p + "feed_forward.output_dense.bias", (H,), "normal", 0.02))
        S.append(PSpec(p + "final_layer_norm.weight", (H,), "ln_w"))
        S.append(PSpec(p + "final_layer_norm.bias", (H,), "ln_b"))
    S.append(PSpec("encoder.layer_norm.weight", (H,), "ln_w"))
    S.append(PSpec("encoder.layer_norm.bias", (H,), "ln_b"))
    return S


def _head_linear(name: str, i: int, o: int) -> list[PSpec]:
    k = 1.0 / math.sqrt(i)  # nn.Linear default init range
    return [PSpec(name + ".weight", (o, i), "uniform", k), PSpec(name + ".bias", (o,), "uniform", k)]


def _head_bn(name: str, c: int) -> list[PSpec]:
    return [PSpec(name + ".weight", (c,), "bn_w"), PSpec(name + ".bias", (c,), "bn_b")]


def projector_specs(i: int, h: int, o: int) -> list[PSpec]:
    """ProjectionHead: Linear -> BN -> ReLU -> Linear -> BN (multi_layer_heads.py:16-20)."""
    return _head_linear("layers.0", i, h) + _head_bn("layers.1", h) + _head_linear("layers.3", h, o) + \
        _head_bn("layers.4", o)


def predictor_specs(i: int, h: int, o: int) -> list[PSpec]:
    """PredictionHead: Lin -> BN -> ReLU -> Lin -> BN -> ReLU -> Lin (multi_layer_heads.py:39-45)."""
    return _head_linear("layers.0", i, h) + _head_bn("layers.1", h) + _head_linear("layers.3", h, h) + \
        _head_bn("layers.4", h) + _head_linear("layers.6", h, o)


def bn_buffers(prefix: str, c: int) -> dict:
    return {prefix + ".running_mean": torch.zeros(c), prefix + ".running_var": torch.ones(c),
            prefix + ".num_batches_tracked": torch.zeros((), dtype=torch.long)}


def _gen(seed: int, role: str, name: str) -> torch.Generator:
    g = torch.Generator()
    g.manual_seed((seed * 1000003 + zlib.crc32(f"{role}/{name}".encode())) & 0x7FFFFFFFFFFF)
    return g


def init_tensor(spec: PSpec, seed: int, role: str, companion: torch.Tensor | None = None) -> torch.Tensor:
    g = _gen(seed, role, spec.name)
    shp = spec.shape
    r = spec.init
    if r == "normal" or r == "kaiming":
        return torch.randn(shp, generator=g) * spec.scale
    if r == "uniform":
        return (torch.rand(shp, generator=g) * 2 - 1) * spec.scale
    if r == "uniform01":
        return torch.rand(shp, generator=g)
    if r in ("ln_w", "bn_w"):
        return 1.0 + 0.05 * torch.randn(shp, generator=g)
    if r in ("ln_b", "bn_b"):
        return 0.05 * torch.randn(shp, generator=g)
    if r == "gru_const":
        return 1.0 + 0.1 * torch.randn(shp, generator=g)
    if r == "wn_g":
        # weight_norm(dim=2) initialises g = ||v|| per kernel tap; perturb so g matters.
        assert companion is not None
        nrm = companion.pow(2).sum(dim=(0, 1)).sqrt().reshape(shp)
        return nrm * (1.0 + 0.05 * torch.randn(shp, generator=g))
    raise ValueError(r)


def init_group(specs: list[PSpec], seed: int, role: str) -> dict:
    out = {}
    by_name = {s.name: s for s in specs}
    for s in specs:
        if s.init == "wn_g":
            continue
        out[s.name] = init_tensor(s, seed, role)
    for s in specs:
        if s.init == "wn_g":
            v = out[s.name.replace("original0", "original1")]
            out[s.name] = init_tensor(s, seed, role, companion=v)
    return {s.name: out[s.name] for s in specs}


@dataclass
class ByolLayout:
    """Flat f32 layout of the online network: [encoder | projector | predictor]; the target
    network mirrors the first `ema_numel` elements (encoder + projector)."""
    arch: WavLMArch
    proj_dim: int
    pred_dim: int
    specs: list            # (group, PSpec)
    offsets: dict          # state-dict key -> (offset, numel, shape)
    ema_numel: int
    numel: int

    def keys(self, group: str | None = None):
        return [k for (g, s), k in zip(self.specs, self.offsets) if group is None or g == group]


GROUP_PREFIX = {"encoder": "online_encoder.model.", "projector": "online_projector.",
                "predictor": "online_predictor."}
TARGET_PREFIX = {"encoder": "target_encoder.model.", "projector": "target_projector."}


def byol_layout(arch: WavLMArch, proj_dim: int, pred_dim: int) -> ByolLayout:
    groups = [("encoder", encoder_specs(arch)),
              ("projector", projector_specs(arch.hidden, proj_dim, proj_dim)),
              ("predictor", predictor_specs(proj_dim, pred_dim, proj_dim))]
    specs, offsets = [], {}
    off = 0
    ema_numel = 0
    for gname, gs in groups:
        for s in gs:
            key = GROUP_PREFIX[gname] + s.name
            n = 1
            for d in s.shape:
                n *= d
            offsets[key] = (off, n, s.shape)
            specs.append((gname, s))
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        if gname == "projector":
            ema_numel = off
    return ByolLayout(arch, proj_dim, pred_dim, specs, offsets, ema_numel, off)


def init_byol_flat(layout: ByolLayout, seed: int) -> torch.Tensor:
    """Online flat parameter vector (CPU f32); the target starts as a copy of its prefix
    (src/models/byol.py:48-49)."""
    flat = torch.zeros(layout.numel)
    for gname in ("encoder", "projector", "predictor"):
        gs = [s for g, s in layout.specs if g == gname]
        vals = init_group(gs, seed, gname)
        for s in gs:
            off, n, shp = layout.offsets[GROUP_PREFIX[gname] + s.name]
            flat[off:off + n] = vals[s.name].reshape(-1)
    return flat


def named_views(layout: ByolLayout, flat: torch.Tensor, target: bool = False) -> dict:
    """state-dict-keyed views into a flat vector (online, or target when `target`)."""
    out = {}
    for (gname, s) in layout.specs:
        key = GROUP_PREFIX[gname] + s.name
        off, n, shp = layout.offsets[key]
        if target:
            if gname not in TARGET_PREFIX:
                continue
            key = TARGET_PREFIX[gname] + s.name
        out[key] = flat[off:off + n].view(shp)
    return out


def count_params(specs: list[PSpec]) -> int:
    t = 0
    for s in specs:
        n = 1
        for d in s.shape:
            n *= d
        t += n
    return t


def layer_range(layout: ByolLayout, arch: WavLMArch, li: int) -> tuple:
    """[start, end) of online transformer layer li's parameters in the flat buffer (the unit
    of the overlapped gradient all-reduce, nrse_amd/ddp.py)."""
    pre = GROUP_PREFIX["encoder"]
    start = layout.offsets[pre + f"encoder.layers.{li}.attention.q_proj.weight"][0]
    nxt = (f"encoder.layers.{li + 1}.attention.q_proj.weight" if li + 1 < arch.layers else "encoder.layer_norm.weight")
    return start, layout.offsets[pre + nxt][0]



def grad_groups(layout: ByolLayout, arch: WavLMArch) -> dict:
    """The flat gradient cut into the units the overlapped all-reduce sends (nrse_amd/engine.py
    backward), each a list of [start, end) ranges; together they tile the buffer exactly once.
    "heads" = projector + predictor, "final" = the final LN, ("layer", li) = transformer layer li
    (layer 0 without its rel_attn_embed, which is "rel"), "posconv", "proj" = the feature
    projection, its LN and the SpecAugment embedding, "conv<i>" = conv layer i's weight and LN."""
    pre = GROUP_PREFIX["encoder"]
    off = lambda name: layout.offsets[pre + name][0]   # noqa: E731
    starts = sorted(v[0] for v in layout.offsets.values())
    head0 = min(v[0] for k, v in layout.offsets.items() if not k.startswith(pre))
    g = {"heads": [(head0, layout.numel)], "final": [(off("encoder.layer_norm.weight"), head0)]}
    rel = off("encoder.layers.0.attention.rel_attn_embed.weight")
    rel_end = next(o for o in starts if o > rel)
    for li in range(arch.layers):
        s, e = layer_range(layout, arch, li)
        g[("layer", li)] = [(s, rel), (rel_end, e)] if li == 0 else [(s, e)]
    g["rel"] = [(rel, rel_end)]
    pos0 = off("encoder.pos_conv_embed.conv.bias")
    g["posconv"] = [(pos0, layer_range(layout, arch, 0)[0])]
    conv = [off(f"feature_extractor.conv_layers.{i}.conv.weight") for i in range(len(arch.conv_dim))]
    fp0 = off("feature_projection.layer_norm.weight")
    g["proj"] = [(fp0, pos0)] + ([(0, conv[0])] if conv[0] > 0 else [])
    for i in range(len(conv)):
        g[f"conv{i}"] = [(conv[i], conv[i + 1] if i + 1 < len(conv) else fp0)]
    return g


def grad_group_order(arch: WavLMArch) -> list:
    """The order the engine's backward sends grad_groups() when no layer is skipped."""
    order = ["heads"]
    for li in reversed(range(arch.layers)):
        order.append(("layer", li))
        if li == arch.layers - 1:
            order.append("final")
    order += ["rel", "posconv", "proj"] + [f"conv{i}" for i in reversed(range(1, len(arch.conv_dim)))] + ["conv0"]
    return order
