"""WavLM architecture description and the BYOL parameter inventory.

Mirrors the configuration the reference instantiates through `AutoModel.from_pretrained`
(src/models/encoder.py:14) for `config['model']['name']` (config/default_wavlm-large_byol.yaml:3),
i.e. transformers' WavLMConfig fields ([TF]configuration_wavlm.py:159-213) with
feat_extract_norm="layer" and do_stable_layer_norm=True (WavLM-Large).
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field, replace


@dataclass(frozen=True)
class WavLMArch:
    hidden: int = 1024
    layers: int = 24
    heads: int = 16
    ffn: int = 4096
    conv_dim: tuple = (512,) * 7
    conv_kernel: tuple = (10, 3, 3, 3, 3, 2, 2)
    conv_stride: tuple = (5, 2, 2, 2, 2, 2, 2)
    pos_kernel: int = 128
    pos_groups: int = 16
    num_buckets: int = 320
    max_distance: int = 800
    eps: float = 1e-5
    # stochastic features (train mode), hub defaults for microsoft/wavlm-large (unverified
    # offline, SURVEY.md §8c "stoch")
    hidden_dropout: float = 0.1
    attention_dropout: float = 0.1
    activation_dropout: float = 0.0
    feat_proj_dropout: float = 0.1
    layerdrop: float = 0.1
    mask_time_prob: float = 0.075
    mask_time_length: int = 10
    mask_time_min_masks: int = 2

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    def frames(self, samples: int) -> int:
        """Output frames of the conv feature encoder for `samples` input samples
        ([TF]modeling_wavlm.py:640-646)."""
        n = samples
        for k, s in zip(self.conv_kernel, self.conv_stride):
            n = (n - k) // s + 1
        return n

    def deterministic(self) -> "WavLMArch":
        """'det' variant: every stochastic feature off."""
        return replace(self, hidden_dropout=0.0, attention_dropout=0.0, activation_dropout=0.0,
                       feat_proj_dropout=0.0, layerdrop=0.0, mask_time_prob=0.0)

    def to_hf_config(self) -> dict:
        """WavLMConfig kwargs (used by the golden-fixture generator to build the reference)."""
        return dict(hidden_size=self.hidden, num_hidden_layers=self.layers, num_attention_heads=self.heads,
                    intermediate_size=self.ffn, conv_dim=list(self.conv_dim), conv_kernel=list(self.conv_kernel),
                    conv_stride=list(self.conv_stride), conv_bias=False, feat_extract_norm="layer",
                    do_stable_layer_norm=True, num_conv_pos_embeddings=self.pos_kernel,
                    num_conv_pos_embedding_groups=self.pos_groups, num_buckets=self.num_buckets,
                    max_bucket_distance=self.max_distance, layer_norm_eps=self.eps,
                    hidden_dropout=self.hidden_dropout, attention_dropout=self.attention_dropout,
                    activation_dropout=self.activation_dropout, feat_proj_dropout=self.feat_proj_dropout,
                    layerdrop=self.layerdrop, mask_time_prob=self.mask_time_prob,
                    mask_time_length=self.mask_time_length, mask_time_min_masks=self.mask_time_min_masks,
                    feat_extract_activation="gelu", hidden_act="gelu", apply_spec_augment=True)


LARGE = WavLMArch()
TINY = WavLMArch(hidden=256, layers=2, heads=4, ffn=512, conv_dim=(256,) * 7)

_PRESETS = {
    "microsoft/wavlm-large": LARGE,
    "nrse/wavlm-large": LARGE,
    "nrse/wavlm-tiny": TINY,
}


def arch_from_name(name: str) -> WavLMArch:
    """Resolve `config['model']['name']`: a known hub name, or a local directory holding a
    transformers WavLM config.json (as AutoModel.from_pretrained would)."""
    if name in _PRESETS:
        return _PRESETS[name]
    cfg_path = os.path.join(name, "config.json")
    if os.path.isfile(cfg_path):
        with open(cfg_path) as f:
            c = json.load(f)
        if not (c.get("feat_extract_norm") == "layer" and c.get("do_stable_layer_norm")):
            raise ValueError(f"{name}: only the stable-layer-norm WavLM variant (WavLM-Large family) is supported")
        return WavLMArch(
            hidden=c["hidden_size"], layers=c["num_hidden_layers"], heads=c["num_attention_heads"],
            ffn=c["intermediate_size"], conv_dim=tuple(c["conv_dim"]), conv_kernel=tuple(c["conv_kernel"]),
            conv_stride=tuple(c["conv_stride"]), pos_kernel=c["num_conv_pos_embeddings"],
            pos_groups=c["num_conv_pos_embedding_groups"], num_buckets=c["num_buckets"],
            max_distance=c["max_bucket_distance"], eps=c.get("layer_norm_eps", 1e-5),
            hidden_dropout=c.get("hidden_dropout", 0.1), attention_dropout=c.get("attention_dropout", 0.1),
            activation_dropout=c.get("activation_dropout", 0.1), feat_proj_dropout=c.get("feat_proj_dropout", 0.0),
            layerdrop=c.get("layerdrop", 0.1), mask_time_prob=c.get("mask_time_prob", 0.05),
            mask_time_length=c.get("mask_time_length", 10), mask_time_min_masks=c.get("mask_time_min_masks", 2))
    raise ValueError(f"unknown model name {name!r} (no local config.json; pretrained hub weights are not "
                     f"available offline)")


def arch_dict(a: WavLMArch) -> dict:
    return asdict(a)
