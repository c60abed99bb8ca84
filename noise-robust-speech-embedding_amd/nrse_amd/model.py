"""Drop-in mirror of the reference BYOL model API (src/models/byol.py, src/models/encoder.py),
backed by the fused engine (nrse_amd/engine.py) and its HIP kernels.

  BYOLSpeechModel(config)                 src/models/byol.py:10-55
    .forward(clean, noisy) -> (online_pred, target_proj)      :75-97 (autograd-enabled)
    ._update_target_network()            :62-73  (one fused EMA kernel instead of 496 pairs)
    .get_encoder()                       :99-101
    .state_dict() / .load_state_dict()   reference key layout
  byol_loss(online_pred, target_proj)    src/models/byol.py:104-128 (fused fwd+bwd kernel)
  WavLMEncoder(model_name)               src/models/encoder.py:5-32
    .forward(input_values, attention_mask=None) -> time-mean embedding [B, H]
    .forward_sequence(...) -> last_hidden_state is available via engine hooks (3-D output)
    .output_dim, .model (parameter namespace with `named_parameters()` for layers.{i} matching)

Documented deviation: the reference's encoder returns the 3-D
last_hidden_state, which crashes its own projector; the embedding here is its time mean.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import kernels as K
from .arch import WavLMArch, arch_from_name
from .engine import ByolEngine, StepConfig
from . import params as PR


def _device_default():
    return torch.device("cuda", torch.cuda.current_device())


class _OnlineBranch(torch.autograd.Function):
    """(clean, noisy, flat online params) -> (online_pred, target_proj); backward runs the
    engine's explicit encoder/heads backward and returns the flat gradient."""

    @staticmethod
    def forward(ctx, clean, noisy, flat, model, need):
        eng = model.engine
        pred, tproj, c = eng.forward(clean, noisy, train=model.training, step_seed=model._next_seed(),
                                     need_grad=need)
        ctx.model = model
        ctx.c = c
        ctx.mark_non_differentiable(tproj)
        return pred, tproj

    @staticmethod
    def backward(ctx, dpred, dtproj):
        eng = ctx.model.engine
        # the engine writes this backward's gradient into a fresh buffer that it then lets go of,
        # so autograd adopts it as (or adds it into) online_flat.grad without a 1.3 GB copy
        g = torch.zeros_like(eng.online)
        home = eng.grad
        eng.grad = g
        try:
            eng.backward(dpred.contiguous().float(), ctx.c)
        finally:
            eng.grad = home
        ctx.c = None
        return None, None, g, None, None


class _Loss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p, z):
        p = p.contiguous().float()
        z = z.contiguous().float()
        loss = torch.zeros(1, device=p.device, dtype=torch.float32)
        dp = torch.empty_like(p)
        stats = torch.zeros(2, device=p.device, dtype=torch.float32)
        K.byol_loss(p, z, loss, dp, stats)
        ctx.save_for_backward(dp)
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        (dp,) = ctx.saved_tensors
        return dp * g, None


def byol_loss(online_pred: torch.Tensor, target_proj: torch.Tensor) -> torch.Tensor:
    """2 - 2 * mean cos(p + 1e-10, z + 1e-10), clamped to [-1, 1] (src/models/byol.py:104-128)."""
    return _Loss.apply(online_pred, target_proj)


class _ParamNamespace(nn.Module):
    """`.model` of the encoder: named views into the flat parameter buffer with the
    transformers WavLMModel names (so `named_parameters()` matching on `layers.{i}` works,
    src/models/emotion.py:122, 127-128)."""

    def __init__(self, views: dict):
        super().__init__()
        self._views = views

    def named_parameters(self, prefix: str = "", recurse: bool = True, remove_duplicate: bool = True):
        for k, v in self._views.items():
            yield (prefix + k, v)

    def parameters(self, recurse: bool = True):
        for _, v in self.named_parameters():
            yield v


class WavLMEncoder(nn.Module):
    """WavLMEncoder(model_name) (src/models/encoder.py:5-32) on the HIP path."""

    def __init__(self, model_name: str | None = None, *, engine: ByolEngine | None = None, which: str = "online",
                 device=None, compute_dtype=torch.bfloat16):
        super().__init__()
        if engine is None:
            arch = arch_from_name(model_name)
            engine = ByolEngine(arch, arch.hidden, arch.hidden, device=device or _device_default(),
                                compute_dtype=compute_dtype)
        self.engine = engine
        self.which = which
        self.output_dim = engine.arch.hidden
        flat = engine.online if which == "online" else engine.target
        # uncached views: user code may edit these objects without touching the engine's own views
        self.model = _ParamNamespace(engine.group_views(flat, "encoder", cached=False))

    def forward(self, input_values: torch.Tensor, attention_mask=None) -> torch.Tensor:
        # [B, 1, L] -> [B, L] (encoder.py:20-21); the attention mask is ignored (encoder.py:23-25)
        if input_values.dim() == 3:
            input_values = input_values.squeeze(1)
        x = input_values.to(self.engine.dev, torch.float32).contiguous()
        with torch.no_grad():
            return self.engine.embed(x, self.which)


class BYOLSpeechModel(nn.Module):
    def __init__(self, config: dict, *, device=None, compute_dtype=torch.bfloat16, seed: int | None = None,
                 arch: WavLMArch | None = None, weight_split: bool = False):
        super().__init__()
        m = config["model"]
        arch = arch or arch_from_name(m["name"])
        self.ema_decay = float(m["ema_decay"])
        tr = config.get("training", {})
        # the engine's own loop (train_one_epoch -> engine.train_step) clears the gradient inside the
        # AdamW pass (no 1.3 GB fill kernel between steps); the autograd path below writes each
        # backward into a fresh buffer, and FusedAdamW.step copies it in before the update
        cfg = StepConfig(lr=float(tr.get("learning_rate", 1e-5)), weight_decay=float(tr.get("weight_decay", 1e-5)),
                         ema_decay=self.ema_decay, overlap_optimizer=True, fused_zero_grad=True)
        seed = seed if seed is not None else int(tr.get("seed", 42))
        self.engine = ByolEngine(arch, int(m["projection_dim"]), int(m["prediction_dim"]),
                                 device=device or _device_default(), compute_dtype=compute_dtype, seed=seed,
                                 step_cfg=cfg, weight_split=weight_split)
        # the single trainable parameter: the flat online buffer (views carry the reference names)
        self.online_flat = nn.Parameter(self.engine.online, requires_grad=True)
        self._seed_counter = seed * 1000003
        self._shadow_version = self.online_flat._version

    def _next_seed(self) -> int:
        self._seed_counter += 1
        return self._seed_counter & 0x7FFFFFFF

    def forward(self, clean_input_values: torch.Tensor, noisy_input_values: torch.Tensor):
        def prep(x):
            if x.dim() == 3:
                x = x.squeeze(1)
            return x.to(self.engine.dev, torch.float32).contiguous()
        self._sync_shadows()
        # grad mode is off inside Function.forward, so decide here whether to keep the tape
        need = torch.is_grad_enabled() and self.online_flat.requires_grad and self.training
        return _OnlineBranch.apply(prep(clean_input_values), prep(noisy_input_values), self.online_flat, self, need)

    def _sync_shadows(self) -> None:
        """Re-cast the bf16 GEMM-operand copy of the online weights if online_flat was modified
        in place since the last cast (a torch optimizer's step(), a user's in-place edit). The
        fused engine path (FusedAdamW / engine.train_step) writes the shadow itself."""
        e = self.engine
        e.sync_optimizer()
        v = self.online_flat._version
        if v != self._shadow_version:
            e.refresh_shadows(("online",))
            self._shadow_version = v

    def _update_target_network(self) -> None:
        e = self.engine
        e.sync_optimizer()
        self._sync_shadows()
        K.ema(e.target, e.online[:e.layout.ema_numel], e.target_sh, self.ema_decay, shadow_lo=e.target_lo)
        if e.target_lo8 is not None:
            # the split-weight mode's fp8 correction plane of the updated target (the fused AdamW + EMA
            # pass writes it in the engine's own step; nrse_ema has no fp8 output)
            K.split_lo8(e.target, e.target_lo8, e.lo8_exp, sat=e.sat_buf[0:1])

    def _copy_weights(self, *args) -> None:
        e = self.engine
        e.sync_optimizer()
        e.target.copy_(e.online[:e.layout.ema_numel])
        e.refresh_shadows(("target",))

    def refresh_shadows(self) -> None:
        """Re-derive the bf16 operand copies after the f32 weights were changed outside the
        fused optimizer (e.g. by torch.optim or load_state_dict)."""
        e = self.engine
        e.sync_optimizer()
        e.refresh_shadows()
        self._shadow_version = self.online_flat._version

    def get_encoder(self) -> WavLMEncoder:
        return WavLMEncoder(engine=self.engine, which="online")

    # ---------------------------------------------------------------- checkpoints
    def _state_items(self):
        """(key, tensor) of the checkpoint: the reference BYOLSpeechModel.state_dict() key set,
        shapes and dtypes (pinned by tests/golden/state_manifest.json): online encoder / projector
        / predictor, target encoder / projector, each BatchNorm's buffers after its bias. Within
        the encoder the order is the flat layout's, not transformers' module order (consumers
        match by key)."""
        e = self.engine
        for views in (PR.named_views(e.layout, e.online), PR.named_views(e.layout, e.target, target=True)):
            for k, v in views.items():
                yield k, v
                if k.endswith(".bias") and k[:-5] in e.bn:
                    rm, rv, nbt = e.bn_state(k[:-5])
                    yield k[:-5] + ".running_mean", rm
                    yield k[:-5] + ".running_var", rv
                    yield k[:-5] + ".num_batches_tracked", nbt

    def state_dict(self, *args, **kwargs):
        self.engine.sync_optimizer()
        return {k: v.detach().clone() for k, v in self._state_items()}

    def load_state_dict(self, sd: dict, strict: bool = True):
        """torch.nn.Module.load_state_dict semantics over the reference key layout: shape
        mismatches always raise; with strict, missing or unexpected keys raise; returns
        (missing_keys, unexpected_keys)."""
        from torch.nn.modules.module import _IncompatibleKeys
        self.engine.sync_optimizer()
        own = dict(self._state_items())
        missing = [k for k in own if k not in sd]
        unexpected = [k for k in sd if k not in own]
        bad = [f"{k}: checkpoint {tuple(sd[k].shape)} vs model {tuple(v.shape)}" for k, v in own.items()
               if k in sd and tuple(sd[k].shape) != tuple(v.shape)]
        if bad or (strict and (missing or unexpected)):
            msg = [f"size mismatch for {b}" for b in bad]
            if strict and missing:
                msg.append(f"Missing key(s): {missing[:8]}{'...' if len(missing) > 8 else ''}")
            if strict and unexpected:
                msg.append(f"Unexpected key(s): {unexpected[:8]}{'...' if len(unexpected) > 8 else ''}")
            raise RuntimeError("Error(s) in loading state_dict for BYOLSpeechModel:\n\t" + "\n\t".join(msg))
        with torch.no_grad():
            for k, v in own.items():
                if k in sd:
                    v.copy_(sd[k].to(v.device, v.dtype))
        self.engine.bn_counts_from_buffers()
        self.refresh_shadows()
        return _IncompatibleKeys(missing, unexpected)

    def train(self, mode: bool = True):
        self.training = mode
        return self
