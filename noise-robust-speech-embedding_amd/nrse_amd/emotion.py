"""Downstream dimensional-emotion head over the frozen BYOL encoder (BASELINE configs[3],
config/default_wavlm-large_emotion_dim_ft.yaml), on libnrse_hip.so.

Reference:
  EmotionClassifier            src/models/emotion.py:8-133 (forward :63-96, task='dimensional')
  AttentiveStatisticsPooling   src/models/pool.py:11-58
  ccc_loss                     src/train/dimentional_emotions.py:427-450
  train_one_epoch_dimensional  src/train/dimentional_emotions.py:306-338 (zero_grad, backward,
                               clip_grad_norm_(1.0), AdamW step); the encoder is frozen
                               (:57-58) but the model is in train mode, so WavLM's dropout,
                               LayerDrop and SpecAugment stay on in its forward.

Layout: the head's parameters are one flat f32 buffer (+ a compute-dtype shadow of it, written by
the AdamW kernel) named like EmotionClassifier's state_dict minus `encoder.`; grads and AdamW
moments mirror it. Per step:
  encoder (frozen, no tape) -> last_hidden_state [B, T, C] (compute dtype)
  sap_linear + tanh: one GEMM over B*T rows (NRSE_EPI_TANH), f32 out
  nrse_asp_fwd: softmax(h . attention) statistics over each utterance's first feat_len frames
  shared_fc / dimensional_fc: split-K Linear -> LayerNorm+ReLU (NRSE_LN_RELU) -> dropout
  dimensional_out: Linear(hidden, 3) (computed 4 wide: operand strides must be 16-byte multiples)
  nrse_ccc_loss (fwd + bwd), then the mirror-image backward and clip + AdamW.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from . import kernels as K
from . import rng as R

F32 = torch.float32
ALIGN = 64


def head_specs(C: int, hidden: int, num_emotions: int = 8) -> list:
    """(name, shape, init) in EmotionClassifier's parameter order (encoder excluded)."""
    S = [("pooling.sap_linear.weight", (C, C), ("lin", C)), ("pooling.sap_linear.bias", (C,), ("lin", C)),
         ("pooling.attention", (C, 1), ("normal", 1.0))]
    for blk, fan in (("shared_fc", 2 * C), ("categorical_fc", hidden), ("dimensional_fc", hidden)):
        S += [(f"{blk}.0.weight", (hidden, fan), ("lin", fan)), (f"{blk}.0.bias", (hidden,), ("lin", fan)),
              (f"{blk}.1.weight", (hidden,), ("one", 0)), (f"{blk}.1.bias", (hidden,), ("zero", 0))]
        if blk == "categorical_fc":
            S += [("categorical_out.weight", (num_emotions, hidden), ("lin", hidden)),
                  ("categorical_out.bias", (num_emotions,), ("lin", hidden))]
    S += [("dimensional_out.weight", (3, hidden), ("lin", hidden)), ("dimensional_out.bias", (3,), ("lin", hidden))]
    return S


def init_head_flat(specs, offsets, numel, seed: int) -> torch.Tensor:
    """torch defaults (nn.Linear: U(+-1/sqrt(fan_in)); LayerNorm 1/0; attention N(0, 1),
    pool.py:32-33), drawn from a seeded CPU generator so any box rebuilds the same head."""
    flat = torch.zeros(numel)
    g = torch.Generator().manual_seed(seed)
    for name, shp, (kind, a) in specs:
        off, n = offsets[name]
        if kind == "lin":
            v = (torch.rand(shp, generator=g) * 2 - 1) / math.sqrt(a)
        elif kind == "normal":
            v = torch.randn(shp, generator=g) * a
        elif kind == "one":
            v = torch.ones(shp)
        else:
            v = torch.zeros(shp)
        flat[off:off + n] = v.reshape(-1)
    return flat


def feat_lengths(lengths_samples: torch.Tensor) -> torch.Tensor:
    """pool.py:11-19: frames (20 ms hop) from per-utterance valid sample counts, int32."""
    return (torch.div(lengths_samples.to(torch.int64) - 1, 320, rounding_mode="floor") + 1).to(torch.int32)


class EmotionHead:
    """Flat-buffer EmotionClassifier head (pooling + shared + categorical + dimensional)."""

    def __init__(self, C: int, hidden: int = 1024, num_emotions: int = 8, dropout: float = 0.5, *, device="cuda",
                 compute_dtype=torch.bfloat16, seed: int = 42, init_flat: torch.Tensor | None = None):
        if C % 256 or hidden % 256:
            raise _lib.NrseError(f"emotion head: C={C}, hidden={hidden} must be multiples of 256")
        self.C, self.hidden, self.num_emotions, self.p = C, hidden, num_emotions, float(dropout)
        self.dev = torch.device(device)
        self.cdt = compute_dtype
        self.specs = head_specs(C, hidden, num_emotions)
        self.offsets, off = {}, 0
        for name, shp, _ in self.specs:
            n = math.prod(shp)
            self.offsets[name] = (off, n)
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        flat = init_flat if init_flat is not None else init_head_flat(self.specs, self.offsets, self.numel, seed)
        self.params = flat.to(self.dev, F32).contiguous()
        self.grad = torch.zeros_like(self.params)
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.shadow = None if self.cdt == F32 else torch.empty(self.numel, device=self.dev, dtype=self.cdt)
        if self.shadow is not None:
            K.cast(self.params, self.shadow)
        self.sumsq_buf = torch.zeros(1, device=self.dev, dtype=torch.float64)
        self.loss_buf = torch.zeros(1, device=self.dev, dtype=F32)
        self.step_count = 0
        # dimensional_out padded to 4 rows (zero 4th row / bias)
        self._wout4 = torch.zeros(4, hidden, device=self.dev, dtype=F32)
        self._bout4 = torch.zeros(4, device=self.dev, dtype=F32)

    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        off, n = self.offsets[name]
        shp = next(s for nm, s, _ in self.specs if nm == name)
        return flat[off:off + n].view(shp)

    def named_parameters(self):
        for name, _, _ in self.specs:
            yield name, self.view(self.params, name)

    # ------------------------------------------------------------------ forward
    def _block(self, x, name, train, seed, tape):
        """Linear -> LayerNorm -> ReLU -> Dropout (emotion.py:34-58)."""
        P = self.params
        B = x.shape[0]
        z = torch.empty(B, self.hidden, device=self.dev, dtype=F32)
        K.linear_fwd_small(x, self.view(P, name + ".0.weight"), z, bias=self.view(P, name + ".0.bias"))
        a = torch.empty_like(z)
        mu = torch.empty(B, device=self.dev, dtype=F32)
        rs = torch.empty(B, device=self.dev, dtype=F32)
        K.ln_fwd(z, self.view(P, name + ".1.weight"), self.view(P, name + ".1.bias"), a, mu, rs, 1e-5, relu=True)
        if train and self.p > 0:
            d = torch.empty_like(a)
            K.dropout_cast(a, d, self.p, seed)
        else:
            d = a
        tape[name] = dict(x=x, z=z, mu=mu, rs=rs, out=d, seed=seed)
        return d

    def forward(self, hid: torch.Tensor, flens: torch.Tensor, *, train: bool, step_seed: int = 0, task="dimensional"):
        """hid [B, T, C] (compute dtype) -> (categorical logits or None, dimensional [B, 3] view, tape)."""
        B, T, C = hid.shape
        assert C == self.C and flens.dtype == torch.int32 and flens.shape == (B,)
        P = self.params
        S = self.shadow if self.shadow is not None else P
        x2 = hid.reshape(B * T, C)
        h = torch.empty(B * T, C, device=self.dev, dtype=F32)
        K.linear_fwd(x2, self.view(S, "pooling.sap_linear.weight"), h, bias=self.view(P, "pooling.sap_linear.bias"),
                     flags=_lib.EPI_TANH)
        w = torch.empty(B, T, device=self.dev, dtype=F32)
        var = torch.empty(B, C, device=self.dev, dtype=F32)
        pooled = torch.empty(B, 2 * C, device=self.dev, dtype=F32)
        K.asp_fwd(hid, h.view(B, T, C), self.view(P, "pooling.attention"), flens, w, var, pooled)
        tape = dict(hid=hid, h=h, w=w, var=var, pooled=pooled, flens=flens)
        s = self._block(pooled, "shared_fc", train, R.site_seed(step_seed, 901), tape)
        cat = None
        if task in ("categorical", "both"):
            c = self._block(s, "categorical_fc", train, R.site_seed(step_seed, 902), tape)
            cat = torch.empty(B, self.num_emotions, device=self.dev, dtype=F32)
            K.linear_fwd_small(c, self.view(P, "categorical_out.weight"), cat, bias=self.view(P, "categorical_out.bias"))
        dim = None
        if task in ("dimensional", "both"):
            d = self._block(s, "dimensional_fc", train, R.site_seed(step_seed, 903), tape)
            K.cast(self.view(P, "dimensional_out.weight").reshape(-1), self._wout4[:3].reshape(-1))
            K.cast(self.view(P, "dimensional_out.bias"), self._bout4[:3])
            out4 = torch.empty(B, 4, device=self.dev, dtype=F32)
            K.linear_fwd_small(d, self._wout4, out4, bias=self._bout4)
            tape["out4"] = out4
            dim = out4[:, :3]
        return cat, dim, tape

    # ------------------------------------------------------------------ backward
    def _block_bwd(self, dout, name, tape):
        G, P = self.grad, self.params
        c = tape[name]
        B = dout.shape[0]
        da = dout
        if self._train:  # the forward's dropout mask (same counter-hash seed)
            da = torch.empty_like(dout)
            K.dropout_cast(dout, da, self.p, c["seed"])
        dz = torch.empty_like(dout)
        K.ln_bwd(da, c["z"], self.view(P, name + ".1.weight"), c["mu"], c["rs"], dz, beta=self.view(P, name + ".1.bias"),
                 relu=True, dgamma=self.view(G, name + ".1.weight"), dbeta=self.view(G, name + ".1.bias"))
        K.linear_wgrad(dz, c["x"], self.view(G, name + ".0.weight"))
        K.colsum(dz, self.view(G, name + ".0.bias"))
        dx = torch.empty(B, c["x"].shape[1], device=self.dev, dtype=F32)
        K.linear_dgrad_small(dz, self.view(P, name + ".0.weight"), dx)
        return dx

    def backward(self, dout4: torch.Tensor, tape: dict, train: bool) -> None:
        """d(loss)/d(out4) [B, 4] (column 3 zero) -> head gradients (accumulated into self.grad)."""
        self._train = train and self.p > 0
        G = self.grad
        d = tape["dimensional_fc"]["out"]
        B = d.shape[0]
        gw4 = torch.zeros(4, self.hidden, device=self.dev, dtype=F32)
        K.linear_wgrad(dout4, d, gw4)
        K.cast(gw4[:3].reshape(-1), self.view(G, "dimensional_out.weight").reshape(-1))
        gb4 = torch.zeros(4, device=self.dev, dtype=F32)
        K.colsum(dout4, gb4)
        K.cast(gb4[:3], self.view(G, "dimensional_out.bias"))
        dd = torch.empty(B, self.hidden, device=self.dev, dtype=F32)
        K.linear_dgrad_small(dout4, self._wout4, dd)
        ds = self._block_bwd(dd, "dimensional_fc", tape)
        dpooled = self._block_bwd(ds, "shared_fc", tape)
        hid, h = tape["hid"], tape["h"]
        Bh, T, C = hid.shape
        dpre = torch.empty(Bh * T, C, device=self.dev, dtype=self.cdt)
        K.asp_bwd(hid, h.view(Bh, T, C), self.view(self.params, "pooling.attention"), tape["flens"], tape["w"],
                  tape["var"], tape["pooled"], dpooled, dpre, self.view(G, "pooling.attention"))
        K.linear_wgrad(dpre, hid.reshape(Bh * T, C), self.view(G, "pooling.sap_linear.weight"))
        K.colsum(dpre, self.view(G, "pooling.sap_linear.bias"))

    def optimizer_step(self, lr: float, weight_decay: float, max_norm: float = 1.0) -> None:
        """clip_grad_norm_(max_norm) + AdamW (dimentional_emotions.py:336-338, :105-111); the
        categorical branch has zero gradient in the dimensional task and torch's AdamW skips
        it (grad None), so only the pooling, shared and dimensional ranges are stepped."""
        self.step_count += 1
        self.sumsq_buf.zero_()
        K.sumsq(self.grad, self.sumsq_buf)
        for lo, hi in self._trainable_ranges():
            sh = self.shadow[lo:hi] if self.shadow is not None else None
            K.adamw(self.params[lo:hi], self.grad[lo:hi], self.m[lo:hi], self.v[lo:hi], sh, lr=lr, beta1=0.9,
                    beta2=0.999, eps=1e-8, weight_decay=weight_decay, step=self.step_count, max_norm=max_norm,
                    sumsq_buf=self.sumsq_buf)

    def _trainable_ranges(self):
        names = [n for n, _, _ in self.specs if not n.startswith("categorical")]
        ranges = []
        for n in names:
            off, cnt = self.offsets[n]
            end = off + (cnt + ALIGN - 1) // ALIGN * ALIGN
            if ranges and ranges[-1][1] == off:
                ranges[-1] = (ranges[-1][0], end)
            else:
                ranges.append((off, end))
        return ranges


class EmotionDimTrainer:
    """One dimensional-emotion training iteration over the frozen BYOL encoder of `engine`
    (train_one_epoch_dimensional body, dimentional_emotions.py:314-338)."""

    def __init__(self, engine, head: EmotionHead, *, lr: float = 1e-5, weight_decay: float = 1e-4,
                 encoder_train_mode: bool = True):
        self.engine, self.head = engine, head
        self.lr, self.wd = lr, weight_decay
        self.encoder_train_mode = encoder_train_mode

    def encode(self, wav: torch.Tensor, step_seed: int):
        eng = self.engine
        B, L = wav.shape
        T = eng.arch.frames(L)
        skips, masks = eng.stochastic_inputs(step_seed, B, T, self.encoder_train_mode)
        with torch.no_grad():
            hid, _, _ = eng.encoder_forward(eng.weights("online"), wav, train=self.encoder_train_mode,
                                            fseed=R.forward_seed(step_seed, 2, 0), skip=skips[0], mask_np=masks[0],
                                            need_grad=False, hidden_dtype=eng.cdt)
        return hid

    def train_step(self, wav: torch.Tensor, labels: torch.Tensor, lengths: torch.Tensor, step_seed: int):
        """wav [B, L] input values, labels [B, 3] (A, V, D), lengths [B] valid samples (the
        attention-mask sums) -> device loss."""
        head = self.head
        hid = self.encode(wav, step_seed)
        flens = feat_lengths(lengths).to(head.dev)
        _, dim, tape = head.forward(hid, flens, train=True, step_seed=step_seed)
        dout4 = torch.zeros(wav.shape[0], 4, device=head.dev, dtype=F32)
        head.loss_buf.zero_()
        K.ccc_loss(dim, labels.to(head.dev, F32).contiguous(), head.loss_buf, dout4[:, :3])
        head.grad.zero_()
        head.backward(dout4, tape, train=True)
        head.optimizer_step(self.lr, self.wd)
        return head.loss_buf
