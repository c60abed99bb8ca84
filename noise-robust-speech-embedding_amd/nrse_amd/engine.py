"""MI355X-native BYOL-on-WavLM training engine over libnrse_hip.so.

One object holds the whole training state in HBM as flat buffers (SURVEY.md §8a layout):
  online   f32 [numel]        master weights: encoder | projector | predictor
  target   f32 [ema_numel]    target encoder + projector (EMA of the online prefix)
  grad     f32 [numel]        gradient buffer (zeroed per step; DDP all-reduces it in buckets)
  m, v     f32 [numel]        AdamW moments
  *_sh     bf16 shadows       GEMM operand copies written by the AdamW / EMA kernels
Activations are channels-last ([B*T, C] rows); the residual stream is f32, every GEMM operand
is in the compute dtype (bf16, or f32 in parity mode). Forward and backward are explicit
kernel sequences (no autograd), mirroring:
  train_one_epoch body  train_byol.py:47-77
  BYOLSpeechModel       src/models/byol.py:75-97 (+ time-mean shim)
  WavLMModel            [TF]modeling_wavlm.py:1032-1096
"""
from __future__ import annotations

import contextlib
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from . import kernels as K
from . import params as PR
from . import rng as R
from .arch import WavLMArch
from .hostside import bucket_runs, bucket_vector, layerdrop_decisions

F32 = torch.float32
# NRSE_SERIAL_TARGET=1 runs the target view and the backward weight gradients on the main
# stream (profiling: kernel durations without the concurrent streams' interference)
_SERIAL_TARGET = os.environ.get("NRSE_SERIAL_TARGET", "0") == "1"


def compute_mode(name: str) -> tuple:
    """CLI compute mode -> (compute dtype, weight_split): "bf16" (benchmarked), "bf16sw" (bf16
    activations, split hi + lo bf16 weights in the forward GEMMs: embeddings within the
    north-star 1e-3), "f32" (exact-f32 parity mode)."""
    modes = {"bf16": (torch.bfloat16, False), "bf16sw": (torch.bfloat16, True), "f32": (torch.float32, False)}
    if name not in modes:
        raise ValueError(f"unknown compute mode {name!r} (one of {sorted(modes)})")
    return modes[name]


def _divisor_at_most(n: int, cap: int) -> int:
    cap = max(1, min(n, cap))
    for d in range(cap, 0, -1):
        if n % d == 0:
            return d
    return 1


# the gate path's dx1 contribution added by the LN1 backward (nrse_gate_bwd_dp + gate_dp) instead
# of a read-modify-write of dx1 by nrse_gate_bwd; NRSE_GATE_INTO_LN=0 restores the latter (A/B)
_GATE_INTO_LN = os.environ.get("NRSE_GATE_INTO_LN", "1") != "0"
# the attention-probability dropout bits computed ahead on a mask stream and read by the forward
# (nrse_attn_dropout_mask); opt-in with NRSE_MASK_AHEAD=1: the mask kernel (29 us) costs more
# than the forward saves (73 -> 58 us) when the two views already overlap (step 552 vs 554 pairs/s)
_MASK_AHEAD = os.environ.get("NRSE_MASK_AHEAD", "0") == "1"
# the target EMA in the AdamW pass (nrse_adamw_params.ema_t) instead of a second pass re-reading
# the updated weights (nrse_ema); NRSE_FUSED_EMA=0 restores the two launches (A/B)
_FUSED_EMA = os.environ.get("NRSE_FUSED_EMA", "1") != "0"
# split-weight mode: the layer GEMMs' correction segment x (w - w_hi) on the fp8 MFMA (fp8 x times the
# fp8 correction plane of the weights, 2x the bf16 rate) instead of a second bf16 segment;
# NRSE_SPLIT_LO8=0 restores the bf16 lo plane everywhere (A/B)
_SPLIT_LO8 = os.environ.get("NRSE_SPLIT_LO8", "1") != "0"
# ... and the conv stack's two correction segments (x_lo w_hi + x_hi w_lo) as fp8 segments against
# the activations' fp8 planes [fp8(x_lo 2^e) | fp8(x_hi)] (ABI 7) instead of two more bf16 segments;
# NRSE_CONV_SPLIT8=0 restores the three bf16 planes. The exponent (ABI 10: derived, no longer fixed)
# keeps both (w - w_hi) 2^e and (x - x_hi) 2^e (each <= 2^-8 |.|) inside half of fp8's +-448: the
# conv activations are GELU(LayerNorm) outputs, |x| <= sqrt(C) max|gamma| + max|beta| (23.6 at
# gamma = 1, beta = 0: e = 11), so ByolEngine._set_lo8_planes takes e from the conv LayerNorms'
# gamma / beta and the conv weights' range; NRSE_CONV_LO8_EXP pins it (A/B)
# ABI 9: the backward's per-layer gradient reductions batched on the side stream (0: on the dX
# chain's stream, one launch each, as before)
_DEFER_REDUCE = os.environ.get("NRSE_DEFER_REDUCE", "1") != "0"
_CONV_SPLIT8 = os.environ.get("NRSE_CONV_SPLIT8", "1") != "0"
CONV_LO8_EXP = 11   # the derived value at the seeded init (gamma = 1, beta = 0)
_CONV_LO8_PIN = os.environ.get("NRSE_CONV_LO8_EXP")
FP8 = K.FP8


SAT_WEIGHTS, SAT_CONV, SAT_ACT = 0, 1, 2   # rows of ByolEngine.sat_buf


def _headroom_exp(W: float) -> int:
    """The fp8 correction exponent of values bounded by W: |v - bf16(v)| <= 2^-8 W, scaled by 2^e
    to at most 224 (half of e4m3's 448: 2x headroom), e = floor(log2(224 * 256 / W))."""
    e = int(math.floor(math.log2(224.0 * 256.0 / W))) if W > 0 else 0
    return max(-60, min(60, e))


@dataclass
class StepConfig:
    lr: float = 1e-5
    weight_decay: float = 1e-5
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    max_norm: float = 1.0
    ema_decay: float = 0.997
    # Run clip/AdamW/EMA on their own stream in per-layer segments and let the NEXT step's forward
    # wait per layer (see ByolEngine.optimizer_step). Same kernels, same per-element arithmetic:
    # parameters are bit-identical to the serial order (tests/test_engine_gpu.py).
    overlap_optimizer: bool = False
    # The AdamW pass zeroes the gradient buffer after reading it (nrse_adamw_params.zero_grad), so
    # the next step accumulates without a separate 1.3 GB fill on the critical path. self.grad
    # then no longer holds the last step's gradient after train_step (tests that read it keep False).
    fused_zero_grad: bool = False


@dataclass
class Tape:
    """Activations the backward pass needs (one encoder forward)."""
    B: int = 0
    T: int = 0
    wav: torch.Tensor | None = None
    conv: list = field(default_factory=list)
    feats: torch.Tensor | None = None
    fp_mean: torch.Tensor | None = None
    fp_rstd: torch.Tensor | None = None
    xn: torch.Tensor | None = None
    mask: torch.Tensor | None = None
    hpad: torch.Tensor | None = None
    pos_pre: torch.Tensor | None = None
    pos: dict | None = None
    bias_tab: torch.Tensor | None = None
    bias_vec: torch.Tensor | None = None
    layers: list = field(default_factory=list)
    final: tuple | None = None
    fseed: int = 0


class EncoderWeights:
    """Per-forward view of one encoder's weights: f32 master views, compute-dtype shadow views,
    and the per-step derived layouts (conv weights in implicit-GEMM order, weight-normed
    pos-conv in forward and flipped-dgrad order)."""

    def __init__(self, eng: "ByolEngine", master: torch.Tensor, shadow: torch.Tensor | None, lo_stride: int = 0,
                 lo8: torch.Tensor | None = None):
        self.eng = eng
        self.m = eng.group_views(master, "encoder")
        self.s = eng.group_views(shadow, "encoder") if shadow is not None else self.m
        # split-weight mode, fp8 form: the fp8 correction plane of the weights (views, and the flat
        # buffer for the fused QKV view); None: the bf16 lo plane serves every correction
        self.s8 = eng.group_views(lo8, "encoder") if lo8 is not None else None
        self.s8_flat = lo8
        self.lo8_exp = eng.lo8_exp
        # split-weight mode: every bf16 weight view of the forward GEMMs has its lo plane
        # lo_stride elements further on (shadows: the [2, n] plane buffers; the derived conv /
        # pos-conv layouts below: [2, ...] tensors, plane 0 = hi)
        self.lo = lo_stride
        a = eng.arch
        cdt = eng.cdt
        # conv 1..6 weights [co][ci][k] -> [co][k][ci] in the compute dtype
        self.conv_r, self.conv_lo = [], []   # conv_lo[i]: lo-plane offset of conv_r[i] (0: none)
        # fp8 form: conv_w8[i] = [fp8(w_hi) | fp8((w - w_hi) 2^conv_lo8_exp)] against the activations'
        # [fp8((x - x_hi) 2^e) | fp8(x_hi)]: x_hi w_hi (bf16) + 2^-e (x_lo8 w_hi8 + x_hi8 w_lo8)
        self.conv_split8 = bool(self.lo) and lo8 is not None and eng.conv_split8
        self.conv_lo8_exp = eng.conv_lo8_exp
        self.conv_w8 = []
        for i in range(1, len(a.conv_dim)):
            w = self.m[f"feature_extractor.conv_layers.{i}.conv.weight"]
            co, ci, k = w.shape
            if self.conv_split8:
                r32 = torch.empty(co, k * ci, device=eng.dev, dtype=F32)
                K.swap12(w, r32, co, ci, k)
                r = torch.empty(co, k * ci, device=eng.dev, dtype=cdt)
                K.cast(r32, r)
                w8 = torch.empty(2, co, k * ci, device=eng.dev, dtype=eng.corr_dt)
                K.cast_fp8(r, w8[0])
                K.split_lo8(r32, w8[1], self.conv_lo8_exp, sat=eng.sat_buf[SAT_CONV:SAT_CONV + 1])
                self.conv_r.append(r)
                self.conv_lo.append(0)
                self.conv_w8.append(w8)
            elif self.lo:
                # planes [hi | hi | lo] against the split activations' [hi | lo | hi] (NRSE_BF16X3):
                # three K segments of one GEMM, x_hi w_hi + x_lo w_hi + x_hi w_lo
                r32 = torch.empty(co, k * ci, device=eng.dev, dtype=F32)
                K.swap12(w, r32, co, ci, k)
                r3 = torch.empty(3, co, k * ci, device=eng.dev, dtype=cdt)
                K.split_bf16(r32, r3[0], r3[2])
                K.cast(r3[0], r3[1])
                self.conv_r.append(r3[0])
                self.conv_lo.append(r32.numel())
            else:
                r = torch.empty(co, k * ci, device=eng.dev, dtype=cdt)
                K.swap12(w, r, co, ci, k)
                self.conv_r.append(r)
                self.conv_lo.append(0)
        # pos-conv weight norm
        H, G, pk = a.hidden, a.pos_groups, a.pos_kernel
        cpg = H // G
        pre = "encoder.pos_conv_embed.conv.parametrizations.weight."
        self.wn_norms = torch.empty(pk, device=eng.dev, dtype=F32)
        if self.lo:
            wf32 = torch.empty(G, cpg, pk * cpg, device=eng.dev, dtype=F32)
            wd32 = torch.empty(G, cpg, pk * cpg, device=eng.dev, dtype=F32)
            K.weight_norm_fwd(self.m[pre + "original0"], self.m[pre + "original1"], wf32, wd32, self.wn_norms, H,
                              cpg, pk)
            wf2 = torch.empty(2, G, cpg, pk * cpg, device=eng.dev, dtype=cdt)
            K.split_bf16(wf32, wf2[0], wf2[1])
            self.wf, self.wf_lo = wf2[0], wf32.numel()
            self.wd = torch.empty(G, cpg, pk * cpg, device=eng.dev, dtype=cdt)
            K.cast(wd32, self.wd)   # the backward's dgrad reads the hi plane only
        else:
            self.wf = torch.empty(G, cpg, pk * cpg, device=eng.dev, dtype=cdt)
            self.wd = torch.empty(G, cpg, pk * cpg, device=eng.dev, dtype=cdt)
            self.wf_lo = 0
            K.weight_norm_fwd(self.m[pre + "original0"], self.m[pre + "original1"], self.wf, self.wd,
                              self.wn_norms, H, cpg, pk)


class ByolEngine:
    def __init__(self, arch: WavLMArch, proj_dim: int, pred_dim: int, *, device="cuda", compute_dtype=torch.bfloat16,
                 seed: int = 1234, step_cfg: StepConfig | None = None, init_flat: torch.Tensor | None = None,
                 do_normalize: bool = True, weight_split: bool = False, split_lo8: bool | None = None):
        if arch.head_dim != 64:
            raise _lib.NrseError(f"head_dim {arch.head_dim} unsupported (attention kernels are head_dim 64)")
        if weight_split and compute_dtype != torch.bfloat16:
            raise _lib.NrseError("weight_split is a bf16-mode option")
        self.arch = arch
        self.dev = torch.device(device)
        _lib.init_device(self.dev.index or 0)
        self.cdt = compute_dtype
        # split-weight mode: the forward GEMMs multiply by the weights' hi + lo bf16
        # pair (the f32 master to ~2^-17), activations stay bf16 -- the north-star 1e-3 embedding
        # bound at bf16 activation cost. The backward's dgrad uses the hi plane.
        self.wsplit = bool(weight_split)
        self.cfg = step_cfg or StepConfig()
        self.layout = PR.byol_layout(arch, proj_dim, pred_dim)
        self.proj_dim, self.pred_dim = proj_dim, pred_dim
        self.do_normalize = do_normalize
        flat = init_flat if init_flat is not None else PR.init_byol_flat(self.layout, seed)
        n, ne = self.layout.numel, self.layout.ema_numel
        self.online = flat.to(self.dev, F32).contiguous()
        self.target = self.online[:ne].clone()
        self.grad = torch.zeros(n, device=self.dev, dtype=F32)
        self.m = torch.zeros(n, device=self.dev, dtype=F32)
        self.v = torch.zeros(n, device=self.dev, dtype=F32)
        self.online_lo = self.target_lo = None
        # fp8 correction planes of the split-weight mode: fp8((w - bf16(w)) 2^lo8_exp)
        self.online_lo8 = self.target_lo8 = None
        self.lo8_exp = 0
        self.conv_lo8_exp = CONV_LO8_EXP if _CONV_LO8_PIN is None else int(_CONV_LO8_PIN)
        # ABI 10 saturation counters of the fp8 correction producers (cumulative since the last
        # re-derivation of the exponents): [SAT_WEIGHTS] the layer weights' planes (AdamW / EMA,
        # nrse_split_lo8), [SAT_CONV] the conv stack's weight and activation planes, [SAT_ACT] the
        # layer LayerNorms' fp8(bf16 y) copies. Read back lagged by health.HealthMonitor, which calls
        # rederive_split_exponents() when a count moves (no host sync in the step)
        self.sat_buf = torch.zeros(4, device=self.dev, dtype=torch.int32)
        self.sat_epoch = 0
        # the bf16 lo planes of the layer weights are skipped by the overlapped optimizer's layer
        # segments in the fp8 form (nothing reads them); a forward that falls back to them (fewer
        # than 128 frames in the batch: no fp8 segments) rebuilds them first (_ensure_lo_planes)
        self._lo_stale = {"online": False, "target": False}
        # the correction planes' dtype: fp8 e4m3 (ABI 8-10's MXFP6 alternative, measured slower at the
        # same accuracy in profiles/r05_mx6_ab.txt, was retired in ABI 11)
        self.corr_dt = FP8
        if self.cdt == F32:
            self.online_sh = None
            self.target_sh = None
        elif self.wsplit:
            # [2, n] planes: hi = bf16(w), lo = bf16(w - hi); a weight view's lo is n (ne) further on
            on2 = torch.empty(2, n, device=self.dev, dtype=self.cdt)
            tg2 = torch.empty(2, ne, device=self.dev, dtype=self.cdt)
            self.online_sh, self.online_lo = on2[0], on2[1]
            self.target_sh, self.target_lo = tg2[0], tg2[1]
            K.split_bf16(self.online, self.online_sh, self.online_lo)
            K.split_bf16(self.target, self.target_sh, self.target_lo)
            if _SPLIT_LO8 if split_lo8 is None else split_lo8:
                self.online_lo8 = torch.empty(n, device=self.dev, dtype=self.corr_dt)
                self.target_lo8 = torch.empty(ne, device=self.dev, dtype=self.corr_dt)
        else:
            self.online_sh = torch.empty(n, device=self.dev, dtype=self.cdt)
            self.target_sh = torch.empty(ne, device=self.dev, dtype=self.cdt)
            K.cast(self.online, self.online_sh)
            K.cast(self.target, self.target_sh)
        self.step_count = 0
        # the attention dropout keep bits computed ahead on a mask stream (NRSE_MASK_AHEAD, opt-in)
        self.mask_ahead = _MASK_AHEAD
        # split-weight fp8 form: the conv stack's correction segments in fp8 too (NRSE_CONV_SPLIT8);
        # conv_split8_used: whether the last forward ran them (frames >= 128, see encoder_forward)
        self.conv_split8 = _CONV_SPLIT8
        self.conv_split8_used = False
        self._offsets = {}
        self._view_cache = {}
        for gname, s in self.layout.specs:
            off, cnt, shp = self.layout.offsets[PR.GROUP_PREFIX[gname] + s.name]
            self._offsets.setdefault(gname, {})[s.name] = (off, cnt, shp)
        self._check_fused_views()
        if self.online_lo8 is not None:
            self._set_lo8_planes()
        # BatchNorm running statistics (buffers, not EMA'd: src/models/byol.py:62-73)
        self.bn = {}
        for net, dims in (("online_projector", (proj_dim, proj_dim)), ("target_projector", (proj_dim, proj_dim)),
                          ("online_predictor", (pred_dim, pred_dim))):
            for li, c in zip((1, 4), dims):
                self.bn[f"{net}.layers.{li}"] = (torch.zeros(c, device=self.dev), torch.ones(c, device=self.dev),
                                                 torch.zeros((), dtype=torch.long, device=self.dev))
        self._bn_count = {k: 0 for k in self.bn}   # num_batches_tracked, kept on the host (no step kernel)
        self._grad_zeroed = True                    # self.grad holds zeros (fresh, or a zero_grad AdamW ran)
        self._buckets = {}
        self.sumsq_buf = torch.zeros(1, device=self.dev, dtype=torch.float64)
        self.loss_buf = torch.zeros(1, device=self.dev, dtype=F32)
        self.health_buf = torch.zeros(4, 4, device=self.dev, dtype=F32)
        self.loss_stats = torch.zeros(2, device=self.dev, dtype=F32)
        self.executed_layers = [0, 0]
        # DDP option (nrse_amd/ddp.SyncBN): head BatchNorm statistics over all ranks' rows
        self.sync_bn = None
        # overlapped optimizer: per-segment "updated" events of the last step, and "done"
        self._opt_stream = None
        self._opt_events = None
        self._opt_done = None
        self._segments = self._param_segments()
        # ar_timing: record (end of backward, all exchanges done) events per step on the main
        # stream (bench.py reports the exposed all-reduce time from them)
        self.ar_timing = False
        self.ar_events = []

    def rederive_split_exponents(self) -> dict:
        """Re-derive lo8_exp / conv_lo8_exp from the current weights and rewrite the fp8 correction
        planes (host sync). Called when a saturation counter moved: the weights (or the conv
        LayerNorms' gamma / beta) grew past the exponents' 2x headroom during training."""
        self.sync_optimizer()
        torch.cuda.current_stream(self.dev).synchronize()
        counts = [int(v) for v in self.sat_buf.cpu()]
        old = (self.lo8_exp, self.conv_lo8_exp)
        if self.online_lo8 is not None:
            self._set_lo8_planes()
        torch.cuda.current_stream(self.dev).synchronize()
        self.sat_buf.zero_()
        self.sat_epoch += 1
        return dict(counts=counts, old=old, new=(self.lo8_exp, self.conv_lo8_exp))

    def _ensure_lo_planes(self, W: "EncoderWeights") -> None:
        """Rebuild network W's bf16 lo plane if the overlapped optimizer skipped it (fp8 form) and a
        forward is about to read it (the fallback for batches under 128 frames)."""
        net = W.net
        if not self._lo_stale.get(net):
            return
        self.sync_optimizer()
        master, lo = (self.online, self.online_lo) if net == "online" else (self.target, self.target_lo)
        scratch = torch.empty_like(lo)   # the hi plane is current: only lo is written
        K.split_bf16(master, scratch, lo)
        self._lo_stale[net] = False

    def refresh_shadows(self, which=("online", "target")) -> None:
        """Re-derive the bf16 GEMM-operand copies (and the split mode's lo planes) of the f32
        weights after they were changed outside the fused AdamW / EMA kernels."""
        for w in which:
            src, sh, lo = ((self.online, self.online_sh, self.online_lo) if w == "online"
                           else (self.target, self.target_sh, self.target_lo))
            if sh is None:
                continue
            if lo is not None:
                K.split_bf16(src, sh, lo)
            else:
                K.cast(src, sh)
        if self.online_lo8 is not None:
            self._set_lo8_planes()   # the exponent follows the (possibly loaded) weights' range

    def _lo8_weights(self, flat: torch.Tensor) -> list:
        """The weight matrices whose forward GEMM takes the fp8 correction segment (the layers'
        QKV, out-projection, FFN-up, FFN-down; encoder_forward)."""
        out = []
        for li in range(self.arch.layers):
            p = f"encoder.layers.{li}."
            out.append(self.fused(flat, li, "qkv_w"))
            for n in ("attention.out_proj.weight", "feed_forward.intermediate_dense.weight",
                      "feed_forward.output_dense.weight"):
                off, cnt, shp = self._offsets["encoder"][p + n]
                out.append(flat[off:off + cnt])
        return out

    def _set_lo8_planes(self) -> None:
        """Choose lo8_exp from the range of the fp8-corrected weights and write both networks' fp8
        correction planes (nrse_split_lo8). |w - bf16(w)| <= 2^-8 |w|, so with W = max |w| the plane's
        values stay below 448 / 2 (2x headroom for weights that grow in training; beyond it the
        conversion saturates) at lo8_exp = floor(log2(224 / (2^-8 W))); the smallest weights fall to
        fp8 subnormals, whose absolute error (2^-9 2^-lo8_exp) is far below the bf16 residual itself."""
        W = max(float(t.abs().max()) for f in (self.online, self.target) for t in self._lo8_weights(f))
        self.lo8_exp = _headroom_exp(W)
        if _CONV_LO8_PIN is None:
            self.conv_lo8_exp = _headroom_exp(self._conv_plane_bound())
        K.split_lo8(self.online, self.online_lo8, self.lo8_exp)
        K.split_lo8(self.target, self.target_lo8, self.lo8_exp)
        # the saturation count over the planes the layer GEMMs read (the rest of the buffer --
        # norms, biases, heads -- is outside the exponent's range and never read): rewritten
        # per matrix with the counter (the same bytes)
        sat = self.sat_buf[SAT_WEIGHTS:SAT_WEIGHTS + 1]
        for flat, plane in ((self.online, self.online_lo8), (self.target, self.target_lo8)):
            for s, e in self._lo8_ranges():
                K.split_lo8(flat[s:e], plane[s:e], self.lo8_exp, sat=sat)

    def _lo8_ranges(self) -> list:
        """Sorted [start, end) flat ranges of the fp8-corrected layer matrices (QKV, out-projection,
        FFN-up, FFN-down of every layer)."""
        if getattr(self, "_lo8_rng", None) is None:
            out = []
            for li in range(self.arch.layers):
                p = f"encoder.layers.{li}."
                off = self._offsets["encoder"][p + "attention.q_proj.weight"][0]
                out.append((off, off + 3 * self.arch.hidden ** 2))
                for n in ("attention.out_proj.weight", "feed_forward.intermediate_dense.weight",
                          "feed_forward.output_dense.weight"):
                    off, cnt, _ = self._offsets["encoder"][p + n]
                    out.append((off, off + cnt))
            self._lo8_rng = sorted(out)
            self._lo8_rng_dev = torch.tensor(self._lo8_rng, dtype=torch.int64, device=self.dev).contiguous()
        return self._lo8_rng

    def _conv_plane_bound(self) -> float:
        """The largest value the conv stack's fp8 correction planes carry unscaled (host sync): the
        conv activations feeding conv 1..n-1 are GELU(LayerNorm_C) outputs, |x| <= sqrt(C) max|gamma|
        + max|beta| (GELU(z) <= max(z, 0) + 0.17), and the conv weights' |w|; each residual is at
        most 2^-8 of it (oracle/wavlm_byol.py conv_lo8_exponent restates this)."""
        a = self.arch
        B = 0.0
        for flat in (self.online, self.target):
            P = self.group_views(flat, "encoder")
            for i in range(len(a.conv_dim) - 1):
                pre = f"feature_extractor.conv_layers.{i}."
                g = float(P[pre + "layer_norm.weight"].abs().max())
                b = float(P[pre + "layer_norm.bias"].abs().max())
                B = max(B, math.sqrt(a.conv_dim[i]) * g + b)
            for i in range(1, len(a.conv_dim)):
                B = max(B, float(P[f"feature_extractor.conv_layers.{i}.conv.weight"].abs().max()))
        return B

    def bn_state(self, key: str) -> tuple:
        """(running_mean, running_var, num_batches_tracked) of a head BatchNorm; the counter is kept
        on the host during training and written into its buffer here."""
        rm, rv, nbt = self.bn[key]
        nbt.fill_(self._bn_count[key])
        return rm, rv, nbt

    def bn_counts_from_buffers(self) -> None:
        """Adopt num_batches_tracked values written into the buffers (a loaded checkpoint)."""
        for k, (_, _, nbt) in self.bn.items():
            self._bn_count[k] = int(nbt)

    # ------------------------------------------------------------------ overlapped optimizer
    def _param_segments(self) -> list:
        """Flat-buffer ranges in the order the forward consumes them: [front end .. layer 0],
        layer 1, ..., layer L-1, [final LN + heads]. Boundaries are rounded UP to 4 elements
        (the kernels' float4 alignment), which can only move an element into an EARLIER segment."""
        a = self.arch
        n = self.layout.numel
        cuts = [0] + [PR.layer_range(self.layout, a, li)[0] for li in range(1, a.layers)]
        cuts.append(PR.layer_range(self.layout, a, a.layers - 1)[1])
        cuts = [min(n, (c + 3) // 4 * 4) for c in cuts] + [n]
        return [(cuts[i], cuts[i + 1]) for i in range(len(cuts) - 1)]

    def _param_wait(self, seg: int) -> None:
        """The current stream waits until segment `seg` of the last optimizer step is updated
        (no-op unless the optimizer step was overlapped)."""
        if self._opt_events is not None:
            torch.cuda.current_stream(self.dev).wait_event(self._opt_events[seg])

    def sync_optimizer(self) -> None:
        """The current stream waits for the whole last optimizer step (parameters, moments, EMA,
        grad buffer reads). Called by every entry point that reads or writes the flat buffers
        outside the overlapped forward."""
        if self._opt_done is not None:
            torch.cuda.current_stream(self.dev).wait_event(self._opt_done)

    # ------------------------------------------------------------------ views
    def group_views(self, flat: torch.Tensor, group: str, cached: bool = True) -> dict:
        """name -> view of `flat` for every parameter of `group`. Cached per (buffer object,
        group): building the encoder's ~400 views costs ~1.5 ms of host time, and the step asks
        for them five times (both views' master and shadow weights, the gradient), which delayed
        the enqueue of each step's first kernels. The cache holds the buffer itself and is keyed
        on its identity, so a replaced buffer (load_state_dict) gets fresh views."""
        key = (id(flat), group)
        hit = self._view_cache.get(key) if cached else None
        if hit is not None and hit[0] is flat:
            return hit[1]
        out = {}
        for name, (off, cnt, shp) in self._offsets[group].items():
            out[name] = flat[off:off + cnt].view(shp)
        if not cached:   # a caller that hands the views out (WavLMEncoder.model): its own objects
            return out
        if len(self._view_cache) >= 32:   # callers passing transient buffers: stay bounded
            self._view_cache.clear()
        self._view_cache[key] = (flat, out)
        return out

    def fused(self, flat: torch.Tensor, layer: int, kind: str) -> torch.Tensor:
        H = self.arch.hidden
        pre = f"encoder.layers.{layer}.attention."
        if kind == "qkv_w":
            off = self._offsets["encoder"][pre + "q_proj.weight"][0]
            return flat[off:off + 3 * H * H].view(3 * H, H)
        off = self._offsets["encoder"][pre + "q_proj.bias"][0]
        return flat[off:off + 3 * H]

    def _check_fused_views(self):
        H = self.arch.hidden
        for li in range(self.arch.layers):
            pre = f"encoder.layers.{li}.attention."
            o = self._offsets["encoder"]
            qw, kw, vw = (o[pre + n + "_proj.weight"][0] for n in "qkv")
            qb, kb, vb = (o[pre + n + "_proj.bias"][0] for n in "qkv")
            assert kw == qw + H * H and vw == kw + H * H, "q/k/v weights must be adjacent in the flat layout"
            assert kb == qb + H and vb == kb + H, "q/k/v biases must be adjacent in the flat layout"

    def buckets(self, T: int) -> torch.Tensor:
        if T not in self._buckets:
            a = self.arch
            self._buckets[T] = torch.from_numpy(bucket_vector(T, a.num_buckets, a.max_distance)).to(self.dev)
        return self._buckets[T]

    def bucket_runs(self, T: int) -> tuple[torch.Tensor, torch.Tensor]:
        """(order, offsets) of buckets(T) for the gather-form rel-pos bias backward."""
        key = ("runs", T)
        if key not in self._buckets:
            order, offsets = bucket_runs(bucket_vector(T, self.arch.num_buckets, self.arch.max_distance),
                                         self.arch.num_buckets)
            self._buckets[key] = (torch.from_numpy(order).to(self.dev), torch.from_numpy(offsets).to(self.dev))
        return self._buckets[key]

    # ------------------------------------------------------------------ encoder forward
    def encoder_forward(self, W: EncoderWeights, wav: torch.Tensor, *, train: bool, fseed: int = 0, skip=None,
                        mask_np=None, need_grad: bool = False, hidden_dtype=None):
        """WavLMModel.forward -> time-mean embedding [B, H] (f32) and the backward tape; with
        hidden_dtype, the last_hidden_state [B, T, H] in that dtype instead of the embedding
        (src/models/encoder.py:25-32, the emotion head's input; no tape)."""
        a = self.arch
        cdt = self.cdt
        dev = self.dev
        B, L = wav.shape
        Pm, Ps = W.m, W.s
        tape = Tape(B=B, wav=wav, fseed=fseed) if need_grad else None
        # -------- conv feature encoder ([TF]modeling_wavlm.py:712-720, 773-783)
        k0, s0, C0 = a.conv_kernel[0], a.conv_stride[0], a.conv_dim[0]
        T0 = (L - k0) // s0 + 1
        # split-weight mode: the conv stack also carries its activations as split bf16 planes
        # (NRSE_BF16X3 [hi | lo | hi], read by 3-segment GEMMs) and its pre-activations in f32 --
        # the activation roundings that remain in this mode are otherwise dominated by the conv
        # stack (tools/ablate_bf16_sites.py: 6e-4 of 7e-4 at 8 s, more at 3 s)
        # fp8 form (W.conv_split8, ABI 7): a bf16 hi plane + the fp8 planes [fp8(x_lo 2^e) | fp8(x_hi)],
        # read by one bf16 and two fp8 K segments
        split = self.wsplit
        # (the fp8 segments run on the 256x256 kernel only, which needs M = frames >= 128 per
        # utterance at every conv layer: audio shorter than ~2.6 s keeps the three bf16 planes)
        t_last = T0
        for k_, s_ in zip(a.conv_kernel[1:], a.conv_stride[1:]):
            t_last = (t_last - k_) // s_ + 1
        s8 = split and W.conv_split8 and t_last >= 128
        self.conv_split8_used = s8
        split3 = split and not s8
        e8 = W.conv_lo8_exp
        nconv = len(a.conv_dim)
        y = torch.empty((3, B * T0, C0) if split3 else (B * T0, C0), device=dev, dtype=cdt)
        x8 = torch.empty(2, B * T0, C0, device=dev, dtype=self.corr_dt) if s8 else None
        mean = torch.empty(B * T0, device=dev, dtype=F32)
        rstd = torch.empty(B * T0, device=dev, dtype=F32)
        pre0 = "feature_extractor.conv_layers.0."
        K.conv0_fwd(wav, Pm[pre0 + "conv.weight"], Pm[pre0 + "layer_norm.weight"], Pm[pre0 + "layer_norm.bias"], y,
                    mean, rstd, T0, k0, s0, a.eps, split3=split3, y8=x8, y8_exp=e8,
                    sat=self.sat_buf[SAT_CONV:SAT_CONV + 1] if s8 else None)
        if need_grad:
            tape.conv.append(dict(mean=mean, rstd=rstd, T=T0))
        x, Tin, Cin = (y[0] if split3 else y), T0, C0
        for i in range(1, nconv):
            k, s, C = a.conv_kernel[i], a.conv_stride[i], a.conv_dim[i]
            Tout = (Tin - k) // s + 1
            pre_out = torch.empty(B * Tout, C, device=dev, dtype=F32 if split else cdt)
            f8 = {}
            if s8:
                f8 = dict(a8=K.Operand(x8, True, s * Cin, z1=Tin * Cin, seg_stride=B * Tin * Cin),
                          b8=K.Operand(W.conv_w8[i - 1], True, k * Cin, seg_stride=C * k * Cin), nseg8=2, b8_exp=e8)
            K.gemm(K.Operand(x, True, s * Cin, z1=Tin * Cin, seg_stride=B * Tin * Cin if split3 else 0),
                   K.Operand(W.conv_r[i - 1], True, k * Cin, seg_stride=W.conv_lo[i - 1]), pre_out,
                   Tout, C, k * Cin, ldc=C, batch=B, c_z1=Tout * C, nseg=3 if split3 else 1, **f8)
            # the last layer's output feeds only the feature-projection LN: f32 in the split mode
            last = i == nconv - 1
            yo8 = None
            if split and last:
                yo3 = torch.empty(B * Tout, C, device=dev, dtype=F32)
            elif split3:
                yo3 = torch.empty(3, B * Tout, C, device=dev, dtype=cdt)
            else:
                yo3 = torch.empty(B * Tout, C, device=dev, dtype=cdt)
                if s8:
                    yo8 = torch.empty(2, B * Tout, C, device=dev, dtype=self.corr_dt)
            mo = torch.empty(B * Tout, device=dev, dtype=F32)
            ro = torch.empty(B * Tout, device=dev, dtype=F32)
            p = f"feature_extractor.conv_layers.{i}."
            K.ln_fwd(pre_out, Pm[p + "layer_norm.weight"], Pm[p + "layer_norm.bias"], yo3, mo, ro, a.eps, gelu=True,
                     split3=split3 and not last, y8=yo8, y8_exp=e8 if yo8 is not None else None,
                     sat=self.sat_buf[SAT_CONV:SAT_CONV + 1] if yo8 is not None else None)
            if need_grad:
                tape.conv.append(dict(x=x, pre=pre_out, mean=mo, rstd=ro, Tin=Tin, T=Tout, k=k, s=s))
            x, x8, Tin, Cin = (yo3[0] if split3 and not last else yo3), yo8, Tout, C
        T = Tin
        C = Cin
        H = a.hidden
        BT = B * T
        feats = x
        # -------- feature projection + dropout ([TF]modeling_wavlm.py:93-105)
        xn = torch.empty(BT, C, device=dev, dtype=cdt)
        fm = torch.empty(BT, device=dev, dtype=F32)
        fr = torch.empty(BT, device=dev, dtype=F32)
        K.ln_fwd(feats, Pm["feature_projection.layer_norm.weight"], Pm["feature_projection.layer_norm.bias"], xn, fm,
                 fr, a.eps)
        h = torch.empty(BT, H, device=dev, dtype=F32)
        pfp = a.feat_proj_dropout if train else 0.0
        K.linear_fwd(xn, Ps["feature_projection.projection.weight"], h, bias=Pm["feature_projection.projection.bias"],
                     dropout_p=pfp, seed=R.site_seed(fseed, R.SITE_FEAT_PROJ), w_lo=W.lo)
        # -------- SpecAugment ([TF]modeling_wavlm.py:985-1011) + padded copy for the pos-conv
        pk, G = a.pos_kernel, a.pos_groups
        cpg = H // G
        mask = None
        if train and isinstance(mask_np, (int, np.integer)):
            # the time masks drawn on the device from the forward's mask seed (nrse_specaug_mask,
            # ABI 10): no host RNG and no host-to-device copy in the step
            if a.mask_time_prob > 0 and a.mask_time_length >= 1:
                mask = torch.empty(B, T, device=dev, dtype=torch.uint8)
                K.specaug_mask(mask, a.mask_time_prob, a.mask_time_length, a.mask_time_min_masks, int(mask_np))
        elif train and mask_np is not None and mask_np.any():
            # explicit host masks (tests, replays): pinned staging -- a copy from pageable memory
            # blocks the host until the stream reaches it
            mask = torch.from_numpy(mask_np.astype(np.uint8)).pin_memory().to(dev, non_blocking=True)
        hpad = torch.empty(B, T + pk, H, device=dev, dtype=cdt)
        K.specaug_pad(h, mask, Pm.get("masked_spec_embed"), hpad, B, T, H, pk // 2, pk - pk // 2)
        # -------- positional conv + residual + dropout ([TF]modeling_wavlm.py:48-90, 476-483)
        h0 = torch.empty(BT, H, device=dev, dtype=F32)
        pos_pre = torch.empty(BT, H, device=dev, dtype=cdt)
        php = a.hidden_dropout if train else 0.0
        cs = int(math.log2(cpg))
        K.gemm(K.Operand(hpad, True, H, chunk_shift=cs, ld_chunk=H, z1=(T + pk) * H, z2=cpg),
               K.Operand(W.wf, True, pk * cpg, z2=cpg * pk * cpg, seg_stride=W.wf_lo), h0, T, cpg, pk * cpg, ldc=H,
               batch=B * G, zdiv=G, nseg=2 if W.wf_lo else 1,
               c_z1=T * H, c_z2=cpg, bias=Pm["encoder.pos_conv_embed.conv.bias"], bias_z2=cpg,
               flags=_lib.EPI_GELU | _lib.EPI_DROP_AFTER, aux=pos_pre, ldaux=H, aux_z1=T * H, aux_z2=cpg,
               resid=h, ldr=H, r_z1=T * H, r_z2=cpg, dropout_p=php, seed=R.site_seed(fseed, R.SITE_POS))
        # -------- relative position bias table (layer 0 computes it, every layer reuses it)
        nh = a.heads
        # bf16 (MFMA) attention reads the Toeplitz vector [nh, 2T-1] (the bias depends on j - i
        # only); the f32 parity kernels read the [nh, T, Tb] table
        E_rel = Pm["encoder.layers.0.attention.rel_attn_embed.weight"]
        if cdt == torch.bfloat16:
            bias_tab = None
            bias_vec = torch.empty(nh, 2 * T - 1, device=dev, dtype=F32)
            K.rel_bias_vec(E_rel, self.buckets(T), bias_vec, nh, T)
        else:
            bias_vec = None
            bias_tab = torch.empty(nh, T, K.bias_ld(T), device=dev, dtype=F32)
            K.rel_bias_fwd(E_rel, self.buckets(T), bias_tab, nh, T)
        if need_grad:
            tape.T = T
            tape.feats, tape.fp_mean, tape.fp_rstd, tape.xn = feats, fm, fr, xn
            tape.mask, tape.hpad, tape.pos_pre, tape.bias_tab, tape.bias_vec = mask, hpad, pos_pre, bias_tab, bias_vec
            tape.pos = dict(W=W)
        del xn, feats
        # -------- transformer layers ([TF]modeling_wavlm.py:488-513, 355-373)
        F_ = a.ffn
        hcur = h0
        # the fp8 correction segments need the 256x256 kernel (M = B*T >= 128 rows); a smaller batch
        # (one clip under ~2.6 s, a short validation tail) takes the bf16 lo plane instead, rebuilt
        # first if the overlapped optimizer skipped it
        lo8 = W.s8 is not None and BT >= 128
        if W.s8 is not None and not lo8:
            self._ensure_lo_planes(W)
        sat_a = self.sat_buf[SAT_ACT:SAT_ACT + 1] if lo8 else None

        def corr(x8, w8):
            # the weight correction of a layer GEMM: the fp8 segment (x8, w8) or the bf16 lo plane
            return dict(x8=x8, w8=w8, lo8_exp=W.lo8_exp) if lo8 else dict(w_lo=W.lo)
        pat = a.attention_dropout if train else 0.0
        pact = a.activation_dropout if train else 0.0
        executed = 0
        for li in range(a.layers):
            if li > 0:
                self._param_wait(li)  # layer li's parameters of the overlapped optimizer step
            if train and skip is not None and skip[li]:
                continue
            executed += 1
            p = f"encoder.layers.{li}."
            # the probability-dropout keep bits of this layer (bf16 path): computed ahead on a mask
            # stream, beside this layer's LN1 / QKV GEMM (a pure-VALU kernel whose waves fit on the
            # GEMM's SIMDs), then read by the attention forward instead of hashed in it; the online
            # view keeps them for the backward
            dmask, mask_ev = None, None
            if pat > 0 and bias_vec is not None:
                dmask = torch.empty(K.attn_mask_elems(B, T, nh), device=dev, dtype=torch.int16)
                if self.mask_ahead:
                    cur = torch.cuda.current_stream(dev)
                    ms = self._mask_stream(cur)
                    ms.wait_stream(cur)
                    with torch.cuda.stream(ms):
                        K.attn_dropout_mask(dmask, B, T, nh, pat, R.site_seed(fseed, R.site_attn_probs(li)))
                        mask_ev = torch.cuda.Event()
                        mask_ev.record(ms)
                elif not need_grad:
                    dmask = None  # hashed in the forward, not recorded
            x1 = torch.empty(BT, H, device=dev, dtype=cdt)
            m1 = torch.empty(BT, device=dev, dtype=F32)
            r1 = torch.empty(BT, device=dev, dtype=F32)
            # split-weight mode, fp8 form: the LN outputs' fp8 copies feed the correction segments
            x1_8 = torch.empty(BT, H, device=dev, dtype=self.corr_dt) if lo8 else None
            K.ln_fwd(hcur, Pm[p + "layer_norm.weight"], Pm[p + "layer_norm.bias"], x1, m1, r1, a.eps, y8=x1_8,
                     sat=sat_a)
            qkv = torch.empty(BT, 3 * H, device=dev, dtype=cdt)
            K.linear_fwd(x1, self.fused(W.s_flat, li, "qkv_w"), qkv, bias=self.fused(W.m_flat, li, "qkv_b"),
                         **corr(x1_8, self.fused(W.s8_flat, li, "qkv_w") if lo8 else None))
            del x1_8
            gate = torch.empty(B, nh, T, device=dev, dtype=F32)
            at = p + "attention."
            K.gate_fwd(x1, Pm[at + "gru_rel_pos_linear.weight"], Pm[at + "gru_rel_pos_linear.bias"],
                       Pm[at + "gru_rel_pos_const"], gate, B, T, nh)
            ctx = torch.empty(BT, H, device=dev, dtype=cdt)
            ctx8 = torch.empty(BT, H, device=dev, dtype=self.corr_dt) if lo8 else None
            lse = torch.empty(B, nh, T, device=dev, dtype=F32)
            if mask_ev is not None:
                torch.cuda.current_stream(dev).wait_event(mask_ev)
            # (without the mask stream the forward hashes and, for the online view, records the bits)
            K.attn_fwd(qkv, gate, bias_tab, ctx, lse, B, T, nh, pat, R.site_seed(fseed, R.site_attn_probs(li)),
                       bias_vec=bias_vec, drop_mask=dmask, mask_in=mask_ev is not None, ctx8=ctx8)
            hmid = torch.empty(BT, H, device=dev, dtype=F32)
            K.linear_fwd(ctx, Ps[at + "out_proj.weight"], hmid, bias=Pm[at + "out_proj.bias"], resid=hcur, ldr=H,
                         dropout_p=php, seed=R.site_seed(fseed, R.site_attn_out(li)),
                         **corr(ctx8, W.s8[at + "out_proj.weight"] if lo8 else None))
            del ctx8
            x2 = torch.empty(BT, H, device=dev, dtype=cdt)
            m2 = torch.empty(BT, device=dev, dtype=F32)
            r2 = torch.empty(BT, device=dev, dtype=F32)
            x2_8 = torch.empty(BT, H, device=dev, dtype=self.corr_dt) if lo8 else None
            K.ln_fwd(hmid, Pm[p + "final_layer_norm.weight"], Pm[p + "final_layer_norm.bias"], x2, m2, r2, a.eps,
                     y8=x2_8, sat=sat_a)
            f1pre = torch.empty(BT, F_, device=dev, dtype=cdt) if need_grad else None
            g1 = torch.empty(BT, F_, device=dev, dtype=cdt)
            # (fp8 form: the FFN-up epilogue also writes fp8(g1), FFN-down's correction operand; the
            # activation dropout, 0 in the step, would come before that copy is taken)
            g1_8 = torch.empty(BT, F_, device=dev, dtype=self.corr_dt) if lo8 else None
            K.linear_fwd(x2, Ps[p + "feed_forward.intermediate_dense.weight"], g1,
                         bias=Pm[p + "feed_forward.intermediate_dense.bias"], flags=_lib.EPI_GELU, aux=f1pre,
                         ldaux=F_, dropout_p=pact, seed=R.site_seed(fseed, R.site_act(li)), out8=g1_8,
                         **corr(x2_8, W.s8[p + "feed_forward.intermediate_dense.weight"] if lo8 else None))
            del x2_8
            hout = torch.empty(BT, H, device=dev, dtype=F32)
            K.linear_fwd(g1, Ps[p + "feed_forward.output_dense.weight"], hout,
                         bias=Pm[p + "feed_forward.output_dense.bias"], resid=hmid, ldr=H, dropout_p=php,
                         seed=R.site_seed(fseed, R.site_ffn_out(li)),
                         **corr(g1_8, W.s8[p + "feed_forward.output_dense.weight"] if lo8 else None))
            del g1_8
            if need_grad:
                tape.layers.append(dict(li=li, h_in=hcur, x1=x1, m1=m1, r1=r1, qkv=qkv, gate=gate, ctx=ctx, lse=lse,
                                        hmid=hmid, x2=x2, m2=m2, r2=r2, f1pre=f1pre, g1=g1, dmask=dmask))
            hcur = hout
        self._param_wait(a.layers)  # final LN (+ the heads that follow)
        if hidden_dtype is not None:
            # -------- final LN -> last_hidden_state ([TF]modeling_wavlm.py:513)
            y = torch.empty(BT, H, device=dev, dtype=hidden_dtype)
            mf = torch.empty(BT, device=dev, dtype=F32)
            rf = torch.empty(BT, device=dev, dtype=F32)
            K.ln_fwd(hcur, Pm["encoder.layer_norm.weight"], Pm["encoder.layer_norm.bias"], y, mf, rf, a.eps)
            return y.view(B, T, H), None, executed
        # -------- final LN + time-mean shim
        emb = torch.empty(B, H, device=dev, dtype=F32)
        K.zero(emb)
        mf = torch.empty(BT, device=dev, dtype=F32)
        rf = torch.empty(BT, device=dev, dtype=F32)
        K.ln_mean_fwd(hcur, Pm["encoder.layer_norm.weight"], Pm["encoder.layer_norm.bias"], emb, mf, rf, B, T, H,
                      a.eps)
        if need_grad:
            tape.final = (hcur, mf, rf)
        return emb, tape, executed

    # ------------------------------------------------------------------ encoder backward
    def encoder_backward(self, tape: Tape, demb: torch.Tensor, Gv: dict, W: EncoderWeights, on_layer=None,
                         on_front=None) -> None:
        """Accumulate d(loss)/d(encoder params) into the grad views Gv given d(loss)/d(emb).
        on_layer(li), if given, is called once layer li's gradients are all enqueued (main and
        side stream) and no later kernel writes them (layer 0 excepted: rel_attn_embed).
        on_front(name), if given, likewise for the front-end groups of _grad_groups(): "rel",
        "posconv", "proj", "conv6" .. "conv1", "conv0" (in that order)."""
        def front(name):
            if on_front is not None:
                on_front(name)
        a = self.arch
        cdt = self.cdt
        dev = self.dev
        B, T = tape.B, tape.T
        H, F_, nh = a.hidden, a.ffn, a.heads
        BT = B * T
        Pm, Ps = W.m, W.s
        fseed = tape.fseed
        train = True
        php, pat, pact = a.hidden_dropout, a.attention_dropout, a.activation_dropout
        # final LN (+ time-mean): dy[b,t] = demb[b] / T
        hfin, mf, rf = tape.final
        dh = torch.empty(BT, H, device=dev, dtype=F32)
        order = list(reversed(tape.layers))

        dv2_next, kw = self._ffn_out_dropout(order, 0, Gv, BT, fseed)
        K.ln_bwd(demb, hfin, Pm["encoder.layer_norm.weight"], mf, rf, dh, dgamma=Gv["encoder.layer_norm.weight"],
                 dbeta=Gv["encoder.layer_norm.bias"], mode=_lib.DY_BCAST, bcast_t=T, dy_scale=1.0 / T, rows=BT, **kw)
        tape.final = None
        diag = torch.empty(nh, 2 * T - 1, device=dev, dtype=F32)
        K.zero(diag)
        delta = torch.empty(B, nh, T, device=dev, dtype=F32)
        # the transformer layers' weight gradients (off the dX critical path) run on a side stream
        main = torch.cuda.current_stream(dev)
        # each layer's ordered gradient reductions (LayerNorm gamma / beta and fused bias column
        # sums, the FFN-up bias column sums, the rel-pos diagonals, the gate parameters: ~6 small
        # launches) are queued and run batched on the side stream after the layer (ABI 9), off
        # the dX chain; their destinations are read only by the all-reduce units (enqueued on the
        # side stream after them), the rel-pos bias backward and the optimizer (after the joins)
        defer = _DEFER_REDUCE and not _SERIAL_TARGET
        if defer and K.reduce_pending():
            raise _lib.NrseError(f"{K.reduce_pending()} deferred reductions pending before the backward")
        try:
            dh = self._layers_backward(order, tape, Gv, W, dh, dv2_next, diag, delta, defer, on_layer)
        except BaseException:
            if defer:
                K.reduce_discard()   # the queued jobs' workspaces are about to be released: never flush them
            raise
        self._front_backward(tape, Gv, W, dh, diag, front)

    def _ffn_out_dropout(self, order, j, Gv, BT, fseed):
        """The fused consumer of a layer-output gradient: layer order[j]'s FFN output-dropout
        backward + output_dense bias gradient (kwargs of K.ln_bwd), and its bf16/f32 result."""
        if j >= len(order):
            return None, {}
        lj = order[j]["li"]
        dv = torch.empty(BT, self.arch.hidden, device=self.dev, dtype=self.cdt)
        return dv, dict(dv=dv, dv_colsum=Gv[f"encoder.layers.{lj}.feed_forward.output_dense.bias"],
                        dv_p=self.arch.hidden_dropout, dv_seed=R.site_seed(fseed, R.site_ffn_out(lj)))

    def _layers_backward(self, order, tape, Gv, W, dh, dv2_next, diag, delta, defer, on_layer):
        """The transformer layers' backward, top layer first (encoder_backward); returns the
        gradient of the first layer's input."""
        a = self.arch
        cdt = self.cdt
        dev = self.dev
        B, T = tape.B, tape.T
        H, F_, nh = a.hidden, a.ffn, a.heads
        BT = B * T
        Pm, Ps = W.m, W.s
        fseed = tape.fseed
        php, pat, pact = a.hidden_dropout, a.attention_dropout, a.activation_dropout
        main = torch.cuda.current_stream(dev)
        for j, L_ in enumerate(order):
            li = L_["li"]
            p = f"encoder.layers.{li}."
            at = p + "attention."
            if defer:
                K.reduce_defer(True)
            # FFN branch (its output-dropout backward was fused into the LN backward that made dh)
            dv2 = dv2_next
            df1 = torch.empty(BT, F_, device=dev, dtype=cdt)
            K.linear_dgrad(dv2, Ps[p + "feed_forward.output_dense.weight"], df1, flags=_lib.EPI_GELU_BWD,
                           aux=L_["f1pre"], ldaux=F_, dropout_p=pact, seed=R.site_seed(fseed, R.site_act(li)),
                           colsum=Gv[p + "feed_forward.intermediate_dense.bias"])
            with self._wgrad_stream(main, dv2, df1, L_["g1"], L_["x2"]):
                K.linear_wgrad(dv2, L_["g1"], Gv[p + "feed_forward.output_dense.weight"])
                K.linear_wgrad(df1, L_["x2"], Gv[p + "feed_forward.intermediate_dense.weight"])
            dx2 = torch.empty(BT, H, device=dev, dtype=F32)
            K.linear_dgrad(df1, Ps[p + "feed_forward.intermediate_dense.weight"], dx2)
            del df1, dv2
            dhmid = torch.empty(BT, H, device=dev, dtype=F32)
            dv1 = torch.empty(BT, H, device=dev, dtype=cdt)
            # + the attention output-dropout backward and out_proj bias gradient, fused
            K.ln_bwd(dx2, L_["hmid"], Pm[p + "final_layer_norm.weight"], L_["m2"], L_["r2"], dhmid, resid=dh,
                     dgamma=Gv[p + "final_layer_norm.weight"], dbeta=Gv[p + "final_layer_norm.bias"],
                     dv=dv1, dv_colsum=Gv[at + "out_proj.bias"], dv_p=php,
                     dv_seed=R.site_seed(fseed, R.site_attn_out(li)))
            del dx2
            # attention branch
            dctx = torch.empty(BT, H, device=dev, dtype=cdt)
            K.linear_dgrad(dv1, Ps[at + "out_proj.weight"], dctx)
            with self._wgrad_stream(main, dv1, L_["ctx"]):
                K.linear_wgrad(dv1, L_["ctx"], Gv[at + "out_proj.weight"])
            del dv1
            dqkv = torch.empty(BT, 3 * H, device=dev, dtype=cdt)
            dgate = torch.empty(B, nh, T, device=dev, dtype=F32)
            K.attn_bwd(L_["qkv"], L_["gate"], tape.bias_tab, L_["ctx"], dctx, L_["lse"], delta, dqkv, dgate, diag, B,
                       T, nh, pat, R.site_seed(fseed, R.site_attn_probs(li)), bias_vec=tape.bias_vec,
                       drop_mask=L_["dmask"])
            del dctx
            # the gate path's backward: its parameter gradients and each (row, head)'s (dpa, dpb),
            # which the LN1 backward below adds to dx1 as it reads it (no dx1 read-modify-write)
            gdp = torch.empty(BT, nh, 2, device=dev, dtype=F32) if _GATE_INTO_LN else None
            if gdp is not None:
                K.gate_bwd_dp(L_["x1"], Pm[at + "gru_rel_pos_linear.weight"], Pm[at + "gru_rel_pos_linear.bias"],
                              Pm[at + "gru_rel_pos_const"], dgate, gdp, Gv[at + "gru_rel_pos_linear.weight"],
                              Gv[at + "gru_rel_pos_linear.bias"], Gv[at + "gru_rel_pos_const"], B, T, nh)
            with self._wgrad_stream(main, dqkv, L_["x1"]):
                K.linear_wgrad(dqkv, L_["x1"], self.fused(self.grad_flat_for(Gv), li, "qkv_w"))
                K.colsum(dqkv, self.fused(self.grad_flat_for(Gv), li, "qkv_b"))
            dx1 = torch.empty(BT, H, device=dev, dtype=F32)
            K.linear_dgrad(dqkv, self.fused(W.s_flat, li, "qkv_w"), dx1)
            del dqkv
            if gdp is None:  # the read-modify-write form (NRSE_GATE_INTO_LN=0, A/B)
                K.gate_bwd(L_["x1"], Pm[at + "gru_rel_pos_linear.weight"], Pm[at + "gru_rel_pos_linear.bias"],
                           Pm[at + "gru_rel_pos_const"], dgate, dx1, Gv[at + "gru_rel_pos_linear.weight"],
                           Gv[at + "gru_rel_pos_linear.bias"], Gv[at + "gru_rel_pos_const"], B, T, nh)
            dhin = torch.empty(BT, H, device=dev, dtype=F32)
            # + the next (lower) layer's FFN output-dropout backward, fused
            dv2_next, kw = self._ffn_out_dropout(order, j + 1, Gv, BT, fseed)
            K.ln_bwd(dx1, L_["h_in"], Pm[p + "layer_norm.weight"], L_["m1"], L_["r1"], dhin, resid=dhmid,
                     dgamma=Gv[p + "layer_norm.weight"], dbeta=Gv[p + "layer_norm.bias"], gate_dp=gdp,
                     gate_w=Pm[at + "gru_rel_pos_linear.weight"] if gdp is not None else None, **kw)
            del dx1, dhmid, gdp
            L_.clear()
            dh = dhin
            if defer:
                K.reduce_defer(False)
                side = self._bwd_side_stream()
                side.wait_stream(main)
                K.reduce_flush(side)
            if on_layer is not None:
                on_layer(li)
        tape.layers = []
        return dh

    def _front_backward(self, tape, Gv, W, dh, diag, front):
        """The rel-pos bias, positional conv, feature projection and conv stack backward
        (encoder_backward, after the transformer layers)."""
        a = self.arch
        cdt = self.cdt
        dev = self.dev
        B, T = tape.B, tape.T
        H, nh = a.hidden, a.heads
        BT = B * T
        Pm = W.m
        Ps = W.s
        fseed = tape.fseed
        php = a.hidden_dropout
        main = torch.cuda.current_stream(dev)
        main.wait_stream(self._bwd_side_stream())
        K.rel_bias_bwd(diag, *self.bucket_runs(T), Gv["encoder.layers.0.attention.rel_attn_embed.weight"], nh, T)
        front("rel")
        # positional conv block: h0 = drop(h + gelu(conv(hpad) + b))
        pk, G = a.pos_kernel, a.pos_groups
        cpg = H // G
        cs = int(math.log2(cpg))
        ds = torch.empty(BT, H, device=dev, dtype=F32)
        K.dropout_cast(dh, ds, php, R.site_seed(fseed, R.SITE_POS))
        del dh
        dypad = torch.empty(B, T + pk, H, device=dev, dtype=cdt)
        K.gelu_bwd_pad(ds, tape.pos_pre, dypad, B, T, H, pk // 2 - 1, pk - pk // 2 + 1)
        # bias + weight gradients (wgrad over (b, t) -> dWf [G][cpg][pk*cpg], weight-norm
        # backward) on the side stream, beside the dgrad chain down the front end
        with self._wgrad_stream(main, dypad, tape.hpad):
            K.colsum(dypad, Gv["encoder.pos_conv_embed.conv.bias"])
            S = _divisor_at_most(B, 8)
            off = (pk // 2 - 1) * H
            A_op = K.Operand(dypad, False, H, offset=off, seg_stride=(T + pk) * H, z1=cpg)
            B_op = K.Operand(tape.hpad, False, H, chunk_shift=cs, ld_chunk=H, seg_stride=(T + pk) * H, z1=cpg)
            if cdt == torch.bfloat16 and cpg == 64 and B % 2 == 0:
                # the bf16 pos-conv wgrad kernel of posconv.hip (64-channel groups): two halves of
                # the utterances, each stored whole into its slab, summed in slab order
                dWf = torch.empty(G, cpg, pk * cpg, device=dev, dtype=F32)
                slab = torch.empty(2, G, cpg, pk * cpg, device=dev, dtype=F32)
                K.gemm(A_op, B_op, slab, cpg, pk * cpg, T, ldc=pk * cpg, nseg=B // 2, splits=2, batch=G,
                       c_z1=cpg * pk * cpg, c_split=dWf.numel())
                K.splitk_reduce(dWf, slab, 2, accumulate=False)
                del slab
            elif S <= 2 or (cdt == torch.bfloat16 and cpg == 64):
                # at most two partial sums per element onto the zeroed dWf: an order-independent,
                # deterministic f32 sum
                dWf = torch.empty(G, cpg, pk * cpg, device=dev, dtype=F32)
                K.zero(dWf)   # (the library's fill: no ATen kernel in the step)
                K.gemm(A_op, B_op, dWf, cpg, pk * cpg, T, ldc=pk * cpg, nseg=B // S, splits=S, batch=G,
                       c_z1=cpg * pk * cpg, flags=_lib.EPI_ATOMIC)
            else:
                dWf = torch.empty(G, cpg, pk * cpg, device=dev, dtype=F32)
                # other shapes (generic kernels): split slabs added in split order
                slab = torch.empty(S, G, cpg, pk * cpg, device=dev, dtype=F32)
                K.gemm(A_op, B_op, slab, cpg, pk * cpg, T, ldc=pk * cpg, nseg=B // S, splits=S, batch=G,
                       c_z1=cpg * pk * cpg, c_split=dWf.numel())
                K.splitk_reduce(dWf, slab, S, accumulate=False)
                del slab
            pre = "encoder.pos_conv_embed.conv.parametrizations.weight."
            wn_scratch = torch.empty(pk, device=dev, dtype=F32)
            K.weight_norm_bwd(dWf, Pm[pre + "original0"], Pm[pre + "original1"], W.wn_norms, Gv[pre + "original0"],
                              Gv[pre + "original1"], wn_scratch, H, cpg, pk)
            del dWf
            front("posconv")
        # dgrad: ds += conv_transpose(dpre) (flipped taps, dypad has pk/2-1 leading zero rows)
        K.gemm(K.Operand(dypad, True, H, chunk_shift=cs, ld_chunk=H, z1=(T + pk) * H, z2=cpg),
               K.Operand(W.wd, True, pk * cpg, z2=cpg * pk * cpg), ds, T, cpg, pk * cpg, ldc=H, batch=B * G, zdiv=G,
               c_z1=T * H, c_z2=cpg, flags=_lib.EPI_ACCUM)
        del dypad
        # SpecAugment + feature-projection dropout backward
        dproj = torch.empty(BT, H, device=dev, dtype=cdt)
        K.specaug_bwd(ds, tape.mask, Gv.get("masked_spec_embed"), dproj, B, T, H, a.feat_proj_dropout,
                      R.site_seed(fseed, R.SITE_FEAT_PROJ))
        del ds
        with self._wgrad_stream(main, dproj, tape.xn):
            K.linear_wgrad(dproj, tape.xn, Gv["feature_projection.projection.weight"])
            K.colsum(dproj, Gv["feature_projection.projection.bias"])
        C = a.conv_dim[-1]
        dxn = torch.empty(BT, C, device=dev, dtype=F32)
        K.linear_dgrad(dproj, Ps["feature_projection.projection.weight"], dxn)
        del dproj
        dfeat = torch.empty(BT, C, device=dev, dtype=cdt)
        K.ln_bwd(dxn, tape.feats, Pm["feature_projection.layer_norm.weight"], tape.fp_mean, tape.fp_rstd, dfeat,
                 dgamma=Gv["feature_projection.layer_norm.weight"], dbeta=Gv["feature_projection.layer_norm.bias"])
        del dxn
        front("proj")
        tape.feats = tape.xn = tape.hpad = tape.pos_pre = None
        # conv stack backward (LN+GELU bwd with col2im of the next layer's dgrad GEMM)
        dy_src, col = dfeat, None
        for i in range(len(a.conv_dim) - 1, 0, -1):
            c = tape.conv[i]
            p = f"feature_extractor.conv_layers.{i}."
            Cc = a.conv_dim[i]
            Cin = a.conv_dim[i - 1]
            Tout, Tin, k, s = c["T"], c["Tin"], c["k"], c["s"]
            dpre = torch.empty(B * Tout, Cc, device=dev, dtype=cdt)
            if col is None:
                K.ln_bwd(dy_src, c["pre"], Pm[p + "layer_norm.weight"], c["mean"], c["rstd"], dpre,
                         beta=Pm[p + "layer_norm.bias"], gelu=True, dgamma=Gv[p + "layer_norm.weight"],
                         dbeta=Gv[p + "layer_norm.bias"])
            else:
                K.ln_bwd(dy_src, c["pre"], Pm[p + "layer_norm.weight"], c["mean"], c["rstd"], dpre,
                         beta=Pm[p + "layer_norm.bias"], gelu=True, dgamma=Gv[p + "layer_norm.weight"],
                         dbeta=Gv[p + "layer_norm.bias"], mode=_lib.DY_COL2IM, col=col)
            del dy_src
            # wgrad -> [co][k*ci] then into the [co][ci][k] grad layout, on the side stream beside
            # the dgrad / LN backward chain down the conv stack
            with self._wgrad_stream(main, dpre, c["x"]):
                A_op = K.Operand(dpre, False, Cc, seg_stride=Tout * Cc)
                B_op = K.Operand(c["x"], False, s * Cin, seg_stride=Tin * Cin)
                if cdt == torch.bfloat16:
                    # split-K over utterances into f32 slabs on the 256x256 kernel + ordered reduce
                    dWr = torch.empty(Cc, k * Cin, device=dev, dtype=F32)
                    S = K.slab_splits_for(((Cc + 255) // 256) * ((k * Cin + 255) // 256), B)
                    K.gemm_slab(A_op, B_op, dWr, Cc, k * Cin, Tout, nseg=B // S, splits=S, accumulate=False)
                else:
                    # f32 parity mode: the same ordered slab reduction on the generic kernels
                    dWr = torch.empty(Cc, k * Cin, device=dev, dtype=F32)
                    tiles = ((Cc + 127) // 128) * ((k * Cin + 127) // 128)
                    S = _divisor_at_most(B, max(1, 512 // tiles))
                    K.gemm_slab(A_op, B_op, dWr, Cc, k * Cin, Tout, nseg=B // S, splits=S, accumulate=False)
                K.swap12(dWr, Gv[p + "conv.weight"], Cc, k, Cin, accumulate=True)
                del dWr
                front(f"conv{i}")
            # dgrad -> G [B*Tout, k*Cin] (col2im folded into the next LN backward)
            Gd = torch.empty(B * Tout, k * Cin, device=dev, dtype=cdt)
            K.gemm(K.Operand(dpre, True, Cc), K.Operand(W.conv_r[i - 1], False, k * Cin), Gd, B * Tout, k * Cin, Cc,
                   ldc=k * Cin)
            del dpre
            tape.conv[i] = None
            dy_src, col = Gd, (k, s, Tout, Tin)
        c0 = tape.conv[0]
        p = "feature_extractor.conv_layers.0."
        K.conv0_bwd(tape.wav, Pm[p + "conv.weight"], Pm[p + "layer_norm.weight"], Pm[p + "layer_norm.bias"],
                    c0["mean"], c0["rstd"], dy_src, Gv[p + "conv.weight"], Gv[p + "layer_norm.weight"],
                    Gv[p + "layer_norm.bias"], c0["T"], a.conv_kernel[0], a.conv_stride[0], col[:3])
        front("conv0")
        tape.conv = []
        main.wait_stream(self._bwd_side_stream())  # every gradient written before clip / AdamW

    def grad_flat_for(self, Gv):
        return self.grad

    # ------------------------------------------------------------------ heads
    def _linear(self, x, w, b, out_dim):
        y = torch.empty(x.shape[0], out_dim, device=self.dev, dtype=F32)
        K.linear_fwd_small(x, w, y, bias=b)
        return y

    def _bn(self, x, P, name, bn_key, train, relu):
        C = x.shape[1]
        y = torch.empty_like(x)
        sm = torch.empty(C, device=self.dev, dtype=F32)
        si = torch.empty(C, device=self.dev, dtype=F32)
        rm, rv, nbt = self.bn[bn_key]
        if train and self.sync_bn is not None:
            # SyncBatchNorm: batch statistics over every rank's rows (one small all-reduce); the
            # rank's row count rides along, so ranks with uneven batches still normalise over the
            # true global count (one host read of it per BN layer: SyncBN is the opt-in parity mode)
            sums = torch.empty(2 * C + 1, device=self.dev, dtype=torch.float64)
            K.bn_stats(x, sums[:2 * C])
            sums[2 * C] = float(x.shape[0])
            self.sync_bn.all_reduce(sums)
            n = int(round(float(sums[2 * C])))
            K.bn_fwd_global(x, P[name + ".weight"], P[name + ".bias"], y, rm, rv, sm, si, sums[:2 * C], n, relu)
            if train:
                self._bn_count[bn_key] += 1
            return y, (x, y, sm, si, n)
        else:
            K.bn_fwd(x, P[name + ".weight"], P[name + ".bias"], y, rm, rv, sm, si, train, relu)
        if train:
            self._bn_count[bn_key] += 1
        return y, (x, y, sm, si)

    def projector_forward(self, emb, P, net, train):
        z0 = self._linear(emb, P["layers.0.weight"], P["layers.0.bias"], P["layers.0.weight"].shape[0])
        z1, c1 = self._bn(z0, P, "layers.1", f"{net}.layers.1", train, True)
        z3 = self._linear(z1, P["layers.3.weight"], P["layers.3.bias"], P["layers.3.weight"].shape[0])
        z4, c4 = self._bn(z3, P, "layers.4", f"{net}.layers.4", train, False)
        return z4, dict(emb=emb, z1=z1, c1=c1, c4=c4)

    def predictor_forward(self, x, P, train):
        net = "online_predictor"
        q0 = self._linear(x, P["layers.0.weight"], P["layers.0.bias"], P["layers.0.weight"].shape[0])
        q1, c1 = self._bn(q0, P, "layers.1", f"{net}.layers.1", train, True)
        q3 = self._linear(q1, P["layers.3.weight"], P["layers.3.bias"], P["layers.3.weight"].shape[0])
        q4, c4 = self._bn(q3, P, "layers.4", f"{net}.layers.4", train, True)
        q6 = self._linear(q4, P["layers.6.weight"], P["layers.6.bias"], P["layers.6.weight"].shape[0])
        return q6, dict(x=x, q1=q1, c1=c1, q4=q4, c4=c4)

    def _lin_bwd(self, dy, x, w, Gw, Gb):
        K.linear_wgrad(dy, x, Gw)
        K.colsum(dy, Gb)
        dx = torch.empty(dy.shape[0], w.shape[1], device=self.dev, dtype=F32)
        K.linear_dgrad_small(dy, w, dx)
        return dx

    def _bn_bwd(self, dy, cache, P, G, name, relu):
        x, y, sm, si = cache[:4]
        dx = torch.empty_like(x)
        if self.sync_bn is not None:
            C = x.shape[1]
            loc = torch.empty(2 * C, device=self.dev, dtype=F32)
            K.bn_bwd_sums(dy, x, y, sm, si, loc, relu)
            glob = loc.clone()
            self.sync_bn.all_reduce(glob)
            K.bn_bwd_global(dy, x, y, P[name + ".weight"], sm, si, loc, glob, cache[4], dx,
                            G[name + ".weight"], G[name + ".bias"], relu)
        else:
            K.bn_bwd(dy, x, y, P[name + ".weight"], sm, si, dx, G[name + ".weight"], G[name + ".bias"], relu)
        return dx

    def predictor_backward(self, dpred, cache, P, G):
        dq4 = self._lin_bwd(dpred, cache["q4"], P["layers.6.weight"], G["layers.6.weight"], G["layers.6.bias"])
        dq3 = self._bn_bwd(dq4, cache["c4"], P, G, "layers.4", True)
        dq1 = self._lin_bwd(dq3, cache["q1"], P["layers.3.weight"], G["layers.3.weight"], G["layers.3.bias"])
        dq0 = self._bn_bwd(dq1, cache["c1"], P, G, "layers.1", True)
        return self._lin_bwd(dq0, cache["x"], P["layers.0.weight"], G["layers.0.weight"], G["layers.0.bias"])

    def projector_backward(self, dz4, cache, P, G):
        dz3 = self._bn_bwd(dz4, cache["c4"], P, G, "layers.4", False)
        dz1 = self._lin_bwd(dz3, cache["z1"], P["layers.3.weight"], G["layers.3.weight"], G["layers.3.bias"])
        dz0 = self._bn_bwd(dz1, cache["c1"], P, G, "layers.1", True)
        return self._lin_bwd(dz0, cache["emb"], P["layers.0.weight"], G["layers.0.weight"], G["layers.0.bias"])

    # ------------------------------------------------------------------ public API
    def weights(self, which: str) -> EncoderWeights:
        """Encoder weight views (+ the derived conv / pos-conv GEMM layouts, computed on the
        current stream). Inside forward() the caller has waited for the front-end segment."""
        if which == "online":
            W = EncoderWeights(self, self.online, self.online_sh, self.online.numel() if self.wsplit else 0,
                               lo8=self.online_lo8)
            W.m_flat, W.s_flat = self.online, (self.online_sh if self.online_sh is not None else self.online)
            W.net = "online"
        else:
            W = EncoderWeights(self, self.target, self.target_sh, self.target.numel() if self.wsplit else 0,
                               lo8=self.target_lo8)
            W.m_flat, W.s_flat = self.target, (self.target_sh if self.target_sh is not None else self.target)
            W.net = "target"
        return W

    def _bwd_side_stream(self) -> torch.cuda.Stream:
        if getattr(self, "_bwd_side", None) is None:
            self._bwd_side = torch.cuda.Stream(self.dev)
        return self._bwd_side

    @contextlib.contextmanager
    def _wgrad_stream(self, main: torch.cuda.Stream, *used: torch.Tensor):
        """Enqueue the enclosed weight-gradient GEMMs on the backward side stream, after all work
        issued so far on `main` (their inputs); `used` tensors are kept alive for that stream.
        The wgrads fill the CUs the dX chain's partial GEMM waves and small kernels leave idle."""
        if _SERIAL_TARGET:
            yield
            return
        side = self._bwd_side_stream()
        side.wait_stream(main)
        for t in used:
            t.record_stream(side)
        with torch.cuda.stream(side):
            yield

    def _mask_stream(self, view_stream: torch.cuda.Stream) -> torch.cuda.Stream:
        """One dropout-mask stream per view stream (the two views' forwards run concurrently)."""
        if getattr(self, "_mask_streams", None) is None:
            self._mask_streams = {}
        key = view_stream.cuda_stream
        if key not in self._mask_streams:
            self._mask_streams[key] = torch.cuda.Stream(self.dev)
        return self._mask_streams[key]

    def _side_stream(self) -> torch.cuda.Stream:
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.dev)
        return self._side

    def stochastic_inputs(self, step_seed: int, B: int, T: int, train: bool, rank: int = 0):
        """LayerDrop decisions for both branches from a rank-SHARED stream (every replica skips
        the same layers, so skipped layers carry zero gradient everywhere and are not sent), and
        the SpecAugment mask SEEDS of both views, rank-DISTINCT (each rank masks its own utterances,
        as dropout does through the rank in forward_seed): the masks themselves are drawn on the
        device by nrse_specaug_mask inside the forward (spec_masks() reads them back for replays)."""
        a = self.arch
        if not train:
            return (None, None), (None, None)
        g = np.random.default_rng([step_seed, 7])
        skips = (layerdrop_decisions(g, a.layers, a.layerdrop), layerdrop_decisions(g, a.layers, a.layerdrop))
        masks = tuple(R.site_seed(R.forward_seed(step_seed, v, rank), R.SITE_SPEC) for v in (0, 1))
        return skips, masks

    def spec_masks(self, seeds, B: int, T: int):
        """The [B, T] bool SpecAugment masks the forward draws from `seeds` (host copies, for the
        oracle replay and tests; a host sync)."""
        a = self.arch
        out = []
        for s in seeds:
            m = torch.empty(B, T, device=self.dev, dtype=torch.uint8)
            K.specaug_mask(m, a.mask_time_prob, a.mask_time_length, a.mask_time_min_masks, int(s))
            out.append(m.cpu().numpy().astype(bool))
        return tuple(out)

    def forward(self, clean: torch.Tensor, noisy: torch.Tensor, *, train: bool, step_seed: int = 0, rank: int = 0,
                need_grad: bool = False, skips=None, masks=None):
        """BYOLSpeechModel.forward -> (online_pred, target_proj, ctx for backward)."""
        B, L = clean.shape
        T = self.arch.frames(L)
        if skips is None or masks is None:
            s2, m2 = self.stochastic_inputs(step_seed, B, T, train, rank)
            skips = skips if skips is not None else s2
            masks = masks if masks is not None else m2
        # The target view (no tape, no grad) runs on a side stream concurrently with the online
        # view: the two encoders are independent until the loss, and each one's small kernels and
        # GEMM tail waves leave CUs idle that the other fills.
        main = torch.cuda.current_stream(self.dev)
        side = main if _SERIAL_TARGET else self._side_stream()
        side.wait_stream(main)
        noisy.record_stream(side)
        with torch.cuda.stream(side):
            self._param_wait(0)
            Wt = self.weights("target")
            temb, _, ex1 = self.encoder_forward(Wt, noisy, train=train, fseed=R.forward_seed(step_seed, 1, rank),
                                                skip=skips[1], mask_np=masks[1], need_grad=False)
            Ptp = self.group_views(self.target, "projector")
            tproj, _ = self.projector_forward(temb, Ptp, "target_projector", train)
        self._param_wait(0)
        Wo = self.weights("online")
        emb, tape, ex0 = self.encoder_forward(Wo, clean, train=train, fseed=R.forward_seed(step_seed, 0, rank),
                                              skip=skips[0], mask_np=masks[0], need_grad=need_grad)
        Pon = self.group_views(self.online, "projector")
        Ppr = self.group_views(self.online, "predictor")
        proj, pc = self.projector_forward(emb, Pon, "online_projector", train)
        pred, qc = self.predictor_forward(proj, Ppr, train)
        main.wait_stream(side)
        tproj.record_stream(main)
        self.executed_layers = [ex0, ex1]
        ctx = dict(tape=tape, W=Wo, pc=pc, qc=qc, emb=emb, Pon=Pon, Ppr=Ppr)
        return pred, tproj, ctx

    def layer_range(self, li: int) -> tuple:
        """[start, end) of transformer layer li's parameters in the flat buffers."""
        return PR.layer_range(self.layout, self.arch, li)

    def _grad_groups(self) -> dict:
        """The units of the overlapped gradient all-reduce (params.grad_groups)."""
        if getattr(self, "_groups", None) is None:
            self._groups = PR.grad_groups(self.layout, self.arch)
        return self._groups

    def backward(self, dpred: torch.Tensor, ctx: dict, allreduce=None) -> None:
        """Accumulate all online-parameter gradients into self.grad from d(loss)/d(pred).
        With a GradAllReduce, every unit of _grad_groups() is all-reduced as soon as backward
        has finished writing it, so the exchange overlaps the rest of backward: the heads right
        after their backward (before the encoder's), each transformer layer when its backward
        (main-stream LN / bias / gate gradients and side-stream weight gradients) is done, the
        final LN with the top layer, layer 0 without its rel_attn_embed row (sent after the
        rel-pos bias backward), then the front end group by group as its weight gradients land
        (pos-conv, feature projection, conv 6 .. 1, conv 0): only conv 0's 5k parameters and
        the exchanges still in flight remain after the last backward kernel. Layers LayerDrop
        skipped hold zero gradient on every rank (rank-shared decisions) and are not sent."""
        Gp = self.group_views(self.grad, "predictor")
        Gj = self.group_views(self.grad, "projector")
        Ge = self.group_views(self.grad, "encoder")
        on = allreduce is not None and allreduce.active()
        main = torch.cuda.current_stream(self.dev)
        groups = self._grad_groups() if on else None

        def send(key):
            # the unit's producers ran on main and/or the backward side stream: enqueue the
            # exchange on the side stream behind both
            side = main if _SERIAL_TARGET else self._bwd_side_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                for s, e in groups[key]:
                    allreduce.issue(self.grad[s:e])

        if on:
            allreduce.start()
        dproj = self.predictor_backward(dpred, ctx["qc"], ctx["Ppr"], Gp)
        demb = self.projector_backward(dproj, ctx["pc"], ctx["Pon"], Gj)
        if on:
            send("heads")
        top = max((L_["li"] for L_ in ctx["tape"].layers), default=None)

        def on_layer(li):
            send(("layer", li))
            if li == top:
                send("final")   # written by the first kernel of the encoder backward
        self.encoder_backward(ctx["tape"], demb, Ge, ctx["W"], on_layer=on_layer if on else None,
                              on_front=send if on else None)
        if on:
            if top is None:
                send("final")
            if self.ar_timing:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record(main)
            allreduce.finish()
            if self.ar_timing:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record(main)
                self.ar_events.append((ev0, ev1))

    def optimizer_step(self, lr: float, grad_scale: float = 1.0) -> None:
        """clip_grad_norm_(1.0) + AdamW + target EMA (train_byol.py:67-71), no host sync.

        With cfg.overlap_optimizer the HBM-bound AdamW + EMA (~3 ms at B = 32) leave the main
        stream: after the global gradient norm (which every segment's clip coefficient needs), a
        dedicated stream updates the parameters segment by segment in forward order and records
        an event per segment; the next step's forward waits per layer, so the update streams
        underneath the MFMA-bound GEMMs of the next step's first layers instead of running alone.
        Per element the arithmetic is identical, so the parameters are bit-identical to the
        serial order."""
        c = self.cfg
        self.step_count += 1
        self.sync_optimizer()  # the previous step's update has read sumsq_buf
        K.zero(self.sumsq_buf)
        K.sumsq(self.grad, self.sumsq_buf)
        kw = dict(lr=lr, beta1=c.betas[0], beta2=c.betas[1], eps=c.eps, weight_decay=c.weight_decay,
                  step=self.step_count, max_norm=c.max_norm, sumsq_buf=self.sumsq_buf, grad_scale=grad_scale,
                  lo8_exp=self.lo8_exp, zero_grad=c.fused_zero_grad,
                  sat=self.sat_buf[SAT_WEIGHTS:SAT_WEIGHTS + 1] if self.online_lo8 is not None else None)
        if self.online_lo8 is not None:
            self._lo8_ranges()
            kw["sat_ranges"] = self._lo8_rng_dev
        self._grad_zeroed = c.fused_zero_grad
        ne = self.layout.ema_numel
        o8, t8 = self.online_lo8, self.target_lo8
        if not c.overlap_optimizer:
            if _FUSED_EMA:
                K.adamw(self.online, self.grad, self.m, self.v, self.online_sh, shadow_lo=self.online_lo,
                        ema_t=self.target, ema_shadow=self.target_sh, ema_shadow_lo=self.target_lo,
                        ema_decay=c.ema_decay, shadow_lo8=o8, ema_shadow_lo8=t8, **kw)
            else:
                K.adamw(self.online, self.grad, self.m, self.v, self.online_sh, shadow_lo=self.online_lo,
                        shadow_lo8=o8, **kw)
                K.ema(self.target, self.online[:ne], self.target_sh, c.ema_decay, shadow_lo=self.target_lo)
                if t8 is not None:
                    K.split_lo8(self.target, t8, self.lo8_exp)   # (the two-launch A/B form: uncounted)
            self._opt_events = self._opt_done = None
            return
        main = torch.cuda.current_stream(self.dev)
        if self._opt_stream is None:
            self._opt_stream = torch.cuda.Stream(self.dev)
        st = self._opt_stream
        st.wait_stream(main)
        events = []
        sh, tsh = self.online_sh, self.target_sh
        with torch.cuda.stream(st):
            for si, (s, e) in enumerate(self._segments):
                # fp8 form: the encoder layers' GEMMs read the fp8 correction planes, never the bf16
                # lo plane, so the pure layer segments (1 .. L-1) skip its writes (2 B per weight
                # for each network)
                layer_only = o8 is not None and 1 <= si < len(self._segments) - 1
                if layer_only:
                    self._lo_stale = {"online": True, "target": True}
                slo = None if layer_only else self.online_lo
                tlo = None if layer_only else self.target_lo
                if e > s:
                    te = min(e, ne)
                    fuse = _FUSED_EMA and te > s
                    K.adamw(self.online[s:e], self.grad[s:e], self.m[s:e], self.v[s:e],
                            sh[s:e] if sh is not None else None, shadow_lo=slo[s:e] if slo is not None else None,
                            ema_t=self.target[s:te] if fuse else None,
                            ema_shadow=tsh[s:te] if fuse and tsh is not None else None,
                            ema_shadow_lo=tlo[s:te] if fuse and tlo is not None else None,
                            ema_decay=c.ema_decay, shadow_lo8=o8[s:e] if o8 is not None else None,
                            ema_shadow_lo8=t8[s:te] if fuse and t8 is not None else None, sat_offset=s, **kw)
                    if te > s and not fuse:
                        K.ema(self.target[s:te], self.online[s:te], tsh[s:te] if tsh is not None else None,
                              c.ema_decay, shadow_lo=tlo[s:te] if tlo is not None else None)
                        if t8 is not None:
                            K.split_lo8(self.target[s:te], t8[s:te], self.lo8_exp)
                ev = torch.cuda.Event()
                ev.record(st)
                events.append(ev)
        self._opt_events = events
        self._opt_done = events[-1]

    def grad_norm(self, world_size: int = 1) -> float:
        """Pre-clip global gradient norm of the last step (host sync)."""
        return float(self.sumsq_buf.sqrt()) / world_size

    def train_step(self, clean: torch.Tensor, noisy: torch.Tensor, *, lr: float, step_seed: int, rank: int = 0,
                   allreduce=None, world_size: int = 1, loss_out: torch.Tensor | None = None) -> torch.Tensor:
        """One iteration of train_one_epoch (train_byol.py:47-77): forward, loss, backward,
        clip, AdamW, EMA. Returns the device-resident loss (no sync): loss_buf, or loss_out (a
        one-element f32 device view, e.g. a slot of the epoch's loss array) when given, so a loop
        that keeps every step's loss needs no copy of loss_buf per step."""
        B = clean.shape[0]
        K.zero(self.health_buf)   # rows: clean, noisy, online_pred, target_proj (nrse_amd/health.py)
        K.health(clean, self.health_buf[0])
        K.health(noisy, self.health_buf[1])
        pred, tproj, ctx = self.forward(clean, noisy, train=True, step_seed=step_seed, rank=rank, need_grad=True)
        K.health(pred, self.health_buf[2])
        K.health(tproj, self.health_buf[3])
        loss = self.loss_buf if loss_out is None else loss_out
        assert loss.dtype == F32 and loss.numel() == 1 and loss.is_contiguous() and loss.device == self.loss_buf.device
        K.zero(loss)
        dpred = torch.empty_like(pred)
        K.byol_loss(pred, tproj, loss, dpred, self.loss_stats)
        self.sync_optimizer()  # the last update has read (and with fused_zero_grad zeroed) the gradient
        if not self._grad_zeroed:
            K.zero(self.grad)
        self._grad_zeroed = False
        self.backward(dpred, ctx, allreduce=allreduce)
        self.optimizer_step(lr, grad_scale=1.0 / world_size)
        return loss

    def eval_forward(self, clean, noisy):
        self.sync_optimizer()
        with torch.no_grad():
            pred, tproj, _ = self.forward(clean, noisy, train=False, need_grad=False)
        loss = torch.zeros(1, device=self.dev, dtype=F32)
        K.byol_loss(pred, tproj, loss)
        return pred, tproj, loss

    def embed(self, wav: torch.Tensor, which: str = "online") -> torch.Tensor:
        self.sync_optimizer()
        emb, _, _ = self.encoder_forward(self.weights(which), wav, train=False)
        return emb
