"""Thin typed wrappers over the C-ABI (include/nrse_hip.h) taking torch device tensors.

PyTorch is used only for device memory and the current HIP stream; every arithmetic op here
is a libnrse_hip.so kernel. Wrappers validate shapes on the host before launching.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import (AdamWParams, AttnBwdParams, AttnFwdParams, Conv0Params, GemmOperand, GemmParams, LnBwdParams,
                   LnFwdParams)

_DT = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16, torch.float8_e4m3fn: _lib.FP8}
FP8 = torch.float8_e4m3fn  # NRSE_FP8: OCP e4m3fn, the split-weight mode's correction operands
CORR = (FP8,)              # the correction-plane dtypes (ABI 8-10's MXFP6 retired in ABI 11)


def dtype_code(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise _lib.NrseError(f"unsupported dtype {t.dtype}") from None


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t: torch.Tensor | None, offset_elems: int = 0):
    if t is None:
        return None
    if not t.is_cuda:
        raise _lib.NrseError("libnrse_hip ops take device tensors")
    return t.data_ptr() + offset_elems * t.element_size()


def _call(name, *args):
    _lib.check(getattr(_lib.lib(), name)(*args), name)


# Deterministic reductions (default): the per-workgroup column sums of the gradient reductions
# are written to a workspace of partial rows and added in a fixed order (nrse_rows_reduce)
# instead of f32 atomics, so a step's gradients are bit-identical run to run.
# NRSE_ATOMIC_REDUCTIONS=1 (timing comparisons only) switches ONLY the reductions that take a
# workspace back to f32 atomics: the GEMM COLSUM bias gradients, colsum / dropout_cast_colsum,
# the LayerNorm dgamma / dbeta (and fused dropout column sums), ln_mean, the attention rel-pos
# diagonals, the gate-parameter and conv0 reductions, the SpecAugment embedding, the BYOL loss and
# the gradient sum of squares. The split-K weight gradients keep their f32 slabs + ordered
# nrse_splitk_reduce under both settings (linear_fwd_small, linear_dgrad_small, the linear_wgrad
# fallback, the f32 conv / pos-conv weight gradients): an A/B with the flag measures the
# partial-row reductions only.
DETERMINISTIC = os.environ.get("NRSE_ATOMIC_REDUCTIONS", "0") != "1"


# ABI 9 deferred reductions (nrse_reduce_defer / nrse_reduce_flush): while on, the workspaces the
# queued reductions read are kept here until reduce_flush hands them to the flushing stream
_DEFER_KEEP = None


def workspace(nfloats: int) -> torch.Tensor:
    """f32 scratch on the current device and stream (the caching allocator keeps it stream-ordered)."""
    t = torch.empty(max(int(nfloats), 4), device="cuda", dtype=torch.float32)
    if _DEFER_KEEP is not None:
        _DEFER_KEEP.append(t)
    return t


def reduce_defer(on: bool) -> None:
    """Queue (on) the ordered gradient reductions that the following calls end with, instead of
    launching them on the current stream (nrse_reduce_defer, ABI 9); reduce_flush runs the queue.
    Their workspaces are held until then."""
    global _DEFER_KEEP
    _lib.lib().nrse_reduce_defer(1 if on else 0)
    if on and _DEFER_KEEP is None:
        _DEFER_KEEP = []


def reduce_discard() -> None:
    """Drop the queued reductions unrun and turn deferral off (nrse_reduce_discard, ABI 10): the
    error path of a backward that raised mid-layer, whose queued jobs' workspaces are released."""
    global _DEFER_KEEP
    _call("nrse_reduce_discard")
    _DEFER_KEEP = None


def reduce_pending() -> int:
    return int(_lib.lib().nrse_reduce_pending())


def _ws_floats(fn: str, p) -> int:
    """A *_workspace query of a params struct; a negative answer is the ABI 10 refusal."""
    n = int(getattr(_lib.lib(), fn)(ctypes.byref(p)))
    if n < 0:
        _lib.check(n, fn)
    return n


def reduce_flush(stream: torch.cuda.Stream | None = None) -> None:
    """Run the queued reductions on `stream` (default: the current one), batched; the queued
    workspaces are recorded on that stream, so the allocator reuses them only after its work."""
    global _DEFER_KEEP
    st = stream if stream is not None else torch.cuda.current_stream()
    for t in _DEFER_KEEP or ():
        t.record_stream(st)
    _call("nrse_reduce_flush", ctypes.c_void_p(st.cuda_stream))
    on = _lib.lib().nrse_reduce_defer(0)
    _lib.lib().nrse_reduce_defer(on)
    _DEFER_KEEP = [] if on else None


def splitk_reduce(out: torch.Tensor, slab: torch.Tensor, S: int, accumulate: bool) -> None:
    """out (+)= sum_s slab[s] in split order (nrse_splitk_reduce; out contiguous f32)."""
    assert out.is_contiguous() and slab.numel() == S * out.numel()
    _call("nrse_splitk_reduce", ptr(out), ptr(slab), S, out.numel(), 1 if accumulate else 0, stream_ptr())


def rows_reduce(slab: torch.Tensor, S: int, *dsts, batch: int = 1, accumulate: bool = True) -> None:
    """Ordered sum of S partial rows [d0 | d1 | d2] into the destinations (nrse_rows_reduce);
    with batch > 1 the slab is [batch, S, n] and each destination [batch, n_j]."""
    assert 1 <= len(dsts) <= 3
    d = list(dsts) + [None] * (3 - len(dsts))
    n = [0 if t is None else t.numel() // batch for t in d]
    _call("nrse_rows_reduce", ptr(d[0]), n[0], ptr(d[1]), n[1], ptr(d[2]), n[2], ptr(slab), S, batch,
          1 if accumulate else 0, stream_ptr())


@dataclass
class Operand:
    """GEMM operand descriptor (see nrse_gemm_operand in include/nrse_hip.h)."""
    t: torch.Tensor
    kcontig: bool
    ld: int
    offset: int = 0
    chunk_shift: int = 0
    ld_chunk: int = 0
    seg_stride: int = 0
    z1: int = 0
    z2: int = 0

    def c(self) -> GemmOperand:
        return GemmOperand(ptr(self.t, self.offset), dtype_code(self.t), int(self.kcontig), self.chunk_shift,
                           self.ld, self.ld_chunk, self.seg_stride, self.z1, self.z2)


def gemm(A: Operand, B: Operand, C: torch.Tensor, M: int, N: int, K: int, *, ldc: int, c_offset: int = 0,
         nseg: int = 1, splits: int = 1, batch: int = 1, zdiv: int = 1, c_z1: int = 0, c_z2: int = 0,
         c_split: int = 0, alpha: float = 1.0, flags: int = 0, bias: torch.Tensor | None = None,
         bias_z1: int = 0, bias_z2: int = 0,
         aux: torch.Tensor | None = None, ldaux: int = 0, aux_z1: int = 0, aux_z2: int = 0,
         resid: torch.Tensor | None = None, ldr: int = 0, r_z1: int = 0, r_z2: int = 0,
         dropout_p: float = 0.0, seed: int = 0, colsum: torch.Tensor | None = None,
         a8: Operand | None = None, b8: Operand | None = None, nseg8: int = 0, b8_exp: int = 0,
         c8: torch.Tensor | None = None, ldc8: int = 0) -> None:
    """C[m,n] = epilogue(alpha * sum_k A(m,k) B(n,k)); see nrse_gemm. a8 / b8 / nseg8 / b8_exp: the
    split-weight mode's fp8 correction segments (+ 2^-b8_exp sum a8 b8); c8: an fp8 copy of a bf16 C."""
    if bias is not None:
        assert bias.dtype == torch.float32
        flags |= _lib.EPI_BIAS
    if colsum is not None:
        assert colsum.dtype == torch.float32
        flags |= _lib.EPI_COLSUM
    if resid is not None:
        flags |= _lib.EPI_RESID
    if dropout_p > 0:
        flags |= _lib.EPI_DROPOUT
    p = GemmParams()
    p.a = A.c()
    p.b = B.c()
    p.M, p.N, p.K, p.nseg, p.splits, p.batch, p.zdiv = M, N, K, nseg, splits, batch, zdiv
    p.alpha = alpha
    p.flags = flags
    p.c = ptr(C, c_offset)
    p.c_dtype = dtype_code(C)
    p.ldc, p.c_z1, p.c_z2, p.c_split = ldc, c_z1, c_z2, c_split
    p.bias = ptr(bias)
    p.bias_z1, p.bias_z2 = bias_z1, bias_z2
    if aux is not None:
        p.aux = ptr(aux)
        p.aux_dtype = dtype_code(aux)
        p.ldaux, p.aux_z1, p.aux_z2 = ldaux, aux_z1, aux_z2
    if resid is not None:
        p.resid = ptr(resid)
        p.resid_dtype = dtype_code(resid)
        p.ldr, p.r_z1, p.r_z2 = ldr, r_z1, r_z2
    p.dropout_p = dropout_p
    p.seed = seed & 0xFFFFFFFF
    p.colsum = ptr(colsum)
    if nseg8:
        assert a8 is not None and b8 is not None and a8.t.dtype == b8.t.dtype and a8.t.dtype in CORR
        p.a8, p.b8, p.nseg8 = a8.c(), b8.c(), nseg8
        p.b8_exp = b8_exp
    if c8 is not None:
        assert c8.dtype in CORR
        p.c8, p.ldc8, p.c8_dtype = ptr(c8), ldc8, dtype_code(c8)
    ws = None
    if colsum is not None and DETERMINISTIC:
        ws = workspace(_ws_floats("nrse_gemm_colsum_workspace", p))
        p.colsum_part = ptr(ws)
    probe = _GEMM_PROBE
    if probe is not None:
        # algorithmic HBM bytes: A and B read once, C written once (read too when accumulated),
        # epilogue operands (bias, aux, residual) once
        ea = A.t.element_size()
        nb = (M * K * nseg * splits + N * K * nseg * splits) * ea * batch + (M + N) * K * nseg8 * batch
        cb = M * N * C.element_size() * batch * (splits if flags & _lib.EPI_ATOMIC else 1)
        nb += cb * (2 if flags & (_lib.EPI_ACCUM | _lib.EPI_ATOMIC) else 1)
        if aux is not None:
            nb += M * N * aux.element_size() * batch
        if resid is not None:
            nb += M * N * resid.element_size() * batch
        _GEMM_PROBE_BYTES.append(nb)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
    _lib.check(_lib.lib().nrse_gemm(ctypes.byref(p), stream_ptr()), "nrse_gemm")
    if probe is not None:
        e1.record()
        # bf16-equivalent work: an fp8 correction segment runs at twice the bf16 MFMA rate, so its
        # FLOPs count 1/2 against the bf16 dense peak
        w8 = 0.5 if nseg8 else 0.0
        tag = "fp8" if nseg8 else ""
        # shape key: M, N, K, batch (+ the correction form), the operand orientation (T: k-contiguous)
        # and the epilogue flags and split count (bench.py --detail)
        orient = ("T" if A.kcontig else "N") + ("T" if B.kcontig else "N") + f"/f{flags}/s{splits}"
        probe.append((2.0 * M * N * K * (nseg * splits + w8 * nseg8) * batch, e0, e1,
                      (M, N, K * nseg * splits, batch, orient) if not nseg8
                      else (M, N, K * nseg, batch, f"{tag}x{nseg8}", orient)))


# When set to a list, every nrse_gemm launch appends (algorithmic FLOPs, start event, end event,
# shape) recorded on the launch stream: bench.py's live roofline measurement.
_GEMM_PROBE = None


def gemm_select(generation: int) -> int:
    """Pin nrse_gemm's bf16 kernel generation (0 auto, 1/2 = 128x128, 3 = 256x256); returns the old one."""
    return int(_lib.lib().nrse_gemm_select(int(generation)))


def gemm_tile_rows(rows: int) -> int:
    """Pin the 256-column kernel's tile rows (0 auto, 256, 224); returns the old setting."""
    return int(_lib.lib().nrse_gemm_tile_rows(int(rows)))


_GEMM_PROBE_BYTES = []


_GEMM_PROBE_OWNER = None


def set_gemm_probe(lst):
    """Record (flops, start event, end event, shape) of every GEMM launch into `lst` while set
    (None: off). Re-enabling with the same list keeps appending (bytes included)."""
    global _GEMM_PROBE, _GEMM_PROBE_OWNER
    _GEMM_PROBE = lst
    if lst is not None and lst is not _GEMM_PROBE_OWNER:
        _GEMM_PROBE_BYTES.clear()
        _GEMM_PROBE_OWNER = lst


def gemm_probe_bytes():
    return list(_GEMM_PROBE_BYTES)


# ----------------------------------------------------------------------------- linear helpers
def linear_fwd(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, *, bias=None, flags: int = 0, w_lo: int = 0,
               x8: torch.Tensor | None = None, w8: torch.Tensor | None = None, lo8_exp: int = 0,
               out8: torch.Tensor | None = None, **kw) -> None:
    """out[M,N] = x[M,K] @ w[N,K]^T (+ epilogue). x, w share the compute dtype. w_lo != 0: the
    split-weight mode, w's lo plane sits w_lo elements after it and the product is
    x @ (w_hi + w_lo)^T, two K segments of one launch (A read twice, one epilogue). x8, w8 (fp8,
    the split-weight mode's fp8 form): x @ w_hi^T + 2^-lo8_exp x8 @ w8^T, the
    correction segment on the MX-scaled fp8 MFMA (x8 = fp8(x), w8 = fp8((w - w_hi) 2^lo8_exp)).
    out8 (fp8, bf16 out): an fp8 copy of the stored output (the next GEMM's x8)."""
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K and out.shape[-1] >= N
    f8 = {}
    if x8 is not None or w8 is not None:
        assert not w_lo and x8 is not None and w8 is not None
        assert x8.shape == x.shape and x8.stride(0) == x.stride(0) and w8.shape == w.shape and w8.stride(0) == w.stride(0)
        f8 = dict(a8=Operand(x8, True, x8.stride(0)), b8=Operand(w8, True, w8.stride(0)), nseg8=1, b8_exp=lo8_exp)
    if out8 is not None:
        assert out8.shape[0] == M and out8.shape[1] >= N
        f8.update(c8=out8, ldc8=out8.stride(0))
    gemm(Operand(x, True, x.stride(0)), Operand(w, True, w.stride(0), seg_stride=w_lo), out, M, N, K,
         ldc=out.stride(0), nseg=2 if w_lo else 1, bias=bias, flags=flags, **f8, **kw)


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, dx: torch.Tensor, *, flags: int = 0, **kw) -> None:
    """dx[M,K] = dy[M,N] @ w[N,K]."""
    M, N = dy.shape
    K = w.shape[1]
    assert w.shape[0] == N
    gemm(Operand(dy, True, dy.stride(0)), Operand(w, False, w.stride(0)), dx, M, K, N, ldc=dx.stride(0),
         flags=flags, **kw)


def _small_m_splits(M: int, N: int, K: int) -> int:
    """K splits for a GEMM with few output tiles (the [32, *] head layers): one 128x128 tile
    column per N/128, so without a split a 1024-wide layer runs 8 workgroups on 256 CUs."""
    if M > 128 or K < 512:
        return 1
    tiles = (N + 127) // 128
    s = 1
    while s * 2 * tiles <= 256 and K % (s * 2) == 0 and (K // (s * 2)) % 128 == 0:
        s *= 2
    return s


def _slab_ok(out: torch.Tensor, M: int, N: int) -> bool:
    """out can take the slab split-K (contiguous f32 [M, N], nrse_splitk_reduce's layout)."""
    return (out.dtype == torch.float32 and out.is_contiguous() and out.numel() == M * N and (M * N) % 4 == 0
            and out.data_ptr() % 16 == 0)


def linear_fwd_small(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, *, bias=None) -> None:
    """out[M,N] = x @ w^T (+ bias) for small M: split-K into f32 slabs (the bias joins split 0),
    added in split order by nrse_splitk_reduce (deterministic; out is overwritten)."""
    M, K = x.shape
    N = w.shape[0]
    S = _small_m_splits(M, N, K)
    if S == 1 or not _slab_ok(out, M, N):
        linear_fwd(x, w, out, bias=bias)
        return
    ks = K // S
    slab = torch.empty(S, M, N, device=out.device, dtype=torch.float32)
    gemm(Operand(x, True, x.stride(0), seg_stride=ks), Operand(w, True, w.stride(0), seg_stride=ks), slab, M, N, ks,
         ldc=N, splits=S, c_split=M * N, bias=bias)
    _call("nrse_splitk_reduce", ptr(out), ptr(slab), S, M * N, 0, stream_ptr())


def linear_dgrad_small(dy: torch.Tensor, w: torch.Tensor, dx: torch.Tensor) -> None:
    """dx[M,K] = dy[M,N] @ w[N,K] for small M: split over N into f32 slabs, added in split order
    (deterministic; dx is overwritten)."""
    M, N = dy.shape
    K = w.shape[1]
    S = _small_m_splits(M, K, N)
    if S == 1 or not _slab_ok(dx, M, K):
        linear_dgrad(dy, w, dx)
        return
    ns = N // S
    slab = torch.empty(S, M, K, device=dx.device, dtype=torch.float32)
    gemm(Operand(dy, True, dy.stride(0), seg_stride=ns), Operand(w, False, w.stride(0), seg_stride=ns * w.stride(0)),
         slab, M, K, ns, ldc=K, splits=S, c_split=M * K)
    _call("nrse_splitk_reduce", ptr(dx), ptr(slab), S, M * K, 0, stream_ptr())


def _slab_splits(M: int, N: int, K: int) -> int:
    """Split count of the slab wgrad: a divisor S of the token count M with ceil(N/256) *
    ceil(K/256) * S 256x256 tiles filling 70-100 % of one wave on the 256 CUs (0: none fits)."""
    tiles = ((N + 255) // 256) * ((K + 255) // 256)
    cap = _SLAB_MAX_TILES
    best = 0
    for s in range(1, 65):
        if M % s or M // s < 256 or tiles * s > cap:
            continue
        if tiles * s >= 0.7 * cap:
            best = s
    if _SLAB_FORCE256 and best and tiles * best < 128:
        # below 128 tiles nrse_gemm hands the problem to the 128x128 kernel: take the smallest
        # split that keeps it on the 256x256 one
        for s in range(best + 1, 65):
            if M % s == 0 and M // s >= 256 and tiles * s >= 128:
                return s
    return best


# The slab wgrads run on the backward side stream beside the dgrad chain's GEMMs, so they size
# their split-K to half a wave of 256x256 workgroups (fewer, longer K ranges: less slab traffic and
# prologue/epilogue per FLOP) rather than to the whole chip: 128 measured +0.6 % pairs/s vs 256,
# 64 -5 % (NRSE_SLAB_MAX_TILES overrides, for tuning). A split landing below 128 tiles (the QKV
# wgrad's 48 x 2) is raised to the smallest one at or above it, so the problem stays on the 256x256
# kernel instead of falling to the 128x128 one (same-box 522 -> 525 pairs/s; NRSE_SLAB_FORCE256=0
# restores the fall-through).
_SLAB_MAX_TILES = int(os.environ.get("NRSE_SLAB_MAX_TILES", "128"))
_SLAB_FORCE256 = os.environ.get("NRSE_SLAB_FORCE256", "1") == "1"


_SLAB_WGRAD = True


def slab_splits_for(tiles256: int, n_units: int) -> int:
    """Largest divisor S of n_units with tiles256 * S <= the slab tile cap (see _SLAB_MAX_TILES)."""
    best = 1
    for s in range(1, n_units + 1):
        if n_units % s == 0 and tiles256 * s <= _CONV_SLAB_MAX_TILES:
            best = s
    return best


# the conv-stack wgrads keep a full wave (their long token ranges; 128 measured -0.6 %)
_CONV_SLAB_MAX_TILES = int(os.environ.get("NRSE_CONV_SLAB_MAX_TILES", "256"))


def gemm_slab(A: "Operand", B: "Operand", out: torch.Tensor, M: int, N: int, K: int, *, nseg: int, splits: int,
              accumulate: bool) -> None:
    """out[M,N] (+)= sum over `splits` K-ranges of A B^T (each split: nseg segments of K), the
    partials stored as f32 slabs by the 256x256 kernel and summed in split order by one streaming
    nrse_splitk_reduce: the deterministic, atomic-free split-K of linear_wgrad, for any operands."""
    assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == M * N
    slab = torch.empty(splits, M, N, device=out.device, dtype=torch.float32)
    gemm(A, B, slab, M, N, K, ldc=N, nseg=nseg, splits=splits, c_split=M * N)
    _call("nrse_splitk_reduce", ptr(out), ptr(slab), splits, M * N, 1 if accumulate else 0, stream_ptr())


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, *, splits: int = 0) -> None:
    """dw[N,K] += dy[M,N]^T @ x[M,K]  (f32 dw).

    Large bf16 problems (the per-layer Linear wgrads, M = B*T tokens): split-K over S equal token
    ranges on the 256x256 kernel, each split storing its f32 partial to a slab (plain stores,
    c_split), then one streaming nrse_splitk_reduce adds the S slabs into dw in split order
    (deterministic; ~6x cheaper than the same partials as f32 atomics at the chip's ~1.3 TB/s
    atomic rate). Otherwise split-K with f32 atomics on the 128x128 kernel."""
    M, N = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and dw.shape == (N, K) and dw.dtype == torch.float32
    S = _slab_splits(M, N, K) if (_SLAB_WGRAD and splits <= 0 and dy.dtype == torch.bfloat16
                                  and dw.is_contiguous()) else 0
    if S:
        seg = M // S
        slab = torch.empty(S, N, K, device=dw.device, dtype=torch.float32)
        gemm(Operand(dy, False, dy.stride(0), seg_stride=seg * dy.stride(0)),
             Operand(x, False, x.stride(0), seg_stride=seg * x.stride(0)),
             slab, N, K, seg, ldc=K, nseg=1, splits=S, c_split=N * K)
        _call("nrse_splitk_reduce", ptr(dw), ptr(slab), S, N * K, 1, stream_ptr())
        return
    if splits <= 0:
        tiles = ((N + 127) // 128) * ((K + 127) // 128)
        splits = max(1, min(16, 512 // max(tiles, 1)))
    splits = max(1, min(splits, M // 64, 4096))
    # equal token segments (the reduction dim is the outer index of both operands, so any
    # segment length works): prefer a divisor of M to avoid a ragged tail launch
    for s in range(splits, 0, -1):
        if M % s == 0 and (splits <= 2 or s * 2 > splits):
            splits = s
            break
    seg = (M + splits - 1) // splits
    bulk = (M // seg) * seg
    if bulk and bulk // seg > 1 and _slab_ok(dw, N, K):
        # the splits' partials as slabs added in split order (deterministic)
        gemm_slab(Operand(dy, False, dy.stride(0), seg_stride=seg * dy.stride(0)),
                  Operand(x, False, x.stride(0), seg_stride=seg * x.stride(0)),
                  dw, N, K, seg, nseg=1, splits=bulk // seg, accumulate=True)
    elif bulk:
        gemm(Operand(dy, False, dy.stride(0), seg_stride=seg * dy.stride(0)),
             Operand(x, False, x.stride(0), seg_stride=seg * x.stride(0)),
             dw, N, K, seg, ldc=dw.stride(0), nseg=1, splits=bulk // seg, flags=_lib.EPI_ATOMIC)
    if bulk < M:
        gemm(Operand(dy, False, dy.stride(0), offset=bulk * dy.stride(0)),
             Operand(x, False, x.stride(0), offset=bulk * x.stride(0)),
             dw, N, K, M - bulk, ldc=dw.stride(0), flags=_lib.EPI_ATOMIC)


# ----------------------------------------------------------------------------- layernorm
def _out_code(y: torch.Tensor, n: int, split3: bool) -> int:
    """dtype code of a kernel output; split3: y is the [3, n] bf16 planes [hi | lo | hi] of the
    split-weight mode's conv stack (NRSE_BF16X3)."""
    if not split3:
        return dtype_code(y)
    assert y.dtype == torch.bfloat16 and y.is_contiguous() and y.shape[0] == 3 and y.numel() == 3 * n, y.shape
    return _lib.BF16X3


def _sat_ptr(sat):
    """The ABI 10 saturation counter (int32 device tensor, element 0) or None."""
    if sat is None:
        return None
    assert sat.dtype == torch.int32 and sat.is_cuda
    return ptr(sat)


def ln_fwd(x, gamma, beta, y, mean, rstd, eps, gelu=False, relu=False, split3=False, y8=None, y8_exp=None, sat=None):
    """y8 (fp8 [rows, C], bf16 y): also y8 = fp8(y), the split-weight mode's next correction operand;
    with y8_exp (fp8 [2, rows, C]): the two correction planes [fp8((o - bf16 o) 2^y8_exp) | fp8(bf16 o)]
    of the exact output o (the conv stack's form, ABI 7). sat (int32 device tensor): += the number
    of y8 conversions that saturated (ABI 10)."""
    rows, C = x.shape[0] if x.dim() == 2 else x.numel() // x.shape[-1], x.shape[-1]
    if y8 is not None:
        n8 = rows * C * (1 if y8_exp is None else 2)
        assert y8.dtype in CORR and y8.numel() == n8 and y8.is_contiguous()
    p = LnFwdParams(ptr(x), dtype_code(x), ptr(gamma), ptr(beta), ptr(y), _out_code(y, rows * C, split3), ptr(mean),
                    ptr(rstd), rows, C, eps, (_lib.LN_GELU if gelu else 0) | (_lib.LN_RELU if relu else 0), ptr(y8),
                    0 if y8_exp is None else 1, 0 if y8_exp is None else int(y8_exp),
                    dtype_code(y8) if y8 is not None else 0, _sat_ptr(sat))
    _call("nrse_layernorm_fwd", ctypes.byref(p), stream_ptr())


def ln_bwd(dy, x, gamma, mean, rstd, dx, *, beta=None, gelu=False, relu=False, resid=None, dgamma=None, dbeta=None,
           mode=_lib.DY_DIRECT, col=(0, 0, 0, 0), bcast_t=0, dy_scale=1.0, rows=None,
           dv=None, dv_colsum=None, dv_p=0.0, dv_seed=0, gate_dp=None, gate_w=None):
    """LayerNorm backward; with `dv`, also the fused dropout_cast_colsum of dx: dv = dropout(dx)
    (cast to dv's dtype), dv_colsum += column sums of dv. gate_dp / gate_w (encoder form): dy plus
    the gate path's gradient from gate_bwd_dp's (dpa, dpb) and gru_rel_pos_linear.weight."""
    C = x.shape[-1]
    rows = rows if rows is not None else x.numel() // C
    p = LnBwdParams()
    p.dy, p.dy_dtype, p.dy_mode = ptr(dy), dtype_code(dy), mode
    p.col_k, p.col_s, p.col_tout, p.col_tin = col
    p.bcast_t, p.dy_scale = bcast_t, dy_scale
    p.x, p.x_dtype = ptr(x), dtype_code(x)
    p.gamma, p.beta, p.mean, p.rstd = ptr(gamma), ptr(beta), ptr(mean), ptr(rstd)
    p.dx, p.dx_dtype = ptr(dx), dtype_code(dx)
    p.resid = ptr(resid)
    p.dgamma, p.dbeta = ptr(dgamma), ptr(dbeta)
    p.rows, p.C, p.flags = rows, C, (_lib.LN_GELU if gelu else 0) | (_lib.LN_RELU if relu else 0)
    if dv is not None:
        assert dv.numel() == rows * C and (dv_colsum is None or dv_colsum.dtype == torch.float32)
        p.dv, p.dv_dtype, p.dv_colsum = ptr(dv), dtype_code(dv), ptr(dv_colsum)
        p.dv_p, p.dv_seed = dv_p, dv_seed & 0xFFFFFFFF
    if gate_dp is not None:
        assert gate_dp.dtype == torch.float32 and gate_dp.numel() == rows * (C // 64) * 2 and gate_w is not None
        p.gate_dp, p.gate_w = ptr(gate_dp), ptr(gate_w)
    ws = None
    if DETERMINISTIC and (dgamma is not None or (dv is not None and dv_colsum is not None)):
        ws = workspace(_ws_floats("nrse_layernorm_bwd_workspace", p))
        p.part = ptr(ws)
    _call("nrse_layernorm_bwd", ctypes.byref(p), stream_ptr())


def ln_mean_fwd(h, gamma, beta, emb, mean, rstd, batch, T, C, eps):
    ws = workspace(batch * ((T + 31) // 32) * C) if DETERMINISTIC else None
    _call("nrse_ln_mean_fwd", ptr(h), ptr(gamma), ptr(beta), ptr(emb), ptr(mean), ptr(rstd), batch, T, C, eps,
          ptr(ws), stream_ptr())


# ----------------------------------------------------------------------------- attention
def bias_ld(T: int) -> int:
    """Row stride of the [H, T, Tb] relative-position bias table (nrse_bias_ld)."""
    return int(_lib.lib().nrse_bias_ld(T))


def rel_bias_fwd(E, bucket, bias, H, T):
    assert bias.shape[-1] == bias_ld(T)
    _call("nrse_rel_bias_fwd", ptr(E), ptr(bucket), ptr(bias), H, T, E.shape[0], stream_ptr())


def rel_bias_vec(E, bucket, vec, H, T):
    """Toeplitz form of the rel-pos bias: vec [H, 2T-1], vec[h, j-i+T-1] = E[bucket(j-i), h]."""
    assert vec.shape == (H, 2 * T - 1) and vec.is_contiguous()
    _call("nrse_rel_bias_vec", ptr(E), ptr(bucket), ptr(vec), H, T, E.shape[0], stream_ptr())


def rel_bias_bwd(diag, order, offsets, dE, H, T):
    """dE[bucket(d), h] += diag[h, d], gathered per bucket in a fixed order (hostside.bucket_runs)."""
    _call("nrse_rel_bias_bwd", ptr(diag), ptr(order), ptr(offsets), ptr(dE), H, T, offsets.numel() - 1, stream_ptr())


def gate_fwd(x1, W, b, c, gate, batch, T, H):
    _call("nrse_gate_fwd", ptr(x1), dtype_code(x1), ptr(W), ptr(b), ptr(c), ptr(gate), batch, T, H, stream_ptr())


def gate_bwd(x1, W, b, c, dgate, dx1, dW, db, dc, batch, T, H):
    """dx1 += gate-path gradient; dW/db/dc accumulated (one fused kernel)."""
    assert dx1.dtype == torch.float32 and dW.dtype == db.dtype == dc.dtype == torch.float32
    ws = workspace(_lib.lib().nrse_gate_bwd_workspace(H)) if DETERMINISTIC else None
    _call("nrse_gate_bwd", ptr(x1), dtype_code(x1), ptr(W), ptr(b), ptr(c), ptr(dgate), ptr(dx1), ptr(dW), ptr(db),
          ptr(dc), batch, T, H, ptr(ws), stream_ptr())


def gate_bwd_dp(x1, W, b, c, dgate, dp, dW, db, dc, batch, T, H):
    """The gate backward without the dx1 read-modify-write: dp [B*T, H, 2] f32 receives each
    (row, head)'s (dpa, dpb) for the LN backward (ln_bwd(gate_dp=dp, gate_w=W)); dW/db/dc as gate_bwd."""
    assert dp.dtype == torch.float32 and dp.numel() == batch * T * H * 2
    assert dW.dtype == db.dtype == dc.dtype == torch.float32
    ws = workspace(_lib.lib().nrse_gate_bwd_workspace(H)) if DETERMINISTIC else None
    _call("nrse_gate_bwd_dp", ptr(x1), dtype_code(x1), ptr(W), ptr(b), ptr(c), ptr(dgate), ptr(dp), ptr(dW), ptr(db),
          ptr(dc), batch, T, H, ptr(ws), stream_ptr())


def attn_mask_elems(batch, T, H) -> int:
    """u16 words of the forward's dropout keep-bit mask (nrse_attn_fwd_params.drop_mask)."""
    return int(_lib.lib().nrse_attn_mask_elems(batch, T, H))


def attn_dropout_mask(mask, batch, T, H, dropout_p, seed):
    """The probability-dropout keep bits of one attention layer (drop_mask layout), computed ahead
    of attn_fwd(..., drop_mask=mask, mask_in=True) by a pure-VALU kernel (nrse_attn_dropout_mask)."""
    assert mask.dtype == torch.int16 and mask.numel() >= attn_mask_elems(batch, T, H)
    _call("nrse_attn_dropout_mask", ptr(mask), batch, T, H, dropout_p, seed & 0xFFFFFFFF, stream_ptr())


def attn_fwd(qkv, gate, bias, ctx, lse, batch, T, H, dropout_p=0.0, seed=0, bias_vec=None, drop_mask=None,
             mask_in=False, ctx8=None):
    """bias: [H, T, Tb] table (f32 parity path), bias_vec: [H, 2T-1] Toeplitz vector (bf16 path);
    drop_mask (optional, int16 [attn_mask_elems]): the keep bits for the backward, recorded by the
    forward, or (mask_in) read by it (attn_dropout_mask wrote them); ctx8 (fp8, bf16 path): an fp8
    copy of ctx (the split-weight mode's out-projection correction operand)."""
    if drop_mask is not None:
        assert drop_mask.dtype == torch.int16 and drop_mask.numel() >= attn_mask_elems(batch, T, H)
    if ctx8 is not None:
        assert ctx8.dtype in CORR and ctx8.numel() == ctx.numel() and qkv.dtype == torch.bfloat16
    p = AttnFwdParams(ptr(qkv), dtype_code(qkv), ptr(gate), ptr(bias), ptr(ctx), ptr(lse), batch, T, H, 64,
                      0.125, dropout_p, seed & 0xFFFFFFFF, ptr(bias_vec), ptr(drop_mask),
                      1 if (mask_in and drop_mask is not None) else 0, ptr(ctx8),
                      dtype_code(ctx8) if ctx8 is not None else 0)
    _call("nrse_attn_fwd", ctypes.byref(p), stream_ptr())


def attn_bwd(qkv, gate, bias, ctx, dctx, lse, delta, dqkv, dgate, diag, batch, T, H, dropout_p=0.0, seed=0,
             bias_vec=None, drop_mask=None):
    p = AttnBwdParams(ptr(qkv), dtype_code(qkv), ptr(gate), ptr(bias), ptr(ctx), ptr(dctx), ptr(lse), ptr(delta),
                      ptr(dqkv), ptr(dgate), ptr(diag), batch, T, H, 64, 0.125, dropout_p, seed & 0xFFFFFFFF,
                      ptr(bias_vec))
    p.drop_mask = ptr(drop_mask)
    ws = None
    if DETERMINISTIC and diag is not None:
        ws = workspace(_ws_floats("nrse_attn_bwd_workspace", p))
        p.diag_part = ptr(ws)
    _call("nrse_attn_bwd", ctypes.byref(p), stream_ptr())


# ----------------------------------------------------------------------------- conv front end
def conv0_fwd(wav, w, gamma, beta, out, mean, rstd, T0, k, s, eps, split3=False, y8=None, y8_exp=0, sat=None):
    """y8 (fp8 [2, B*T0, C], bf16 out): the exact output's fp8 correction planes (ABI 7); sat: the
    saturation counter of those conversions (ABI 10)."""
    B, L = wav.shape
    C = w.shape[0]
    p = Conv0Params()
    if y8 is not None:
        assert y8.dtype in CORR and y8.numel() == 2 * B * T0 * C and y8.is_contiguous() and not split3
        p.y8, p.y8_exp, p.y8_dtype = ptr(y8), int(y8_exp), dtype_code(y8)
        p.sat_count = _sat_ptr(sat)
    p.wav, p.L, p.w, p.gamma, p.beta = ptr(wav), L, ptr(w), ptr(gamma), ptr(beta)
    p.out, p.out_dtype, p.mean, p.rstd = ptr(out), _out_code(out, B * T0 * C, split3), ptr(mean), ptr(rstd)
    p.batch, p.T0, p.C, p.k, p.s, p.eps = B, T0, C, k, s, eps
    _call("nrse_conv0_fwd", ctypes.byref(p), stream_ptr())


def conv0_bwd(wav, w, gamma, beta, mean, rstd, dy, dw, dgamma, dbeta, T0, k, s, col):
    """dw ([C, k] or [C, 1, k] f32) += the conv0 weight gradient (the kernel accumulates a
    tap-major [k, C] copy, transposed into dw here)."""
    B, L = wav.shape
    C = w.shape[0]
    dwT = torch.empty(k, C, device=wav.device, dtype=torch.float32)
    zero(dwT)   # nrse_zero: no ATen fill kernel in the step
    p = Conv0Params()
    p.wav, p.L, p.w, p.gamma, p.beta = ptr(wav), L, ptr(w), ptr(gamma), ptr(beta)
    p.mean, p.rstd = ptr(mean), ptr(rstd)
    p.dy, p.dy_dtype = ptr(dy), dtype_code(dy)
    if col is None:
        p.dy_mode = _lib.DY_DIRECT
    else:
        p.dy_mode = _lib.DY_COL2IM
        p.col_k, p.col_s, p.col_tout = col
    p.dw, p.dgamma, p.dbeta = ptr(dwT), ptr(dgamma), ptr(dbeta)
    p.batch, p.T0, p.C, p.k, p.s = B, T0, C, k, s
    ws = None
    if DETERMINISTIC:
        ws = workspace(_ws_floats("nrse_conv0_bwd_workspace", p))
        p.part = ptr(ws)
    _call("nrse_conv0_bwd", ctypes.byref(p), stream_ptr())
    swap12(dwT, dw, 1, k, C, accumulate=True)


def _wn_part(v, K):
    """Scratch of the coalesced two-stage per-tap reduction (256 * K doubles) or None."""
    return torch.empty(256 * K, device=v.device, dtype=torch.float64) if K <= 256 and 256 % K == 0 else None


def weight_norm_fwd(g, v, wf, wd, norms, H, cpg, K):
    part = _wn_part(v, K)
    _call("nrse_weight_norm_fwd", ptr(g), ptr(v), ptr(wf), ptr(wd), dtype_code(wf), ptr(norms), H, cpg, K,
          ptr(part), stream_ptr())


def weight_norm_bwd(dWf, g, v, norms, dg, dv, scratch, H, cpg, K):
    part = _wn_part(v, K)
    _call("nrse_weight_norm_bwd", ptr(dWf), ptr(g), ptr(v), ptr(norms), ptr(dg), ptr(dv), ptr(scratch), H, cpg, K,
          ptr(part), stream_ptr())


# ----------------------------------------------------------------------------- elementwise
def specaug_pad(h, mask, embed, dst, batch, T, C, pf, pb):
    _call("nrse_specaug_pad", ptr(h), ptr(mask), ptr(embed), ptr(dst), dtype_code(dst), batch, T, C, pf, pb,
          stream_ptr())


def specaug_mask(mask, mask_prob, mask_length, min_masks, seed):
    """mask [B, T] u8 <- the SpecAugment time masks drawn on the device (nrse_specaug_mask, ABI 10)."""
    assert mask.dtype == torch.uint8 and mask.dim() == 2 and mask.is_contiguous()
    B, T = mask.shape
    _call("nrse_specaug_mask", ptr(mask), B, T, float(mask_prob), int(mask_length), int(min_masks), seed & 0xFFFFFFFF,
          stream_ptr())


def pad_rows(src, dst, batch, T, C, pf, pb):
    _call("nrse_pad_rows", ptr(src), dtype_code(src), ptr(dst), dtype_code(dst), batch, T, C, pf, pb, stream_ptr())


def specaug_bwd(dh, mask, dembed, out, batch, T, C, p, seed):
    ws = None
    if DETERMINISTIC and mask is not None and dembed is not None:
        ws = workspace(min(batch * T, 2048) * C)
    _call("nrse_specaug_bwd", ptr(dh), ptr(mask), ptr(dembed), ptr(out), dtype_code(out), batch, T, C, p,
          seed & 0xFFFFFFFF, ptr(ws), stream_ptr())


def dropout_cast(x, out, p=0.0, seed=0):
    assert x.dtype == torch.float32 and x.numel() == out.numel()
    _call("nrse_dropout_cast", ptr(x), ptr(out), dtype_code(out), x.numel(), p, seed & 0xFFFFFFFF, stream_ptr())


def _colsum_ws(rows: int, C: int):
    return workspace(_lib.lib().nrse_colsum_workspace(rows, C)) if DETERMINISTIC else None


def dropout_cast_colsum(x, out, colsum, p=0.0, seed=0):
    """out = dropout(x) (cast), colsum += column sums of out: one pass."""
    assert x.dtype == torch.float32 and x.numel() == out.numel() and colsum.dtype == torch.float32
    C = x.shape[-1]
    ws = _colsum_ws(x.numel() // C, C)
    _call("nrse_dropout_cast_colsum", ptr(x), ptr(out), dtype_code(out), x.numel() // C, C, p, seed & 0xFFFFFFFF,
          ptr(colsum), ptr(ws), stream_ptr())


def colsum(x, out):
    C = x.shape[-1]
    ws = _colsum_ws(x.numel() // C, C)
    _call("nrse_colsum", ptr(x), dtype_code(x), ptr(out), x.numel() // C, C, ptr(ws), stream_ptr())


def cast(x, y):
    assert x.numel() == y.numel()
    _call("nrse_cast", ptr(x), dtype_code(x), ptr(y), dtype_code(y), x.numel(), stream_ptr())


def swap12(src, dst, d0, d1, d2, accumulate=False):
    _call("nrse_swap12", ptr(src), dtype_code(src), ptr(dst), dtype_code(dst), d0, d1, d2, int(accumulate),
          stream_ptr())


def gelu_bwd_pad(dy, pre, out, batch, T, C, pf, pb):
    _call("nrse_gelu_bwd_pad", ptr(dy), ptr(pre), dtype_code(pre), ptr(out), dtype_code(out), batch, T, C, pf, pb,
          stream_ptr())


# ----------------------------------------------------------------------------- heads / loss / optim
def bn_fwd(x, w, b, y, rm, rv, sm, si, train, relu, momentum=0.1, eps=1e-5):
    rows, C = x.shape
    _call("nrse_bn_fwd", ptr(x), ptr(w), ptr(b), ptr(y), ptr(rm), ptr(rv), ptr(sm), ptr(si), rows, C, momentum, eps,
          int(train), int(relu), stream_ptr())


def bn_bwd(dy, x, y, w, sm, si, dx, dw, db, relu):
    rows, C = x.shape
    _call("nrse_bn_bwd", ptr(dy), ptr(x), ptr(y), ptr(w), ptr(sm), ptr(si), ptr(dx), ptr(dw), ptr(db), rows, C,
          int(relu), stream_ptr())


def bn_stats(x, sums):
    rows, C = x.shape
    _call("nrse_bn_stats", ptr(x), ptr(sums), rows, C, stream_ptr())


def bn_fwd_global(x, w, b, y, rm, rv, sm, si, gsums, nglobal, relu, momentum=0.1, eps=1e-5):
    rows, C = x.shape
    _call("nrse_bn_fwd_global", ptr(x), ptr(w), ptr(b), ptr(y), ptr(rm), ptr(rv), ptr(sm), ptr(si), ptr(gsums),
          int(nglobal), rows, C, momentum, eps, int(relu), stream_ptr())


def bn_bwd_sums(dy, x, y, sm, si, sums, relu):
    rows, C = x.shape
    _call("nrse_bn_bwd_sums", ptr(dy), ptr(x), ptr(y), ptr(sm), ptr(si), ptr(sums), rows, C, int(relu), stream_ptr())


def bn_bwd_global(dy, x, y, w, sm, si, lsums, gsums, nglobal, dx, dw, db, relu):
    rows, C = x.shape
    _call("nrse_bn_bwd_global", ptr(dy), ptr(x), ptr(y), ptr(w), ptr(sm), ptr(si), ptr(lsums), ptr(gsums),
          int(nglobal), ptr(dx), ptr(dw), ptr(db), rows, C, int(relu), stream_ptr())


def byol_loss(p, z, loss, dp=None, stats=None, grad_scale=1.0):
    rows, D = p.shape
    ws = workspace(rows * (3 if stats is not None else 1)) if DETERMINISTIC else None
    _call("nrse_byol_loss", ptr(p), ptr(z), ptr(loss), ptr(dp), ptr(stats), rows, D, grad_scale, ptr(ws),
          stream_ptr())


def sumsq(x, out):
    ws = torch.empty(4096, device=x.device, dtype=torch.float64) if DETERMINISTIC else None
    _call("nrse_sumsq", ptr(x), x.numel(), ptr(out), ptr(ws), stream_ptr())


def adamw(p, g, m, v, shadow, *, lr, beta1, beta2, eps, weight_decay, step, max_norm, sumsq_buf, grad_scale=1.0,
          shadow_lo=None, ema_t=None, ema_shadow=None, ema_shadow_lo=None, ema_decay=0.0, shadow_lo8=None,
          ema_shadow_lo8=None, lo8_exp=0, zero_grad=False, sat=None, sat_ranges=None, sat_offset=0):
    """clip + AdamW; shadow (bf16/f32) gets the updated weights, shadow_lo (bf16, with a bf16
    shadow) the split-weight mode's lo plane bf16(p - shadow). ema_t (f32, numel <= p's): the
    target EMA of the first ema_t.numel() updated weights in the same pass (as ema() after).
    shadow_lo8 / ema_shadow_lo8 (fp8): the fp8 correction planes fp8((w - bf16(w)) 2^lo8_exp);
    zero_grad: g is zeroed by the pass after it is read. sat (int32 device tensor): += the number of
    fp8 corrections that saturated (ABI 10); sat_ranges (int64 device [n, 2], sorted [start, end) flat
    indices, p[i] = flat index sat_offset + i): only saturations inside them count."""
    if ema_t is not None:
        assert ema_t.dtype == torch.float32 and ema_t.numel() <= p.numel()
    for t, n in ((shadow_lo8, p.numel()), (ema_shadow_lo8, ema_t.numel() if ema_t is not None else 0)):
        assert t is None or (t.dtype in CORR and t.numel() == n)
    lo8_dt = dtype_code(shadow_lo8 if shadow_lo8 is not None else ema_shadow_lo8) \
        if (shadow_lo8 is not None or ema_shadow_lo8 is not None) else 0
    prm = AdamWParams(ptr(p), ptr(g), ptr(m), ptr(v), ptr(shadow),
                      dtype_code(shadow) if shadow is not None else 0, p.numel(), lr, beta1, beta2, eps,
                      weight_decay, step, max_norm, ptr(sumsq_buf), grad_scale, ptr(shadow_lo),
                      ptr(ema_t), ptr(ema_shadow), ptr(ema_shadow_lo),
                      dtype_code(ema_shadow) if ema_shadow is not None else 0, ema_decay,
                      ema_t.numel() if ema_t is not None else 0, ptr(shadow_lo8), ptr(ema_shadow_lo8), lo8_exp,
                      1 if zero_grad else 0, lo8_dt, _sat_ptr(sat))
    if sat_ranges is not None:
        assert sat is not None and sat_ranges.dtype == torch.int64 and sat_ranges.is_contiguous()
        prm.sat_ranges, prm.sat_nranges, prm.sat_offset = ptr(sat_ranges), sat_ranges.shape[0], int(sat_offset)
    _call("nrse_adamw", ctypes.byref(prm), stream_ptr())


def ema(t, o, shadow, decay, shadow_lo=None):
    _call("nrse_ema", ptr(t), ptr(o), ptr(shadow), dtype_code(shadow) if shadow is not None else 0, t.numel(), decay,
          ptr(shadow_lo), stream_ptr())


def split_bf16(x, hi, lo):
    """hi = bf16(x), lo = bf16(x - hi) (nrse_split_bf16)."""
    assert x.dtype == torch.float32 and hi.dtype == lo.dtype == torch.bfloat16
    assert hi.numel() == lo.numel() == x.numel()
    _call("nrse_split_bf16", ptr(x), ptr(hi), ptr(lo), x.numel(), stream_ptr())


def split_lo8(x, lo8, lo8_exp=0, sat=None):
    """lo8 = fp8((x - bf16(x)) 2^lo8_exp) (nrse_split_lo8): the fp8 correction plane of x. sat: the
    saturation counter (ABI 10)."""
    assert x.dtype == torch.float32 and lo8.dtype in CORR and lo8.numel() == x.numel()
    _call("nrse_split_lo8", ptr(x), ptr(lo8), int(lo8_exp), x.numel(), _sat_ptr(sat), stream_ptr())


def cast_fp8(x, y8):
    """y8 = fp8(x) (nrse_cast_fp8; x f32 or bf16)."""
    assert y8.dtype in CORR and y8.numel() == x.numel()
    _call("nrse_cast_fp8", ptr(x), dtype_code(x), ptr(y8), x.numel(), stream_ptr())


def zero(t):
    """t[:] = 0 for an f32 tensor (nrse_zero; the step's small accumulators, no torch fill)."""
    assert t.dtype in (torch.float32, torch.float64) and t.is_contiguous()
    _call("nrse_zero", ptr(t), t.numel() * t.element_size() // 4, stream_ptr())


def health(x, stats):
    _call("nrse_health", ptr(x), dtype_code(x), x.numel(), ptr(stats), stream_ptr())


SNR_RAW, SNR_PEAK, SNR_PEAK_ZMUV = 0, 1, 2
SNR_SCRATCH_PER_PAIR = 256  # NRSE_SNR_SCRATCH_PER_PAIR (include/nrse_hip.h)


def snr_mix(clean, noise, noise_len, snr_db, clean_out, noisy_out, status, kscale, mode=SNR_PEAK_ZMUV):
    """Fused on-GPU SNR mix (nrse_snr_mix); mode 0 raw / 1 peak / 2 peak + feature-extractor norm."""
    B, L = clean.shape
    assert noise.dim() == 2 and noise.shape[0] == B and clean.is_contiguous() and noise.stride(1) == 1
    scratch = torch.empty(B * SNR_SCRATCH_PER_PAIR, device=clean.device, dtype=torch.float64)
    _call("nrse_snr_mix", ptr(clean), ptr(noise), ptr(noise_len), noise.stride(0), ptr(snr_db), ptr(clean_out),
          ptr(noisy_out), ptr(status), ptr(kscale), ptr(scratch), B, L, int(mode), stream_ptr())


# ----------------------------------------------------------------------------- emotion head
def asp_fwd(x, h, att, lens, w_out, var_out, pooled):
    """Attentive statistics pooling (src/models/pool.py:25-58); x [B, T, C], h f32 [B, T, C]."""
    B, T, C = x.shape
    assert h.dtype == torch.float32 and lens.dtype == torch.int32
    _call("nrse_asp_fwd", ptr(x), dtype_code(x), ptr(h), ptr(att), ptr(lens), B, T, C, ptr(w_out), ptr(var_out),
          ptr(pooled), stream_ptr())


def asp_bwd(x, h, att, lens, w_in, var_in, pooled, dpooled, dpre, datt):
    B, T, C = x.shape
    _call("nrse_asp_bwd", ptr(x), dtype_code(x), ptr(h), ptr(att), ptr(lens), B, T, C, ptr(w_in), ptr(var_in),
          ptr(pooled), ptr(dpooled), ptr(dpre), dtype_code(dpre), ptr(datt), stream_ptr())


def ccc_loss(pred, target, loss, dpred=None):
    """pred (and dpred) may be a column slice of a wider row-major buffer (row stride >= D)."""
    rows, D = target.shape
    assert pred.shape == (rows, D) and pred.stride(1) == 1 and (dpred is None or dpred.stride(0) == pred.stride(0))
    _call("nrse_ccc_loss", ptr(pred), pred.stride(0), ptr(target), ptr(loss), ptr(dpred), rows, D, stream_ptr())

