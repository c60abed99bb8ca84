"""Thin typed wrappers over the C-ABI (include/nrse_hip.h) taking torch device tensors.

PyTorch is used only for device memory and the current HIP stream; every arithmetic op here
is a libnrse_hip.so kernel. Wrappers validate shapes on the host before launching.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import GemmOperand, GemmParams

_DT = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16}


def dtype_code(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise _lib.NrseError(f"unsupported dtype {t.dtype}") from None


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t: torch.Tensor | None, offset_elems: int = 0) -> int | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise _lib.NrseError("libnrse_hip ops take device tensors")
    return t.data_ptr() + offset_elems * t.element_size()


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
         aux: torch.Tensor | None = None, ldaux: int = 0, aux_z1: int = 0, aux_z2: int = 0,
         resid: torch.Tensor | None = None, ldr: int = 0, r_z1: int = 0, r_z2: int = 0,
         dropout_p: float = 0.0, seed: int = 0, colsum: torch.Tensor | None = None) -> None:
    """C[m,n] = epilogue(alpha * sum_k A(m,k) B(n,k)); see nrse_gemm."""
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous()
    if colsum is not None:
        assert colsum.dtype == torch.float32
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
    _lib.check(_lib.lib().nrse_gemm(ctypes.byref(p), stream_ptr()), "nrse_gemm")


# ----------------------------------------------------------------------------- linear helpers
def linear_fwd(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, *, bias=None, flags: int = 0, **kw) -> None:
    """out[M,N] = x[M,K] @ w[N,K]^T (+ epilogue). x, w share the compute dtype."""
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K and out.shape[-1] >= N
    if bias is not None:
        flags |= _lib.EPI_BIAS
    gemm(Operand(x, True, x.stride(0)), Operand(w, True, w.stride(0)), out, M, N, K, ldc=out.stride(0),
         bias=bias, flags=flags, **kw)


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, dx: torch.Tensor, *, flags: int = 0, **kw) -> None:
    """dx[M,K] = dy[M,N] @ w[N,K]."""
    M, N = dy.shape
    K = w.shape[1]
    assert w.shape[0] == N
    gemm(Operand(dy, True, dy.stride(0)), Operand(w, False, w.stride(0)), dx, M, K, N, ldc=dx.stride(0),
         flags=flags, **kw)


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, *, splits: int = 1, colsum=None,
                 accumulate: bool = True) -> None:
    """dw[N,K] (+)= dy[M,N]^T @ x[M,K]  (f32 dw). Optionally colsum(dy) -> bias grad."""
    M, N = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and dw.shape == (N, K) and dw.dtype == torch.float32
    splits = max(1, min(splits, M // 256))
    seg = (M + splits - 1) // splits
    seg = (seg + 7) // 8 * 8
    nseg_total = (M + seg - 1) // seg
    if nseg_total * seg != M:
        # ragged last split: run the bulk split-K and the tail separately
        bulk = (M // seg) * seg
        if bulk:
            linear_wgrad(dy[:bulk], x[:bulk], dw, splits=bulk // seg, accumulate=accumulate)
        linear_wgrad(dy[bulk:], x[bulk:], dw, splits=1, accumulate=True)
        if colsum is not None:
            from . import ops_small
            ops_small.colsum(dy, colsum)
        return
    flags = _lib.EPI_ATOMIC if (splits > 1 or accumulate) else 0
    gemm(Operand(dy, False, dy.stride(0), seg_stride=seg * dy.stride(0)),
         Operand(x, False, x.stride(0), seg_stride=seg * x.stride(0)),
         dw, N, K, seg, ldc=dw.stride(0), nseg=1, splits=splits, flags=flags)
    if colsum is not None:
        from . import ops_small
        ops_small.colsum(dy, colsum)
