"""ctypes binding of libnrse_hip.so (the C-ABI declared in include/nrse_hip.h).

The library is the only compute path: if it cannot be loaded, or the device is not gfx950,
every op raises instead of falling back to PyTorch/CPU arithmetic.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# NRSE_LIB_PATH: load a differently built copy of the same library (diagnostic builds)
LIB_PATH = os.environ.get("NRSE_LIB_PATH") or os.path.join(_HERE, "libnrse_hip.so")

F32 = 0
BF16 = 1
BF16X3 = 2   # output-only split-bf16 planes [hi | lo | hi] (include/nrse_hip.h)
FP8 = 3      # OCP fp8 e4m3fn, the split-weight mode's correction operands (ABI 6)

EPI_BIAS = 1 << 0
EPI_GELU = 1 << 1
EPI_GELU_BWD = 1 << 2
EPI_DROPOUT = 1 << 3
EPI_RESID = 1 << 4
EPI_DROP_AFTER = 1 << 5
EPI_ACCUM = 1 << 6
EPI_ATOMIC = 1 << 7
EPI_COLSUM = 1 << 8
EPI_RELU = 1 << 9
EPI_TANH = 1 << 10

LN_GELU = 1
LN_RELU = 2
DY_DIRECT, DY_COL2IM, DY_BCAST = 0, 1, 2

c_ll = ctypes.c_longlong
c_vp = ctypes.c_void_p
c_int = ctypes.c_int
c_f = ctypes.c_float
c_u32 = ctypes.c_uint32


class NrseCaps(ctypes.Structure):
    _fields_ = [("device", c_int), ("cu_count", c_int), ("xcd_count", c_int),
                ("lds_bytes_per_cu", c_int), ("hbm_bytes", c_ll), ("arch", ctypes.c_char * 32)]


ABI_VERSION = 11   # NRSE_ABI_VERSION of include/nrse_hip.h this binding is written against


class _Sized(ctypes.Structure):
    """A params struct of the ABI 10 handshake: its first field is `struct_size`, stamped with
    sizeof(struct) as laid out here; the library refuses any other value (NRSE_ERR_ARG), so a
    binding out of step with the header fails loudly instead of having its struct over-read.
    Positional constructor arguments fill the fields after struct_size."""

    def __init__(self, *args, **kw):
        super().__init__(ctypes.sizeof(type(self)), *args, **kw)


class GemmOperand(ctypes.Structure):
    _fields_ = [("ptr", c_vp), ("dtype", c_int), ("kcontig", c_int), ("chunk_shift", c_int),
                ("ld", c_ll), ("ld_chunk", c_ll), ("seg_stride", c_ll), ("z1", c_ll), ("z2", c_ll)]


class GemmParams(_Sized):
    _fields_ = [("struct_size", c_u32), ("a", GemmOperand), ("b", GemmOperand),
                ("M", c_int), ("N", c_int), ("K", c_int), ("nseg", c_int),
                ("splits", c_int), ("batch", c_int), ("zdiv", c_int),
                ("alpha", c_f), ("flags", c_int),
                ("c", c_vp), ("c_dtype", c_int), ("ldc", c_ll), ("c_z1", c_ll), ("c_z2", c_ll),
                ("c_split", c_ll),
                ("bias", c_vp), ("bias_z1", c_ll), ("bias_z2", c_ll),
                ("aux", c_vp), ("aux_dtype", c_int), ("ldaux", c_ll), ("aux_z1", c_ll),
                ("aux_z2", c_ll), ("resid", c_vp), ("resid_dtype", c_int), ("ldr", c_ll), ("r_z1", c_ll),
                ("r_z2", c_ll), ("dropout_p", c_f), ("seed", c_u32), ("colsum", c_vp),
                ("colsum_part", c_vp),
                ("a8", GemmOperand), ("b8", GemmOperand), ("nseg8", c_int), ("b8_exp", c_int),
                ("c8", c_vp), ("ldc8", c_ll), ("c8_dtype", c_int)]


class LnFwdParams(_Sized):
    _fields_ = [("struct_size", c_u32), ("x", c_vp), ("x_dtype", c_int), ("gamma", c_vp), ("beta", c_vp), ("y", c_vp), ("y_dtype", c_int),
                ("mean", c_vp), ("rstd", c_vp), ("rows", c_ll), ("C", c_int), ("eps", c_f), ("flags", c_int),
                ("y8", c_vp), ("y8_split", c_int), ("y8_exp", c_int), ("y8_dtype", c_int), ("sat_count", c_vp)]


class LnBwdParams(_Sized):
    _fields_ = [("struct_size", c_u32), ("dy", c_vp), ("dy_dtype", c_int), ("dy_mode", c_int),
                ("col_k", c_int), ("col_s", c_int), ("col_tout", c_int), ("col_tin", c_int),
                ("bcast_t", c_int), ("dy_scale", c_f),
                ("x", c_vp), ("x_dtype", c_int), ("gamma", c_vp), ("beta", c_vp), ("mean", c_vp), ("rstd", c_vp),
                ("dx", c_vp), ("dx_dtype", c_int), ("resid", c_vp), ("dgamma", c_vp), ("dbeta", c_vp),
                ("rows", c_ll), ("C", c_int), ("flags", c_int),
                ("dv", c_vp), ("dv_dtype", c_int), ("dv_colsum", c_vp), ("dv_p", c_f), ("dv_seed", c_u32),
                ("part", c_vp), ("gate_dp", c_vp), ("gate_w", c_vp)]


class AttnFwdParams(_Sized):
    _fields_ = [("struct_size", c_u32), ("qkv", c_vp), ("dtype", c_int), ("gate", c_vp), ("bias", c_vp), ("ctx", c_vp), ("lse", c_vp),
                ("batch", c_int), ("T", c_int), ("H", c_int), ("head_dim", c_int), ("scale", c_f),
                ("dropout_p", c_f), ("seed", c_u32), ("bias_vec", c_vp), ("drop_mask", c_vp),
                ("drop_mask_in", c_int), ("ctx8", c_vp), ("ctx8_dtype", c_int)]


class AttnBwdParams(_Sized):
    _fields_ = [("struct_size", c_u32), ("qkv", c_vp), ("dtype", c_int), ("gate", c_vp), ("bias", c_vp), ("ctx", c_vp), ("dctx", c_vp),
                ("lse", c_vp), ("delta", c_vp), ("dqkv", c_vp), ("dgate", c_vp), ("diag", c_vp),
                ("batch", c_int), ("T", c_int), ("H", c_int), ("head_dim", c_int), ("scale", c_f),
                ("dropout_p", c_f), ("seed", c_u32), ("bias_vec", c_vp), ("diag_part", c_vp), ("drop_mask", c_vp)]


class Conv0Params(_Sized):
    _fields_ = [("struct_size", c_u32), ("wav", c_vp), ("L", c_int), ("w", c_vp), ("gamma", c_vp), ("beta", c_vp), ("out", c_vp),
                ("out_dtype", c_int), ("mean", c_vp), ("rstd", c_vp),
                ("dy", c_vp), ("dy_dtype", c_int), ("dy_mode", c_int), ("col_k", c_int), ("col_s", c_int),
                ("col_tout", c_int), ("dw", c_vp), ("dgamma", c_vp), ("dbeta", c_vp),
                ("batch", c_int), ("T0", c_int), ("C", c_int), ("k", c_int), ("s", c_int), ("eps", c_f),
                ("part", c_vp), ("y8", c_vp), ("y8_exp", c_int), ("y8_dtype", c_int), ("sat_count", c_vp)]


class AdamWParams(_Sized):
    _fields_ = [("struct_size", c_u32), ("p", c_vp), ("g", c_vp), ("m", c_vp), ("v", c_vp), ("p_shadow", c_vp), ("shadow_dtype", c_int),
                ("n", c_ll), ("lr", c_f), ("beta1", c_f), ("beta2", c_f), ("eps", c_f), ("weight_decay", c_f),
                ("step", c_int), ("max_norm", c_f), ("sumsq", c_vp), ("grad_scale", c_f),
                ("p_shadow_lo", c_vp), ("ema_t", c_vp), ("ema_shadow", c_vp), ("ema_shadow_lo", c_vp),
                ("ema_shadow_dtype", c_int), ("ema_decay", c_f), ("ema_n", c_ll),
                ("p_shadow_lo8", c_vp), ("ema_shadow_lo8", c_vp), ("lo8_exp", c_int), ("zero_grad", c_int),
                ("lo8_dtype", c_int), ("sat_count", c_vp), ("sat_ranges", c_vp), ("sat_nranges", c_int),
                ("sat_offset", c_ll)]


_P = ctypes.POINTER
# Every symbol include/nrse_hip.h declares, with its ctypes signature (argtypes, restype).
# tests/test_abi.py checks this table against the header.
_SIGNATURES = {
    "nrse_init": ([c_int, _P(NrseCaps)], c_int),
    "nrse_last_error": ([], ctypes.c_char_p),
    "nrse_abi_version": ([], c_int),
    "nrse_gemm": ([_P(GemmParams), c_vp], c_int),
    "nrse_gemm_colsum_workspace": ([_P(GemmParams)], c_ll),
    "nrse_gemm_select": ([c_int], c_int),
    "nrse_gemm_tile_rows": ([c_int], c_int),
    "nrse_layernorm_fwd": ([_P(LnFwdParams), c_vp], c_int),
    "nrse_layernorm_bwd": ([_P(LnBwdParams), c_vp], c_int),
    "nrse_layernorm_bwd_workspace": ([_P(LnBwdParams)], c_ll),
    "nrse_ln_mean_fwd": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_f, c_vp, c_vp], c_int),
    "nrse_bias_ld": ([c_int], c_int),
    "nrse_rel_bias_fwd": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp], c_int),
    "nrse_rel_bias_vec": ([c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp], c_int),
    "nrse_rel_bias_bwd": ([c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp], c_int),
    "nrse_gate_fwd": ([c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp], c_int),
    "nrse_gate_bwd_workspace": ([c_int], c_ll),
    "nrse_gate_bwd": ([c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp],
                      c_int),
    "nrse_gate_bwd_dp": ([c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp,
                          c_vp], c_int),
    "nrse_attn_dropout_mask": ([c_vp, c_int, c_int, c_int, c_f, c_u32, c_vp], c_int),
    "nrse_attn_fwd": ([_P(AttnFwdParams), c_vp], c_int),
    "nrse_attn_bwd": ([_P(AttnBwdParams), c_vp], c_int),
    "nrse_attn_bwd_workspace": ([_P(AttnBwdParams)], c_ll),
    "nrse_attn_mask_elems": ([c_int, c_int, c_int], c_ll),
    "nrse_conv0_fwd": ([_P(Conv0Params), c_vp], c_int),
    "nrse_conv0_bwd": ([_P(Conv0Params), c_vp], c_int),
    "nrse_conv0_bwd_workspace": ([_P(Conv0Params)], c_ll),
    "nrse_weight_norm_fwd": ([c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_vp, c_vp], c_int),
    "nrse_weight_norm_bwd": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp], c_int),
    "nrse_specaug_pad": ([c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
    "nrse_specaug_mask": ([c_vp, c_int, c_int, ctypes.c_double, c_int, c_int, c_u32, c_vp], c_int),
    "nrse_pad_rows": ([c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
    "nrse_specaug_bwd": ([c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_f, c_u32, c_vp, c_vp], c_int),
    "nrse_dropout_cast": ([c_vp, c_vp, c_int, c_ll, c_f, c_u32, c_vp], c_int),
    "nrse_dropout_cast_colsum": ([c_vp, c_vp, c_int, c_ll, c_int, c_f, c_u32, c_vp, c_vp, c_vp], c_int),
    "nrse_colsum": ([c_vp, c_int, c_vp, c_ll, c_int, c_vp, c_vp], c_int),
    "nrse_colsum_workspace": ([c_ll, c_int], c_ll),
    "nrse_cast": ([c_vp, c_int, c_vp, c_int, c_ll, c_vp], c_int),
    "nrse_split_bf16": ([c_vp, c_vp, c_vp, c_ll, c_vp], c_int),
    "nrse_split_lo8": ([c_vp, c_vp, c_int, c_ll, c_vp, c_vp], c_int),
    "nrse_cast_fp8": ([c_vp, c_int, c_vp, c_ll, c_vp], c_int),
    "nrse_zero": ([c_vp, c_ll, c_vp], c_int),
    "nrse_splitk_reduce": ([c_vp, c_vp, c_int, c_ll, c_int, c_vp], c_int),
    "nrse_rows_reduce": ([c_vp, c_ll, c_vp, c_ll, c_vp, c_ll, c_vp, c_int, c_int, c_int, c_vp], c_int),
    "nrse_reduce_defer": ([c_int], c_int),
    "nrse_reduce_pending": ([], c_int),
    "nrse_reduce_flush": ([c_vp], c_int),
    "nrse_reduce_discard": ([], c_int),
    "nrse_swap12": ([c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
    "nrse_gelu_bwd_pad": ([c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
    "nrse_bn_fwd": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_f, c_f, c_int, c_int, c_vp], c_int),
    "nrse_bn_bwd": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp], c_int),
    "nrse_bn_stats": ([c_vp, c_vp, c_int, c_int, c_vp], c_int),
    "nrse_bn_fwd_global": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_int, c_int, c_f, c_f, c_int,
                            c_vp], c_int),
    "nrse_bn_bwd_sums": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp], c_int),
    "nrse_bn_bwd_global": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_vp, c_vp, c_vp, c_int, c_int,
                            c_int, c_vp], c_int),
    "nrse_byol_loss": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_f, c_vp, c_vp], c_int),
    "nrse_sumsq": ([c_vp, c_ll, c_vp, c_vp, c_vp], c_int),
    "nrse_adamw": ([_P(AdamWParams), c_vp], c_int),
    "nrse_ema": ([c_vp, c_vp, c_vp, c_int, c_ll, c_f, c_vp, c_vp], c_int),
    "nrse_health": ([c_vp, c_int, c_ll, c_vp, c_vp], c_int),
    "nrse_asp_fwd": ([c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp], c_int),
    "nrse_asp_bwd": ([c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp,
                      c_vp], c_int),
    "nrse_ccc_loss": ([c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp], c_int),
    "nrse_snr_mix": ([c_vp, c_vp, c_vp, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp], c_int),
}


class NrseError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libnrse_hip.so (raises if missing: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NrseError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (argt, rest) in _SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = rest
        v = int(L.nrse_abi_version())
        if v != ABI_VERSION:
            raise NrseError(f"{LIB_PATH} is ABI {v}, this binding is ABI {ABI_VERSION}: rebuild the library")
        _lib = L
    return _lib


def exported_symbols():
    return sorted(_SIGNATURES)


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().nrse_last_error().decode(errors="replace")
        raise NrseError(f"{what} failed (status {rc}): {msg}")


_initialised_devices = set()


def init_device(device: int = 0) -> NrseCaps:
    caps = NrseCaps()
    check(lib().nrse_init(device, ctypes.byref(caps)), "nrse_init")
    _initialised_devices.add(device)
    return caps


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)
