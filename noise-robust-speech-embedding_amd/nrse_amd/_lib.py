"""ctypes binding of libnrse_hip.so (the C-ABI declared in include/nrse_hip.h).

The library is the only compute path: if it cannot be loaded, or the device is not gfx950,
every op raises instead of falling back to PyTorch/CPU arithmetic.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libnrse_hip.so")

F32 = 0
BF16 = 1

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

c_ll = ctypes.c_longlong
c_vp = ctypes.c_void_p


class NrseCaps(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("cu_count", ctypes.c_int), ("xcd_count", ctypes.c_int),
                ("lds_bytes_per_cu", ctypes.c_int), ("hbm_bytes", c_ll), ("arch", ctypes.c_char * 32)]


class GemmOperand(ctypes.Structure):
    _fields_ = [("ptr", c_vp), ("dtype", ctypes.c_int), ("kcontig", ctypes.c_int), ("chunk_shift", ctypes.c_int),
                ("ld", c_ll), ("ld_chunk", c_ll), ("seg_stride", c_ll), ("z1", c_ll), ("z2", c_ll)]


class GemmParams(ctypes.Structure):
    _fields_ = [("a", GemmOperand), ("b", GemmOperand),
                ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int), ("nseg", ctypes.c_int),
                ("splits", ctypes.c_int), ("batch", ctypes.c_int), ("zdiv", ctypes.c_int),
                ("alpha", ctypes.c_float), ("flags", ctypes.c_int),
                ("c", c_vp), ("c_dtype", ctypes.c_int), ("ldc", c_ll), ("c_z1", c_ll), ("c_z2", c_ll),
                ("c_split", c_ll),
                ("bias", c_vp), ("aux", c_vp), ("aux_dtype", ctypes.c_int), ("ldaux", c_ll), ("aux_z1", c_ll),
                ("aux_z2", c_ll), ("resid", c_vp), ("resid_dtype", ctypes.c_int), ("ldr", c_ll), ("r_z1", c_ll),
                ("r_z2", c_ll), ("dropout_p", ctypes.c_float), ("seed", ctypes.c_uint32), ("colsum", c_vp)]


# Every symbol include/nrse_hip.h declares, with its ctypes signature (argtypes, restype).
# tests/test_abi.py checks this table against the header.
_SIGNATURES = {
    "nrse_init": ([ctypes.c_int, ctypes.POINTER(NrseCaps)], ctypes.c_int),
    "nrse_last_error": ([], ctypes.c_char_p),
    "nrse_abi_version": ([], ctypes.c_int),
    "nrse_gemm": ([ctypes.POINTER(GemmParams), c_vp], ctypes.c_int),
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
