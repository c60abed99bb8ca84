"""CPU restatement of NRSE_MX6 (include/nrse_hip.h, ABI 8): OCP MXFP6 e2m3 in blocks of 32
consecutive elements along the last axis, one E8M0 scale per block, in fp8's byte footprint.

TEST INFRASTRUCTURE ONLY (tests/, bench.py's cpu_baseline, __graft_entry__.smoke()): the checker
the kernels' MXFP6 producers (nrse_cast_mx6, nrse_split_lo_mx6, the LayerNorm / conv0 / attention /
GEMM-epilogue / AdamW forms) are compared with byte for byte, and the quantiser the oracle's
split-weight restatement (oracle/wavlm_byol.py, set_split8(..., fmt="mx6")) applies. The format is
this framework's own (the reference computes in f32 and has no such operand); it follows the OCP
Microscaling spec's e2m3 element (1 sign, 2 exponent bits with bias 1, 3 mantissa bits, max 7.5, no
inf / NaN) and E8M0 scale (2^(s - 127)). Block b of a row, at byte 32b:
  bytes 0..23   value j at bits 6j .. 6j+5 (little-endian bit order across the 24 bytes)
  byte 24       s = X + 127, X the smallest exponent with max|x| <= 7.5 * 2^X (X >= -127)
  bytes 25..31  zero
Values are x * 2^-X rounded to nearest even (subnormals m/8 below 1), |.| clamped to 7.5.
"""
import numpy as np


def _exp(amax: np.ndarray) -> np.ndarray:
    """Block exponent X of float32 amax (csrc/common.h mx6_exp)."""
    b = amax.astype(np.float32).view(np.uint32).astype(np.int64)
    X = (b >> 23) - 129 + ((b & 0x7FFFFF) > 0x700000)
    return np.maximum(X, -127)


def _e2m3(q: np.ndarray) -> np.ndarray:
    """e2m3 codes (sign bit 5) of float32 q, RNE, |q| clamped to 7.5 (csrc/common.h e2m3)."""
    q = q.astype(np.float32)
    s = np.signbit(q).astype(np.int64) << 5
    a = np.minimum(np.abs(q), np.float32(7.5)).astype(np.float32)
    sub = np.rint(a * np.float32(8.0)).astype(np.int64)
    b = a.view(np.uint32).astype(np.int64)
    b = b + 0x7FFFF + ((b >> 20) & 1)
    nrm = (((b >> 23) - 126) << 3) | ((b >> 20) & 7)
    return s | np.where(a < 1.0, sub, nrm)


def _value(code: np.ndarray) -> np.ndarray:
    code = code.astype(np.int64)
    e = (code >> 3) & 3
    m = (code & 7).astype(np.float64)
    v = np.where(e == 0, m / 8.0, (1.0 + m / 8.0) * np.exp2(e - 1.0))
    return np.where(code & 32, -v, v)


def encode(x) -> np.ndarray:
    """x [..., K] (K % 32 == 0) -> uint8 [..., K]: the NRSE_MX6 bytes."""
    x = np.asarray(x, dtype=np.float32)
    K = x.shape[-1]
    assert K % 32 == 0, K
    xb = x.reshape(*x.shape[:-1], K // 32, 32)
    X = _exp(np.abs(xb).max(-1))
    inv = ((127 - X).astype(np.uint32) << 23).view(np.float32)
    codes = _e2m3(xb * inv[..., None])
    out = np.zeros(xb.shape[:-1] + (32,), dtype=np.int64)
    for j in range(32):
        bit = 6 * j
        byte, off = bit >> 3, bit & 7
        out[..., byte] |= (codes[..., j] << off) & 0xFF
        if off > 2:
            out[..., byte + 1] |= codes[..., j] >> (8 - off)
    out[..., 24] = X + 127
    return out.astype(np.uint8).reshape(x.shape)


def decode(y) -> np.ndarray:
    """uint8 NRSE_MX6 bytes [..., K] -> float64 values [..., K]."""
    y = np.asarray(y, dtype=np.uint8)
    K = y.shape[-1]
    yb = y.reshape(*y.shape[:-1], K // 32, 32).astype(np.int64)
    codes = np.zeros(yb.shape[:-1] + (32,), dtype=np.int64)
    for j in range(32):
        bit = 6 * j
        byte, off = bit >> 3, bit & 7
        c = yb[..., byte] >> off
        if off > 2:
            c = c | (yb[..., byte + 1] << (8 - off))
        codes[..., j] = c & 63
    scale = np.exp2(yb[..., 24].astype(np.float64) - 127.0)
    return (_value(codes) * scale[..., None]).reshape(y.shape)


def round_trip(x) -> np.ndarray:
    """The value an MXFP6 operand carries for x (float64)."""
    return decode(encode(x))
