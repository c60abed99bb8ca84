// Shared device helpers for the gfx950 kernels of libnrse_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/nrse_hip.h"

typedef unsigned short bf16_t;  // storage type for bf16 in memory
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define NRSE_DEV __device__ __forceinline__

// Load through an explicit global (addrspace 1) pointer: a generic pointer the compiler cannot
// prove global becomes a flat load, which also counts in lgkmcnt, so every LDS / shuffle wait
// after it (lgkmcnt(0)) waits for the memory load too.
template <typename T>
NRSE_DEV T ldg(const T* p) {  // scalars and ext-vector types
  return *(const __attribute__((address_space(1))) T*)p;
}
NRSE_DEV uint2 ldg(const uint2* p) {  // HIP vector struct: load as an ext vector, bit-cast
  typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint2, *(const __attribute__((address_space(1))) u32x2v*)p);
}
NRSE_DEV uint4 ldg(const uint4* p) {
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(uint4, *(const __attribute__((address_space(1))) u32x4v*)p);
}

NRSE_DEV float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }
NRSE_DEV bf16_t f2bf(float x) {
  __bf16 b = (__bf16)x;  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN stays NaN
  return *reinterpret_cast<bf16_t*>(&b);
}
// low half of the split-bf16 pair of x: bf16(x - float(bf16(x)))
NRSE_DEV bf16_t bf16_lo(float x) {
  const bf16_t h = f2bf(x);
  return f2bf(x - __uint_as_float((uint32_t)h << 16));
}

// 4 consecutive values at element i of an output in dtype dt: f32, bf16, or the three-plane split
// bf16 form NRSE_BF16X3 ([hi | lo | hi], planes `plane` elements apart; include/nrse_hip.h)
NRSE_DEV void store4_out(void* p, int dt, long long i, long long plane, const float* o) {
  if (dt == NRSE_F32) {
    *reinterpret_cast<float4*>((float*)p + i) = make_float4(o[0], o[1], o[2], o[3]);
    return;
  }
  uint2 u;
  u.x = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
  u.y = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
  bf16_t* b = (bf16_t*)p + i;
  *reinterpret_cast<uint2*>(b) = u;
  if (dt == NRSE_BF16X3) {
    uint2 w;
    w.x = (uint32_t)f2bf(o[0] - __uint_as_float(u.x << 16)) | ((uint32_t)f2bf(o[1] - __uint_as_float(u.x & 0xffff0000u)) << 16);
    w.y = (uint32_t)f2bf(o[2] - __uint_as_float(u.y << 16)) | ((uint32_t)f2bf(o[3] - __uint_as_float(u.y & 0xffff0000u)) << 16);
    *reinterpret_cast<uint2*>(b + plane) = w;
    *reinterpret_cast<uint2*>(b + 2 * plane) = u;
  }
}

// OCP fp8 e4m3fn (NRSE_FP8, gfx950's native fp8): v_cvt_pk_fp8_f32 rounds to nearest even; the
// inputs are clamped to the largest finite value first (+-448), so out-of-range values saturate
// instead of becoming NaN. fp8x4 packs a, b, c, d into bytes 0..3 (little-endian element order).
NRSE_DEV uint32_t fp8x4(float a, float b, float c, float d) {
  a = __builtin_amdgcn_fmed3f(a, -448.f, 448.f);
  b = __builtin_amdgcn_fmed3f(b, -448.f, 448.f);
  c = __builtin_amdgcn_fmed3f(c, -448.f, 448.f);
  d = __builtin_amdgcn_fmed3f(d, -448.f, 448.f);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}
NRSE_DEV unsigned char fp8_1(float a) { return (unsigned char)(fp8x4(a, 0.f, 0.f, 0.f) & 0xffu); }
// ABI 10: how many of 4 values fp8x4 saturates (|v| > 448, clamped instead of rounded), and the
// producers' counter update (an atomic only when something saturated: never in normal operation).
// The common case (nothing saturates) costs two max and one compare; the exact count runs only
// in a wave where some lane saturated (wave-uniform branch)
#ifndef NRSE_SAT_FAST
#define NRSE_SAT_FAST 1   // 0: the exact count on every call (A/B)
#endif
NRSE_DEV int fp8_nsat4(float a, float b, float c, float d) {
#if NRSE_SAT_FAST
  const float m = fmaxf(fmaxf(fabsf(a), fabsf(b)), fmaxf(fabsf(c), fabsf(d)));
  if (!__builtin_amdgcn_ballot_w64(m > 448.f)) return 0;
#endif
  return (int)(fabsf(a) > 448.f) + (int)(fabsf(b) > 448.f) + (int)(fabsf(c) > 448.f) + (int)(fabsf(d) > 448.f);
}
NRSE_DEV void sat_count_add(unsigned int* cnt, int n) {
  if (n && cnt) atomicAdd(cnt, (unsigned int)n);
}
// the split-weight mode's fp8 correction of x (nrse_split_lo8): (x - bf16(x)) * sc, sc = 2^lo8_exp
NRSE_DEV float lo_resid(float x) { return x - __uint_as_float((uint32_t)f2bf(x) << 16); }
// fp8 of 4 values as they are stored in bf16 (the a8 operand is fp8(bf16 y), one rounding path)
NRSE_DEV uint32_t fp8x4_of_bf(const float* o) {
  return fp8x4(bf2f(f2bf(o[0])), bf2f(f2bf(o[1])), bf2f(f2bf(o[2])), bf2f(f2bf(o[3])));
}
// the two fp8 correction planes of 4 exact values o (ABI 7, y8_split): lo8 = fp8((o - bf16(o)) sc)
// (sc = 2^y8_exp), hi8 = fp8(bf16(o)) -- the conv stack's a8 segments of the split-weight mode
NRSE_DEV void fp8x4_split(const float* o, float sc, uint32_t& lo8, uint32_t& hi8, int* nsat = nullptr) {
  float h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = bf2f(f2bf(o[e]));
    l[e] = (o[e] - h[e]) * sc;
  }
  lo8 = fp8x4(l[0], l[1], l[2], l[3]);
  hi8 = fp8x4(h[0], h[1], h[2], h[3]);
  if (nsat) *nsat += fp8_nsat4(l[0], l[1], l[2], l[3]) + fp8_nsat4(h[0], h[1], h[2], h[3]);
}
// 8 packed bf16 (a 16-B row chunk) -> 8 fp8 bytes
NRSE_DEV uint2 fp8x8_from_bf16x8(uint4 u) {
  uint2 r;
  r.x = fp8x4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
              __uint_as_float(u.y & 0xffff0000u));
  r.y = fp8x4(__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u), __uint_as_float(u.w << 16),
              __uint_as_float(u.w & 0xffff0000u));
  return r;
}

template <typename T> NRSE_DEV float to_f(T x);
template <> NRSE_DEV float to_f<float>(float x) { return x; }
template <> NRSE_DEV float to_f<bf16_t>(bf16_t x) { return bf2f(x); }
template <typename T> NRSE_DEV T from_f(float x);
template <> NRSE_DEV float from_f<float>(float x) { return x; }
template <> NRSE_DEV bf16_t from_f<bf16_t>(float x) { return f2bf(x); }

NRSE_DEV float load_as_f(const void* p, int dtype, long long i) {
  return dtype == NRSE_BF16 ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}
NRSE_DEV void store_from_f(void* p, int dtype, long long i, float v) {
  if (dtype == NRSE_BF16) ((bf16_t*)p)[i] = f2bf(v);
  else ((float*)p)[i] = v;
}


// Fast erf: odd/even rational minimax approximation on [-4, 4] (the single-precision
// coefficient set used by XLA / Eigen), |error| < 7e-8 in exact arithmetic and < 5e-7 evaluated
// in f32 (erff: ~35 VALU instructions with both branches taken in a divergent wave; this: 14).
NRSE_DEV float erf_fast(float x) {
  x = fminf(fmaxf(x, -4.f), 4.f);
  const float x2 = x * x;
  float p = fmaf(x2, -2.72614225801306e-10f, 2.77068142495902e-08f);
  p = fmaf(x2, p, -2.10102402082508e-06f);
  p = fmaf(x2, p, -5.69250639462346e-05f);
  p = fmaf(x2, p, -7.34990630326855e-04f);
  p = fmaf(x2, p, -2.95459980854025e-03f);
  p = fmaf(x2, p, -1.60960333262415e-02f);
  float q = fmaf(x2, -1.45660718464996e-05f, -2.13374055278905e-04f);
  q = fmaf(x2, q, -1.68282697438203e-03f);
  q = fmaf(x2, q, -7.37332916720468e-03f);
  q = fmaf(x2, q, -1.42647390514189e-02f);
  return x * p * __builtin_amdgcn_rcpf(q);
}
NRSE_DEV float gelu_fast(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
// GELU'(x) = Phi(x) + x phi(x) with ONE exponential shared by both terms: Phi from the
// Abramowitz-Stegun 7.1.26 form erfc(a) = poly(t) e^{-a^2}, t = 1 / (1 + p a), a = |x| / sqrt2,
// so e = exp(-x^2 / 2) is also sqrt(2 pi) phi(x). |error| < 3.0e-7 over all x evaluated in f32
// (the rational-erf form it replaces: 2.6e-7), 16 instructions instead of 22 (both with one rcp
// and one exp): the GELU' of the conv0 / conv-stack LN backward and of the GELU_BWD epilogues.
NRSE_DEV float gelu_grad_fast(float x) {
  const float t = __builtin_amdgcn_rcpf(fmaf(__builtin_fabsf(x), 0.3275911f * 0.70710678118654752f, 1.0f));
  float q = fmaf(t, 1.061405429f, -1.453152027f);
  q = fmaf(t, q, 1.421413741f);
  q = fmaf(t, q, -0.284496736f);
  q = fmaf(t, q, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f((x * (-0.5f * 1.4426950408889634f)) * x);
  const float h = 0.5f * (t * q) * e;  // 0.5 erfc(|x| / sqrt2)
  const float cdf = x >= 0.f ? 1.0f - h : h;
  return fmaf(x * 0.39894228040143268f, e, cdf);
}
// Two-lane (packed FP32) forms of the same evaluation, op for op: the polynomial FMAs and
// products issue as v_pk_fma_f32 / v_pk_mul_f32 (two elements per VALU instruction); the clamp
// (v_med3), rcp and exp stay per element. Used where measured faster (conv0 forward, 5%; the
// 256x256 GEMM's register epilogue, FFN-up +1.4 % isolated in r03 -- an r02 GEMM epilogue had
// measured 1 % slower with it); in the LN kernels and conv0 backward the packed form was neutral
// or slower.
typedef float f32x2 __attribute__((ext_vector_type(2)));
NRSE_DEV f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
NRSE_DEV f32x2 splat2(float v) { return f32x2{v, v}; }
NRSE_DEV f32x2 erf_fast2(f32x2 x) {
  x = f32x2{__builtin_amdgcn_fmed3f(x.x, -4.f, 4.f), __builtin_amdgcn_fmed3f(x.y, -4.f, 4.f)};
  const f32x2 x2 = x * x;
  f32x2 p = pk_fma(x2, splat2(-2.72614225801306e-10f), splat2(2.77068142495902e-08f));
  p = pk_fma(x2, p, splat2(-2.10102402082508e-06f));
  p = pk_fma(x2, p, splat2(-5.69250639462346e-05f));
  p = pk_fma(x2, p, splat2(-7.34990630326855e-04f));
  p = pk_fma(x2, p, splat2(-2.95459980854025e-03f));
  p = pk_fma(x2, p, splat2(-1.60960333262415e-02f));
  f32x2 q = pk_fma(x2, splat2(-1.45660718464996e-05f), splat2(-2.13374055278905e-04f));
  q = pk_fma(x2, q, splat2(-1.68282697438203e-03f));
  q = pk_fma(x2, q, splat2(-7.37332916720468e-03f));
  q = pk_fma(x2, q, splat2(-1.42647390514189e-02f));
  return x * p * f32x2{__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
}
NRSE_DEV f32x2 gelu2(f32x2 x) { return splat2(0.5f) * x * (splat2(1.0f) + erf_fast2(x * splat2(0.70710678118654752f))); }
// gelu_grad_fast of two lanes, op for op (same values): the polynomial and products packed, rcp /
// exp2 / the sign select per element
NRSE_DEV f32x2 gelu_grad2(f32x2 x) {
  const f32x2 ax = f32x2{__builtin_fabsf(x.x), __builtin_fabsf(x.y)};
  const f32x2 d = pk_fma(ax, splat2(0.3275911f * 0.70710678118654752f), splat2(1.0f));
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 q = pk_fma(t, splat2(1.061405429f), splat2(-1.453152027f));
  q = pk_fma(t, q, splat2(1.421413741f));
  q = pk_fma(t, q, splat2(-0.284496736f));
  q = pk_fma(t, q, splat2(0.254829592f));
  const f32x2 ea = (x * splat2(-0.5f * 1.4426950408889634f)) * x;
  const f32x2 e = f32x2{__builtin_amdgcn_exp2f(ea.x), __builtin_amdgcn_exp2f(ea.y)};
  const f32x2 h = splat2(0.5f) * (t * q) * e;
  const f32x2 cdf = f32x2{x.x >= 0.f ? 1.0f - h.x : h.x, x.y >= 0.f ? 1.0f - h.y : h.y};
  return pk_fma(x * splat2(0.39894228040143268f), e, cdf);
}

// erf GELU as ACT2FN["gelu"] ([TF] activations.GELUActivation -> F.gelu default), evaluated with
// erf_fast everywhere (|error| ~5e-7, the order of f32 erff's own; the parity tolerances are
// 1e-5 rel-L2 per kernel and 1e-3 on embeddings).
NRSE_DEV float gelu_f(float x) { return gelu_fast(x); }
NRSE_DEV float gelu_grad_f(float x) { return gelu_grad_fast(x); }

// Column sums of the COLSUM epilogue: with p.colsum_part, each workgroup writes its two half-tile
// partial sums to rows (z * mt + m_tile) * 2 + {0, 1} of the [rows][N] slab (added in order by
// nrse_rows_reduce in nrse_gemm: deterministic); without it, f32 atomics into p.colsum.
NRSE_DEV void colsum_out(const nrse_gemm_params& p, int z, int mt, int mtile, int sub, int n, float v) {
  if (p.colsum_part) p.colsum_part[(((long long)z * mt + mtile) * 2 + sub) * p.N + n] = v;
  else atomicAdd(p.colsum + n, v);
}

// Counter-based dropout hash (bijective 32-bit mixer, "lowbias32"), one hash per PAIR of
// elements, 16 bits each: the mask of flat element i at a dropout site seeded with `seed` is
//   h = mix32((i >> 1) ^ site_key(seed)), keep = (i odd ? h >> 16 : h & 0xffff) >= thr16,
//   thr16 = round(p * 65536) (P(drop) within 8e-6 of p).
// mix32's two 32-bit multiplies are quarter-rate VALU (16 cycles per wave64 instruction): per
// element they cost more than the rest of a GEMM epilogue's dropout, so pairs halve that.
// Deterministic and stateless, so backward regenerates the forward mask from (seed, i).
NRSE_DEV uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
NRSE_DEV uint32_t site_key(uint32_t seed) { return mix32(seed * 0x9e3779b9U + 0x632be5abU); }
__host__ __device__ inline uint32_t dropout_threshold(float p) {
  const double t = (double)p * 65536.0 + 0.5;
  return t >= 65536.0 ? 65536u : (uint32_t)t;
}
NRSE_DEV bool dropout_keep(uint32_t key, uint32_t idx, uint32_t thr16) {
  const uint32_t h = mix32((idx >> 1) ^ key);
  return ((idx & 1u) ? (h >> 16) : (h & 0xffffu)) >= thr16;
}
// keep[0..N-1] of elements idx0 .. idx0+N-1, idx0 EVEN (N even): N/2 hashes
template <int N>
NRSE_DEV void dropout_keep_run(uint32_t key, uint32_t idx0, uint32_t thr16, bool (&keep)[N]) {
  static_assert(N % 2 == 0, "pairs");
#pragma unroll
  for (int j = 0; j < N / 2; ++j) {
    const uint32_t h = mix32(((idx0 >> 1) + (uint32_t)j) ^ key);
    keep[2 * j] = (h & 0xffffu) >= thr16;
    keep[2 * j + 1] = (h >> 16) >= thr16;
  }
}
// o[e] = keep(idx0 + e) ? o[e] * sc : 0 -- pairs when idx0 is even (every vector site of the
// step: row strides and column groups are even), per element otherwise
template <int N>
NRSE_DEV void dropout_apply(uint32_t key, uint32_t idx0, uint32_t thr16, float sc, float (&o)[N]) {
  if constexpr (N % 2 == 0) {
    if (!(idx0 & 1u)) {
      bool k[N];
      dropout_keep_run<N>(key, idx0, thr16, k);
#pragma unroll
      for (int e = 0; e < N; ++e) o[e] = k[e] ? o[e] * sc : 0.f;
      return;
    }
  }
#pragma unroll
  for (int e = 0; e < N; ++e) o[e] = dropout_keep(key, idx0 + (uint32_t)e, thr16) ? o[e] * sc : 0.f;
}

// Attention-probability dropout (the [B, H, T, T] site, the largest): one mixer hash per PAIR of
// keys of a query row, 16 bits per element, so the two 32-bit multiplies of mix32 (quarter-rate
// VALU) are paid once per two elements. Element (row, k), row = (b*H + h)*T + q:
//   hash = attn_mix((row * ((T + 1) / 2) + k / 2) ^ key), half = k odd ? hash >> 16 : hash & 0xffff,
//   keep = half >= thr16, thr16 = round(p * 65536) (P(drop) within 8e-6 of p).
__host__ __device__ inline uint32_t dropout_threshold16(float p) {
  const double t = (double)p * 65536.0 + 0.5;
  return t >= 65536.0 ? 65536u : (uint32_t)t;
}
// ABI 10: the pair hash is attn_mix, a mixer of full-rate VALU only -- two 24-bit multiplies
// (v_mul_u32_u24) between xor-shifts that fold every input bit into the multiplied 24 (6 issue
// slots against mix32's ~12: its two 32-bit multiplies are quarter-rate); the attention forward
// hashes 8 pairs per lane and key tile, about a third of its vector work. Drop rate and pair /
// neighbour / row independence match mix32's (tests/test_hostside.py, oracle/masks.py attn_mix).
// NRSE_ATTN_MIX32=1 builds the former mix32 form (timing A/B only: the oracle replays attn_mix).
NRSE_DEV uint32_t attn_mix(uint32_t x) {
#if NRSE_ATTN_MIX32
  return mix32(x);
#else
  x ^= x >> 16;
  x = (x & 0xffffffu) * 0xebca6bu;
  x ^= x >> 13;
  x = (x & 0xffffffu) * 0xb2ae35u;
  x ^= x >> 16;
  return x;
#endif
}
NRSE_DEV uint32_t attn_pair_hash(uint32_t key, uint32_t row, uint32_t tp2, int k) {
  return attn_mix((row * tp2 + (uint32_t)(k >> 1)) ^ key);
}
NRSE_DEV bool attn_half_keep(uint32_t hash, int odd, uint32_t thr16) {
  return (odd ? (hash >> 16) : (hash & 0xffffu)) >= thr16;
}
NRSE_DEV bool attn_keep(uint32_t key, uint32_t row, uint32_t tp2, int k, uint32_t thr16) {
  return attn_half_keep(attn_pair_hash(key, row, tp2, k), k & 1, thr16);
}

// n / d for n < 2^31 and a runtime d >= 1 as one multiply-high (round-up form of Granlund and
// Montgomery): l = ceil(log2 d), m = ceil(2^(31+l) / d) < 2^32, and (n * m) >> (31 + l) = n / d
// exactly for every n < 2^31 (m d - 2^(31+l) < d <= 2^l). A row -> (utterance, frame) split as a
// software 64-bit divide on the scalar unit cost ~180 SALU instructions per row and wave in the
// conv0 backward (PMC); set up once per kernel, this is a few scalar ops per use.
struct UDiv31 {
  unsigned m;
  int sh;
  NRSE_DEV void init(unsigned d) {
    int l = 0;
    while ((1u << l) < d) ++l;
    sh = 31 + l;
    m = (unsigned)(((1ull << sh) + d - 1) / d);
  }
  NRSE_DEV unsigned div(unsigned n) const { return (unsigned)(((unsigned long long)n * m) >> sh); }
};

// Wave-wide reductions (wave64).
// Butterfly steps across the 16-lane rows of a wave64 with the gfx950 row-swap VALU ops instead
// of ds_bpermute (no LDS round trip, no lane-address arithmetic): v_permlane16_swap exchanges rows
// 1, 3 of its first operand with rows 0, 2 of its second, so with both operands = v every lane
// gets {own, lane ^ 16} in some order; permlane32_swap likewise for lane ^ 32. max / + of the two
// are order-independent (bitwise equal to the __shfl_xor form).
NRSE_DEV float xor16_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
NRSE_DEV float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
NRSE_DEV float xor16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
NRSE_DEV float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

NRSE_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// DPP all-reduce: quad swaps, half-row and row mirrors give every lane its 16-lane row sum, two
// row broadcasts accumulate the rows into lane 63, readlane makes it wave-uniform (no LDS
// crossbar traffic, unlike the ds_bpermute butterfly above; conv0 fwd / bwd 6-8 % faster). A
// different summation order than wave_sum, so it is used where the order was chosen with it.
NRSE_DEV float wave_sum_dpp(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x143, 0xC, 0xF, false));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
NRSE_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
NRSE_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Error reporting shared by the C-ABI translation units.
void nrse_set_error(const char* fmt, ...);
int nrse_check_launch(const char* what);

#define NRSE_REQUIRE(cond, ...)              \
  do {                                       \
    if (!(cond)) {                           \
      nrse_set_error(__VA_ARGS__);           \
      return NRSE_ERR_ARG;                   \
    }                                        \
  } while (0)

// ABI 10 handshake: a params struct whose struct_size is not this build's sizeof is refused before
// any other field is read (a caller compiled against another nrse_hip.h passes a shorter or longer
// struct). RET is the entry point's error value (NRSE_ERR_ARG for both int and long long returns).
#define NRSE_CHECK_PARAMS(p, fn)                                                                        \
  do {                                                                                                \
    if (!(p)) {                                                                                       \
      nrse_set_error("%s: null params", fn);                                                          \
      return NRSE_ERR_ARG;                                                                            \
    }                                                                                                 \
    if ((p)->struct_size != (uint32_t)sizeof(*(p))) {                                                 \
      nrse_set_error("%s: struct_size %u, this library's is %u (caller built against another "        \
                     "nrse_hip.h; library ABI %d)", fn, (unsigned)(p)->struct_size,                   \
                     (unsigned)sizeof(*(p)), NRSE_ABI_VERSION);                                       \
      return NRSE_ERR_ARG;                                                                            \
    }                                                                                                 \
  } while (0)

static inline int nrse_cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
