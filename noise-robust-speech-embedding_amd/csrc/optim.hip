// Optimiser tail over the flat f32 buffers (HBM-bound, float4 per lane):
//   clip_grad_norm_(max_norm=1.0)   train_byol.py:67  (sum of squares in f64: a single f32
//                                   reduction over 3.3e8 entries loses the small ones)
//   AdamW.step (decoupled wd)       train_byol.py:68, torch.optim.AdamW semantics
//   target EMA                      src/models/byol.py:62-73
//   health checks                   train_byol.py:52-59, src/utils/debugging_utils.py:4-30
// The clip coefficient is read from device memory by the AdamW kernel: no host sync.
#include "common.h"

namespace {

// bf16 shadow of 4 consecutive f32 values at float4 index q; with lo (the split-weight mode), also
// the residual plane lo = bf16(x - hi), so hi + lo carries the f32 weight to ~2^-17 relative
NRSE_DEV void store_bf16x4(void* hi, void* lo, long long q, const float* x) {
  uint2 u;
  u.x = (uint32_t)f2bf(x[0]) | ((uint32_t)f2bf(x[1]) << 16);
  u.y = (uint32_t)f2bf(x[2]) | ((uint32_t)f2bf(x[3]) << 16);
  reinterpret_cast<uint2*>(hi)[q] = u;
  if (lo) {
    uint2 w;
    w.x = (uint32_t)f2bf(x[0] - __uint_as_float(u.x << 16)) | ((uint32_t)f2bf(x[1] - __uint_as_float(u.x & 0xffff0000u)) << 16);
    w.y = (uint32_t)f2bf(x[2] - __uint_as_float(u.y << 16)) | ((uint32_t)f2bf(x[3] - __uint_as_float(u.y & 0xffff0000u)) << 16);
    reinterpret_cast<uint2*>(lo)[q] = w;
  }
}

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, long long n, double* __restrict__ out,
                                                    double* __restrict__ part) {
  __shared__ double red[4];
  double a = 0.0;
  const long long n4 = n / 4;
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < n4; q += (long long)gridDim.x * 256) {
    const float4 v = reinterpret_cast<const float4*>(x)[q];
    a += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    a += (double)x[i] * x[i];
  a = wave_sum_d(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double s = red[0] + red[1] + red[2] + red[3];
    if (part) part[blockIdx.x] = s;  // added in block order by sum_parts_kernel
    else atomicAdd(out, s);
  }
}

// out += sum_b part[b], b < nb, in a fixed order (per-lane strided sums, then fixed trees)
__global__ __launch_bounds__(256) void sum_parts_kernel(const double* __restrict__ part, int nb,
                                                        double* __restrict__ out) {
  __shared__ double red[4];
  double a = 0.0;
  for (int b = threadIdx.x; b < nb; b += 256) a += part[b];
  a = wave_sum_d(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) *out += red[0] + red[1] + red[2] + red[3];
}

// t' = decay t + (1 - decay) o with one explicit rounding order at every EMA site (ema_kernel and
// the fused form in adamw_kernel), so the two forms agree bit for bit whatever the contraction
NRSE_DEV float ema_mix(float t, float o, float decay, float om) { return fmaf(decay, t, om * o); }

// ABI 10: whether flat index sat_offset + i lies in one of the counted ranges (the saturating path
// only: a binary search over the sorted [start, end) pairs)
NRSE_DEV bool sat_member(const nrse_adamw_params& p, long long i) {
  if (!p.sat_ranges) return true;
  const long long gi = p.sat_offset + i;
  int lo = 0, hi = p.sat_nranges;   // first range whose end > gi
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (p.sat_ranges[2 * mid + 1] <= gi) lo = mid + 1;
    else hi = mid;
  }
  return lo < p.sat_nranges && p.sat_ranges[2 * lo] <= gi;
}
// the counted saturations among 4 elements from index i0 (bit e of m: element i0 + e saturated)
NRSE_DEV int sat_members4(const nrse_adamw_params& p, long long i0, unsigned m) {
  int c = 0;
  for (int e = 0; e < 4; ++e)
    if ((m >> e) & 1u) c += sat_member(p, i0 + e) ? 1 : 0;
  return c;
}

// one element of the fused target EMA (nrse_adamw_params.ema_t), as ema_kernel's scalar tail
NRSE_DEV void ema_one(const nrse_adamw_params& p, long long i, float pn, float eom, float sc8, int& ns) {
  const float t = ema_mix(p.ema_t[i], pn, p.ema_decay, eom);
  p.ema_t[i] = t;
  if (p.ema_shadow) store_from_f(p.ema_shadow, p.ema_shadow_dtype, i, t);
  if (p.ema_shadow_lo) ((bf16_t*)p.ema_shadow_lo)[i] = bf16_lo(t);
  if (p.ema_shadow_lo8) {
    const float l = lo_resid(t) * sc8;
    ((unsigned char*)p.ema_shadow_lo8)[i] = fp8_1(l);
    if (fabsf(l) > 448.f) ns += sat_member(p, i) ? 1 : 0;
  }
}

// the fp8 correction plane of 4 consecutive weights at float4 index q (ABI 6)
NRSE_DEV void store_lo8x4(const nrse_adamw_params& p, void* lo8, long long q, const float* x, float sc8, int& ns) {
  const float a = lo_resid(x[0]) * sc8, b = lo_resid(x[1]) * sc8, c = lo_resid(x[2]) * sc8, d = lo_resid(x[3]) * sc8;
  reinterpret_cast<uint32_t*>(lo8)[q] = fp8x4(a, b, c, d);
  const unsigned m = (fabsf(a) > 448.f ? 1u : 0u) | (fabsf(b) > 448.f ? 2u : 0u) | (fabsf(c) > 448.f ? 4u : 0u) |
                     (fabsf(d) > 448.f ? 8u : 0u);
  if (m) ns += sat_members4(p, 4 * q, m);
}

__global__ __launch_bounds__(256) void adamw_kernel(const nrse_adamw_params p) {
  const double ss = p.sumsq ? *p.sumsq : 0.0;
  float coef = 1.f;
  if (p.sumsq) {
    // sumsq is over the (possibly summed-over-ranks) gradient; the clipped gradient is
    // grad_scale * g (the rank average), whose norm is grad_scale * sqrt(sumsq).
    const float tn = (float)sqrt(ss) * p.grad_scale;
    coef = fminf(1.f, p.max_norm / (tn + 1e-6f));
  }
  coef *= p.grad_scale;
  const float bc1 = 1.f - powf(p.beta1, (float)p.step);
  const float bc2 = 1.f - powf(p.beta2, (float)p.step);
  const float step_size = p.lr / bc1;
  const float bc2s = sqrtf(bc2);
  const float decay = 1.f - p.lr * p.weight_decay;
  const long long n4 = p.n / 4;
  const long long e4 = p.ema_n / 4;  // whole quads of the fused EMA range
  const float eom = 1.f - p.ema_decay;
  const float sc8 = ldexpf(1.f, p.lo8_exp);
  const bool ema4 = p.ema_t && e4 > 0;  // uniform: a whole EMA quad exists to load
  int ns = 0;                           // saturated fp8 corrections (ABI 10 sat_count)
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < n4; q += (long long)gridDim.x * 256) {
    // the five operand quads issued together: the target's quad (from a clamped index past the
    // EMA range) before the stores below, which may alias it and would otherwise order its load
    // after them as a second memory round trip per iteration
    float4 pv = reinterpret_cast<float4*>(p.p)[q];
    const float4 gv = reinterpret_cast<const float4*>(p.g)[q];
    float4 mv = reinterpret_cast<float4*>(p.m)[q];
    float4 vv = reinterpret_cast<float4*>(p.v)[q];
    float4 tv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ema4) tv = reinterpret_cast<const float4*>(p.ema_t)[q < e4 ? q : 0];
    // zero_grad: the gradient buffer is cleared for the next step's accumulation by this pass
    if (p.zero_grad) reinterpret_cast<float4*>(const_cast<float*>(p.g))[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    float* pa = &pv.x; const float* ga = &gv.x; float* ma = &mv.x; float* va = &vv.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float g = ga[e] * coef;
      float w = pa[e] * decay;
      ma[e] = p.beta1 * ma[e] + (1.f - p.beta1) * g;
      va[e] = p.beta2 * va[e] + (1.f - p.beta2) * g * g;
      const float denom = sqrtf(va[e]) / bc2s + p.eps;
      pa[e] = w - step_size * ma[e] / denom;
    }
    reinterpret_cast<float4*>(p.p)[q] = pv;
    reinterpret_cast<float4*>(p.m)[q] = mv;
    reinterpret_cast<float4*>(p.v)[q] = vv;
    if (p.p_shadow) {
      if (p.shadow_dtype == NRSE_BF16) {
        store_bf16x4(p.p_shadow, p.p_shadow_lo, q, pa);
      } else {
        reinterpret_cast<float4*>(p.p_shadow)[q] = pv;
      }
    }
    if (p.p_shadow_lo8) store_lo8x4(p, p.p_shadow_lo8, q, pa, sc8, ns);
    if (p.ema_t) {
      if (q < e4) {
        tv.x = ema_mix(tv.x, pv.x, p.ema_decay, eom); tv.y = ema_mix(tv.y, pv.y, p.ema_decay, eom);
        tv.z = ema_mix(tv.z, pv.z, p.ema_decay, eom); tv.w = ema_mix(tv.w, pv.w, p.ema_decay, eom);
        reinterpret_cast<float4*>(p.ema_t)[q] = tv;
        if (p.ema_shadow) {
          if (p.ema_shadow_dtype == NRSE_BF16) store_bf16x4(p.ema_shadow, p.ema_shadow_lo, q, &tv.x);
          else reinterpret_cast<float4*>(p.ema_shadow)[q] = tv;
        }
        if (p.ema_shadow_lo8) store_lo8x4(p, p.ema_shadow_lo8, q, &tv.x, sc8, ns);
      } else if (q == e4) {
        // the quad holding the EMA range's end: its first ema_n - 4 q elements, from this thread's
        // updated registers
#pragma unroll
        for (int e = 0; e < 3; ++e)
          if (4 * q + e < p.ema_n) ema_one(p, 4 * q + e, pa[e], eom, sc8, ns);
      }
    }
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * 256 + threadIdx.x; i < p.n; i += (long long)gridDim.x * 256) {
    const float g = p.g[i] * coef;
    if (p.zero_grad) const_cast<float*>(p.g)[i] = 0.f;
    const float w = p.p[i] * decay;
    p.m[i] = p.beta1 * p.m[i] + (1.f - p.beta1) * g;
    p.v[i] = p.beta2 * p.v[i] + (1.f - p.beta2) * g * g;
    const float denom = sqrtf(p.v[i]) / bc2s + p.eps;
    p.p[i] = w - step_size * p.m[i] / denom;
    if (p.p_shadow) store_from_f(p.p_shadow, p.shadow_dtype, i, p.p[i]);
    if (p.p_shadow_lo) ((bf16_t*)p.p_shadow_lo)[i] = bf16_lo(p.p[i]);
    if (p.p_shadow_lo8) {
      const float l = lo_resid(p.p[i]) * sc8;
      ((unsigned char*)p.p_shadow_lo8)[i] = fp8_1(l);
      if (fabsf(l) > 448.f) ns += sat_member(p, i) ? 1 : 0;
    }
    if (p.ema_t && i < p.ema_n) ema_one(p, i, p.p[i], eom, sc8, ns);
  }
  sat_count_add(p.sat_count, ns);
}

__global__ __launch_bounds__(256) void ema_kernel(float* __restrict__ t, const float* __restrict__ o,
                                                  void* __restrict__ ts, int sdt, long long n, float decay,
                                                  void* __restrict__ tlo) {
  const float om = 1.f - decay;
  const long long n4 = n / 4;
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < n4; q += (long long)gridDim.x * 256) {
    float4 tv = reinterpret_cast<float4*>(t)[q];
    const float4 ov = reinterpret_cast<const float4*>(o)[q];
    tv.x = ema_mix(tv.x, ov.x, decay, om); tv.y = ema_mix(tv.y, ov.y, decay, om);
    tv.z = ema_mix(tv.z, ov.z, decay, om); tv.w = ema_mix(tv.w, ov.w, decay, om);
    reinterpret_cast<float4*>(t)[q] = tv;
    if (ts) {
      if (sdt == NRSE_BF16) {
        store_bf16x4(ts, tlo, q, &tv.x);
      } else {
        reinterpret_cast<float4*>(ts)[q] = tv;
      }
    }
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    t[i] = ema_mix(t[i], o[i], decay, om);
    if (ts) store_from_f(ts, sdt, i, t[i]);
    if (tlo) ((bf16_t*)tlo)[i] = bf16_lo(t[i]);
  }
}

__global__ __launch_bounds__(256) void health_kernel(const void* __restrict__ x, int dt, long long n,
                                                     float* __restrict__ stats) {
  __shared__ float red[3][4];
  float nan = 0.f, inf = 0.f, sabs = 0.f, mabs = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float v = load_as_f(x, dt, i);
    if (isnan(v)) nan += 1.f;
    else if (isinf(v)) inf += 1.f;
    else { sabs += fabsf(v); mabs = fmaxf(mabs, fabsf(v)); }
  }
  nan = wave_sum(nan); inf = wave_sum(inf); sabs = wave_sum(sabs); mabs = wave_max(mabs);
  const int w = threadIdx.x >> 6;
  __shared__ float rmax[4];
  if ((threadIdx.x & 63) == 0) { red[0][w] = nan; red[1][w] = inf; red[2][w] = sabs; rmax[w] = mabs; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float a = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const float b = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    const float c = red[2][0] + red[2][1] + red[2][2] + red[2][3];
    const float m = fmaxf(fmaxf(rmax[0], rmax[1]), fmaxf(rmax[2], rmax[3]));
    if (a != 0.f) atomicAdd(stats + 0, a);
    if (b != 0.f) atomicAdd(stats + 1, b);
    atomicAdd(stats + 2, c);
    atomicMax(reinterpret_cast<int*>(stats + 3), __float_as_int(m));  // non-negative floats order as ints
  }
}

int grid_for(long long n) {
  long long b = (n / 4 + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" int nrse_sumsq(const float* x, long long n, double* out, double* part, void* stream) {
  NRSE_REQUIRE(x && out && n >= 0, "nrse_sumsq: bad args");
  NRSE_REQUIRE(((uintptr_t)x & 15) == 0, "nrse_sumsq: x must be 16-byte aligned");
  if (n == 0) return NRSE_OK;
  const int nb = (int)grid_for(n);
  hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, x, n, out, part);
  if (part) hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, part, nb, out);
  return nrse_check_launch("nrse_sumsq");
}

extern "C" int nrse_adamw(const nrse_adamw_params* p, void* stream) {
  NRSE_CHECK_PARAMS(p, "nrse_adamw");
  NRSE_REQUIRE(p && p->p && p->g && p->m && p->v && p->n >= 0 && p->step >= 1, "nrse_adamw: bad args");
  NRSE_REQUIRE((((uintptr_t)p->p | (uintptr_t)p->g | (uintptr_t)p->m | (uintptr_t)p->v) & 15) == 0,
               "nrse_adamw: buffers must be 16-byte aligned");
  NRSE_REQUIRE(!p->p_shadow_lo || (p->p_shadow && p->shadow_dtype == NRSE_BF16 && ((uintptr_t)p->p_shadow_lo & 7) == 0),
               "nrse_adamw: p_shadow_lo needs a bf16 p_shadow and 8-byte alignment");
  NRSE_REQUIRE(!p->ema_t || (p->ema_n >= 0 && p->ema_n <= p->n && ((uintptr_t)p->ema_t & 15) == 0),
               "nrse_adamw: ema_t needs ema_n <= n and 16-byte alignment");
  NRSE_REQUIRE(!p->ema_shadow_lo ||
                   (p->ema_shadow && p->ema_shadow_dtype == NRSE_BF16 && ((uintptr_t)p->ema_shadow_lo & 7) == 0),
               "nrse_adamw: ema_shadow_lo needs a bf16 ema_shadow and 8-byte alignment");
  // the shadows are written as 4-element vectors: uint2 (bf16) or float4 (f32) per quad
  auto shadow_ok = [](const void* sh, int dt) {
    return !sh || (dt == NRSE_BF16 && ((uintptr_t)sh & 7) == 0) || (dt == NRSE_F32 && ((uintptr_t)sh & 15) == 0);
  };
  NRSE_REQUIRE(shadow_ok(p->p_shadow, p->shadow_dtype),
               "nrse_adamw: p_shadow must be bf16 (8-byte aligned) or f32 (16-byte aligned)");
  NRSE_REQUIRE(!p->ema_shadow || (p->ema_t && shadow_ok(p->ema_shadow, p->ema_shadow_dtype)),
               "nrse_adamw: ema_shadow needs ema_t and must be bf16 (8-byte aligned) or f32 (16-byte aligned)");
  NRSE_REQUIRE((!p->p_shadow_lo8 && !p->ema_shadow_lo8) || (p->lo8_exp > -64 && p->lo8_exp < 64),
               "nrse_adamw: lo8_exp out of range");
  NRSE_REQUIRE(((uintptr_t)p->p_shadow_lo8 & 3) == 0 && ((uintptr_t)p->ema_shadow_lo8 & 3) == 0 &&
                   (!p->ema_shadow_lo8 || p->ema_t),
               "nrse_adamw: fp8 planes need 4-byte alignment (and ema_t for ema_shadow_lo8)");
  NRSE_REQUIRE(!p->sat_ranges || (p->sat_count && p->sat_nranges >= 0), "nrse_adamw: sat_ranges without sat_count");
  NRSE_REQUIRE(p->lo8_dtype == 0 || p->lo8_dtype == NRSE_FP8, "nrse_adamw: lo8_dtype %d (0 or NRSE_FP8)",
               p->lo8_dtype);
  if (p->n == 0) return NRSE_OK;
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(p->n)), dim3(256), 0, (hipStream_t)stream, *p);
  return nrse_check_launch("nrse_adamw");
}

extern "C" int nrse_ema(float* t, const float* o, void* ts, int sdt, long long n, float decay, void* ts_lo,
                        void* stream) {
  NRSE_REQUIRE(t && o && n >= 0, "nrse_ema: bad args");
  NRSE_REQUIRE((((uintptr_t)t | (uintptr_t)o) & 15) == 0, "nrse_ema: buffers must be 16-byte aligned");
  NRSE_REQUIRE(!ts_lo || (ts && sdt == NRSE_BF16 && ((uintptr_t)ts_lo & 7) == 0),
               "nrse_ema: t_shadow_lo needs a bf16 t_shadow and 8-byte alignment");
  if (n == 0) return NRSE_OK;
  hipLaunchKernelGGL(ema_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, t, o, ts, sdt, n, decay, ts_lo);
  return nrse_check_launch("nrse_ema");
}

extern "C" int nrse_health(const void* x, int dt, long long n, float* stats, void* stream) {
  NRSE_REQUIRE(x && stats && n >= 0, "nrse_health: bad args");
  if (n == 0) return NRSE_OK;
  long long b = (n + 255) / 256;
  if (b > 1024) b = 1024;
  hipLaunchKernelGGL(health_kernel, dim3((int)b), dim3(256), 0, (hipStream_t)stream, x, dt, n, stats);
  return nrse_check_launch("nrse_health");
}
