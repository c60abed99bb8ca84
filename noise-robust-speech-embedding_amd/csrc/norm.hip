// Row LayerNorm kernels (one wave64 per row, fp32 statistics by wave shuffles).
//   conv LN+GELU      [TF]modeling_wavlm.py:712-720
//   feature-proj LN   [TF]modeling_wavlm.py:101
//   encoder LNs       [TF]modeling_wavlm.py:357, 369, 513 (+ time-mean shim)
// Memory-bound: each lane moves 4-element vectors (8 B bf16 / 16 B f32) so one wave
// instruction covers 512 B - 1 KiB of a row; gamma/beta grads are accumulated per lane across
// the rows a wave visits (grid-stride), reduced across the block in LDS, then one f32 atomic
// per column per block.
#include <cstdlib>
#include "common.h"

namespace {

constexpr int CH = 4;  // elements per lane-vector

template <typename T> struct V4;
template <> struct V4<float> {
  static NRSE_DEV void load(const float* p, float* o) {
    float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  static NRSE_DEV void store(float* p, const float* o) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  }
};
template <> struct V4<bf16_t> {
  static NRSE_DEV void load(const bf16_t* p, float* o) {
    uint2 v = *reinterpret_cast<const uint2*>(p);
    o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
    o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
  }
  static NRSE_DEV void store(bf16_t* p, const float* o) {
    uint2 v;
    v.x = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
    v.y = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
    *reinterpret_cast<uint2*>(p) = v;
  }
};

NRSE_DEV void load4(const void* p, int dt, long long i, float* o) {
  if (dt == NRSE_BF16) V4<bf16_t>::load((const bf16_t*)p + i, o);
  else V4<float>::load((const float*)p + i, o);
}
NRSE_DEV void store4(void* p, int dt, long long i, const float* o) {
  if (dt == NRSE_BF16) V4<bf16_t>::store((bf16_t*)p + i, o);
  else V4<float>::store((float*)p + i, o);
}

NRSE_DEV void unpack_bf4(uint2 v, float* o) {
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
}

// the fp8 copies of 4 outputs at element i: fp8(bf16 o) (ABI 6), or the split planes (ABI 7)
NRSE_DEV void store_y8(const nrse_ln_fwd_params& p, long long i, const float* o) {
  unsigned char* y8 = (unsigned char*)p.y8 + i;
  if (p.y8_split) {
    uint32_t lo, hi;
    int ns = 0;
    fp8x4_split(o, __builtin_ldexpf(1.f, p.y8_exp), lo, hi, &ns);
    *reinterpret_cast<uint32_t*>(y8) = lo;
    *reinterpret_cast<uint32_t*>(y8 + p.rows * p.C) = hi;
    sat_count_add(p.sat_count, ns);
  } else {
    *reinterpret_cast<uint32_t*>(y8) = fp8x4_of_bf(o);
    // (|bf16 o| > 448 iff |o| >= 448 + half a bf16 ulp: the stored value decides)
    sat_count_add(p.sat_count, fp8_nsat4(bf2f(f2bf(o[0])), bf2f(f2bf(o[1])), bf2f(f2bf(o[2])), bf2f(f2bf(o[3]))));
  }
}

// element c of a row held by this lane: c = (k*64 + lane)*4 + e, k < NK = C/256
template <int NK>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const nrse_ln_fwd_params p) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row >= p.rows) return;
  const int C = p.C;
  float v[NK][CH];
  const long long base = row * C;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    load4(p.x, p.x_dtype, base + (k * 64 + lane) * CH, v[k]);
#pragma unroll
    for (int e = 0; e < CH; ++e) s += v[k][e];
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < CH; ++e) { const float d = v[k][e] - mean; q += d * d; }
  const float rstd = rsqrtf(wave_sum(q) / C + p.eps);
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c0 = (k * 64 + lane) * CH;
    float4 g = *reinterpret_cast<const float4*>(p.gamma + c0);
    float4 b = *reinterpret_cast<const float4*>(p.beta + c0);
    float o[CH] = {(v[k][0] - mean) * rstd * g.x + b.x, (v[k][1] - mean) * rstd * g.y + b.y,
                   (v[k][2] - mean) * rstd * g.z + b.z, (v[k][3] - mean) * rstd * g.w + b.w};
    if (p.flags & NRSE_LN_GELU) {
#pragma unroll
      for (int e = 0; e < CH; ++e) o[e] = gelu_f(o[e]);
    } else if (p.flags & NRSE_LN_RELU) {
#pragma unroll
      for (int e = 0; e < CH; ++e) o[e] = fmaxf(o[e], 0.f);
    }
    store4_out(p.y, p.y_dtype, base + c0, p.rows * C, o);
    if (p.y8) store_y8(p, base + c0, o);
  }
  if (lane == 0) {
    if (p.mean) p.mean[row] = mean;
    if (p.rstd) p.rstd[row] = rstd;
  }
}

// f32-in form (the encoder LNs: x is the f32 residual stream): the row's four 16-B words and
// the lane's gamma / beta issued together, unconditionally, before the reductions. The generic
// kernel's runtime dtype branch per word made the compiler wait for each load before issuing
// the next (four serial round trips per row).
template <int NK>
__global__ __launch_bounds__(256) void ln_fwd_f32_kernel(const nrse_ln_fwd_params p) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row >= p.rows) return;
  const int C = p.C;
  const float* xr = (const float*)p.x + row * C;
  float4 xv[NK], gv[NK], bv[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) xv[k] = *reinterpret_cast<const float4*>(xr + (k * 64 + lane) * CH);
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    gv[k] = *reinterpret_cast<const float4*>(p.gamma + (k * 64 + lane) * CH);
    bv[k] = *reinterpret_cast<const float4*>(p.beta + (k * 64 + lane) * CH);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) s += (xv[k].x + xv[k].y) + (xv[k].z + xv[k].w);
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const float d0 = xv[k].x - mean, d1 = xv[k].y - mean, d2 = xv[k].z - mean, d3 = xv[k].w - mean;
    q += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
  }
  const float rstd = rsqrtf(wave_sum(q) / C + p.eps);
  const long long base = row * C;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c0 = (k * 64 + lane) * CH;
    float o[CH] = {(xv[k].x - mean) * rstd * gv[k].x + bv[k].x, (xv[k].y - mean) * rstd * gv[k].y + bv[k].y,
                   (xv[k].z - mean) * rstd * gv[k].z + bv[k].z, (xv[k].w - mean) * rstd * gv[k].w + bv[k].w};
    if (p.flags & NRSE_LN_GELU) {
#pragma unroll
      for (int e = 0; e < CH; ++e) o[e] = gelu_f(o[e]);
    } else if (p.flags & NRSE_LN_RELU) {
#pragma unroll
      for (int e = 0; e < CH; ++e) o[e] = fmaxf(o[e], 0.f);
    }
    store4_out(p.y, p.y_dtype, base + c0, p.rows * C, o);
    if (p.y8) store_y8(p, base + c0, o);
  }
  if (lane == 0) {
    if (p.mean) p.mean[row] = mean;
    if (p.rstd) p.rstd[row] = rstd;
  }
}

// bf16-in form of the forward for the long row sweeps of the conv stack (x bf16, C <= 512):
// each wave takes RPW rows, all of their raw 8-byte words loaded first (clamped rows, no
// branches), so RPW KiB are in flight per wave instead of one row's 1 KiB
template <int NK, int RPW>
__global__ __launch_bounds__(256) void ln_fwd_bf16_kernel(const nrse_ln_fwd_params p) {
  const int lane = threadIdx.x & 63;
  const long long row0 = ((long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * RPW;
  if (row0 >= p.rows) return;
  const int C = p.C;
  const float invC = 1.f / C;
  uint2 raw[RPW][NK];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const long long row = min(row0 + r, p.rows - 1);
#pragma unroll
    for (int k = 0; k < NK; ++k)
      raw[r][k] = ldg(reinterpret_cast<const uint2*>((const bf16_t*)p.x + row * C + (k * 64 + lane) * CH));
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const long long row = row0 + r;
    float v[NK][CH];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      unpack_bf4(raw[r][k], v[k]);
#pragma unroll
      for (int e = 0; e < CH; ++e) s += v[k][e];
    }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int e = 0; e < CH; ++e) { const float d = v[k][e] - mean; q += d * d; }
    const float rstd = rsqrtf(wave_sum(q) / C + p.eps);
    (void)invC;
    if (row >= p.rows) break;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c0 = (k * 64 + lane) * CH;
      float4 g = *reinterpret_cast<const float4*>(p.gamma + c0);
      float4 b = *reinterpret_cast<const float4*>(p.beta + c0);
      float o[CH] = {(v[k][0] - mean) * rstd * g.x + b.x, (v[k][1] - mean) * rstd * g.y + b.y,
                     (v[k][2] - mean) * rstd * g.z + b.z, (v[k][3] - mean) * rstd * g.w + b.w};
      if (p.flags & NRSE_LN_GELU) {
#pragma unroll
        for (int e = 0; e < CH; ++e) o[e] = gelu_f(o[e]);
      } else if (p.flags & NRSE_LN_RELU) {
#pragma unroll
        for (int e = 0; e < CH; ++e) o[e] = fmaxf(o[e], 0.f);
      }
      store4_out(p.y, p.y_dtype, row * C + c0, p.rows * C, o);
    }
    if (lane == 0) {
      if (p.mean) p.mean[row] = mean;
      if (p.rstd) p.rstd[row] = rstd;
    }
  }
}

NRSE_DEV float load_dy(const nrse_ln_bwd_params& p, long long row, int c, float* o) {
  // fills o[0..3] = dy[row, c..c+3]
  if (p.dy_mode == NRSE_DY_DIRECT) {
    load4(p.dy, p.dy_dtype, row * p.C + c, o);
  } else if (p.dy_mode == NRSE_DY_BCAST) {
    const long long b = row / p.bcast_t;
    load4(p.dy, p.dy_dtype, b * p.C + c, o);
#pragma unroll
    for (int e = 0; e < CH; ++e) o[e] *= p.dy_scale;
  } else {
    const long long b = row / p.col_tin;
    const int tau = (int)(row - b * p.col_tin);
    o[0] = o[1] = o[2] = o[3] = 0.f;
    const long long kc = (long long)p.col_k * p.C;
    for (int j = 0; j < p.col_k; ++j) {
      const int d = tau - j;
      if (d < 0 || (d % p.col_s) != 0) continue;
      const int t = d / p.col_s;
      if (t >= p.col_tout) continue;
      float w[CH];
      load4(p.dy, p.dy_dtype, (b * p.col_tout + t) * kc + (long long)j * p.C + c, w);
#pragma unroll
      for (int e = 0; e < CH; ++e) o[e] += w[e];
    }
  }
  return 0.f;
}

// LayerNorm backward, one wave per row, grid-stride over rows with the next row's operands
// (x, dy, residual, mean, rstd) loaded while the current row is reduced, so each wave keeps two
// rows of loads in flight. Optional fused consumer (the residual branch's dropout backward that
// feeds the next GEMM, misc.hip dropout_cast_colsum): dv = dropout(dx) cast to dv_dtype and
// dv_colsum[c] += sum_r dv[r, c], with the same counter-hash mask (element index r*C + c), so dx
// is not read back. gamma / beta / dv column sums: per-lane accumulators across the rows of a
// wave, reduced over the block's 4 waves in one 16 KB LDS buffer, one f32 atomic per column and
// block.
// COL: col2im dy with at most two taps per row (k <= 2s, every conv layer of the feature
// encoder): both taps are loaded into their own registers and summed in compute().
// BF: x and dy are bf16 (the bf16 conv / feature-projection LNs): the row keeps the raw 8-byte
// words and compute() unpacks them, so no unpack (and no wait for the load) sits between the
// prefetch of the next row and its use; converting at load time put an s_waitcnt vmcnt(0)
// after every dy / x load and serialised the prefetch away.
// XF (with BF): x is f32 (the split-weight step's f32 conv pre-activations), kept as raw 16-B words
template <int NK, bool RES, bool COL, bool BF, bool XF = false>
struct LnRow {
  float x[BF ? 1 : NK][CH], dy[BF ? 1 : NK][CH], r[RES ? NK : 1][CH], dy2[COL && !BF ? NK : 1][CH];
  uint2 xr[BF && !XF ? NK : 1], dyr[BF ? NK : 1], dy2r[COL && BF ? NK : 1];
  uint4 xw[XF ? NK : 1];
  float gd[RES ? NK : 1][2];  // GT: the row's gate-path (dpa, dpb) of this lane's head per k
  float mean, rstd;
  bool v0, v1;  // BF: col2im taps present (their loads are issued regardless, from a valid address)
};


// element offsets of the (up to) two col rows feeding LN row `row` (-1: no such tap)
// (rows < 2^31, host check; the divides by multiply-high, UDiv31: set up once per kernel in cd)
struct ColDiv { UDiv31 tin, s; };
NRSE_DEV void col_taps(const nrse_ln_bwd_params& p, const ColDiv& cd, long long row, long long& o0, long long& o1) {
  const long long b = cd.tin.div((unsigned)row);
  const int tau = (int)((unsigned)row - (unsigned)b * (unsigned)p.col_tin);
  const int q = (int)cd.s.div((unsigned)tau);
  const int j0 = tau - q * p.col_s;
  long long o[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = j0 + u * p.col_s;
    const int t = q - u;  // (tau - j) / s where tau >= j (checked below)
    o[u] = (j < p.col_k && tau >= j && t < p.col_tout)
               ? ((b * p.col_tout + t) * p.col_k + j) * (long long)p.C : -1;
  }
  o0 = o[0];
  o1 = o[1];
}

// FD (encoder form, RES): x, dy and the residual all f32, dy direct: three unconditional 16-B
// loads per word, no dtype / mode branches (each of which had made the compiler wait for the load)
template <int NK, bool RES, bool COL, bool BF, bool FD, bool GT, bool XF = false>
NRSE_DEV void ln_bwd_load(const nrse_ln_bwd_params& p, const ColDiv& cd, long long row, int lane,
                          LnRow<NK, RES, COL, BF, XF>& b) {
  b.mean = p.mean[row];
  b.rstd = p.rstd[row];
  if constexpr (GT) {
    // head of channel (k * 64 + lane) * CH: 4k + lane / 16 of the row's C / 64
    const float* gp = p.gate_dp + (row * (p.C >> 6) + (lane >> 4)) * 2;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const float2 v = *reinterpret_cast<const float2*>(gp + 8 * k);
      b.gd[k][0] = v.x;
      b.gd[k][1] = v.y;
    }
  }
  if constexpr (FD) {
    const float* xr = (const float*)p.x + row * p.C;
    const float* dr = (const float*)p.dy + row * p.C;
    const float* rr = p.resid + row * p.C;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c0 = (k * 64 + lane) * CH;
      const float4 xv = *reinterpret_cast<const float4*>(xr + c0);
      const float4 dv = *reinterpret_cast<const float4*>(dr + c0);
      const float4 rv = *reinterpret_cast<const float4*>(rr + c0);
      b.x[k][0] = xv.x; b.x[k][1] = xv.y; b.x[k][2] = xv.z; b.x[k][3] = xv.w;
      b.dy[k][0] = dv.x; b.dy[k][1] = dv.y; b.dy[k][2] = dv.z; b.dy[k][3] = dv.w;
      b.r[RES ? k : 0][0] = rv.x; b.r[RES ? k : 0][1] = rv.y; b.r[RES ? k : 0][2] = rv.z; b.r[RES ? k : 0][3] = rv.w;
    }
    return;
  }
  long long o0 = -1, o1 = -1;
  if constexpr (COL) col_taps(p, cd, row, o0, o1);
  else if constexpr (BF) o0 = row * p.C;  // direct dy
  if constexpr (BF) {
    // every load is issued on every row: a load skipped on some path leaves the wait-count pass
    // no static count for the rows in flight, and it then waits for all of them
    b.v0 = o0 >= 0;
    b.v1 = o1 >= 0;
    o0 = o0 < 0 ? 0 : o0;
    o1 = o1 < 0 ? 0 : o1;
  }
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c0 = (k * 64 + lane) * CH;
    if constexpr (BF) {
      const bf16_t* dyp = (const bf16_t*)p.dy;
      if constexpr (XF) b.xw[k] = ldg(reinterpret_cast<const uint4*>((const float*)p.x + row * p.C + c0));
      else b.xr[k] = ldg(reinterpret_cast<const uint2*>((const bf16_t*)p.x + row * p.C + c0));
      b.dyr[k] = ldg(reinterpret_cast<const uint2*>(dyp + o0 + c0));
      if constexpr (COL) b.dy2r[k] = ldg(reinterpret_cast<const uint2*>(dyp + o1 + c0));
    } else {
      load4(p.x, p.x_dtype, row * p.C + c0, b.x[k]);
      if constexpr (COL) {
        if (o0 >= 0) load4(p.dy, p.dy_dtype, o0 + c0, b.dy[k]);
        else b.dy[k][0] = b.dy[k][1] = b.dy[k][2] = b.dy[k][3] = 0.f;
        if (o1 >= 0) load4(p.dy, p.dy_dtype, o1 + c0, b.dy2[k]);
        else b.dy2[k][0] = b.dy2[k][1] = b.dy2[k][2] = b.dy2[k][3] = 0.f;
      } else {
        load_dy(p, row, c0, b.dy[k]);
      }
    }
    if constexpr (RES) {
      if (p.resid) V4<float>::load(p.resid + row * p.C + c0, b.r[k]);
    }
  }
}

// RES: the encoder-layer form (residual input, fused dropout-cast consumer); !RES (conv / feature
// projection LNs) drops their registers: 137 -> fewer VGPRs, more waves for the long row sweeps
// GT (with FD): dy += the gate path's gradient, nrse_ln_bwd_params.gate_dp
template <int NK, bool RES, bool COL, bool BF, bool FD = false, bool GT = false, bool XF = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const nrse_ln_bwd_params p) {
  static_assert(!XF || BF, "XF: f32 x beside the bf16 dy words");
  static_assert(!GT || FD, "the gate term rides on the encoder form");
  constexpr bool GBL = RES && !FD;  // gamma / beta read from global memory per row
  __shared__ float red[4][NK * 64 * CH];
  // gamma / beta staged once: read per row from LDS (lgkmcnt), not global memory, whose per-row
  // loads were the youngest vmcnt entries and made every row wait for the prefetched next row
  // (the encoder form keeps global reads: hoisted LDS copies would cost it 32 VGPRs)
  __shared__ __attribute__((aligned(16))) float gb[GBL ? 1 : 2][GBL ? 4 : NK * 64 * CH];
  if constexpr (!GBL) {
    for (int c = threadIdx.x; c < p.C; c += 256) {
      gb[0][c] = p.gamma[c];
      gb[1][c] = (p.flags & (NRSE_LN_GELU | NRSE_LN_RELU)) ? p.beta[c] : 0.f;
    }
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: row math (col2im divisions) on the SALU
  const int C = p.C;
  const bool fuse = RES && p.dv != nullptr;
  // GT: the pair-summed gate weights of this lane's head dims d = 4 (lane % 16) + e (the same for
  // every k), summed in gate_bwd's order
  float gwa[CH], gwb[CH];
#pragma unroll
  for (int e = 0; e < CH; ++e) {
    gwa[e] = gwb[e] = 0.f;
    if constexpr (GT) {
      const int d = (lane & 15) * CH + e;
      gwa[e] = p.gate_w[d] + p.gate_w[64 + d] + p.gate_w[128 + d] + p.gate_w[192 + d];
      gwb[e] = p.gate_w[256 + d] + p.gate_w[320 + d] + p.gate_w[384 + d] + p.gate_w[448 + d];
    }
  }
  const uint32_t key = site_key(p.dv_seed);
  const uint32_t thr = dropout_threshold(p.dv_p);
  const float dsc = p.dv_p > 0.f ? 1.f / (1.f - p.dv_p) : 1.f;
  float dg[NK][CH], db[NK][CH], dc[RES ? NK : 1][CH];
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < CH; ++e) dg[k][e] = db[k][e] = 0.f;
#pragma unroll
  for (int k = 0; k < (RES ? NK : 1); ++k)
#pragma unroll
    for (int e = 0; e < CH; ++e) dc[k][e] = 0.f;

  auto compute = [&](const LnRow<NK, RES, COL, BF, XF>& b, long long row) {
    float xh[NK][CH], g[NK][CH];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c0 = (k * 64 + lane) * CH;
      float gam[CH], be[CH] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (GBL) {
        const float4 ga = *reinterpret_cast<const float4*>(p.gamma + c0);
        gam[0] = ga.x; gam[1] = ga.y; gam[2] = ga.z; gam[3] = ga.w;
        if (p.flags & (NRSE_LN_GELU | NRSE_LN_RELU)) {
          const float4 bb = *reinterpret_cast<const float4*>(p.beta + c0);
          be[0] = bb.x; be[1] = bb.y; be[2] = bb.z; be[3] = bb.w;
        }
      } else {
        const float4 ga = *reinterpret_cast<const float4*>(&gb[0][c0]);
        gam[0] = ga.x; gam[1] = ga.y; gam[2] = ga.z; gam[3] = ga.w;
        const float4 bb = *reinterpret_cast<const float4*>(&gb[GBL ? 0 : 1][c0]);
        be[0] = bb.x; be[1] = bb.y; be[2] = bb.z; be[3] = bb.w;
      }
      float xv[CH], dv0[CH], dv1[CH] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BF) {
        const uint2 z2 = make_uint2(0u, 0u);
        if constexpr (XF) {
          xv[0] = __uint_as_float(b.xw[k].x); xv[1] = __uint_as_float(b.xw[k].y);
          xv[2] = __uint_as_float(b.xw[k].z); xv[3] = __uint_as_float(b.xw[k].w);
        } else {
          unpack_bf4(b.xr[k], xv);
        }
        unpack_bf4(b.v0 ? b.dyr[k] : z2, dv0);
        if constexpr (COL) unpack_bf4(b.v1 ? b.dy2r[k] : z2, dv1);
      } else {
#pragma unroll
        for (int e = 0; e < CH; ++e) {
          xv[e] = b.x[k][e];
          dv0[e] = b.dy[k][e];
          if constexpr (GT) dv0[e] += b.gd[RES ? k : 0][0] * gwa[e] + b.gd[RES ? k : 0][1] * gwb[e];
          if constexpr (COL) dv1[e] = b.dy2[k][e];
        }
      }
#pragma unroll
      for (int e = 0; e < CH; ++e) {
        xh[k][e] = (xv[e] - b.mean) * b.rstd;
        float gg = dv0[e];
        if constexpr (COL) gg += dv1[e];
        if (p.flags & NRSE_LN_GELU) gg *= gelu_grad_f(xh[k][e] * gam[e] + be[e]);
        else if (p.flags & NRSE_LN_RELU) gg = (xh[k][e] * gam[e] + be[e] > 0.f) ? gg : 0.f;
        dg[k][e] += gg * xh[k][e];
        db[k][e] += gg;
        g[k][e] = gg * gam[e];
        s1 += g[k][e];
        s2 += g[k][e] * xh[k][e];
      }
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c0 = (k * 64 + lane) * CH;
      float o[CH];
#pragma unroll
      for (int e = 0; e < CH; ++e) {
        o[e] = b.rstd * (g[k][e] - s1 - xh[k][e] * s2);
        if constexpr (RES) {
          if (p.resid) o[e] += b.r[RES ? k : 0][e];
        }
      }
      store4(p.dx, p.dx_dtype, row * C + c0, o);
      if (fuse) {
        const long long i = row * C + c0;
        if (p.dv_p > 0.f) {
          dropout_apply<CH>(key, (uint32_t)i, thr, dsc, o);
        }
#pragma unroll
        for (int e = 0; e < CH; ++e) dc[RES ? k : 0][e] += o[e];
        store4(p.dv, p.dv_dtype, i, o);
      }
    }
  };

  const long long nw = (long long)gridDim.x * 4;
  long long row = (long long)blockIdx.x * 4 + w;
  ColDiv cd;
  if constexpr (COL) {
    cd.tin.init((unsigned)p.col_tin);
    cd.s.init((unsigned)p.col_s);
  }
  LnRow<NK, RES, COL, BF, XF> ba, bb;
  const long long last = p.rows - 1;
  if (row < p.rows) ln_bwd_load<NK, RES, COL, BF, FD, GT, XF>(p, cd, row, lane, ba);
  for (; row < p.rows; row += 2 * nw) {
    const long long rb = row + nw;
    // BF: unconditional (clamped) prefetch, fenced from the scheduler, which otherwise sinks the
    // loads below part of the current row's math to save registers (and then waits for them)
    if (BF || FD) {
      ln_bwd_load<NK, RES, COL, BF, FD, GT, XF>(p, cd, rb < last ? rb : last, lane, bb);
      __builtin_amdgcn_sched_barrier(0);
    } else if (rb < p.rows) {
      ln_bwd_load<NK, RES, COL, BF, FD, GT, XF>(p, cd, rb, lane, bb);
    }
    compute(ba, row);
    if (rb >= p.rows) break;
    if (BF || FD) {
      ln_bwd_load<NK, RES, COL, BF, FD, GT, XF>(p, cd, rb + nw < last ? rb + nw : last, lane, ba);
      __builtin_amdgcn_sched_barrier(0);
    } else if (rb + nw < p.rows) {
      ln_bwd_load<NK, RES, COL, BF, FD, GT, XF>(p, cd, rb + nw, lane, ba);
    }
    compute(bb, rb);
  }

  // the workgroup's column sums: into its row of the partial slab (p.part, added in workgroup
  // order by nrse_rows_reduce: deterministic), or f32 atomics into dst (no workspace)
  const int nd = (p.dgamma ? 2 : 0) + ((RES && fuse && p.dv_colsum) ? 1 : 0);
  auto reduce = [&](auto& acc, float* dst, int j) {
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int e = 0; e < CH; ++e) red[w][(k * 64 + lane) * CH + e] = acc[k][e];
    __syncthreads();
    float* prow = p.part ? p.part + ((long long)blockIdx.x * nd + j) * C : nullptr;
    for (int c = threadIdx.x; c < C; c += 256) {
      const float v = red[0][c] + red[1][c] + red[2][c] + red[3][c];
      if (prow) prow[c] = v;
      else atomicAdd(dst + c, v);
    }
    __syncthreads();
  };
  if (p.dgamma) {
    reduce(dg, p.dgamma, 0);
    reduce(db, p.dbeta, 1);
  }
  if constexpr (RES) {
    if (fuse && p.dv_colsum) reduce(dc, p.dv_colsum, p.dgamma ? 2 : 0);
  }
}

// Final LN + time-mean: grid (ceil(T / RPB), batch); 4 waves, each a row at a time.
template <int NK>
__global__ __launch_bounds__(256) void ln_mean_kernel(const float* __restrict__ h, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, float* __restrict__ emb,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      int T, int C, float eps, int rpb, float* __restrict__ part) {
  __shared__ float red[4][NK * 64 * CH];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * rpb;
  const int t1 = min(T, t0 + rpb);
  float acc[NK][CH];
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < CH; ++e) acc[k][e] = 0.f;
  for (int t = t0 + w; t < t1; t += 4) {
    const long long row = (long long)b * T + t;
    float v[NK][CH];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      V4<float>::load(h + row * C + (k * 64 + lane) * CH, v[k]);
#pragma unroll
      for (int e = 0; e < CH; ++e) s += v[k][e];
    }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int e = 0; e < CH; ++e) { const float d = v[k][e] - mean; q += d * d; }
    const float rstd = rsqrtf(wave_sum(q) / C + eps);
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c0 = (k * 64 + lane) * CH;
#pragma unroll
      for (int e = 0; e < CH; ++e) acc[k][e] += (v[k][e] - mean) * rstd * gamma[c0 + e] + beta[c0 + e];
    }
    if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
  }
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < CH; ++e) red[w][(k * 64 + lane) * CH + e] = acc[k][e];
  __syncthreads();
  const float inv = 1.0f / T;
  // partial row of this time chunk ([batch][chunk][C], added in chunk order by nrse_rows_reduce)
  // or f32 atomics (no workspace)
  float* prow = part ? part + ((long long)b * gridDim.x + blockIdx.x) * C : nullptr;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float v = (red[0][c] + red[1][c] + red[2][c] + red[3][c]) * inv;
    if (prow) prow[c] = v;
    else atomicAdd(emb + (long long)b * C + c, v);
  }
}

#define NRSE_DISPATCH_NK(KERNEL, C, GRID, ST, ARG)                                  \
  switch ((C) / 256) {                                                              \
    case 1: hipLaunchKernelGGL(KERNEL<1>, GRID, dim3(256), 0, ST, ARG); break;     \
    case 2: hipLaunchKernelGGL(KERNEL<2>, GRID, dim3(256), 0, ST, ARG); break;     \
    default: hipLaunchKernelGGL(KERNEL<4>, GRID, dim3(256), 0, ST, ARG); break;    \
  }

bool c_ok(int C) { return C == 256 || C == 512 || C == 1024; }

}  // namespace

extern "C" int nrse_layernorm_fwd(const nrse_ln_fwd_params* p, void* stream) {
  NRSE_CHECK_PARAMS(p, "nrse_layernorm_fwd");
  NRSE_REQUIRE(p && p->x && p->y && p->gamma && p->beta && p->rows > 0, "nrse_layernorm_fwd: bad args");
  if (!c_ok(p->C)) { nrse_set_error("nrse_layernorm_fwd: C=%d not in {256,512,1024}", p->C); return NRSE_ERR_UNSUPPORTED; }
  NRSE_REQUIRE(p->y_dtype == NRSE_F32 || p->y_dtype == NRSE_BF16 || p->y_dtype == NRSE_BF16X3,
               "nrse_layernorm_fwd: bad y_dtype %d", p->y_dtype);
  NRSE_REQUIRE(!p->y8 || (p->y_dtype == NRSE_BF16 && ((uintptr_t)p->y8 & 3) == 0),
               "nrse_layernorm_fwd: y8 needs a bf16 y and 4-byte alignment");
  NRSE_REQUIRE((p->y8_split == 0 || p->y8_split == 1) && p->y8_exp >= -60 && p->y8_exp <= 60,
               "nrse_layernorm_fwd: y8_split %d / y8_exp %d out of range", p->y8_split, p->y8_exp);
  NRSE_REQUIRE(!p->y8 || p->y8_dtype == 0 || p->y8_dtype == NRSE_FP8,
               "nrse_layernorm_fwd: y8_dtype %d (0 or NRSE_FP8)", p->y8_dtype);
  if (p->x_dtype == NRSE_BF16 && p->C <= 512 && ((uintptr_t)p->x & 7) == 0 && !p->y8) {
    constexpr int RPW = 4;
    const dim3 g((unsigned)((p->rows + 4 * RPW - 1) / (4 * RPW)));
    if (p->C == 512) hipLaunchKernelGGL((ln_fwd_bf16_kernel<2, RPW>), g, dim3(256), 0, (hipStream_t)stream, *p);
    else hipLaunchKernelGGL((ln_fwd_bf16_kernel<1, RPW>), g, dim3(256), 0, (hipStream_t)stream, *p);
    return nrse_check_launch("nrse_layernorm_fwd");
  }
  dim3 grid((unsigned)((p->rows + 3) / 4));
  if (p->x_dtype == NRSE_F32 && ((uintptr_t)p->x & 15) == 0) {
    NRSE_DISPATCH_NK(ln_fwd_f32_kernel, p->C, grid, (hipStream_t)stream, *p);
  } else {
    NRSE_DISPATCH_NK(ln_fwd_kernel, p->C, grid, (hipStream_t)stream, *p);
  }
  return nrse_check_launch("nrse_layernorm_fwd");
}

// grid-stride: 2 blocks per CU (8 waves, each with two rows of loads in flight) when the
// column sums are accumulated, so the per-block partial rows stay ~3 * C * 512
static long long ln_bwd_blocks(const nrse_ln_bwd_params* p) {
  long long blocks = (p->rows + 3) / 4;
  long long cap = 8192;
  if (p->dgamma || p->dv_colsum) {
    // >= 2 blocks per CU; long row sweeps (the conv layers' 4e5 rows) get up to 8 per CU
    cap = p->rows / 192;
    cap = cap < 512 ? 512 : (cap > 2048 ? 2048 : cap);
  }
  static const long long cap_env = getenv("NRSE_LN_BWD_CAP") ? atoll(getenv("NRSE_LN_BWD_CAP")) : 0;
  if (cap_env > 0) cap = cap_env;  // tuning experiments (tools/bench_ln.py)
  return blocks > cap ? cap : blocks;
}
// column-sum vectors per workgroup: dgamma, dbeta, the fused dropout consumer's colsum
static int ln_bwd_nd(const nrse_ln_bwd_params* p) { return (p->dgamma ? 2 : 0) + ((p->dv && p->dv_colsum) ? 1 : 0); }

// NRSE_LN_XF=0 keeps the generic form for f32 x with bf16 col2im dy (A/B)
static bool xf_enabled() {
  static int v = -1;
  if (v < 0) v = (getenv("NRSE_LN_XF") && atoi(getenv("NRSE_LN_XF")) == 0) ? 0 : 1;
  return v == 1;
}

extern "C" int nrse_layernorm_bwd(const nrse_ln_bwd_params* p, void* stream) {
  NRSE_CHECK_PARAMS(p, "nrse_layernorm_bwd");
  NRSE_REQUIRE(p && p->dy && p->x && p->gamma && p->mean && p->rstd && p->dx && p->rows > 0,
               "nrse_layernorm_bwd: bad args");
  NRSE_REQUIRE(!(p->flags & (NRSE_LN_GELU | NRSE_LN_RELU)) || p->beta, "nrse_layernorm_bwd: GELU/ReLU need beta");
  NRSE_REQUIRE((p->dgamma == nullptr) == (p->dbeta == nullptr), "nrse_layernorm_bwd: dgamma/dbeta together");
  NRSE_REQUIRE(p->rows < (1LL << 31), "nrse_layernorm_bwd: too many rows");
  if (p->dy_mode == NRSE_DY_COL2IM)
    NRSE_REQUIRE(p->col_k > 0 && p->col_s > 0 && p->col_tin > 0 && p->col_tout > 0 && p->rows % p->col_tin == 0,
                 "nrse_layernorm_bwd: bad col2im geometry");
  if (p->dy_mode == NRSE_DY_BCAST) NRSE_REQUIRE(p->bcast_t > 0, "nrse_layernorm_bwd: bad bcast_t");
  if (!c_ok(p->C)) { nrse_set_error("nrse_layernorm_bwd: C=%d not in {256,512,1024}", p->C); return NRSE_ERR_UNSUPPORTED; }
  NRSE_REQUIRE(!p->dv || (p->dv_dtype == NRSE_BF16 || p->dv_dtype == NRSE_F32), "nrse_layernorm_bwd: bad dv dtype");
  const long long blocks = ln_bwd_blocks(p);
  const int nd = ln_bwd_nd(p);
  NRSE_REQUIRE(!p->part || nd > 0, "nrse_layernorm_bwd: workspace given without column sums");
  const dim3 grid((unsigned)blocks);
  hipStream_t st = (hipStream_t)stream;
  const bool res = p->resid || p->dv;
  const bool col2 = !res && p->dy_mode == NRSE_DY_COL2IM && p->col_k <= 2 * p->col_s;
  // bf16 x and dy (conv / feature-projection LNs of the bf16 step), direct or two-tap col2im dy
  const bool bf = !res && p->x_dtype == NRSE_BF16 && p->dy_dtype == NRSE_BF16 &&
                  (col2 || p->dy_mode == NRSE_DY_DIRECT);
  // encoder form with every operand f32 and dy direct: the branch-free loads
  // f32 x (the split-weight step's conv pre-activations), bf16 two-tap col2im dy: the bf16 form's
  // raw-word loads with x as 16-B f32 words
  const bool xf = !res && p->x_dtype == NRSE_F32 && p->dy_dtype == NRSE_BF16 && col2 &&
                  (((uintptr_t)p->x) & 15) == 0 && xf_enabled();
  const bool fd = res && p->resid && p->x_dtype == NRSE_F32 && p->dy_dtype == NRSE_F32 &&
                  p->dy_mode == NRSE_DY_DIRECT &&
                  ((((uintptr_t)p->x) | ((uintptr_t)p->dy) | ((uintptr_t)p->resid)) & 15) == 0;
  NRSE_REQUIRE(!p->gate_dp || (fd && p->gate_w && p->C % 64 == 0 && ((uintptr_t)p->gate_dp & 7) == 0),
               "nrse_layernorm_bwd: gate_dp needs the encoder form (resid, f32 x / dy / resid, dy direct) and gate_w");
#define NRSE_LN_BWD_NK(NK)                                                                          \
  if (fd && p->gate_dp) hipLaunchKernelGGL((ln_bwd_kernel<NK, true, false, false, true, true>), grid, dim3(256), 0, st, *p); \
  else if (fd) hipLaunchKernelGGL((ln_bwd_kernel<NK, true, false, false, true>), grid, dim3(256), 0, st, *p); \
  else if (res) hipLaunchKernelGGL((ln_bwd_kernel<NK, true, false, false>), grid, dim3(256), 0, st, *p);    \
  else if (bf && col2) hipLaunchKernelGGL((ln_bwd_kernel<NK, false, true, true>), grid, dim3(256), 0, st, *p); \
  else if (xf) hipLaunchKernelGGL((ln_bwd_kernel<NK, false, true, true, false, false, true>), grid, dim3(256), 0, st, *p); \
  else if (bf) hipLaunchKernelGGL((ln_bwd_kernel<NK, false, false, true>), grid, dim3(256), 0, st, *p); \
  else if (col2) hipLaunchKernelGGL((ln_bwd_kernel<NK, false, true, false>), grid, dim3(256), 0, st, *p); \
  else hipLaunchKernelGGL((ln_bwd_kernel<NK, false, false, false>), grid, dim3(256), 0, st, *p);
  switch (p->C / 256) {
    case 1: NRSE_LN_BWD_NK(1) break;
    case 2: NRSE_LN_BWD_NK(2) break;
    default: NRSE_LN_BWD_NK(4) break;
  }
#undef NRSE_LN_BWD_NK
  const int rc = nrse_check_launch("nrse_layernorm_bwd");
  if (rc || !p->part) return rc;
  float* d[3] = {nullptr, nullptr, nullptr};
  int j = 0;
  if (p->dgamma) { d[j++] = p->dgamma; d[j++] = p->dbeta; }
  if (j < nd) d[j++] = p->dv_colsum;
  const long long C = p->C;
  return nrse_rows_reduce(d[0], C, d[1], d[1] ? C : 0, d[2], d[2] ? C : 0, p->part, (int)blocks, 1, 1, stream);
}

extern "C" long long nrse_layernorm_bwd_workspace(const nrse_ln_bwd_params* p) {
  NRSE_CHECK_PARAMS(p, "nrse_layernorm_bwd_workspace");
  if (!p || p->rows <= 0) return 0;
  return ln_bwd_blocks(p) * ln_bwd_nd(p) * (long long)p->C;
}

extern "C" int nrse_ln_mean_fwd(const float* h, const float* gamma, const float* beta, float* emb, float* mean,
                                float* rstd, int batch, int T, int C, float eps, float* part, void* stream) {
  NRSE_REQUIRE(h && gamma && beta && emb && mean && rstd && batch > 0 && T > 0, "nrse_ln_mean_fwd: bad args");
  if (!c_ok(C)) { nrse_set_error("nrse_ln_mean_fwd: C=%d unsupported", C); return NRSE_ERR_UNSUPPORTED; }
  const int rpb = 32;
  dim3 grid((T + rpb - 1) / rpb, batch);
  hipStream_t st = (hipStream_t)stream;
  switch (C / 256) {
    case 1: hipLaunchKernelGGL(ln_mean_kernel<1>, grid, dim3(256), 0, st, h, gamma, beta, emb, mean, rstd, T, C, eps, rpb, part); break;
    case 2: hipLaunchKernelGGL(ln_mean_kernel<2>, grid, dim3(256), 0, st, h, gamma, beta, emb, mean, rstd, T, C, eps, rpb, part); break;
    default: hipLaunchKernelGGL(ln_mean_kernel<4>, grid, dim3(256), 0, st, h, gamma, beta, emb, mean, rstd, T, C, eps, rpb, part); break;
  }
  const int rc = nrse_check_launch("nrse_ln_mean_fwd");
  if (rc || !part) return rc;
  return nrse_rows_reduce(emb, C, nullptr, 0, nullptr, 0, part, (int)grid.x, batch, 1, stream);
}
