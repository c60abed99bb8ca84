// Conv feature-encoder front end (conv0 + LN + GELU, fused fwd and fused bwd/wgrad) and the
// weight_norm of the grouped positional conv. Conv layers 1..6 and the pos-conv contraction run
// as implicit GEMMs in gemm.hip / gemm_dma.hip.
//   conv0         [TF]modeling_wavlm.py:712-720 (Conv1d(1, C, 10, 5, bias=False), LN, GELU)
//   weight norm   [TF]modeling_wavlm.py:61-77 (parametrizations.weight_norm, dim=2)
// conv0 has K = 10: vector-ALU work, HBM-bound on its [B*T0, C] output (the largest activation
// of the step). One wave per output row; the [k][C] weight is held in LDS (read as float4 per
// tap), lane owns 4*NQ channels.
#include <cstdlib>

#include "common.h"

namespace {

// NRSE_CONV0_MFMA=0 keeps the VALU forward for bf16 outputs too (A/B measurements)
bool conv0_mfma_on() {
  static int v = -1;
  if (v < 0) v = getenv("NRSE_CONV0_MFMA") ? atoi(getenv("NRSE_CONV0_MFMA")) : 1;
  return v != 0;
}

constexpr int KMAX = 10;

NRSE_DEV long long uniform_ll(long long v) {
  const int lo = __builtin_amdgcn_readfirstlane((int)(v & 0xffffffff));
  const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
  return ((long long)hi << 32) | (unsigned)lo;
}

// LDS weight image wT[j][c] (tap-major) so lane reads 4 consecutive channels per tap
NRSE_DEV void load_wT(float* wT, const float* w, int C, int k) {
  for (int e = threadIdx.x; e < C * KMAX; e += blockDim.x) {
    const int j = e / C, c = e % C;
    wT[e] = j < k ? w[c * k + j] : 0.f;
  }
}

// conv0 forward: VALU-bound (10-tap conv, LN, GELU per element), so channel pairs run as
// packed FP32 (v_pk_fma_f32 / v_pk_mul_f32): lane owns 4*NQ channels as 2*NQ pairs.
// K10: the model's geometry (k = KMAX = 10) as a compile-time constant -- with a runtime k every
// tap load is conditional, a branch per tap per row
template <int NQ, bool K10>
__global__ __launch_bounds__(256) void conv0_fwd_kernel(const nrse_conv0_params p) {
  __shared__ __attribute__((aligned(16))) float wT[KMAX * 512];
  const int lane = threadIdx.x & 63;
  const int C = p.C;
  load_wT(wT, p.w, C, p.k);
  __syncthreads();
  f32x2 ga[NQ][2], be[NQ][2];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = (q * 64 + lane) * 4 + 2 * h;
      ga[q][h] = f32x2{p.gamma[c], p.gamma[c + 1]};
      be[q][h] = f32x2{p.beta[c], p.beta[c + 1]};
    }
  const float invC = 1.f / C;
  const long long rows = (long long)p.batch * p.T0;
  const long long nw = (long long)gridDim.x * 4;
  UDiv31 dT0;
  dT0.init((unsigned)p.T0);
  for (long long r0 = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); r0 < rows; r0 += nw) {
    const long long row = uniform_ll(r0);
    const unsigned b = dT0.div((unsigned)row);  // rows < 2^31 (host check)
    const int t = (int)((unsigned)row - b * (unsigned)p.T0);
    const float* x = p.wav + (long long)b * p.L + (long long)t * p.s;
    float xs[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) xs[j] = (K10 || j < p.k) ? x[j] : 0.f;
    f32x2 y[NQ][2];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int c0 = (q * 64 + lane) * 4;
      y[q][0] = y[q][1] = f32x2{0.f, 0.f};
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        const float4 wv = *reinterpret_cast<const float4*>(wT + j * C + c0);
        y[q][0] = pk_fma(f32x2{wv.x, wv.y}, splat2(xs[j]), y[q][0]);
        y[q][1] = pk_fma(f32x2{wv.z, wv.w}, splat2(xs[j]), y[q][1]);
      }
    }
    f32x2 s2 = f32x2{0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NQ; ++q) s2 += y[q][0] + y[q][1];
    const float mean = wave_sum_dpp(s2.x + s2.y) * invC;
    f32x2 v2 = f32x2{0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x2 d = y[q][h] - mean;
        v2 = pk_fma(d, d, v2);
      }
    const float rstd = rsqrtf(wave_sum_dpp(v2.x + v2.y) * invC + p.eps);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      f32x2 o[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) o[h] = gelu2(pk_fma((y[q][h] - mean) * rstd, ga[q][h], be[q][h]));
      const long long off = row * C + (q * 64 + lane) * 4;
      const float ov[4] = {o[0].x, o[0].y, o[1].x, o[1].y};
      store4_out(p.out, p.out_dtype, off, rows * C, ov);
    }
    if (lane == 0) {
      p.mean[row] = mean;
      p.rstd[row] = rstd;
    }
  }
}

// conv0 forward on the matrix cores, for bf16 and split-bf16 (NRSE_BF16X3) outputs at k = 10:
// one wave = 16 rows x C channels per step. The 10-tap contraction is an MFMA 16x16x32 bf16 per
// 16-channel block with both operands split into bf16 hi + lo parts packed along K,
//   K = [x_hi . w_hi | x_lo . w_hi | x_hi . w_lo | 0 0]   (3 x 10 products, relative error ~2^-16),
// X3 adds x_lo . w_lo in a second MFMA (the three-plane output carries ~16 bits). The product is
// formed transposed (D = W'^T X'^T), so lane (g, l) holds row l of the block and, in channel
// block n, channels ch(n, 4g + r) = 32 (n >> 1) + 8 g + 4 (n & 1) + r: the row's LayerNorm sums
// are lane-local over 4 C / 16 values plus two lane swaps (the VALU kernel above paid two wave
// reductions per row), and each lane stores 8 consecutive channels (16 B) per block pair. The
// weight fragments live in LDS in fragment order (one conflict-free ds_read_b128 per block).
// S8 (ABI 7, y8): the split-planes contraction, stored as bf16 hi + the two fp8 correction planes
// [fp8((o - hi) 2^y8_exp) | fp8(hi)] (4 instead of 6 bytes per element).
// Exact f32 outputs (the parity mode) keep conv0_fwd_kernel.
template <int NB, bool X3, bool S8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void conv0_fwd_mfma_kernel(
    const nrse_conv0_params p) {
  constexpr int C = NB * 16, NF = X3 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) bf16x8 wimg[NF * NB * 64];
  __shared__ __attribute__((aligned(16))) float gb[2 * C];
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = lane >> 4, l = lane & 15;
  // weight fragments: fragment m, block n, lane (g', l') holds W'[k = 8 g' + e][ch(n, l')]
  for (int idx = tid; idx < NF * NB * 64; idx += 256) {
    const int m = idx / (NB * 64), rem = idx - m * (NB * 64);
    const int n = rem >> 6, gg = (rem >> 4) & 3, ll = rem & 15;
    const int ch = 32 * (n >> 1) + 8 * (ll >> 2) + 4 * (n & 1) + (ll & 3);
    bf16x8 v;
    // the 8 weight loads unconditional (tap k % 10 is always in range), the selection after: behind
    // the conditions each load had waited for its own round trip, 8 per fragment
    float wl[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) wl[e] = p.w[ch * KMAX + (8 * gg + e) % 10];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * gg + e;
      const float w = wl[e];
      const float hi = bf2f(f2bf(w));
      float wv = 0.f;
      if (m == 0 && k < 30) wv = k < 20 ? hi : w - hi;  // [w_hi | w_hi | w_lo]; w_lo rounds to bf16 below
      else if (m == 1 && k < 10) wv = w - hi;
      v[e] = (__bf16)wv;
    }
    wimg[idx] = v;
  }
  for (int c = tid; c < C; c += 256) {
    gb[c] = p.gamma[c];
    gb[C + c] = p.beta[c];
  }
  __syncthreads();

  // this lane's K positions: element e is k = 8g + e -> tap k % 10, part k / 10 (0 hi, 1 lo, 2 hi, 3 zero)
  int tap[8], part[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * g + e;
    tap[e] = k < 30 ? k % 10 : 0;
    part[e] = k / 10;
  }
  const long long rows = (long long)p.batch * p.T0;
  const long long nblk = (rows + 15) >> 4;
  const long long wstride = (long long)gridDim.x * 4;
  UDiv31 dT0;
  dT0.init((unsigned)p.T0);
  const float invC = 1.f / C;
  const float sc8 = __builtin_ldexpf(1.f, p.y8_exp);
  auto load_x = [&](long long blk, float (&xs)[8]) {
    long long row = blk * 16 + l;
    row = row < rows ? row : rows - 1;
    const unsigned b = dT0.div((unsigned)row);
    const int t = (int)((unsigned)row - b * (unsigned)p.T0);
    const float* x = p.wav + (long long)b * p.L + (long long)t * p.s;
#pragma unroll
    for (int e = 0; e < 8; ++e) xs[e] = ldg(x + tap[e]);
  };
  long long blk = (long long)blockIdx.x * 4 + (tid >> 6);
  float xn[8];
  if (blk < nblk) load_x(blk, xn);
  for (; blk < nblk; blk += wstride) {
    bf16x8 xf, xf2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float hi = bf2f(f2bf(xn[e]));
      const float lo = xn[e] - hi;
      xf[e] = (__bf16)(part[e] == 1 ? lo : (part[e] == 3 ? 0.f : hi));
      xf2[e] = (__bf16)(8 * g + e < 10 ? lo : 0.f);
    }
    if (blk + wstride < nblk) load_x(blk + wstride, xn);  // next block's samples in flight
    f32x4 acc[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wimg[n * 64 + lane], xf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      if constexpr (X3) acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wimg[(NB + n) * 64 + lane], xf2, acc[n], 0, 0, 0);
    }
    // LayerNorm over the row's C channels: this lane's 4 NB values + the lanes l ^ 16, l ^ 32
    f32x2 s2 = f32x2{0.f, 0.f};
#pragma unroll
    for (int n = 0; n < NB; ++n) s2 += f32x2{acc[n][0], acc[n][1]} + f32x2{acc[n][2], acc[n][3]};
    const float mean = xor32_sum(xor16_sum(s2.x + s2.y)) * invC;
    f32x2 v2 = f32x2{0.f, 0.f};
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const f32x2 d0 = f32x2{acc[n][0], acc[n][1]} - mean, d1 = f32x2{acc[n][2], acc[n][3]} - mean;
      acc[n] = f32x4{d0.x, d0.y, d1.x, d1.y};
      v2 = pk_fma(d0, d0, pk_fma(d1, d1, v2));
    }
    const float rstd = rsqrtf(xor32_sum(xor16_sum(v2.x + v2.y)) * invC + p.eps);
    const long long row = blk * 16 + l;
    const bool ok = row < rows;
    const f32x2 rs2 = f32x2{rstd, rstd};
#pragma unroll
    for (int q = 0; q < NB / 2; ++q) {
      const int c0 = 32 * q + 8 * g;
      float o[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 ga = *reinterpret_cast<const float4*>(gb + c0 + 4 * h);
        const float4 be = *reinterpret_cast<const float4*>(gb + C + c0 + 4 * h);
        const f32x4 a = acc[2 * q + h];
        const f32x2 z0 = pk_fma(f32x2{a[0], a[1]} * rs2, f32x2{ga.x, ga.y}, f32x2{be.x, be.y});
        const f32x2 z1 = pk_fma(f32x2{a[2], a[3]} * rs2, f32x2{ga.z, ga.w}, f32x2{be.z, be.w});
        const f32x2 y0 = gelu2(z0), y1 = gelu2(z1);
        o[4 * h + 0] = y0.x; o[4 * h + 1] = y0.y; o[4 * h + 2] = y1.x; o[4 * h + 3] = y1.y;
      }
      uint4 u;
      u.x = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
      u.y = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
      u.z = (uint32_t)f2bf(o[4]) | ((uint32_t)f2bf(o[5]) << 16);
      u.w = (uint32_t)f2bf(o[6]) | ((uint32_t)f2bf(o[7]) << 16);
      bf16_t* dst = (bf16_t*)p.out + row * C + c0;
      if (ok) {
        *reinterpret_cast<uint4*>(dst) = u;
        if constexpr (S8) {
          uint2 l8, h8;
          int ns = 0;
          fp8x4_split(o, sc8, l8.x, h8.x, &ns);
          fp8x4_split(o + 4, sc8, l8.y, h8.y, &ns);
          sat_count_add(p.sat_count, ns);
          unsigned char* d8 = (unsigned char*)p.y8 + row * C + c0;
          *reinterpret_cast<uint2*>(d8) = l8;
          *reinterpret_cast<uint2*>(d8 + rows * C) = h8;
        } else if constexpr (X3) {
          const unsigned uw[4] = {u.x, u.y, u.z, u.w};
          unsigned lw[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            lw[e] = (uint32_t)f2bf(o[2 * e] - __uint_as_float(uw[e] << 16)) |
                    ((uint32_t)f2bf(o[2 * e + 1] - __uint_as_float(uw[e] & 0xffff0000u)) << 16);
          *reinterpret_cast<uint4*>(dst + rows * C) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
          *reinterpret_cast<uint4*>(dst + 2 * rows * C) = u;
        }
      }
      // one block pair at a time: hoisting every pair's gamma / beta reads to the top of the
      // loop (what the scheduler does otherwise) spilled the accumulators
      __builtin_amdgcn_sched_barrier(0);
    }
    if (g == 0 && ok) {
      p.mean[row] = mean;
      p.rstd[row] = rstd;
    }
  }
}

NRSE_DEV void ld4(const void* p, int dt, long long i, float* o) {
  if (dt == NRSE_BF16) {
    uint2 v = *reinterpret_cast<const uint2*>((const bf16_t*)p + i);
    o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
    o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
  } else {
    float4 v = *reinterpret_cast<const float4*>((const float*)p + i);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
}

// conv0 backward: LN + GELU backward, the conv weight gradient dW[j][c] = sum_rows dc[c] * x[j],
// dgamma, dbeta. VALU-bound (conv recompute, GELU', dW: ~50 operations per element), so:
//  - a row is shared by C/256 waves (lane = 4 channels, 40 dW accumulators instead of 80), the
//    two waves of a C = 512 row exchange their LN partial sums through LDS (one barrier per row,
//    double-buffered slots), which keeps the kernel near 128 VGPRs (4 waves per SIMD);
//  - the conv and dW FMAs run as packed fp32 (v_pk_fma_f32: two channels per instruction);
//  - the next row's operands (10 samples, mean / rstd, up to two col2im taps of dy) are loaded
//    while the current row computes, the two taps into separate registers (no load -> add chain).

// One row's operands. BF (bf16 dy, the bf16 step): raw 8-byte words, unpacked at use, so no
// unpack (and no wait for the load) sits between the prefetch and the use. Every load is issued
// on every row from a valid address (clamped row, dummy tap offset + flag): a load skipped on
// some path leaves the wait-count pass no static count of the loads in flight.
template <bool BF>
struct C0Row {
  float xs[KMAX];
  float mean, rstd;
  uint2 r0, r1;     // BF
  f32x4 f0, f1;     // !BF
  bool v0, v1;
};

template <bool BF, bool K10>
NRSE_DEV void c0_load(const nrse_conv0_params& p, const UDiv31& dT0, const UDiv31& dS, long long row, int c0,
                      bool col2, C0Row<BF>& r) {
  const long long b = dT0.div((unsigned)row);  // rows < 2^31 (host check)
  const int t = (int)((unsigned)row - (unsigned)b * (unsigned)p.T0);
  const float* x = p.wav + b * p.L + (long long)t * p.s;
#pragma unroll
  for (int j = 0; j < KMAX; ++j) r.xs[j] = (K10 || j < p.k) ? ldg(x + j) : 0.f;
  r.mean = ldg(p.mean + row);
  r.rstd = ldg(p.rstd + row);
  long long o0 = row * p.C, o1 = 0;
  bool v0 = true, v1 = false;
  if (p.dy_mode == NRSE_DY_COL2IM) {
    // taps j0 = t mod s and j0 + s (k <= 2s): col row (t - j) / s of tap j
    const int q = (int)dS.div((unsigned)t);
    const int j0 = t - q * p.col_s;
    const int j1 = j0 + p.col_s;
    const int t0 = q, t1 = q - 1;  // (t - j1) / s where t >= j1 (v1); unused otherwise
    v0 = j0 < p.col_k && t0 < p.col_tout;
    v1 = j1 < p.col_k && t >= j1 && t1 < p.col_tout;
    o0 = v0 ? ((b * p.col_tout + t0) * p.col_k + j0) * (long long)p.C : 0;
    o1 = v1 ? ((b * p.col_tout + t1) * p.col_k + j1) * (long long)p.C : 0;
  }
  r.v0 = v0;
  r.v1 = v1;
  if constexpr (BF) {
    const bf16_t* dy = (const bf16_t*)p.dy;
    r.r0 = ldg(reinterpret_cast<const uint2*>(dy + o0 + c0));
    r.r1 = ldg(reinterpret_cast<const uint2*>(dy + o1 + c0));
  } else {
    const float* dy = (const float*)p.dy;
    r.f0 = ldg(reinterpret_cast<const f32x4*>(dy + o0 + c0));
    r.f1 = ldg(reinterpret_cast<const f32x4*>(dy + o1 + c0));
  }
}

NRSE_DEV f32x4 unpack_bf4v(uint2 v) {
  return f32x4{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
               __uint_as_float(v.y & 0xffff0000u)};
}

// generic col2im fold (k > 2s): the tap loop, dy summed into f0 (rare geometry; no prefetch)
NRSE_DEV f32x4 c0_dy_generic(const nrse_conv0_params& p, long long row, int c0) {
  const long long b = row / p.T0;
  const int t = (int)(row - b * p.T0);
  f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < p.col_k; ++j) {
    const int dd = t - j;
    if (dd < 0) break;
    if (dd % p.col_s) continue;
    const int tt = dd / p.col_s;
    if (tt >= p.col_tout) continue;
    const long long i = ((b * p.col_tout + tt) * p.col_k + j) * (long long)p.C + c0;
    d += p.dy_dtype == NRSE_BF16 ? unpack_bf4v(*reinterpret_cast<const uint2*>((const bf16_t*)p.dy + i))
                                 : *reinterpret_cast<const f32x4*>((const float*)p.dy + i);
  }
  return d;
}

// K10: k = KMAX and a two-tap col2im (col_k <= 2 col_s): unconditional tap loads, no generic fold
template <int WPR, bool BF, bool K10>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void conv0_bwd_kernel(const nrse_conv0_params p) {
  constexpr int RPB = 4 / WPR;  // rows in flight per block
  __shared__ __attribute__((aligned(16))) float wT[KMAX * 512];
  __shared__ float red[RPB][WPR * 256];
  __shared__ f32x2 xch[2][4];  // [row parity][wave]: the wave's (sum g, sum g*xh)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rg = w / WPR, half = w % WPR;
  const int C = p.C;
  const int c0 = (half * 64 + lane) * 4;
  load_wT(wT, p.w, C, p.k);
  __syncthreads();
  f32x2 dw[KMAX][2], dga[2], dbe[2], ga[2], be[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int j = 0; j < KMAX; ++j) dw[j][h] = f32x2{0.f, 0.f};
    dga[h] = dbe[h] = f32x2{0.f, 0.f};
    ga[h] = f32x2{p.gamma[c0 + 2 * h], p.gamma[c0 + 2 * h + 1]};
    be[h] = f32x2{p.beta[c0 + 2 * h], p.beta[c0 + 2 * h + 1]};
  }
  const long long rows = (long long)p.batch * p.T0;
  const long long last = rows - 1;
  const long long stride = (long long)gridDim.x * RPB;
  const long long first = (long long)blockIdx.x * RPB;
  // uniform trip count over the block (the row exchange is a block barrier)
  const long long iters = first < rows ? (rows - first + stride - 1) / stride : 0;
  const bool generic = !K10 && p.dy_mode == NRSE_DY_COL2IM && p.col_k > 2 * p.col_s;
  UDiv31 dT0, dS;
  dT0.init((unsigned)p.T0);
  dS.init(p.col_s > 0 ? (unsigned)p.col_s : 1u);
  const float invC = 1.f / C;

  auto step = [&](const C0Row<BF>& cur, C0Row<BF>& nxt, long long it, long long row) {
    const long long rn = row + stride;
    c0_load<BF, K10>(p, dT0, dS, rn < last ? rn : last, c0, !generic, nxt);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this row's math
    const bool live = row < rows;
    f32x2 xh[2], g[2];
    float s1 = 0.f, s2 = 0.f;
    if (live) {
      f32x4 dd;
      if (generic) {
        dd = c0_dy_generic(p, row, c0);
      } else if constexpr (BF) {
        const uint2 z = make_uint2(0u, 0u);
        dd = unpack_bf4v(cur.v0 ? cur.r0 : z) + unpack_bf4v(cur.v1 ? cur.r1 : z);
      } else {
        const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        dd = (cur.v0 ? cur.f0 : z) + (cur.v1 ? cur.f1 : z);
      }
      f32x2 y[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}};
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {  // weights from LDS: one ds_read_b128 per tap
        const float4 q = *reinterpret_cast<const float4*>(wT + j * C + c0);
        y[0] += f32x2{q.x, q.y} * cur.xs[j];
        y[1] += f32x2{q.z, q.w} * cur.xs[j];
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        xh[h] = (y[h] - cur.mean) * cur.rstd;
        const f32x2 z = xh[h] * ga[h] + be[h];
        const f32x2 dy = h == 0 ? f32x2{dd.x, dd.y} : f32x2{dd.z, dd.w};
        const f32x2 gg = dy * f32x2{gelu_grad_f(z.x), gelu_grad_f(z.y)};  // (packed form measured slower here)
        dga[h] += gg * xh[h];
        dbe[h] += gg;
        g[h] = gg * ga[h];
        s1 += g[h].x + g[h].y;
        const f32x2 gx = g[h] * xh[h];
        s2 += gx.x + gx.y;
      }
    }
    s1 = wave_sum_dpp(s1);
    s2 = wave_sum_dpp(s2);
    if constexpr (WPR > 1) {
      const int par = (int)(it & 1);
      if (lane == 0) xch[par][w] = f32x2{s1, s2};
      __syncthreads();
      s1 = 0.f;
      s2 = 0.f;
#pragma unroll
      for (int q = 0; q < WPR; ++q) {  // fixed order: both waves of the row get identical sums
        const f32x2 v = xch[par][rg * WPR + q];
        s1 += v.x;
        s2 += v.y;
      }
    }
    if (live) {
      s1 *= invC;
      s2 *= invC;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x2 dc = (g[h] - s1 - xh[h] * s2) * cur.rstd;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) dw[j][h] += dc * cur.xs[j];
      }
    }
  };

  C0Row<BF> ra, rb;
  long long row = first + rg;
  if (iters > 0) c0_load<BF, K10>(p, dT0, dS, row < last ? row : last, c0, !generic, ra);
  for (long long it = 0; it < iters; it += 2) {  // two row buffers, alternated (no copies)
    step(ra, rb, it, row);
    row += stride;
    if (it + 1 >= iters) break;
    step(rb, ra, it + 1, row);
    row += stride;
  }
  // block reduce: dw (k x C), dgamma, dbeta (the RPB row groups hold disjoint rows)
  const int kk = K10 ? KMAX : p.k;
  for (int j = 0; j < kk + 2; ++j) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x2 v = dbe[h];
#pragma unroll
      for (int jj = 0; jj < KMAX; ++jj)
        if (jj == j && jj < kk) v = dw[jj][h];  // rows kk, kk + 1 are dgamma, dbeta
      if (j == kk) v = dga[h];
      red[rg][c0 + 2 * h] = v.x;
      red[rg][c0 + 2 * h + 1] = v.y;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < RPB; ++q) v += red[q][c];
      if (p.part) p.part[((long long)blockIdx.x * (kk + 2) + j) * C + c] = v;  // row [dw | dgamma | dbeta]
      else if (j < kk) atomicAdd(p.dw + (long long)j * C + c, v);  // [k][C]: 256-B atomic wave-instructions
      else if (j == kk) atomicAdd(p.dgamma + c, v);
      else atomicAdd(p.dbeta + c, v);
    }
    __syncthreads();
  }
}

// conv0 backward on the matrix cores (bf16 dy, k = 10, two-tap col2im or direct dy, C = 256 | 512):
// the VALU kernel above spent ~20 of its ~50 operations per element on the conv recompute and the
// dW FMAs and exchanged LN sums through a barrier per row. Here a workgroup's 4 waves take a
// 16-row chunk together, each wave C/4 channels (NBW 16-channel blocks, lane column c owning
// channels w C/4 + NBW c .. + NBW - 1: one 16-byte dy load per row and tap):
//  - the conv is recomputed as the forward computes it (one MFMA 16x16x32 bf16 per block, the
//    split-bf16 packing K = [x_hi w_hi | x_lo w_hi | x_hi w_lo]), not transposed: lane (g, c)
//    holds rows 4g .. 4g+3 of its channel, so the per-channel sums (dgamma, dbeta) are lane-local
//    and the LN backward's row sums reduce over 16 lanes, then over the 4 waves through LDS (one
//    barrier per chunk, double-buffered slots);
//  - dW[c][j] = sum_rows dc[row][c] x[row][j] is an MFMA 16x16x16 bf16 per block whose A fragment
//    (channel on the lane column, rows 4g .. 4g+3 along k) is exactly the lane's dc values, in split
//    bf16 (dc_hi x_hi + dc_lo x_hi + dc_hi x_lo, three MFMAs: ~2^-16, the f32 kernel's accuracy);
//  - the waves own disjoint channels, so each workgroup stores its partial rows [dW | dgamma |
//    dbeta] whole (nrse_rows_reduce adds them in workgroup order) without a cross-wave reduction.
typedef short short4x __attribute__((ext_vector_type(4)));
NRSE_DEV short4x pk4_hi(const float* v, float* lo) {  // bf16 hi of 4 values; lo[e] = v[e] - hi
  short4x r;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bf16_t h = f2bf(v[e]);
    r[e] = (short)h;
    lo[e] = v[e] - bf2f(h);
  }
  return r;
}
NRSE_DEV short4x pk4(const float* v) {
  short4x r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = (short)f2bf(v[e]);
  return r;
}

// one 16-row chunk's operands of a lane (loaded a chunk ahead: two buffers alternate)
template <int NBW>
struct C0Chunk {
  float xa[8];          // X' fragment samples of row R0 + c
  float xb[4];          // dW B fragment: rows R0 + 4g + r, tap c
  float mu[4], rs[4];
  uint32_t d0[4][NBW / 2], d1[4][NBW / 2];  // the two col2im taps of dy, NBW bf16 per row
  uint32_t vmask;       // bit r: tap 0 valid, bit 4 + r: tap 1 valid
};

template <int NW, int NBW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2))) void conv0_bwd_mfma_kernel(
    const nrse_conv0_params p) {
  constexpr int C = NW * NBW * 16, CW = NBW * 16;
  __shared__ __attribute__((aligned(16))) bf16x8 wimg[NW * NBW * 64];  // [wave][block][lane] W' fragments
  __shared__ __attribute__((aligned(16))) f32x2 xch[2][16][NW];          // [parity][chunk row][wave]
  __shared__ __attribute__((aligned(16))) float gbs[2 * C];              // gamma | beta
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  const int cbase = w * CW + c * NBW;  // this lane's channels: cbase + n, n < NBW
  for (int idx = tid; idx < NW * NBW * 64; idx += NW * 64) {
    const int ww = idx / (NBW * 64), n = (idx / 64) % NBW, ln = idx & 63;
    const int ch = ww * CW + (ln & 15) * NBW + n;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * (ln >> 4) + e;
      float wv = 0.f;
      if (k < 30) {
        const float wf = p.w[ch * KMAX + k % 10];
        const float hi = bf2f(f2bf(wf));
        wv = k < 20 ? hi : wf - hi;
      }
      v[e] = (__bf16)wv;
    }
    wimg[idx] = v;
  }
  for (int i = tid; i < C; i += NW * 64) {
    gbs[i] = p.gamma[i];
    gbs[C + i] = p.beta[i];
  }
  __syncthreads();

  int tap[8], part[8];  // this lane's K positions of the X' fragment (as the forward)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * g + e;
    tap[e] = k < 30 ? k % 10 : 0;
    part[e] = k / 10;
  }
  const long long rows = (long long)p.batch * p.T0;
  const long long nch = (rows + 15) >> 4;
  UDiv31 dT0, dS;
  dT0.init((unsigned)p.T0);
  dS.init(p.col_s > 0 ? (unsigned)p.col_s : 1u);
  const bool col = p.dy_mode == NRSE_DY_COL2IM;
  const float invC = 1.f / C;
  const bf16_t* dyp = (const bf16_t*)p.dy;
  f32x4 dwa[NBW];
  f32x2 dga2[NBW / 2], dbe2[NBW / 2];
#pragma unroll
  for (int n = 0; n < NBW; ++n) dwa[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < NBW / 2; ++m) dga2[m] = dbe2[m] = f32x2{0.f, 0.f};
  auto xrow = [&](long long row) {  // waveform of conv0 row (row < rows)
    const unsigned b = dT0.div((unsigned)row);
    const int t = (int)((unsigned)row - b * (unsigned)p.T0);
    return p.wav + (long long)b * p.L + (long long)t * p.s;
  };
  // every load issued from a valid address (clamped rows, tap offsets 0 when invalid + mask bits),
  // so the wait-count pass sees a fixed number of loads in flight
  auto load = [&](long long ck, C0Chunk<NBW>& q) {
    const long long R0 = (ck < nch ? ck : nch - 1) * 16;
    {
      const long long ra = R0 + c < rows ? R0 + c : rows - 1;
      const float* x = xrow(ra);
#pragma unroll
      for (int e = 0; e < 8; ++e) q.xa[e] = ldg(x + tap[e]);
    }
    uint32_t vm = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long row = R0 + 4 * g + r;
      const bool live = row < rows;
      const long long rw = live ? row : rows - 1;
      q.xb[r] = ldg(xrow(rw) + (c < KMAX ? c : 0));
      q.mu[r] = ldg(p.mean + rw);
      q.rs[r] = ldg(p.rstd + rw);
      long long o0 = rw * C, o1 = 0;
      bool a0 = true, a1 = false;
      if (col) {
        const unsigned b = dT0.div((unsigned)rw);
        const int t = (int)((unsigned)rw - b * (unsigned)p.T0);
        const int qq = (int)dS.div((unsigned)t);
        const int j0 = t - qq * p.col_s, j1 = j0 + p.col_s;
        a0 = j0 < p.col_k && qq < p.col_tout;
        a1 = j1 < p.col_k && t >= j1 && qq - 1 < p.col_tout;
        o0 = a0 ? (((long long)b * p.col_tout + qq) * p.col_k + j0) * (long long)C : 0;
        o1 = a1 ? (((long long)b * p.col_tout + qq - 1) * p.col_k + j1) * (long long)C : 0;
      }
      vm |= (a0 && live ? 1u : 0u) << r;
      vm |= (a1 && live ? 1u : 0u) << (4 + r);
      if constexpr (NBW == 8) {
        const uint4 e0 = ldg(reinterpret_cast<const uint4*>(dyp + o0 + cbase));
        const uint4 e1 = ldg(reinterpret_cast<const uint4*>(dyp + o1 + cbase));
        q.d0[r][0] = e0.x; q.d0[r][1] = e0.y; q.d0[r][2] = e0.z; q.d0[r][3] = e0.w;
        q.d1[r][0] = e1.x; q.d1[r][1] = e1.y; q.d1[r][2] = e1.z; q.d1[r][3] = e1.w;
      } else {
        const uint2 e0 = ldg(reinterpret_cast<const uint2*>(dyp + o0 + cbase));
        const uint2 e1 = ldg(reinterpret_cast<const uint2*>(dyp + o1 + cbase));
        q.d0[r][0] = e0.x; q.d0[r][1] = e0.y;
        q.d1[r][0] = e1.x; q.d1[r][1] = e1.y;
      }
    }
    q.vmask = vm;
  };

  auto step = [&](long long ck, int it) {
    C0Chunk<NBW> q;
    load(ck, q);  // (a register prefetch of the next chunk pushed the kernel past 256 VGPRs)
    // ---- the conv, recomputed: D[row 4g + r][channel cbase + n]
    bf16x8 xf;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float hi = bf2f(f2bf(q.xa[e]));
      xf[e] = (__bf16)(part[e] == 1 ? q.xa[e] - hi : (part[e] == 3 ? 0.f : hi));
    }
    f32x4 acc[NBW];
#pragma unroll
    for (int n = 0; n < NBW; ++n)
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, wimg[(w * NBW + n) * 64 + lane], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    // ---- LN + GELU backward, first half, in channel pairs (n, n + 1) as packed FP32 (the dy word
    // of a pair holds both): gg, dgamma, dbeta, g = gg gamma and the row sums
    constexpr int NP = NBW / 2;
    f32x2 gv[NP][4], xh2[NP][4], s1[4], s2[4];
    f32x2 ga[NP], be[NP];
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      ga[m] = *reinterpret_cast<const f32x2*>(gbs + cbase + 2 * m);
      be[m] = *reinterpret_cast<const f32x2*>(gbs + C + cbase + 2 * m);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s1[r] = s2[r] = f32x2{0.f, 0.f};
      const bool v0 = (q.vmask >> r) & 1u, v1 = (q.vmask >> (4 + r)) & 1u;
      const f32x2 rs2 = splat2(q.rs[r]), nm2 = splat2(-q.mu[r] * q.rs[r]);
#pragma unroll
      for (int m = 0; m < NP; ++m) {
        const uint32_t u0 = v0 ? q.d0[r][m] : 0u, u1 = v1 ? q.d1[r][m] : 0u;
        const f32x2 dyv = f32x2{__uint_as_float(u0 << 16), __uint_as_float(u0 & 0xffff0000u)} +
                          f32x2{__uint_as_float(u1 << 16), __uint_as_float(u1 & 0xffff0000u)};
        const f32x2 xh = pk_fma(f32x2{acc[2 * m][r], acc[2 * m + 1][r]}, rs2, nm2);
        const f32x2 gg = dyv * gelu_grad2(pk_fma(xh, ga[m], be[m]));
        dga2[m] = pk_fma(gg, xh, dga2[m]);
        dbe2[m] += gg;
        const f32x2 gq = gg * ga[m];
        gv[m][r] = gq;
        xh2[m][r] = xh;
        s1[r] += gq;
        s2[r] = pk_fma(gq, xh, s2[r]);
      }
    }
    float rsc[4], xbc[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      rsc[r] = q.rs[r];
      xbc[r] = q.xb[r];
    }
    // row sums over the wave's channels (16 lane columns), then over the NW waves (fixed order)
    float t1[4], t2[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      t1[r] = s1[r].x + s1[r].y;
      t2[r] = s2[r].x + s2[r].y;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        t1[r] += __shfl_xor(t1[r], o, 16);
        t2[r] += __shfl_xor(t2[r], o, 16);
      }
    }
    const int par = it & 1;
    if (c == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) xch[par][4 * g + r][w] = f32x2{t1[r], t2[r]};
    }
    __syncthreads();
    f32x2 S1[4], S2[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = 0.f, b2 = 0.f;
#pragma unroll
      for (int qq = 0; qq < NW; ++qq) {
        const f32x2 v = xch[par][4 * g + r][qq];
        a += v.x;
        b2 += v.y;
      }
      S1[r] = splat2(a * invC);
      S2[r] = splat2(b2 * invC);
    }
    // ---- second half: dc, and dW += dc^T x on the matrix cores (split bf16)
    float xv[4], xlo[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) xv[r] = c < KMAX ? xbc[r] : 0.f;
    const short4x xbh = pk4_hi(xv, xlo);
    const short4x xbl = pk4(xlo);
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      float dc[2][4], dlo[2][4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f32x2 v = pk_fma(-xh2[m][r], S2[r], gv[m][r] - S1[r]) * splat2(rsc[r]);
        dc[0][r] = v.x;
        dc[1][r] = v.y;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int n = 2 * m + h;
        const short4x ah = pk4_hi(dc[h], dlo[h]);
        const short4x al = pk4(dlo[h]);
        dwa[n] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, xbh, dwa[n], 0, 0, 0);
        dwa[n] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(al, xbh, dwa[n], 0, 0, 0);
        dwa[n] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, xbl, dwa[n], 0, 0, 0);
      }
    }
  };

  // uniform trip count over the workgroup (the LN-sum exchange is a workgroup barrier)
  int it = 0;
#pragma unroll 1
  for (long long ck = blockIdx.x; ck < nch; ck += gridDim.x) step(ck, it++);
  // ---- the workgroup's partial rows: dW (lane (g, j): channels w CW + (4g + r) NBW + n, tap j),
  // dgamma / dbeta (summed over the 4 row groups g)
  const int kk = KMAX;
#pragma unroll
  for (int n = 0; n < NBW; ++n) {
    const float a = xor32_sum(xor16_sum((n & 1) ? dga2[n >> 1].y : dga2[n >> 1].x));
    const float b2 = xor32_sum(xor16_sum((n & 1) ? dbe2[n >> 1].y : dbe2[n >> 1].x));
    if (g == 0) {
      const int ch = cbase + n;
      if (p.part) {
        p.part[((long long)blockIdx.x * (kk + 2) + kk) * C + ch] = a;
        p.part[((long long)blockIdx.x * (kk + 2) + kk + 1) * C + ch] = b2;
      } else {
        atomicAdd(p.dgamma + ch, a);
        atomicAdd(p.dbeta + ch, b2);
      }
    }
    if (c < KMAX) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ch = w * CW + (4 * g + r) * NBW + n;
        if (p.part) p.part[((long long)blockIdx.x * (kk + 2) + c) * C + ch] = dwa[n][r];
        else atomicAdd(p.dw + (long long)c * C + ch, dwa[n][r]);
      }
    }
  }
}

// ---------------------------------------------------------------- weight norm (dim = 2)
// v [H][cpg][K] ; per tap j: norm_j = ||v[:, :, j]||
__global__ __launch_bounds__(256) void wn_norm_kernel(const float* __restrict__ v, float* __restrict__ norms,
                                                      const float* __restrict__ dWf, float* __restrict__ sdot, int H,
                                                      int cpg, int K) {
  __shared__ double red[4];
  const int j = blockIdx.x;
  const long long n = (long long)H * cpg;
  double a = 0.0;
  for (long long e = threadIdx.x; e < n; e += 256) {
    const float x = v[e * K + j];
    if (dWf) {
      // dWf layout [g][o][j*cpg + i], e = (g*cpg + o)*cpg + i
      const long long go = e / cpg;
      const int i = (int)(e % cpg);
      a += (double)x * dWf[go * (long long)K * cpg + (long long)j * cpg + i];
    } else {
      a += (double)x * x;
    }
  }
  a = wave_sum_d(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double s = red[0] + red[1] + red[2] + red[3];
    if (dWf) sdot[j] = (float)s;
    else norms[j] = (float)sqrt(s);
  }
}

// Coalesced form for K <= 256 dividing 256: thread (jj = tid % K, eo = tid / K) sums e = eo,
// eo + 256/K, ... over this block's e range, the partials of one j reduced in LDS, one double per
// (block, j) stored; wn_norm_final_kernel adds the blocks in order (deterministic). v is read in
// full 512-B rows (the [H*cpg][K] layout's K-contiguous rows).
__global__ __launch_bounds__(256) void wn_norm_part_kernel(const float* __restrict__ v, const float* __restrict__ dWf,
                                                           double* __restrict__ part, int H, int cpg, int K,
                                                           long long epb) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  const int j = tid % K, eo = tid / K, es = 256 / K;
  const long long n = (long long)H * cpg;
  const long long e0 = (long long)blockIdx.x * epb, e1 = min(n, e0 + epb);
  double a = 0.0;
#pragma unroll 8
  for (long long e = e0 + eo; e < e1; e += es) {
    const float x = v[e * K + j];
    if (dWf) {
      const long long go = e / cpg;
      const int i = (int)(e - go * cpg);
      a += (double)x * dWf[go * (long long)K * cpg + (long long)j * cpg + i];
    } else {
      a += (double)x * x;
    }
  }
  red[tid] = a;
  __syncthreads();
  if (tid < K) {
    double s = 0.0;
    for (int q = 0; q < es; ++q) s += red[q * K + tid];
    part[(long long)blockIdx.x * K + tid] = s;
  }
}

// Backward per-tap dot products sdot[j] = <v[:, :, j], dW[:, :, j]> with both operands read
// coalesced: v[go] is [cpg][K] (j contiguous) and dWf[go] is [K][cpg] (i contiguous), transposes
// of each other, so each output-channel slab of dWf goes through LDS ([j][i], row pad 1 float:
// the column reads by thread j are conflict-free). Thread (j, ih) accumulates i-half ih of tap j
// over the block's go range in f64; the two halves meet in LDS; part[block][j] as in the norm
// form (wn_norm_final_kernel adds the blocks in order). Needs K * cpg <= 8192, 2 * K <= 256.
constexpr int WN_DOT_LDS = 128 * 65;
__global__ __launch_bounds__(256) void wn_dot_part_kernel(const float* __restrict__ v, const float* __restrict__ dWf,
                                                          double* __restrict__ part, int ngo, int cpg, int K, int gpb) {
  __shared__ float tr[WN_DOT_LDS];
  __shared__ double red[256];
  const int tid = threadIdx.x;
  const int j = tid % K, ih = tid / K;  // 2 * K threads active
  const int ihalf = cpg / 2;
  const int ld = cpg + 1;
  double acc = 0.0;
  const int go0 = blockIdx.x * gpb, go1 = min(ngo, go0 + gpb);
  for (int go = go0; go < go1; ++go) {
    const float* d = dWf + (long long)go * K * cpg;
    __syncthreads();
    for (int e = tid; e < K * cpg; e += 256) tr[(e / cpg) * ld + (e % cpg)] = d[e];  // [j][i]
    __syncthreads();
    if (tid < 2 * K) {
      const float* vv = v + (long long)go * cpg * K;
      for (int i = ih * ihalf; i < (ih + 1) * ihalf; ++i) acc += (double)vv[(long long)i * K + j] * tr[j * ld + i];
    }
  }
  red[tid] = tid < 2 * K ? acc : 0.0;
  __syncthreads();
  if (tid < K) part[(long long)blockIdx.x * K + tid] = red[tid] + red[tid + K];
}

// one block per tap: thread b loads block b's partial, fixed-order tree (wave shuffles, then the
// 4 wave sums in order): deterministic, one load latency instead of nb dependent ones
__global__ __launch_bounds__(256) void wn_norm_final_kernel(const double* __restrict__ part, int nb, int K,
                                                            float* __restrict__ norms, float* __restrict__ sdot) {
  __shared__ double red[4];
  const int j = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < nb; b += 256) s += part[(long long)b * K + j];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = red[0] + red[1] + red[2] + red[3];
    if (sdot) sdot[j] = (float)t;
    else norms[j] = (float)sqrt(t);
  }
}

// norms[j] = ||v[:, :, j]|| (dWf null) or sdot[j] = <v[:, :, j], dW[:, :, j]> (dWf layout [g][o][j*cpg + i])
constexpr int WN_NB = 256;  // blocks of the two-stage reduction (part holds WN_NB * K doubles)
void wn_norm(hipStream_t st, const float* v, float* norms, const float* dWf, float* sdot, int H, int cpg, int K,
             double* part) {
  if (part && dWf && 2 * K <= 256 && K * cpg <= 8192 && cpg % 2 == 0 && K * (cpg + 1) <= WN_DOT_LDS) {
    const int ngo = H;  // [go][cpg][K] slabs of v, [go][K][cpg] of dWf
    const int gpb = (ngo + WN_NB - 1) / WN_NB;
    hipLaunchKernelGGL(wn_dot_part_kernel, dim3(WN_NB), dim3(256), 0, st, v, dWf, part, ngo, cpg, K, gpb);
    hipLaunchKernelGGL(wn_norm_final_kernel, dim3(K), dim3(256), 0, st, part, WN_NB, K, norms, sdot);
    return;
  }
  if (part && K <= 256 && 256 % K == 0) {
    const long long n = (long long)H * cpg;
    const long long epb = (n + WN_NB - 1) / WN_NB;
    hipLaunchKernelGGL(wn_norm_part_kernel, dim3(WN_NB), dim3(256), 0, st, v, dWf, part, H, cpg, K, epb);
    hipLaunchKernelGGL(wn_norm_final_kernel, dim3(K), dim3(256), 0, st, part, WN_NB, K, norms, sdot);
    return;
  }
  hipLaunchKernelGGL(wn_norm_kernel, dim3(K), dim3(256), 0, st, v, norms, dWf, sdot, H, cpg, K);
}

template <typename T>
__global__ void wn_apply_kernel(const float* __restrict__ g, const float* __restrict__ v,
                                const float* __restrict__ norms, T* __restrict__ wf, T* __restrict__ wd, int H, int cpg,
                                int K) {
  const long long total = (long long)H * cpg * K;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    // e enumerates wf: [G][o][j][i]
    const int i = (int)(e % cpg);
    const long long r = e / cpg;
    const int j = (int)(r % K);
    const long long go = r / K;          // g*cpg + o
    const long long gi = go / cpg;
    const int o = (int)(go % cpg);
    const float wv = v[(go * cpg + i) * K + j] * (g[j] / norms[j]);
    wf[e] = from_f<T>(wv);
    // wd[g][i][(K-1-j)*cpg + o]
    wd[((gi * cpg + i) * K + (K - 1 - j)) * cpg + o] = from_f<T>(wv);
  }
}

// dv (+)= (g_j / n_j) (dW - (sdot_j / n_j^2) v) per output-channel slab, dWf's [j][i] slab read
// coalesced into LDS (transposed to v's [i][j] order), v / dv streamed coalesced
__global__ __launch_bounds__(256) void wn_bwd_slab_kernel(const float* __restrict__ dWf, const float* __restrict__ g,
                                                          const float* __restrict__ v, const float* __restrict__ norms,
                                                          const float* __restrict__ sdot, float* __restrict__ dv,
                                                          int ngo, int cpg, int K, int gpb) {
  __shared__ float tr[WN_DOT_LDS];
  const int tid = threadIdx.x;
  const int ld = cpg + 1;
  const int go0 = blockIdx.x * gpb, go1 = min(ngo, go0 + gpb);
  for (int go = go0; go < go1; ++go) {
    const float* d = dWf + (long long)go * K * cpg;
    __syncthreads();
    for (int e = tid; e < K * cpg; e += 256) tr[(e / cpg) * ld + (e % cpg)] = d[e];  // [j][i]
    __syncthreads();
    const long long base = (long long)go * cpg * K;
    for (int e = tid; e < cpg * K; e += 256) {
      const int i = e / K, j = e - i * K;
      const float nj = norms[j];
      dv[base + e] += (g[j] / nj) * (tr[j * ld + i] - (sdot[j] / (nj * nj)) * v[base + e]);
    }
  }
}

__global__ void wn_bwd_kernel(const float* __restrict__ dWf, const float* __restrict__ g, const float* __restrict__ v,
                              const float* __restrict__ norms, const float* __restrict__ sdot, float* __restrict__ dv,
                              int H, int cpg, int K) {
  const long long total = (long long)H * cpg * K;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    // e enumerates v: [go][i][j]
    const int j = (int)(e % K);
    const long long r = e / K;
    const int i = (int)(r % cpg);
    const long long go = r / cpg;
    const float nj = norms[j];
    const float dw = dWf[go * (long long)K * cpg + (long long)j * cpg + i];
    dv[e] += (g[j] / nj) * (dw - (sdot[j] / (nj * nj)) * v[e]);
  }
}

__global__ void wn_dg_kernel(const float* __restrict__ sdot, const float* __restrict__ norms, float* __restrict__ dg,
                             int K) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < K) dg[j] += sdot[j] / norms[j];
}

}  // namespace

extern "C" int nrse_conv0_fwd(const nrse_conv0_params* p, void* stream) {
  NRSE_CHECK_PARAMS(p, "nrse_conv0_fwd");
  NRSE_REQUIRE(p && p->wav && p->w && p->gamma && p->beta && p->out && p->mean && p->rstd, "nrse_conv0_fwd: bad args");
  NRSE_REQUIRE(p->k > 0 && p->k <= KMAX && p->T0 == (p->L - p->k) / p->s + 1, "nrse_conv0_fwd: bad geometry");
  NRSE_REQUIRE((long long)p->batch * p->T0 < (1LL << 31), "nrse_conv0_fwd: too many rows");
  NRSE_REQUIRE(p->out_dtype == NRSE_F32 || p->out_dtype == NRSE_BF16 || p->out_dtype == NRSE_BF16X3,
               "nrse_conv0_fwd: bad out_dtype %d", p->out_dtype);
  const long long rows = (long long)p->batch * p->T0;
  long long blocks = (rows + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  hipStream_t st = (hipStream_t)stream;
  const bool k10 = p->k == KMAX;
  if (p->y8) {
    // ABI 7 fp8 correction planes: the matrix-core kernel's split-planes form only
    NRSE_REQUIRE(k10 && p->out_dtype == NRSE_BF16 && (p->C == 512 || p->C == 256) && conv0_mfma_on() &&
                     ((uintptr_t)p->y8 & 31) == 0 && p->y8_exp >= -60 && p->y8_exp <= 60 &&
                     (p->y8_dtype == 0 || p->y8_dtype == NRSE_FP8),
                 "nrse_conv0_fwd: y8 needs k = 10, a bf16 out, C = 256 | 512, the MFMA form (NRSE_CONV0_MFMA), "
                 "32-byte alignment, |y8_exp| <= 60 and y8_dtype 0 / NRSE_FP8");
  }
  if (k10 && p->out_dtype != NRSE_F32 && (p->C == 512 || p->C == 256) && conv0_mfma_on()) {
    // matrix-core form (bf16 / split-bf16 outputs): 2 workgroups per CU, waves loop over 16-row blocks
    const long long nblk = (rows + 15) / 16;
    long long wg = (nblk + 3) / 4;
    if (wg > 1024) wg = 1024;
    const bool x3 = p->out_dtype == NRSE_BF16X3, s8 = p->y8 != nullptr;
#define NRSE_C0F(NB)                                                                                   \
  if (s8) hipLaunchKernelGGL((conv0_fwd_mfma_kernel<NB, true, true>), dim3(wg), dim3(256), 0, st, *p); \
  else if (x3) hipLaunchKernelGGL((conv0_fwd_mfma_kernel<NB, true, false>), dim3(wg), dim3(256), 0, st, *p); \
  else hipLaunchKernelGGL((conv0_fwd_mfma_kernel<NB, false, false>), dim3(wg), dim3(256), 0, st, *p)
    if (p->C == 512) {
      NRSE_C0F(32);
    } else {
      NRSE_C0F(16);
    }
#undef NRSE_C0F
    return nrse_check_launch("nrse_conv0_fwd");
  }
  switch (p->C) {
    case 256:
      if (k10) hipLaunchKernelGGL((conv0_fwd_kernel<1, true>), dim3(blocks), dim3(256), 0, st, *p);
      else hipLaunchKernelGGL((conv0_fwd_kernel<1, false>), dim3(blocks), dim3(256), 0, st, *p);
      break;
    case 512:
      if (k10) hipLaunchKernelGGL((conv0_fwd_kernel<2, true>), dim3(blocks), dim3(256), 0, st, *p);
      else hipLaunchKernelGGL((conv0_fwd_kernel<2, false>), dim3(blocks), dim3(256), 0, st, *p);
      break;
    default: nrse_set_error("nrse_conv0_fwd: C=%d unsupported", p->C); return NRSE_ERR_UNSUPPORTED;
  }
  return nrse_check_launch("nrse_conv0_fwd");
}

// the matrix-core backward's conditions (the bf16 step's form); NRSE_CONV0_MFMA=0 keeps the VALU one
static bool conv0_bwd_mfma(const nrse_conv0_params* p) {
  return p->dy_dtype == NRSE_BF16 && p->k == KMAX && (p->C == 512 || p->C == 256) && conv0_mfma_on() &&
         (p->dy_mode == NRSE_DY_DIRECT || (p->dy_mode == NRSE_DY_COL2IM && p->col_k <= 2 * p->col_s));
}

// each block adds (k + 2) * C partial sums at the end (atomics or its partial row)
static long long conv0_bwd_blocks(const nrse_conv0_params* p) {
  const long long rows = (long long)p->batch * p->T0;
  if (conv0_bwd_mfma(p)) {  // 16-row chunks
    const long long ch = (rows + 15) / 16;
    return ch > 1024 ? 1024 : ch;
  }
  const int rpb = p->C == 512 ? 2 : 4;
  const long long blocks = (rows + rpb - 1) / rpb;
  return blocks > 1024 ? 1024 : blocks;
}

extern "C" int nrse_conv0_bwd(const nrse_conv0_params* p, void* stream) {
  NRSE_CHECK_PARAMS(p, "nrse_conv0_bwd");
  NRSE_REQUIRE(p && p->wav && p->w && p->gamma && p->beta && p->mean && p->rstd && p->dy && p->dw && p->dgamma &&
               p->dbeta, "nrse_conv0_bwd: bad args");
  NRSE_REQUIRE(p->k > 0 && p->k <= KMAX, "nrse_conv0_bwd: bad k");
  NRSE_REQUIRE((long long)p->batch * p->T0 < (1LL << 31), "nrse_conv0_bwd: too many rows");
  if (p->dy_mode == NRSE_DY_COL2IM) NRSE_REQUIRE(p->col_k > 0 && p->col_s > 0 && p->col_tout > 0, "nrse_conv0_bwd: col2im");
  const long long rows = (long long)p->batch * p->T0;
  const int rpb = p->C == 512 ? 2 : 4;
  const bool bf = p->dy_dtype == NRSE_BF16;
  const long long blocks = conv0_bwd_blocks(p);
  hipStream_t st = (hipStream_t)stream;
  // the model's geometry (k = 10, two-tap col2im) specialised; anything else takes the generic form
  const bool k10 = p->k == KMAX && (p->dy_mode != NRSE_DY_COL2IM || p->col_k <= 2 * p->col_s);
#define NRSE_C0B(W, B, K) hipLaunchKernelGGL((conv0_bwd_kernel<W, B, K>), dim3(blocks), dim3(256), 0, st, *p)
  if (conv0_bwd_mfma(p)) {
    if (p->C == 512) hipLaunchKernelGGL((conv0_bwd_mfma_kernel<4, 8>), dim3(blocks), dim3(256), 0, st, *p);
    else hipLaunchKernelGGL((conv0_bwd_mfma_kernel<4, 4>), dim3(blocks), dim3(256), 0, st, *p);
  } else
  switch (p->C) {
    case 256:
      if (k10) { if (bf) NRSE_C0B(1, true, true); else NRSE_C0B(1, false, true); }
      else { if (bf) NRSE_C0B(1, true, false); else NRSE_C0B(1, false, false); }
      break;
    case 512:  // 2 waves per row
      if (k10) { if (bf) NRSE_C0B(2, true, true); else NRSE_C0B(2, false, true); }
      else { if (bf) NRSE_C0B(2, true, false); else NRSE_C0B(2, false, false); }
      break;
    default: nrse_set_error("nrse_conv0_bwd: C=%d unsupported", p->C); return NRSE_ERR_UNSUPPORTED;
  }
#undef NRSE_C0B
  const int rc = nrse_check_launch("nrse_conv0_bwd");
  if (rc || !p->part) return rc;
  return nrse_rows_reduce(p->dw, (long long)p->k * p->C, p->dgamma, p->C, p->dbeta, p->C, p->part, (int)blocks, 1, 1,
                          st);
}

extern "C" long long nrse_conv0_bwd_workspace(const nrse_conv0_params* p) {
  NRSE_CHECK_PARAMS(p, "nrse_conv0_bwd_workspace");
  if (!p || p->batch <= 0 || p->T0 <= 0) return 0;
  return conv0_bwd_blocks(p) * (p->k + 2) * (long long)p->C;
}

extern "C" int nrse_weight_norm_fwd(const float* g, const float* v, void* wf, void* wd, int w_dtype, float* norms,
                                    int H, int cpg, int K, double* part, void* stream) {
  NRSE_REQUIRE(g && v && wf && wd && norms && H > 0 && cpg > 0 && K > 0 && H % cpg == 0, "nrse_weight_norm_fwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  wn_norm(st, v, norms, nullptr, nullptr, H, cpg, K, part);
  const long long total = (long long)H * cpg * K;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  if (w_dtype == NRSE_BF16)
    hipLaunchKernelGGL(wn_apply_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, g, v, norms, (bf16_t*)wf, (bf16_t*)wd,
                       H, cpg, K);
  else
    hipLaunchKernelGGL(wn_apply_kernel<float>, dim3(blocks), dim3(256), 0, st, g, v, norms, (float*)wf, (float*)wd, H,
                       cpg, K);
  return nrse_check_launch("nrse_weight_norm_fwd");
}

extern "C" int nrse_weight_norm_bwd(const float* dWf, const float* g, const float* v, const float* norms, float* dg,
                                    float* dv, float* scratch, int H, int cpg, int K, double* part, void* stream) {
  NRSE_REQUIRE(dWf && g && v && norms && dg && dv && scratch, "nrse_weight_norm_bwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  wn_norm(st, v, nullptr, dWf, scratch, H, cpg, K, part);
  const long long total = (long long)H * cpg * K;
  if (K * (cpg + 1) <= WN_DOT_LDS) {
    const int gpb = (H + WN_NB - 1) / WN_NB;
    hipLaunchKernelGGL(wn_bwd_slab_kernel, dim3(WN_NB), dim3(256), 0, st, dWf, g, v, norms, scratch, dv, H, cpg, K, gpb);
  } else {
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(wn_bwd_kernel, dim3(blocks), dim3(256), 0, st, dWf, g, v, norms, scratch, dv, H, cpg, K);
  }
  hipLaunchKernelGGL(wn_dg_kernel, dim3((K + 255) / 256), dim3(256), 0, st, scratch, norms, dg, K);
  return nrse_check_launch("nrse_weight_norm_bwd");
}
