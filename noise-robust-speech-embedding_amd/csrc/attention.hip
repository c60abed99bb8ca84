// Gated relative-position attention pieces of WavLMAttention ([TF]modeling_wavlm.py:147-271):
// rel-pos bias table, gate fwd/bwd, bias-table backward, and the exact-f32 attention kernels
// (one query/key row per lane). The f32 kernels are the parity path (fp32 mode) and the
// fallback for shapes the MFMA flash kernels (attention_mfma.hip) do not cover; they compute
// in f32 for both storage dtypes.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int HD = 64;  // head_dim (WavLM base/large)

template <typename T> NRSE_DEV float ld(const void* p, long long i) { return to_f<T>(((const T*)p)[i]); }
template <typename T> NRSE_DEV void st(void* p, long long i, float v) { ((T*)p)[i] = from_f<T>(v); }

NRSE_DEV int bias_ld_dev(int T) { return (T + 63) & ~63; }

__global__ void rel_bias_kernel(const float* __restrict__ E, const int* __restrict__ bucket, float* __restrict__ bias,
                                int H, int T) {
  const int Tb = bias_ld_dev(T);
  const long long n = (long long)T * Tb;
  const int h = blockIdx.y;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(e / Tb), j = (int)(e % Tb);
    bias[(long long)h * n + e] = j < T ? E[bucket[j - i + T - 1] * H + h] : 0.f;
  }
}

// Toeplitz form of the same table: vec[h, e] = E[bucket[e], h], e = j - i + T - 1
__global__ void rel_bias_vec_kernel(const float* __restrict__ E, const int* __restrict__ bucket, float* __restrict__ vec,
                                    int H, int T) {
  const int nd = 2 * T - 1;
  const int h = blockIdx.y;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < nd; e += gridDim.x * blockDim.x)
    vec[(long long)h * nd + e] = E[bucket[e] * H + h];
}

// dE[k, h] += sum of diag[h, d] over the offsets d of bucket k, in increasing d: a gather over
// the bucket's index list (order[offsets[k] .. offsets[k+1]), the d sorted by bucket) instead of a
// scatter with f32 atomics, so the sum order is fixed
__global__ void rel_bias_bwd_kernel(const float* __restrict__ diag, const int* __restrict__ order,
                                    const int* __restrict__ offsets, float* __restrict__ dE, int H, int T, int nb) {
  const int nd = 2 * T - 1;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int h = blockIdx.y;
  if (k >= nb) return;
  float s = 0.f;
  for (int i = offsets[k]; i < offsets[k + 1]; ++i) s += diag[(long long)h * nd + order[i]];
  dE[k * H + h] += s;
}

// Gate projections. gru_rel_pos_linear is Linear(64 -> 8) shared by all heads, and only the
// pair sums of its outputs are used (view(.., 2, 4).sum(-1), [TF]modeling_wavlm.py:168-176),
// so the 8 rows of W fold into two 64-vectors wa = sum_{r<4} W[r], wb = sum_{r>=4} W[r]:
// a = sigmoid(x.wa + sum_{r<4} b[r]), b = sigmoid(x.wb + sum_{r>=4} b[r]).
// Item n = row * H + h is the head-h slice x1[row, 64h : 64h + 64] (64 contiguous values);
// one 8-lane group per item, lane sub holds dims 8*sub .. 8*sub + 7 (one 16-byte bf16 load).
template <typename T> NRSE_DEV void ld8v(const void* p, long long i, float* o);
template <> NRSE_DEV void ld8v<bf16_t>(const void* p, long long i, float* o) {
  const uint4 u = *reinterpret_cast<const uint4*>((const bf16_t*)p + i);
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    o[2 * e] = __uint_as_float(w[e] << 16);
    o[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
}
template <> NRSE_DEV void ld8v<float>(const void* p, long long i, float* o) {
  const float4 a = *reinterpret_cast<const float4*>((const float*)p + i);
  const float4 b = *reinterpret_cast<const float4*>((const float*)p + i + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

struct GateW {
  float wa[8], wb[8], ba, bb;
  NRSE_DEV GateW(const float* W, const float* bv, int sub) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int i = 8 * sub + e;
      wa[e] = W[i] + W[HD + i] + W[2 * HD + i] + W[3 * HD + i];
      wb[e] = W[4 * HD + i] + W[5 * HD + i] + W[6 * HD + i] + W[7 * HD + i];
    }
    ba = bv[0] + bv[1] + bv[2] + bv[3];
    bb = bv[4] + bv[5] + bv[6] + bv[7];
  }
  // (a, b) of the item whose 8 values this lane holds (sums over the 8-lane group)
  NRSE_DEV void ab(const float* x, float& a, float& b) const {
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { sa += x[e] * wa[e]; sb += x[e] * wb[e]; }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) { sa += __shfl_xor(sa, o, 64); sb += __shfl_xor(sb, o, 64); }
    a = 1.f / (1.f + __expf(-(sa + ba)));
    b = 1.f / (1.f + __expf(-(sb + bb)));
  }
};

// GATE_U item groups per wave and iteration, their loads issued together (clamped, no branch):
// one group's 1 KiB per wave in flight left the sweep latency-bound (1.9 TB/s)
constexpr int GATE_U = 4;
template <typename T>
__global__ __launch_bounds__(256) void gate_fwd_kernel(const void* __restrict__ x1, const float* __restrict__ W,
                                                       const float* __restrict__ bv, const float* __restrict__ c,
                                                       float* __restrict__ gate, int batch, int Tn, int H) {
  const int lane = threadIdx.x & 63, sub = lane & 7, ig = lane >> 3;
  const GateW gw(W, bv, sub);
  const long long total = (long long)batch * Tn * H;
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nwave = (long long)gridDim.x * (blockDim.x >> 6);
  UDiv31 dH, dT;
  dH.init((unsigned)H);
  dT.init((unsigned)Tn);
  for (long long n0 = wave * 8 * GATE_U; n0 < total; n0 += nwave * 8 * GATE_U) {
    float x[GATE_U][8];
#pragma unroll
    for (int j = 0; j < GATE_U; ++j) {
      const long long n = n0 + 8 * j + ig;
      ld8v<T>(x1, (n < total ? n : total - 1) * HD + 8 * sub, x[j]);
    }
#pragma unroll
    for (int j = 0; j < GATE_U; ++j) {
      const long long n = n0 + 8 * j + ig;
      float a, b;
      gw.ab(x[j], a, b);
      if (sub == 0 && n < total) {
        const unsigned row = dH.div((unsigned)n);  // total < 2^31 (host check): multiply-high divides
        const int h = (int)((unsigned)n - row * (unsigned)H);
        const unsigned bi = dT.div(row), t = row - bi * (unsigned)Tn;
        gate[((long long)bi * H + h) * Tn + t] = a * (b * c[h] - 1.f) + 2.f;
      }
    }
  }
}

// Gate backward, fully fused: dx1 += dpa * wa + dpb * wb (f32 read-modify-write), and the
// parameter gradients reduced in registers -> LDS -> one set of atomics per workgroup:
//   dW[r < 4] += sum_n dpa_n x_n,  dW[r >= 4] += sum_n dpb_n x_n,  db likewise,
//   dc[h] += sum_{n of head h} dgate * a * b.
// The grid is a multiple of H workgroups, so the item stride (8 per wave per step) is a
// multiple of H and every 8-lane group keeps one head for the whole loop.
// DP (nrse_gate_bwd_dp): instead of the dx1 read-modify-write (104 MB per layer at WavLM-Large),
// store the item's (dpa, dpb) to dp[n] (float2); the encoder LayerNorm backward that reads dx1
// next adds dpa * wa + dpb * wb itself (nrse_ln_bwd_params.gate_dp).
constexpr int GATE_BWD_BLOCKS_PER_HEAD = 16;
constexpr int GATE_BU = 4;
template <typename T, bool DP>
__global__ __launch_bounds__(256) void gate_bwd_kernel(const void* __restrict__ x1, const float* __restrict__ W,
                                                       const float* __restrict__ bv, const float* __restrict__ c,
                                                       const float* __restrict__ dgate, float* __restrict__ dx1,
                                                       float* __restrict__ dW, float* __restrict__ db,
                                                       float* __restrict__ dc, int batch, int Tn, int H,
                                                       float* __restrict__ part) {
  __shared__ float red[4][2][HD];
  __shared__ float reds[4][2];
  __shared__ float redc[4][8];
  const int lane = threadIdx.x & 63, sub = lane & 7, ig = lane >> 3, w = threadIdx.x >> 6;
  const GateW gw(W, bv, sub);
  const long long total = (long long)batch * Tn * H;
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nwave = (long long)gridDim.x * (blockDim.x >> 6);
  const int h = (int)((wave * 8 + ig) % H);
  const float ch = c[h];
  float accA[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, accB[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float sdpa = 0.f, sdpb = 0.f, sdc = 0.f;
  // GATE_BU items per lane and iteration, one grid stride apart (so the lane's head is the same
  // for all of them), every load issued up front from a clamped index; 32-bit index math (the
  // host checks total < 2^31)
  const int tot = (int)total, stride = (int)(nwave * 8);
  for (int n0 = (int)(wave * 8) + ig; n0 < tot; n0 += stride * GATE_BU) {
    float x[GATE_BU][8], dgv[GATE_BU];
    float4 du[GATE_BU], dw[GATE_BU];
#pragma unroll
    for (int j = 0; j < GATE_BU; ++j) {
      const int n = n0 + j * stride;
      const int nc = n < tot ? n : tot - 1;
      ld8v<T>(x1, (long long)nc * HD + 8 * sub, x[j]);
      const int row = nc / H;
      const int bi = row / Tn, t = row - bi * Tn;
      dgv[j] = dgate[((long long)bi * H + h) * Tn + t];
      if constexpr (!DP) {
        const float4* d = reinterpret_cast<const float4*>(dx1 + (long long)nc * HD + 8 * sub);
        du[j] = d[0];
        dw[j] = d[1];
      }
    }
#pragma unroll
    for (int j = 0; j < GATE_BU; ++j) {
      const int n = n0 + j * stride;
      const bool ok = n < tot;
      float a, b;
      gw.ab(x[j], a, b);
      const float dg = ok ? dgv[j] : 0.f;
      const float dpa = dg * (b * ch - 1.f) * a * (1.f - a);
      const float dpb = dg * a * ch * b * (1.f - b);
      if constexpr (DP) {
        if (ok && sub == 0) *reinterpret_cast<float2*>(dx1 + 2LL * n) = make_float2(dpa, dpb);
      } else if (ok) {
        float4 u = du[j], v = dw[j];
        u.x += dpa * gw.wa[0] + dpb * gw.wb[0]; u.y += dpa * gw.wa[1] + dpb * gw.wb[1];
        u.z += dpa * gw.wa[2] + dpb * gw.wb[2]; u.w += dpa * gw.wa[3] + dpb * gw.wb[3];
        v.x += dpa * gw.wa[4] + dpb * gw.wb[4]; v.y += dpa * gw.wa[5] + dpb * gw.wb[5];
        v.z += dpa * gw.wa[6] + dpb * gw.wb[6]; v.w += dpa * gw.wa[7] + dpb * gw.wb[7];
        float4* d = reinterpret_cast<float4*>(dx1 + (long long)n * HD + 8 * sub);
        d[0] = u; d[1] = v;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) { accA[e] += dpa * x[j][e]; accB[e] += dpb * x[j][e]; }
      sdpa += dpa; sdpb += dpb; sdc += dg * a * b;
    }
  }
  // per-head term: one atomic per 8-lane group (or, with the partial-row workspace, the groups'
  // sums per head added in group order below)
  if (part) {
    if (sub == 0) redc[w][ig] = sdc;
  } else if (sub == 0 && sdc != 0.f) {
    atomicAdd(dc + h, sdc);
  }
  // sum over the 8 groups of the wave (lanes with equal sub hold the same dims)
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { accA[e] += __shfl_xor(accA[e], o, 64); accB[e] += __shfl_xor(accB[e], o, 64); }
    sdpa += __shfl_xor(sdpa, o, 64);
    sdpb += __shfl_xor(sdpb, o, 64);
  }
  if (ig == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[w][0][8 * sub + e] = accA[e]; red[w][1][8 * sub + e] = accB[e]; }
    if (sub == 0) { reds[w][0] = sdpa; reds[w][1] = sdpb; }
  }
  __syncthreads();
  // partial row [dW 8 x HD | db 8 | dc H] of this workgroup (nrse_rows_reduce adds the rows in
  // workgroup order), or f32 atomics
  float* prow = part ? part + (long long)blockIdx.x * (8 * HD + 8 + H) : nullptr;
  if (threadIdx.x < 2 * HD) {
    const int j = threadIdx.x / HD, i = threadIdx.x % HD;
    const float v = red[0][j][i] + red[1][j][i] + red[2][j][i] + red[3][j][i];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (prow) prow[(4 * j + r) * HD + i] = v;
      else atomicAdd(dW + (4 * j + r) * HD + i, v);
    }
  } else if (threadIdx.x < 2 * HD + 8) {
    const int r = threadIdx.x - 2 * HD;
    const int j = r >> 2;
    const float v = reds[0][j] + reds[1][j] + reds[2][j] + reds[3][j];
    if (prow) prow[8 * HD + r] = v;
    else atomicAdd(db + r, v);
  } else if (prow && threadIdx.x < 2 * HD + 8 + H) {
    // head hh: the 8-lane groups of this workgroup with (global wave * 8 + group) % H == hh
    const int hh = threadIdx.x - 2 * HD - 8;
    const long long wave0 = (long long)blockIdx.x * (blockDim.x >> 6);
    float v = 0.f;
    for (int ww = 0; ww < 4; ++ww)
      for (int gg = 0; gg < 8; ++gg)
        if ((int)(((wave0 + ww) * 8 + gg) % H) == hh) v += redc[ww][gg];
    prow[8 * HD + 8 + hh] = v;
  }
}

// ---------------------------------------------------------------- f32 attention (row per lane)
// grid (ceil(T/64), H, B), 64 threads; lane = query row.
template <typename T>
__global__ __launch_bounds__(64) void attn_fwd_f32_kernel(const nrse_attn_fwd_params p) {
  __shared__ float Ks[64][HD + 1];
  __shared__ float Vs[64][HD + 1];
  const int Tn = p.T, H = p.H, Hd = H * HD;
  const int b = blockIdx.z, h = blockIdx.y;
  const int i = blockIdx.x * 64 + threadIdx.x;
  const bool valid = i < Tn;
  const long long ld3 = 3LL * Hd;
  float q[HD], o[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    q[d] = valid ? ld<T>(p.qkv, ((long long)b * Tn + i) * ld3 + h * HD + d) * p.scale : 0.f;
    o[d] = 0.f;
  }
  const float g = valid ? p.gate[((long long)b * H + h) * Tn + i] : 0.f;
  const float* brow = p.bias + ((long long)h * Tn + (valid ? i : 0)) * bias_ld_dev(Tn);
  const uint32_t key = site_key(p.seed);
  const uint32_t thr = dropout_threshold16(p.dropout_p);
  const uint32_t tp2 = (uint32_t)((Tn + 1) >> 1);
  const float dsc = p.dropout_p > 0.f ? 1.f / (1.f - p.dropout_p) : 1.f;
  const uint32_t arow = (uint32_t)(((long long)b * H + h) * Tn + i);
  float m = -INFINITY, l = 0.f;
  for (int j0 = 0; j0 < Tn; j0 += 64) {
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * HD; e += 64) {
      const int jj = e / HD, d = e % HD;
      const int j = j0 + jj;
      const long long r = ((long long)b * Tn + (j < Tn ? j : 0)) * ld3;
      Ks[jj][d] = j < Tn ? ld<T>(p.qkv, r + Hd + h * HD + d) : 0.f;
      Vs[jj][d] = j < Tn ? ld<T>(p.qkv, r + 2 * Hd + h * HD + d) : 0.f;
    }
    __syncthreads();
    const int nj = min(64, Tn - j0);
    float s[64];
    float tmax = -INFINITY;
    for (int jj = 0; jj < nj; ++jj) {
      float a = 0.f;
#pragma unroll
      for (int d = 0; d < HD; ++d) a += q[d] * Ks[jj][d];
      a += g * brow[j0 + jj];
      s[jj] = a;
      tmax = fmaxf(tmax, a);
    }
    const float mn = fmaxf(m, tmax);
    const float alpha = __expf(m - mn);
    l *= alpha;
#pragma unroll
    for (int d = 0; d < HD; ++d) o[d] *= alpha;
    m = mn;
    for (int jj = 0; jj < nj; ++jj) {
      const float pj = __expf(s[jj] - m);
      l += pj;
      float pd = pj;
      if (p.dropout_p > 0.f) pd = attn_keep(key, arow, tp2, j0 + jj, thr) ? pj * dsc : 0.f;
#pragma unroll
      for (int d = 0; d < HD; ++d) o[d] += pd * Vs[jj][d];
    }
  }
  if (!valid) return;
  const float inv = 1.f / l;
#pragma unroll
  for (int d = 0; d < HD; ++d) st<T>(p.ctx, ((long long)b * Tn + i) * Hd + h * HD + d, o[d] * inv);
  p.lse[((long long)b * H + h) * Tn + i] = m + __logf(l);
}

// delta[b,h,i] = sum_d dO * O ; one thread per (b,h,i)
template <typename T>
__global__ void attn_delta_kernel(const nrse_attn_bwd_params p) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)p.batch * p.H * p.T;
  if (n >= total) return;
  const int i = (int)(n % p.T);
  const long long bh = n / p.T;
  const int h = (int)(bh % p.H);
  const long long b = bh / p.H;
  const long long base = (b * p.T + i) * (long long)p.H * HD + h * HD;
  float s = 0.f;
  for (int d = 0; d < HD; ++d) s += ld<T>(p.ctx, base + d) * ld<T>(p.dctx, base + d);
  p.delta[n] = s;
}

// dK, dV, diag: grid (ceil(T/64), H, B); lane = key row j
template <typename T>
__global__ __launch_bounds__(64) void attn_bwd_kv_f32_kernel(const nrse_attn_bwd_params p) {
  __shared__ float Qs[64][HD + 1];
  __shared__ float Os[64][HD + 1];   // dO tile
  __shared__ float rowc[4][64];      // lse, delta, gate per query
  // rel-pos diagonal sums of this key tile over ALL query tiles (dynamic LDS, f32_diag_len(T)
  // floats): diagonal j - i at dg[(j - i) - (j0 - Tq + 1)], Tq = T rounded up to the query tile
  extern __shared__ float dg[];
  const int Tn = p.T, H = p.H, Hd = H * HD;
  const int b = blockIdx.z, h = blockIdx.y;
  const int j = blockIdx.x * 64 + threadIdx.x;
  const bool valid = j < Tn;
  const long long ld3 = 3LL * Hd;
  float k[HD], v[HD], dk[HD], dv[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    const long long r = ((long long)b * Tn + (valid ? j : 0)) * ld3;
    k[d] = valid ? ld<T>(p.qkv, r + Hd + h * HD + d) : 0.f;
    v[d] = valid ? ld<T>(p.qkv, r + 2 * Hd + h * HD + d) : 0.f;
    dk[d] = dv[d] = 0.f;
  }
  const uint32_t key = site_key(p.seed);
  const uint32_t thr = dropout_threshold16(p.dropout_p);
  const float dsc = p.dropout_p > 0.f ? 1.f / (1.f - p.dropout_p) : 1.f;
  const int nd = 2 * Tn - 1;
  const int nq = (Tn + 63) / 64;
  const int ndg = nq * 64 + 63;       // diagonals j - i of this key tile: (j0 - Tq + 1) .. (j0 + 63)
  const int dg0 = blockIdx.x * 64 - nq * 64 + 1;
  for (int e = threadIdx.x; e < ndg; e += 64) dg[e] = 0.f;
  for (int i0 = 0; i0 < Tn; i0 += 64) {
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * HD; e += 64) {
      const int ii = e / HD, d = e % HD;
      const int i = i0 + ii;
      const bool ok = i < Tn;
      Qs[ii][d] = ok ? ld<T>(p.qkv, ((long long)b * Tn + i) * ld3 + h * HD + d) * p.scale : 0.f;
      Os[ii][d] = ok ? ld<T>(p.dctx, ((long long)b * Tn + i) * Hd + h * HD + d) : 0.f;
    }
    {
      const int i = i0 + threadIdx.x;
      const bool ok = i < Tn;
      const long long ri = ((long long)b * H + h) * Tn + (ok ? i : 0);
      rowc[0][threadIdx.x] = ok ? p.lse[ri] : 0.f;
      rowc[1][threadIdx.x] = ok ? p.delta[ri] : 0.f;
      rowc[2][threadIdx.x] = ok ? p.gate[ri] : 0.f;
    }
    __syncthreads();
    const int ni = min(64, Tn - i0);
    if (valid) {
      for (int ii = 0; ii < ni; ++ii) {
        const int i = i0 + ii;
        float s = 0.f, dpd = 0.f;
#pragma unroll
        for (int d = 0; d < HD; ++d) { s += Qs[ii][d] * k[d]; dpd += Os[ii][d] * v[d]; }
        const float gi = rowc[2][ii];
        const float bij = p.bias[((long long)h * Tn + i) * bias_ld_dev(Tn) + j];
        s += gi * bij;
        const float pr = __expf(s - rowc[0][ii]);
        float pd = pr, dp = dpd;
        if (p.dropout_p > 0.f) {
          const bool keep = attn_keep(key, (uint32_t)(((long long)b * H + h) * Tn + i), (uint32_t)((Tn + 1) >> 1), j, thr);
          pd = keep ? pr * dsc : 0.f;
          dp = keep ? dpd * dsc : 0.f;
        }
        const float ds = pr * (dp - rowc[1][ii]);
#pragma unroll
        for (int d = 0; d < HD; ++d) { dv[d] += pd * Os[ii][d]; dk[d] += ds * Qs[ii][d]; }
        // one wave: for a given ii the 64 lanes add to 64 distinct diagonals, and the ii / i0
        // order is program order, so the sums are deterministic
        atomicAdd(&dg[(j - i) - dg0], ds * gi);
      }
    }
  }
  __syncthreads();
  if (p.diag && p.diag_part) {
    // row (h, b, key tile) of the partial slab: this key tile's diagonals, zeros elsewhere
    // (added in (b, key tile) order by nrse_rows_reduce: deterministic)
    float* prow = p.diag_part + (((long long)h * p.batch + b) * gridDim.x + blockIdx.x) * nd;
    for (int dd = threadIdx.x; dd < nd; dd += 64) {
      const int e = dd - (Tn - 1) - dg0;
      prow[dd] = (e >= 0 && e < ndg) ? dg[e] : 0.f;
    }
  } else if (p.diag) {
    for (int e = threadIdx.x; e < ndg; e += 64) {
      const int dd = dg0 + e + Tn - 1;
      if (dd >= 0 && dd < nd && dg[e] != 0.f) atomicAdd(p.diag + (long long)h * nd + dd, dg[e]);
    }
  }
  if (!valid) return;
  const long long r = ((long long)b * Tn + j) * ld3;
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    st<T>(p.dqkv, r + Hd + h * HD + d, dk[d]);  // Qs carried the scale: dK = dS^T (Q*scale)
    st<T>(p.dqkv, r + 2 * Hd + h * HD + d, dv[d]);
  }
}

// dQ, dgate: grid (ceil(T/64), H, B); lane = query row i
template <typename T>
__global__ __launch_bounds__(64) void attn_bwd_q_f32_kernel(const nrse_attn_bwd_params p) {
  __shared__ float Ks[64][HD + 1];
  __shared__ float Vs[64][HD + 1];
  const int Tn = p.T, H = p.H, Hd = H * HD;
  const int b = blockIdx.z, h = blockIdx.y;
  const int i = blockIdx.x * 64 + threadIdx.x;
  const bool valid = i < Tn;
  const long long ld3 = 3LL * Hd;
  float q[HD], dO[HD], dq[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    q[d] = valid ? ld<T>(p.qkv, ((long long)b * Tn + i) * ld3 + h * HD + d) * p.scale : 0.f;
    dO[d] = valid ? ld<T>(p.dctx, ((long long)b * Tn + i) * Hd + h * HD + d) : 0.f;
    dq[d] = 0.f;
  }
  const long long ri = ((long long)b * H + h) * Tn + (valid ? i : 0);
  const float lse = valid ? p.lse[ri] : 0.f;
  const float delta = valid ? p.delta[ri] : 0.f;
  const float g = valid ? p.gate[ri] : 0.f;
  const float* brow = p.bias + ((long long)h * Tn + (valid ? i : 0)) * bias_ld_dev(Tn);
  const uint32_t key = site_key(p.seed);
  const uint32_t thr = dropout_threshold16(p.dropout_p);
  const float dsc = p.dropout_p > 0.f ? 1.f / (1.f - p.dropout_p) : 1.f;
  float dgate = 0.f;
  for (int j0 = 0; j0 < Tn; j0 += 64) {
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * HD; e += 64) {
      const int jj = e / HD, d = e % HD;
      const int j = j0 + jj;
      const long long r = ((long long)b * Tn + (j < Tn ? j : 0)) * ld3;
      Ks[jj][d] = j < Tn ? ld<T>(p.qkv, r + Hd + h * HD + d) : 0.f;
      Vs[jj][d] = j < Tn ? ld<T>(p.qkv, r + 2 * Hd + h * HD + d) : 0.f;
    }
    __syncthreads();
    if (!valid) continue;
    const int nj = min(64, Tn - j0);
    for (int jj = 0; jj < nj; ++jj) {
      const int j = j0 + jj;
      float s = 0.f, dpd = 0.f;
#pragma unroll
      for (int d = 0; d < HD; ++d) { s += q[d] * Ks[jj][d]; dpd += dO[d] * Vs[jj][d]; }
      const float bij = brow[j];
      s += g * bij;
      const float pr = __expf(s - lse);
      float dp = dpd;
      if (p.dropout_p > 0.f) {
        const bool keep = attn_keep(key, (uint32_t)(((long long)b * H + h) * Tn + i), (uint32_t)((Tn + 1) >> 1), j, thr);
        dp = keep ? dpd * dsc : 0.f;
      }
      const float ds = pr * (dp - delta);
      dgate += ds * bij;
#pragma unroll
      for (int d = 0; d < HD; ++d) dq[d] += ds * Ks[jj][d];
    }
  }
  if (!valid) return;
#pragma unroll
  for (int d = 0; d < HD; ++d) st<T>(p.dqkv, ((long long)b * Tn + i) * ld3 + h * HD + d, dq[d] * p.scale);
  p.dgate[ri] = dgate;
}

}  // namespace

extern "C" int nrse_bias_ld(int T) { return (T + 63) & ~63; }

extern "C" int nrse_rel_bias_fwd(const float* E, const int* bucket, float* bias, int H, int T, int nb, void* stream) {
  NRSE_REQUIRE(E && bucket && bias && H > 0 && T > 0 && nb > 0, "nrse_rel_bias_fwd: bad args");
  long long n = (long long)T * ((T + 63) & ~63);
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(rel_bias_kernel, dim3(blocks, H), dim3(256), 0, (hipStream_t)stream, E, bucket, bias, H, T);
  return nrse_check_launch("nrse_rel_bias_fwd");
}

extern "C" int nrse_rel_bias_vec(const float* E, const int* bucket, float* vec, int H, int T, int nb, void* stream) {
  NRSE_REQUIRE(E && bucket && vec && H > 0 && T > 0 && nb > 0, "nrse_rel_bias_vec: bad args");
  const int nd = 2 * T - 1;
  hipLaunchKernelGGL(rel_bias_vec_kernel, dim3((nd + 255) / 256, H), dim3(256), 0, (hipStream_t)stream, E, bucket, vec,
                     H, T);
  return nrse_check_launch("nrse_rel_bias_vec");
}

extern "C" int nrse_rel_bias_bwd(const float* diag, const int* order, const int* offsets, float* dE, int H, int T,
                                 int nb, void* stream) {
  NRSE_REQUIRE(diag && order && offsets && dE && H > 0 && T > 0 && nb > 0, "nrse_rel_bias_bwd: bad args");
  hipLaunchKernelGGL(rel_bias_bwd_kernel, dim3((nb + 63) / 64, H), dim3(64), 0, (hipStream_t)stream, diag, order,
                     offsets, dE, H, T, nb);
  return nrse_check_launch("nrse_rel_bias_bwd");
}

extern "C" int nrse_gate_fwd(const void* x1, int x_dtype, const float* W, const float* bvec, const float* c,
                             float* gate, int batch, int T, int H, void* stream) {
  NRSE_REQUIRE(x1 && W && bvec && c && gate && batch > 0 && T > 0 && H > 0, "nrse_gate_fwd: bad args");
  NRSE_REQUIRE(((uintptr_t)x1 & 15) == 0, "nrse_gate_fwd: x1 not 16-byte aligned");
  const long long total = (long long)batch * T * H;
  NRSE_REQUIRE(total < (1LL << 31), "nrse_gate_fwd: too many items");
  const long long blocks = (total + 32 * GATE_U - 1) / (32 * GATE_U);  // 8 * GATE_U items per wave, 4 waves
  dim3 grid((unsigned)(blocks < 2048 ? blocks : 2048));
  hipStream_t st = (hipStream_t)stream;
  if (x_dtype == NRSE_BF16) hipLaunchKernelGGL(gate_fwd_kernel<bf16_t>, grid, dim3(256), 0, st, x1, W, bvec, c, gate, batch, T, H);
  else hipLaunchKernelGGL(gate_fwd_kernel<float>, grid, dim3(256), 0, st, x1, W, bvec, c, gate, batch, T, H);
  return nrse_check_launch("nrse_gate_fwd");
}

static int gate_bwd_bph() {
  static const int bph = [] {
    const char* e = getenv("NRSE_GATE_BWD_BPH");
    const int v = e ? atoi(e) : GATE_BWD_BLOCKS_PER_HEAD;
    return v < 1 ? 1 : (v > GATE_BWD_BLOCKS_PER_HEAD * 8 ? GATE_BWD_BLOCKS_PER_HEAD * 8 : v);
  }();
  return bph;
}

// floats of nrse_gate_bwd's partial-row workspace
extern "C" long long nrse_gate_bwd_workspace(int H) { return (long long)gate_bwd_bph() * H * (8 * HD + 8 + H); }

extern "C" int nrse_gate_bwd(const void* x1, int x_dtype, const float* W, const float* bvec, const float* c,
                             const float* dgate, float* dx1, float* dW, float* db, float* dc, int batch, int T, int H,
                             float* part, void* stream) {
  NRSE_REQUIRE(x1 && W && bvec && c && dgate && dx1 && dW && db && dc && batch > 0 && T > 0 && H > 0,
               "nrse_gate_bwd: bad args");
  NRSE_REQUIRE(((uintptr_t)x1 & 15) == 0 && ((uintptr_t)dx1 & 15) == 0, "nrse_gate_bwd: x1/dx1 not 16-byte aligned");
  NRSE_REQUIRE((long long)batch * T * H < (1LL << 31) - (1LL << 24), "nrse_gate_bwd: too many items");
  hipStream_t st = (hipStream_t)stream;
  // a multiple of H workgroups: each 8-lane item group then keeps one head (see the kernel)
  // NRSE_GATE_BWD_BPH (tuning override) is clamped: <= 0 would launch an empty grid, a large value
  // would overflow the kernel's 32-bit item stride
  NRSE_REQUIRE(!part || H <= 256 - 2 * HD - 8, "nrse_gate_bwd: H too large for the partial-row form");
  dim3 grid((unsigned)(gate_bwd_bph() * H));
  if (x_dtype == NRSE_BF16)
    hipLaunchKernelGGL((gate_bwd_kernel<bf16_t, false>), grid, dim3(256), 0, st, x1, W, bvec, c, dgate, dx1, dW, db, dc,
                       batch, T, H, part);
  else
    hipLaunchKernelGGL((gate_bwd_kernel<float, false>), grid, dim3(256), 0, st, x1, W, bvec, c, dgate, dx1, dW, db, dc,
                       batch, T, H, part);
  const int rc = nrse_check_launch("nrse_gate_bwd");
  if (rc || !part) return rc;
  return nrse_rows_reduce(dW, 8 * HD, db, 8, dc, H, part, (int)grid.x, 1, 1, st);
}

extern "C" int nrse_gate_bwd_dp(const void* x1, int x_dtype, const float* W, const float* bvec, const float* c,
                                const float* dgate, float* dp, float* dW, float* db, float* dc, int batch, int T, int H,
                                float* part, void* stream) {
  NRSE_REQUIRE(x1 && W && bvec && c && dgate && dp && dW && db && dc && batch > 0 && T > 0 && H > 0,
               "nrse_gate_bwd_dp: bad args");
  NRSE_REQUIRE(((uintptr_t)x1 & 15) == 0 && ((uintptr_t)dp & 7) == 0, "nrse_gate_bwd_dp: x1 / dp misaligned");
  NRSE_REQUIRE((long long)batch * T * H < (1LL << 31) - (1LL << 24), "nrse_gate_bwd_dp: too many items");
  NRSE_REQUIRE(!part || H <= 256 - 2 * HD - 8, "nrse_gate_bwd_dp: H too large for the partial-row form");
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)(gate_bwd_bph() * H));
  if (x_dtype == NRSE_BF16)
    hipLaunchKernelGGL((gate_bwd_kernel<bf16_t, true>), grid, dim3(256), 0, st, x1, W, bvec, c, dgate, dp, dW, db, dc,
                       batch, T, H, part);
  else
    hipLaunchKernelGGL((gate_bwd_kernel<float, true>), grid, dim3(256), 0, st, x1, W, bvec, c, dgate, dp, dW, db, dc,
                       batch, T, H, part);
  const int rc = nrse_check_launch("nrse_gate_bwd_dp");
  if (rc || !part) return rc;
  return nrse_rows_reduce(dW, 8 * HD, db, 8, dc, H, part, (int)grid.x, 1, 1, st);
}

int nrse_attn_fwd_mfma(const nrse_attn_fwd_params* p, hipStream_t st);  // attention_mfma.hip
int nrse_attn_bwd_mfma(const nrse_attn_bwd_params* p, hipStream_t st);
int nrse_attn_use_mfma(int dtype, int head_dim);

extern "C" int nrse_attn_fwd(const nrse_attn_fwd_params* p, void* stream) {
  NRSE_CHECK_PARAMS(p, "nrse_attn_fwd");
  NRSE_REQUIRE(p && p->qkv && p->gate && (p->bias || p->bias_vec) && p->ctx && p->lse && p->batch > 0 && p->T > 0 && p->H > 0,
               "nrse_attn_fwd: bad args");
  if (p->head_dim != HD) { nrse_set_error("nrse_attn_fwd: head_dim %d != 64", p->head_dim); return NRSE_ERR_UNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  NRSE_REQUIRE(!p->ctx8 || (nrse_attn_use_mfma(p->dtype, p->head_dim) && ((uintptr_t)p->ctx8 & 3) == 0),
               "nrse_attn_fwd: ctx8 needs the bf16 MFMA path and 4-byte alignment");
  NRSE_REQUIRE(!p->ctx8 || p->ctx8_dtype == 0 || p->ctx8_dtype == NRSE_FP8,
               "nrse_attn_fwd: ctx8_dtype %d (0 or NRSE_FP8)", p->ctx8_dtype);
  if (nrse_attn_use_mfma(p->dtype, p->head_dim)) return nrse_attn_fwd_mfma(p, st);
  NRSE_REQUIRE(p->bias, "nrse_attn_fwd: the f32 path needs the [H, T, Tb] bias table");
  dim3 grid((p->T + 63) / 64, p->H, p->batch);
  if (p->dtype == NRSE_BF16) hipLaunchKernelGGL(attn_fwd_f32_kernel<bf16_t>, grid, dim3(64), 0, st, *p);
  else hipLaunchKernelGGL(attn_fwd_f32_kernel<float>, grid, dim3(64), 0, st, *p);
  return nrse_check_launch("nrse_attn_fwd");
}

// diag partial rows: one per (h, b, key tile) on both paths
extern "C" long long nrse_attn_bwd_workspace(const nrse_attn_bwd_params* p) {
  NRSE_CHECK_PARAMS(p, "nrse_attn_bwd_workspace");
  if (!p || p->T <= 0 || p->batch <= 0 || p->H <= 0) return 0;
  const long long nt = (p->T + 63) / 64;
  return (long long)p->H * p->batch * nt * (2LL * p->T - 1);
}

extern "C" int nrse_attn_bwd(const nrse_attn_bwd_params* p, void* stream) {
  NRSE_CHECK_PARAMS(p, "nrse_attn_bwd");
  NRSE_REQUIRE(p && p->qkv && p->gate && (p->bias || p->bias_vec) && p->ctx && p->dctx && p->lse && p->delta && p->dqkv && p->dgate &&
               p->batch > 0 && p->T > 0 && p->H > 0, "nrse_attn_bwd: bad args");
  if (p->head_dim != HD) { nrse_set_error("nrse_attn_bwd: head_dim %d != 64", p->head_dim); return NRSE_ERR_UNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  if (nrse_attn_use_mfma(p->dtype, p->head_dim)) return nrse_attn_bwd_mfma(p, st);  // computes delta itself
  NRSE_REQUIRE(p->bias, "nrse_attn_bwd: the f32 path needs the [H, T, Tb] bias table");
  const long long total = (long long)p->batch * p->H * p->T;
  dim3 g1((unsigned)((total + 255) / 256));
  if (p->dtype == NRSE_BF16) hipLaunchKernelGGL(attn_delta_kernel<bf16_t>, g1, dim3(256), 0, st, *p);
  else hipLaunchKernelGGL(attn_delta_kernel<float>, g1, dim3(256), 0, st, *p);
  dim3 grid((p->T + 63) / 64, p->H, p->batch);
  const size_t dg_lds = (size_t)(((p->T + 63) / 64) * 64 + 63) * sizeof(float);
  NRSE_REQUIRE(dg_lds <= 96 * 1024, "nrse_attn_bwd: T=%d too long for the f32 path's diagonal accumulator", p->T);
  if (p->dtype == NRSE_BF16) {
    hipLaunchKernelGGL(attn_bwd_kv_f32_kernel<bf16_t>, grid, dim3(64), dg_lds, st, *p);
    hipLaunchKernelGGL(attn_bwd_q_f32_kernel<bf16_t>, grid, dim3(64), 0, st, *p);
  } else {
    hipLaunchKernelGGL(attn_bwd_kv_f32_kernel<float>, grid, dim3(64), dg_lds, st, *p);
    hipLaunchKernelGGL(attn_bwd_q_f32_kernel<float>, grid, dim3(64), 0, st, *p);
  }
  const int rc = nrse_check_launch("nrse_attn_bwd");
  if (rc || !p->diag || !p->diag_part) return rc;
  const int nt = (p->T + 63) / 64;
  return nrse_rows_reduce(p->diag, 2LL * p->T - 1, nullptr, 0, nullptr, 0, p->diag_part, p->batch * nt, p->H, 1, st);
}
