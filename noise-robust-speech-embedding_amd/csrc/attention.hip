// Gated relative-position attention pieces of WavLMAttention ([TF]modeling_wavlm.py:147-271):
// rel-pos bias table, gate fwd/bwd, bias-table backward, and the exact-f32 attention kernels
// (one query/key row per lane). The f32 kernels are the parity path (fp32 mode) and the
// fallback for shapes the MFMA flash kernels (attention_mfma.hip) do not cover; they compute
// in f32 for both storage dtypes.
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

__global__ void rel_bias_bwd_kernel(const float* __restrict__ diag, const int* __restrict__ bucket,
                                    float* __restrict__ dE, int H, int T) {
  const int nd = 2 * T - 1;
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  const int h = blockIdx.y;
  if (d < nd) atomicAdd(dE + bucket[d] * H + h, diag[(long long)h * nd + d]);
}

// gate: one thread per (row, head)
template <typename T>
__global__ void gate_fwd_kernel(const void* __restrict__ x1, const float* __restrict__ W, const float* __restrict__ bv,
                                const float* __restrict__ c, float* __restrict__ gate, int batch, int Tn, int H) {
  __shared__ float w[8 * HD];
  for (int i = threadIdx.x; i < 8 * HD; i += blockDim.x) w[i] = W[i];
  __syncthreads();
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)batch * Tn * H;
  if (n >= total) return;
  const long long row = n / H;
  const int h = (int)(n % H);
  float pr[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) pr[r] = bv[r];
  const long long base = row * (long long)H * HD + h * HD;
  for (int i = 0; i < HD; ++i) {
    const float x = ld<T>(x1, base + i);
#pragma unroll
    for (int r = 0; r < 8; ++r) pr[r] += x * w[r * HD + i];
  }
  const float a = 1.f / (1.f + __expf(-(pr[0] + pr[1] + pr[2] + pr[3])));
  const float b = 1.f / (1.f + __expf(-(pr[4] + pr[5] + pr[6] + pr[7])));
  const long long bi = row / Tn, t = row % Tn;
  gate[(bi * H + h) * Tn + t] = a * (b * c[h] - 1.f) + 2.f;
}

// gate backward: one wave per (row, head), lane = head dim i. Recomputes the 8 projections
// with wave reductions, then dx1[i] += sum_r dproj[r] W[r][i] (coalesced read-modify-write),
// dproj [n][8] and dcterm [n] out for the GEMM / column-sum reductions done by the caller.
template <typename T>
__global__ __launch_bounds__(256) void gate_bwd_kernel(const void* __restrict__ x1, const float* __restrict__ W,
                                                       const float* __restrict__ bv, const float* __restrict__ c,
                                                       const float* __restrict__ dgate, float* __restrict__ dx1,
                                                       T* __restrict__ dproj, float* __restrict__ dcterm, int batch,
                                                       int Tn, int H) {
  const int lane = threadIdx.x & 63;
  const long long n = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long long total = (long long)batch * Tn * H;
  if (n >= total) return;
  const long long row = n / H;
  const int h = (int)(n % H);
  const long long base = row * (long long)H * HD + h * HD;
  const float x = ld<T>(x1, base + lane);
  float w[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) w[r] = W[r * HD + lane];
  float sa = 0.f, sb = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) { sa += x * w[r]; sb += x * w[4 + r]; }
  sa = wave_sum(sa) + bv[0] + bv[1] + bv[2] + bv[3];
  sb = wave_sum(sb) + bv[4] + bv[5] + bv[6] + bv[7];
  const float a = 1.f / (1.f + __expf(-sa));
  const float b = 1.f / (1.f + __expf(-sb));
  const long long bi = row / Tn, t = row % Tn;
  const float dg = dgate[(bi * H + h) * Tn + t];
  const float ch = c[h];
  const float dpa = dg * (b * ch - 1.f) * a * (1.f - a);
  const float dpb = dg * a * ch * b * (1.f - b);
  dx1[base + lane] += dpa * (w[0] + w[1] + w[2] + w[3]) + dpb * (w[4] + w[5] + w[6] + w[7]);
  if (lane < 8) dproj[n * 8 + lane] = from_f<T>(lane < 4 ? dpa : dpb);
  if (lane == 8) dcterm[n] = dg * a * b;
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
  const uint32_t thr = dropout_threshold(p.dropout_p);
  const float dsc = p.dropout_p > 0.f ? 1.f / (1.f - p.dropout_p) : 1.f;
  const uint32_t rowidx = (uint32_t)((((long long)b * H + h) * Tn + i) * Tn);
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
      if (p.dropout_p > 0.f) pd = dropout_keep(key, rowidx + j0 + jj, thr) ? pj * dsc : 0.f;
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
  __shared__ float dg[128];
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
  const uint32_t thr = dropout_threshold(p.dropout_p);
  const float dsc = p.dropout_p > 0.f ? 1.f / (1.f - p.dropout_p) : 1.f;
  const int nd = 2 * Tn - 1;
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
    dg[threadIdx.x] = 0.f;
    dg[64 + threadIdx.x] = 0.f;
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
          const bool keep = dropout_keep(key, (uint32_t)((((long long)b * H + h) * Tn + i) * Tn + j), thr);
          pd = keep ? pr * dsc : 0.f;
          dp = keep ? dpd * dsc : 0.f;
        }
        const float ds = pr * (dp - rowc[1][ii]);
#pragma unroll
        for (int d = 0; d < HD; ++d) { dv[d] += pd * Os[ii][d]; dk[d] += ds * Qs[ii][d]; }
        // diag index relative to this tile pair: (j - i) - (j0 - i0) + 63 in [0, 127)
        atomicAdd(&dg[(j - blockIdx.x * 64) - ii + 63], ds * gi);
      }
    }
    __syncthreads();
    if (p.diag) {
      for (int e = threadIdx.x; e < 127; e += 64) {
        const int dd = (blockIdx.x * 64 - i0) + e - 63 + Tn - 1;
        if (dd >= 0 && dd < nd && dg[e] != 0.f) atomicAdd(p.diag + (long long)h * nd + dd, dg[e]);
      }
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
  const uint32_t thr = dropout_threshold(p.dropout_p);
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
        const bool keep = dropout_keep(key, (uint32_t)((((long long)b * H + h) * Tn + i) * Tn + j), thr);
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

extern "C" int nrse_rel_bias_bwd(const float* diag, const int* bucket, float* dE, int H, int T, void* stream) {
  NRSE_REQUIRE(diag && bucket && dE && H > 0 && T > 0, "nrse_rel_bias_bwd: bad args");
  const int nd = 2 * T - 1;
  hipLaunchKernelGGL(rel_bias_bwd_kernel, dim3((nd + 255) / 256, H), dim3(256), 0, (hipStream_t)stream, diag, bucket,
                     dE, H, T);
  return nrse_check_launch("nrse_rel_bias_bwd");
}

extern "C" int nrse_gate_fwd(const void* x1, int x_dtype, const float* W, const float* bvec, const float* c,
                             float* gate, int batch, int T, int H, void* stream) {
  NRSE_REQUIRE(x1 && W && bvec && c && gate && batch > 0 && T > 0 && H > 0, "nrse_gate_fwd: bad args");
  const long long total = (long long)batch * T * H;
  dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  if (x_dtype == NRSE_BF16) hipLaunchKernelGGL(gate_fwd_kernel<bf16_t>, grid, dim3(256), 0, st, x1, W, bvec, c, gate, batch, T, H);
  else hipLaunchKernelGGL(gate_fwd_kernel<float>, grid, dim3(256), 0, st, x1, W, bvec, c, gate, batch, T, H);
  return nrse_check_launch("nrse_gate_fwd");
}

extern "C" int nrse_gate_bwd(const void* x1, int x_dtype, const float* W, const float* bvec, const float* c,
                             const float* dgate, float* dx1, void* dproj, float* dcterm, int batch, int T, int H,
                             void* stream) {
  NRSE_REQUIRE(x1 && W && bvec && c && dgate && dx1 && dproj && dcterm && batch > 0 && T > 0 && H > 0,
               "nrse_gate_bwd: bad args");
  const long long total = (long long)batch * T * H;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((total + 3) / 4));
  if (x_dtype == NRSE_BF16)
    hipLaunchKernelGGL(gate_bwd_kernel<bf16_t>, grid, dim3(256), 0, st, x1, W, bvec, c, dgate, dx1, (bf16_t*)dproj,
                       dcterm, batch, T, H);
  else
    hipLaunchKernelGGL(gate_bwd_kernel<float>, grid, dim3(256), 0, st, x1, W, bvec, c, dgate, dx1, (float*)dproj,
                       dcterm, batch, T, H);
  return nrse_check_launch("nrse_gate_bwd");
}

int nrse_attn_fwd_mfma(const nrse_attn_fwd_params* p, hipStream_t st);  // attention_mfma.hip
int nrse_attn_bwd_mfma(const nrse_attn_bwd_params* p, hipStream_t st);
int nrse_attn_use_mfma(int dtype, int head_dim);

extern "C" int nrse_attn_fwd(const nrse_attn_fwd_params* p, void* stream) {
  NRSE_REQUIRE(p && p->qkv && p->gate && p->bias && p->ctx && p->lse && p->batch > 0 && p->T > 0 && p->H > 0,
               "nrse_attn_fwd: bad args");
  if (p->head_dim != HD) { nrse_set_error("nrse_attn_fwd: head_dim %d != 64", p->head_dim); return NRSE_ERR_UNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  if (nrse_attn_use_mfma(p->dtype, p->head_dim)) return nrse_attn_fwd_mfma(p, st);
  dim3 grid((p->T + 63) / 64, p->H, p->batch);
  if (p->dtype == NRSE_BF16) hipLaunchKernelGGL(attn_fwd_f32_kernel<bf16_t>, grid, dim3(64), 0, st, *p);
  else hipLaunchKernelGGL(attn_fwd_f32_kernel<float>, grid, dim3(64), 0, st, *p);
  return nrse_check_launch("nrse_attn_fwd");
}

extern "C" int nrse_attn_bwd(const nrse_attn_bwd_params* p, void* stream) {
  NRSE_REQUIRE(p && p->qkv && p->gate && p->bias && p->ctx && p->dctx && p->lse && p->delta && p->dqkv && p->dgate &&
               p->batch > 0 && p->T > 0 && p->H > 0, "nrse_attn_bwd: bad args");
  if (p->head_dim != HD) { nrse_set_error("nrse_attn_bwd: head_dim %d != 64", p->head_dim); return NRSE_ERR_UNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  if (nrse_attn_use_mfma(p->dtype, p->head_dim)) return nrse_attn_bwd_mfma(p, st);  // computes delta itself
  const long long total = (long long)p->batch * p->H * p->T;
  dim3 g1((unsigned)((total + 255) / 256));
  if (p->dtype == NRSE_BF16) hipLaunchKernelGGL(attn_delta_kernel<bf16_t>, g1, dim3(256), 0, st, *p);
  else hipLaunchKernelGGL(attn_delta_kernel<float>, g1, dim3(256), 0, st, *p);
  dim3 grid((p->T + 63) / 64, p->H, p->batch);
  if (p->dtype == NRSE_BF16) {
    hipLaunchKernelGGL(attn_bwd_kv_f32_kernel<bf16_t>, grid, dim3(64), 0, st, *p);
    hipLaunchKernelGGL(attn_bwd_q_f32_kernel<bf16_t>, grid, dim3(64), 0, st, *p);
  } else {
    hipLaunchKernelGGL(attn_bwd_kv_f32_kernel<float>, grid, dim3(64), 0, st, *p);
    hipLaunchKernelGGL(attn_bwd_q_f32_kernel<float>, grid, dim3(64), 0, st, *p);
  }
  return nrse_check_launch("nrse_attn_bwd");
}
