// Elementwise / data-movement kernels of the step (HBM-bound; 16-byte vectors where the row
// width allows).
//   SpecAugment apply/bwd  [TF]modeling_wavlm.py:1006-1011
//   dropout backward       [TF]modeling_wavlm.py:99, 294, 482 (nn.Dropout)
//   bias gradients         column sums of the output gradients of every nn.Linear
#include <algorithm>

#include <cstdlib>
#include "common.h"

namespace {

template <typename T> NRSE_DEV void st1(void* p, long long i, float v) { ((T*)p)[i] = from_f<T>(v); }

__global__ void specaug_pad_kernel(float* __restrict__ h, const unsigned char* __restrict__ mask,
                                   const float* __restrict__ embed, void* __restrict__ dst, int dst_dtype, int batch,
                                   int T, int C, int pf, int pb) {
  const int Tp = T + pf + pb;
  const long long total = (long long)batch * Tp * C;
  UDiv31 dC, dTp;
  dC.init((unsigned)C);
  dTp.init((unsigned)Tp);
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const unsigned r = dC.div((unsigned)e);  // total < 2^31 (host check): multiply-high divides
    const int c = (int)((unsigned)e - r * (unsigned)C);
    const long long b = dTp.div(r);
    const int tp = (int)(r - (unsigned)b * (unsigned)Tp);
    const int t = tp - pf;
    float v = 0.f;
    if (t >= 0 && t < T) {
      const long long si = (b * T + t) * C + c;
      if (mask && mask[b * T + t]) {
        v = embed[c];
        if (h) h[si] = v;
      } else {
        v = h ? h[si] : 0.f;
      }
    }
    store_from_f(dst, dst_dtype, e, v);
  }
}

__global__ void pad_rows_kernel(const void* __restrict__ src, int sdt, void* __restrict__ dst, int ddt, int batch,
                                int T, int C, int pf, int pb) {
  const int Tp = T + pf + pb;
  const long long total = (long long)batch * Tp * C;
  UDiv31 dC, dTp;
  dC.init((unsigned)C);
  dTp.init((unsigned)Tp);
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const unsigned r = dC.div((unsigned)e);  // total < 2^31 (host check): multiply-high divides
    const int c = (int)((unsigned)e - r * (unsigned)C);
    const long long b = dTp.div(r);
    const int tp = (int)(r - (unsigned)b * (unsigned)Tp);
    const int t = tp - pf;
    const float v = (t >= 0 && t < T) ? load_as_f(src, sdt, (b * T + t) * C + c) : 0.f;
    store_from_f(dst, ddt, e, v);
  }
}

// one block per row chunk; thread per column
// ABI 10: the SpecAugment time masks drawn on the device ([TF]modeling_wavlm.py:834-954,
// _compute_mask_indices without an attention mask: every utterance has the full T). Utterance b
// masks n spans of L frames whose starts are a uniformly random n-subset of the C = T - L + 1
// candidates: the n candidates with the smallest 64-bit keys (mix32 of the flat candidate index
// b*C + k under the step's key, then k itself, so keys never tie). The reference draws the subset
// with numpy (np.random.choice(..., replace=False)); the distribution is the same, the stream is
// a counter hash that oracle/masks.py specaug_mask replays bit for bit. One workgroup per
// utterance: keys in LDS, each candidate ranked by one broadcast sweep (8 LDS reads in flight per
// step: the sweep had waited for each read, ~44 us per launch at T = 399), then each frame ORs the
// selection flags of the L starts that cover it (one coalesced byte store per frame).
constexpr int SPEC_CMAX = 4096, SPEC_NT = 512;
__global__ __launch_bounds__(SPEC_NT) void specaug_mask_kernel(unsigned char* __restrict__ mask, int T, int L, int n,
                                                               uint32_t key) {
  __shared__ unsigned long long keys[SPEC_CMAX + 8];
  __shared__ unsigned char sel[SPEC_CMAX];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int C = T - L + 1;
  if (n > 0) {
    const int C8 = (C + 7) & ~7;
    for (int k = tid; k < C8; k += SPEC_NT) {
      const uint32_t h = mix32(((uint32_t)b * (uint32_t)C + (uint32_t)k) ^ key);
      // padding past C: the largest key, never below a candidate's
      keys[k] = k < C ? ((unsigned long long)h << 32) | (unsigned long long)(unsigned)k : ~0ull;
    }
    __syncthreads();
    for (int k = tid; k < C; k += SPEC_NT) {
      const unsigned long long mine = keys[k];
      int rank = 0;
      for (int j = 0; j < C8; j += 8) {
        unsigned long long v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = keys[j + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) rank += v[u] < mine ? 1 : 0;
      }
      sel[k] = rank < n ? 1 : 0;
    }
    __syncthreads();
  }
  for (int t = tid; t < T; t += SPEC_NT) {
    unsigned char m = 0;
    if (n > 0) {
      const int lo = t - L + 1 < 0 ? 0 : t - L + 1, hi = t < C - 1 ? t : C - 1;
      for (int s2 = lo; s2 <= hi; ++s2) m |= sel[s2];
    }
    mask[(long long)b * T + t] = m;
  }
}

__global__ void specaug_bwd_kernel(const float* __restrict__ dh, const unsigned char* __restrict__ mask,
                                   float* __restrict__ dembed, void* __restrict__ out, int odt, int batch, int T, int C,
                                   float p, uint32_t seed, float* __restrict__ part) {
  const long long rows = (long long)batch * T;
  const uint32_t key = site_key(seed);
  const uint32_t thr = dropout_threshold(p);
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float acc = 0.f;
    for (long long r = blockIdx.x; r < rows; r += gridDim.x) {
      const long long i = r * C + c;
      const float g = dh[i];
      float o;
      if (mask && mask[r]) {
        acc += g;
        o = 0.f;
      } else {
        o = g;
        if (p > 0.f) o = dropout_keep(key, (uint32_t)i, thr) ? g * sc : 0.f;
      }
      store_from_f(out, odt, i, o);
    }
    if (mask && dembed) {
      if (part) part[(long long)blockIdx.x * C + c] = acc;  // added in block order (nrse_rows_reduce)
      else if (acc != 0.f) atomicAdd(dembed + c, acc);
    }
  }
}

__global__ void dropout_cast_kernel(const float* __restrict__ in, void* __restrict__ out, int odt, long long n, float p,
                                    uint32_t seed) {
  const uint32_t key = site_key(seed);
  const uint32_t thr = dropout_threshold(p);
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const long long n4 = n / 4;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (long long)gridDim.x * blockDim.x) {
    float4 v = reinterpret_cast<const float4*>(in)[q];
    float o[4] = {v.x, v.y, v.z, v.w};
    if (p > 0.f) {
      dropout_apply<4>(key, (uint32_t)(q * 4), thr, sc, o);
    }
    if (odt == NRSE_BF16) {
      uint2 u;
      u.x = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
      u.y = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
      reinterpret_cast<uint2*>(out)[q] = u;
    } else {
      reinterpret_cast<float4*>(out)[q] = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float v = in[i];
    if (p > 0.f) v = dropout_keep(key, (uint32_t)i, thr) ? v * sc : 0.f;
    store_from_f(out, odt, i, v);
  }
}

// colsum, vector form (C % 8 == 0): a block covers 512 columns (64 lanes x 8 columns, one
// 16-byte bf16 / 32-byte f32 load per lane per row) x 4 row lanes (the 4 waves) over a chunk of
// rows; the 4 partial sums meet in LDS and leave as 256-byte atomic wave-instructions (lane i on
// column i: the full memory-side atomic rate, MI355X_MICROARCH.md "Global float atomics").
template <typename T>
__global__ __launch_bounds__(256) void colsum8_kernel(const void* __restrict__ x, float* __restrict__ out,
                                                      long long rows, int C, int chunk, float* __restrict__ pr) {
  __shared__ float part[4][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cb0 = blockIdx.x * 512;
  const int c0 = cb0 + lane * 8;
  const long long r0 = (long long)blockIdx.y * chunk;
  const long long r1 = min(rows, r0 + chunk);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < C) {
#pragma unroll 4
    for (long long r = r0 + w; r < r1; r += 4) {
      if constexpr (sizeof(T) == 2) {
        const uint4 u = *reinterpret_cast<const uint4*>((const bf16_t*)x + r * C + c0);
        const unsigned v[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[2 * e] += __uint_as_float(v[e] << 16);
          a[2 * e + 1] += __uint_as_float(v[e] & 0xffff0000u);
        }
      } else {
        const float4 u = *reinterpret_cast<const float4*>((const float*)x + r * C + c0);
        const float4 v = *reinterpret_cast<const float4*>((const float*)x + r * C + c0 + 4);
        a[0] += u.x; a[1] += u.y; a[2] += u.z; a[3] += u.w; a[4] += v.x; a[5] += v.y; a[6] += v.z; a[7] += v.w;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[w][lane * 8 + e] = a[e];
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int col = threadIdx.x + 256 * h;
    if (cb0 + col < C) {
      const float s = part[0][col] + part[1][col] + part[2][col] + part[3][col];
      if (pr) pr[(long long)blockIdx.y * C + cb0 + col] = s;  // partial row of this row chunk
      else atomicAdd(out + cb0 + col, s);
    }
  }
}

// Dropout backward + cast + bias gradient in one pass over [rows, C] f32 rows (C % 8 == 0):
// out = dropout(in) in the output dtype, colsum[c] += sum_r out[r, c] (the f32 value before the
// cast). Same block geometry and atomic shape as colsum8_kernel.
template <typename TO>
__global__ __launch_bounds__(256) void dropout_cast_colsum_kernel(const float* __restrict__ in, TO* __restrict__ out,
                                                                  float* __restrict__ colsum, long long rows, int C,
                                                                  int chunk, float p, uint32_t seed,
                                                                  float* __restrict__ pr) {
  __shared__ float part[4][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cb0 = blockIdx.x * 512;
  const int c0 = cb0 + lane * 8;
  const long long r0 = (long long)blockIdx.y * chunk;
  const long long r1 = min(rows, r0 + chunk);
  const uint32_t key = site_key(seed);
  const uint32_t thr = dropout_threshold(p);
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < C) {
#pragma unroll 2
    for (long long r = r0 + w; r < r1; r += 4) {
      const long long i = r * C + c0;
      const float4 u = *reinterpret_cast<const float4*>(in + i);
      const float4 v = *reinterpret_cast<const float4*>(in + i + 4);
      float o[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
      if (p > 0.f) {
        dropout_apply<8>(key, (uint32_t)i, thr, sc, o);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += o[e];
      if constexpr (sizeof(TO) == 2) {
        uint4 q;
        q.x = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
        q.y = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
        q.z = (uint32_t)f2bf(o[4]) | ((uint32_t)f2bf(o[5]) << 16);
        q.w = (uint32_t)f2bf(o[6]) | ((uint32_t)f2bf(o[7]) << 16);
        *reinterpret_cast<uint4*>(out + i) = q;
      } else {
        *reinterpret_cast<float4*>(out + i) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(out + i + 4) = make_float4(o[4], o[5], o[6], o[7]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[w][lane * 8 + e] = a[e];
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int col = threadIdx.x + 256 * h;
    if (cb0 + col < C) {
      const float s = part[0][col] + part[1][col] + part[2][col] + part[3][col];
      if (pr) pr[(long long)blockIdx.y * C + cb0 + col] = s;
      else atomicAdd(colsum + cb0 + col, s);
    }
  }
}

// rows per block of the row-sweep kernels above: ~1024 blocks, a multiple of 16 rows
long long sweep_chunk(long long rows, int C) {
  const int cb = (C + 511) / 512;
  long long chunk = (rows * cb + 1023) / 1024;
  return ((chunk + 15) / 16) * 16;
}

// colsum, scalar form: grid (ceil(C/256), row chunks)
__global__ void colsum_kernel(const void* __restrict__ x, int dt, float* __restrict__ out, long long rows, int C,
                              int chunk, float* __restrict__ pr) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const long long r0 = (long long)blockIdx.y * chunk;
  const long long r1 = min(rows, r0 + chunk);
  float a = 0.f;
  for (long long r = r0; r < r1; ++r) a += load_as_f(x, dt, r * C + c);
  if (pr) pr[(long long)blockIdx.y * C + c] = a;
  else atomicAdd(out + c, a);
}

__global__ void cast_kernel(const void* __restrict__ x, int xdt, void* __restrict__ y, int ydt, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    store_from_f(y, ydt, i, load_as_f(x, xdt, i));
}

__global__ void split_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ hi, bf16_t* __restrict__ lo,
                                  long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = x[i];
    hi[i] = f2bf(v);
    lo[i] = bf16_lo(v);
  }
}

// the fp8 correction plane of the split (nrse_split_lo8), 4 elements (one u32 of fp8) per lane
__global__ void split_lo8_kernel(const float* __restrict__ x, uint32_t* __restrict__ lo8, float sc, long long n,
                                 unsigned int* __restrict__ sat) {
  const long long n4 = n / 4;
  int ns = 0;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (long long)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[q];
    const float a = lo_resid(v.x) * sc, b = lo_resid(v.y) * sc, c = lo_resid(v.z) * sc, d = lo_resid(v.w) * sc;
    lo8[q] = fp8x4(a, b, c, d);
    ns += fp8_nsat4(a, b, c, d);
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float a = lo_resid(x[i]) * sc;
    reinterpret_cast<unsigned char*>(lo8)[i] = fp8_1(a);
    ns += fp8_nsat4(a, 0.f, 0.f, 0.f);
  }
  sat_count_add(sat, ns);
}

__global__ void cast_fp8_kernel(const void* __restrict__ x, int xdt, unsigned char* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = fp8_1(load_as_f(x, xdt, i));
}

__global__ void zero_kernel(float* __restrict__ d, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    d[i] = 0.f;
}

__global__ void swap12_kernel(const void* __restrict__ src, int sdt, void* __restrict__ dst, int ddt, int d0, int d1,
                              int d2, int acc) {
  const long long total = (long long)d0 * d1 * d2;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    // e enumerates dst [a][c][b]
    const int b = (int)(e % d1);
    const long long r = e / d1;
    const int c = (int)(r % d2);
    const long long a = r / d2;
    float v = load_as_f(src, sdt, (a * d1 + b) * d2 + c);
    if (acc) v += load_as_f(dst, ddt, e);
    store_from_f(dst, ddt, e, v);
  }
}

__global__ void gelu_bwd_pad_kernel(const float* __restrict__ dy, const void* __restrict__ pre, int pdt,
                                    void* __restrict__ out, int odt, int batch, int T, int C, int pf, int pb) {
  const int Tp = T + pf + pb;
  const long long total = (long long)batch * Tp * C;
  UDiv31 dC, dTp;
  dC.init((unsigned)C);
  dTp.init((unsigned)Tp);
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const unsigned r = dC.div((unsigned)e);  // total < 2^31 (host check): multiply-high divides
    const int c = (int)((unsigned)e - r * (unsigned)C);
    const long long b = dTp.div(r);
    const int tp = (int)(r - (unsigned)b * (unsigned)Tp);
    const int t = tp - pf;
    float v = 0.f;
    if (t >= 0 && t < T) {
      const long long i = (b * T + t) * C + c;
      v = dy[i] * gelu_grad_f(load_as_f(pre, pdt, i));
    }
    store_from_f(out, odt, e, v);
  }
}

int blocks_for(long long n, int per = 256, int cap = 8192) {
  long long b = (n + per - 1) / per;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" int nrse_specaug_pad(float* h, const unsigned char* mask, const float* embed, void* dst, int dst_dtype,
                                int batch, int T, int C, int pf, int pb, void* stream) {
  NRSE_REQUIRE(dst && batch > 0 && T > 0 && C > 0 && pf >= 0 && pb >= 0, "nrse_specaug_pad: bad args");
  NRSE_REQUIRE(!mask || embed, "nrse_specaug_pad: mask without embed");
  const long long total = (long long)batch * (T + pf + pb) * C;
  NRSE_REQUIRE(total < (1LL << 31), "nrse_specaug_pad: too many elements");
  hipLaunchKernelGGL(specaug_pad_kernel, dim3(blocks_for(total)), dim3(256), 0, (hipStream_t)stream, h, mask, embed,
                     dst, dst_dtype, batch, T, C, pf, pb);
  return nrse_check_launch("nrse_specaug_pad");
}

// host restatement of common.h's mix32 / site_key (the span count needs eps on the host)
static uint32_t mix32_host(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

extern "C" int nrse_specaug_mask(unsigned char* mask, int batch, int T, double mask_prob, int mask_length,
                                 int min_masks, uint32_t seed, void* stream) {
  NRSE_REQUIRE(mask && batch > 0 && T > 0, "nrse_specaug_mask: bad args");
  int n = 0, L = mask_length < 1 ? 1 : mask_length;
  if (mask_prob > 0 && mask_length >= 1) {
    NRSE_REQUIRE(mask_length <= T, "nrse_specaug_mask: mask_length %d > sequence_length %d", mask_length, T);
    NRSE_REQUIRE(T - mask_length + 1 <= SPEC_CMAX, "nrse_specaug_mask: more than %d span starts", SPEC_CMAX);
    const uint32_t key = mix32_host(seed * 0x9e3779b9U + 0x632be5abU);
    // the reference's one eps per call (np.random.rand()), 24 random bits
    const double eps = (double)(mix32_host(key ^ 0x2545f491U) >> 8) * (1.0 / 16777216.0);
    n = (int)(mask_prob * T / mask_length + eps);
    if (n < min_masks) n = min_masks;
    if (n * mask_length > T) n = T / mask_length;
    if (T - (mask_length - 1) < n) n = T - (mask_length - 1) > 0 ? T - (mask_length - 1) : 0;
    seed = mix32_host(key ^ 0x5bd1e995U);
  }
  hipLaunchKernelGGL(specaug_mask_kernel, dim3(batch), dim3(SPEC_NT), 0, (hipStream_t)stream, mask, T, L, n, seed);
  return nrse_check_launch("nrse_specaug_mask");
}

extern "C" int nrse_pad_rows(const void* src, int sdt, void* dst, int ddt, int batch, int T, int C, int pf, int pb,
                             void* stream) {
  NRSE_REQUIRE(src && dst && batch > 0 && T > 0 && C > 0, "nrse_pad_rows: bad args");
  const long long total = (long long)batch * (T + pf + pb) * C;
  NRSE_REQUIRE(total < (1LL << 31), "nrse_pad_rows: too many elements");
  hipLaunchKernelGGL(pad_rows_kernel, dim3(blocks_for(total)), dim3(256), 0, (hipStream_t)stream, src, sdt, dst, ddt,
                     batch, T, C, pf, pb);
  return nrse_check_launch("nrse_pad_rows");
}

extern "C" int nrse_specaug_bwd(const float* dh, const unsigned char* mask, float* dembed, void* out, int odt,
                                int batch, int T, int C, float p, uint32_t seed, float* part, void* stream) {
  NRSE_REQUIRE(dh && out && batch > 0 && T > 0 && C > 0, "nrse_specaug_bwd: bad args");
  const long long rows = (long long)batch * T;
  const int blocks = (int)(rows < 2048 ? rows : 2048);
  if (!mask || !dembed) part = nullptr;
  hipLaunchKernelGGL(specaug_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dh, mask, dembed, out, odt,
                     batch, T, C, p, seed, part);
  const int rc = nrse_check_launch("nrse_specaug_bwd");
  if (rc || !part) return rc;
  return nrse_rows_reduce(dembed, C, nullptr, 0, nullptr, 0, part, blocks, 1, 1, stream);
}

extern "C" int nrse_dropout_cast(const float* in, void* out, int odt, long long n, float p, uint32_t seed,
                                 void* stream) {
  NRSE_REQUIRE(in && out && n >= 0, "nrse_dropout_cast: bad args");
  if (n == 0) return NRSE_OK;
  hipLaunchKernelGGL(dropout_cast_kernel, dim3(blocks_for(n / 4 + 1)), dim3(256), 0, (hipStream_t)stream, in, out, odt,
                     n, p, seed);
  return nrse_check_launch("nrse_dropout_cast");
}

// row chunks of the column-sum sweeps (vector form: C % 8 == 0 and x 16-byte aligned)
static long long colsum_chunks(long long rows, int C, bool vec, long long* chunk_out) {
  long long chunk;
  if (vec) {
    chunk = sweep_chunk(rows, C);
  } else {
    chunk = 64;
    while ((rows + chunk - 1) / chunk > 4096) chunk *= 2;
  }
  *chunk_out = chunk;
  return (rows + chunk - 1) / chunk;
}

// floats of the partial-row workspace of nrse_colsum / nrse_dropout_cast_colsum
extern "C" long long nrse_colsum_workspace(long long rows, int C) {
  if (rows <= 0 || C <= 0) return 0;
  long long c0, c1;
  const long long a = colsum_chunks(rows, C, true, &c0), b = colsum_chunks(rows, C, false, &c1);
  return (a > b ? a : b) * C;
}

extern "C" int nrse_dropout_cast_colsum(const float* in, void* out, int out_dtype, long long rows, int C, float p,
                                        uint32_t seed, float* colsum, float* part, void* stream) {
  NRSE_REQUIRE(in && out && colsum && rows > 0 && C > 0 && C % 8 == 0, "nrse_dropout_cast_colsum: bad args");
  NRSE_REQUIRE(((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0, "nrse_dropout_cast_colsum: unaligned");
  const int cb = (C + 511) / 512;
  long long chunk;
  const long long nchunks = colsum_chunks(rows, C, true, &chunk);
  const dim3 grid(cb, (unsigned)nchunks);
  if (out_dtype == NRSE_BF16)
    hipLaunchKernelGGL(dropout_cast_colsum_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, in, (bf16_t*)out,
                       colsum, rows, C, (int)chunk, p, seed, part);
  else
    hipLaunchKernelGGL(dropout_cast_colsum_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, in, (float*)out,
                       colsum, rows, C, (int)chunk, p, seed, part);
  const int rc = nrse_check_launch("nrse_dropout_cast_colsum");
  if (rc || !part) return rc;
  return nrse_rows_reduce(colsum, C, nullptr, 0, nullptr, 0, part, (int)nchunks, 1, 1, stream);
}

extern "C" int nrse_colsum(const void* x, int dt, float* colsum, long long rows, int C, float* part, void* stream) {
  NRSE_REQUIRE(x && colsum && rows > 0 && C > 0, "nrse_colsum: bad args");
  const bool vec = C % 8 == 0 && ((uintptr_t)x & 15) == 0;
  long long chunk;
  const long long nchunks = colsum_chunks(rows, C, vec, &chunk);
  if (vec) {
    // ~1024 blocks; each row lane reads >= 4 rows
    const int cb = (C + 511) / 512;
    if (dt == NRSE_BF16)
      hipLaunchKernelGGL(colsum8_kernel<bf16_t>, dim3(cb, (unsigned)nchunks), dim3(256), 0, (hipStream_t)stream, x,
                         colsum, rows, C, (int)chunk, part);
    else
      hipLaunchKernelGGL(colsum8_kernel<float>, dim3(cb, (unsigned)nchunks), dim3(256), 0, (hipStream_t)stream, x,
                         colsum, rows, C, (int)chunk, part);
  } else {
    hipLaunchKernelGGL(colsum_kernel, dim3((C + 255) / 256, (unsigned)nchunks), dim3(256), 0, (hipStream_t)stream, x,
                       dt, colsum, rows, C, (int)chunk, part);
  }
  const int rc = nrse_check_launch("nrse_colsum");
  if (rc || !part) return rc;
  return nrse_rows_reduce(colsum, C, nullptr, 0, nullptr, 0, part, (int)nchunks, 1, 1, stream);
}

extern "C" int nrse_split_bf16(const float* x, void* hi, void* lo, long long n, void* stream) {
  NRSE_REQUIRE(x && hi && lo && n >= 0, "nrse_split_bf16: bad args");
  if (n == 0) return NRSE_OK;
  hipLaunchKernelGGL(split_bf16_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, x, (bf16_t*)hi,
                     (bf16_t*)lo, n);
  return nrse_check_launch("nrse_split_bf16");
}

extern "C" int nrse_split_lo8(const float* x, void* lo8, int lo8_exp, long long n, unsigned int* sat_count,
                              void* stream) {
  NRSE_REQUIRE(x && lo8 && n >= 0 && lo8_exp > -64 && lo8_exp < 64, "nrse_split_lo8: bad args");
  NRSE_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)lo8 & 3) == 0, "nrse_split_lo8: x 16-byte, lo8 4-byte aligned");
  if (n == 0) return NRSE_OK;
  hipLaunchKernelGGL(split_lo8_kernel, dim3(blocks_for(n / 4 + 1)), dim3(256), 0, (hipStream_t)stream, x,
                     (uint32_t*)lo8, ldexpf(1.f, lo8_exp), n, sat_count);
  return nrse_check_launch("nrse_split_lo8");
}

extern "C" int nrse_cast_fp8(const void* x, int xdt, void* y8, long long n, void* stream) {
  NRSE_REQUIRE(x && y8 && n >= 0 && (xdt == NRSE_F32 || xdt == NRSE_BF16), "nrse_cast_fp8: bad args");
  if (n == 0) return NRSE_OK;
  hipLaunchKernelGGL(cast_fp8_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, x, xdt,
                     (unsigned char*)y8, n);
  return nrse_check_launch("nrse_cast_fp8");
}

extern "C" int nrse_zero(float* dst, long long n, void* stream) {
  NRSE_REQUIRE(dst && n >= 0, "nrse_zero: bad args");
  if (n == 0) return NRSE_OK;
  hipLaunchKernelGGL(zero_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, dst, n);
  return nrse_check_launch("nrse_zero");
}

extern "C" int nrse_cast(const void* x, int xdt, void* y, int ydt, long long n, void* stream) {
  NRSE_REQUIRE(x && y && n >= 0, "nrse_cast: bad args");
  if (n == 0) return NRSE_OK;
  hipLaunchKernelGGL(cast_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, x, xdt, y, ydt, n);
  return nrse_check_launch("nrse_cast");
}

// dst (+)= sum over splits of the f32 partial slabs, 16 B per lane, grid-stride; the slabs are
// streamed once (HBM-bound: (splits + 1 or 2) * n * 4 bytes). S > 0: the split count as a
// template constant, so every slab's load (and dst's) is issued before the first add; with the
// runtime count the loop waited for each load in turn. The sum order (dst, slab 0, 1, ...) is
// the same in both forms.
template <int S, bool ACC = false>
static __global__ __launch_bounds__(256) void splitk_reduce_kernel(float* __restrict__ dst, const float* __restrict__ slabs,
                                                                   int splits, long long n4, long long n, int acc) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    float4 s;
    if constexpr (S > 0) {
      float4 v[S];
      s = ACC ? reinterpret_cast<const float4*>(dst)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < S; ++k) v[k] = reinterpret_cast<const float4*>(slabs + (long long)k * n)[i];
#pragma unroll
      for (int k = 0; k < S; ++k) { s.x += v[k].x; s.y += v[k].y; s.z += v[k].z; s.w += v[k].w; }
    } else {
      s = acc ? reinterpret_cast<const float4*>(dst)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      for (int k = 0; k < splits; ++k) {
        const float4 v = reinterpret_cast<const float4*>(slabs + (long long)k * n)[i];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
    }
    reinterpret_cast<float4*>(dst)[i] = s;
  }
  // scalar tail (n % 4)
  for (long long i = n4 * 4 + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    float s = acc ? dst[i] : 0.f;
    for (int k = 0; k < splits; ++k) s += slabs[(long long)k * n + i];
    dst[i] = s;
  }
}

extern "C" int nrse_splitk_reduce(float* dst, const float* slabs, int splits, long long n, int accumulate,
                                  void* stream) {
  NRSE_REQUIRE(dst && slabs && splits >= 1 && n > 0, "nrse_splitk_reduce: bad args");
  NRSE_REQUIRE(((uintptr_t)dst & 15) == 0 && ((uintptr_t)slabs & 15) == 0 && (n % 4 == 0 || splits == 1),
               "nrse_splitk_reduce: dst / slabs must be 16-byte aligned and n a multiple of 4");
  const long long n4 = n / 4;
  const long long blocks = std::min<long long>((n4 + 255) / 256, 2048);
  const dim3 g((unsigned)std::max<long long>(blocks, 1));
  hipStream_t st = (hipStream_t)stream;
  switch (splits) {
    case 1:
      if (accumulate) hipLaunchKernelGGL((splitk_reduce_kernel<1, true>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate);
      else hipLaunchKernelGGL((splitk_reduce_kernel<1, false>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate);
      break;
    case 2:
      if (accumulate) hipLaunchKernelGGL((splitk_reduce_kernel<2, true>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate);
      else hipLaunchKernelGGL((splitk_reduce_kernel<2, false>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate);
      break;
    case 3:
      if (accumulate) hipLaunchKernelGGL((splitk_reduce_kernel<3, true>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate);
      else hipLaunchKernelGGL((splitk_reduce_kernel<3, false>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate);
      break;
    case 4:
      if (accumulate) hipLaunchKernelGGL((splitk_reduce_kernel<4, true>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate);
      else hipLaunchKernelGGL((splitk_reduce_kernel<4, false>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate);
      break;
    case 8:
      if (accumulate) hipLaunchKernelGGL((splitk_reduce_kernel<8, true>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate);
      else hipLaunchKernelGGL((splitk_reduce_kernel<8, false>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate);
      break;
    default: hipLaunchKernelGGL((splitk_reduce_kernel<0>), g, dim3(256), 0, st, dst, slabs, splits, n4, n, accumulate); break;
  }
  return nrse_check_launch("nrse_splitk_reduce");
}

extern "C" int nrse_swap12(const void* src, int sdt, void* dst, int ddt, int d0, int d1, int d2, int acc,
                           void* stream) {
  NRSE_REQUIRE(src && dst && d0 > 0 && d1 > 0 && d2 > 0, "nrse_swap12: bad args");
  const long long total = (long long)d0 * d1 * d2;
  hipLaunchKernelGGL(swap12_kernel, dim3(blocks_for(total)), dim3(256), 0, (hipStream_t)stream, src, sdt, dst, ddt, d0,
                     d1, d2, acc);
  return nrse_check_launch("nrse_swap12");
}

extern "C" int nrse_gelu_bwd_pad(const float* dy, const void* pre, int pdt, void* out, int odt, int batch, int T, int C,
                                 int pf, int pb, void* stream) {
  NRSE_REQUIRE(dy && pre && out && batch > 0 && T > 0 && C > 0, "nrse_gelu_bwd_pad: bad args");
  const long long total = (long long)batch * (T + pf + pb) * C;
  NRSE_REQUIRE(total < (1LL << 31), "nrse_gelu_bwd_pad: too many elements");
  hipLaunchKernelGGL(gelu_bwd_pad_kernel, dim3(blocks_for(total)), dim3(256), 0, (hipStream_t)stream, dy, pre, pdt,
                     out, odt, batch, T, C, pf, pb);
  return nrse_check_launch("nrse_gelu_bwd_pad");
}

// ------------------------------------------------------------------ ordered partial-row reduction
// The deterministic replacement of the per-workgroup f32 atomics of the gradient reductions
// (LayerNorm dgamma / dbeta, bias column sums, conv / gate / rel-pos parameter gradients, loss
// and norm accumulators): each producing workgroup writes its partial row to slab[s][0..n) and
// this kernel adds the rows in a fixed order into up to three destination vectors,
//   row = [d0: n0 | d1: n1 | d2: n2],   d_j[c] (+)= sum_s slab[s][off_j + c],
// so the result is the same on every run whatever the workgroups' completion order. 1024 threads
// per 256 columns: thread (r, q) sums rows r, r + 16, ... of columns 4q..4q+3 (16 B loads, 8
// independent loads in flight), then the 16 row-group sums are added in order r = 0..15.
// Row groups of `batch` (slab [batch][S][n], dst_j + b * n_j): per-utterance sums.
struct RowsDst { float* d[3]; long long n[3]; };

// RG row groups x (1024 / RG) column quads per workgroup: RG = 16 (256 columns) by default; RG =
// 64 (64 columns) when that grid would leave most CUs idle (r04: the encoder LayerNorm's 512
// partial rows x 3072 columns ran on 12 workgroups at ~1 TB/s). The bodies are device functions
// of the workgroup's (column block bx, row group by) so that the batched form below runs them
// unchanged (bitwise the same sums).
template <int RG>
NRSE_DEV void rows_reduce_body(float4 (*red)[1024 / RG], const RowsDst& dst, const float* __restrict__ slab, int S,
                               long long n, int acc, long long bx, int by) {
  constexpr int NQ = 1024 / RG;
  const int q = threadIdx.x % NQ, r = threadIdx.x / NQ;
  const long long col = bx * (4 * NQ) + 4 * q;
  const float* sl = slab + (long long)by * S * n;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < n) {
    int k = r;
    for (; k + 7 * RG < S; k += 8 * RG) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(sl + (long long)(k + RG * u) * n + col);
#pragma unroll
      for (int u = 0; u < 8; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
    for (; k < S; k += RG) {
      const float4 v = *reinterpret_cast<const float4*>(sl + (long long)k * n + col);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[r][q] = s;
  __syncthreads();
  if (r == 0 && col < n) {
    float4 t = red[0][q];
    // (unrolled by 8, not whole: at RG = 64 the compiler put all 63 LDS reads in flight at once
    // and spilled ~138 VGPRs of the 1024-thread workgroup's 128; same adds in the same order)
#pragma unroll 8
    for (int i = 1; i < RG; ++i) { t.x += red[i][q].x; t.y += red[i][q].y; t.z += red[i][q].z; t.w += red[i][q].w; }
    int j = 0;
    long long c = col;
    while (j < 2 && c >= dst.n[j]) { c -= dst.n[j]; ++j; }
    float* d = dst.d[j] + (long long)by * dst.n[j] + c;
    if (acc) {
      const float4 o = *reinterpret_cast<const float4*>(d);
      t.x += o.x; t.y += o.y; t.z += o.z; t.w += o.w;
    }
    *reinterpret_cast<float4*>(d) = t;
  }
}

// the same with one column per thread (lengths that are not multiples of 4, unaligned vectors)
NRSE_DEV void rows_reduce1_body(float (*red)[64], const RowsDst& dst, const float* __restrict__ slab, int S,
                                long long n, int acc, long long bx, int by) {
  const int q = threadIdx.x & 63, r = threadIdx.x >> 6;
  const long long col = bx * 64 + q;
  const float* sl = slab + (long long)by * S * n;
  float s = 0.f;
  if (col < n) {
    int k = r;
    for (; k + 112 < S; k += 128) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = sl[(long long)(k + 16 * u) * n + col];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < S; k += 16) s += sl[(long long)k * n + col];
  }
  red[r][q] = s;
  __syncthreads();
  if (r == 0 && col < n) {
    float t = red[0][q];
#pragma unroll
    for (int i = 1; i < 16; ++i) t += red[i][q];
    int j = 0;
    long long c = col;
    while (j < 2 && c >= dst.n[j]) { c -= dst.n[j]; ++j; }
    float* d = dst.d[j] + (long long)by * dst.n[j] + c;
    *d = acc ? *d + t : t;
  }
}

template <int RG>
__global__ __launch_bounds__(1024) void rows_reduce_kernel(RowsDst dst, const float* __restrict__ slab, int S,
                                                           long long n, int acc) {
  __shared__ float4 red[RG][1024 / RG];
  rows_reduce_body<RG>(red, dst, slab, S, n, acc, blockIdx.x, blockIdx.y);
}

__global__ __launch_bounds__(1024) void rows_reduce1_kernel(RowsDst dst, const float* __restrict__ slab, int S,
                                                            long long n, int acc) {
  __shared__ float red[16][64];
  rows_reduce1_body(red, dst, slab, S, n, acc, blockIdx.x, blockIdx.y);
}

// One reduction as nrse_rows_reduce launches it: the form (0: RG 16, 1: RG 64, 2: one column per
// thread) and its grid (gx column blocks x batch row groups).
struct RowsJob {
  RowsDst dst;
  const float* slab;
  long long n;
  int S, batch, acc, form, gx;
};

static RowsJob rows_job(float* d0, long long n0, float* d1, long long n1, float* d2, long long n2, const float* slab, int S,
                 int batch, int accumulate) {
  auto al16 = [](const void* x) { return ((uintptr_t)x & 15) == 0; };
  RowsJob j;
  j.dst.d[0] = d0; j.dst.d[1] = d1; j.dst.d[2] = d2;
  j.dst.n[0] = n0; j.dst.n[1] = d1 ? n1 : 0; j.dst.n[2] = d2 ? n2 : 0;
  j.n = j.dst.n[0] + j.dst.n[1] + j.dst.n[2];
  j.slab = slab; j.S = S; j.batch = batch; j.acc = accumulate;
  const bool vec = n0 % 4 == 0 && j.dst.n[1] % 4 == 0 && j.dst.n[2] % 4 == 0 && al16(d0) && (!d1 || al16(d1)) &&
                   (!d2 || al16(d2)) && al16(slab);
  if (vec && S >= 128 && ((j.n + 255) / 256) * batch < 128) { j.form = 1; j.gx = (int)((j.n + 63) / 64); }
  else if (vec) { j.form = 0; j.gx = (int)((j.n + 255) / 256); }
  else { j.form = 2; j.gx = (int)((j.n + 63) / 64); }
  return j;
}

// ABI 9: deferred reductions. While deferral is on, every nrse_rows_reduce (the gradient
// reductions the LayerNorm, attention, gate, GEMM column-sum and colsum entry points end with) is
// queued instead of launched; nrse_reduce_flush then runs the queue as batched launches of up to
// RJ_MAX jobs each, on the stream it is given. The step's backward queues one transformer layer's
// reductions on the dX chain's stream and flushes them on the weight-gradient stream, so the
// ~6 small launches per layer leave the critical stream (each job's arithmetic is the
// single-launch form's: the sums are bitwise the same).
constexpr int RJ_MAX = 12;
struct RowsJobs {
  RowsJob j[RJ_MAX];
  int begin[RJ_MAX + 1];  // first flat workgroup of job i
  int count;
};

__global__ __launch_bounds__(1024) void rows_reduce_multi_kernel(const RowsJobs jobs) {
  __shared__ __attribute__((aligned(16))) float4 red[1024];
  int i = 0;
  while (i + 1 < jobs.count && (int)blockIdx.x >= jobs.begin[i + 1]) ++i;
  const RowsJob& j = jobs.j[i];
  const int local = (int)blockIdx.x - jobs.begin[i];
  const int bx = local % j.gx, by = local / j.gx;
  if (j.form == 0) rows_reduce_body<16>(reinterpret_cast<float4(*)[64]>(red), j.dst, j.slab, j.S, j.n, j.acc, bx, by);
  else if (j.form == 1) rows_reduce_body<64>(reinterpret_cast<float4(*)[16]>(red), j.dst, j.slab, j.S, j.n, j.acc, bx, by);
  else rows_reduce1_body(reinterpret_cast<float(*)[64]>(red), j.dst, j.slab, j.S, j.n, j.acc, bx, by);
}

struct DeferQueue {
  bool on = false;
  int count = 0;
  RowsJob q[256];
};
static DeferQueue g_defer;

static int launch_job(const RowsJob& j, hipStream_t st) {
  const dim3 grid((unsigned)j.gx, (unsigned)j.batch);
  if (j.form == 1) hipLaunchKernelGGL(rows_reduce_kernel<64>, grid, dim3(1024), 0, st, j.dst, j.slab, j.S, j.n, j.acc);
  else if (j.form == 0) hipLaunchKernelGGL(rows_reduce_kernel<16>, grid, dim3(1024), 0, st, j.dst, j.slab, j.S, j.n, j.acc);
  else hipLaunchKernelGGL(rows_reduce1_kernel, grid, dim3(1024), 0, st, j.dst, j.slab, j.S, j.n, j.acc);
  return nrse_check_launch("nrse_rows_reduce");
}

extern "C" int nrse_rows_reduce(float* d0, long long n0, float* d1, long long n1, float* d2, long long n2,
                                const float* slab, int S, int batch, int accumulate, void* stream) {
  NRSE_REQUIRE(d0 && n0 > 0 && slab && S >= 1 && batch >= 1, "nrse_rows_reduce: bad args");
  NRSE_REQUIRE((!d1 || n1 > 0) && (!d2 || (d1 && n2 > 0)), "nrse_rows_reduce: destinations d0[, d1[, d2]] in order");
  const RowsJob job = rows_job(d0, n0, d1, n1, d2, n2, slab, S, batch, accumulate);
  if (g_defer.on) {
    NRSE_REQUIRE(g_defer.count < 256, "nrse_rows_reduce: more than 256 deferred reductions (flush first)");
    g_defer.q[g_defer.count++] = job;
    return 0;
  }
  return launch_job(job, (hipStream_t)stream);
}

extern "C" int nrse_reduce_defer(int on) {
  const int prev = g_defer.on ? 1 : 0;
  g_defer.on = on != 0;
  return prev;
}

extern "C" int nrse_reduce_pending(void) { return g_defer.count; }

extern "C" int nrse_reduce_discard(void) {
  g_defer.count = 0;
  g_defer.on = false;
  return 0;
}

extern "C" int nrse_reduce_flush(void* stream) {
  const hipStream_t st = (hipStream_t)stream;
  int k = 0;
  while (k < g_defer.count) {
    const int m = g_defer.count - k < RJ_MAX ? g_defer.count - k : RJ_MAX;
    if (m == 1) {
      const int rc = launch_job(g_defer.q[k], st);
      if (rc) { g_defer.count = 0; return rc; }
      ++k;
      continue;
    }
    RowsJobs jobs;
    jobs.count = m;
    long long total = 0;
    for (int i = 0; i < m; ++i) {
      jobs.j[i] = g_defer.q[k + i];
      jobs.begin[i] = (int)total;
      total += (long long)jobs.j[i].gx * jobs.j[i].batch;
    }
    jobs.begin[m] = (int)total;
    hipLaunchKernelGGL(rows_reduce_multi_kernel, dim3((unsigned)total), dim3(1024), 0, st, jobs);
    const int rc = nrse_check_launch("nrse_reduce_flush");
    if (rc) { g_defer.count = 0; return rc; }
    k += m;
  }
  g_defer.count = 0;
  return 0;
}
