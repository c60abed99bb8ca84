// Downstream emotion head kernels (BASELINE configs[3]: the dimensional-emotion head over the
// frozen BYOL encoder, src/models/emotion.py):
//   attentive statistics pooling  src/models/pool.py:25-58 (AttentiveStatisticsPooling)
//   CCC loss                      src/train/dimentional_emotions.py:427-450 (ccc_loss)
// The sap_linear projection (+tanh) runs on nrse_gemm (NRSE_EPI_TANH) and the FC/LayerNorm/ReLU
// layers on nrse_gemm / nrse_layernorm (NRSE_LN_RELU); these kernels hold the per-utterance
// softmax-weighted statistics, whose length mask (feat_len = (wav_len - 1) // 320 + 1,
// pool.py:11-19) makes them a ragged per-row reduction rather than a GEMM.
//
// One workgroup (256 threads = 4 waves) per utterance; C % 256 == 0, C <= 2048. Column sweeps:
// each thread owns 4 consecutive channels per 1024; frame dot products: one wave per frame,
// each lane C/256 groups of 4 channels.
#include "common.h"

namespace {

constexpr float ASP_VAR_MIN = 1e-5f;  // clamp(min=1e-5) inside the sqrt (pool.py:53)

template <typename T> NRSE_DEV void ld4x(const void* p, long long i, float* o);
template <> NRSE_DEV void ld4x<float>(const void* p, long long i, float* o) {
  const float4 v = *reinterpret_cast<const float4*>((const float*)p + i);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <> NRSE_DEV void ld4x<bf16_t>(const void* p, long long i, float* o) {
  const uint2 v = *reinterpret_cast<const uint2*>((const bf16_t*)p + i);
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
}
template <typename T> NRSE_DEV void st4x(void* p, long long i, const float* v);
template <> NRSE_DEV void st4x<float>(void* p, long long i, const float* v) {
  *reinterpret_cast<float4*>((float*)p + i) = make_float4(v[0], v[1], v[2], v[3]);
}
template <> NRSE_DEV void st4x<bf16_t>(void* p, long long i, const float* v) {
  uint2 u;
  u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *reinterpret_cast<uint2*>((bf16_t*)p + i) = u;
}

NRSE_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}
NRSE_DEV float block_max(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// logits[t] = h[t, :] . att for t < len (one wave per frame, lane = 4-channel groups)
template <int NG>
NRSE_DEV void frame_dots(const float* h, const float* att, int C, int len, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float a[NG][4];
#pragma unroll
  for (int g = 0; g < NG; ++g) ld4x<float>(att, (g * 64 + lane) * 4, a[g]);
  for (int t = w; t < len; t += 4) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      float x[4];
      ld4x<float>(h, (long long)t * C + (g * 64 + lane) * 4, x);
      s += x[0] * a[g][0] + x[1] * a[g][1] + x[2] * a[g][2] + x[3] * a[g][3];
    }
    s = wave_sum(s);
    if (lane == 0) out[t] = s;
  }
}

// pooled[b] = [mu, sqrt(max(var, 1e-5))], mu = sum_t w_t x_t, var = sum_t w_t x_t^2 - mu^2,
// w = softmax_t(tanh(sap(x)) . att) over the first len frames. Saves w [B, T] and var [B, C].
template <typename T, int NG>
__global__ __launch_bounds__(256) void asp_fwd_kernel(const void* __restrict__ x, const float* __restrict__ h,
                                                      const float* __restrict__ att, const int* __restrict__ lens,
                                                      int Tn, int C, float* __restrict__ w_out,
                                                      float* __restrict__ var_out, float* __restrict__ pooled) {
  extern __shared__ float lg[];  // [Tn]
  __shared__ float red[4];
  const int b = blockIdx.x;
  const int len = min(max(lens[b], 1), Tn);
  const float* hb = h + (long long)b * Tn * C;
  frame_dots<NG / 4>(hb, att, C, len, lg);
  __syncthreads();
  float mx = -INFINITY;
  for (int t = threadIdx.x; t < len; t += 256) mx = fmaxf(mx, lg[t]);
  mx = block_max(mx, red);
  float se = 0.f;
  for (int t = threadIdx.x; t < len; t += 256) {
    const float e = __expf(lg[t] - mx);
    lg[t] = e;
    se += e;
  }
  se = block_sum(se, red);
  const float inv = 1.f / se;
  for (int t = threadIdx.x; t < Tn; t += 256) {
    const float wt = t < len ? lg[t] * inv : 0.f;
    if (t < len) lg[t] = wt;
    w_out[(long long)b * Tn + t] = wt;
  }
  __syncthreads();
  const long long xb = (long long)b * Tn * C;
  for (int c0 = threadIdx.x * 4; c0 < C; c0 += 1024) {
    float mu[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < len; ++t) {
      float v[4];
      ld4x<T>(x, xb + (long long)t * C + c0, v);
      const float wt = lg[t];
#pragma unroll
      for (int e = 0; e < 4; ++e) { mu[e] = fmaf(wt, v[e], mu[e]); s2[e] = fmaf(wt, v[e] * v[e], s2[e]); }
    }
    float var[4], rh[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      var[e] = s2[e] - mu[e] * mu[e];
      rh[e] = sqrtf(fmaxf(var[e], ASP_VAR_MIN));
    }
    st4x<float>(pooled, (long long)b * 2 * C + c0, mu);
    st4x<float>(pooled, (long long)b * 2 * C + C + c0, rh);
    st4x<float>(var_out, (long long)b * C + c0, var);
  }
}

// Backward to the pooling's inputs that carry parameters: dpre [B, T, C] = d(sap pre-activation)
// (zero on frames >= len) and datt [C] (accumulated). The encoder is frozen: no dx.
template <typename T, typename TD, int NG>
__global__ __launch_bounds__(256) void asp_bwd_kernel(const void* __restrict__ x, const float* __restrict__ h,
                                                      const float* __restrict__ att, const int* __restrict__ lens,
                                                      int Tn, int C, const float* __restrict__ w_in,
                                                      const float* __restrict__ var_in, const float* __restrict__ pooled,
                                                      const float* __restrict__ dpooled, void* __restrict__ dpre,
                                                      float* __restrict__ datt) {
  extern __shared__ float sm[];  // dA [C], dB [C], dw [Tn]
  float* dA = sm;
  float* dB = sm + C;
  float* dw = sm + 2 * C;
  __shared__ float red[4];
  const int b = blockIdx.x;
  const int len = min(max(lens[b], 1), Tn);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // per channel: mu = sum w x, var = sum w x^2 - mu^2, rh = sqrt(max(var, 1e-5))
  //   dvar = drh / (2 rh) (0 where clamped), dA = dmu - 2 mu dvar, dB = dvar
  for (int c = threadIdx.x; c < C; c += 256) {
    const float mu = pooled[(long long)b * 2 * C + c], rh = pooled[(long long)b * 2 * C + C + c];
    const float dmu = dpooled[(long long)b * 2 * C + c], drh = dpooled[(long long)b * 2 * C + C + c];
    const float dvar = var_in[(long long)b * C + c] > ASP_VAR_MIN ? drh / (2.f * rh) : 0.f;
    dA[c] = dmu - 2.f * mu * dvar;
    dB[c] = dvar;
  }
  __syncthreads();
  // dw_t = sum_c dA x + dB x^2
  const long long xb = (long long)b * Tn * C;
  for (int t = w; t < len; t += 4) {
    float s = 0.f;
    for (int g = 0; g < NG / 4; ++g) {
      const int c0 = (g * 64 + lane) * 4;
      float v[4];
      ld4x<T>(x, xb + (long long)t * C + c0, v);
#pragma unroll
      for (int e = 0; e < 4; ++e) s += v[e] * (dA[c0 + e] + dB[c0 + e] * v[e]);
    }
    s = wave_sum(s);
    if (lane == 0) dw[t] = s;
  }
  __syncthreads();
  // softmax backward: dlogit_t = w_t (dw_t - sum_tau w_tau dw_tau)
  float sw = 0.f;
  for (int t = threadIdx.x; t < len; t += 256) sw += w_in[(long long)b * Tn + t] * dw[t];
  sw = block_sum(sw, red);
  for (int t = threadIdx.x; t < len; t += 256) dw[t] = w_in[(long long)b * Tn + t] * (dw[t] - sw);
  __syncthreads();
  // dpre = dlogit_t att (1 - h^2); datt += sum_t dlogit_t h
  const float* hb = h + (long long)b * Tn * C;
  for (int c0 = threadIdx.x * 4; c0 < C; c0 += 1024) {
    float a[4], da[4] = {0.f, 0.f, 0.f, 0.f};
    ld4x<float>(att, c0, a);
    for (int t = 0; t < Tn; ++t) {
      float o[4] = {0.f, 0.f, 0.f, 0.f};
      if (t < len) {
        float hv[4];
        ld4x<float>(hb, (long long)t * C + c0, hv);
        const float dl = dw[t];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = dl * a[e] * (1.f - hv[e] * hv[e]);
          da[e] = fmaf(dl, hv[e], da[e]);
        }
      }
      st4x<TD>(dpre, xb + (long long)t * C + c0, o);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(datt + c0 + e, da[e]);
  }
}

// ccc_loss (dimentional_emotions.py:427-450): loss = mean_d (1 - 2 cov / (var_p + var_t +
// (mean_p - mean_t)^2 + 1e-10)), biased variances; 0 (and zero gradient) when rows <= 1.
__global__ __launch_bounds__(256) void ccc_kernel(const float* __restrict__ pred, int ld,
                                                  const float* __restrict__ tgt, float* __restrict__ loss,
                                                  float* __restrict__ dpred, int rows, int D) {
  __shared__ float red[4];
  float total = 0.f;
  for (int d = 0; d < D; ++d) {
    if (rows <= 1) break;
    float sp = 0.f, st = 0.f;
    for (int i = threadIdx.x; i < rows; i += 256) { sp += pred[i * ld + d]; st += tgt[i * D + d]; }
    const float mp = block_sum(sp, red) / rows;
    const float mt = block_sum(st, red) / rows;
    float vp = 0.f, vt = 0.f, cv = 0.f;
    for (int i = threadIdx.x; i < rows; i += 256) {
      const float a = pred[i * ld + d] - mp, c = tgt[i * D + d] - mt;
      vp += a * a; vt += c * c; cv += a * c;
    }
    vp = block_sum(vp, red) / rows;
    vt = block_sum(vt, red) / rows;
    cv = block_sum(cv, red) / rows;
    const float dm = mp - mt;
    const float N = vp + vt + dm * dm + 1e-10f;
    const float ccc = 2.f * cv / N;
    total += 1.f - ccc;
    if (dpred) {
      // dloss/dp_i = -(1/D) [2 (t_i - mt) / (rows N) - 2 cv (2 (p_i - mp) + 2 dm) / (rows N^2)]
      for (int i = threadIdx.x; i < rows; i += 256) {
        const float a = pred[i * ld + d] - mp, c = tgt[i * D + d] - mt;
        const float g = 2.f * c / (rows * N) - 2.f * cv * (2.f * a + 2.f * dm) / (rows * N * N);
        dpred[i * ld + d] = -g / D;
      }
    }
  }
  if (rows <= 1 && dpred)
    for (int i = threadIdx.x; i < rows * D; i += 256) dpred[(i / D) * ld + i % D] = 0.f;
  if (threadIdx.x == 0) loss[0] = total / D;
}

}  // namespace

extern "C" int nrse_asp_fwd(const void* x, int x_dtype, const float* h, const float* att, const int* lens, int batch,
                            int T, int C, float* w_out, float* var_out, float* pooled, void* stream) {
  NRSE_REQUIRE(x && h && att && lens && w_out && var_out && pooled && batch > 0 && T > 0, "nrse_asp_fwd: bad args");
  NRSE_REQUIRE(C % 256 == 0 && C <= 2048, "nrse_asp_fwd: C=%d must be a multiple of 256, <= 2048", C);
  const size_t lds = (size_t)T * sizeof(float);
  NRSE_REQUIRE(lds <= 64 * 1024, "nrse_asp_fwd: T=%d too long", T);
  hipStream_t st = (hipStream_t)stream;
  const int NG = C / 64;
#define NRSE_ASP_FWD(TT, G) \
  hipLaunchKernelGGL((asp_fwd_kernel<TT, G>), dim3(batch), dim3(256), lds, st, x, h, att, lens, T, C, w_out, var_out, pooled)
  if (x_dtype == NRSE_BF16) {
    switch (NG) {
      case 4: NRSE_ASP_FWD(bf16_t, 4); break;
      case 8: NRSE_ASP_FWD(bf16_t, 8); break;
      case 16: NRSE_ASP_FWD(bf16_t, 16); break;
      case 32: NRSE_ASP_FWD(bf16_t, 32); break;
      default: nrse_set_error("nrse_asp_fwd: C=%d", C); return NRSE_ERR_UNSUPPORTED;
    }
  } else {
    switch (NG) {
      case 4: NRSE_ASP_FWD(float, 4); break;
      case 8: NRSE_ASP_FWD(float, 8); break;
      case 16: NRSE_ASP_FWD(float, 16); break;
      case 32: NRSE_ASP_FWD(float, 32); break;
      default: nrse_set_error("nrse_asp_fwd: C=%d", C); return NRSE_ERR_UNSUPPORTED;
    }
  }
#undef NRSE_ASP_FWD
  return nrse_check_launch("nrse_asp_fwd");
}

extern "C" int nrse_asp_bwd(const void* x, int x_dtype, const float* h, const float* att, const int* lens, int batch,
                            int T, int C, const float* w_in, const float* var_in, const float* pooled,
                            const float* dpooled, void* dpre, int dpre_dtype, float* datt, void* stream) {
  NRSE_REQUIRE(x && h && att && lens && w_in && var_in && pooled && dpooled && dpre && datt && batch > 0 && T > 0,
               "nrse_asp_bwd: bad args");
  NRSE_REQUIRE(C % 256 == 0 && C <= 2048, "nrse_asp_bwd: C=%d must be a multiple of 256, <= 2048", C);
  const size_t lds = (size_t)(2 * C + T) * sizeof(float);
  NRSE_REQUIRE(lds <= 64 * 1024, "nrse_asp_bwd: T=%d too long", T);
  hipStream_t st = (hipStream_t)stream;
  const int NG = C / 64;
#define NRSE_ASP_BWD(TT, TD, G)                                                                                  \
  hipLaunchKernelGGL((asp_bwd_kernel<TT, TD, G>), dim3(batch), dim3(256), lds, st, x, h, att, lens, T, C, w_in, \
                     var_in, pooled, dpooled, dpre, datt)
#define NRSE_ASP_BWD_G(TT, TD)                                              \
  switch (NG) {                                                             \
    case 4: NRSE_ASP_BWD(TT, TD, 4); break;                                 \
    case 8: NRSE_ASP_BWD(TT, TD, 8); break;                                 \
    case 16: NRSE_ASP_BWD(TT, TD, 16); break;                               \
    case 32: NRSE_ASP_BWD(TT, TD, 32); break;                               \
    default: nrse_set_error("nrse_asp_bwd: C=%d", C); return NRSE_ERR_UNSUPPORTED; \
  }
  if (x_dtype == NRSE_BF16 && dpre_dtype == NRSE_BF16) { NRSE_ASP_BWD_G(bf16_t, bf16_t) }
  else if (x_dtype == NRSE_BF16) { NRSE_ASP_BWD_G(bf16_t, float) }
  else if (dpre_dtype == NRSE_BF16) { NRSE_ASP_BWD_G(float, bf16_t) }
  else { NRSE_ASP_BWD_G(float, float) }
#undef NRSE_ASP_BWD_G
#undef NRSE_ASP_BWD
  return nrse_check_launch("nrse_asp_bwd");
}

extern "C" int nrse_ccc_loss(const float* pred, int ld, const float* target, float* loss, float* dpred, int rows,
                             int D, void* stream) {
  NRSE_REQUIRE(pred && target && loss && rows > 0 && D > 0 && ld >= D, "nrse_ccc_loss: bad args");
  hipLaunchKernelGGL(ccc_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, pred, ld, target, loss, dpred, rows, D);
  return nrse_check_launch("nrse_ccc_loss");
}
