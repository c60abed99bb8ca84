// BYOL heads and loss: BatchNorm1d (+ReLU) forward/backward over [rows = batch, C] and the
// fused normalised-MSE BYOL loss forward+backward.
//   ProjectionHead / PredictionHead  src/models/multi_layer_heads.py:4-48
//   byol_loss                        src/models/byol.py:104-128
// Tiny (batch x 1-2K) and latency-bound: one thread per column for BN, one wave per row for
// the loss. The Linear layers of the heads run through nrse_gemm (exact f32 path).
#include "common.h"

namespace {

__global__ void bn_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                              float* __restrict__ y, float* __restrict__ rm, float* __restrict__ rv,
                              float* __restrict__ sm, float* __restrict__ si, int rows, int C, float momentum,
                              float eps, int train, int relu) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mean, invstd;
  if (train) {
    float s = 0.f;
    for (int r = 0; r < rows; ++r) s += x[(long long)r * C + c];
    mean = s / rows;
    float q = 0.f;
    for (int r = 0; r < rows; ++r) { const float d = x[(long long)r * C + c] - mean; q += d * d; }
    const float var = q / rows;
    invstd = rsqrtf(var + eps);
    if (rm) rm[c] = (1.f - momentum) * rm[c] + momentum * mean;
    if (rv) rv[c] = (1.f - momentum) * rv[c] + momentum * (rows > 1 ? q / (rows - 1) : var);
  } else {
    mean = rm[c];
    invstd = rsqrtf(rv[c] + eps);
  }
  if (sm) sm[c] = mean;
  if (si) si[c] = invstd;
  const float ww = w[c], bb = b[c];
  for (int r = 0; r < rows; ++r) {
    float v = (x[(long long)r * C + c] - mean) * invstd * ww + bb;
    if (relu) v = fmaxf(v, 0.f);
    y[(long long)r * C + c] = v;
  }
}

__global__ void bn_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ y,
                              const float* __restrict__ w, const float* __restrict__ sm, const float* __restrict__ si,
                              float* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db, int rows, int C,
                              int relu) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mean = sm[c], invstd = si[c];
  float sdy = 0.f, sdyx = 0.f;
  for (int r = 0; r < rows; ++r) {
    const long long i = (long long)r * C + c;
    float g = dy[i];
    if (relu && !(y[i] > 0.f)) g = 0.f;
    sdy += g;
    sdyx += g * (x[i] - mean) * invstd;
  }
  dw[c] += sdyx;
  db[c] += sdy;
  const float k = w[c] * invstd / rows;
  for (int r = 0; r < rows; ++r) {
    const long long i = (long long)r * C + c;
    float g = dy[i];
    if (relu && !(y[i] > 0.f)) g = 0.f;
    const float xh = (x[i] - mean) * invstd;
    dx[i] = k * (rows * g - sdy - xh * sdyx);
  }
}

// ---- SyncBatchNorm (DDP option): batch statistics over every rank's rows. Phase 1 reduces the
// local rows into sums, the caller all-reduces them (RCCL), phase 2 normalises with the global
// statistics (torch.nn.SyncBatchNorm semantics: biased var to normalise, unbiased N/(N-1) into
// the running var; backward with the all-reduced sum(dy), sum(dy*xhat)).
__global__ void bn_stats_kernel(const float* __restrict__ x, double* __restrict__ sums, int rows, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int r = 0; r < rows; ++r) { const double v = x[(long long)r * C + c]; s += v; q += v * v; }
  sums[c] = s;
  sums[C + c] = q;
}

__global__ void bn_fwd_global_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                     const float* __restrict__ b, float* __restrict__ y, float* __restrict__ rm,
                                     float* __restrict__ rv, float* __restrict__ sm, float* __restrict__ si,
                                     const double* __restrict__ gsums, long long N, int rows, int C, float momentum,
                                     float eps, int relu) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double m = gsums[c] / (double)N;
  const double var = fmax(gsums[C + c] / (double)N - m * m, 0.0);
  const float mean = (float)m, invstd = rsqrtf((float)var + eps);
  if (rm) rm[c] = (1.f - momentum) * rm[c] + momentum * mean;
  if (rv) rv[c] = (1.f - momentum) * rv[c] + momentum * (float)(N > 1 ? var * N / (N - 1) : var);
  sm[c] = mean;
  si[c] = invstd;
  const float ww = w[c], bb = b[c];
  for (int r = 0; r < rows; ++r) {
    float v = (x[(long long)r * C + c] - mean) * invstd * ww + bb;
    if (relu) v = fmaxf(v, 0.f);
    y[(long long)r * C + c] = v;
  }
}

__global__ void bn_bwd_sums_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                   const float* __restrict__ y, const float* __restrict__ sm,
                                   const float* __restrict__ si, float* __restrict__ sums, int rows, int C, int relu) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mean = sm[c], invstd = si[c];
  float sdy = 0.f, sdyx = 0.f;
  for (int r = 0; r < rows; ++r) {
    const long long i = (long long)r * C + c;
    float g = dy[i];
    if (relu && !(y[i] > 0.f)) g = 0.f;
    sdy += g;
    sdyx += g * (x[i] - mean) * invstd;
  }
  sums[c] = sdy;
  sums[C + c] = sdyx;
}

__global__ void bn_bwd_global_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                     const float* __restrict__ y, const float* __restrict__ w,
                                     const float* __restrict__ sm, const float* __restrict__ si,
                                     const float* __restrict__ lsums, const float* __restrict__ gsums, long long N,
                                     float* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db, int rows,
                                     int C, int relu) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mean = sm[c], invstd = si[c];
  dw[c] += lsums[C + c];   // this rank's share; the gradient all-reduce sums the shares
  db[c] += lsums[c];
  const float gm = gsums[c] / (float)N, gx = gsums[C + c] / (float)N;
  const float k = w[c] * invstd;
  for (int r = 0; r < rows; ++r) {
    const long long i = (long long)r * C + c;
    float g = dy[i];
    if (relu && !(y[i] > 0.f)) g = 0.f;
    const float xh = (x[i] - mean) * invstd;
    dx[i] = k * (g - gm - xh * gx);
  }
}

// one wave per row
__global__ __launch_bounds__(256) void byol_loss_kernel(const float* __restrict__ p, const float* __restrict__ z,
                                                        float* __restrict__ loss, float* __restrict__ dp,
                                                        float* __restrict__ stats, int rows, int D, float gscale,
                                                        float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* pr = p + (long long)r * D;
  const float* zr = z + (long long)r * D;
  float spp = 0.f, szz = 0.f, spz = 0.f;
  int nan0 = 0;
  for (int d = lane; d < D; d += 64) {
    const float a = pr[d], b = zr[d];
    nan0 |= (isnan(a) || isnan(b));
    const float a1 = a + 1e-10f, b1 = b + 1e-10f;
    spp += a1 * a1; szz += b1 * b1; spz += a1 * b1;
  }
  spp = wave_sum(spp); szz = wave_sum(szz); spz = wave_sum(spz);
  const float np_ = sqrtf(spp), nz = sqrtf(szz);
  const float dp_ = fmaxf(np_, 1e-10f), dz = fmaxf(nz, 1e-10f);
  const float s = spz / (dp_ * dz);
  const float sc = fminf(fmaxf(s, -1.f), 1.f);
  nan0 = __any(nan0);
  const int nan1 = isnan(s);
  if (lane == 0) {
    const float lr = -2.f * sc / rows + (r == 0 ? 2.f : 0.f);
    if (part) {
      // row r of the [rows][1 (+2)] partial slab: loss term (and NaN flags), added in row order
      float* pr_ = part + (long long)r * (stats ? 3 : 1);
      pr_[0] = lr;
      if (stats) { pr_[1] = nan0 ? 1.f : 0.f; pr_[2] = nan1 ? 1.f : 0.f; }
    } else {
      atomicAdd(loss, lr);
      if (stats) {
        if (nan0) atomicAdd(stats + 0, 1.f);
        if (nan1) atomicAdd(stats + 1, 1.f);
      }
    }
  }
  if (!dp) return;
  // dL/ds = -2/rows inside the clamp range (torch.clamp passes the gradient at the bounds)
  const float gs = (s >= -1.f && s <= 1.f) ? (-2.f / rows) * gscale : 0.f;
  for (int d = lane; d < D; d += 64) {
    const float a1 = pr[d] + 1e-10f, b1 = zr[d] + 1e-10f;
    // s = <a1, b1> / (max(|a1|,eps) max(|b1|,eps))
    float g = b1 / (dp_ * dz);
    if (np_ > 1e-10f) g -= s * a1 / (np_ * np_);
    dp[(long long)r * D + d] = gs * g;
  }
}

}  // namespace

extern "C" int nrse_bn_fwd(const float* x, const float* w, const float* b, float* y, float* rm, float* rv, float* sm,
                           float* si, int rows, int C, float momentum, float eps, int train, int relu, void* stream) {
  NRSE_REQUIRE(x && w && b && y && rows > 0 && C > 0, "nrse_bn_fwd: bad args");
  NRSE_REQUIRE(train || (rm && rv), "nrse_bn_fwd: eval mode needs running stats");
  if (train && rows < 2) { nrse_set_error("nrse_bn_fwd: Expected more than 1 value per channel when training"); return NRSE_ERR_ARG; }
  hipLaunchKernelGGL(bn_fwd_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, w, b, y, rm, rv, sm,
                     si, rows, C, momentum, eps, train, relu);
  return nrse_check_launch("nrse_bn_fwd");
}

extern "C" int nrse_bn_bwd(const float* dy, const float* x, const float* y, const float* w, const float* sm,
                           const float* si, float* dx, float* dw, float* db, int rows, int C, int relu, void* stream) {
  NRSE_REQUIRE(dy && x && w && sm && si && dx && dw && db && rows > 0 && C > 0 && (!relu || y), "nrse_bn_bwd: bad args");
  hipLaunchKernelGGL(bn_bwd_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, dy, x, y, w, sm, si, dx,
                     dw, db, rows, C, relu);
  return nrse_check_launch("nrse_bn_bwd");
}

extern "C" int nrse_bn_stats(const float* x, double* sums, int rows, int C, void* stream) {
  NRSE_REQUIRE(x && sums && rows > 0 && C > 0, "nrse_bn_stats: bad args");
  hipLaunchKernelGGL(bn_stats_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, sums, rows, C);
  return nrse_check_launch("nrse_bn_stats");
}

extern "C" int nrse_bn_fwd_global(const float* x, const float* w, const float* b, float* y, float* rm, float* rv,
                                  float* sm, float* si, const double* gsums, long long nglobal, int rows, int C,
                                  float momentum, float eps, int relu, void* stream) {
  NRSE_REQUIRE(x && w && b && y && sm && si && gsums && rows > 0 && C > 0 && nglobal >= rows,
               "nrse_bn_fwd_global: bad args");
  if (nglobal < 2) { nrse_set_error("nrse_bn_fwd_global: Expected more than 1 value per channel when training"); return NRSE_ERR_ARG; }
  hipLaunchKernelGGL(bn_fwd_global_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, w, b, y, rm,
                     rv, sm, si, gsums, nglobal, rows, C, momentum, eps, relu);
  return nrse_check_launch("nrse_bn_fwd_global");
}

extern "C" int nrse_bn_bwd_sums(const float* dy, const float* x, const float* y, const float* sm, const float* si,
                                float* sums, int rows, int C, int relu, void* stream) {
  NRSE_REQUIRE(dy && x && sm && si && sums && rows > 0 && C > 0 && (!relu || y), "nrse_bn_bwd_sums: bad args");
  hipLaunchKernelGGL(bn_bwd_sums_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, dy, x, y, sm, si,
                     sums, rows, C, relu);
  return nrse_check_launch("nrse_bn_bwd_sums");
}

extern "C" int nrse_bn_bwd_global(const float* dy, const float* x, const float* y, const float* w, const float* sm,
                                  const float* si, const float* local_sums, const float* global_sums, long long nglobal,
                                  float* dx, float* dw, float* db, int rows, int C, int relu, void* stream) {
  NRSE_REQUIRE(dy && x && w && sm && si && local_sums && global_sums && dx && dw && db && rows > 0 && C > 0 &&
               nglobal >= rows && (!relu || y), "nrse_bn_bwd_global: bad args");
  hipLaunchKernelGGL(bn_bwd_global_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, dy, x, y, w, sm,
                     si, local_sums, global_sums, nglobal, dx, dw, db, rows, C, relu);
  return nrse_check_launch("nrse_bn_bwd_global");
}

extern "C" int nrse_byol_loss(const float* p, const float* z, float* loss, float* dp, float* stats, int rows, int D,
                              float gscale, float* part, void* stream) {
  NRSE_REQUIRE(p && z && loss && rows > 0 && D > 0, "nrse_byol_loss: bad args");
  hipLaunchKernelGGL(byol_loss_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, p, z, loss, dp, stats,
                     rows, D, gscale, part);
  const int rc = nrse_check_launch("nrse_byol_loss");
  if (rc || !part) return rc;
  return nrse_rows_reduce(loss, 1, stats, stats ? 2 : 0, nullptr, 0, part, rows, 1, 1, stream);
}
