// Fused on-GPU SNR mix: the per-pair noise augmentation + normalisation the reference runs in
// CPU DataLoader workers (src/data/augment.py:4-66, src/data/noisy_speech_dataset.py:77-129,
// [TF] feature_extraction_wav2vec2.py:78-97 zero_mean_unit_var_norm).
// Four streaming passes over L (reductions in f64), as one 1024-thread workgroup per pair (no
// scratch) or as four launches over (chunk, pair) workgroups (scratch, below):
//   1: sum/sumsq of speech and tiled noise, max|s|, NaN flags   -> k = sqrt(Ps/(Pn*10^(snr/10)))
//   2: max|s + k n|
//   3: mean/var of the peak-normalised views (feature-extractor normalisation)
//   4: write clean_input_values / noisy_input_values
// Status codes match oracle/snr_mix.py (0 ok; failing pairs get zeroed outputs).
#include "common.h"

namespace {

constexpr int NT = 1024;

NRSE_DEV double block_sum(double v, double* red) {
  v = wave_sum_d(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}
NRSE_DEV float block_max(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = red[0];
  for (int i = 1; i < NT / 64; ++i) s = fmaxf(s, red[i]);
  return s;
}

__global__ __launch_bounds__(NT) void snr_mix_kernel(const float* __restrict__ clean, const float* __restrict__ noise,
                                                     const int* __restrict__ nlen, long long nstride,
                                                     const float* __restrict__ snr_db, float* __restrict__ cout,
                                                     float* __restrict__ nout, int* __restrict__ status,
                                                     float* __restrict__ kscale, int L, int do_norm) {
  __shared__ double redd[NT / 64];
  __shared__ float redf[NT / 64];
  const int b = blockIdx.x;
  const float* s = clean + (long long)b * L;
  const float* n = noise + (long long)b * nstride;
  const int Ln = nlen[b];
  float* co = cout + (long long)b * L;
  float* no = nout + (long long)b * L;

  // pass 1
  double ss = 0.0, ssq = 0.0, nsq = 0.0;
  float smax = 0.f;
  int snan = 0, nnan = 0;
  for (int t = threadIdx.x; t < L; t += NT) {
    const float a = s[t];
    snan |= isnan(a);
    const float c = n[Ln >= L ? t : t % Ln];
    ss += a;
    ssq += (double)a * a;
    nsq += (double)c * c;
    smax = fmaxf(smax, fabsf(a));
  }
  for (int t = threadIdx.x; t < Ln; t += NT) nnan |= isnan(n[t]);
  ss = block_sum(ss, redd);
  ssq = block_sum(ssq, redd);
  nsq = block_sum(nsq, redd);
  smax = block_max(smax, redf);
  snan = __syncthreads_or(snan);
  nnan = __syncthreads_or(nnan);

  const float ps = (float)(ssq / L), pn = (float)(nsq / L);
  int st = 0;
  float k = 0.f;
  if (snan) st = 1;
  else if (nnan) st = 2;
  else if (ps < 1e-10f) st = 3;
  else if (pn < 1e-10f) st = 4;
  else {
    const float snr_lin = (float)pow(10.0, (double)snr_db[b] / 10.0);
    k = sqrtf(ps / (pn * snr_lin));
    if (isinf(k) || isnan(k)) st = 5;
    else if (k > 1e6f) st = 6;
  }
  // pass 2: noisy peak
  float ymax = 0.f;
  int ynan = 0;
  if (st == 0) {
    for (int t = threadIdx.x; t < L; t += NT) {
      const float y = s[t] + n[Ln >= L ? t : t % Ln] * k;
      ynan |= isnan(y);
      ymax = fmaxf(ymax, fabsf(y));
    }
  }
  ymax = block_max(ymax, redf);
  ynan = __syncthreads_or(ynan);
  if (st == 0 && ynan) st = 7;
  // mode 0 = add_noise_to_speech only (augment.py:4-66); 1 = + peak normalisation
  // (noisy_speech_dataset.py:88-103); 2 = + feature-extractor zero-mean/unit-var
  const int mode = do_norm;
  if (mode >= 1 && st == 0 && smax < 1e-8f) st = 8;
  if (mode >= 1 && st == 0 && ymax < 1e-8f) st = 9;
  const float cden = mode >= 1 ? smax + 1e-8f : 1.f, yden = mode >= 1 ? ymax + 1e-8f : 1.f;
  do_norm = mode == 2;
  // pass 3: statistics of the peak-normalised views
  double cs = 0.0, cq = 0.0, ys = 0.0, yq = 0.0;
  if (st == 0 && do_norm) {
    for (int t = threadIdx.x; t < L; t += NT) {
      const float c = s[t] / cden;
      const float y = (s[t] + n[Ln >= L ? t : t % Ln] * k) / yden;
      cs += c; cq += (double)c * c; ys += y; yq += (double)y * y;
    }
  }
  cs = block_sum(cs, redd);
  cq = block_sum(cq, redd);
  ys = block_sum(ys, redd);
  yq = block_sum(yq, redd);
  const double cm = cs / L, ym = ys / L;
  const float cmean = (float)cm, ymean = (float)ym;
  const float cinv = do_norm ? (float)(1.0 / sqrt(fmax(cq / L - cm * cm, 0.0) + 1e-7)) : 1.f;
  const float yinv = do_norm ? (float)(1.0 / sqrt(fmax(yq / L - ym * ym, 0.0) + 1e-7)) : 1.f;
  // pass 4
  for (int t = threadIdx.x; t < L; t += NT) {
    float c = 0.f, y = 0.f;
    if (st == 0) {
      c = s[t] / cden;
      y = (s[t] + n[Ln >= L ? t : t % Ln] * k) / yden;
      if (do_norm) { c = (c - cmean) * cinv; y = (y - ymean) * yinv; }
    }
    co[t] = c;
    no[t] = y;
  }
  if (threadIdx.x == 0) {
    status[b] = st;
    if (kscale) kscale[b] = k;
  }
}

// ---------------------------------------------------------------------------------------------
// Chunked form (scratch given): the same four passes as four launches over (chunk, pair) grids of
// SNR_CHUNKS x batch workgroups, so 32 pairs occupy 512 workgroups instead of 32 (the one-
// workgroup-per-pair kernel ran ~0.6 ms, latency-bound on 32 CUs). Each pass writes per-chunk
// partials (f64) to scratch; the next pass first folds its pair's partials in chunk order
// (deterministic, every workgroup of the pair computes the same values), then streams its chunk.
constexpr int SNR_CHUNKS = 16;
constexpr int SNR_REC = 16;  // doubles per (pair, chunk) record
enum { R_SS, R_SSQ, R_NSQ, R_SMAX, R_SNAN, R_NNAN, R_YMAX, R_YNAN, R_CS, R_CQ, R_YS, R_YQ };
constexpr int CT = 256;

NRSE_DEV double cblock_sum(double v, double* red) {
  v = wave_sum_d(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}
NRSE_DEV float cblock_max(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

struct SnrState {
  int st;
  float k, cden, yden, cmean, ymean, cinv, yinv;
  bool norm;
};

// fold the pair's chunk records up to `phase` and derive the mix constants (the single-workgroup
// kernel's formulas, in the same order)
NRSE_DEV SnrState snr_state(const double* rec, int phase, float snr_db, int L, int mode) {
  double a[SNR_REC];
#pragma unroll
  for (int f = 0; f < SNR_REC; ++f) a[f] = 0.0;
  for (int c = 0; c < SNR_CHUNKS; ++c) {
    const double* r = rec + c * SNR_REC;
    a[R_SS] += r[R_SS]; a[R_SSQ] += r[R_SSQ]; a[R_NSQ] += r[R_NSQ];
    a[R_SMAX] = fmax(a[R_SMAX], r[R_SMAX]);
    a[R_SNAN] += r[R_SNAN]; a[R_NNAN] += r[R_NNAN];
    if (phase >= 3) { a[R_YMAX] = fmax(a[R_YMAX], r[R_YMAX]); a[R_YNAN] += r[R_YNAN]; }
    if (phase >= 4) { a[R_CS] += r[R_CS]; a[R_CQ] += r[R_CQ]; a[R_YS] += r[R_YS]; a[R_YQ] += r[R_YQ]; }
  }
  SnrState S{};
  const float ps = (float)(a[R_SSQ] / L), pn = (float)(a[R_NSQ] / L);
  S.st = 0;
  S.k = 0.f;
  if (a[R_SNAN] > 0) S.st = 1;
  else if (a[R_NNAN] > 0) S.st = 2;
  else if (ps < 1e-10f) S.st = 3;
  else if (pn < 1e-10f) S.st = 4;
  else {
    const float snr_lin = (float)pow(10.0, (double)snr_db / 10.0);
    S.k = sqrtf(ps / (pn * snr_lin));
    if (isinf(S.k) || isnan(S.k)) S.st = 5;
    else if (S.k > 1e6f) S.st = 6;
  }
  if (phase < 3) return S;
  const float smax = (float)a[R_SMAX], ymax = (float)a[R_YMAX];
  if (S.st == 0 && a[R_YNAN] > 0) S.st = 7;
  if (mode >= 1 && S.st == 0 && smax < 1e-8f) S.st = 8;
  if (mode >= 1 && S.st == 0 && ymax < 1e-8f) S.st = 9;
  S.cden = mode >= 1 ? smax + 1e-8f : 1.f;
  S.yden = mode >= 1 ? ymax + 1e-8f : 1.f;
  S.norm = mode == 2;
  if (phase < 4) return S;
  const double cm = a[R_CS] / L, ym = a[R_YS] / L;
  S.cmean = (float)cm;
  S.ymean = (float)ym;
  S.cinv = S.norm ? (float)(1.0 / sqrt(fmax(a[R_CQ] / L - cm * cm, 0.0) + 1e-7)) : 1.f;
  S.yinv = S.norm ? (float)(1.0 / sqrt(fmax(a[R_YQ] / L - ym * ym, 0.0) + 1e-7)) : 1.f;
  return S;
}

__global__ __launch_bounds__(CT) void snr_chunk_kernel(int phase, const float* __restrict__ clean,
                                                       const float* __restrict__ noise, const int* __restrict__ nlen,
                                                       long long nstride, const float* __restrict__ snr_db,
                                                       float* __restrict__ cout, float* __restrict__ nout,
                                                       int* __restrict__ status, float* __restrict__ kscale,
                                                       double* __restrict__ scratch, int L, int mode) {
  __shared__ double redd[4];
  __shared__ float redf[4];
  const int chunk = blockIdx.x, b = blockIdx.y;
  const float* s = clean + (long long)b * L;
  const float* n = noise + (long long)b * nstride;
  const int Ln = nlen[b];
  double* rec = scratch + (long long)b * SNR_CHUNKS * SNR_REC;
  double* mine = rec + chunk * SNR_REC;
  const int cl = (L + SNR_CHUNKS - 1) / SNR_CHUNKS;
  const int t0 = chunk * cl, t1 = min(L, t0 + cl);
  auto nidx = [&](int t) { return Ln >= L ? t : t % Ln; };
  if (phase == 1) {
    double ss = 0.0, ssq = 0.0, nsq = 0.0;
    float smax = 0.f;
    int snan = 0, nnan = 0;
    for (int t = t0 + threadIdx.x; t < t1; t += CT) {
      const float a = s[t];
      snan |= isnan(a);
      const float c = n[nidx(t)];
      ss += a;
      ssq += (double)a * a;
      nsq += (double)c * c;
      smax = fmaxf(smax, fabsf(a));
    }
    const int nl = (Ln + SNR_CHUNKS - 1) / SNR_CHUNKS;
    for (int t = chunk * nl + threadIdx.x; t < min(Ln, (chunk + 1) * nl); t += CT) nnan |= isnan(n[t]);
    ss = cblock_sum(ss, redd);
    ssq = cblock_sum(ssq, redd);
    nsq = cblock_sum(nsq, redd);
    smax = cblock_max(smax, redf);
    snan = __syncthreads_or(snan);
    nnan = __syncthreads_or(nnan);
    if (threadIdx.x == 0) {
      mine[R_SS] = ss; mine[R_SSQ] = ssq; mine[R_NSQ] = nsq; mine[R_SMAX] = smax;
      mine[R_SNAN] = snan; mine[R_NNAN] = nnan;
    }
    return;
  }
  const SnrState S = snr_state(rec, phase, snr_db[b], L, mode);
  if (phase == 2) {
    float ymax = 0.f;
    int ynan = 0;
    if (S.st == 0) {
      for (int t = t0 + threadIdx.x; t < t1; t += CT) {
        const float y = s[t] + n[nidx(t)] * S.k;
        ynan |= isnan(y);
        ymax = fmaxf(ymax, fabsf(y));
      }
    }
    ymax = cblock_max(ymax, redf);
    ynan = __syncthreads_or(ynan);
    if (threadIdx.x == 0) { mine[R_YMAX] = ymax; mine[R_YNAN] = ynan; }
    return;
  }
  if (phase == 3) {
    double cs = 0.0, cq = 0.0, ys = 0.0, yq = 0.0;
    if (S.st == 0 && S.norm) {
      for (int t = t0 + threadIdx.x; t < t1; t += CT) {
        const float c = s[t] / S.cden;
        const float y = (s[t] + n[nidx(t)] * S.k) / S.yden;
        cs += c; cq += (double)c * c; ys += y; yq += (double)y * y;
      }
    }
    cs = cblock_sum(cs, redd);
    cq = cblock_sum(cq, redd);
    ys = cblock_sum(ys, redd);
    yq = cblock_sum(yq, redd);
    if (threadIdx.x == 0) { mine[R_CS] = cs; mine[R_CQ] = cq; mine[R_YS] = ys; mine[R_YQ] = yq; }
    return;
  }
  float* co = cout + (long long)b * L;
  float* no = nout + (long long)b * L;
  for (int t = t0 + threadIdx.x; t < t1; t += CT) {
    float c = 0.f, y = 0.f;
    if (S.st == 0) {
      c = s[t] / S.cden;
      y = (s[t] + n[nidx(t)] * S.k) / S.yden;
      if (S.norm) { c = (c - S.cmean) * S.cinv; y = (y - S.ymean) * S.yinv; }
    }
    co[t] = c;
    no[t] = y;
  }
  if (chunk == 0 && threadIdx.x == 0) {
    status[b] = S.st;
    if (kscale) kscale[b] = S.k;
  }
}

}  // namespace

extern "C" int nrse_snr_mix(const float* clean, const float* noise, const int* noise_len, long long noise_stride,
                            const float* snr_db, float* clean_out, float* noisy_out, int* status, float* kscale,
                            double* scratch, int batch, int L, int do_normalize, void* stream) {
  NRSE_REQUIRE(clean && noise && noise_len && snr_db && clean_out && noisy_out && status && batch > 0 && L > 0,
               "nrse_snr_mix: bad args");
  hipStream_t st = (hipStream_t)stream;
  if (!scratch) {
    hipLaunchKernelGGL(snr_mix_kernel, dim3(batch), dim3(NT), 0, st, clean, noise, noise_len, noise_stride, snr_db,
                       clean_out, noisy_out, status, kscale, L, do_normalize);
    return nrse_check_launch("nrse_snr_mix");
  }
  const dim3 grid(SNR_CHUNKS, batch);
  for (int phase = 1; phase <= 4; ++phase)
    hipLaunchKernelGGL(snr_chunk_kernel, grid, dim3(CT), 0, st, phase, clean, noise, noise_len, noise_stride, snr_db,
                       clean_out, noisy_out, status, kscale, scratch, L, do_normalize);
  return nrse_check_launch("nrse_snr_mix(chunked)");
}
