// Fused on-GPU SNR mix: the per-pair noise augmentation + normalisation the reference runs in
// CPU DataLoader workers (src/data/augment.py:4-66, src/data/noisy_speech_dataset.py:77-129,
// [TF] feature_extraction_wav2vec2.py:78-97 zero_mean_unit_var_norm).
// One 1024-thread workgroup per pair, four streaming passes over L (reductions in f64):
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

}  // namespace

extern "C" int nrse_snr_mix(const float* clean, const float* noise, const int* noise_len, long long noise_stride,
                            const float* snr_db, float* clean_out, float* noisy_out, int* status, float* kscale,
                            double* scratch, int batch, int L, int do_normalize, void* stream) {
  (void)scratch;
  NRSE_REQUIRE(clean && noise && noise_len && snr_db && clean_out && noisy_out && status && batch > 0 && L > 0,
               "nrse_snr_mix: bad args");
  hipLaunchKernelGGL(snr_mix_kernel, dim3(batch), dim3(NT), 0, (hipStream_t)stream, clean, noise, noise_len,
                     noise_stride, snr_db, clean_out, noisy_out, status, kscale, L, do_normalize);
  return nrse_check_launch("nrse_snr_mix");
}
