// Bit-exactness probe of gfx950's scaled fp6 conversions against the software MXFP6 encoder
// (csrc/common.h e2m3 / mx6_exp, restated by oracle/mx6.py): one lane per 32-value block, random
// bf16 / f32 blocks over a wide exponent range plus the edge values (zeros, ties, the clamp at
// 7.5, subnormals); prints the blocks whose 24 payload bytes differ, for the scale passed as 2^X
// and as 2^-X.
// Build: hipcc --offload-arch=gfx950 -O3 -I noise-robust-speech-embedding_amd/csrc tools/probe_fp6cvt.hip -o tools/probe_fp6cvt
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>

#include "common.h"

typedef __bf16 bf16x32 __attribute__((ext_vector_type(32)));
typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef int i32x6 __attribute__((ext_vector_type(6)));

__global__ void probe(const float* x, int nblk, uint32_t* sw, uint32_t* hw_bf_a, uint32_t* hw_bf_b, uint32_t* hw_f_a,
                      uint32_t* hw_f_b) {
  const int blk = blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= nblk) return;
  const float* v = x + 32LL * blk;
  float am = 0.f;
  for (int j = 0; j < 32; ++j) am = fmaxf(am, fabsf(v[j]));
  const int X = mx6_exp(am);
  const float inv = mx6_inv(X);
  // software: 32 codes packed little-endian at 6j
  uint32_t d[6] = {0, 0, 0, 0, 0, 0};
  for (int j = 0; j < 32; ++j) {
    const uint64_t c = e2m3(v[j] * inv);
    const int bit = 6 * j, w = bit >> 5, o = bit & 31;
    d[w] |= (uint32_t)(c << o);
    if (o > 26) d[w + 1] |= (uint32_t)(c >> (32 - o));
  }
  for (int k = 0; k < 6; ++k) sw[6 * blk + k] = d[k];
  bf16x32 b;
  f32x16v f0, f1;
  for (int j = 0; j < 32; ++j) b[j] = (__bf16)v[j];
  for (int j = 0; j < 16; ++j) { f0[j] = v[j]; f1[j] = v[16 + j]; }
  const float sa = __uint_as_float((uint32_t)(127 + X) << 23);  // 2^X
  const float sb = inv;                                          // 2^-X
  const i32x6 ra = __builtin_amdgcn_cvt_scalef32_pk32_fp6_bf16(b, sa);
  const i32x6 rb = __builtin_amdgcn_cvt_scalef32_pk32_fp6_bf16(b, sb);
  const i32x6 fa = __builtin_amdgcn_cvt_scalef32_2xpk16_fp6_f32(f0, f1, sa);
  const i32x6 fb = __builtin_amdgcn_cvt_scalef32_2xpk16_fp6_f32(f0, f1, sb);
  for (int k = 0; k < 6; ++k) {
    hw_bf_a[6 * blk + k] = ra[k];
    hw_bf_b[6 * blk + k] = rb[k];
    hw_f_a[6 * blk + k] = fa[k];
    hw_f_b[6 * blk + k] = fb[k];
  }
}

static float bf16_round(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u = (u + 0x7fff + ((u >> 16) & 1)) & 0xffff0000u;
  memcpy(&f, &u, 4);
  return f;
}

int main() {
  const int nblk = 1 << 16;
  std::vector<float> h(32LL * nblk);
  srand(7);
  for (int b = 0; b < nblk; ++b) {
    const int e = (rand() % 60) - 30;
    for (int j = 0; j < 32; ++j) {
      float r = ((float)rand() / RAND_MAX * 2.f - 1.f) * ldexpf(1.f, e);
      if (b % 7 == 0 && j % 5 == 0) r = 0.f;
      if (b % 11 == 0) r = ldexpf((float)((rand() % 121) - 60) / 8.f, e);  // grid points, ties
      h[32LL * b + j] = bf16_round(r);  // bf16-representable: both forms see the same values
    }
  }
  float* dx;
  uint32_t *sw, *a, *bb, *fa, *fb;
  hipMalloc(&dx, h.size() * 4);
  hipMalloc(&sw, 24LL * nblk); hipMalloc(&a, 24LL * nblk); hipMalloc(&bb, 24LL * nblk);
  hipMalloc(&fa, 24LL * nblk); hipMalloc(&fb, 24LL * nblk);
  hipMemcpy(dx, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(nblk / 256), dim3(256), 0, 0, dx, nblk, sw, a, bb, fa, fb);
  hipDeviceSynchronize();
  std::vector<uint32_t> S(6LL * nblk), A(6LL * nblk), B(6LL * nblk), FA(6LL * nblk), FB(6LL * nblk);
  hipMemcpy(S.data(), sw, 24LL * nblk, hipMemcpyDeviceToHost);
  hipMemcpy(A.data(), a, 24LL * nblk, hipMemcpyDeviceToHost);
  hipMemcpy(B.data(), bb, 24LL * nblk, hipMemcpyDeviceToHost);
  hipMemcpy(FA.data(), fa, 24LL * nblk, hipMemcpyDeviceToHost);
  hipMemcpy(FB.data(), fb, 24LL * nblk, hipMemcpyDeviceToHost);
  const char* names[4] = {"pk32_bf16 scale 2^X", "pk32_bf16 scale 2^-X", "2xpk16_f32 scale 2^X", "2xpk16_f32 scale 2^-X"};
  std::vector<uint32_t>* hv[4] = {&A, &B, &FA, &FB};
  for (int m = 0; m < 4; ++m) {
    long bad = 0;
    int shown = 0;
    for (int b = 0; b < nblk; ++b) {
      if (memcmp(&S[6LL * b], &(*hv[m])[6LL * b], 24) == 0) continue;
      ++bad;
      if (shown < 3) {
        ++shown;
        printf("  %s block %d:", names[m], b);
        for (int j = 0; j < 32; ++j) {
          const int bit = 6 * j, w = bit >> 5, o = bit & 31;
          uint64_t ws = ((uint64_t)S[6LL * b + w] | ((w < 5 ? (uint64_t)S[6LL * b + w + 1] : 0) << 32)) >> o;
          uint64_t wh = ((uint64_t)(*hv[m])[6LL * b + w] | ((w < 5 ? (uint64_t)(*hv[m])[6LL * b + w + 1] : 0) << 32)) >> o;
          if ((ws & 63) != (wh & 63)) printf(" [%d] x=%g sw=%02llx hw=%02llx", j, h[32LL * b + j], (unsigned long long)(ws & 63), (unsigned long long)(wh & 63));
        }
        printf("\n");
      }
    }
    printf("%-24s %ld of %d blocks differ\n", names[m], bad, nblk);
  }
  return 0;
}
