// Probe of the MX-scaled MFMA's operand layout for fp6 / fp4 (v_mfma_scale_f32_16x16x128_f8f6f4):
// one wave, exact small-integer data, per-lane block scales; the host checks each format against
// the hypothesis "lane (g, i) holds row i's k = 32g .. 32g+31, value j at bits [w j, w j + w) of the
// little-endian register string (w = 8 / 6 / 4), and its scale byte scales that 32-k block".
// Build: hipcc --offload-arch=gfx950 -O2 tools/probe_mx.hip -o tools/probe_mx ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int FMT>
__global__ void probe(const int* a, const int* b, const int* sa, const int* sb, float* c) {
  const int l = threadIdx.x;
  i32x8 av, bv;
  for (int r = 0; r < 8; ++r) {
    av[r] = a[l * 8 + r];
    bv[r] = b[l * 8 + r];
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, FMT, FMT, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 4; ++r) c[l * 4 + r] = acc[r];
}

// encodings of small integers (and halves for fp4)
static unsigned enc(int fmt, float v) {
  const unsigned s = v < 0 ? 1u : 0u;
  float m = std::fabs(v);
  if (fmt == 0) {  // e4m3fn, bias 7
    if (m == 0) return s << 7;
    int e = (int)std::floor(std::log2(m));
    int mant = (int)std::lround((m / std::ldexp(1.f, e) - 1.f) * 8.f);
    return (s << 7) | ((unsigned)(e + 7) << 3) | (unsigned)mant;
  }
  if (fmt == 2) {  // e2m3, bias 1: normal (1 + m/8) 2^(e-1), e = 1..3; subnormal m/8
    if (m < 1.f) return (s << 5) | (unsigned)std::lround(m * 8.f);
    int e = (int)std::floor(std::log2(m));
    int mant = (int)std::lround((m / std::ldexp(1.f, e) - 1.f) * 8.f);
    return (s << 5) | ((unsigned)(e + 1) << 3) | (unsigned)mant;
  }
  // fmt 4: e2m1, bias 1: normal (1 + m/2) 2^(e-1), e = 1..3; subnormal 0.5 m
  if (m < 1.f) return (s << 3) | (unsigned)std::lround(m * 2.f);
  int e = (int)std::floor(std::log2(m));
  int mant = (int)std::lround((m / std::ldexp(1.f, e) - 1.f) * 2.f);
  return (s << 3) | ((unsigned)(e + 1) << 1) | (unsigned)mant;
}

static void pack(int w, const unsigned* vals, int* out) {  // 32 values of w bits -> dwords
  unsigned char bytes[32];
  std::memset(bytes, 0, sizeof(bytes));
  for (int j = 0; j < 32; ++j)
    for (int t = 0; t < w; ++t)
      if (vals[j] >> t & 1u) bytes[(w * j + t) >> 3] |= (unsigned char)(1u << ((w * j + t) & 7));
  std::memcpy(out, bytes, 32);
}

template <int FMT>
static int run(int w) {
  srand(12345 + FMT);
  static const float pool8[] = {0, 1, 2, 3, 4, 5, 6, 7, -1, -2, -3, -5, -7};
  static const float pool4[] = {0, 0.5f, 1, 1.5f, 2, 3, 4, 6, -1, -2, -3, -0.5f};
  const float* pool = FMT == 4 ? pool4 : pool8;
  const int np = FMT == 4 ? 12 : 13;
  float A[16][128], B[128][16];
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 128; ++k) A[i][k] = pool[rand() % np];
  for (int k = 0; k < 128; ++k)
    for (int j = 0; j < 16; ++j) B[k][j] = pool[rand() % np];
  int sa_blk[16][4], sb_blk[16][4];
  for (int i = 0; i < 16; ++i)
    for (int g = 0; g < 4; ++g) {
      sa_blk[i][g] = 127 + (i + 2 * g) % 3;
      sb_blk[i][g] = 126 + (3 * i + g) % 3;
    }
  std::vector<int> ha(64 * 8), hb(64 * 8), hsa(64), hsb(64);
  for (int l = 0; l < 64; ++l) {
    const int g = l >> 4, i = l & 15;
    unsigned va[32], vb[32];
    for (int j = 0; j < 32; ++j) {
      va[j] = enc(FMT, A[i][32 * g + j]);
      vb[j] = enc(FMT, B[32 * g + j][i]);
    }
    pack(w, va, &ha[l * 8]);
    pack(w, vb, &hb[l * 8]);
    hsa[l] = sa_blk[i][g];
    hsb[l] = sb_blk[i][g];
  }
  int *da, *db, *dsa, *dsb;
  float* dc;
  hipMalloc(&da, 64 * 8 * 4); hipMalloc(&db, 64 * 8 * 4); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256);
  hipMalloc(&dc, 64 * 4 * 4);
  hipMemcpy(da, ha.data(), 64 * 8 * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, hb.data(), 64 * 8 * 4, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa.data(), 256, hipMemcpyHostToDevice);
  hipMemcpy(dsb, hsb.data(), 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe<FMT>, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dc);
  float hc[256];
  hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
  double maxerr = 0, maxref = 0;
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * (l >> 4) + r, col = l & 15;
      double ref = 0;
      for (int k = 0; k < 128; ++k)
        ref += (double)A[row][k] * std::ldexp(1.0, sa_blk[row][k / 32] - 127) * B[k][col] *
               std::ldexp(1.0, sb_blk[col][k / 32] - 127);
      const double err = std::fabs(ref - hc[l * 4 + r]);
      if (err > 1e-6 * (1 + std::fabs(ref))) ++bad;
      maxerr = err > maxerr ? err : maxerr;
      maxref = std::fabs(ref) > maxref ? std::fabs(ref) : maxref;
    }
  printf("fmt %d (w=%d): %d of 256 outputs differ, max err %.4g (max |ref| %.4g) c[0..3] = %g %g %g %g\n", FMT, w, bad,
         maxerr, maxref, hc[0], hc[1], hc[2], hc[3]);
  hipFree(da); hipFree(db); hipFree(dsa); hipFree(dsb); hipFree(dc);
  return bad;
}

int main() {
  int bad = run<0>(8);
  bad += run<2>(6);
  bad += run<4>(4);
  printf(bad ? "PROBE MISMATCH\n" : "PROBE OK\n");
  return 0;
}
