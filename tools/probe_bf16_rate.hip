// Issue-rate probe of the bf16 MFMA shapes: v_mfma_f32_16x16x32_bf16 (8 independent 4-register
// accumulators) against v_mfma_f32_32x32x16_bf16 (4 independent 16-register accumulators), the
// operands loop-invariant registers (no VALU in the loop), 2 workgroups of 4 waves per CU;
// prints the whole-grid rate (dense FLOPs).
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_bf16_rate.hip -o tools/probe_bf16_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int SHAPE>
__global__ __launch_bounds__(256) void rate(float* out, int iters) {
  const int l = threadIdx.x & 63;
  bf16x8 a[4], b[4];  // distinct operand registers per MFMA (one shared pair measured the 16x16 shape low)
  for (int q = 0; q < 4; ++q)
    for (int r = 0; r < 8; ++r) { a[q][r] = (__bf16)(0.001f * (l + r + q)); b[q][r] = (__bf16)(0.002f * (l ^ (r + q))); }
  float s = 0.f;
  if constexpr (SHAPE == 16) {
    f32x4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i & 3], b[(i >> 1) & 3], acc[i], 0, 0, 0);
    }
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  } else {
    f32x16 acc[4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i & 3], b[(i + 1) & 3], acc[i], 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 16; ++j) s += acc[i][j];
  }
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int SHAPE>
static void run() {
  const int blocks = 256 * 2, iters = 8192;
  float* out;
  hipMalloc(&out, blocks * 256 * 4);
  hipLaunchKernelGGL(rate<SHAPE>, dim3(blocks), dim3(256), 0, 0, out, 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(rate<SHAPE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  // per wave per iteration: 8 x 16x16x32 or 4 x 32x32x16 = the same 131072 x 2 FLOPs
  const double flop = (double)blocks * 4 * iters * (SHAPE == 16 ? 8.0 * 2 * 16 * 16 * 32 : 4.0 * 2 * 32 * 32 * 16);
  printf("bf16 %dx%d: %8.3f ms  %.0f TFLOP/s dense\n", SHAPE, SHAPE, ms, flop / (ms * 1e-3) / 1e12);
  hipFree(out);
}

int main() {
  for (int r = 0; r < 2; ++r) {
    run<16>();
    run<32>();
  }
  return 0;
}
