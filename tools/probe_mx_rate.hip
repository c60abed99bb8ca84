// Issue-rate probe of v_mfma_scale_f32_16x16x128_f8f6f4 per operand format (fp8 e4m3 = 0,
// fp6 e2m3 = 2, fp4 e2m1 = 4) against v_mfma_f32_16x16x32_bf16: one workgroup of 4 waves per CU
// (one per SIMD), each issuing a long chain over 8 independent accumulators; prints the cycles per
// MFMA per SIMD from s_memtime and the whole-grid rate.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_mx_rate.hip -o tools/probe_mx_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int FMT>
__global__ __launch_bounds__(256) void rate(float* out, long long* cyc, int iters, int sbase) {
  const int l = threadIdx.x & 63;
  i32x8 a, b;
  for (int r = 0; r < 8; ++r) { a[r] = 0x01010101 * (l + r); b[r] = 0x02020202 * (l ^ r); }
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int sa = sbase + (l & 3), sb = sbase + ((l >> 2) & 3);
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (FMT < 0) {
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, __builtin_shufflevector(a, a, 0, 1, 2, 3)),
                                                          __builtin_bit_cast(bf16x8, __builtin_shufflevector(b, b, 0, 1, 2, 3)),
                                                          acc[i], 0, 0, 0);
      } else {
        acc[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[i], FMT, FMT, 0, sa, 0, sb);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// the 32x32x64 shape: 4 independent 16-register accumulators
template <int FMT>
__global__ __launch_bounds__(256) void rate32(float* out, long long* cyc, int iters, int sbase) {
  const int l = threadIdx.x & 63;
  i32x8 a, b;
  for (int r = 0; r < 8; ++r) { a[r] = 0x01010101 * (l + r); b[r] = 0x02020202 * (l ^ r); }
  f32x16 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  const int sa = sbase + (l & 3), sb = sbase + ((l >> 2) & 3);
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[i], FMT, FMT, 0, sa, 0, sb);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 16; ++j) s += acc[i][j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int FMT>
static void run32(const char* name) {
  const int blocks = 256 * 2, iters = 4096;
  float* out;
  long long* cyc;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 8);
  hipLaunchKernelGGL(rate32<FMT>, dim3(blocks), dim3(256), 0, 0, out, cyc, 16, 120);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(rate32<FMT>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 120);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double n = (double)iters * 4;
  const double tf = blocks * 4.0 * n * (2.0 * 32 * 32 * 64) / (ms * 1e-3) / 1e12;
  printf("%-10s %8.3f ms  32x32x64  %.0f TFLOP/s dense\n", name, ms, tf);
  hipFree(out); hipFree(cyc);
}

template <int FMT>
static void run(const char* name, double flop_per_mfma) {
  const int blocks = 256 * 2, iters = 4096;
  float* out;
  long long* cyc;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 8);
  hipLaunchKernelGGL(rate<FMT>, dim3(blocks), dim3(256), 0, 0, out, cyc, 16, 120);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(rate<FMT>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 120);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  long long c0;
  hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);
  const double n = (double)iters * 8;  // MFMAs per wave
  const double tf = blocks * 4.0 * n * flop_per_mfma / (ms * 1e-3) / 1e12;
  printf("%-10s %8.3f ms  memtime/MFMA/wave %.2f (100 MHz ticks)  %.0f TFLOP/s dense\n", name, ms, c0 / n, tf);
  hipFree(out); hipFree(cyc);
}

int main() {
  run<-1>("bf16", 2.0 * 16 * 16 * 32);
  run<0>("fp8", 2.0 * 16 * 16 * 128);
  run<2>("fp6", 2.0 * 16 * 16 * 128);
  run<4>("fp4", 2.0 * 16 * 16 * 128);
  run32<0>("fp8");
  run32<2>("fp6");
  run32<4>("fp4");
  return 0;
}
