// Grouped positional convolution as a sliding-window MFMA kernel
// ([TF]modeling_wavlm.py:48-90: Conv1d(H, H, kernel = 128, padding = 64, groups = 16) over the
// time axis; here forward and its dgrad, the transposed conv with flipped taps).
//
// nrse_gemm describes the conv as a grouped implicit GEMM whose A operand is "chunked": row m,
// column k = tap * 64 + i reads Xp[m + tap, g * 64 + i] (chunk_shift = 6, ld_chunk = ld: the tap
// stride equals the row stride). N = 64 output channels per group. The generic LDS-DMA kernels
// reload the A rows of every tap from L2 (a 256-row tile touches 383 distinct input rows but
// loads 256 x 128 of them) and waste half of a 128-wide N tile.
//
// This kernel: one workgroup = 256 output rows x the group's 64 output channels, 4 waves of
// 64 x 64. The input WINDOW of the tile (256 + 127 rows x 64 channels, 48 KiB) is staged into
// LDS once; every tap reads its A fragments from the window shifted by `tap` rows. Only the
// weights stream (8 KiB per tap, a ring of 3 LDS slots filled by LDS-DMA two taps ahead). The
// window's 16-B chunks are XOR-swizzled by (row & 7), which keeps ds_read_b128 fragment reads
// conflict-free at every row shift (the (row >> 1) & 7 swizzle of the GEMM images conflicts
// 2-way at odd shifts). K is consumed tap by tap in the same order and with the same MFMA as the
// GEMM kernels, and the epilogue is the shared epi8, so the results are the GEMM path's.
#include "gemm_common.h"

namespace {
using namespace nrse_gemm_detail;

constexpr int PBM = 256;               // output rows per workgroup
constexpr int PCH = 64;                // channels per group (N and the tap's K)
constexpr int PNTHR = 256;             // 4 waves
constexpr int WIN_ROWS = PBM + 128;    // window rows staged (>= PBM + taps - 1 for taps <= 129)
constexpr int WIN_BYTES = WIN_ROWS * 128;
constexpr int WSLOT = PCH * 128;       // one tap of weights: 64 rows x 64 k bf16 = 8 KiB
constexpr int WRING = 3;
constexpr int P_LDS = WIN_BYTES + WRING * WSLOT;  // 72 KiB: 2 workgroups per CU
constexpr int PCT_LD = 68;             // f32 epilogue row stride (256 x 68 x 4 B fits in P_LDS)
static_assert(PBM * PCT_LD * 4 <= P_LDS, "epilogue tile must fit the LDS");

// fragment of rows base..base+15 (any base), k-substep s, from a [row][64 k] image whose 16-B
// chunk ch of row R sits at position ch ^ (R & 7)
NRSE_DEV bf16x8 frag7(const char* lds, int base, int s, int lane) {
  const int row = base + (lane & 15);
  const int chunk = s * 4 + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((chunk ^ (row & 7)) << 4));
}

__global__ __launch_bounds__(PNTHR, 2) void posconv_kernel(const nrse_gemm_params p, int mt, int taps,
                                                           long long a_rows) {
  __shared__ __attribute__((aligned(16))) char smem[P_LDS];
  char* win = smem;
  char* wring = smem + WIN_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // XCD-aware order: consecutive logical tiles run on one XCD, and logical tiles are numbered
  // group-major (g, b, m-tile), so an XCD's tiles share one or two groups' weights in its L2
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int G = p.zdiv, Bt = p.batch / p.zdiv;
  const int g = lt / (Bt * mt);
  const int rem = lt - g * Bt * mt;
  const int b = rem / mt;
  const int m0 = (rem - b * mt) * PBM;
  (void)G;

  const char* abase = (const char*)p.a.ptr + ((long long)b * p.a.z1 + (long long)g * p.a.z2) * 2;
  const char* bbase = (const char*)p.b.ptr + ((long long)b * p.b.z1 + (long long)g * p.b.z2) * 2;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(abase);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(bbase);

  // window: 384 rows x 8 chunks; 48 wave-instructions (8 rows each), 12 per wave. Rows past the
  // batch's padded extent (a_rows = rows of Xp per batch) load zeros.
#pragma unroll
  for (int j = 0; j < WIN_ROWS / 8 / 4; ++j) {
    const int inst = wave * (WIN_ROWS / 32) + j;
    const int r = inst * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const long long grow = (long long)m0 + r;
    const unsigned voff = grow < a_rows ? (unsigned)((grow * p.a.ld + c * 8) * 2) : OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(win + inst * 1024), 16, voff, 0, 0, 0);
  }
  // weights of tap t: 64 rows (o) x 64 k; 8 wave-instructions, 2 per wave, same (row & 7) swizzle
  unsigned wvoff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = (wave * 2 + j) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    wvoff[j] = (unsigned)(((long long)r * p.b.ld + c * 8) * 2);
  }
  auto stage_w = [&](int t) {
    char* dst = wring + (t % WRING) * WSLOT;
    const unsigned soff = (unsigned)(t * PCH * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(dst + (wave * 2 + j) * 1024), 16, wvoff[j], soff, 0, 0);
  };
  stage_w(0);
  if (taps > 1) stage_w(1);

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int t = 0; t < taps; ++t) {
    // tap t's weights (and, at t = 0, the window) landed for this wave; the barrier makes every
    // wave's DMAs visible and retires the reads of the slot restaged below (tap t - 1's)
    if (t + 1 < taps) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // raw barrier: no fence, so tap t + 1's DMAs stay in flight across it
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < taps) stage_w(t + 2);
    const char* ws = wring + (t % WRING) * WSLOT;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fb[4], fa[4];
#pragma unroll
      for (int fj = 0; fj < 4; ++fj) fb[fj] = frag7(ws, fj * 16, s, lane);
#pragma unroll
      for (int fi = 0; fi < 4; ++fi) fa[fi] = frag7(win, wave * 64 + fi * 16 + t, s, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int fi = 0; fi < 4; ++fi)
#pragma unroll
        for (int fj = 0; fj < 4; ++fj)
          // transposed product: lane (q, i) holds output row i, columns 4q..4q+3
          acc[fi][fj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[fj], fa[fi], acc[fi][fj], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  __syncthreads();

  // epilogue: the 256 x 64 f32 tile through LDS, then epi8 on 8 contiguous columns per thread
  float* ct = reinterpret_cast<float*>(smem);
  {
    const int q = lane >> 4, i = lane & 15;
#pragma unroll
    for (int fi = 0; fi < 4; ++fi)
#pragma unroll
      for (int fj = 0; fj < 4; ++fj)
        *reinterpret_cast<f32x4*>(ct + (wave * 64 + fi * 16 + i) * PCT_LD + fj * 16 + 4 * q) = acc[fi][fj];
  }
  __syncthreads();
  Epi epi(p, b, g, 0);
  const int n = (tid & 7) * 8;
  epi.load_bias(p, n);
#pragma unroll 1
  for (int it = 0; it < PBM / 32; ++it) {
    const int row = (tid >> 3) + 32 * it;
    const int m = m0 + row;
    if (m < p.M) epi8(p, epi, m, n, ct + row * PCT_LD + n, false);
  }
}

}  // namespace

// The conv pattern nrse_gemm routes here (see the header comment).
bool nrse_posconv_ok(const nrse_gemm_params* p) {
  const nrse_gemm_operand& a = p->a;
  const nrse_gemm_operand& b = p->b;
  if (a.dtype != NRSE_BF16 || b.dtype != NRSE_BF16 || !a.kcontig || !b.kcontig) return false;
  if (a.chunk_shift != 6 || a.ld_chunk != a.ld || b.chunk_shift != 0) return false;
  if (p->N != PCH || p->nseg != 1 || p->splits != 1 || p->K % PCH != 0) return false;
  const int taps = p->K / PCH;
  if (taps < 1 || taps > WIN_ROWS - PBM + 1) return false;
  if (p->flags & (NRSE_EPI_ATOMIC | NRSE_EPI_COLSUM)) return false;
  if (p->batch % p->zdiv != 0) return false;
  // the window of the last tile reads up to a_rows rows per batch: the padded input must hold
  // M + taps - 1 rows, whose row stride is the batch stride / ld
  if (a.z1 % a.ld != 0 || a.z1 / a.ld < (long long)p->M + taps - 1) return false;
  return dma_layout_ok(p, 0);
}

int nrse_posconv(const nrse_gemm_params* p, hipStream_t st) {
  const int mt = nrse_cdiv(p->M, PBM);
  const long long total = (long long)mt * p->batch;
  const int taps = p->K / PCH;
  const long long a_rows = p->a.z1 / p->a.ld;  // padded rows of one batch
  hipLaunchKernelGGL(posconv_kernel, dim3((unsigned)total), dim3(PNTHR), 0, st, *p, mt, taps, a_rows);
  return nrse_check_launch("nrse_gemm(posconv)");
}
