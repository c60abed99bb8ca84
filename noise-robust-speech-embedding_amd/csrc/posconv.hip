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
  // iteration t runs tap t % taps of weight segment t / taps: nseg = 2 is the split-weight mode
  // (hi and lo bf16 planes seg_stride apart, A's window read again for the lo plane)
  const int iters = taps * p.nseg;
  auto stage_w = [&](int t) {
    char* dst = wring + (t % WRING) * WSLOT;
    const int sg = t >= taps ? 1 : 0;
    const unsigned soff = (unsigned)((t - sg * taps) * PCH * 2 + (long long)sg * p.b.seg_stride * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(dst + (wave * 2 + j) * 1024), 16, wvoff[j], soff, 0, 0);
  };
  stage_w(0);
  if (iters > 1) stage_w(1);

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int t = 0, tap = 0; t < iters; ++t, tap = (tap + 1 == taps ? 0 : tap + 1)) {
    // tap t's weights (and, at t = 0, the window) landed for this wave; the barrier makes every
    // wave's DMAs visible and retires the reads of the slot restaged below (tap t - 1's)
    if (t + 1 < iters) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // raw barrier: no fence, so tap t + 1's DMAs stay in flight across it
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < iters) stage_w(t + 2);
    const char* ws = wring + (t % WRING) * WSLOT;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fb[4], fa[4];
#pragma unroll
      for (int fj = 0; fj < 4; ++fj) fb[fj] = frag7(ws, fj * 16, s, lane);
#pragma unroll
      for (int fi = 0; fi < 4; ++fi) fa[fi] = frag7(win, wave * 64 + fi * 16 + tap, s, lane);
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

// ---------------------------------------------------------------------------------------------
// Weight gradient of the grouped pos-conv (the backward's dWf[g][o][tap * 64 + i] =
// sum over (b, t) of dy[b, t, g * 64 + o] * Xp[b, t + tap, g * 64 + i]), as nrse_gemm poses it:
// M = 64 (o), N = taps * 64, K = T per segment (one segment per utterance), A = dy and B = the
// chunked Xp both row-contiguous, f32 atomics into the zeroed dWf. The generic 128 x 128 kernel
// wastes half of its M tile on it and re-reads the Xp rows of every tap.
//
// Here: one workgroup = group g x 8 taps (64 x 512 outputs, 4 waves of 64 x 128 = 2 taps) x one
// share of the segments. Per K-tile of 64 time steps it stages the dy tile (64 t x 64 o) and
// the Xp WINDOW (64 + 7 rows x 64 i) once; tap j's B fragments are the window read j rows down.
// Both images are [k][row] with 128-B k-rows (chunk c of k-row r at c ^ swk(r)) read with the
// transposing ds_read_b64_tr_b16, so the MFMA gets K-contiguous fragments from row-contiguous
// operands. A ring of 3 stages (17 KiB each) keeps two K-tiles of LDS-DMA in flight.
constexpr int WTB = 8;                       // taps per workgroup
constexpr int WDY = 64 * 128;                // dy tile image
constexpr int WWIN_ROWS = 72;                // window rows staged (64 + WTB - 1 used)
constexpr int WSTAGE = WDY + WWIN_ROWS * 128;
constexpr int WNST = 3;
constexpr int W_LDS = WSTAGE * WNST;         // 51 KiB
constexpr int W_INST = (64 + WWIN_ROWS) / 8; // 17 DMA wave-instructions per stage
constexpr int W_PER_WAVE = 5;                // per wave (the last one repeated by waves 1-3)

NRSE_DEV int swk(int k) { return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1; }

// fragment of rows base..base+15 (16 rows of the image's 64), k rows kb..kb+31 of a [k][64 rows]
// image: the row-contiguous counterpart of frag<false> for 128-B k-rows
NRSE_DEV bf16x8 fragT(const char* lds, int base, int kb, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int q = i >> 2, pp = i & 3;
  const int col = base + 4 * pp;
  const int k0 = kb + 8 * g + q, k1 = k0 + 4;
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)(lds + k0 * 128 + (((col >> 3) ^ swk(k0)) << 4) + ((col >> 2) & 1) * 8));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)(lds + k1 * 128 + (((col >> 3) ^ swk(k1)) << 4) + ((col >> 2) & 1) * 8));
  typedef short short8v __attribute__((ext_vector_type(8)));
  short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__global__ __launch_bounds__(PNTHR, 2) void posconv_wgrad_kernel(const nrse_gemm_params p, int ntb, int nshare,
                                                                 int nseg_total, int ktiles, long long b_rows) {
  __shared__ __attribute__((aligned(16))) char smem[W_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // XCD-aware order: the ntb tap blocks of one (group, share) are consecutive logical tiles on
  // one XCD, so they read the same dy / Xp rows through its L2
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tb = lt % ntb;
  const int gs = lt / ntb;
  const int sh = gs % nshare;
  const int g = gs / nshare;
  const int sg0 = (int)((long long)nseg_total * sh / nshare);
  const int sg1 = (int)((long long)nseg_total * (sh + 1) / nshare);
  const int n_it = (sg1 - sg0) * ktiles;

  const char* abase = (const char*)p.a.ptr + (long long)g * p.a.z1 * 2;
  const char* bbase = (const char*)p.b.ptr + (long long)g * p.b.z1 * 2;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(abase);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(bbase);
  const int tap0 = tb * WTB;

  // stage iteration `it` (segment sg0 + it / ktiles, K-tile it % ktiles) into ring slot it % 3:
  // instructions 0-7 the dy tile (rows t < K, zeros past it), 8-16 the window (rows
  // t0 + tap0 + w, zeros past the segment's padded extent)
  auto stage = [&](int it) {
    const int sg = sg0 + it / ktiles;
    const int t0 = (it % ktiles) * 64;
    char* dst = smem + (it % WNST) * WSTAGE;
#pragma unroll
    for (int j = 0; j < W_PER_WAVE; ++j) {
      const int inst = min(wave + 4 * j, W_INST - 1);
      const int r = (inst < 8 ? inst : inst - 8) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ swk(r);
      unsigned voff;
      if (inst < 8) {
        const int t = t0 + r;
        voff = t < p.K ? (unsigned)(((long long)sg * p.a.seg_stride + (long long)t * p.a.ld + c * 8) * 2) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(dst + inst * 1024), 16, voff, 0, 0, 0);
      } else {
        const long long row = (long long)t0 + tap0 + r;
        voff = row < b_rows ? (unsigned)(((long long)sg * p.b.seg_stride + row * p.b.ld + c * 8) * 2) : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(dst + inst * 1024), 16, voff, 0, 0, 0);
      }
    }
  };

  f32x4 acc[2][4][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[a][b][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (n_it > 0) stage(0);
  if (n_it > 1) stage(1);
#pragma unroll 1
  for (int it = 0; it < n_it; ++it) {
    // stage it landed for this wave (stage it + 1 may still be in flight); the barrier makes
    // every wave's DMAs visible and retires the reads of slot (it + 2) % 3 (stage it - 1's)
    if (it + 1 < n_it) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + 2 < n_it) stage(it + 2);
    const char* dy = smem + (it % WNST) * WSTAGE;
    const char* win = dy + WDY;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fa[4];
#pragma unroll
      for (int fi = 0; fi < 4; ++fi) fa[fi] = fragT(dy, fi * 16, s * 32, lane);
#pragma unroll
      for (int tl = 0; tl < 2; ++tl) {
        const int tap = wave * 2 + tl;
        bf16x8 fb[4];
#pragma unroll
        for (int fj = 0; fj < 4; ++fj) fb[fj] = fragT(win, fj * 16, s * 32 + tap, lane);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int fi = 0; fi < 4; ++fi)
#pragma unroll
          for (int fj = 0; fj < 4; ++fj)
            // transposed product: lane (q, i) holds output row o = 16 fi + i, columns 4q..4q+3
            acc[tl][fi][fj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[fj], fa[fi], acc[tl][fi][fj], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }

  // c_split > 0: share sh's partial sums stored whole into slab sh (16-byte stores, summed in
  // slab order by the caller); else f32 atomics into dWf (zeroed by the caller; nshare partial
  // sums per element). The atomics cost 32 B of write traffic per 4-byte add.
  const bool slabs = p.c_split != 0;
  float* cbase = (float*)p.c + (long long)g * p.c_z1 + (slabs ? (long long)sh * p.c_split : 0);
  const int q = lane >> 4, i = lane & 15;
#pragma unroll
  for (int tl = 0; tl < 2; ++tl) {
    const int n0 = (tap0 + wave * 2 + tl) * 64;
#pragma unroll
    for (int fi = 0; fi < 4; ++fi)
#pragma unroll
      for (int fj = 0; fj < 4; ++fj) {
        float* dst = cbase + (long long)(fi * 16 + i) * p.ldc + n0 + fj * 16 + 4 * q;
        if (slabs) {
          *reinterpret_cast<float4*>(dst) =
              make_float4(acc[tl][fi][fj][0], acc[tl][fi][fj][1], acc[tl][fi][fj][2], acc[tl][fi][fj][3]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) atomicAdd(dst + e, acc[tl][fi][fj][e]);
        }
      }
  }
}

}  // namespace

// The conv pattern nrse_gemm routes here (see the header comment).
bool nrse_posconv_ok(const nrse_gemm_params* p) {
  const nrse_gemm_operand& a = p->a;
  const nrse_gemm_operand& b = p->b;
  if (a.dtype != NRSE_BF16 || b.dtype != NRSE_BF16 || !a.kcontig || !b.kcontig) return false;
  if (a.chunk_shift != 6 || a.ld_chunk != a.ld || b.chunk_shift != 0) return false;
  if (p->N != PCH || p->splits != 1 || p->K % PCH != 0) return false;
  // nseg = 2: the split-weight mode (the same window against two weight planes)
  if (p->nseg != 1 && !(p->nseg == 2 && a.seg_stride == 0 && b.seg_stride > 0)) return false;
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

// The pos-conv weight-gradient pattern nrse_gemm routes to posconv_wgrad_kernel.
bool nrse_posconv_wgrad_ok(const nrse_gemm_params* p) {
  const nrse_gemm_operand& a = p->a;
  const nrse_gemm_operand& b = p->b;
  if (a.dtype != NRSE_BF16 || b.dtype != NRSE_BF16 || a.kcontig || b.kcontig) return false;
  if (a.chunk_shift != 0 || b.chunk_shift != 6 || b.ld_chunk != b.ld) return false;
  if (p->M != PCH || p->N % (WTB * PCH) != 0 || p->K < 1 || p->zdiv != 1) return false;
  // either two partial sums per element added straight into C (EPI_ATOMIC; the caller zeroes it)
  // or, with splits = 2 and per-split slabs (c_split > 0), each split's sum stored into its slab
  if (p->c_dtype != NRSE_F32 || p->ldc < p->N || p->alpha != 1.f || (p->ldc & 3) || (p->c_z1 & 3)) return false;
  if (p->c_split == 0 ? p->flags != NRSE_EPI_ATOMIC
                      : (p->flags != 0 || p->splits != 2 || (p->c_split & 3) ||
                         p->c_split < (long long)(p->batch - 1) * p->c_z1 + (long long)(p->M - 1) * p->ldc + p->N))
    return false;
  if (((uintptr_t)p->c) & 15) return false;
  if (a.ld % 8 || b.ld % 8 || a.seg_stride % 8 || b.seg_stride % 8 || a.z1 % 8 || b.z1 % 8) return false;
  if (b.seg_stride % b.ld != 0 || b.seg_stride / b.ld < (long long)p->K + p->N / PCH - 1) return false;
  if ((((uintptr_t)a.ptr) | ((uintptr_t)b.ptr)) & 15) return false;
  const long long nseg_total = (long long)p->nseg * p->splits;
  // byte offsets inside one group's buffer descriptor stay below 2^31
  const long long amax = (nseg_total * a.seg_stride + (long long)a.z1 * 0) * 2;
  const long long bmax = (nseg_total * b.seg_stride) * 2;
  return amax < (1LL << 31) && bmax < (1LL << 31);
}

int nrse_posconv_wgrad(const nrse_gemm_params* p, hipStream_t st) {
  const int ntb = p->N / (WTB * PCH);
  const int nseg_total = p->nseg * p->splits;
  // two shares of the segments: 2 workgroups per CU at 16 groups x 16 tap blocks, and with two
  // partial sums per element onto the zeroed dWf the atomic result is order-independent
  // (slab mode: one share per split, splits = 2)
  const int nshare = p->c_split != 0 ? 2 : nseg_total >= 2 ? 2 : 1;
  const int ktiles = nrse_cdiv(p->K, 64);
  const long long b_rows = p->b.seg_stride / p->b.ld;
  const long long total = (long long)p->batch * nshare * ntb;
  hipLaunchKernelGGL(posconv_wgrad_kernel, dim3((unsigned)total), dim3(PNTHR), 0, st, *p, ntb, nshare, nseg_total,
                     ktiles, b_rows);
  return nrse_check_launch("nrse_gemm(posconv wgrad)");
}
