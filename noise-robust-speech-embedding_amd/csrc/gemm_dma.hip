// bf16 MFMA GEMM, generation 2: LDS-DMA staging + LDS-staged coalesced epilogue.
//
// Same contract as nrse_gemm (include/nrse_hip.h); nrse_gemm dispatches here for bf16 problems
// whose strides/alignments fit (see nrse_gemm_dma_ok). Differences from gemm.hip's kernel:
//  - operand tiles are filled by `buffer_load_dwordx4 ... lds` (LDS-DMA): no staging VGPRs and
//    no ds_write pass. The LDS image is lane-linear per wave instruction (1 KiB), so the XOR
//    swizzle that keeps the fragment reads conflict-free is applied on the per-lane SOURCE
//    address. Buffer descriptors give free zero-fill: a lane whose element is outside the
//    operand (M/N/K tails, segment ends) gets an out-of-range offset and loads zeros.
//  - 2 LDS stages, one barrier per 64-deep K step: the DMA for step t+1 is in flight while
//    step t's MFMAs run; 2 workgroups per CU (72 KiB LDS each) hide each other's waits.
//  - the 128x128 f32 accumulator tile goes through LDS so every epilogue access (bias,
//    residual, GELU pre-activation, output) is a 16-32 B vector per lane on contiguous rows.
#include "gemm_common.h"

namespace {
using namespace nrse_gemm_detail;

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;
constexpr int TILE = 16384;
constexpr int STAGE = 2 * TILE;
constexpr int CT_LD = 132;                       // f32 epilogue tile row stride
constexpr int LDS_BYTES = BM * CT_LD * 4 + 1024; // >= 2 stages (64 KiB)

struct OpLoad {
  __amdgpu_buffer_rsrc_t rs;
  long long ld, ldc, seg, cmask;
  int cs;
  unsigned base_off[4];  // KC: row offset (elements); !KC: column offset (elements)
  int aux[4];            // KC: logical chunk; !KC: k row within tile
  bool ok[4];
};

template <bool KC>
NRSE_DEV void op_init(OpLoad& o, const nrse_gemm_operand& d, const char* base, int wave, int lane, int row0,
                      int rows_total) {
  o.rs = make_rsrc(base);
  o.ld = d.ld; o.ldc = d.ld_chunk; o.seg = d.seg_stride;
  o.cs = d.chunk_shift > 0 ? d.chunk_shift : 62;
  o.cmask = d.chunk_shift > 0 ? ((1LL << d.chunk_shift) - 1) : -1LL;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = wave * 4 + j;
    if constexpr (KC) {
      const int row = 8 * i + (lane >> 3);
      const int lc = (lane & 7) ^ ((row >> 1) & 7);
      o.base_off[j] = (unsigned)((long long)(row0 + row) * o.ld);
      o.aux[j] = lc;
      o.ok[j] = row0 + row < rows_total;
    } else {
      const int row = 4 * i + (lane >> 4);
      const int fb = ((row & 3) | (((row >> 3) & 1) << 2)) << 1;
      const int lc = (lane & 15) ^ fb;
      const long long col = row0 + lc * 8;
      o.base_off[j] = (unsigned)coff(col, o.cs, o.cmask, o.ldc);
      o.aux[j] = row;
      o.ok[j] = col < rows_total;
    }
  }
}

template <bool KC>
NRSE_DEV void op_issue(const OpLoad& o, char* lds_tile, int wave, long long segoff, int k0, int kseg) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    unsigned voff;
    if constexpr (KC) {
      const int k = k0 + o.aux[j] * 8;
      const bool v = o.ok[j] && k < kseg;
      voff = v ? (unsigned)((segoff + o.base_off[j] + coff(k, o.cs, o.cmask, o.ldc)) * 2) : OOB;
    } else {
      const int k = k0 + o.aux[j];
      const bool v = o.ok[j] && k < kseg;
      voff = v ? (unsigned)((segoff + (long long)k * o.ld + o.base_off[j]) * 2) : OOB;
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(o.rs, (lds_void*)(lds_tile + (wave * 4 + j) * 1024), 16, voff, 0, 0, 0);
  }
}

template <bool AKC, bool BKC>
__global__ __launch_bounds__(NTHR, 2) void gemm_dma_kernel(const nrse_gemm_params p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware, M-grouped tile order (as gemm256.hip): workgroup i runs on XCD i % 8, so the
  // ids are renumbered to give each XCD a contiguous run of tiles, walked GM M-tiles deep, and
  // the tiles an XCD holds at once share their A and B panels in its L2. (Row-major grid order
  // put one N column on each XCD: every XCD streamed all of A, 4x the algorithmic traffic on
  // the weight-gradient GEMMs.)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int mt = (p.M + BM - 1) / BM, nt = (p.N + BN - 1) / BN;
  const int per_z = mt * nt;
  const int z = wg / per_z;
  const int tt = wg - z * per_z;
  constexpr int GM = 8;
  const int group = tt / (GM * nt);
  const int first_m = group * GM;
  const int gm = min(GM, mt - first_m);
  const int in_g = tt - group * GM * nt;
  const int m0 = (first_m + in_g % gm) * BM;
  const int n0 = (in_g / gm) * BN;
  const int zb = z / p.splits;
  const int split = z % p.splits;
  const long long zq = zb / p.zdiv, zr = zb % p.zdiv;

  OpLoad la, lb;
  op_init<AKC>(la, p.a, (const char*)p.a.ptr + (zq * p.a.z1 + zr * p.a.z2) * 2, wave, lane, m0, p.M);
  op_init<BKC>(lb, p.b, (const char*)p.b.ptr + (zq * p.b.z1 + zr * p.b.z2) * 2, wave, lane, n0, p.N);

  const int tps = (p.K + BK - 1) / BK;
  const int seg0 = split * p.nseg;
  const int ntiles = p.nseg * tps;

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t, int stage) {
    const int sg = seg0 + t / tps;
    const int k0 = (t % tps) * BK;
    char* st = smem + stage * STAGE;
    op_issue<AKC>(la, st, wave, (long long)sg * la.seg, k0, p.K);
    op_issue<BKC>(lb, st + TILE, wave, (long long)sg * lb.seg, k0, p.K);
  };

  if (ntiles > 0) issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) issue(t + 1, (t + 1) & 1);
    const char* la_s = smem + (t & 1) * STAGE;
    const char* lb_s = la_s + TILE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) fa[tm] = frag<AKC>(la_s, wm * 64 + tm * 16, s, lane);
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) fb[tn] = frag<BKC>(lb_s, wn * 64 + tn * 16, s, lane);
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int tn = 0; tn < 4; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[tm], fb[tn], acc[tm][tn], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue through LDS
  float* ct = reinterpret_cast<float*>(smem);
  {
    const int g = lane >> 4, li = lane & 15;
#pragma unroll
    for (int tm = 0; tm < 4; ++tm)
#pragma unroll
      for (int tn = 0; tn < 4; ++tn)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ct[(wm * 64 + tm * 16 + 4 * g + r) * CT_LD + wn * 64 + tn * 16 + li] = acc[tm][tn][r];
  }
  __syncthreads();
  const int flags = p.flags;
  const long long cbase = zq * p.c_z1 + zr * p.c_z2 + (long long)split * p.c_split;
  if (flags & NRSE_EPI_ATOMIC) {
    // split-K / accumulate-into-gradient: one row per wave instruction, 64 lanes on 64
    // consecutive columns = 256 contiguous bytes per atomic wave-instruction (full atomic rate)
    for (int row = wave; row < BM; row += 4) {
      const int m = m0 + row;
      if (m >= p.M) break;
#pragma unroll
      for (int hc = 0; hc < 2; ++hc) {
        const int col = hc * 64 + lane;
        const int n = n0 + col;
        if (n < p.N) atomicAdd((float*)p.c + cbase + (long long)m * p.ldc + n, ct[row * CT_LD + col] * p.alpha);
      }
    }
    return;
  }
  Epi epi(p, zq, zr, split);
  epi.load_bias(p, n0 + (tid & 15) * 8);  // the epilogue columns of this thread (see the loop)
  const bool colsum = (flags & NRSE_EPI_COLSUM) != 0;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int sgi = tid + NTHR * it;
    const int row = sgi >> 4;
    const int cs = (sgi & 15) * 8;
    const int m = m0 + row, n = n0 + cs;
    float* cr = ct + row * CT_LD + cs;
    if (m >= p.M || n >= p.N) {
      if (colsum) {
#pragma unroll
        for (int e = 0; e < 8; ++e) cr[e] = 0.f;
      }
      continue;
    }
    epi8(p, epi, m, n, cr, colsum);
  }
  if (colsum) {
    __syncthreads();
    const int col = tid & 127, half = tid >> 7;
    if (n0 + col < p.N) {
      float s = 0.f;
      for (int r = half * 64; r < half * 64 + 64; ++r) s += ct[r * CT_LD + col];
      colsum_out(p, z, mt, m0 / BM, half, n0 + col, s);
    }
  }
}

template <bool AKC, bool BKC>
int launch(const nrse_gemm_params* p, hipStream_t st) {
  const long long total = (long long)nrse_cdiv(p->N, BN) * nrse_cdiv(p->M, BM) * p->batch * p->splits;
  hipLaunchKernelGGL((gemm_dma_kernel<AKC, BKC>), dim3((unsigned)total), dim3(NTHR), 0, st, *p);
  return nrse_check_launch("nrse_gemm(dma)");
}

}  // namespace

bool nrse_gemm_dma_ok(const nrse_gemm_params* p) {
  return p->M >= 64 && dma_layout_ok(p, 64) &&
         (long long)nrse_cdiv(p->N, BN) * nrse_cdiv(p->M, BM) * p->batch * p->splits < (1LL << 31);
}

int nrse_gemm_dma(const nrse_gemm_params* p, hipStream_t st) {
  if (p->a.kcontig && p->b.kcontig) return launch<true, true>(p, st);
  if (p->a.kcontig && !p->b.kcontig) return launch<true, false>(p, st);
  if (!p->a.kcontig && p->b.kcontig) return launch<false, true>(p, st);
  return launch<false, false>(p, st);
}
