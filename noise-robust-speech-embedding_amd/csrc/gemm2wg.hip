// bf16 MFMA GEMM, generation 5: two workgroups per CU, each a BM x 256 tile (BM = 128 or 112)
// with 4 waves, for the forward (A and B k-contiguous) problems of the step.
//
// Why (profiles): the 256x256 kernel owns a whole CU (160 KiB of LDS, 8 waves
// x 217 VGPRs), so its prologue (~5k cycles of DMA latency) and epilogue (~17k cycles, ~32k
// with GELU + pre-activation) run with the matrix pipe idle: 30-40 % of a tile at K = 1024.
// Here two independent workgroups share each CU (72 KiB of LDS and 4 waves of <= 256 VGPRs
// each), so one's epilogue and prologue overlap the other's main loop, and their main loops
// interleave on every SIMD without an explicit ping-pong.
//  - wave w computes rows 0..BM-1 x columns 64w..64w+63 of the tile: BM/16 x 4 accumulators of
//    16x16 (transposed MFMA: lane (g, i) holds row i, columns 4g..4g+3);
//  - K-tiles of 32: A image [BM][32] (8 / 7 KiB), B image [256][32] (16 KiB), 64-B rows whose
//    16-B chunks sit at chunk ^ ((row >> 1) & 3): conflict-free ds_read_b128 fragments for the
//    16-row x 4-chunk lane pattern (checked against the gfx950 lane groups);
//  - a 3-stage ring of K-tiles (72 KiB), filled by LDS-DMA two K-tiles ahead; one barrier per
//    K-tile: [barrier] issue K-tile t+2 into the slot read in t-1, read + 32 MFMAs on t,
//    vmcnt(6) (K-tile t+1 landed, t+2 in flight), [barrier];
//  - the epilogue finishes values in registers (bias, GELU + bf16 pre-activation, dropout,
//    f32 residual) and stores through an LDS image in two 64-row passes (16-B row stores).
#include "gemm_common.h"
#ifndef NRSE_2WG_DIAG
#define NRSE_2WG_DIAG 0
#endif

namespace {
using namespace nrse_gemm_detail;

constexpr int BN = 256, BK = 32, NTHR = 256;
constexpr int STAGE = (128 + 256) * BK * 2;  // 24 KiB per K-tile (A image sized for 128 rows)
constexpr int LDS_BYTES = 3 * STAGE;         // 72 KiB: two workgroups per CU
constexpr int A_IMG = 0, B_IMG = 128 * BK * 2;

NRSE_DEV int sw(int row) { return (row >> 1) & 3; }

// 16x16x32 operand fragment: rows base..base+15 of a [rows][32] image, lane (g, i) -> row i,
// k 8g..8g+7
NRSE_DEV bf16x8 frag32(const char* img, int base, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = base + i;
  return *reinterpret_cast<const bf16x8*>(img + row * 64 + ((g ^ sw(row)) << 4));
}

// LDS-DMA loader of one k-contiguous operand: instruction j of wave w fills image rows
// 16 (4j + w) .. +15; lane l -> row 16 (4j + w) + l / 4, LDS chunk l % 4 holding source chunk
// (l % 4) ^ sw(row). Rows past the operand (or past the tile's BM) load zeros.
template <int NI>
struct Ldr {
  __amdgpu_buffer_rsrc_t rs, dead;
  unsigned voff[NI];
  int kpos[NI];
  long long ld, seg;
};

template <int NI>
NRSE_DEV void ldr_init(Ldr<NI>& o, const nrse_gemm_operand& d, const char* base, int wave, int lane, int row0,
                       int rows_total, int rows_tile) {
  o.rs = make_rsrc(base);
  o.dead = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0, 0x00020000);
  o.ld = d.ld;
  o.seg = d.seg_stride;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int r = 16 * (4 * j + wave) + (lane >> 2);
    const int c = (lane & 3) ^ sw(r);
    const int grow = row0 + r;
    o.voff[j] = (r < rows_tile && grow < rows_total) ? (unsigned)(((long long)grow * o.ld + c * 8) * 2) : OOB;
    o.kpos[j] = c * 8;
  }
}

template <int NI>
NRSE_DEV void ldr_issue(const Ldr<NI>& o, char* img, int wave, unsigned soff, int krem, bool live) {
  const __amdgpu_buffer_rsrc_t rs = live ? o.rs : o.dead;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    unsigned voff = o.voff[j];
    if (krem < BK) voff = o.kpos[j] < krem ? voff : OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + (4 * j + wave) * 1024), 16, voff, soff, 0, 0);
  }
}

enum : int { F_BIAS = 1, F_GELU = 2, F_DROP = 4, F_RESID = 8, F_OBF = 16 };

// compile-time epilogue mode of the flag set, or -1 (not supported here)
NRSE_DEV int epi_mode(const nrse_gemm_params& p) {
  const int f = p.flags;
  if (f & ~(NRSE_EPI_BIAS | NRSE_EPI_GELU | NRSE_EPI_DROPOUT | NRSE_EPI_RESID | NRSE_EPI_DROP_AFTER)) return -1;
  int m = 0;
  if (f & NRSE_EPI_BIAS) m |= F_BIAS;
  if (f & NRSE_EPI_GELU) m |= F_GELU;
  if (f & NRSE_EPI_DROPOUT) m |= F_DROP;
  if (f & NRSE_EPI_RESID) m |= F_RESID;
  if (p.c_dtype == NRSE_BF16) m |= F_OBF;
  return m;
}

template <int FE, int BM>
NRSE_DEV void epilogue(const nrse_gemm_params& p, const f32x4 (&acc)[8][4], char* smem, int m0, int n0, int wave,
                       int lane, int tid, long long zq, long long zr) {
  constexpr bool BIAS = FE & F_BIAS, GELU = FE & F_GELU, DROP = FE & F_DROP, RESID = FE & F_RESID;
  constexpr bool OBF = FE & F_OBF;
  constexpr int NA = BM / 16;
  constexpr int ES = OBF ? 2 : 4;
  constexpr int PITCH = 256 * ES + 16;
  constexpr int APITCH = 256 * 2 + 16;
  const int g = lane >> 4, li = lane & 15;
  const Epi epi(p, zq, zr, 0);
  char* const oimg = smem;
  char* const aimg = smem + 64 * PITCH;  // GELU pre-activation (bf16 output: 33 + 33 KiB)
  float b4[4][4];
#pragma unroll
  for (int fn = 0; fn < 4; ++fn) {
    const int n = n0 + wave * 64 + fn * 16 + 4 * g;
    float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
    if (BIAS && n < p.N) bb = *reinterpret_cast<const float4*>(p.bias + epi.bbase + n);
    b4[fn][0] = bb.x; b4[fn][1] = bb.y; b4[fn][2] = bb.z; b4[fn][3] = bb.w;
  }
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int fi = 0; fi < 4; ++fi) {
      const int a = pass * 4 + fi;
      if (a >= NA) continue;
      const int prow = fi * 16 + li;
      const int m = m0 + pass * 64 + prow;
      const bool mok = m < p.M;
#pragma unroll
      for (int fn = 0; fn < 4; ++fn) {
        const int tcol = wave * 64 + fn * 16 + 4 * g;
        const int n = n0 + tcol;
        const bool ok = mok && n < p.N;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(acc[a][fn][e], p.alpha, b4[fn][e]);
        if constexpr (GELU) {
          if (p.aux) {
            uint2 u;
            u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
            u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
            *reinterpret_cast<uint2*>(aimg + prow * APITCH + tcol * 2) = u;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = gelu_fast(v[e]);
        }
        const long long ci = epi.cbase + (long long)m * p.ldc + n;
        if constexpr (DROP) {
          if (!(p.flags & NRSE_EPI_DROP_AFTER)) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = dropout_keep(epi.key, (uint32_t)(ci + e), epi.thresh) ? v[e] * epi.dscale : 0.f;
          }
        }
        if constexpr (RESID) {
          float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
          if (ok) {
            if (p.resid_dtype == NRSE_BF16) {
              const uint2 u = *reinterpret_cast<const uint2*>((const bf16_t*)p.resid + epi.rbase + (long long)m * p.ldr + n);
              r = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                              __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
            } else {
              r = *reinterpret_cast<const float4*>((const float*)p.resid + epi.rbase + (long long)m * p.ldr + n);
            }
          }
          v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
        }
        if constexpr (DROP) {
          if (p.flags & NRSE_EPI_DROP_AFTER) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = dropout_keep(epi.key, (uint32_t)(ci + e), epi.thresh) ? v[e] * epi.dscale : 0.f;
          }
        }
        if constexpr (OBF) {
          uint2 u;
          u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          *reinterpret_cast<uint2*>(oimg + prow * PITCH + tcol * 2) = u;
        } else {
          *reinterpret_cast<float4*>(oimg + prow * PITCH + tcol * 4) = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    }
    __syncthreads();
    constexpr int CPR = 256 * ES / 16;
    const int prows = (pass == 1) ? BM - 64 : 64;
    for (int idx = tid; idx < prows * CPR; idx += NTHR) {
      const int prow = idx / CPR, ch = idx - prow * CPR;
      const int m = m0 + pass * 64 + prow;
      const int n = n0 + ch * (16 / ES);
      if (m >= p.M || n >= p.N) continue;
      const uint4 u = *reinterpret_cast<const uint4*>(oimg + prow * PITCH + ch * 16);
      *reinterpret_cast<uint4*>((char*)p.c + (epi.cbase + (long long)m * p.ldc + n) * ES) = u;
      if constexpr (GELU) {
        if (p.aux) {
          const uint4 w = *reinterpret_cast<const uint4*>(aimg + prow * APITCH + ch * 16);
          *reinterpret_cast<uint4*>((bf16_t*)p.aux + epi.abase + (long long)m * p.ldaux + n) = w;
        }
      }
    }
    __syncthreads();
  }
}

template <int BM>
__global__ __launch_bounds__(NTHR, 2) void gemm2wg_kernel(const nrse_gemm_params p, int mt, int nt) {
  static_assert(BM == 128 || BM == 112, "tile rows");
  constexpr int NA = BM / 16;           // accumulator row blocks per wave
  constexpr int NIA = (BM + 63) / 64;   // DMA instructions per thread for A (2)
  constexpr int NIB = 256 / 64;         // ... for B (4)
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // XCD-aware, M-grouped tile order (as the 256-column kernel)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int per_z = mt * nt;
  const int zb = wg / per_z;
  const int tt = wg - zb * per_z;
  constexpr int GM = 16;
  const int group = tt / (GM * nt);
  const int first_m = group * GM;
  const int gm = min(GM, mt - first_m);
  const int in_g = tt - group * GM * nt;
  const int m0 = (first_m + in_g % gm) * BM;
  const int n0 = (in_g / gm) * BN;
  const long long zq = zb / p.zdiv, zr = zb % p.zdiv;

  Ldr<NIA> la;
  Ldr<NIB> lb;
  ldr_init<NIA>(la, p.a, (const char*)p.a.ptr + (zq * p.a.z1 + zr * p.a.z2) * 2, wave, lane, m0, p.M, BM);
  ldr_init<NIB>(lb, p.b, (const char*)p.b.ptr + (zq * p.b.z1 + zr * p.b.z2) * 2, wave, lane, n0, p.N, 256);

  const int tps = (p.K + BK - 1) / BK;
  const int ntiles = p.nseg * tps;
  // K-tile (segment, index within it) of the tile being staged, advanced by one per K-tile
  auto stage = [&](int slot, bool live, int sg, int ki) {
    const int k0 = (live ? ki : 0) * BK;
    const long long sgo = (long long)(live ? sg : 0);
    const unsigned sa = (unsigned)((sgo * la.seg + k0) * 2);
    const unsigned sb = (unsigned)((sgo * lb.seg + k0) * 2);
    char* st = smem + slot * STAGE;
    ldr_issue<NIA>(la, st + A_IMG, wave, sa, p.K - k0, live);
    ldr_issue<NIB>(lb, st + B_IMG, wave, sb, p.K - k0, live);
  };
  int s_sg = 0, s_k = 0;  // next K-tile to stage
  auto advance = [&]() { if (++s_k == tps) { s_k = 0; ++s_sg; } };

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-tiles 0 and 1
  stage(0, 0 < ntiles, s_sg, s_k);
  advance();
  stage(1, 1 < ntiles, s_sg, s_k);
  advance();
  constexpr int NDMA = NIA + NIB;
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();  // raw: K-tile 1 stays in flight
  asm volatile("" ::: "memory");

  int slot = 0;
#pragma unroll 1
  for (int t = 0; t < ntiles; ++t) {
    // K-tile t+2 into the slot read in iteration t-1 (all its reads retired before the barrier)
    const int sn = slot == 0 ? 2 : slot - 1;
#if NRSE_2WG_DIAG == 1
    if (t < 0)
#endif
    stage(sn, t + 2 < ntiles, s_sg, s_k);
    advance();
    const char* st = smem + slot * STAGE;
    bf16x8 fb[4], fa[8];
#pragma unroll
    for (int fj = 0; fj < 4; ++fj) fb[fj] = frag32(st + B_IMG, wave * 64 + fj * 16, lane);
#pragma unroll
    for (int fi = 0; fi < NA; ++fi) fa[fi] = frag32(st + A_IMG, fi * 16, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int fi = 0; fi < NA; ++fi)
#pragma unroll
      for (int fj = 0; fj < 4; ++fj)
        acc[fi][fj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[fj], fa[fi], acc[fi][fj], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // K-tile t+1 landed (this wave's DMAs); t+2's stay in flight across the raw barrier
#if NRSE_2WG_DIAG != 2
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
#endif
    asm volatile("" ::: "memory");
#if NRSE_2WG_DIAG != 3
    __builtin_amdgcn_s_barrier();
#endif
    asm volatile("" ::: "memory");
    slot = slot == 2 ? 0 : slot + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing zero-fill DMAs
  __syncthreads();
  switch (epi_mode(p)) {
#define NRSE_E(M) case M: epilogue<M, BM>(p, acc, smem, m0, n0, wave, lane, tid, zq, zr); break;
    NRSE_E(0) NRSE_E(F_OBF) NRSE_E(F_BIAS) NRSE_E(F_BIAS | F_OBF) NRSE_E(F_BIAS | F_GELU | F_OBF)
    NRSE_E(F_BIAS | F_GELU | F_DROP | F_OBF) NRSE_E(F_BIAS | F_RESID) NRSE_E(F_BIAS | F_RESID | F_DROP)
    NRSE_E(F_RESID) NRSE_E(F_RESID | F_DROP)
#undef NRSE_E
    default: break;
  }
}

// modes the kernel instantiates (host mirror of the device switch above)
bool mode_ok(const nrse_gemm_params* p) {
  const int f = p->flags;
  if (f & ~(NRSE_EPI_BIAS | NRSE_EPI_GELU | NRSE_EPI_DROPOUT | NRSE_EPI_RESID | NRSE_EPI_DROP_AFTER)) return false;
  if (p->c_dtype != NRSE_BF16 && p->c_dtype != NRSE_F32) return false;
  const bool obf = p->c_dtype == NRSE_BF16;
  if (f & NRSE_EPI_GELU) {
    if (!obf || !(f & NRSE_EPI_BIAS) || (f & NRSE_EPI_RESID)) return false;
    if (p->aux && p->aux_dtype != NRSE_BF16) return false;
    return true;
  }
  if (f & NRSE_EPI_RESID) return !obf && p->resid_dtype == NRSE_F32;
  return !(f & NRSE_EPI_DROPOUT);
}

}  // namespace

// 112 rows when they need no more tile waves of 512 workgroups (two per CU) than 128 rows
static int bm2(const nrse_gemm_params* p) {
  const long long per = (long long)nrse_cdiv(p->N, BN) * p->batch;
  const long long w128 = (nrse_cdiv(p->M, 128) * per + 511) / 512;
  const long long w112 = (nrse_cdiv(p->M, 112) * per + 511) / 512;
  return w112 <= w128 ? 112 : 128;
}

bool nrse_gemm2wg_ok(const nrse_gemm_params* p) {
  if (!p->a.kcontig || !p->b.kcontig || p->splits != 1) return false;
  if (p->a.chunk_shift != 0 || p->b.chunk_shift != 0 || p->a.seg_stride < 0 || p->b.seg_stride < 0) return false;
  if (p->M < 128 || p->N < 256 || p->K % 8) return false;
  if (!mode_ok(p) || !dma_layout_ok(p, 0)) return false;
  return (long long)nrse_cdiv(p->M, 112) * nrse_cdiv(p->N, BN) * p->batch < (1LL << 31);
}

int nrse_gemm2wg(const nrse_gemm_params* p, hipStream_t st) {
  const int bm = bm2(p);
  const int mt = nrse_cdiv(p->M, bm), nt = nrse_cdiv(p->N, BN);
  const long long total = (long long)mt * nt * p->batch;
  if (bm == 112)
    hipLaunchKernelGGL(gemm2wg_kernel<112>, dim3((unsigned)total), dim3(NTHR), 0, st, *p, mt, nt);
  else
    hipLaunchKernelGGL(gemm2wg_kernel<128>, dim3((unsigned)total), dim3(NTHR), 0, st, *p, mt, nt);
  return nrse_check_launch("nrse_gemm(2wg)");
}
