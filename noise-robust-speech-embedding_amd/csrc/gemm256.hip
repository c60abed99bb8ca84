// bf16 MFMA GEMM, generation 3: 256x256 output tile per workgroup, 8 waves, LDS-DMA staging
// pipelined across barriers.
//
// Same contract as nrse_gemm (include/nrse_hip.h); nrse_gemm dispatches here for large bf16
// problems (nrse_gemm256_ok). Why this shape (MI355X_MICROARCH.md / cdna_hip_programming.md §5):
//  - a 128x128 tile moves 64 FLOP per L2 byte; at ~30 TB/s of L2 that caps a GEMM near 2 PF
//    only with perfect L2 hits, and the 2-stage loop with a vmcnt(0) per K-step exposes the
//    load latency. 256x256 halves the bytes per FLOP and the per-wave tile (128x64, 32
//    accumulators of 16x16) doubles the MFMAs per LDS byte read.
//  - one K-tile (BK = 64) is 4 half-tiles of 16 KiB: A-lo = A rows {0-63,128-191}, A-hi = A rows
//    {64-127,192-255}, B-lo = B cols {wn*64 + 0..31}, B-hi = B cols {wn*64 + 32..63}. Each wave
//    computes its 128x64 output as 4 quadrants (64x32, 16 MFMAs) in 2 phases per K-tile:
//    phase 0 reads A-lo, B-lo, B-hi and runs quadrants (A-lo,B-lo), (A-lo,B-hi); phase 1 reads
//    A-hi into the A-lo registers and runs (A-hi,B-hi), (A-hi,B-lo) with the B fragments kept.
//    (r04: the r03 loop ran 4 phases of 16 MFMAs, 8 barriers per K-tile; 2 phases of 32 MFMAs
//    halve the barrier syncs, and a phase-0 read burst of 16 ds_read_b128 per wave (64 KiB per
//    CU, ~256 LDS cycles) still fits beside the partner's 512-cycle MFMA segment.)
//  - LDS is a ring of 10 half-tile slots (160 KiB). Half-tiles are numbered in first-read order
//    (seq = 4t + {A-lo, B-lo, B-hi, A-hi}), seq n lives in slot n % 10; phase 0 of K-tile t
//    stages seq 4t+8, 4t+9 and phase 1 seq 4t+10, 4t+11 (K-tile t+2): every DMA has >= 3 phases
//    (~1.5 us) before its data is needed.
//  - ping-pong: the waves with wm = 1 run one barrier behind those with wm = 0, so each SIMD
//    alternates one wave's 32-MFMA segment with the other wave's read+stage segment.
//    With the barriers numbered globally, group 0's phase P reads in (#2P-1, #2P) and its
//    MFMAs run in (#2P, #2P+1); group 1 is shifted by one. Hand-off rules that follow:
//      RAW: data read in phase Q is waited for (vmcnt) by every issuing wave before the FIRST
//           barrier of phase Q-1: vmcnt(12) in phase 0 retires A-hi(t), vmcnt(10) in phase 1
//           retires A-lo, B-lo, B-hi of K-tile t+1.
//      WAR: a slot is restaged one or two phases after its last read. Every read of the old
//           contents (both groups) has RETURNED before the barrier that precedes the restaging
//           DMA's issue (lgkmcnt(0) in that wait): merely issued was not enough -- a read queued
//           behind the phase's read burst was now and then overtaken by an L2-warm DMA.
//    No wait is vmcnt(0) and the barriers are raw s_barrier (no fence), so DMAs stay in flight
//    across them.
//  - tiles are numbered XCD-aware (consecutive tile ids on one XCD, T1) and grouped 8 M-tiles
//    deep so the 32 tiles an XCD runs at once share 8 A panels and 4 B panels in its L2.
//  - the 256x256 f32 result leaves through LDS in four 64-row passes with the same fused
//    epilogue as gemm_dma.hip (epi8).
#include <cstdlib>
#include <type_traits>

#include "gemm_common.h"

// NRSE_G3_STAMPS (diagnostic builds only): thread 0 of each workgroup writes s_memtime to
// ((u64*)p.colsum)[8 * wg + i] when the COLSUM flag is off (tools/diag_stamps.py): 0 entry,
// 1 after the prologue wait, 2 after the main loop, 3 after the epilogue's DMA drain, 4 / 5
// after pass 0's LDS staging / stores, 6 after pass 1's staging (general epilogue: after pass 1),
// 7 at the end.
#ifndef NRSE_G3_STAMPS
#define NRSE_G3_STAMPS 0
#endif
#if NRSE_G3_STAMPS
#define NRSE_STAMP(I)                                                                                 \
  do {                                                                                                \
    if (tid == 0 && p.colsum && !(p.flags & NRSE_EPI_COLSUM))                                         \
      reinterpret_cast<unsigned long long*>(p.colsum)[8 * (long long)blockIdx.x + (I)] =              \
          __builtin_amdgcn_s_memtime();                                                               \
  } while (0)
#else
#define NRSE_STAMP(I) ((void)0)
#endif
// NRSE_G3_PHASE_STAMPS (diagnostic builds only): threads 0 and 256 (one wave of each ping-pong
// group) of workgroup 0 write s_memtime after every main-loop barrier to ((u64*)p.aux)[group *
// 1024 + 8 * t + i] (tools/diag_phases.py; plain launches, where aux is unused).
#ifndef NRSE_G3_PHASE_STAMPS
#define NRSE_G3_PHASE_STAMPS 0
#endif
#if NRSE_G3_PHASE_STAMPS
#define NRSE_PSTAMP(I)                                                                                \
  do {                                                                                                \
    if (blockIdx.x == 0 && (tid & 255) == 0 && t < 128)                                               \
      ((unsigned long long*)(p.aux))[(tid >> 8) * 1024 + 8 * t + (I)] =                              \
          __builtin_amdgcn_s_memtime();                                                               \
  } while (0)
#else
#define NRSE_PSTAMP(I) ((void)0)
#endif

namespace {
using namespace nrse_gemm_detail;

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int HALF = 16384;             // 128 rows x 64 k bf16
constexpr int SLOTS = 10;               // ring of half-tile slots (2.5 K-tiles)
constexpr int LDS_BYTES = SLOTS * HALF; // 160 KiB: the whole LDS
constexpr int LEAD = 8;                 // half-tiles staged ahead of the phase being computed
constexpr int CT_LD = 260;          // f32 row stride of a 64 x 256 epilogue pass
static_assert(64 * CT_LD * 4 <= LDS_BYTES, "epilogue pass must fit the staging LDS");

// Row r (0..127) of half-tile hh of a panel -> row of the tile, or -1 (slot unused: zero fill).
//  A (BMT = 256 or 224 rows; M-wave wm owns rows wm*BMT/2 ..): the 64-row blocks
//    {wm*BMT/2 + hh*64 + (r & 63)}: the M-half mh = hh of both M-waves. At BMT = 224 an M-wave
//    has 112 rows, so its high half holds 48 (rows 48..63 of that block are unused).
//  B: the 32-col blocks {wn*64 + hh*32 : wn < 4} (the N-half nh = hh of all four N-waves)
template <bool IS_A, int BMT>
NRSE_DEV int tile_row(int hh, int r) {
  if constexpr (IS_A) {
    const int ri = r & 63;
    if (BMT != 256 && hh == 1 && ri >= BMT / 2 - 64) return -1;
    return (r >> 6) * (BMT / 2) + hh * 64 + ri;
  } else {
    return (r >> 5) * 64 + hh * 32 + (r & 31);
  }
}


// Operand loader. Every DMA source offset splits into a per-lane part fixed for the whole kernel
// (row/column inside the tile, 16-B chunk, k row inside the K-tile) and a wave-uniform part fixed
// per K-tile (segment + k0), which goes in the instruction's SGPR soffset: the main loop spends no
// vector instructions on addresses. Lanes outside the operand hold an out-of-range offset (zero
// fill); dead K-tiles (past the end) use a zero-record descriptor.
struct Ld {
  __amdgpu_buffer_rsrc_t rs, dead;
  long long ld, seg;
  unsigned voff[2][2];  // [half][instr] per-lane byte offset, or OOB
  int kpos[2][2];       // k of the lane inside the K-tile (K-tail masking)
};

template <bool KC, bool IS_A, int BMT>
NRSE_DEV void ld_init(Ld& o, const nrse_gemm_operand& d, const char* base, int wave, int lane, int row0,
                      int rows_total) {
  o.rs = make_rsrc(base);
  o.dead = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0, 0x00020000);
  o.ld = d.ld; o.seg = d.seg_stride;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = wave * 2 + j;
      if constexpr (KC) {
        // [row][k] image: 8 rows x 8 chunks per instruction, chunk position ^ ((row>>1)&7)
        const int r = 8 * i + (lane >> 3);
        const int tr = tile_row<IS_A, BMT>(hh, r);
        const int grow = row0 + tr;
        const int lc = (lane & 7) ^ ((r >> 1) & 7);
        o.voff[hh][j] = (tr >= 0 && grow < rows_total) ? (unsigned)(((long long)grow * o.ld + lc * 8) * 2) : OOB;
        o.kpos[hh][j] = lc * 8;
      } else {
        // [k][row] image: 4 k rows x 16 chunks per instruction, chunk position ^ fbank(k)
        const int k = 4 * i + (lane >> 4);
        const int lc = (lane & 15) ^ fbank(k);
        const int tr = tile_row<IS_A, BMT>(hh, lc * 8);   // 8-row chunks: wholly used or unused
        const int gcol = row0 + tr;
        o.voff[hh][j] = (tr >= 0 && gcol < rows_total) ? (unsigned)(((long long)k * o.ld + gcol) * 2) : OOB;
        o.kpos[hh][j] = k;
      }
    }
}

// uniform byte offset of K-tile (segment sg, k0)
template <bool KC>
NRSE_DEV unsigned ld_soff(const Ld& o, int sg, int k0) {
  return (unsigned)(((long long)sg * o.seg + (KC ? (long long)k0 : (long long)k0 * o.ld)) * 2);
}

// stage half-tile hh: the 2 DMA instructions of this thread; krem = K - k0 (< BK only on a tail)
NRSE_DEV void ld_issue(const Ld& o, char* dst, int wave, int hh, unsigned soff, int krem, bool live) {
  const __amdgpu_buffer_rsrc_t rs = live ? o.rs : o.dead;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    unsigned voff = o.voff[hh][j];
    if (krem < BK) voff = o.kpos[hh][j] < krem ? voff : OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + (wave * 2 + j) * 1024), 16, voff, soff, 0, 0);
  }
}

// fp8 correction-segment loader (ABI 6, nrse_gemm_params.a8 / b8): k-contiguous [row][k] bytes
// with the bf16 operand's element pitch (a8.ld == a.ld, a multiple of 64). One fp8 K-tile is 128 k
// = 128 bytes per row, the bf16 K-tile's bytes, so the LDS image, its swizzle, the ring and the
// fragment reads are the bf16 loader's, and so are the per-lane source offsets up to the pitch:
// bf16 row r, chunk c sits at 2 r ld + 16 c (2 r ld a multiple of 128), fp8 at r ld + 16 c. The fp8
// offsets are derived from the bf16 loader's at issue (no registers held for them). No K tail
// (the host requires K % 128 == 0).
struct Ld8 {
  __amdgpu_buffer_rsrc_t rs;
  long long seg;
};

NRSE_DEV void ld8_init(Ld8& o, const nrse_gemm_operand& d, const char* base) {
  o.rs = make_rsrc(base);
  o.seg = d.seg_stride;
}

NRSE_DEV unsigned ld8_soff(const Ld8& o, int sg, int ki) { return (unsigned)((long long)sg * o.seg + (long long)ki * 128); }

NRSE_DEV void ld8_issue(const Ld8& o, const Ld& l16, char* dst, int wave, int hh, unsigned soff, bool live = true) {
  const __amdgpu_buffer_rsrc_t rs = live ? o.rs : l16.dead;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const unsigned v = l16.voff[hh][j];
    const unsigned v8 = v >= OOB ? OOB : ((v & ~127u) >> 1) + (v & 127u);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + (wave * 2 + j) * 1024), 16, v8, soff, 0, 0);
  }
}

typedef int i32x4v __attribute__((ext_vector_type(4)));
typedef int i32x8v __attribute__((ext_vector_type(8)));
// both 32-deep fragments of a 64-deep bf16 K-tile (k-substeps 0, 1) as one 8-register tuple, which
// is also the operand of the fp8 MFMA over the same 128 bytes: A and B lanes read the same byte
// positions, so every byte of a row meets its partner whatever k the hardware assigns it
NRSE_DEV i32x8v frag2(const char* lds, int base, int lane) {
  const i32x4v a = __builtin_bit_cast(i32x4v, frag<true>(lds, base, 0, lane));
  const i32x4v b = __builtin_bit_cast(i32x4v, frag<true>(lds, base, 1, lane));
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
NRSE_DEV bf16x8 frag_half(i32x8v v, int s) {
  return s == 0 ? __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 0, 1, 2, 3))
                : __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 4, 5, 6, 7));
}
// fp8 operand of the 32x32x64 shape (F8 == 4): lane (h, r) = (lane >> 5, lane & 31) reads row
// base + r's 32-byte group 2s + h of the 128-k K-tile (k = 64s + 32h .. +31): chunks 2(2s+h),
// 2(2s+h)+1, conflict-free under the row swizzle like frag's chunk pairs
NRSE_DEV i32x8v frag_f32(const char* lds, int base, int s, int lane) {
  const int h = lane >> 5, row = base + (lane & 31), sw = (row >> 1) & 7, c = 2 * (2 * s + h);
  const char* r = lds + row * 128;
  const i32x4v a = *reinterpret_cast<const i32x4v*>(r + ((c ^ sw) << 4));
  const i32x4v b = *reinterpret_cast<const i32x4v*>(r + (((c + 1) ^ sw) << 4));
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------ register epilogue
// The common epilogues of the step run with their flags fixed at compile time: the lane's
// accumulator values are finished in registers -- bias, GELU (+ bf16 pre-activation to aux),
// GELU' from the bf16 aux, dropout, residual -- and only the final values go through LDS,
// packed as the output dtype, for 16-B coalesced row stores; column sums (bias gradients) are
// taken from the staged image. Lane (g, li) of accumulator [mh*4 + fi][fn] holds tile row
// wm*BMT/2 + mh*64 + fi*16 + li, columns wn*64 + fn*16 + 4g .. +3 (transposed MFMA). Two passes,
// one per M-half mh of both M-waves (128 image rows; an f32 image is 130 KB, a bf16 one leaves
// room for the pre-activation image). The dropout mask index is the general epilogue's.
// Other flag sets (atomic, accumulate, ReLU, tanh, f32 aux, ...) take the general epilogue.
// FE_NOAUX: GELU without the pre-activation image (the target view's FFN-up keeps no tape; it
// had fallen to the general epilogue's four f32 passes)
enum : int { FE_BIAS = 1, FE_GELU = 2, FE_GELUB = 4, FE_DROP = 8, FE_RESID = 16, FE_OBF = 32, FE_RBF = 64,
             FE_NOAUX = 128 };

// compile-time mode of the flag set, or -1 (general epilogue)
NRSE_DEV int fast_epi_mode(const nrse_gemm_params& p) {
  const int f = p.flags & ~NRSE_EPI_COLSUM;
  if (f & ~(NRSE_EPI_BIAS | NRSE_EPI_GELU | NRSE_EPI_GELU_BWD | NRSE_EPI_DROPOUT | NRSE_EPI_RESID)) return -1;
  if (p.c_dtype != NRSE_BF16 && p.c_dtype != NRSE_F32) return -1;
  int m = 0;
  if (f & NRSE_EPI_BIAS) m |= FE_BIAS;
  if (f & NRSE_EPI_GELU) {
    if (p.c_dtype != NRSE_BF16) return -1;
    if (!p.aux) m |= FE_NOAUX;
    else if (p.aux_dtype != NRSE_BF16) return -1;
    m |= FE_GELU;
  }
  if (f & NRSE_EPI_GELU_BWD) {
    if (!p.aux || p.aux_dtype != NRSE_BF16) return -1;
    m |= FE_GELUB;
  }
  if (f & NRSE_EPI_DROPOUT) m |= FE_DROP;
  if (f & NRSE_EPI_RESID) {
    if (p.resid_dtype != NRSE_F32) return -1;
    m |= FE_RESID;
  }
  if (p.c_dtype == NRSE_BF16) m |= FE_OBF;
  return m;
}

#ifndef NRSE_EPI_LDSBAR
#define NRSE_EPI_LDSBAR 1  // 0: the general epilogue's passes behind __syncthreads (A/B)
#endif
#ifndef NRSE_EPI_FASTBAR
#define NRSE_EPI_FASTBAR 1  // 0: the register epilogue's passes behind __syncthreads (A/B)
#endif
template <int FE, int BMT>
NRSE_DEV void fast_epilogue(const nrse_gemm_params& p, const f32x4 (&acc)[8][4], char* smem, int m0, int n0, int wm,
                            int wn, int lane, int tid, long long zq, long long zr, int split,
                            const float4 (&bpre)[4], int z, int mt) {
  constexpr bool BIAS = FE & FE_BIAS, GELU = FE & FE_GELU, GELUB = FE & FE_GELUB, DROP = FE & FE_DROP;
  constexpr bool RESID = FE & FE_RESID, OBF = FE & FE_OBF;
  constexpr bool GAUX = GELU && !(FE & FE_NOAUX);  // pre-activation image + stores
  constexpr int NFI_HI = (BMT / 2 - 64) / 16;
  constexpr int ES = OBF ? 2 : 4;
  constexpr int PITCH = 256 * ES + 16;               // image row pitch (bytes), bank-spread
  constexpr int APITCH = 256 * 2 + 16;
  const int g = lane >> 4, li = lane & 15;
  const Epi epi(p, zq, zr, split);
  const bool colsum = (p.flags & NRSE_EPI_COLSUM) != 0;
  // f32 output without column sums: stored straight from the registers (4 lanes write a row's
  // 64 contiguous bytes; measured 8 % faster on the out-proj shape than the LDS-staged rows,
  // while 32-byte bf16 row pieces measured slower, so those keep the staging)
  const bool DIRECT = !OBF && !colsum;
  const bool bias_on = BIAS && epi.bias_on;
  char* const oimg = smem;
  char* const aimg = smem + 128 * APITCH;            // pre-activation image (bf16 output only)
  float* const colacc = reinterpret_cast<float*>(smem + 150 * 1024);  // [2 M-waves][256 columns]
  float bias4[4][4];  // loaded before the main loop (bpre): no global-load latency here
#pragma unroll
  for (int fn = 0; fn < 4; ++fn) {
    bias4[fn][0] = bpre[fn].x; bias4[fn][1] = bpre[fn].y; bias4[fn][2] = bpre[fn].z; bias4[fn][3] = bpre[fn].w;
  }
  // The residual (RESID) and pre-activation (GELUB) operands of a pass are loaded as one batch of
  // branch-free buffer loads before its math (elements past M / N read zeros): loaded per element
  // group behind an `if (ok)`, each load sat in its own basic block and the pass waited for the
  // memory latency 16 times (s_waitcnt vmcnt(0) after every load; the out-projection's epilogue
  // was then longer than its main loop)
  // the image hand-offs between the passes need the LDS accesses retired, not the row stores
  // (NRSE_EPI_FASTBAR=0: __syncthreads, which also waits for every store of the pass)
  auto fast_bar = [] {
#if NRSE_EPI_FASTBAR
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#else
    __syncthreads();
#endif
  };
  __amdgpu_buffer_rsrc_t rrs, ars;
  if constexpr (RESID)
    rrs = make_rsrc(reinterpret_cast<const char*>((const float*)p.resid + epi.rbase + (long long)m0 * p.ldr + n0));
  if constexpr (GELUB)
    ars = make_rsrc(reinterpret_cast<const char*>((const bf16_t*)p.aux + epi.abase + (long long)m0 * p.ldaux + n0));
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    float4 rpre[4][4];
    uint2 apre[4][4];
    if constexpr (RESID || GELUB) {
#pragma unroll
      for (int fi = 0; fi < 4; ++fi) {
        if (pass == 1 && fi >= NFI_HI) continue;
        const int trow = wm * (BMT / 2) + pass * 64 + fi * 16 + li;
        const bool mok = m0 + trow < p.M;
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) {
          const int tcol = wn * 64 + fn * 16 + 4 * g;
          const bool ok = mok && n0 + tcol < p.N;
          if constexpr (RESID) {
            const unsigned off = ok ? (unsigned)((trow * p.ldr + tcol) * 4) : OOB;
            const auto r = __builtin_amdgcn_raw_buffer_load_b128(rrs, off, 0, 0);
            rpre[fi][fn] = make_float4(__uint_as_float(r[0]), __uint_as_float(r[1]), __uint_as_float(r[2]),
                                       __uint_as_float(r[3]));
          }
          if constexpr (GELUB) {
            const unsigned off = ok ? (unsigned)((trow * p.ldaux + tcol) * 2) : OOB;
            const auto r = __builtin_amdgcn_raw_buffer_load_b64(ars, off, 0, 0);
            apre[fi][fn] = make_uint2(r[0], r[1]);
          }
        }
      }
    }
#pragma unroll
    for (int fi = 0; fi < 4; ++fi) {
      if (pass == 1 && fi >= NFI_HI) continue;
      const int a = pass * 4 + fi;
      const int trow = wm * (BMT / 2) + pass * 64 + fi * 16 + li;
      const int prow = wm * 64 + fi * 16 + li;
      const int m = m0 + trow;
      const bool mok = m < p.M;
#pragma unroll
      for (int fn = 0; fn < 4; ++fn) {
        const int tcol = wn * 64 + fn * 16 + 4 * g;
        const int n = n0 + tcol;
        const bool ok = mok && n < p.N;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(acc[a][fn][e], p.alpha, BIAS ? bias4[fn][e] : 0.f);
        if constexpr (GELU) {
          if constexpr (GAUX) {
            uint2 u;
            u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
            u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
            *reinterpret_cast<uint2*>(aimg + prow * APITCH + tcol * 2) = u;
          }
          {  // packed FP32 pairs (FFN-up 773-775 -> 781-789 TF isolated; step neutral)
            const f32x2 g0 = gelu2(f32x2{v[0], v[1]}), g1 = gelu2(f32x2{v[2], v[3]});
            v[0] = g0.x; v[1] = g0.y; v[2] = g1.x; v[3] = g1.y;
          }
        }
        if constexpr (GELUB) {
          const uint2 u = apre[fi][fn];
          v[0] *= gelu_grad_fast(__uint_as_float(u.x << 16));
          v[1] *= gelu_grad_fast(__uint_as_float(u.x & 0xffff0000u));
          v[2] *= gelu_grad_fast(__uint_as_float(u.y << 16));
          v[3] *= gelu_grad_fast(__uint_as_float(u.y & 0xffff0000u));
        }
        if constexpr (DROP) {
          const long long ci = epi.cbase + (long long)m * p.ldc + n;
          if (!(p.flags & NRSE_EPI_DROP_AFTER)) {
            dropout_apply<4>(epi.key, (uint32_t)ci, epi.thresh, epi.dscale, v);
          }
        }
        if constexpr (RESID) {
          const float4 r = rpre[fi][fn];
          v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
        }
        if constexpr (DROP) {
          const long long ci = epi.cbase + (long long)m * p.ldc + n;
          if (p.flags & NRSE_EPI_DROP_AFTER) {
            dropout_apply<4>(epi.key, (uint32_t)ci, epi.thresh, epi.dscale, v);
          }
        }
        if constexpr (OBF) {
          uint2 u;
          u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          *reinterpret_cast<uint2*>(oimg + prow * PITCH + tcol * 2) = u;
        } else {
          if (DIRECT) {
            if (ok) *reinterpret_cast<float4*>((float*)p.c + epi.cbase + (long long)m * p.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
            *reinterpret_cast<float4*>(oimg + prow * PITCH + tcol * 4) = make_float4(v[0], v[1], v[2], v[3]);
          }
        }
      }
    }
    if (DIRECT) continue;
    fast_bar();
    NRSE_STAMP(4 + 2 * pass);
    if (colsum) {
      // column sums of the staged values (as stored: bf16-rounded for bf16 output): thread
      // (column c, M-wave h) sums the image rows of M-wave h; both passes into its own slot
      const int c = tid & 255, h = tid >> 8;
      const int vrows = pass == 1 ? NFI_HI * 16 : 64;
      const int mlim = p.M - (m0 + h * (BMT / 2) + pass * 64);
      const int nr = vrows < mlim ? vrows : (mlim > 0 ? mlim : 0);
      float sum = 0.f;
      const char* col = oimg + (h * 64) * PITCH + c * ES;
      auto at = [&](int r) {
        if constexpr (OBF) return bf2f(*reinterpret_cast<const bf16_t*>(col + r * PITCH));
        else return *reinterpret_cast<const float*>(col + r * PITCH);
      };
      if (nr == 64) {
        // full pass: 16 LDS reads in flight per batch, added in the same row order (the runtime
        // trip count had kept each read's latency in front of its add: +15 us on the FFN-down
        // dgrad, tools/bench_dgrad_gelu.py)
#pragma unroll
        for (int r0 = 0; r0 < 64; r0 += 16) {
          float t[16];
#pragma unroll
          for (int i = 0; i < 16; ++i) t[i] = at(r0 + i);
#pragma unroll
          for (int i = 0; i < 16; ++i) sum += t[i];
        }
      } else {
        for (int r = 0; r < nr; ++r) sum += at(r);
      }
      colacc[tid] = pass == 0 ? sum : colacc[tid] + sum;
    }
    // coalesced 16-B row stores of the image (and of the pre-activation image)
    constexpr int CPR = 256 * ES / 16;               // 16-B chunks per image row
#pragma unroll 4
    for (int idx = tid; idx < 128 * CPR; idx += 512) {
      const int prow = idx / CPR, ch = idx - prow * CPR;
      if (pass == 1 && (prow & 63) >= NFI_HI * 16) continue;
      const int m = m0 + (prow >> 6) * (BMT / 2) + pass * 64 + (prow & 63);
      const int n = n0 + ch * (16 / ES);
      if (m >= p.M || n >= p.N) continue;
      const uint4 u = *reinterpret_cast<const uint4*>(oimg + prow * PITCH + ch * 16);
      *reinterpret_cast<uint4*>((char*)p.c + (epi.cbase + (long long)m * p.ldc + n) * ES) = u;
      if constexpr (OBF) {
        // the fp8 copy of the stored bf16 values (ABI 6 c8: the next GEMM's correction operand)
        if (p.c8) {
          const uint2 w = fp8x8_from_bf16x8(u);
          *reinterpret_cast<uint2*>((unsigned char*)p.c8 + (long long)m * p.ldc8 + n) = w;
        }
      }
      if constexpr (GAUX) {
        const uint4 w = *reinterpret_cast<const uint4*>(aimg + prow * APITCH + ch * 16);
        *reinterpret_cast<uint4*>((bf16_t*)p.aux + epi.abase + (long long)m * p.ldaux + n) = w;
      }
    }
    fast_bar();
    if (pass == 0) NRSE_STAMP(5);
  }
  if (colsum && tid < 512 && n0 + (tid & 255) < p.N)
    colsum_out(p, z, mt, m0 / BMT, tid >> 8, n0 + (tid & 255), colacc[tid]);
}

// raw workgroup barrier: orders LDS accesses for the compiler, emits no vmcnt wait
#define NRSE_BAR()                            \
  do {                                        \
    asm volatile("" ::: "memory");            \
    __builtin_amdgcn_s_barrier();             \
    asm volatile("" ::: "memory");            \
  } while (0)

// BMT: tile rows, 256 or 224 (= 7 x 32: e.g. M = 12768 = 57 x 224 frames of 32 utterances fills
// 228 of the 256 CUs per N-column of tiles instead of 200; nrse_gemm256 picks the one that
// needs fewer tile waves, see bm_choice)
// F8: 0 bf16 K-tiles only; 1 the split-weight mode's fp8 correction segments after the bf16 K-tiles
// (ABI 6); 4 the fp8 segments on the 32x32x64 MFMA shape, the correction K-tiles first (BMT 256
// only). (2 and 3 were the MXFP6 forms of ABI 8, retired in ABI 11; 5, the bf16 K-tiles on
// 32x32x16, measured 2.5 % slower in the step in r05 and was retired with them.)
template <bool AKC, bool BKC, int BMT, int F8>
__global__ __launch_bounds__(NTHR, 1) void gemm256_kernel(const nrse_gemm_params p, int mt, int nt) {
  static_assert(BMT == 256 || BMT == 224, "tile rows");
  static_assert(!F8 || (AKC && BKC), "fp8 correction segments: k-contiguous operands");
  static_assert(F8 == 0 || F8 == 1 || F8 == 4, "kernel forms");
  static_assert(F8 < 4 || BMT == 256, "the 32x32 blocks tile 256-row tiles");
  constexpr bool W32 = F8 == 4;  // the fp8 correction on the 32x32x64 shape
  constexpr int NFI_HI = (BMT / 2 - 64) / 16;  // 16-row blocks in an M-wave's high half: 4 or 3
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  NRSE_STAMP(0);
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // XCD-aware, M-grouped tile order
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int per_z = mt * nt;
  const int z = wg / per_z;
  const int tt = wg - z * per_z;
#ifndef NRSE_GEMM_GM
#define NRSE_GEMM_GM 4
#endif
  // M-tiles per group of the tile order: r06 same-box step A/B 4 > 8 (+0.4-0.6 %) > 2 > 16 > 1
  // (profiles/r06_gemm_group_ab.txt; NRSE_GEMM_GM rebuilds another)
  constexpr int GM = NRSE_GEMM_GM;
  const int group = tt / (GM * nt);
  const int first_m = group * GM;
  const int gm = min(GM, mt - first_m);
  const int in_g = tt - group * GM * nt;
  const int m0 = (first_m + in_g % gm) * BMT;
  const int n0 = (in_g / gm) * BN;

  const int zb = z / p.splits;
  const int split = z % p.splits;
  const long long zq = zb / p.zdiv, zr = zb % p.zdiv;

  Ld la, lb;
  ld_init<AKC, true, BMT>(la, p.a, (const char*)p.a.ptr + (zq * p.a.z1 + zr * p.a.z2) * 2, wave, lane, m0, p.M);
  ld_init<BKC, false, BMT>(lb, p.b, (const char*)p.b.ptr + (zq * p.b.z1 + zr * p.b.z2) * 2, wave, lane, n0, p.N);

  const int tps = (p.K + BK - 1) / BK;
  const int seg0 = split * p.nseg;
  const int n16 = p.nseg * tps;               // bf16 K-tiles
  // fp8 correction K-tiles (128 k each) after them (F8; splits == 1)
  Ld8 la8, lb8;
  int tps8 = 1;
  if constexpr (F8 != 0) {
    ld8_init(la8, p.a8, (const char*)p.a8.ptr + zq * p.a8.z1 + zr * p.a8.z2);
    ld8_init(lb8, p.b8, (const char*)p.b8.ptr + zq * p.b8.z1 + zr * p.b8.z2);
    tps8 = p.K / 128;
  }
  const int ntiles = n16 + (F8 ? p.nseg8 * tps8 : 0);

  // K-tile t -> uniform source offsets of A and B and the K remainder; t >= ntiles -> dead
  struct TilePos { unsigned sa, sb; int krem; bool live; bool f8; };
  auto tile_pos_at = [&](bool live, int sgi, int ki, bool f8) {
    TilePos q;
    q.live = live;
    q.f8 = F8 && live && f8;
    if (q.f8) {
      q.sa = ld8_soff(la8, sgi, ki);
      q.sb = ld8_soff(lb8, sgi, ki);
      q.krem = BK;
      return q;
    }
    const int sg = seg0 + (live ? sgi : 0);
    const int k0 = (live ? ki : 0) * BK;
    q.sa = ld_soff<AKC>(la, sg, k0);
    q.sb = ld_soff<BKC>(lb, sg, k0);
    q.krem = p.K - k0;
    return q;
  };
  auto tile_pos = [&](int t) {
    if constexpr (W32) {  // correction K-tiles first
      const int n8 = ntiles - n16;
      if (t < n8) return tile_pos_at(true, t / tps8, t % tps8, true);
      return tile_pos_at(t < ntiles, (t - n8) / tps, (t - n8) % tps, false);
    }
    if (F8 && t >= n16) return tile_pos_at(t < ntiles, (t - n16) / tps8, (t - n16) % tps8, true);
    return tile_pos_at(t < ntiles, t / tps, t % tps, false);
  };
  // half-tile index j of a K-tile in staging (= first-read) order: 0 A-lo, 1 B-lo, 2 B-hi, 3 A-hi
  auto stage = [&](int j, const TilePos& q, int slot) {
    char* dst = smem + slot * HALF;
    if constexpr (F8 != 0) {
      if (q.f8) {
        if (j == 0) ld8_issue(la8, la, dst, wave, 0, q.sa);
        else if (j == 1) ld8_issue(lb8, lb, dst, wave, 0, q.sb);
        else if (j == 2) ld8_issue(lb8, lb, dst, wave, 1, q.sb);
        else ld8_issue(la8, la, dst, wave, 1, q.sa);
        return;
      }
    }
    if (j == 0) ld_issue(la, dst, wave, 0, q.sa, q.krem, q.live);
    else if (j == 1) ld_issue(lb, dst, wave, 0, q.sb, q.krem, q.live);
    else if (j == 2) ld_issue(lb, dst, wave, 1, q.sb, q.krem, q.live);
    else ld_issue(la, dst, wave, 1, q.sa, q.krem, q.live);
  };
  auto wrap = [](int x) { return x >= SLOTS ? x - SLOTS : x; };

  // this lane's epilogue bias columns (wn * 64 + fn * 16 + 4g .. +3), fetched now so that their
  // latency is hidden behind the main loop
  // (buffer loads: columns past N, no bias or split > 0 read zeros without a branch, so the
  // loads stay in flight under the prologue)
  float4 bpre[4];
  {
    const bool bon = (p.flags & NRSE_EPI_BIAS) && split == 0;
    const float* bb = bon ? p.bias + zq * p.bias_z1 + zr * p.bias_z2 : nullptr;
    const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc((void*)bb, 0, bon ? 0x7fffffff : 0, 0x00020000);
#pragma unroll
    for (int fn = 0; fn < 4; ++fn) {
      const int n = n0 + wn * 64 + fn * 16 + 4 * (lane >> 4);
      const unsigned off = n < p.N ? (unsigned)n * 4u : OOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(brs, off, 0, 0);
      bpre[fn] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    }
  }

  f32x4 acc[8][4];  // W32: assigned from the 32x32 accumulators after the correction tiles
  if constexpr (!W32) {
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // prologue: K-tiles 0 and 1 (half-tile sequence numbers 0..7, slot = seq % 10), then wait for
  // the three read in phase 0 (A-lo, B-lo, B-hi; 5 younger half-tiles = 10 DMAs may stay in flight)
  {
    const TilePos q0 = tile_pos(0), q1 = tile_pos(1);
#pragma unroll
    for (int j = 0; j < 4; ++j) stage(j, q0, j);
#pragma unroll
    for (int j = 0; j < 4; ++j) stage(j, q1, 4 + j);
  }
  asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  NRSE_BAR();
  NRSE_STAMP(1);

  bf16x8 fa[4][2], fbl[2][2], fbh[2][2];

#define NRSE_FRAG(KC, L, B, S, LN) frag<KC>(L, B, S, LN)
// transposed product (B fragment in the A slot): lane (g, i) of an accumulator holds output row i,
// columns 4g..4g+3, so the epilogue stages each quad into LDS with one 16-byte write
#define NRSE_MFMA(C, A, B) C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B, A, C, 0, 0, 0)
#define NRSE_READ_A(SLOT, NFI)                                                           \
  _Pragma("unroll") for (int fi = 0; fi < (NFI); ++fi)                                 \
  _Pragma("unroll") for (int s = 0; s < 2; ++s)                                        \
    fa[fi][s] = NRSE_FRAG(AKC, smem + (SLOT) * HALF, wm * 64 + fi * 16, s, lane);
#define NRSE_READ_B(SLOT, FB)                                                            \
  _Pragma("unroll") for (int fj = 0; fj < 2; ++fj)                                     \
  _Pragma("unroll") for (int s = 0; s < 2; ++s)                                        \
    FB[fj][s] = NRSE_FRAG(BKC, smem + (SLOT) * HALF, wn * 32 + fj * 16, s, lane);
// per-segment priority flips (r04: a static s_setprio 1 for the younger half instead,
// MI355X_MICROARCH.md two waves per SIMD item 4, measured 6 % slower on the step: 537-540 vs
// 507-508 pairs/s same box)
#define NRSE_QUAD(MH, NH, FB)                                                            \
  __builtin_amdgcn_s_setprio(1);                                                         \
  _Pragma("unroll") for (int s = 0; s < 2; ++s)                                        \
  _Pragma("unroll") for (int fi = 0; fi < ((MH) ? NFI_HI : 4); ++fi)                   \
  _Pragma("unroll") for (int fj = 0; fj < 2; ++fj)                                     \
    NRSE_MFMA(acc[(MH) * 4 + fi][(NH) * 2 + fj], fa[fi][s], FB[fj][s]);                  \
  __builtin_amdgcn_s_setprio(0);
// the wait before each phase's first barrier retires every half-tile the NEXT phase reads:
// phase 0 of K-tile t leaves the 6 youngest half-tiles in flight (retiring A-hi(t)), phase 1
// the 5 youngest (retiring A-lo, B-lo, B-hi of K-tile t+1). It also retires this wave's LDS
// reads of the phase (lgkmcnt(0)): the other group restages those slots right after this
// barrier, and a ds_read still queued behind the phase's read burst (up to ~500 LDS cycles at
// 128 ds_read_b128 per CU) could be overtaken by an L2-warm LDS-DMA landing in ~250-400 cycles
// -- a rare wrong fragment (tools/det_repro.py: target-view results differing in ~1 of 20
// concurrent forwards before this wait)
#define NRSE_WAIT(N) asm volatile("s_waitcnt vmcnt(" #N ") lgkmcnt(0)" ::: "memory")

  // ping-pong start: group 1 falls one barrier behind (schedule and hand-off rules: header)
  if (wm == 1) __builtin_amdgcn_s_barrier();
  int base = 0;  // slot of half-tile sequence number 4t
  if constexpr (F8 == 0) {
  // K-tile t+2 as (segment, K-tile within the segment), advanced by one per iteration: the
  // division by the segment's K-tile count stays out of the loop (done per iteration by all 8
  // waves on the CU's one scalar unit, it lengthened each K-tile's first phase by ~200 cycles)
  int u_sg = 2 / tps, u_k = 2 % tps;
#pragma unroll 1
  for (int t = 0; t < ntiles; ++t) {
    const int s0 = base, s1 = wrap(base + 1), s2 = wrap(base + 2), s3 = wrap(base + 3);
    // K-tile t+2 is staged over the two phases of K-tile t: A-lo, B-lo in phase 0 (sequence
    // 4t+8, 4t+9), B-hi, A-hi in phase 1 (4t+10, 4t+11)
    const TilePos q2 = tile_pos_at(t + 2 < ntiles, u_sg, u_k, false);
    if (++u_k == tps) { u_k = 0; ++u_sg; }
    // phase 0: quadrants (M-half 0, N-half 0) and (0, 1) from A-lo, B-lo, B-hi
    NRSE_READ_A(s0, 4)
    NRSE_READ_B(s1, fbl)
    NRSE_READ_B(s2, fbh)
    stage(0, q2, wrap(base + 8));
    stage(1, q2, wrap(base + 9));
    NRSE_WAIT(12);
    NRSE_BAR();
    NRSE_PSTAMP(0);
    NRSE_QUAD(0, 0, fbl)
    NRSE_QUAD(0, 1, fbh)
    NRSE_BAR();
    NRSE_PSTAMP(1);
    // phase 1: quadrants (1, 1) and (1, 0) from A-hi (into the A-lo registers) and the B
    // fragments still in registers
    NRSE_READ_A(s3, NFI_HI)
    stage(2, q2, base);  // (4t + 10) % 10
    stage(3, q2, s1);    // (4t + 11) % 10
    NRSE_WAIT(10);
    NRSE_BAR();
    NRSE_PSTAMP(2);
    NRSE_QUAD(1, 1, fbh)
    NRSE_QUAD(1, 0, fbl)
    NRSE_BAR();
    NRSE_PSTAMP(3);
    base = wrap(base + 4);
  }
  } else if constexpr (W32) {
  // fp8 correction on the 32x32x64 shape (e4m3 there runs at ~1.08x its 16x16x128 rate,
  // tools/probe_mx_rate.hip). The correction K-tiles run FIRST, into one 32x32 accumulator per
  // 32-row x 32-column block of the wave's 128 x 64 output (c32[MH*4 + NH*2 + bi]: M-half MH,
  // N-half NH, 32-row block bi), which are then permuted in registers into the 16x16 layout that
  // the bf16 K-tiles and the epilogue use. Same ring, phases, waits and hand-off rules as above;
  // per phase 8 MFMAs of 32x32x64 (two k-steps of 64 per 128-k K-tile) instead of 16 of 16x16x128.
  // every operand byte pair meets its partner whatever k the hardware assigns a lane's
  // 32 bytes (A and B lanes read the same positions); the weight operand carries 2^-b8_exp
  const int scw32 = 0x01010101 * (127 - p.b8_exp);
  f32x16 c32[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) c32[i][e] = 0.f;
  i32x8v fa32[2][2], fl32[2], fh32[2];
#define NRSE_READ_A32(SLOT)                                                              \
  _Pragma("unroll") for (int bi = 0; bi < 2; ++bi)                                     \
  _Pragma("unroll") for (int s = 0; s < 2; ++s)                                        \
    fa32[bi][s] = frag_f32(smem + (SLOT) * HALF, wm * 64 + 32 * bi, s, lane);
#define NRSE_READ_B32(SLOT, FB)                                                          \
  _Pragma("unroll") for (int s = 0; s < 2; ++s)                                        \
    FB[s] = frag_f32(smem + (SLOT) * HALF, wn * 32, s, lane);
#define NRSE_QUAD32(MH, NH, FB)                                                          \
  __builtin_amdgcn_s_setprio(1);                                                         \
  _Pragma("unroll") for (int s = 0; s < 2; ++s)                                        \
  _Pragma("unroll") for (int bi = 0; bi < 2; ++bi)                                     \
    c32[(MH) * 4 + (NH) * 2 + bi] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(   \
          FB[s], fa32[bi][s], c32[(MH) * 4 + (NH) * 2 + bi], 0, 0, 0, scw32, 0, 0x7f7f7f7f); \
  __builtin_amdgcn_s_setprio(0);
#define NRSE_BAR8()                          \
  do {                                       \
    __builtin_amdgcn_sched_barrier(0);       \
    NRSE_BAR();                              \
    __builtin_amdgcn_sched_barrier(0);       \
  } while (0)
  const int n8 = ntiles - n16;
  // staging cursors: correction tile t+2 while t+2 < n8, then bf16 tiles from index max(0, 2 - n8)
  int v_sg = 2 / tps8, v_k = 2 % tps8;
  const int b0 = n8 >= 2 ? 0 : 2 - n8;
  int u_sg = b0 / tps, u_k = b0 % tps;
  auto ktile32 = [&](int t, auto stage8) {
    constexpr bool S8 = decltype(stage8)::value;
    const int s0 = base, s1 = wrap(base + 1), s2 = wrap(base + 2), s3 = wrap(base + 3);
    TilePos q2;
    if constexpr (S8) {
      q2.live = true;
      q2.sa = ld8_soff(la8, v_sg, v_k);
      q2.sb = ld8_soff(lb8, v_sg, v_k);
      if (++v_k == tps8) { v_k = 0; ++v_sg; }
    } else {
      q2 = tile_pos_at(t + 2 < ntiles, u_sg, u_k, false);
      if (++u_k == tps) { u_k = 0; ++u_sg; }
    }
    auto stg = [&](int j, int slot) {
      if constexpr (S8) {
        char* dst = smem + slot * HALF;
        if (j == 0) ld8_issue(la8, la, dst, wave, 0, q2.sa);
        else if (j == 1) ld8_issue(lb8, lb, dst, wave, 0, q2.sb);
        else if (j == 2) ld8_issue(lb8, lb, dst, wave, 1, q2.sb);
        else ld8_issue(la8, la, dst, wave, 1, q2.sa);
      } else {
        stage(j, q2, slot);
      }
    };
    NRSE_READ_A32(s0)
    NRSE_READ_B32(s1, fl32)
    NRSE_READ_B32(s2, fh32)
    stg(0, wrap(base + 8));
    stg(1, wrap(base + 9));
    NRSE_WAIT(12);
    NRSE_BAR8();
    NRSE_QUAD32(0, 0, fl32)
    NRSE_QUAD32(0, 1, fh32)
    NRSE_BAR8();
    NRSE_READ_A32(s3)
    stg(2, base);
    stg(3, s1);
    NRSE_WAIT(10);
    NRSE_BAR8();
    NRSE_QUAD32(1, 1, fh32)
    NRSE_QUAD32(1, 0, fl32)
    NRSE_BAR8();
    base = wrap(base + 4);
  };
  int t = 0;
  const int n8a = n8 >= 2 ? n8 - 2 : 0;
#pragma unroll 1
  for (; t < n8a; ++t) ktile32(t, std::true_type{});
#pragma unroll 1
  for (; t < n8; ++t) ktile32(t, std::false_type{});
  // 32x32 -> 16x16: lane l of block (MH, NH, bi) holds row l % 32, columns 8j + 4(l / 32) + r in
  // register 4j + r; the 16x16 blocks [2bi + a][2NH + fj] want row 16a + (l % 16), columns 16fj +
  // 4(l / 16) + r. For each (fj, r) the register pair X0 = c[8fj + r], X1 = c[8fj + 4 + r] (16-lane
  // rows q0..q3) must become [X0.q0, X0.q2, X1.q0, X1.q2] (a = 0) and [X0.q1, X0.q3, X1.q1, X1.q3]
  // (a = 1): a permlane32 swap (X0's upper half <-> X1's lower) then a permlane16 swap (odd rows
  // of the first <-> even rows of the second), in place.
  auto convert = [&]() {
#pragma unroll
    for (int blk = 0; blk < 8; ++blk) {
      const int mh = blk >> 2, nh = (blk >> 1) & 1, bi = blk & 1;
#pragma unroll
      for (int fj = 0; fj < 2; ++fj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto w = __builtin_amdgcn_permlane32_swap(__float_as_uint(c32[blk][8 * fj + r]),
                                                          __float_as_uint(c32[blk][8 * fj + 4 + r]), false, false);
          const auto v = __builtin_amdgcn_permlane16_swap(w[0], w[1], false, false);
          acc[mh * 4 + 2 * bi][nh * 2 + fj][r] = __uint_as_float(v[0]);
          acc[mh * 4 + 2 * bi + 1][nh * 2 + fj][r] = __uint_as_float(v[1]);
        }
    }
  };
  convert();
  // the bf16 K-tiles (t + 2 staged as bf16 or dead)
  auto ktileb = [&](int t) {
    const int s0 = base, s1 = wrap(base + 1), s2 = wrap(base + 2), s3 = wrap(base + 3);
    const TilePos q2 = tile_pos_at(t + 2 < ntiles, u_sg, u_k, false);
    if (++u_k == tps) { u_k = 0; ++u_sg; }
    NRSE_READ_A(s0, 4)
    NRSE_READ_B(s1, fbl)
    NRSE_READ_B(s2, fbh)
    stage(0, q2, wrap(base + 8));
    stage(1, q2, wrap(base + 9));
    NRSE_WAIT(12);
    NRSE_BAR8();
    NRSE_QUAD(0, 0, fbl)
    NRSE_QUAD(0, 1, fbh)
    NRSE_BAR8();
    NRSE_READ_A(s3, 4)
    stage(2, q2, base);
    stage(3, q2, s1);
    NRSE_WAIT(10);
    NRSE_BAR8();
    NRSE_QUAD(1, 1, fbh)
    NRSE_QUAD(1, 0, fbl)
    NRSE_BAR8();
    base = wrap(base + 4);
  };
#pragma unroll 1
  for (; t < ntiles; ++t) ktileb(t);
#undef NRSE_READ_A32
#undef NRSE_READ_B32
#undef NRSE_QUAD32
#undef NRSE_BAR8
  } else {
  // The same schedule with the fp8 correction K-tiles after the bf16 ones (ABI 6). The fragments
  // are held as 8-register tuples (both k-substeps of a bf16 K-tile = one fp8 MFMA operand); a
  // bf16 K-tile runs its 32-deep halves as before, an fp8 K-tile runs one 128-deep MX-scaled MFMA
  // per (fi, fj) -- twice a bf16 MFMA's cycles for 4x its k: half the time per k. The weight
  // operand (our B, in the instruction's A slot) carries the scale 2^-b8_exp (E8M0), the
  // activation operand 1.0.
  i32x8v fa8[4], fbl8[2], fbh8[2];
  const int scw = 0x01010101 * (127 - p.b8_exp), sc1 = 0x7f7f7f7f;
#define NRSE_READ_A8(SLOT, NFI)                                                          \
  _Pragma("unroll") for (int fi = 0; fi < (NFI); ++fi)                                 \
    fa8[fi] = frag2(smem + (SLOT) * HALF, wm * 64 + fi * 16, lane);
#define NRSE_READ_B8(SLOT, FB)                                                           \
  _Pragma("unroll") for (int fj = 0; fj < 2; ++fj)                                     \
    FB[fj] = frag2(smem + (SLOT) * HALF, wn * 32 + fj * 16, lane);
#define NRSE_QUADH(MH, NH, FB)                                                           \
  __builtin_amdgcn_s_setprio(1);                                                         \
  _Pragma("unroll") for (int s = 0; s < 2; ++s)                                        \
  _Pragma("unroll") for (int fi = 0; fi < ((MH) ? NFI_HI : 4); ++fi)                   \
  _Pragma("unroll") for (int fj = 0; fj < 2; ++fj)                                     \
    NRSE_MFMA(acc[(MH) * 4 + fi][(NH) * 2 + fj], frag_half(fa8[fi], s), frag_half(FB[fj], s)); \
  __builtin_amdgcn_s_setprio(0);
// fp8 (F8 == 1): format 0 (e4m3) for both operands
#define NRSE_QUAD8(MH, NH, FB)                                                           \
  __builtin_amdgcn_s_setprio(1);                                                         \
  _Pragma("unroll") for (int fi = 0; fi < ((MH) ? NFI_HI : 4); ++fi)                   \
  _Pragma("unroll") for (int fj = 0; fj < 2; ++fj)                                     \
    acc[(MH) * 4 + fi][(NH) * 2 + fj] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4( \
          FB[fj], fa8[fi], acc[(MH) * 4 + fi][(NH) * 2 + fj], 0, 0, 0, scw, 0, sc1);      \
  __builtin_amdgcn_s_setprio(0);
// the raw barrier with scheduling fences: without them the compiler moved this loop's MFMAs across
// the phase barriers (out of their ping-pong segments), and fp8 K-tiles ran at half the bf16 rate
#define NRSE_BAR8()                          \
  do {                                       \
    __builtin_amdgcn_sched_barrier(0);       \
    NRSE_BAR();                              \
    __builtin_amdgcn_sched_barrier(0);       \
  } while (0)
  // K-tile t+2 as (segment, K-tile, fp8?) advanced per iteration (no divisions in the loop)
  bool u8 = 2 >= n16;
  int u_sg = u8 ? (2 - n16) / tps8 : 2 / tps, u_k = u8 ? (2 - n16) % tps8 : 2 % tps;
  // one K-tile of the schedule; the bf16 tiles and the fp8 tiles run in two loops, so neither
  // body branches around its MFMAs (a branch there made the compiler copy and spill the
  // accumulators between the two forms)
  auto ktile = [&](int t, auto kind) {
    constexpr bool K8 = decltype(kind)::value;
    const int s0 = base, s1 = wrap(base + 1), s2 = wrap(base + 2), s3 = wrap(base + 3);
    // K-tile t+2: in the fp8 loop it is an fp8 tile or dead, staged without a branch (a branch
    // around the DMA issue let the compiler sink this phase's MFMAs out of their segment)
    TilePos q2;
    if constexpr (K8) {
      q2.live = t + 2 < ntiles;
      q2.sa = ld8_soff(la8, u_sg, u_k);
      q2.sb = ld8_soff(lb8, u_sg, u_k);
      if (++u_k == tps8) { u_k = 0; ++u_sg; }
    } else {
      q2 = tile_pos_at(t + 2 < ntiles, u_sg, u_k, u8);
      if (++u_k == (u8 ? tps8 : tps)) {
        u_k = 0;
        if (++u_sg == p.nseg && !u8) { u8 = true; u_sg = 0; }
      }
    }
    auto stg = [&](int j, int slot) {
      if constexpr (K8) {
        char* dst = smem + slot * HALF;
        if (j == 0) ld8_issue(la8, la, dst, wave, 0, q2.sa, q2.live);
        else if (j == 1) ld8_issue(lb8, lb, dst, wave, 0, q2.sb, q2.live);
        else if (j == 2) ld8_issue(lb8, lb, dst, wave, 1, q2.sb, q2.live);
        else ld8_issue(la8, la, dst, wave, 1, q2.sa, q2.live);
      } else {
        stage(j, q2, slot);
      }
    };
    NRSE_READ_A8(s0, 4)
    NRSE_READ_B8(s1, fbl8)
    NRSE_READ_B8(s2, fbh8)
    stg(0, wrap(base + 8));
    stg(1, wrap(base + 9));
    NRSE_WAIT(12);
    NRSE_BAR8();
    if constexpr (K8) {
      NRSE_QUAD8(0, 0, fbl8)
      NRSE_QUAD8(0, 1, fbh8)
    } else {
      NRSE_QUADH(0, 0, fbl8)
      NRSE_QUADH(0, 1, fbh8)
    }
    NRSE_BAR8();
    NRSE_READ_A8(s3, NFI_HI)
    stg(2, base);
    stg(3, s1);
    NRSE_WAIT(10);
    NRSE_BAR8();
    if constexpr (K8) {
      NRSE_QUAD8(1, 1, fbh8)
      NRSE_QUAD8(1, 0, fbl8)
    } else {
      NRSE_QUADH(1, 1, fbh8)
      NRSE_QUADH(1, 0, fbl8)
    }
    NRSE_BAR8();
    base = wrap(base + 4);
  };
  int t = 0;
#pragma unroll 1
  for (; t < n16; ++t) ktile(t, std::false_type{});
#pragma unroll 1
  for (; t < ntiles; ++t) ktile(t, std::true_type{});
#undef NRSE_READ_A8
#undef NRSE_READ_B8
#undef NRSE_QUADH
#undef NRSE_QUAD8
#undef NRSE_BAR8
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();
  NRSE_STAMP(2);
#undef NRSE_READ_A
#undef NRSE_READ_B
#undef NRSE_QUAD
#undef NRSE_WAIT
#undef NRSE_FRAG
#undef NRSE_MFMA

  // ---------------------------------------------------------------- epilogue
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing zero-fill DMAs
  __syncthreads();
  NRSE_STAMP(3);
  const int flags = p.flags;
  {
    const int fe = fast_epi_mode(p);
    // the register epilogue, specialised at compile time for the flag sets the step issues
    // (forward kernels: A and B k-contiguous; dgrad: B row-contiguous)
#define NRSE_FE(MODE)                                                                            \
  case MODE:                                                                                     \
    fast_epilogue<MODE, BMT>(p, acc, smem, m0, n0, wm, wn, lane, tid, zq, zr, split, bpre, z, mt);   \
    NRSE_STAMP(7);                                                                               \
    return;
    if constexpr (AKC && BKC) {
      switch (fe) {
        NRSE_FE(FE_OBF)
        NRSE_FE(FE_OBF | FE_BIAS)
        NRSE_FE(FE_BIAS)
        NRSE_FE(FE_OBF | FE_BIAS | FE_GELU)
        NRSE_FE(FE_OBF | FE_BIAS | FE_GELU | FE_NOAUX)
        NRSE_FE(FE_BIAS | FE_DROP)
        NRSE_FE(FE_BIAS | FE_RESID)
        NRSE_FE(FE_BIAS | FE_RESID | FE_DROP)
        default: break;
      }
    } else if constexpr (AKC && !BKC) {
      switch (fe) {
        NRSE_FE(FE_OBF)
        NRSE_FE(0)
        NRSE_FE(FE_OBF | FE_GELUB)
        NRSE_FE(FE_OBF | FE_GELUB | FE_DROP)
        default: break;
      }
    }
    // (the weight gradients, both operands row-contiguous, keep the general epilogue: its 1-KB
    // row sweeps of the f32 slab measured 1-3 % faster than the register form's 64-B row pieces,
    // r04 same box: qkv / out / ffn1 / ffn2 wgrad 722 / 476 / 722 / 706 vs 709 / 461 / 714 / 685 TF)
#undef NRSE_FE
  }

  // ---------------------------------------------------------------- general epilogue: 4 x 64-row passes
  float* ct = reinterpret_cast<float*>(smem);
  Epi epi(p, zq, zr, split);
  epi.load_bias(p, n0 + (tid & 31) * 8);  // the epilogue columns of this thread (see the loop)
  const bool colsum = (flags & NRSE_EPI_COLSUM) != 0;
  const int ccol = tid & 255, chalf = tid >> 8;
  float csum = 0.f;
  const int g = lane >> 4, li = lane & 15;
  // the passes hand the staging area over with LDS-only barriers: a pass's row stores drain while
  // the next pass stages and stores (__syncthreads waited for every store of the pass, vmcnt(0));
  // epi8's own operand loads keep the compiler's counted waits
  auto gen_bar = [] {
#if NRSE_EPI_LDSBAR
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#else
    __syncthreads();
#endif
  };
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int prows = (pass & 1) ? NFI_HI * 16 : 64;  // rows of this pass: (M-wave, M-half)
    if (wm == (pass >> 1)) {
      const int mh = pass & 1;
#pragma unroll
      for (int fi = 0; fi < (mh ? NFI_HI : 4); ++fi)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          *reinterpret_cast<f32x4*>(ct + (fi * 16 + li) * CT_LD + wn * 64 + fn * 16 + 4 * g) = acc[mh * 4 + fi][fn];
    }
    gen_bar();
    if (pass == 0) NRSE_STAMP(4);
    const int mrow0 = m0 + (pass >> 1) * (BMT / 2) + (pass & 1) * 64;
    if (flags & NRSE_EPI_ATOMIC) {
      // one row per wave instruction: 64 lanes on 64 consecutive columns (256-B atomics)
      for (int row = wave; row < prows; row += 8) {
        const int m = mrow0 + row;
        if (m >= p.M) break;
#pragma unroll
        for (int hc = 0; hc < 4; ++hc) {
          const int col = hc * 64 + lane;
          const int n = n0 + col;
          if (n < p.N) atomicAdd((float*)p.c + epi.cbase + (long long)m * p.ldc + n, ct[row * CT_LD + col] * p.alpha);
        }
      }
    } else {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int sgi = tid + NTHR * it;
        const int row = sgi >> 5;
        const int cs = (sgi & 31) * 8;
        const int m = mrow0 + row, n = n0 + cs;
        float* cr = ct + row * CT_LD + cs;
        if (row >= prows || m >= p.M || n >= p.N) {
          if (colsum) {
#pragma unroll
            for (int e = 0; e < 8; ++e) cr[e] = 0.f;
          }
          continue;
        }
        epi8(p, epi, m, n, cr, colsum);
      }
      if (colsum) {
        gen_bar();
        for (int r = chalf * 32; r < chalf * 32 + 32; ++r) csum += ct[r * CT_LD + ccol];
      }
    }
    gen_bar();
    if (pass == 0) NRSE_STAMP(5);
    if (pass == 1) NRSE_STAMP(6);
  }
  if (colsum && n0 + ccol < p.N) colsum_out(p, z, mt, m0 / BMT, chalf, n0 + ccol, csum);
#if NRSE_G3_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  NRSE_STAMP(7);
}

// Tile rows: 256 by default. The automatic choice (NRSE_GEMM_BM=0) takes 224 when a problem
// needs no more waves of 256 workgroups (one per CU) than 256-row tiles do -- its tiles are 7/8
// the work, so alone on the chip the same number of waves finishes sooner (M = 12768, N = 1024:
// 228 instead of 200 tiles, both one wave; isolated forward / dgrad / wgrad 3-9 % faster). In the
// step the GEMMs share the chip with the other view's or stream's kernels, and the fewer, larger
// tiles leave those CUs: 570.1 / 570.7 vs 553.0 / 553.2 pairs/s same box
// (profiles/r04_s3_tile_rows_ab.txt). NRSE_GEMM_BM=224 pins the other; nrse_gemm_tile_rows too.
int g_tile_rows = -1;  // -1: not read yet, 0: automatic, 256 / 224: pinned

int tile_rows_setting() {
  if (g_tile_rows < 0) g_tile_rows = getenv("NRSE_GEMM_BM") ? atoi(getenv("NRSE_GEMM_BM")) : 256;
  return g_tile_rows;
}

// per-orientation overrides for step-level tuning: NRSE_GEMM_BM_FWD (A and B k-contiguous: the
// forward linears and convs), NRSE_GEMM_BM_DGRAD, NRSE_GEMM_BM_WGRAD (256, 224 or 0 = automatic);
// unset: the process setting above
int orient_rows(const nrse_gemm_params* p) {
  static int v[3] = {-2, -2, -2};
  static const char* names[3] = {"NRSE_GEMM_BM_FWD", "NRSE_GEMM_BM_DGRAD", "NRSE_GEMM_BM_WGRAD"};
  const int o = (p->a.kcontig && p->b.kcontig) ? 0 : (p->a.kcontig ? 1 : 2);
  if (v[o] == -2) v[o] = getenv(names[o]) ? atoi(getenv(names[o])) : -1;
  return v[o];
}

int bm_choice(const nrse_gemm_params* p) {
  const int ov = orient_rows(p);
  const int pinned = ov >= 0 ? ov : tile_rows_setting();
  if (pinned == 256 || pinned == 224) return pinned;
  const long long per = (long long)nrse_cdiv(p->N, BN) * p->batch * p->splits;
  const long long w256 = (nrse_cdiv(p->M, 256) * per + 255) / 256;
  const long long w224 = (nrse_cdiv(p->M, 224) * per + 255) / 256;
  return w224 <= w256 ? 224 : 256;
}

template <bool AKC, bool BKC, int F8 = 0>
int launch(const nrse_gemm_params* p, hipStream_t st) {
  if constexpr (F8 >= 4) {
    const int mt = nrse_cdiv(p->M, 256), nt = nrse_cdiv(p->N, BN);
    const long long total = (long long)mt * nt * p->batch * p->splits;
    hipLaunchKernelGGL((gemm256_kernel<AKC, BKC, 256, F8>), dim3((unsigned)total), dim3(NTHR), 0, st, *p, mt, nt);
    return nrse_check_launch("nrse_gemm(256)");
  }
  const int bm = bm_choice(p);
  const int mt = nrse_cdiv(p->M, bm), nt = nrse_cdiv(p->N, BN);
  const long long total = (long long)mt * nt * p->batch * p->splits;
  if constexpr (F8 < 4) {
    if (bm == 224)
      hipLaunchKernelGGL((gemm256_kernel<AKC, BKC, 224, F8>), dim3((unsigned)total), dim3(NTHR), 0, st, *p, mt, nt);
    else
      hipLaunchKernelGGL((gemm256_kernel<AKC, BKC, 256, F8>), dim3((unsigned)total), dim3(NTHR), 0, st, *p, mt, nt);
  }
  return nrse_check_launch("nrse_gemm(256)");
}

}  // namespace

extern "C" int nrse_gemm_tile_rows(int rows) {
  const int prev = tile_rows_setting();
  g_tile_rows = (rows == 256 || rows == 224) ? rows : 0;
  return prev;
}

long long nrse_gemm256_tiles(const nrse_gemm_params* p) {
  return (long long)nrse_cdiv(p->M, BM) * nrse_cdiv(p->N, BN) * p->batch * p->splits;
}

bool nrse_gemm256_ok(const nrse_gemm_params* p) {
  return p->M >= 128 && p->N >= 128 && p->a.chunk_shift == 0 && p->b.chunk_shift == 0 &&
         p->a.seg_stride >= 0 && p->b.seg_stride >= 0 && dma_layout_ok(p, 256) &&
         nrse_gemm256_tiles(p) < (1LL << 31);
}

int nrse_gemm256_rows(const nrse_gemm_params* p) { return bm_choice(p); }

// the ABI-6 fp8 correction segments' conditions (nrse_gemm checks them before routing here)
bool nrse_gemm256_f8_ok(const nrse_gemm_params* p) {
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  auto m16 = [](long long x) { return (x & 15) == 0; };
  const nrse_gemm_operand* o8[2] = {&p->a8, &p->b8};
  for (const nrse_gemm_operand* o : o8) {
    if (!o->ptr || o->dtype != p->a8.dtype || !o->kcontig || o->chunk_shift != 0 || !al16(o->ptr) ||
        !m16(o->seg_stride) || !m16(o->z1) || !m16(o->z2) || o->seg_stride < 0)
      return false;
  }
  // the fp8 rows share the bf16 operands' element pitch (the loader derives its offsets from theirs)
  if (p->a8.ld != p->a.ld || p->b8.ld != p->b.ld || (p->a.ld & 63) || (p->b.ld & 63)) return false;
  const long long spa = (long long)(p->nseg8 - 1) * p->a8.seg_stride + (long long)p->M * p->a8.ld + p->K;
  const long long spb = (long long)(p->nseg8 - 1) * p->b8.seg_stride + (long long)p->N * p->b8.ld + p->K;
  if (p->a8.dtype != NRSE_FP8) return false;
  return p->K % 128 == 0 && p->splits == 1 && p->a.kcontig && p->b.kcontig && spa < (1LL << 31) &&
         spb < (1LL << 31) && p->b8_exp > -127 && p->b8_exp < 127;
}

// fp8 segments on the 32x32x64 shape (F8 = 4: e4m3 there runs at ~1.08x its 16x16x128 rate,
// tools/probe_mx_rate.hip; bf16sw step +1.4 %, profiles/r05_step_ab.txt) unless NRSE_FP8_SHAPE=16
// (the 16x16x128 form, F8 = 1)
static bool fp8_wide() {
  static int v = -1;
  if (v < 0) v = (getenv("NRSE_FP8_SHAPE") && atoi(getenv("NRSE_FP8_SHAPE")) == 16) ? 0 : 1;
  return v == 1;
}

int nrse_gemm256(const nrse_gemm_params* p, hipStream_t st) {
  if (p->nseg8 > 0) {
    // (the 32x32 form tiles 256 rows: a problem pinned to 224-row tiles keeps the 16x16 form, whose
    // row count the column-sum workspace was sized for)
    const bool r256 = bm_choice(p) == 256;
    return fp8_wide() && r256 ? launch<true, true, 4>(p, st) : launch<true, true, 1>(p, st);
  }
  if (p->a.kcontig && p->b.kcontig) return launch<true, true>(p, st);
  if (p->a.kcontig && !p->b.kcontig) return launch<true, false>(p, st);
  if (!p->a.kcontig && p->b.kcontig) return launch<false, true>(p, st);
  return launch<false, false>(p, st);
}
