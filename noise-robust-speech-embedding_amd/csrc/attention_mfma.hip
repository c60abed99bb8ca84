// MFMA flash attention for the gated relative-position attention of WavLM (bf16 operands, f32
// softmax/accumulation), head_dim 64:
//   scores = (q . k) / 8 + gate[b,h,i] * bias[h,i,j]   ([TF]modeling_wavlm.py:164-184)
//   P = softmax_j(scores), dropout(P), O = P V         ([TORCH]functional.py:6629 SDPA)
// Three kernels, all 256 threads = 4 waves, one wave = 16 rows, 64-row tiles staged in LDS:
//   fwd   : grid (q-blocks, H, B); S^T = K Q^T so the softmax row (one query) is lane-local
//           (lane = query, 16 keys per lane per 64-key tile); online softmax; P feeds P.V
//           straight from registers (permuted k order) with V read by ds_read_b64_tr_b16.
//   bwd_kv: grid (k-blocks, H, B); S = Q K^T (lane = key); dV += Pd^T dO, dK += dS^T Q with the
//           accumulator tiles used as MFMA A operands; sum_b gate*dS accumulated per diagonal
//           j-i in LDS (rel_attn_embed gradient) then one atomic per diagonal per workgroup.
//   bwd_q : grid (q-blocks, H, B); dQ^T += K^T dS^T (K by transposed LDS read; lane = query, so
//           dQ leaves in 8-byte runs), dgate = sum_j dS*bias.
// LDS tiles are [64 rows][64 bf16] (128-byte rows) with the 16-byte chunk XOR-swizzled by
// ((row>>1)&3)<<1 so both ds_read_b128 row reads and ds_read_b64_tr_b16 column reads of one
// image stay (nearly) conflict-free.
#include <type_traits>

#include "common.h"

namespace {

constexpr int D = 64;
constexpr int TILE_B = 64 * 128;  // bytes per 64x64 bf16 tile
// dK/dV kernel: diagonal accumulator arrays of ndiag(T) = Tp + 80 floats, the diagonal d = kj - qi
// of the block at index d - (kb0 - T + 1) + dpad(T); dpad >= Tp - T + 13 covers the lowest index
// (the carried accumulator at qend = Tp), the top is T + 62 + dpad < ndiag
NRSE_DEV int diag_pad(int T) { return ((T + 63) & ~63) - T + 16; }
NRSE_DEV int diag_len(int T) { return ((T + 63) & ~63) + 80; }
// Softmax runs in the base-2 domain (v_exp_f32 is 2^x): scores are formed as
// log2(e) * (q.k / 8 + gate * bias) with the log2(e) folded into the per-row constants, so each
// element costs one fma + one exp; lse is stored in natural-log units.
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
NRSE_DEV float exp2_(float x) { return __builtin_amdgcn_exp2f(x); }
typedef short short8v __attribute__((ext_vector_type(8)));

NRSE_DEV int loff(int row, int chunk) { return row * 128 + ((chunk ^ (((row >> 1) & 3) << 1)) << 4); }

// 16-byte row fragment (MFMA A/B operand "row" layout): row, 8 contiguous d starting at 8*chunk
NRSE_DEV bf16x8 rd_row(const char* t, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(t + loff(row, chunk));
}

// transposed fragment: lane (group g, i=l&15) gets rows r0+4g.. (elements 0..3) and
// r1+4g.. (elements 4..7) of column c0 + i
NRSE_DEV bf16x8 rd_tr(const char* t, int r0, int r1, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int q = i >> 2, p = i & 3;
  const int col = c0 + 4 * p;
  const int chunk = col >> 3, half = (col >> 2) & 1;
  short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)(t + loff(r0 + 4 * g + q, chunk) + half * 8));
  short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)(t + loff(r1 + 4 * g + q, chunk) + half * 8));
  short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Register r of a 16x16 MFMA C block rotated left by r lanes within each 16-lane row (DPP
// row_ror:(16 - r): lane x receives lane (x + r) mod 16), added to the accumulator of its
// diagonal: lo if the rotation did not wrap, hi (16 further down) if it did. The wrap test is a
// per-lane constant, so it enters as 0/1 multipliers (mlo = 1 - mhi) and each half is one fma.
#ifndef NRSE_DIAG_DPPADD
#define NRSE_DIAG_DPPADD 1
#endif
template <int R>
NRSE_DEV void diag_rot(float v, float mlo, float mhi, float& lo, float& hi) {
#if NRSE_DIAG_DPPADD
  // the two halves of the rotation as row shifts (lanes with no source read 0), each folded by
  // the compiler into a v_add_f32 with a DPP source: 2 VALU instead of a DPP move + 2 FMAs
  (void)mlo; (void)mhi;
  lo += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x100 + R, 0xF, 0xF, true));
  hi += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x110 + 16 - R, 0xF, 0xF, true));
#else
  const float u = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + 16 - R, 0xF, 0xF, false));
  lo = fmaf(u, mlo, lo);
  hi = fmaf(u, mhi, hi);
#endif
}

NRSE_DEV bf16x8 pack8(const float* a, const float* b) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = (__bf16)a[j]; v[4 + j] = (__bf16)b[j]; }
  return v;
}

// Workgroup -> (query/key block, head, utterance). The grid is 1-D; workgroup i runs on XCD
// i % 8. With H % 8 == 0 each XCD gets H/8 heads for every utterance, so the [H, T, Tb] f32
// relative-position bias rows of its heads (2 x 0.7 MB at T = 399) stay in that XCD's 4 MB L2
// across all B utterances instead of streaming from the Infinity Cache per workgroup, and the
// blocks of one (b, h) run back to back on one XCD (their K/V tiles shared in L2).
struct BlockPos { int blk, h, b; };
NRSE_DEV BlockPos block_pos(int nblk, int H) {
  const int id = blockIdx.x;
  if ((H & 7) == 0) {
    const int hx = H >> 3;
    const int xcd = id & 7, local = id >> 3;
    const int blk = local % nblk;
    const int r = local / nblk;
    return BlockPos{blk, xcd * hx + r % hx, r / hx};
  }
  return BlockPos{id % nblk, (id / nblk) % H, id / (nblk * H)};
}

// ------------------------------------------------------------------------------ shared staging
// K / V tiles by LDS-DMA (buffer_load ... lds): a 64-row x 128-B tile is 8 wave-instructions of
// 1 KiB (8 rows each); 4 waves issue 2 each. Lane l of instruction j of wave w writes LDS bytes
// (2w+j)*1024 + 16 l = row (2w+j)*8 + l/8, 16-B position l%8, which in the swizzled image holds
// logical chunk (l%8) ^ sw(row): the swizzle goes into the per-lane SOURCE address. Rows past the
// utterance (>= T) are out of the descriptor's range and land as zeros.
typedef __attribute__((address_space(3))) void lds_void_t;

struct KvDma {
  __amdgpu_buffer_rsrc_t rs;
  unsigned voff[2];  // row offset (tile row 0) + column offset of this lane's piece, per instruction
  unsigned ld_b;     // row stride in bytes
};

// col_b: byte offset of the 64-wide column block inside a row
NRSE_DEV KvDma kv_dma_init(const bf16_t* utt_base, int T, long long ld, int col_b, int wave, int lane) {
  KvDma d;
  d.ld_b = (unsigned)(ld * 2);
  d.rs = __builtin_amdgcn_make_buffer_rsrc((void*)utt_base, 0, (int)((long long)T * ld * 2), 0x00020000);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wave * 2 + j) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ (((row >> 1) & 3) << 1);
    d.voff[j] = (unsigned)row * d.ld_b + (unsigned)col_b + (unsigned)chunk * 16;
  }
  return d;
}

// stage rows row0 .. row0+63 into the tile at `tile` (wave-uniform LDS address)
NRSE_DEV void kv_dma_issue(const KvDma& d, char* tile, int row0, int wave) {
  const unsigned roff = (unsigned)row0 * d.ld_b;
#pragma unroll
  for (int j = 0; j < 2; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(d.rs, (lds_void_t*)(tile + (wave * 2 + j) * 1024), 16, d.voff[j] + roff,
                                             0, 0, 0);
}

// The relative-position bias of a query block (64 queries from q0) over all keys, as 4 shifted
// copies of the Toeplitz vector segment it touches: copy s holds vec[e_lo + j + s], e_lo =
// T - 1 - q0 - 63 (values outside [0, 2T-1) are zero). A lane whose 4 consecutive elements start
// at segment index u reads them with one aligned ds_read_b128 from copy (u & 3) at u - (u & 3).
// Copy length: a lane reads 4 floats at (u00 - (u00 & 3)) + kb + 16t <= 72 + (Tp - 64) + 48, so
// Tp + 64 entries cover every read (Tp = T rounded up to the 64-key tile); the fwd kernel's LDS
// is then 32 KB of K/V tiles + 4 (Tp + 64) floats = 40 KB at T = 399: 4 workgroups per CU.
__host__ __device__ inline int bv_len(int T) { return ((T + 63) & ~63) + 64; }
// Inside copy s, segment element j sits at bv_pos(j, s): rotated by 16 s within its 64-float
// block (a 256-B bank row). One ds_read_b128 lane group reads 3 aligned positions 4-12 floats
// apart from all 4 copies; with the copies one bank row apart and unrotated, the 4 copies of a
// position were 4 addresses on the same 4 banks, a 4-way conflict. Rotated by 4 slots per copy,
// the 12 addresses take 12 distinct 16-B slots (PMC, profiles/r04_s3_attn_lds_pmc.txt:
// SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.368 -> 0.0 forward, 0.296 -> 0.0 dQ, 0.302 -> 0.19
// dK/dV; time unchanged, the kernels are VALU-bound). An aligned float4 never straddles a block,
// and bv_pos(j + 64 m, s) = bv_pos(j, s) + 64 m: a lane keeps one offset per 16-key sub-tile.
__host__ __device__ inline int bv_pos(int j, int s) { return (j & ~63) | ((j + 16 * s) & 63); }
// The loads are unconditional (an index outside [0, 2T-1) reads a clamped one and is zeroed after)
// and issued two strides at a time before their LDS stores: behind a conditional each load had
// waited for its own round trip, in every workgroup's prologue.
NRSE_DEV float clamped_ld(const float* v, int e, int n) { return v[e < 0 ? 0 : (e >= n ? n - 1 : e)]; }
NRSE_DEV void bv_stage(float* bv, const float* vec, int T, int q0, int tid) {
  const int len = bv_len(T), nd = 2 * T - 1;
  const int e_lo = T - 1 - q0 - 63;
  for (int j0 = tid; j0 < len; j0 += 512) {
    float v[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int s = 0; s < 4; ++s) v[u][s] = clamped_ld(vec, e_lo + j0 + 256 * u + s, nd);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = j0 + 256 * u;
      if (j < len) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int e = e_lo + j + s;
          bv[s * len + bv_pos(j, s)] = (e >= 0 && e < nd) ? v[u][s] : 0.f;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------ forward
// One workgroup = 64 queries (4 waves x 16) of one (b, h); K/V tiles double-buffered in LDS by
// LDS-DMA, the next tile in flight while the current one is computed (one barrier per tile);
// the gated bias gate[b,h,i] * vec[h, j-i+T-1] from the LDS Toeplitz copies.
// DM: dropout mode, a compile-time branch (the runtime one made the compiler copy every
// probability register across it, 16 v_mov per key tile): 0 none, 1 the pair hash in the kernel
// (and its keep bits recorded to drop_mask if given), 2 the keep bits read from drop_mask
// (nrse_attn_dropout_mask computed them ahead, beside the GEMMs: the hash and the bit assembly
// were about half of this VALU-bound loop's issue cycles)
// 4 waves per SIMD (<= 128 VGPRs; the LDS fits 4 workgroups per CU): the dropout forms had
// allocated 130 VGPRs, 3 waves (r06 A/B: recorded-mask forward 70.6-72.1 -> 68.4-68.5 us, the
// step neutral, profiles/r06_attn_fwd_waves_ab.txt); 0 leaves the occupancy to the compiler
#ifndef NRSE_ATTN_FWD_WAVES
#define NRSE_ATTN_FWD_WAVES 4
#endif
#if NRSE_ATTN_FWD_WAVES
#define NRSE_FWD_OCC __attribute__((amdgpu_waves_per_eu(NRSE_ATTN_FWD_WAVES, NRSE_ATTN_FWD_WAVES)))
#else
#define NRSE_FWD_OCC
#endif
template <int DM>
__global__ __launch_bounds__(256) NRSE_FWD_OCC void attn_fwd_kernel(const nrse_attn_fwd_params p) {
  constexpr bool DROP = DM != 0;
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  char* const kv0 = dyn;                       // [2 buffers][K tile, V tile]
  float* const bv = reinterpret_cast<float*>(dyn + 4 * TILE_B);
  const int T = p.T, H = p.H, Hd = H * D;
  const long long ld3 = 3LL * Hd;
  const BlockPos bp = block_pos((p.T + 63) / 64, p.H);
  const int b = bp.b, h = bp.h;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  const int q0 = bp.blk * 64;
  const int qi = q0 + w * 16 + i16;
  const bool qv = qi < T;
  // a wave whose 16 queries all lie past T (the last query block's tail: 3 of its 4 waves at
  // T = 399) keeps its share of the K/V staging and the barriers but skips the tile math
  const bool wlive = q0 + w * 16 < T;
  const bf16_t* qkv = (const bf16_t*)p.qkv + (long long)b * T * ld3;
  const KvDma kd = kv_dma_init(qkv, T, ld3, (Hd + h * D) * 2, w, lane);
  const KvDma vd = kv_dma_init(qkv, T, ld3, (2 * Hd + h * D) * 2, w, lane);
  const int ntiles = (T + 63) / 64;
  kv_dma_issue(kd, kv0, 0, w);
  kv_dma_issue(vd, kv0 + TILE_B, 0, w);
  bv_stage(bv, p.bias_vec + (long long)h * (2 * T - 1), T, q0, tid);
  // Q fragments (B operand of S^T = K Q^T): Q[qi][8g + 32s .. +8]
  bf16x8 qf[2];
  const int qc = qv ? qi : T - 1;  // loads from a clamped row, zeroed after (no branch around them)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    uint4 u = *reinterpret_cast<const uint4*>(qkv + (long long)qc * ld3 + h * D + 8 * g + 32 * s);
    if (!qv) u = make_uint4(0, 0, 0, 0);
    qf[s] = __builtin_bit_cast(bf16x8, u);
  }
  const long long bh = (long long)b * H + h;
  const float gi0 = p.gate[bh * T + qc];
  const float gi = qv ? gi0 : 0.f;
  const float c1 = p.scale * LOG2E, gl = gi * LOG2E;
  // bias copy and base for this lane: segment index u0 = kb + 4g + 63 - (qi - q0)
  const int bvl = bv_len(T);
  const int u00 = 4 * g + 63 - (w * 16 + i16);
  const int bsel = u00 & 3;
  const float* bvl_base = bv + bsel * bvl;  // copy bsel, rotated as bv_pos
  int boff[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) boff[t] = bv_pos(u00 - bsel + 16 * t, bsel);
  const uint32_t key = site_key(p.seed);
  const uint32_t thr = dropout_threshold16(p.dropout_p);
  constexpr bool drop = DROP;
  const float dsc = drop ? 1.f / (1.f - p.dropout_p) : 1.f;
  const int Tp = ntiles * 64;
  // this lane's query row: key pair (kb + 16t + 4g)/2 + rp holds elements r = 2rp, 2rp + 1
  const uint32_t rowpair = (uint32_t)(bh * T + qi) * (uint32_t)((T + 1) >> 1) + (uint32_t)(2 * g);
  // DM 2: word (bh, key tile, g, qi) of the precomputed bits, the next tile's word loaded while the
  // current tile computes (the top-of-tile vmcnt(0) covers it)
  const uint16_t* mrow = DM == 2 ? p.drop_mask + (bh * ntiles * 4 + g) * (long long)(ntiles * 64) + (qv ? qi : 0)
                                 : nullptr;
  uint32_t mnext = DM == 2 ? (uint32_t)mrow[0] : 0u;
  // Lazy rescaling in the base-2 domain: mref is the row's reference maximum, and a tile's scores
  // are formed relative to it in two packed fmas, v = s * c1 + (gl * bias - mref) (no separate
  // subtract before the exponential). Only when some lane of the wave sees a score more than
  // RESCALE_TAU above its reference (or on the first tile, where mref is not yet set) does the
  // wave shift: mref += shift, v -= shift, o and the row sum by 2^-shift. Probabilities stay
  // <= 2^RESCALE_TAU before normalisation, which f32 holds exactly as well as values <= 1; the
  // output divides by the same row sum, so only bf16 rounding of P differs from rescaling per tile.
  constexpr float RESCALE_TAU = 8.f;
  float mref = 0.f;
  f32x2 lpart2 = {0.f, 0.f};
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // In the last key tile the keys past T get -inf scores, so probability 0 whatever the dropout
  // hash says; every sub-tile is hashed (a per-sub-tile branch made the compiler copy the
  // probability registers across it on every tile).
  // LAST: the tile that may hold keys past T (their masking compiled only into it: in the loop of
  // the other tiles it was 16 compares + 16 selects per tile, if-converted by the compiler)
  auto tile = [&](const int it, auto last_c) {
    constexpr bool LAST = decltype(last_c)::value;
    const int kb = it * 64;
    char* const Kt = kv0 + (it & 1) * 2 * TILE_B;
    char* const Vt = Kt + TILE_B;
    // tile `it` landed (the only DMAs in flight) and, on the first tile, the bias copies written
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // this tile's bias rows, read BEFORE the prefetch is issued: a read of the bias copies after
    // it made the compiler wait for the prefetch (s_waitcnt vmcnt(0): it cannot tell the copies
    // from the DMA's destination) right after the first S MFMAs (r06: p = 0 forward 54-55 -> 52-53 us)
    float4 bb4[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) bb4[t] = *reinterpret_cast<const float4*>(bvl_base + kb + boff[t]);
    // prefetch tile it+1 into the other buffer (its last readers finished before this barrier)
    const uint32_t mcur = mnext;
    if (!LAST || it + 1 < ntiles) {
      char* const Kn = kv0 + ((it + 1) & 1) * 2 * TILE_B;
      kv_dma_issue(kd, Kn, kb + 64, w);
      kv_dma_issue(vd, Kn + TILE_B, kb + 64, w);
      if (DM == 2) mnext = mrow[(long long)(it + 1) * 4 * (ntiles * 64)];
    }
    if (!wlive) return;
    // the MFMAs run on every sub-tile (a conditional MFMA makes the compiler stage its result
    // through AGPRs)
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rd_row(Kt, 16 * t + i16, 4 * ss + g), qf[ss], s[t], 0, 0, 0);
    }
    float v[4][4];
    const f32x2 c12 = {c1, c1}, gl2 = {gl, gl}, nm2 = {-mref, -mref};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 bb = bb4[t];
      const f32x2 r0 = pk_fma(f32x2{s[t][0], s[t][1]}, c12, pk_fma(gl2, f32x2{bb.x, bb.y}, nm2));
      const f32x2 r1 = pk_fma(f32x2{s[t][2], s[t][3]}, c12, pk_fma(gl2, f32x2{bb.z, bb.w}, nm2));
      v[t][0] = r0.x; v[t][1] = r0.y; v[t][2] = r1.x; v[t][3] = r1.y;
    }
    if (LAST && kb + 64 > T) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[t][r] = (kb + 16 * t + 4 * g + r < T) ? v[t][r] : -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) mx = fmaxf(mx, fmaxf(fmaxf(v[t][0], v[t][1]), fmaxf(v[t][2], v[t][3])));
    mx = xor32_max(xor16_max(mx));
    if (it == 0 || __builtin_amdgcn_ballot_w64(mx > RESCALE_TAU)) {
      // shift to the tile's maximum: on the first tile unconditionally (mref = 0 was a
      // placeholder; o and the row sum are still zero), later only upwards
      const float sh = it == 0 ? mx : fmaxf(mx, 0.f);
      const float alpha = it == 0 ? 1.f : exp2_(-sh);
      mref += sh;
      const f32x2 sh2 = {sh, sh}, al2 = {alpha, alpha};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f32x2 a0 = f32x2{v[t][0], v[t][1]} - sh2, a1 = f32x2{v[t][2], v[t][3]} - sh2;
        v[t][0] = a0.x; v[t][1] = a0.y; v[t][2] = a1.x; v[t][3] = a1.y;
      }
      lpart2 *= al2;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f32x2 o0 = f32x2{o[dt][0], o[dt][1]} * al2, o1 = f32x2{o[dt][2], o[dt][3]} * al2;
        o[dt] = f32x4{o0.x, o0.y, o1.x, o1.y};
      }
    }
    float pd[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) pd[t][r] = exp2_(v[t][r]);
#pragma unroll
    for (int t = 0; t < 4; ++t) lpart2 += f32x2{pd[t][0], pd[t][1]} + f32x2{pd[t][2], pd[t][3]};
    if constexpr (DM == 2) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pd[t][r] = (mcur >> (4 * t + r)) & 1u ? pd[t][r] : 0.f;
          asm("" : "+v"(pd[t][r]));  // keep the packed bf16 conversions (see DM 1)
        }
    } else if constexpr (DROP) {
      uint32_t mb = 0;  // this lane's 16 keep bits of the tile: bit 4t + r = key kb + 16t + 4g + r
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rp = 0; rp < 2; ++rp) {
          const uint32_t hh = attn_mix((rowpair + (uint32_t)((kb >> 1) + 8 * t + rp)) ^ key);
          const bool k0 = attn_half_keep(hh, 0, thr), k1 = attn_half_keep(hh, 1, thr);
          pd[t][2 * rp] = k0 ? pd[t][2 * rp] : 0.f;
          pd[t][2 * rp + 1] = k1 ? pd[t][2 * rp + 1] : 0.f;
          mb |= (k0 ? 1u << (4 * t + 2 * rp) : 0u) | (k1 ? 2u << (4 * t + 2 * rp) : 0u);
          // opaque to the optimiser: otherwise it pushes the bf16 conversion into each select
          // (16 conversions + 8 v_perm per tile instead of 8 packed conversions)
          asm("" : "+v"(pd[t][2 * rp]), "+v"(pd[t][2 * rp + 1]));
        }
      // the backward reads the bits instead of re-hashing: [bh][key tile][g][Tp] u16
      if (p.drop_mask && qv) p.drop_mask[((bh * ntiles + it) * 4 + g) * Tp + qi] = (uint16_t)mb;
    }
    // O^T = V^T P^T (V in the A slot): lane (g, i16) holds O[its query][16 dt + 4g + r], so the
    // rescale by its own row's alpha needs no cross-lane broadcast
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16x8 pa = pack8(pd[2 * c], pd[2 * c + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rd_tr(Vt, 32 * c, 32 * c + 16, 16 * dt, lane), pa, o[dt], 0, 0, 0);
    }
  };
#if NRSE_ATTN_NOPEEL
  for (int it = 0; it < ntiles; ++it) tile(it, std::true_type{});
#else
  for (int it = 0; it + 1 < ntiles; ++it) tile(it, std::false_type{});
  tile(ntiles - 1, std::true_type{});
#endif
  const float lpart = lpart2.x + lpart2.y;
  const float m = mref;
  const float l = xor32_sum(xor16_sum(lpart));
  bf16_t* ctx = (bf16_t*)p.ctx;
  if (qv) {
    // this lane's query row: 4 consecutive dims per dt (one 8-byte store each)
    const float inv = dsc / l;
    bf16_t* crow = ctx + ((long long)b * T + qi) * Hd + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      uint2 u;
      u.x = (uint32_t)f2bf(o[dt][0] * inv) | ((uint32_t)f2bf(o[dt][1] * inv) << 16);
      u.y = (uint32_t)f2bf(o[dt][2] * inv) | ((uint32_t)f2bf(o[dt][3] * inv) << 16);
      *reinterpret_cast<uint2*>(crow + 16 * dt) = u;
      if (p.ctx8) {  // ABI 6: fp8(bf16 ctx), the out-projection's operand
        float b4[4] = {bf2f(f2bf(o[dt][0] * inv)), bf2f(f2bf(o[dt][1] * inv)), bf2f(f2bf(o[dt][2] * inv)),
                       bf2f(f2bf(o[dt][3] * inv))};
        *reinterpret_cast<uint32_t*>((unsigned char*)p.ctx8 + ((long long)b * T + qi) * Hd + h * D + 4 * g + 16 * dt) =
            fp8x4(b4[0], b4[1], b4[2], b4[3]);
      }
    }
  }
  if (g == 0 && qv) p.lse[bh * T + qi] = (m + __builtin_amdgcn_logf(l)) * LN2;
}

// ------------------------------------------------------------------------------ bwd: dQ, dgate
// DM: dropout mode, 0 none, 1 re-hashed keep bits, 2 the forward's recorded bits (drop_mask);
// one specialisation each (both paths in one kernel cost 20 VGPRs and a wave per SIMD)
#ifndef NRSE_ATTN_BWDQ_WAVES
#define NRSE_ATTN_BWDQ_WAVES 3
#endif
#if NRSE_ATTN_BWDQ_WAVES
#define NRSE_BWDQ_OCC __attribute__((amdgpu_waves_per_eu(NRSE_ATTN_BWDQ_WAVES, NRSE_ATTN_BWDQ_WAVES)))
#else
#define NRSE_BWDQ_OCC
#endif
template <int DM>
__global__ __launch_bounds__(256) NRSE_BWDQ_OCC void attn_bwd_q_kernel(const nrse_attn_bwd_params p) {
  constexpr bool DROP = DM != 0;
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  char* const kv0 = dyn;  // [2 buffers][K tile, V tile], LDS-DMA double buffer as in the forward
  float* const bv = reinterpret_cast<float*>(dyn + 4 * TILE_B);
  const int T = p.T, H = p.H, Hd = H * D;
  const long long ld3 = 3LL * Hd;
  const BlockPos bp = block_pos((p.T + 63) / 64, p.H);
  const int b = bp.b, h = bp.h;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  const int q0 = bp.blk * 64;
  const int qi = q0 + w * 16 + i16;
  const bool qv = qi < T;
  const bool wlive = q0 + w * 16 < T;  // as the forward: a wave of queries past T skips the math
  const bf16_t* qkv = (const bf16_t*)p.qkv + (long long)b * T * ld3;
  const bf16_t* dctx = (const bf16_t*)p.dctx + (long long)b * T * Hd;
  const KvDma kd = kv_dma_init(qkv, T, ld3, (Hd + h * D) * 2, w, lane);
  const KvDma vd = kv_dma_init(qkv, T, ld3, (2 * Hd + h * D) * 2, w, lane);
  const int ntiles = (T + 63) / 64;
  kv_dma_issue(kd, kv0, 0, w);
  kv_dma_issue(vd, kv0 + TILE_B, 0, w);
  bv_stage(bv, p.bias_vec + (long long)h * (2 * T - 1), T, q0, tid);
  bf16x8 qf[2], dof[2];
  const bf16_t* octx = (const bf16_t*)p.ctx + (long long)b * T * Hd;
  float dsum = 0.f;  // delta = rowsum(dO * O) for this lane's 16 of the 64 dims
  const int qc = qv ? qi : T - 1;  // loads from a clamped row, zeroed after (no branch around them)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    uint4 u = *reinterpret_cast<const uint4*>(qkv + (long long)qc * ld3 + h * D + 8 * g + 32 * s);
    uint4 d = *reinterpret_cast<const uint4*>(dctx + (long long)qc * Hd + h * D + 8 * g + 32 * s);
    uint4 o = *reinterpret_cast<const uint4*>(octx + (long long)qc * Hd + h * D + 8 * g + 32 * s);
    if (!qv) u = d = o = make_uint4(0, 0, 0, 0);
    qf[s] = __builtin_bit_cast(bf16x8, u);
    dof[s] = __builtin_bit_cast(bf16x8, d);
    const unsigned dw[4] = {d.x, d.y, d.z, d.w}, ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      dsum += __uint_as_float(dw[e] << 16) * __uint_as_float(ow[e] << 16) +
              __uint_as_float(dw[e] & 0xffff0000u) * __uint_as_float(ow[e] & 0xffff0000u);
  }
  dsum = xor32_sum(xor16_sum(dsum));
  const long long bh = (long long)b * H + h;
  const float gi0 = p.gate[bh * T + qc], lse0 = p.lse[bh * T + qc];
  const float gi = qv ? gi0 : 0.f;
  const float c1 = p.scale * LOG2E, gl = gi * LOG2E;
  const float lse = qv ? lse0 : 0.f;
  const float lse2 = lse * LOG2E;
  const float delta = dsum;
  if (g == 0 && qv) p.delta[bh * T + qi] = delta;  // consumed by attn_bwd_kv_kernel (launched after)
  const int bvl = bv_len(T);
  const int u00 = 4 * g + 63 - (w * 16 + i16);
  const int bsel = u00 & 3;
  const float* bvl_base = bv + bsel * bvl;  // copy bsel, rotated as bv_pos
  int boff[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) boff[t] = bv_pos(u00 - bsel + 16 * t, bsel);
  const uint32_t key = site_key(p.seed);
  const uint32_t thr = dropout_threshold16(p.dropout_p);
  constexpr bool drop = DROP;
  const float dsc = drop ? 1.f / (1.f - p.dropout_p) : 1.f;
  const uint32_t rowpair = (uint32_t)(bh * T + qi) * (uint32_t)((T + 1) >> 1) + (uint32_t)(2 * g);  // as fwd
  // the forward's keep bits (if recorded): word (bh, key tile, g, qi), bit 4t + r for key 16t + 4g + r;
  // tile it+1's word is loaded while tile it computes (the top-of-tile vmcnt(0) covers it)
  const int Tp = ntiles * 64;
  constexpr bool use_mask = DM == 2;
  const uint16_t* mrow = use_mask ? p.drop_mask + (bh * ntiles * 4 + g) * (long long)Tp + (qv ? qi : 0) : nullptr;
  uint32_t mnext = use_mask ? (uint32_t)mrow[0] : 0u;
  float dgate = 0.f;
  f32x4 dq[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // LAST: the key tile that may reach past T (its sub-tile skips and masking compiled only into it,
  // as the forward's)
  auto tile = [&](const int it, auto last_c) {
    constexpr bool LAST = decltype(last_c)::value;
    const int kb = it * 64;
    char* const Kt = kv0 + (it & 1) * 2 * TILE_B;
    char* const Vt = Kt + TILE_B;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // the bias rows before the prefetch is issued (as the forward's)
    float bb[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 v4 = *reinterpret_cast<const float4*>(bvl_base + kb + boff[t]);
      bb[t][0] = v4.x; bb[t][1] = v4.y; bb[t][2] = v4.z; bb[t][3] = v4.w;
    }
    const uint32_t mcur = mnext;
    if (!LAST || it + 1 < ntiles) {
      char* const Kn = kv0 + ((it + 1) & 1) * 2 * TILE_B;
      kv_dma_issue(kd, Kn, kb + 64, w);
      kv_dma_issue(vd, Kn + TILE_B, kb + 64, w);
      if (use_mask) mnext = mrow[(long long)(it + 1) * 4 * Tp];
    }
    if (!wlive) return;
    const int nt16 = LAST ? min(4, (T - kb + 15) >> 4) : 4;
    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rd_row(Kt, 16 * t + i16, 4 * ss + g), qf[ss], s[t], 0, 0, 0);
        dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rd_row(Vt, 16 * t + i16, 4 * ss + g), dof[ss], dp[t], 0, 0, 0);
      }
    }
    // Straight-line per element; wave-uniform branches for dropout and for the last (partial)
    // key tile. Rows of invalid queries need no mask: their Q, dO, gate, lse and delta are zero,
    // so d = 1 * (0 - 0) = 0.
    float ds[4][4];
    if constexpr (DROP) {
      if constexpr (use_mask) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) dp[t][r] = (mcur >> (4 * t + r)) & 1u ? dp[t][r] * dsc : 0.f;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (t < nt16) {
#pragma unroll
            for (int rp = 0; rp < 2; ++rp) {
              const uint32_t hh = attn_mix((rowpair + (uint32_t)((kb >> 1) + 8 * t + rp)) ^ key);
              dp[t][2 * rp] = attn_half_keep(hh, 0, thr) ? dp[t][2 * rp] * dsc : 0.f;
              dp[t][2 * rp + 1] = attn_half_keep(hh, 1, thr) ? dp[t][2 * rp + 1] * dsc : 0.f;
            }
          }
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < nt16) {
#pragma unroll
        for (int r = 0; r < 4; ++r) ds[t][r] = exp2_(fmaf(s[t][r], c1, gl * bb[t][r]) - lse2) * (dp[t][r] - delta);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) ds[t][r] = 0.f;
      }
    }
    if (LAST && kb + 64 > T) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) ds[t][r] = (kb + 16 * t + 4 * g + r < T) ? ds[t][r] : 0.f;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) dgate += ds[t][r] * bb[t][r];
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16x8 da = pack8(ds[2 * c], ds[2 * c + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        dq[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rd_tr(Kt, 32 * c, 32 * c + 16, 16 * dt, lane), da, dq[dt], 0, 0, 0);
    }
  };
#if NRSE_ATTN_NOPEEL
  for (int it = 0; it < ntiles; ++it) tile(it, std::true_type{});
#else
  for (int it = 0; it + 1 < ntiles; ++it) tile(it, std::false_type{});
  tile(ntiles - 1, std::true_type{});
#endif
  dgate = xor32_sum(xor16_sum(dgate));
  if (g == 0 && qv) p.dgate[bh * T + qi] = dgate;
  // dQ^T accumulated (K^T in the A slot): lane (g, i16) holds query qi, dims 16 dt + 4g .. + 3
  if (qv) {
    bf16_t* qrow = (bf16_t*)p.dqkv + ((long long)b * T + qi) * ld3 + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      uint2 u;
      u.x = (uint32_t)f2bf(dq[dt][0] * p.scale) | ((uint32_t)f2bf(dq[dt][1] * p.scale) << 16);
      u.y = (uint32_t)f2bf(dq[dt][2] * p.scale) | ((uint32_t)f2bf(dq[dt][3] * p.scale) << 16);
      *reinterpret_cast<uint2*>(qrow + 16 * dt) = u;
    }
  }
}

// ------------------------------------------------------------------------------ bwd: dK, dV, diag
// 3 waves per SIMD (<= 168 VGPRs; LDS ~50 KB at T = 399 -> 3 workgroups per CU): the element
// loops are long dependency chains, latency-bound at 2 waves per SIMD
// DM: dropout mode as attn_bwd_q_kernel's
template <int DM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void attn_bwd_kv_kernel(
    const nrse_attn_bwd_params p) {
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  char* const qo0 = dyn;  // [2 buffers][Q tile, dO tile], LDS-DMA double buffer
  const int T = p.T, H = p.H, Hd = H * D;
  const int Tp = (T + 63) & ~63;
  float* const rowall = reinterpret_cast<float*>(dyn + 4 * TILE_B);  // lse*log2e [Tp], delta [Tp], gate [Tp]
  float* const rbv = rowall + 3 * Tp;                                 // 4 reversed bias copies
  const int bvl = bv_len(T);
  float* const diag = rbv + 4 * bvl;                                  // [diag_len(T)]
  float* const dtmp = diag + diag_len(T);                             // [4 waves][4 lane rows][64]
  // [2 buffers][4 g][64 queries] u16: the forward's keep bits of this key block for the query
  // tile, staged by LDS-DMA beside Q / dO (wave 0, lanes 0-31: 512 B)
  char* const mtile0 = reinterpret_cast<char*>(dtmp + 1024);
  const long long ld3 = 3LL * Hd;
  const BlockPos bp = block_pos((p.T + 63) / 64, p.H);
  const int b = bp.b, h = bp.h;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  const int kb0 = bp.blk * 64;
  const int kj = kb0 + w * 16 + i16;
  const bool kv = kj < T;
  // a wave whose 16 keys all lie past T (the last key block's tail) keeps its staging, barriers
  // and (zero) diagonal slots but skips the tile math
  const bool wlive = kb0 + w * 16 < T;
  const float kvf = kv ? 1.f : 0.f;
  const bf16_t* qkv = (const bf16_t*)p.qkv + (long long)b * T * ld3;
  const bf16_t* dctx = (const bf16_t*)p.dctx + (long long)b * T * Hd;
  const KvDma qd = kv_dma_init(qkv, T, ld3, h * D * 2, w, lane);
  const KvDma od = kv_dma_init(dctx, T, Hd, h * D * 2, w, lane);
  const int ntiles = (T + 63) / 64;
  const long long bh = (long long)b * H + h;
  constexpr bool use_mask = DM == 2;
  // mask DMA: lane l < 32 of wave 0 moves 16 B = 8 queries of row g_f = l >> 3
  __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(use_mask ? p.drop_mask + (bh * ntiles + bp.blk) * 4 * (long long)(ntiles * 64) : nullptr), 0,
      use_mask ? ntiles * 64 * 4 * 2 : 0, 0x00020000);
  const unsigned mvoff = (unsigned)(((lane >> 3) * ntiles * 64 + (lane & 7) * 8) * 2);
  auto mask_issue = [&](char* dst, int q0) {
    if (use_mask && w == 0 && lane < 32)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(mrs, (lds_void_t*)dst, 16, mvoff + (unsigned)q0 * 2, 0, 0, 0);
  };
  kv_dma_issue(qd, qo0, 0, w);
  kv_dma_issue(od, qo0 + TILE_B, 0, w);
  mask_issue(mtile0, 0);
  // (loads unconditional from clamped rows, two strides in flight, zeroed past T)
  for (int q0r = tid; q0r < Tp; q0r += 512) {
    float l[2], dl[2], gt[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int qq = q0r + 256 * u, qc = qq < T ? qq : T - 1;
      l[u] = p.lse[bh * T + qc];
      dl[u] = p.delta[bh * T + qc];
      gt[u] = p.gate[bh * T + qc];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int qq = q0r + 256 * u;
      if (qq < Tp) {
        const bool ok = qq < T;
        rowall[qq] = ok ? l[u] * LOG2E : 0.f;
        rowall[Tp + qq] = ok ? dl[u] : 0.f;
        rowall[2 * Tp + qq] = ok ? gt[u] : 0.f;
      }
    }
  }
  // bias of (query q, key kj) = vec[kj - q + T - 1]: reversed copies, copy s index j holds
  // log2e * vec[e_hi - j - s], e_hi = kb0 + 63 + T - 1; element (q, kj) sits at segment index
  // u = 63 - kl + q, so a lane's 4 consecutive queries are one aligned float4 of copy (u & 3)
  // (stored at bv_pos(j, s) within the copy, as the forward's copies).
  {
    const float* vec = p.bias_vec + (long long)h * (2 * T - 1);
    const int nd = 2 * T - 1, e_hi = kb0 + 63 + T - 1;
    for (int j0 = tid; j0 < bvl; j0 += 512) {   // as bv_stage: loads first, clamped
      float v[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) v[u][s4] = clamped_ld(vec, e_hi - (j0 + 256 * u) - s4, nd);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int j = j0 + 256 * u;
        if (j < bvl) {
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const int e = e_hi - j - s4;
            rbv[s4 * bvl + bv_pos(j, s4)] = (e >= 0 && e < nd) ? v[u][s4] * LOG2E : 0.f;
          }
        }
      }
    }
  }
  bf16x8 kf[2], vf[2];
  const int kc = kv ? kj : T - 1;  // clamped row, zeroed after
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    uint4 a = *reinterpret_cast<const uint4*>(qkv + (long long)kc * ld3 + Hd + h * D + 8 * g + 32 * s);
    uint4 c = *reinterpret_cast<const uint4*>(qkv + (long long)kc * ld3 + 2 * Hd + h * D + 8 * g + 32 * s);
    if (!kv) a = c = make_uint4(0, 0, 0, 0);
    kf[s] = __builtin_bit_cast(bf16x8, a);
    vf[s] = __builtin_bit_cast(bf16x8, c);
  }
  // rel_attn_embed gradient: sum over (q, k) of gate[q] * dS[q, k] per diagonal k - q. Lane
  // (g, i16) holds keys i16 and queries 16t + 4g + r; rotating register r left by r lanes
  // within each 16-lane row (DPP) puts diagonal (i16 - 4g - 16t) or (i16 - 4g - 16t - 16) in
  // lane i16 of row g, so 5 per-lane register accumulators (dacc[j], diagonal x - 4g - 16j
  // relative to the block) collect a 64x64 tile; 4 of them are final after each query block
  // and are folded into the workgroup's diagonal array without LDS atomics (ds_add_f32 cost the
  // kernel ~100 of its 300 us): every lane stores its 4 sums to its own slots of a per-tile
  // staging area, and after a barrier one thread per relative diagonal (124 of them) adds the
  // <= 16 staged values that fall on it.
  const int ndiag = diag_len(T);
  const int DPAD = diag_pad(T);
  for (int e = tid; e < ndiag; e += 256) diag[e] = 0.f;
  float* const tw = dtmp + (w * 4 + g) * 64;
  // fold the staged tile of relative diagonals r = 16 w + (slot - 48) - 4 g into diag[cb + r]
  auto fold = [&](int cb) {
    __syncthreads();
    if (tid < 124) {
      // branch-free: all 16 reads issued back to back (an out-of-range slot reads slot 0 and
      // adds zero), summed in the fixed (wave, row) order
      const int r = tid - 60;
      float v[16];
#pragma unroll
      for (int wv = 0; wv < 4; ++wv)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int slot = r - 16 * wv + 4 * gg + 48;
          const bool ok = (unsigned)slot < 64u;
          const float x = dtmp[(wv * 4 + gg) * 64 + (ok ? slot : 0)];
          v[wv * 4 + gg] = ok ? x : 0.f;
        }
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) s += v[i];
      diag[cb + r] += s;
    }
  };
  float dacc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  if (!wlive) {  // this wave's staging row stays zero for every fold (slots i16 + 16 j, j < 4)
#pragma unroll
    for (int j = 0; j < 4; ++j) tw[i16 + 16 * j] = 0.f;
  }
  // rotation by r wraps for lanes i16 >= 16 - r
  const float whi[3] = {i16 >= 15 ? 1.f : 0.f, i16 >= 14 ? 1.f : 0.f, i16 >= 13 ? 1.f : 0.f};
  const float wlo[3] = {1.f - whi[0], 1.f - whi[1], 1.f - whi[2]};
  const uint32_t key = site_key(p.seed);
  const float c1 = p.scale * LOG2E;
  const uint32_t thr = dropout_threshold16(p.dropout_p);
  // dropout: this lane's key kj and its neighbour kj ^ 1 share every pair hash (row q, kj / 2);
  // the even lane hashes rows r = 0, 1 of each 4-row group, the odd lane rows 2, 3, and they swap
  // the results (DPP quad_perm [1,0,3,2])
  const int par = kj & 1;
  const uint32_t tp2 = (uint32_t)((T + 1) >> 1);
  const uint32_t colpair = (uint32_t)(kj >> 1);
  constexpr bool drop = DM != 0;
  const float dsc = drop ? 1.f / (1.f - p.dropout_p) : 1.f;
  const int kl = w * 16 + i16;  // key within the 64-key block
  const int u00 = 63 - kl + 4 * g;
  const int bsel = u00 & 3;
  const float* rb_base = rbv + bsel * bvl;  // copy bsel, rotated as bv_pos
  int boff[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) boff[t] = bv_pos(u00 - bsel + 16 * t, bsel);
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // LDS index of diagonal kj - qi: (kj - qi) - (kb0 - T + 1) + DPAD
  const int dbase = kb0 - T + 1 - DPAD;
  for (int it = 0; it < ntiles; ++it) {
    const int qb = it * 64;
    char* const Qt = qo0 + (it & 1) * 2 * TILE_B;
    char* const Ot = Qt + TILE_B;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + 1 < ntiles) {
      char* const Qn = qo0 + ((it + 1) & 1) * 2 * TILE_B;
      kv_dma_issue(qd, Qn, qb + 64, w);
      kv_dma_issue(od, Qn + TILE_B, qb + 64, w);
      mask_issue(mtile0 + ((it + 1) & 1) * 512, qb + 64);
    }
    float pd[4][4], ds[4][4], gv[4][4];
    if (wlive) {
    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rd_row(Qt, 16 * t + i16, 4 * ss + g), kf[ss], s[t], 0, 0, 0);
        dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rd_row(Ot, 16 * t + i16, 4 * ss + g), vf[ss], dp[t], 0, 0, 0);
      }
    }
    // element (query qb + 16t + 4g + r, key kj). Straight-line per element; the dropout hash
    // behind one wave-uniform branch, its 1/(1-p) on P folded into the final dV scale. Rows of
    // invalid queries contribute zero by construction (zero Q, dO, lse, delta, gate rows);
    // lanes of invalid keys produce dK/dV rows that are never stored, and kvf keeps them out of
    // the diagonal sums.
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ql = qb + 16 * t + 4 * g;
      const float4 l4 = *reinterpret_cast<const float4*>(rowall + ql);
      const float4 g4 = *reinterpret_cast<const float4*>(rowall + 2 * Tp + ql);
      const float4 b4 = *reinterpret_cast<const float4*>(rb_base + qb + boff[t]);
      ds[t][0] = exp2_(fmaf(s[t][0], c1, g4.x * b4.x) - l4.x);  // P (log2 domain)
      ds[t][1] = exp2_(fmaf(s[t][1], c1, g4.y * b4.y) - l4.y);
      ds[t][2] = exp2_(fmaf(s[t][2], c1, g4.z * b4.z) - l4.z);
      ds[t][3] = exp2_(fmaf(s[t][3], c1, g4.w * b4.w) - l4.w);
    }
    if constexpr (use_mask) {
      // element (t, r) = (query qb + 16t + 4g + r, key 16w + i16 of the block): the forward's word
      // (that query, g_f = i16 >> 2), bit 4w + (i16 & 3)
      const char* mt = mtile0 + (it & 1) * 512 + (i16 >> 2) * 128;
      const int sh = 4 * w + (i16 & 3);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint2 mw = *reinterpret_cast<const uint2*>(mt + (16 * t + 4 * g) * 2);
        const uint32_t bits[4] = {mw.x >> sh, mw.x >> (16 + sh), mw.y >> sh, mw.y >> (16 + sh)};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool keep = bits[r] & 1u;
          pd[t][r] = keep ? ds[t][r] : 0.f;
          dp[t][r] = keep ? dp[t][r] * dsc : 0.f;
        }
      }
    } else if constexpr (drop) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t qa = (uint32_t)(bh * T + qb + 16 * t + 4 * g + 2 * par);
        const uint32_t ha = attn_mix((qa * tp2 + colpair) ^ key);
        const uint32_t hb = attn_mix(((qa + 1) * tp2 + colpair) ^ key);
        const uint32_t xa = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ha, 0xB1, 0xF, 0xF, false);
        const uint32_t xb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hb, 0xB1, 0xF, 0xF, false);
        const uint32_t hr[4] = {par ? xa : ha, par ? xb : hb, par ? ha : xa, par ? hb : xb};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool keep = attn_half_keep(hr[r], par, thr);
          pd[t][r] = keep ? ds[t][r] : 0.f;
          dp[t][r] = keep ? dp[t][r] * dsc : 0.f;
        }
      }
    } else
    {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) pd[t][r] = ds[t][r];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ql = qb + 16 * t + 4 * g;
      const float4 d4 = *reinterpret_cast<const float4*>(rowall + Tp + ql);
      const float4 g4 = *reinterpret_cast<const float4*>(rowall + 2 * Tp + ql);
      ds[t][0] *= dp[t][0] - d4.x; gv[t][0] = ds[t][0] * (g4.x * kvf);
      ds[t][1] *= dp[t][1] - d4.y; gv[t][1] = ds[t][1] * (g4.y * kvf);
      ds[t][2] *= dp[t][2] - d4.z; gv[t][2] = ds[t][2] * (g4.z * kvf);
      ds[t][3] *= dp[t][3] - d4.w; gv[t][3] = ds[t][3] * (g4.w * kvf);
    }
    if (p.diag) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        dacc[t] += gv[t][0];
        diag_rot<1>(gv[t][1], wlo[0], whi[0], dacc[t], dacc[t + 1]);
        diag_rot<2>(gv[t][2], wlo[1], whi[1], dacc[t], dacc[t + 1]);
        diag_rot<3>(gv[t][3], wlo[2], whi[2], dacc[t], dacc[t + 1]);
      }
      // diagonals i16 - 4g - 16j + 16w (j < 4) relative to kb0 - qb are complete: stage, fold
#pragma unroll
      for (int j = 0; j < 4; ++j) tw[i16 - 16 * j + 48] = dacc[j];
      dacc[0] = dacc[4];
      dacc[1] = dacc[2] = dacc[3] = dacc[4] = 0.f;
    }
    }  // wlive
    if (p.diag) fold(kb0 - qb - dbase);  // every wave: the fold's barriers
    if (!wlive) continue;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16x8 pa = pack8(pd[2 * c], pd[2 * c + 1]);
      const bf16x8 da = pack8(ds[2 * c], ds[2 * c + 1]);
      // dV^T = dO^T P, dK^T = Q^T dS (the tiles in the A slot): lane (g, i16) accumulates its own
      // key's dims 16 dt + 4g + r, stored as 8-byte runs below
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rd_tr(Ot, 32 * c, 32 * c + 16, 16 * dt, lane), pa, dv[dt], 0, 0, 0);
        dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rd_tr(Qt, 32 * c, 32 * c + 16, 16 * dt, lane), da, dk[dt], 0, 0, 0);
      }
    }
  }
  bf16_t* dqkv = (bf16_t*)p.dqkv + (long long)b * T * ld3;
  if (kv) {
    bf16_t* krow = dqkv + (long long)kj * ld3 + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      uint2 uk, uv;
      uk.x = (uint32_t)f2bf(dk[dt][0] * p.scale) | ((uint32_t)f2bf(dk[dt][1] * p.scale) << 16);
      uk.y = (uint32_t)f2bf(dk[dt][2] * p.scale) | ((uint32_t)f2bf(dk[dt][3] * p.scale) << 16);
      uv.x = (uint32_t)f2bf(dv[dt][0] * dsc) | ((uint32_t)f2bf(dv[dt][1] * dsc) << 16);
      uv.y = (uint32_t)f2bf(dv[dt][2] * dsc) | ((uint32_t)f2bf(dv[dt][3] * dsc) << 16);
      *reinterpret_cast<uint2*>(krow + Hd + 16 * dt) = uk;
      *reinterpret_cast<uint2*>(krow + 2 * Hd + 16 * dt) = uv;
    }
  }
  if (p.diag) {  // the carried accumulator: diagonals i16 - 4g + 16w relative to kb0 - (last qb + 64)
    const int qend = ((T + 63) / 64) * 64;
    __syncthreads();  // the last tile's fold has read the staging area
    tw[i16 + 48] = dacc[0];
    tw[i16 + 32] = tw[i16 + 16] = tw[i16] = 0.f;
    fold(kb0 - qend - dbase);
  }
  __syncthreads();
  if (p.diag) {
    const int nd = 2 * T - 1;
    if (p.diag_part) {
      // this block's whole row of the [H][B * key tiles][2T-1] partial slab (zeros off its band),
      // added in (b, key tile) order by nrse_rows_reduce: deterministic
      float* prow = p.diag_part + (((long long)h * p.batch + b) * ntiles + bp.blk) * nd;
      for (int dd = tid; dd < nd; dd += 256) {
        const int e = dd - (dbase + T - 1);
        prow[dd] = (e >= 0 && e < ndiag) ? diag[e] : 0.f;
      }
    } else {
      for (int e = tid; e < ndiag; e += 256) {
        const int dd = dbase + e + T - 1;  // index of d = kj - qi in [0, 2T-1)
        const float v = diag[e];
        if (dd >= 0 && dd < nd && v != 0.f) atomicAdd(p.diag + (long long)h * nd + dd, v);
      }
    }
  }
}

}  // namespace

int nrse_attn_use_mfma(int dtype, int head_dim) { return dtype == NRSE_BF16 && head_dim == D; }

int nrse_attn_fwd_mfma(const nrse_attn_fwd_params* p, hipStream_t st) {
  if (!p->bias_vec) {
    nrse_set_error("nrse_attn_fwd: the bf16 MFMA path needs bias_vec (nrse_rel_bias_vec)");
    return NRSE_ERR_ARG;
  }
  const dim3 grid((unsigned)((p->T + 63) / 64 * p->H * p->batch));
  const size_t lds = 4 * TILE_B + 4 * (size_t)bv_len(p->T) * sizeof(float);
  if (lds > 160 * 1024) {
    nrse_set_error("nrse_attn_fwd: T=%d too long for the LDS bias copies", p->T);
    return NRSE_ERR_UNSUPPORTED;
  }
  if (p->dropout_p > 0.f && p->drop_mask && p->drop_mask_in)
    hipLaunchKernelGGL(attn_fwd_kernel<2>, grid, dim3(256), lds, st, *p);
  else if (p->dropout_p > 0.f) hipLaunchKernelGGL(attn_fwd_kernel<1>, grid, dim3(256), lds, st, *p);
  else hipLaunchKernelGGL(attn_fwd_kernel<0>, grid, dim3(256), lds, st, *p);
  return nrse_check_launch("nrse_attn_fwd(mfma)");
}

int nrse_attn_bwd_mfma(const nrse_attn_bwd_params* p, hipStream_t st) {
  if (!p->bias_vec) {
    nrse_set_error("nrse_attn_bwd: the bf16 MFMA path needs bias_vec (nrse_rel_bias_vec)");
    return NRSE_ERR_ARG;
  }
  const dim3 grid((unsigned)((p->T + 63) / 64 * p->H * p->batch));
  const size_t bvl = (size_t)bv_len(p->T);
  const size_t lds_q = 4 * TILE_B + 4 * bvl * sizeof(float);
  const size_t lds_kv =
      4 * TILE_B + (3 * (size_t)((p->T + 63) & ~63) + 4 * bvl + (size_t)(((p->T + 63) & ~63) + 80) + 1024) * sizeof(float) +
      2 * 512;  // the double-buffered keep-bit tile
  if (lds_kv > 160 * 1024) {
    nrse_set_error("nrse_attn_bwd: T=%d too long for the LDS bias copies / diagonal accumulator", p->T);
    return NRSE_ERR_UNSUPPORTED;
  }
  // the dQ kernel also produces delta = rowsum(dO * O), which the dK/dV kernel reads
  if (p->dropout_p > 0.f && p->drop_mask) hipLaunchKernelGGL(attn_bwd_q_kernel<2>, grid, dim3(256), lds_q, st, *p);
  else if (p->dropout_p > 0.f) hipLaunchKernelGGL(attn_bwd_q_kernel<1>, grid, dim3(256), lds_q, st, *p);
  else hipLaunchKernelGGL(attn_bwd_q_kernel<0>, grid, dim3(256), lds_q, st, *p);
  if (p->dropout_p > 0.f && p->drop_mask) hipLaunchKernelGGL(attn_bwd_kv_kernel<2>, grid, dim3(256), lds_kv, st, *p);
  else if (p->dropout_p > 0.f) hipLaunchKernelGGL(attn_bwd_kv_kernel<1>, grid, dim3(256), lds_kv, st, *p);
  else hipLaunchKernelGGL(attn_bwd_kv_kernel<0>, grid, dim3(256), lds_kv, st, *p);
  const int rc = nrse_check_launch("nrse_attn_bwd(mfma)");
  if (rc || !p->diag || !p->diag_part) return rc;
  const int ntiles = (p->T + 63) / 64;
  return nrse_rows_reduce(p->diag, 2LL * p->T - 1, nullptr, 0, nullptr, 0, p->diag_part, p->batch * ntiles, p->H, 1,
                          st);
}


namespace {
// One thread per mask word (bh, key tile kt, g, q): the forward's 8 pair hashes of that word
// (attn_fwd_kernel DM 1), bit 4t + 2rp + e = keep(q, key 64 kt + 16 t + 4 g + 2 rp + e).
__global__ __launch_bounds__(256) void attn_mask_kernel(uint16_t* __restrict__ mask, int T, int ntiles, int rows,
                                                        uint32_t seed, uint32_t thr) {
  // one wave per mask row ((bh, key tile, g): Tp words, lane-strided), waves grid-strided over the
  // rows: the launch is sized to sit beside the GEMMs it overlaps (a few waves per CU), not to fill
  // the chip
  const uint32_t key = site_key(seed);
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  const int Tp = ntiles * 64;
  const uint32_t tp2 = (uint32_t)((T + 1) >> 1);
  for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    const int g = r & 3;
    const int kt = (r >> 2) % ntiles;
    const int bh = (r >> 2) / ntiles;
    const int kb = kt * 64;
    uint16_t* out = mask + (long long)r * Tp;
    for (int q = lane; q < Tp; q += 64) {
      uint32_t mb = 0;
      if (q < T) {
        const uint32_t rowpair = (uint32_t)(bh * T + q) * tp2 + (uint32_t)(2 * g);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int rp = 0; rp < 2; ++rp) {
            const uint32_t hh = attn_mix((rowpair + (uint32_t)((kb >> 1) + 8 * t + rp)) ^ key);
            mb |= (attn_half_keep(hh, 0, thr) ? 1u : 0u) << (4 * t + 2 * rp);
            mb |= (attn_half_keep(hh, 1, thr) ? 1u : 0u) << (4 * t + 2 * rp + 1);
          }
      }
      out[q] = (uint16_t)mb;
    }
  }
}
}  // namespace

extern "C" int nrse_attn_dropout_mask(uint16_t* drop_mask, int batch, int T, int H, float dropout_p, uint32_t seed,
                                      void* stream) {
  NRSE_REQUIRE(drop_mask && batch > 0 && T > 0 && H > 0 && dropout_p > 0.f && dropout_p < 1.f,
               "nrse_attn_dropout_mask: bad args");
  NRSE_REQUIRE((long long)batch * H * T < (1LL << 31), "nrse_attn_dropout_mask: too many rows");
  const int ntiles = (T + 63) / 64;
  const int rows = batch * H * ntiles * 4;
  // workgroups (4 waves each): NRSE_MASK_WGS, default 256 (one wave per SIMD) -- the kernel runs
  // on a side stream under the layer's LN1 / QKV GEMM and must leave their waves room
  static const int wgs_env = [] {
    const char* e = getenv("NRSE_MASK_WGS");
    return e ? atoi(e) : 0;
  }();
  const int wgs = std::max(1, std::min(wgs_env > 0 ? wgs_env : 256, (rows + 3) / 4));
  hipLaunchKernelGGL(attn_mask_kernel, dim3((unsigned)wgs), dim3(256), 0, (hipStream_t)stream, drop_mask, T, ntiles,
                     rows, seed, dropout_threshold16(dropout_p));
  return nrse_check_launch("nrse_attn_dropout_mask");
}

extern "C" long long nrse_attn_mask_elems(int batch, int T, int H) {
  if (batch <= 0 || T <= 0 || H <= 0) return 0;
  const long long nt = (T + 63) / 64;
  return (long long)batch * H * nt * 4 * nt * 64;
}
