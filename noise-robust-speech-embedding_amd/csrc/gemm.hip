// Generic MFMA GEMM for gfx950 (CDNA4): every Linear / Conv1d contraction of the BYOL-on-WavLM
// step (see include/nrse_hip.h, nrse_gemm, for the reference call sites it replaces).
//
// Design (MI355X-first, not a CUDA tiling):
//  - 128x128 output tile per 256-thread workgroup (4 waves as 2x2, 64x64 per wave = 4x4 MFMA
//    tiles of 16x16). bf16 path: v_mfma_f32_16x16x32_bf16, BK = 64; f32 parity path:
//    v_mfma_f32_16x16x4_f32 (exact f32, same tile geometry), BK = 32. Both stage 16 KB per
//    operand per K step, double-buffered in LDS (64 KB per workgroup -> 2 workgroups per CU).
//  - Operands may be K-contiguous ("row-major MxK") or M/N-contiguous. K-contiguous tiles are
//    stored [row][k] with an XOR swizzle and read with ds_read_b128; M/N-contiguous tiles are
//    stored [k][row] and read transposed with ds_read_b64_tr_b16 (gfx950 hardware transpose),
//    so dgrad/wgrad never materialise a transposed copy of an activation.
//  - Implicit-GEMM addressing: the contiguous index may be "chunked" (pos-conv groups) and K
//    may be split into segments (per-utterance token ranges), so strided Conv1d and the
//    grouped positional conv run through this kernel without im2col buffers.
//  - Fused epilogues: bias, erf-GELU (+pre-activation store), GELU backward, dropout (counter
//    hash), residual add, accumulate/atomic, column sums (bias gradients).
#include <cstdlib>
#include "common.h"

bool nrse_gemm_dma_ok(const nrse_gemm_params* p);        // gemm_dma.hip
int nrse_gemm_dma(const nrse_gemm_params* p, hipStream_t st);
bool nrse_posconv_ok(const nrse_gemm_params* p);         // posconv.hip
int nrse_posconv(const nrse_gemm_params* p, hipStream_t st);
bool nrse_posconv_wgrad_ok(const nrse_gemm_params* p);
int nrse_posconv_wgrad(const nrse_gemm_params* p, hipStream_t st);
bool nrse_gemm256_ok(const nrse_gemm_params* p);         // gemm256.hip
bool nrse_gemm256_f8_ok(const nrse_gemm_params* p);
long long nrse_gemm256_tiles(const nrse_gemm_params* p);
int nrse_gemm256(const nrse_gemm_params* p, hipStream_t st);
int nrse_gemm256_rows(const nrse_gemm_params* p);           // its tile rows for p (256 or 224)

namespace {

int g_gemm_gen = getenv("NRSE_GEMM_GEN") ? atoi(getenv("NRSE_GEMM_GEN")) : 0;

constexpr int BM = 128;
constexpr int BN = 128;
constexpr int NTHR = 256;
constexpr int TILE_BYTES = 16384;             // one operand tile per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;   // A + B

template <typename T> struct Cfg;
template <> struct Cfg<bf16_t> { static constexpr int BK = 64; static constexpr int EPC = 8; };
template <> struct Cfg<float> { static constexpr int BK = 32; static constexpr int EPC = 4; };

struct OpState {
  const char* base;  // batch-offset base pointer (bytes)
  long long ld, ldc, seg;
  int cs;
  long long cmask;
};

NRSE_DEV long long chunk_off(long long c, int cs, long long cmask, long long ldc) {
  return (c >> cs) * ldc + (c & cmask);
}

// Per-thread staging of one operand tile (4 x 16-byte chunks per thread).
template <typename T, bool KC>
struct Stage {
  static constexpr int EPC = Cfg<T>::EPC;
  static constexpr int BK = Cfg<T>::BK;
  uint4 r[4];
  // KC: fixed k-chunk, 4 rows; !KC: fixed column chunk, 4 k-rows
  long long rowoff[4];  // KC only: outer offsets of the 4 rows
  bool rowok[4];
  int kc;               // KC: chunk index within BK (0..7); !KC: column chunk index
  long long coloff;     // !KC: contiguous offset of the column chunk
  bool colok;
  int krow[4];          // !KC: k row index within tile

  NRSE_DEV void init(const OpState& s, int tid, int row0, int rows_total) {
    if constexpr (KC) {
      kc = tid & 7;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = (tid >> 3) + 32 * i;
        const int row = row0 + rr;
        rowok[i] = row < rows_total;
        rowoff[i] = (long long)row * s.ld;
      }
    } else {
      constexpr int CPR = BM / EPC;  // chunks per LDS row
      constexpr int RSTEP = NTHR / CPR;
      kc = tid % CPR;
      const long long col = row0 + (long long)kc * EPC;
      colok = col < rows_total;
      coloff = chunk_off(col, s.cs, s.cmask, s.ldc);
#pragma unroll
      for (int i = 0; i < 4; ++i) krow[i] = tid / CPR + RSTEP * i;
    }
  }

  NRSE_DEV void load(const OpState& s, long long segoff, int k0, int kseg) {
    if constexpr (KC) {
      const int k = k0 + kc * EPC;
      const bool kok = k < kseg;
      const long long co = chunk_off(k, s.cs, s.cmask, s.ldc);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (kok && rowok[i]) {
          r[i] = *reinterpret_cast<const uint4*>(s.base + (segoff + rowoff[i] + co) * (long long)sizeof(T));
        } else {
          r[i] = make_uint4(0, 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + krow[i];
        if (colok && k < kseg) {
          r[i] = *reinterpret_cast<const uint4*>(s.base + (segoff + (long long)k * s.ld + coloff) * (long long)sizeof(T));
        } else {
          r[i] = make_uint4(0, 0, 0, 0);
        }
      }
    }
  }

  // LDS image byte offset of a 16-byte chunk.
  static NRSE_DEV int lds_off_kc(int row, int chunk) {
    if constexpr (sizeof(T) == 2) return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
    else return row * 128 + ((chunk ^ (row & 7)) << 4);
  }
  static NRSE_DEV int fb(int row) { return ((row & 3) | (((row >> 3) & 1) << 2)) << 1; }
  static NRSE_DEV int lds_off_nk(int row, int chunk) {
    if constexpr (sizeof(T) == 2) return row * 256 + ((chunk ^ fb(row)) << 4);
    else return row * 512 + ((chunk ^ ((row & 1) << 2)) << 4);
  }

  NRSE_DEV void store(char* lds, int tid) const {
    if constexpr (KC) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = (tid >> 3) + 32 * i;
        *reinterpret_cast<uint4*>(lds + lds_off_kc(rr, kc)) = r[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4*>(lds + lds_off_nk(krow[i], kc)) = r[i];
    }
  }
};

// Fragment readers. `base` = first row/column of the 16-wide MFMA tile inside the 128 tile.
template <bool KC>
NRSE_DEV bf16x8 frag_bf16(const char* lds, int base, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  if constexpr (KC) {
    const int row = base + i;
    const int chunk = s * 4 + g;
    const int off = row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
    return *reinterpret_cast<const bf16x8*>(lds + off);
  } else {
    const int q = i >> 2, p = i & 3;
    const int col = base + 4 * p;
    short4v lo, hi;
    {
      const int row = s * 32 + 8 * g + q;
      const int off = row * 256 + (((col >> 3) ^ Stage<bf16_t, false>::fb(row)) << 4) + ((col >> 2) & 1) * 8;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)(lds + off));
    }
    {
      const int row = s * 32 + 8 * g + 4 + q;
      const int off = row * 256 + (((col >> 3) ^ Stage<bf16_t, false>::fb(row)) << 4) + ((col >> 2) & 1) * 8;
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)(lds + off));
    }
    typedef short short8v __attribute__((ext_vector_type(8)));
    short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <bool KC>
NRSE_DEV float frag_f32(const char* lds, int base, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  if constexpr (KC) {
    const int row = base + i;
    const int off = row * 128 + ((s ^ (row & 7)) << 4) + g * 4;  // k = 4s + g
    return *reinterpret_cast<const float*>(lds + off);
  } else {
    const int row = 4 * s + g;
    const int col = base + i;
    const int off = row * 512 + (((col >> 2) ^ ((row & 1) << 2)) << 4) + (col & 3) * 4;
    return *reinterpret_cast<const float*>(lds + off);
  }
}

template <typename T, bool AKC, bool BKC>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(const nrse_gemm_params p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  constexpr int BK = Cfg<T>::BK;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int n0 = blockIdx.x * BN;
  const int m0 = blockIdx.y * BM;
  const int z = blockIdx.z;
  const int zb = z / p.splits;
  const int split = z % p.splits;
  const long long zq = zb / p.zdiv, zr = zb % p.zdiv;

  OpState sa, sb;
  sa.base = (const char*)p.a.ptr + (zq * p.a.z1 + zr * p.a.z2) * (long long)sizeof(T);
  sa.ld = p.a.ld; sa.ldc = p.a.ld_chunk; sa.seg = p.a.seg_stride;
  sa.cs = p.a.chunk_shift > 0 ? p.a.chunk_shift : 62;
  sa.cmask = p.a.chunk_shift > 0 ? ((1LL << p.a.chunk_shift) - 1) : -1LL;
  sb.base = (const char*)p.b.ptr + (zq * p.b.z1 + zr * p.b.z2) * (long long)sizeof(T);
  sb.ld = p.b.ld; sb.ldc = p.b.ld_chunk; sb.seg = p.b.seg_stride;
  sb.cs = p.b.chunk_shift > 0 ? p.b.chunk_shift : 62;
  sb.cmask = p.b.chunk_shift > 0 ? ((1LL << p.b.chunk_shift) - 1) : -1LL;

  Stage<T, AKC> ga;
  Stage<T, BKC> gb;
  ga.init(sa, tid, m0, p.M);
  gb.init(sb, tid, n0, p.N);

  const int tps = (p.K + BK - 1) / BK;  // tiles per segment
  const int seg0 = split * p.nseg;
  const int ntiles = p.nseg * tps;

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load_tile = [&](int t) {
    const int sg = seg0 + t / tps;
    const int k0 = (t % tps) * BK;
    ga.load(sa, (long long)sg * sa.seg, k0, p.K);
    gb.load(sb, (long long)sg * sb.seg, k0, p.K);
  };

  if (ntiles > 0) {
    load_tile(0);
    ga.store(smem, tid);
    gb.store(smem + TILE_BYTES, tid);
    __syncthreads();
  }
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const bool more = (t + 1) < ntiles;
    if (more) load_tile(t + 1);
    const char* la = smem + cur * STAGE_BYTES;
    const char* lb = la + TILE_BYTES;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 fa[4], fb[4];
#pragma unroll
        for (int tm = 0; tm < 4; ++tm) fa[tm] = frag_bf16<AKC>(la, wm * 64 + tm * 16, s, lane);
#pragma unroll
        for (int tn = 0; tn < 4; ++tn) fb[tn] = frag_bf16<BKC>(lb, wn * 64 + tn * 16, s, lane);
#pragma unroll
        for (int tm = 0; tm < 4; ++tm)
#pragma unroll
          for (int tn = 0; tn < 4; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[tm], fb[tn], acc[tm][tn], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        float fa[4], fb[4];
#pragma unroll
        for (int tm = 0; tm < 4; ++tm) fa[tm] = frag_f32<AKC>(la, wm * 64 + tm * 16, s, lane);
#pragma unroll
        for (int tn = 0; tn < 4; ++tn) fb[tn] = frag_f32<BKC>(lb, wn * 64 + tn * 16, s, lane);
#pragma unroll
        for (int tm = 0; tm < 4; ++tm)
#pragma unroll
          for (int tn = 0; tn < 4; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[tm], fb[tn], acc[tm][tn], 0, 0, 0);
      }
    }
    if (more) {
      char* nxt = smem + (cur ^ 1) * STAGE_BYTES;
      ga.store(nxt, tid);
      gb.store(nxt + TILE_BYTES, tid);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  const int g = lane >> 4, li = lane & 15;
  const int flags = p.flags;
  const long long cbase = zq * p.c_z1 + zr * p.c_z2 + (long long)split * p.c_split;
  const long long abase = zq * p.aux_z1 + zr * p.aux_z2;
  const long long rbase = zq * p.r_z1 + zr * p.r_z2;
  const uint32_t key = site_key(p.seed);
  const uint32_t thresh = dropout_threshold(p.dropout_p);
  const float dscale = p.dropout_p < 1.f ? 1.f / (1.f - p.dropout_p) : 0.f;
#pragma unroll
  for (int tn = 0; tn < 4; ++tn) {
    const int n = n0 + wn * 64 + tn * 16 + li;
    const bool nok = n < p.N;
    const float bias = ((flags & NRSE_EPI_BIAS) && nok && split == 0) ? p.bias[zq * p.bias_z1 + zr * p.bias_z2 + n] : 0.f;
    float csum = 0.f;
#pragma unroll
    for (int tm = 0; tm < 4; ++tm) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + tm * 16 + 4 * g + r;
        if (!(nok && m < p.M)) continue;
        float v = acc[tm][tn][r] * p.alpha + bias;
        if (flags & NRSE_EPI_GELU) {
          if (p.aux) store_from_f((void*)p.aux, p.aux_dtype, abase + (long long)m * p.ldaux + n, v);
          v = gelu_f(v);
        }
        if (flags & NRSE_EPI_GELU_BWD) v *= gelu_grad_f(load_as_f(p.aux, p.aux_dtype, abase + (long long)m * p.ldaux + n));
        if (flags & NRSE_EPI_RELU) v = fmaxf(v, 0.f);
        if (flags & NRSE_EPI_TANH) v = tanhf(v);
        const long long ci = cbase + (long long)m * p.ldc + n;
        const uint32_t eidx = (uint32_t)ci;
        if ((flags & NRSE_EPI_DROPOUT) && !(flags & NRSE_EPI_DROP_AFTER))
          v = dropout_keep(key, eidx, thresh) ? v * dscale : 0.f;
        if (flags & NRSE_EPI_RESID) v += load_as_f(p.resid, p.resid_dtype, rbase + (long long)m * p.ldr + n);
        if ((flags & NRSE_EPI_DROPOUT) && (flags & NRSE_EPI_DROP_AFTER))
          v = dropout_keep(key, eidx, thresh) ? v * dscale : 0.f;
        csum += v;
        if (flags & NRSE_EPI_ATOMIC) {
          atomicAdd((float*)p.c + ci, v);
        } else {
          if (flags & NRSE_EPI_ACCUM) v += load_as_f(p.c, p.c_dtype, ci);
          store_from_f(p.c, p.c_dtype, ci, v);
        }
      }
    }
    if (flags & NRSE_EPI_COLSUM) {
      csum += __shfl_xor(csum, 16, 64);
      csum += __shfl_xor(csum, 32, 64);
      if (g == 0 && nok) colsum_out(p, z, gridDim.y, blockIdx.y, wm, n, csum);
    }
  }
}

template <typename T, bool AKC, bool BKC>
int launch_t(const nrse_gemm_params* p, hipStream_t st) {
  dim3 grid(nrse_cdiv(p->N, BN), nrse_cdiv(p->M, BM), p->batch * p->splits);
  hipLaunchKernelGGL((gemm_kernel<T, AKC, BKC>), grid, dim3(NTHR), 0, st, *p);
  return nrse_check_launch("nrse_gemm");
}

template <typename T>
int launch_dt(const nrse_gemm_params* p, hipStream_t st) {
  if (p->a.kcontig && p->b.kcontig) return launch_t<T, true, true>(p, st);
  if (p->a.kcontig && !p->b.kcontig) return launch_t<T, true, false>(p, st);
  if (!p->a.kcontig && p->b.kcontig) return launch_t<T, false, true>(p, st);
  return launch_t<T, false, false>(p, st);
}

}  // namespace

extern "C" int nrse_gemm(const nrse_gemm_params* p, void* stream) {
  NRSE_CHECK_PARAMS(p, "nrse_gemm");
  NRSE_REQUIRE(p->a.ptr && p->b.ptr && p->c, "nrse_gemm: null operand");
  NRSE_REQUIRE(p->M > 0 && p->N > 0 && p->K >= 0 && p->nseg >= 1 && p->splits >= 1 && p->batch >= 1 && p->zdiv >= 1,
               "nrse_gemm: bad sizes M=%d N=%d K=%d nseg=%d splits=%d batch=%d zdiv=%d", p->M, p->N, p->K, p->nseg,
               p->splits, p->batch, p->zdiv);
  if (p->a.dtype != p->b.dtype || (p->a.dtype != NRSE_BF16 && p->a.dtype != NRSE_F32)) {
    nrse_set_error("nrse_gemm: A/B dtype mismatch (%d vs %d)", p->a.dtype, p->b.dtype);
    return NRSE_ERR_DTYPE;
  }
  const int epc = p->a.dtype == NRSE_BF16 ? 8 : 4;
  // 16-byte vector loads: every contiguous extent and leading dimension must be a multiple
  // of the elements per 16 bytes, and chunks must hold whole vectors.
  const nrse_gemm_operand* ops[2] = {&p->a, &p->b};
  const int cdim[2] = {p->M, p->N};
  for (int i = 0; i < 2; ++i) {
    const nrse_gemm_operand* o = ops[i];
    const long long contig = o->kcontig ? p->K : cdim[i];
    NRSE_REQUIRE(contig % epc == 0, "nrse_gemm: operand %c contiguous extent %lld not a multiple of %d", 'A' + i,
                 contig, epc);
    NRSE_REQUIRE(o->ld % epc == 0 && o->seg_stride % epc == 0 && o->z1 % epc == 0 && o->z2 % epc == 0,
                 "nrse_gemm: operand %c strides must be multiples of %d", 'A' + i, epc);
    if (o->chunk_shift > 0) {
      NRSE_REQUIRE((1LL << o->chunk_shift) >= epc && o->ld_chunk % epc == 0,
                   "nrse_gemm: operand %c chunk too small", 'A' + i);
    }
    NRSE_REQUIRE(((uintptr_t)o->ptr & 15) == 0, "nrse_gemm: operand %c not 16-byte aligned", 'A' + i);
  }
  if ((p->flags & NRSE_EPI_ATOMIC) && p->c_dtype != NRSE_F32) {
    nrse_set_error("nrse_gemm: ATOMIC epilogue needs f32 C");
    return NRSE_ERR_DTYPE;
  }
  NRSE_REQUIRE(!(p->flags & NRSE_EPI_BIAS) || p->bias, "nrse_gemm: BIAS without bias");
  NRSE_REQUIRE(!(p->flags & NRSE_EPI_GELU_BWD) || p->aux, "nrse_gemm: GELU_BWD without aux");
  NRSE_REQUIRE(!(p->flags & NRSE_EPI_RESID) || p->resid, "nrse_gemm: RESID without resid");
  NRSE_REQUIRE(!(p->flags & NRSE_EPI_COLSUM) || p->colsum, "nrse_gemm: COLSUM without colsum");
  NRSE_REQUIRE((long long)nrse_cdiv(p->M, BM) <= 65535, "nrse_gemm: M too large for grid.y (%d)", p->M);
  hipStream_t st = (hipStream_t)stream;
  // NRSE_GEMM_GEN=1|2|3 pins one kernel generation (benchmarks); by default the 256x256 kernel
  // takes bf16 problems with enough tiles to fill the chip, the 128x128 one the rest.
  const int gen = g_gemm_gen;
  // (split-K atomic problems stay on 128x128: 4x the tiles of a 256x256 decomposition means 4x
  // fewer K splits for the same occupancy, i.e. 4x less atomic traffic per FLOP)
  const bool big = nrse_gemm256_tiles(p) >= 128 && !(p->flags & NRSE_EPI_ATOMIC);
  // the grouped pos-conv pattern (sliding-window A operand, N = 64): its own kernel unless a
  // generation is pinned (NRSE_GEMM_GEN=1|2|3 benchmarks the generic kernels on it)
  const bool f8 = p->nseg8 != 0 || p->c8;  // ABI 6 fields: the 256x256 kernel only (below)
  if (!f8 && (gen == 0 || gen == 4) && nrse_posconv_ok(p)) return nrse_posconv(p, st);
  if (!f8 && (gen == 0 || gen == 4) && nrse_posconv_wgrad_ok(p)) return nrse_posconv_wgrad(p, st);
  const bool part = (p->flags & NRSE_EPI_COLSUM) && p->colsum_part;
  int rc, mt;
  if (f8) {
    // ABI 6 (split-weight mode): fp8 correction segments / fp8 output copy -- the 256x256
    // kernel only; no other kernel implements them, so anything else is refused, never dropped
    NRSE_REQUIRE(p->nseg8 >= 0, "nrse_gemm: nseg8 < 0");
    if (!nrse_gemm256_ok(p) || (p->nseg8 > 0 && !nrse_gemm256_f8_ok(p))) {
      nrse_set_error("nrse_gemm: fp8 correction segments need the 256x256 kernel's layout, K %% 128 == 0, "
                     "splits == 1 and 16-byte aligned NRSE_FP8 k-contiguous a8 / b8 (M=%d N=%d K=%d)",
                     p->M, p->N, p->K);
      return NRSE_ERR_UNSUPPORTED;
    }
    if (p->c8 && (p->c_dtype != NRSE_BF16 || p->batch != 1 || p->splits != 1 || ((uintptr_t)p->c8 & 7) ||
                  (p->ldc8 & 7) || p->ldc8 < p->N)) {
      nrse_set_error("nrse_gemm: c8 needs a bf16 C, batch == splits == 1, 8-byte aligned c8 and ldc8 >= N");
      return NRSE_ERR_UNSUPPORTED;
    }
    if (p->c8 && p->c8_dtype != 0 && p->c8_dtype != NRSE_FP8) {
      nrse_set_error("nrse_gemm: bad c8_dtype %d", p->c8_dtype);
      return NRSE_ERR_UNSUPPORTED;
    }
    rc = nrse_gemm256(p, st);
    mt = nrse_cdiv(p->M, nrse_gemm256_rows(p));
    if (rc || !part) return rc;
    return nrse_rows_reduce(p->colsum, p->N, nullptr, 0, nullptr, 0, p->colsum_part, 2 * mt, 1, 1, stream);
  }
  if (gen != 1 && gen != 2 && nrse_gemm256_ok(p) && (gen == 3 || big)) {
    rc = nrse_gemm256(p, st);
    mt = nrse_cdiv(p->M, nrse_gemm256_rows(p));
  } else if (gen != 1 && nrse_gemm_dma_ok(p)) {
    rc = nrse_gemm_dma(p, st);
    mt = nrse_cdiv(p->M, 128);
  } else {
    rc = p->a.dtype == NRSE_BF16 ? launch_dt<bf16_t>(p, st) : launch_dt<float>(p, st);
    mt = nrse_cdiv(p->M, BM);
  }
  if (rc || !part) return rc;
  // the kernels wrote 2 partial rows per (z, M-tile): add them in order
  const long long rows = 2LL * mt * p->batch * p->splits;
  return nrse_rows_reduce(p->colsum, p->N, nullptr, 0, nullptr, 0, p->colsum_part, (int)rows, 1, 1, stream);
}

// floats of colsum_part any kernel generation may write: 2 rows of N per (z, 128-row M-tile)
extern "C" long long nrse_gemm_colsum_workspace(const nrse_gemm_params* p) {
  NRSE_CHECK_PARAMS(p, "nrse_gemm_colsum_workspace");
  if (!p || p->M <= 0 || p->N <= 0) return 0;
  return 2LL * nrse_cdiv(p->M, 128) * p->batch * p->splits * p->N;
}

extern "C" int nrse_gemm_select(int generation) {
  const int prev = g_gemm_gen;
  g_gemm_gen = generation;
  return prev;
}
