// Pieces shared by the bf16 LDS-DMA GEMM kernels (gemm_dma.hip: 128x128 tile, gemm256.hip:
// 256x256 tile): buffer descriptors, the two swizzled LDS operand images and their fragment
// readers, 8-wide f32/bf16 vector access, and the fused epilogue applied to 8 output columns.
#pragma once
#include "common.h"

namespace nrse_gemm_detail {

constexpr unsigned OOB = 0x80000000u;  // buffer voffset past num_records: the load returns zeros

typedef __attribute__((address_space(3))) void lds_void;

NRSE_DEV __amdgpu_buffer_rsrc_t make_rsrc(const char* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
}

// element offset of contiguous-dim coordinate c in a (possibly chunked) operand
NRSE_DEV long long coff(long long c, int cs, long long cmask, long long ldc) { return (c >> cs) * ldc + (c & cmask); }

// XOR pattern of the [k][row] image (row-contiguous operands): 16-B chunk position of row
// chunk c on k-row k is c ^ fbank(k)
NRSE_DEV int fbank(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

// MFMA 16x16x32 bf16 operand fragment for rows base..base+15, k-substep s (32 deep), read
// from a 128-row x 64-k LDS image.
//  KC  (k-contiguous operand): [row][k] 128-B rows, 16-B chunk ch stored at ch ^ ((row>>1)&7)
//  !KC (row-contiguous operand): [k][row] 256-B rows, chunk c stored at c ^ fbank(k); read with
//       the transposing ds_read_b64_tr_b16
template <bool KC>
NRSE_DEV bf16x8 frag(const char* lds, int base, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  if constexpr (KC) {
    const int row = base + i;
    const int chunk = s * 4 + g;
    return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
  } else {
    const int q = i >> 2, p = i & 3;
    const int col = base + 4 * p;
    short4v lo, hi;
    {
      const int row = s * 32 + 8 * g + q;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) short4v*)(lds + row * 256 + (((col >> 3) ^ fbank(row)) << 4) +
                                                       ((col >> 2) & 1) * 8));
    }
    {
      const int row = s * 32 + 8 * g + 4 + q;
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) short4v*)(lds + row * 256 + (((col >> 3) ^ fbank(row)) << 4) +
                                                       ((col >> 2) & 1) * 8));
    }
    typedef short short8v __attribute__((ext_vector_type(8)));
    short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

NRSE_DEV void ld8(const void* p, int dt, long long i, float* o) {
  if (dt == NRSE_BF16) {
    const uint4 u = *reinterpret_cast<const uint4*>((const bf16_t*)p + i);
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[2 * e] = __uint_as_float(w[e] << 16);
      o[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
    }
  } else {
    const float4 a = *reinterpret_cast<const float4*>((const float*)p + i);
    const float4 b = *reinterpret_cast<const float4*>((const float*)p + i + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
}
NRSE_DEV void st8(void* p, int dt, long long i, const float* v) {
  if (dt == NRSE_BF16) {
    uint4 u;
    u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    u.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    u.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>((bf16_t*)p + i) = u;
  } else {
    *reinterpret_cast<float4*>((float*)p + i) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>((float*)p + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// Per-launch-block constants of the fused epilogue.
struct Epi {
  long long cbase, abase, rbase, bbase;
  uint32_t key, thresh;
  float dscale;
  bool bias_on;  // split-K: the bias joins the sum once (split 0)
  float bias8[8];  // this thread's 8 bias values (its epilogue columns are fixed per thread)
  NRSE_DEV Epi(const nrse_gemm_params& p, long long zq, long long zr, int split) {
    cbase = zq * p.c_z1 + zr * p.c_z2 + (long long)split * p.c_split;
    abase = zq * p.aux_z1 + zr * p.aux_z2;
    rbase = zq * p.r_z1 + zr * p.r_z2;
    bbase = zq * p.bias_z1 + zr * p.bias_z2;
    key = site_key(p.seed);
    thresh = dropout_threshold(p.dropout_p);
    dscale = p.dropout_p < 1.f ? 1.f / (1.f - p.dropout_p) : 0.f;
    bias_on = split == 0;
  }
  // bias of output columns n..n+7 (call once: every epilogue iteration of a thread has the same n)
  NRSE_DEV void load_bias(const nrse_gemm_params& p, int n) {
    if ((p.flags & NRSE_EPI_BIAS) && bias_on && n < p.N) {
      const float4 a = *reinterpret_cast<const float4*>(p.bias + bbase + n);
      const float4 b = *reinterpret_cast<const float4*>(p.bias + bbase + n + 4);
      bias8[0] = a.x; bias8[1] = a.y; bias8[2] = a.z; bias8[3] = a.w;
      bias8[4] = b.x; bias8[5] = b.y; bias8[6] = b.z; bias8[7] = b.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) bias8[i] = 0.f;
    }
  }
};

// Epilogue of output row m, columns n..n+7 (in range), accumulator values staged in LDS at cr:
// alpha, +bias, GELU (pre-activation saved to aux), GELU' (from aux), ReLU, dropout before or
// after +residual, then store / accumulate / atomic-add. With `keep`, the final values are
// written back to cr (column sums).
NRSE_DEV void epi8(const nrse_gemm_params& p, const Epi& e, int m, int n, float* cr, bool keep) {
  const int flags = p.flags;
  float v[8];
  {
    const float4 a = *reinterpret_cast<const float4*>(cr);
    const float4 b = *reinterpret_cast<const float4*>(cr + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] *= p.alpha;
  if (flags & NRSE_EPI_BIAS) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += e.bias8[i];
  }
  if (flags & NRSE_EPI_GELU) {
    if (p.aux) st8((void*)p.aux, p.aux_dtype, e.abase + (long long)m * p.ldaux + n, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = gelu_fast(v[i]);
  }
  if (flags & NRSE_EPI_GELU_BWD) {
    float a[8];
    ld8(p.aux, p.aux_dtype, e.abase + (long long)m * p.ldaux + n, a);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] *= gelu_grad_fast(a[i]);
  }
  if (flags & NRSE_EPI_RELU) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], 0.f);
  }
  if (flags & NRSE_EPI_TANH) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = tanhf(v[i]);
  }
  const long long ci = e.cbase + (long long)m * p.ldc + n;
  if ((flags & NRSE_EPI_DROPOUT) && !(flags & NRSE_EPI_DROP_AFTER)) {
    dropout_apply<8>(e.key, (uint32_t)ci, e.thresh, e.dscale, v);
  }
  if (flags & NRSE_EPI_RESID) {
    float r[8];
    ld8(p.resid, p.resid_dtype, e.rbase + (long long)m * p.ldr + n, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += r[i];
  }
  if ((flags & NRSE_EPI_DROPOUT) && (flags & NRSE_EPI_DROP_AFTER)) {
    dropout_apply<8>(e.key, (uint32_t)ci, e.thresh, e.dscale, v);
  }
  if (keep) {
#pragma unroll
    for (int i = 0; i < 8; ++i) cr[i] = v[i];
  }
  if (flags & NRSE_EPI_ATOMIC) {
#pragma unroll
    for (int i = 0; i < 8; ++i) atomicAdd((float*)p.c + ci + i, v[i]);
  } else {
    if (flags & NRSE_EPI_ACCUM) {
      float c[8];
      ld8(p.c, p.c_dtype, ci, c);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += c[i];
    }
    st8(p.c, p.c_dtype, ci, v);
    if (p.c8 && p.c_dtype == NRSE_BF16) {  // ABI 6: fp8 copy of the stored bf16 values (batch 1)
      uint2 w;
      w.x = fp8x4_of_bf(v);
      w.y = fp8x4_of_bf(v + 4);
      *reinterpret_cast<uint2*>((unsigned char*)p.c8 + (long long)m * p.ldc8 + n) = w;
    }
  }
}

// max element offset an operand can reach (the buffer offsets are 31-bit byte offsets)
inline long long op_span(const nrse_gemm_operand& o, const nrse_gemm_params* p, int cdim, int pad_rows) {
  const long long segs = (long long)p->nseg * p->splits;
  const long long rows = o.kcontig ? cdim : p->K;
  const long long contig = o.kcontig ? p->K : cdim;
  long long cspan = contig;
  if (o.chunk_shift > 0) cspan = ((contig - 1) >> o.chunk_shift) * o.ld_chunk + (1LL << o.chunk_shift);
  return (segs - 1) * (o.seg_stride < 0 ? -o.seg_stride : o.seg_stride) + rows * o.ld + cspan + (long long)pad_rows * o.ld;
}

// layout/alignment conditions shared by both LDS-DMA kernels
inline bool dma_layout_ok(const nrse_gemm_params* p, int pad_rows) {
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  auto m8 = [](long long x) { return (x & 7) == 0; };
  if (p->a.dtype != NRSE_BF16 || p->b.dtype != NRSE_BF16) return false;
  if (!m8(p->N) || !m8(p->ldc) || !m8(p->c_z1) || !m8(p->c_z2) || !m8(p->c_split) || !al16(p->c)) return false;
  const bool bias = p->flags & NRSE_EPI_BIAS;
  if (bias && (!al16(p->bias) || (p->bias_z1 & 3) || (p->bias_z2 & 3))) return false;
  const bool aux = (p->flags & (NRSE_EPI_GELU | NRSE_EPI_GELU_BWD)) && p->aux;
  if (aux && (!al16(p->aux) || !m8(p->ldaux) || !m8(p->aux_z1) || !m8(p->aux_z2))) return false;
  if ((p->flags & NRSE_EPI_RESID) && (!al16(p->resid) || !m8(p->ldr) || !m8(p->r_z1) || !m8(p->r_z2))) return false;
  if (op_span(p->a, p, p->M, pad_rows) >= (1LL << 30) || op_span(p->b, p, p->N, pad_rows) >= (1LL << 30)) return false;
  return true;
}

}  // namespace nrse_gemm_detail
