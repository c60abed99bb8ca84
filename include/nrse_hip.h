/*
 * nrse_hip.h — C-ABI of libnrse_hip.so, the MI355X (gfx950 / CDNA4) kernels behind the
 * BYOL-on-WavLM training path (drop-in for /root/reference train_byol.py and src/models/).
 *
 * Conventions:
 *   - every entry point is `extern "C"`, takes plain device pointers + sizes, and enqueues on
 *     the caller's HIP stream (`void* stream` = hipStream_t; pass the current torch stream);
 *   - the caller owns all memory (outputs and scratch are preallocated by the caller);
 *   - no host synchronisation, no hidden allocation (graph-capture safe);
 *   - return 0 on success, a negative nrse_status otherwise; nrse_last_error() returns a
 *     thread-local message for the last failure on the calling thread;
 *   - per-sample data validity (the reference's `None` returns) is reported through int32
 *     status arrays, never through the return code.
 *
 * Reference interface each group replaces is cited per entry point (file:line in the
 * reference, [TF] = transformers 5.15.0 modeling_wavlm.py, see SURVEY.md citation rules).
 */
#ifndef NRSE_HIP_H
#define NRSE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  NRSE_OK = 0,
  NRSE_ERR_ARG = -1,        /* bad shape / null pointer / inconsistent sizes */
  NRSE_ERR_DTYPE = -2,      /* unsupported dtype combination */
  NRSE_ERR_ARCH = -3,       /* device is not gfx950 */
  NRSE_ERR_LAUNCH = -4,     /* hipGetLastError() after launch was not hipSuccess */
  NRSE_ERR_UNSUPPORTED = -5 /* configuration outside what the kernels implement */
} nrse_status;

typedef enum { NRSE_F32 = 0, NRSE_BF16 = 1 } nrse_dtype;

typedef struct {
  int device;
  int cu_count;
  int xcd_count;
  int lds_bytes_per_cu;
  long long hbm_bytes;
  char arch[32];
} nrse_caps;

/* Library / device checks. Fails with NRSE_ERR_ARCH on anything that is not gfx950. */
int nrse_init(int device, nrse_caps* caps);
const char* nrse_last_error(void);
int nrse_abi_version(void);

/* ------------------------------------------------------------------------------------------
 * Generic MFMA GEMM (bf16 in / f32 acc via v_mfma_f32_16x16x32_bf16, or exact f32 via
 * v_mfma_f32_16x16x4_f32). Replaces every nn.Linear / Conv1d contraction on the path:
 *   Linear q/k/v/out  [TF]modeling_wavlm.py:206-226 (F.multi_head_attention_forward)
 *   FFN               [TF]modeling_wavlm.py:274-295
 *   feature projection[TF]modeling_wavlm.py:93-105
 *   conv 1..6         [TF]modeling_wavlm.py:696-720 (as implicit GEMM on channels-last data)
 *   pos-conv          [TF]modeling_wavlm.py:48-90   (grouped implicit GEMM, chunked operand)
 *   heads             src/models/multi_layer_heads.py:16-20, 39-45
 *
 *   C[m,n] = epilogue( alpha * sum_k A(m,k) * B(n,k) )
 * Operand addressing (element offsets), for operand X with "outer" index o and contiguous
 * index c:  off = o*ld + (c >> chunk_shift)*ld_chunk + (c & ((1<<chunk_shift)-1))
 *   kcontig=1: o = m (resp. n), c = k      kcontig=0: o = k, c = m (resp. n)
 * K is split into `nseg` segments of `K` elements each (segment s adds s*seg_stride).
 * grid z = batch * splits; batch zb adds (zb / zdiv)*z1 + (zb % zdiv)*z2 to every pointer;
 * split s handles segments [s*nseg, (s+1)*nseg) and (with NRSE_EPI_SPLIT_SLAB) writes to
 * C + s*c_split.
 * ------------------------------------------------------------------------------------------ */
enum {
  NRSE_EPI_BIAS = 1 << 0,         /* v += bias[n] (f32) */
  NRSE_EPI_GELU = 1 << 1,         /* aux <- v (if aux); v = gelu_erf(v) */
  NRSE_EPI_GELU_BWD = 1 << 2,     /* v *= gelu_erf'(aux[m,n]) */
  NRSE_EPI_DROPOUT = 1 << 3,      /* v = keep ? v/(1-p) : 0   (before residual) */
  NRSE_EPI_RESID = 1 << 4,        /* v += R[m,n] */
  NRSE_EPI_DROP_AFTER = 1 << 5,   /* dropout applied after the residual add */
  NRSE_EPI_ACCUM = 1 << 6,        /* v += C[m,n] (read-modify-write) */
  NRSE_EPI_ATOMIC = 1 << 7,       /* atomicAdd into f32 C */
  NRSE_EPI_COLSUM = 1 << 8,       /* colsum[n] += sum over rows of v (f32 atomics) */
  NRSE_EPI_RELU = 1 << 9          /* v = max(v, 0) */
};

typedef struct {
  const void* ptr;
  int dtype;        /* nrse_dtype; A and B must match */
  int kcontig;      /* 1: K is the contiguous index */
  int chunk_shift;  /* log2 of the contiguous chunk length (0: unchunked) */
  long long ld;
  long long ld_chunk;
  long long seg_stride;
  long long z1, z2;
} nrse_gemm_operand;

typedef struct {
  nrse_gemm_operand a, b;
  int M, N, K, nseg, splits, batch, zdiv;
  float alpha;
  int flags;
  /* C */
  void* c;
  int c_dtype;
  long long ldc, c_z1, c_z2, c_split;
  /* epilogue operands */
  const float* bias;
  const void* aux;       /* GELU pre-activation store (GELU) or load (GELU_BWD) */
  int aux_dtype;
  long long ldaux, aux_z1, aux_z2;
  const void* resid;
  int resid_dtype;
  long long ldr, r_z1, r_z2;
  float dropout_p;
  uint32_t seed;         /* dropout mask = hash(seed, m*N + n) */
  float* colsum;
} nrse_gemm_params;

int nrse_gemm(const nrse_gemm_params* p, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NRSE_HIP_H */
