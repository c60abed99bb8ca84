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
 *     status arrays, never through the return code;
 *   - ABI handshake (ABI 10): every params struct starts with `uint32_t struct_size`, which the
 *     caller sets to sizeof(struct) as compiled against THIS header (NRSE_PARAMS_INIT below). An
 *     entry point (and a *_workspace query) refuses any other value with NRSE_ERR_ARG before it
 *     reads a further field, so a caller built against an older or newer header -- whose struct is
 *     shorter or longer -- is refused instead of having its struct read past the end.
 *     nrse_abi_version() returns NRSE_ABI_VERSION for callers that also want to log it.
 *
 * Reference interface each group replaces is cited per entry point (file:line in the
 * reference, [TF] = transformers 5.15.0 modeling_wavlm.py, see SURVEY.md citation rules).
 */
#ifndef NRSE_HIP_H
#define NRSE_HIP_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define NRSE_ABI_VERSION 11
/* ABI 11: the MXFP6 correction-plane dtype (4) and nrse_split_lo_mx6 / nrse_cast_mx6 retired; the
 * params structs are unchanged from ABI 10 (the *_dtype fields now accept 0 / NRSE_FP8 only) */
/* zero-initialise a params struct and stamp its size: nrse_gemm_params p; NRSE_PARAMS_INIT(p); */
#define NRSE_PARAMS_INIT(s)            \
  do {                                 \
    memset(&(s), 0, sizeof(s));        \
    (s).struct_size = sizeof(s);       \
  } while (0)

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

typedef enum { NRSE_F32 = 0, NRSE_BF16 = 1, NRSE_BF16X3 = 2, NRSE_FP8 = 3 } nrse_dtype;
/* (dtype 4 was NRSE_MX6, OCP MXFP6 correction planes, ABI 8-10: measured slower than fp8 at the
 * same accuracy and retired in ABI 11; every entry point refuses it.) */
/* NRSE_FP8 (ABI 6): OCP fp8 e4m3fn (gfx950's native fp8), one byte per element, saturated at +-448;
 * the split-weight mode's correction operands (nrse_gemm_params.a8 / b8). */
/* NRSE_BF16X3 (an OUTPUT format of nrse_layernorm_fwd and nrse_conv0_fwd only): the split-bf16
 * activation of the split-weight mode's conv stack, three bf16 planes of n = rows * C elements
 * each at the output pointer: [hi | lo | hi], hi = bf16(y), lo = bf16(y - hi). A GEMM that reads
 * plane 0 with seg_stride n over nseg = 3 segments against weight planes [hi | hi | lo] computes
 * y_hi w_hi + y_lo w_hi + y_hi w_lo: the f32 product to ~2^-16. */

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
 * split s handles segments [s*nseg, (s+1)*nseg) and writes to C + s*c_split (c_split = 0: every
 * split into C, with NRSE_EPI_ATOMIC; c_split > 0: per-split f32 slabs, summed afterwards by
 * nrse_splitk_reduce).
 * ------------------------------------------------------------------------------------------ */
enum {
  NRSE_EPI_BIAS = 1 << 0,         /* v += bias[n] (f32); with splits > 1 only split 0 adds it */
  NRSE_EPI_GELU = 1 << 1,         /* aux <- v (if aux); v = gelu_erf(v) */
  NRSE_EPI_GELU_BWD = 1 << 2,     /* v *= gelu_erf'(aux[m,n]) */
  NRSE_EPI_DROPOUT = 1 << 3,      /* v = keep ? v/(1-p) : 0   (before residual) */
  NRSE_EPI_RESID = 1 << 4,        /* v += R[m,n] */
  NRSE_EPI_DROP_AFTER = 1 << 5,   /* dropout applied after the residual add */
  NRSE_EPI_ACCUM = 1 << 6,        /* v += C[m,n] (read-modify-write) */
  NRSE_EPI_ATOMIC = 1 << 7,       /* atomicAdd into f32 C */
  NRSE_EPI_COLSUM = 1 << 8,       /* colsum[n] += sum over rows of v (f32 atomics) */
  NRSE_EPI_RELU = 1 << 9,         /* v = max(v, 0) */
  NRSE_EPI_TANH = 1 << 10         /* v = tanh(v) (attentive statistics pooling, src/models/pool.py:43) */
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
  uint32_t struct_size;  /* ABI 10: sizeof(nrse_gemm_params), checked by every entry point taking it */
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
  long long bias_z1, bias_z2;  /* batch offsets of bias (grouped pos-conv) */
  const void* aux;       /* GELU pre-activation store (GELU) or load (GELU_BWD) */
  int aux_dtype;
  long long ldaux, aux_z1, aux_z2;
  const void* resid;
  int resid_dtype;
  long long ldr, r_z1, r_z2;
  float dropout_p;
  uint32_t seed;         /* dropout mask = hash(seed, element offset of C[m,n] from c) */
  float* colsum;
  /* optional f32 workspace of nrse_gemm_colsum_workspace(p) floats (COLSUM): the
   * per-tile column sums are then added in a fixed order (deterministic) instead of by atomics */
  float* colsum_part;
  /* ABI 6, the split-weight mode's fp8 correction segments: after the nseg bf16 segments, nseg8
   * more K segments of K elements each whose operands a8 / b8 are NRSE_FP8, k-contiguous (ld,
   * seg_stride, z1, z2 in bytes = elements), multiplied on the MX-scaled MFMA
   * (v_mfma_scale_f32_16x16x128_f8f6f4, 2x the bf16 rate) with B scaled by 2^-b8_exp:
   *   C[m,n] = epilogue( alpha * (sum_bf16 + 2^-b8_exp * sum_{s<nseg8, k<K} a8(m,k) b8(n,k)) ).
   * Requires the 256x256 kernel's conditions, K % 128 == 0, splits == 1, 16-byte aligned a8 / b8
   * with ld, seg_stride, z1, z2 multiples of 16; nseg8 = 0 (or zeroed trailing fields): none. */
  nrse_gemm_operand a8, b8;
  int nseg8;
  int b8_exp;
  /* ABI 6: optional fp8 copy of a bf16 output, written beside C by the register epilogues of the
   * 256x256 kernel: c8[m * ldc8 + n] = fp8(bf16 C[m, n]) (the next GEMM's a8 operand: FFN-up's
   * GELU output feeding FFN-down's correction segment). ldc8 % 16 == 0, 16-byte aligned. */
  void* c8;
  long long ldc8;
  int c8_dtype;                   /* 0 or NRSE_FP8 (fp8); anything else is refused */
} nrse_gemm_params;

int nrse_gemm(const nrse_gemm_params* p, void* stream);
long long nrse_gemm_colsum_workspace(const nrse_gemm_params* p);  /* floats for p->colsum_part */
/* Kernel generation used by nrse_gemm for bf16 operands: 0 = automatic (default), 1 = register
 * staged 128x128, 2 = LDS-DMA 128x128, 3 = LDS-DMA 256x256 (falls back when a problem does not
 * fit it). Process-wide; for tests and benchmarks. Returns the previous setting. */
int nrse_gemm_select(int generation);
/* Tile rows of the 256-column LDS-DMA kernel: 256 (the default) or 224 pins one, 0 = automatic
 * (224 when that needs no more tile waves than 256, e.g. M = 12768 = 57 x 224: faster alone, slower
 * beside concurrent streams). Process-wide; for tests and benchmarks. Returns the previous setting. */
int nrse_gemm_tile_rows(int rows);

/* ------------------------------------------------------------------------------------------
 * LayerNorm over the last (channel) dim of channels-last rows, fp32 statistics.
 *   conv layers       [TF]modeling_wavlm.py:712-720 (LN(512) + GELU, fused: flags |= NRSE_LN_GELU)
 *   feature projection[TF]modeling_wavlm.py:101
 *   encoder layers    [TF]modeling_wavlm.py:357, 369, final 513
 * fwd: y = act(LN(x)) ; saves mean/rstd per row.
 * bwd: dy is read directly ([rows, C]), through col2im of a conv dgrad GEMM output
 *      (dy_mode = NRSE_DY_COL2IM: dy[b, tau] = sum_j G[b, (tau-j)/s, j*C + c] over valid j), or
 *      broadcast per utterance (NRSE_DY_BCAST: dy[b, t] = dy_vec[b] * dy_scale, the time-mean
 *      shim). dx = resid + LN'(...) (resid optional, f32). dgamma/dbeta accumulate (f32 atomics).
 * ------------------------------------------------------------------------------------------ */
enum { NRSE_LN_GELU = 1, NRSE_LN_RELU = 2 };   /* RELU: emotion heads, src/models/emotion.py:34-58 */
enum { NRSE_DY_DIRECT = 0, NRSE_DY_COL2IM = 1, NRSE_DY_BCAST = 2 };

typedef struct {
  uint32_t struct_size;  /* ABI 10: sizeof(nrse_ln_fwd_params), checked by every entry point taking it */
  const void* x; int x_dtype;
  const float* gamma; const float* beta;
  void* y; int y_dtype;
  float* mean; float* rstd;
  long long rows; int C; float eps; int flags;
  /* ABI 6, optional (bf16 y): y8 [rows, C] NRSE_FP8 = fp8(bf16 y), the next GEMM's a8 operand
   * (split-weight mode); 16-byte aligned */
  void* y8;
  /* ABI 7: y8_split = 1 makes y8 the two fp8 correction planes of the exact output o (the conv
   * stack's split-weight form): y8 [2, rows, C] = [fp8((o - bf16(o)) 2^y8_exp) |
   * fp8(bf16(o))], y = bf16(o); the next conv GEMM's a8 segments against [fp8(w_hi) | fp8(w_lo 2^e)] */
  int y8_split; int y8_exp;
  int y8_dtype;                   /* 0 or NRSE_FP8 (fp8); anything else is refused */
  /* ABI 10, optional: sat_count[0] += the number of y8 values whose fp8 conversion saturated
   * (|v| > 448 before rounding; the scaled correction plane and the unscaled hi / fp8(bf16 y) plane
   * alike). Never touched when nothing saturates; the engine reads it back lagged and re-derives
   * the split-weight exponents when it moves (nrse_amd/engine.py rederive_split_exponents) */
  unsigned int* sat_count;
} nrse_ln_fwd_params;

typedef struct {
  uint32_t struct_size;  /* ABI 10: sizeof(nrse_ln_bwd_params), checked by every entry point taking it */
  const void* dy; int dy_dtype; int dy_mode;
  int col_k, col_s, col_tout, col_tin;   /* NRSE_DY_COL2IM geometry; rows = batch * col_tin */
  int bcast_t; float dy_scale;           /* NRSE_DY_BCAST: rows per utterance, scale */
  const void* x; int x_dtype;
  const float* gamma; const float* beta;
  const float* mean; const float* rstd;
  void* dx; int dx_dtype;
  const float* resid;                    /* optional f32 [rows, C] added to dx */
  float* dgamma; float* dbeta;
  long long rows; int C; int flags;
  /* optional fused consumer of dx (the residual branch's dropout backward, replacing a separate
   * nrse_dropout_cast_colsum pass over dx): dv = dropout(dx; dv_p, dv_seed) in dv_dtype,
   * dv_colsum[c] += sum_r dv[r, c] (if dv_colsum) */
  void* dv; int dv_dtype; float* dv_colsum; float dv_p; uint32_t dv_seed;
  /* optional f32 workspace of nrse_layernorm_bwd_workspace(p) floats: the column sums (dgamma,
   * dbeta, dv_colsum) are then added in a fixed order (deterministic) instead of by f32 atomics */
  float* part;
  /* optional (the encoder form: resid given, x / dy / resid f32, dy direct): the gated rel-pos
   * attention's gate-path gradient added to dy on the fly, so nrse_gate_bwd_dp need not
   * read-modify-write the LN1 gradient: dy[r, 64 h + d] += gate_dp[r, h, 0] * sum_{i<4} gate_w[i, d]
   * + gate_dp[r, h, 1] * sum_{i>=4} gate_w[i, d]; gate_dp [rows, C / 64, 2] f32 (8-byte aligned),
   * gate_w [8, 64] (gru_rel_pos_linear.weight, [TF]modeling_wavlm.py:164-176) */
  const float* gate_dp; const float* gate_w;
} nrse_ln_bwd_params;

int nrse_layernorm_fwd(const nrse_ln_fwd_params* p, void* stream);
int nrse_layernorm_bwd(const nrse_ln_bwd_params* p, void* stream);
long long nrse_layernorm_bwd_workspace(const nrse_ln_bwd_params* p);  /* floats for p->part */

/* Final encoder LN fused with the time-mean pooling shim:
 * emb[b, c] = mean_t LN(h[b, t])[c]; emb must be zeroed by the caller. part: optional f32
 * workspace of batch * ceil(T / 32) * C floats (the 32-frame chunk sums then add in a fixed
 * order, deterministic; NULL: f32 atomics). */
int nrse_ln_mean_fwd(const float* h, const float* gamma, const float* beta, float* emb, float* mean, float* rstd,
                     int batch, int T, int C, float eps, float* part, void* stream);

/* ------------------------------------------------------------------------------------------
 * Gated relative-position attention, WavLMAttention ([TF]modeling_wavlm.py:147-271) with
 * F.multi_head_attention_forward / SDPA ([TORCH]functional.py:6206, 6629).
 * Layouts: qkv [B*T, 3*Hd] rows = (q | k | v), head h at columns h*64..h*64+63 (head_dim 64);
 * ctx [B*T, Hd]; gate, lse, delta [B, H, T] f32; bucket [2T-1] int32 = bucket(j - i) at j-i+T-1.
 * The relative-position bias (layer-0 table, reused by every layer as in [TF]modeling_wavlm.py:505)
 * depends on j - i only: the bf16 MFMA kernels read it as a Toeplitz vector bias_vec [H, 2T-1]
 * (bias_vec[h, j-i+T-1] = E[bucket(j-i), h], nrse_rel_bias_vec), staged per workgroup in LDS; the
 * f32 parity-mode kernels read the expanded table bias [H, T, Tb], Tb = nrse_bias_ld(T) (rows
 * padded to a multiple of 64 with zeros, nrse_rel_bias_fwd).
 * Dropout on the attention probabilities: keep(i) = hash(seed, ((b*H+h)*T+i)*T+j).
 * ------------------------------------------------------------------------------------------ */
int nrse_bias_ld(int T);
int nrse_rel_bias_fwd(const float* E, const int* bucket, float* bias, int H, int T, int nb, void* stream);
/* bias_vec[h, e] = E[bucket[e], h], e in [0, 2T-1) */
int nrse_rel_bias_vec(const float* E, const int* bucket, float* bias_vec, int H, int T, int nb, void* stream);
/* dE[bucket[d], h] += diag[h, d] (compute_bias backward), as a gather in a fixed order: order
 * [2T-1] lists the offsets d sorted by bucket (increasing d within a bucket), offsets [nb+1] the
 * start of each bucket's run (nrse_amd.hostside.bucket_runs). */
int nrse_rel_bias_bwd(const float* diag, const int* order, const int* offsets, float* dE, int H, int T, int nb,
                      void* stream);

/* gate[b,h,t] = a*(b_*c_h - 1) + 2 with (a, b_) = sigmoid(pair sums of gru_rel_pos_linear(x_h))
 * ([TF]modeling_wavlm.py:164-176). x1 [B*T, Hd] (the LN1 output), W [8, 64], bias [8], c [H]. */
int nrse_gate_fwd(const void* x1, int x_dtype, const float* W, const float* bvec, const float* c, float* gate,
                  int batch, int T, int H, void* stream);
/* Gate backward, fused: dx1 (f32 [B*T, Hd]) += the gate-path gradient, and the parameter
 * gradients accumulated: dW [8, 64] (gru_rel_pos_linear.weight), db [8] (its
 * bias), dc [H] (gru_rel_pos_const). x1, dx1 16-byte aligned. */
int nrse_gate_bwd(const void* x1, int x_dtype, const float* W, const float* bvec, const float* c, const float* dgate,
                  float* dx1, float* dW, float* db, float* dc, int batch, int T, int H, float* part, void* stream);
/* The same with the gate-path gradient left for the LN backward to add (nrse_ln_bwd_params.gate_dp):
 * dp [B*T, H, 2] f32 receives (dpa, dpb) per (row, head); dx1 is not touched. */
int nrse_gate_bwd_dp(const void* x1, int x_dtype, const float* W, const float* bvec, const float* c,
                     const float* dgate, float* dp, float* dW, float* db, float* dc, int batch, int T, int H,
                     float* part, void* stream);
/* part (optional): f32 workspace of nrse_gate_bwd_workspace(H) floats; the per-workgroup
 * parameter gradients are then added in a fixed order (deterministic) instead of by atomics */
long long nrse_gate_bwd_workspace(int H);

typedef struct {
  uint32_t struct_size;  /* ABI 10: sizeof(nrse_attn_fwd_params), checked by every entry point taking it */
  const void* qkv; int dtype;     /* q/k/v (bf16 or f32) */
  const float* gate; const float* bias;
  void* ctx;                      /* [B*T, Hd] same dtype as qkv */
  float* lse;                     /* [B, H, T] */
  int batch, T, H, head_dim;
  float scale;                    /* 1/sqrt(head_dim) */
  float dropout_p; uint32_t seed;
  const float* bias_vec;          /* [H, 2T-1] (bf16 MFMA path); bias [H, T, Tb] is the f32 path's */
  uint16_t* drop_mask;            /* optional (bf16 MFMA path, dropout_p > 0): the keep bits of the
                                     probability dropout, [B*H][ntiles][4][Tp] u16 (ntiles = Tp/64,
                                     Tp = T rounded up to 64): word (bh, key tile kt, g, query q) bit
                                     4t + r = keep(q, key 64 kt + 16 t + 4 g + r); the backward reads
                                     them instead of re-hashing (nrse_attn_mask_elems) */
  int drop_mask_in;               /* nonzero (bf16 MFMA path): drop_mask already holds the keep bits
                                     (nrse_attn_dropout_mask, the same function of seed and position)
                                     and the forward reads them instead of hashing */
  void* ctx8;                     /* ABI 6, optional (bf16 MFMA path): [B*T, Hd] NRSE_FP8 copy of ctx,
                                     fp8(bf16 ctx) (the out-projection's fp8 correction operand);
                                     4-byte aligned. NULL: none */
  int ctx8_dtype;                 /* 0 or NRSE_FP8 (fp8); anything else is refused */
} nrse_attn_fwd_params;

typedef struct {
  uint32_t struct_size;  /* ABI 10: sizeof(nrse_attn_bwd_params), checked by every entry point taking it */
  const void* qkv; int dtype;
  const float* gate; const float* bias;
  const void* ctx; const void* dctx;   /* O and dO */
  const float* lse;
  float* delta;                        /* scratch [B, H, T]: rowsum(dO * O) */
  void* dqkv;                          /* [B*T, 3*Hd] */
  float* dgate;                        /* [B, H, T] */
  float* diag;                         /* [H, 2T-1] f32, accumulated: sum_b gate * dS along j-i */
  int batch, T, H, head_dim;
  float scale; float dropout_p; uint32_t seed;
  const float* bias_vec;               /* [H, 2T-1] (bf16 MFMA path) */
  float* diag_part;                    /* optional: f32 workspace of nrse_attn_bwd_workspace(p)
                                          floats; the per-block diag rows are then added in a fixed
                                          order (deterministic) instead of by f32 atomics */
  const uint16_t* drop_mask;           /* optional (ABI 6: trailing, after diag_part): the forward's
                                          keep bits (nrse_attn_fwd_params.drop_mask); NULL re-hashes */
} nrse_attn_bwd_params;

int nrse_attn_fwd(const nrse_attn_fwd_params* p, void* stream);
int nrse_attn_bwd(const nrse_attn_bwd_params* p, void* stream);
long long nrse_attn_bwd_workspace(const nrse_attn_bwd_params* p);  /* floats for p->diag_part */
long long nrse_attn_mask_elems(int batch, int T, int H);           /* u16 words of drop_mask */
/* The attention-probability dropout keep bits of one layer in the drop_mask layout, computed ahead
 * of the forward (a data-independent pure-VALU kernel that needs no LDS and few VGPRs, so its waves
 * run beside the 256x256 GEMMs' on the same SIMDs); the forward then reads them
 * (drop_mask_in = 1). Words of queries q >= T are zero. */
int nrse_attn_dropout_mask(uint16_t* drop_mask, int batch, int T, int H, float dropout_p, uint32_t seed,
                           void* stream);

/* ------------------------------------------------------------------------------------------
 * Conv feature encoder front end and the positional-conv weight norm.
 * conv0 = Conv1d(1 -> C, k, stride s, no bias) + LN(C) + GELU ([TF]modeling_wavlm.py:712-720),
 * channels-last output [B, T0, C]. Backward recomputes conv0 from the waveform, applies the
 * LN+GELU backward and accumulates only dW (the waveform needs no gradient), in TAP-MAJOR
 * layout dw[k][C] (contiguous atomics; the caller transposes into the [C][1][k] parameter
 * gradient); dy may come through col2im of conv1's dgrad GEMM (same geometry fields as
 * nrse_ln_bwd_params).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  uint32_t struct_size;  /* ABI 10: sizeof(nrse_conv0_params), checked by every entry point taking it */
  const float* wav; int L;        /* [B, L] f32 */
  const float* w;                 /* [C, k] */
  const float* gamma; const float* beta;
  void* out; int out_dtype;       /* [B, T0, C] = gelu(LN(conv)) */
  float* mean; float* rstd;       /* [B*T0] */
  const void* dy; int dy_dtype; int dy_mode; int col_k, col_s, col_tout;   /* bwd only */
  float* dw; float* dgamma; float* dbeta;     /* bwd only; dw is [k][C] (tap-major) */
  int batch, T0, C, k, s; float eps;
  float* part;                    /* bwd, optional: f32 workspace of nrse_conv0_bwd_workspace(p)
                                     floats; dw / dgamma / dbeta are then added in a fixed order
                                     (deterministic) instead of by f32 atomics */
  /* fwd, ABI 7, optional (bf16 out, k = 10, C = 256 | 512): the fp8 correction planes of the exact
   * output o, y8 [2, B*T0, C] NRSE_FP8 = [fp8((o - bf16(o)) 2^y8_exp) | fp8(bf16(o))] (as
   * nrse_ln_fwd_params.y8_split); out = bf16(o). 16-byte aligned */
  void* y8; int y8_exp;
  int y8_dtype;                   /* fwd: 0 or NRSE_FP8 (fp8); anything else is refused */
  unsigned int* sat_count;        /* fwd, ABI 10, optional: as nrse_ln_fwd_params.sat_count, for y8 */
} nrse_conv0_params;
int nrse_conv0_fwd(const nrse_conv0_params* p, void* stream);
int nrse_conv0_bwd(const nrse_conv0_params* p, void* stream);
long long nrse_conv0_bwd_workspace(const nrse_conv0_params* p);

/* weight_norm(dim=2) of the grouped pos-conv ([TF]modeling_wavlm.py:61-77):
 * w[o, i, j] = g[j] * v[o, i, j] / ||v[:, :, j]||.  Writes the two GEMM weight layouts
 *   wf [G][cpg][K*cpg]: wf[g][o][j*cpg + i]        (forward:  B operand, n = o)
 *   wd [G][cpg][K*cpg]: wd[g][i][j'*cpg + o] = w[g*cpg+o][i][K-1-j']  (dgrad, flipped taps)
 * and norms[K]. Backward takes dWf in the wf layout (f32) and produces dg [K], dv [H, cpg, K].
 * part: optional scratch of 256 * K doubles (K <= 256 dividing 256) for the coalesced two-stage
 * per-tap reductions (ordered, deterministic); null -> one strided block per tap (slow). */
int nrse_weight_norm_fwd(const float* g, const float* v, void* wf, void* wd, int w_dtype, float* norms, int H,
                         int cpg, int K, double* part, void* stream);
int nrse_weight_norm_bwd(const float* dWf, const float* g, const float* v, const float* norms, float* dg, float* dv,
                         float* scratch, int H, int cpg, int K, double* part, void* stream);

/* ------------------------------------------------------------------------------------------
 * Elementwise / data-movement kernels of the step.
 * ------------------------------------------------------------------------------------------ */
/* dst[b, pad_front + t, :] = (mask[b,t] ? embed : src[b, t, :]) (cast to dst dtype); the pad
 * rows of dst are zeroed. If h_inout is non-null the SpecAugment row replacement is also
 * applied in place to the f32 hidden state ([TF]modeling_wavlm.py:1006-1011). */
int nrse_specaug_pad(float* h_inout, const unsigned char* mask, const float* embed, void* dst, int dst_dtype,
                     int batch, int T, int C, int pad_front, int pad_back, void* stream);
/* ABI 10: the SpecAugment time masks of one forward, drawn on the device ([TF]modeling_wavlm.py:834-954
 * _compute_mask_indices, full-length utterances): mask [batch, T] u8 (1 = masked frame). The span
 * count n = int(mask_prob T / mask_length + eps) (then >= min_masks, <= T / mask_length, <= the
 * T - mask_length + 1 candidate starts), eps = 24 random bits of the seed; per utterance the n starts
 * are a uniform random subset of the candidates (the n smallest counter-hash keys), each masking
 * mask_length frames. mask_prob <= 0: all zeros. T - mask_length + 1 <= 4096. Replaces the reference's
 * numpy draw and the per-step host-to-device copy of its mask (oracle/masks.py specaug_mask replays it). */
int nrse_specaug_mask(unsigned char* mask, int batch, int T, double mask_prob, int mask_length, int min_masks,
                      uint32_t seed, void* stream);
/* generic padded copy: dst[b, pad_front + t, :] = src[b, t, :], pad rows zeroed */
int nrse_pad_rows(const void* src, int src_dtype, void* dst, int dst_dtype, int batch, int T, int C, int pad_front,
                  int pad_back, void* stream);
/* SpecAugment + dropout backward on the feature-projection output:
 * dembed[c] += sum over masked rows of dh; out = (masked ? 0 : dh) * dropout_mask(seed, p). */
int nrse_specaug_bwd(const float* dh, const unsigned char* mask, float* dembed, void* out, int out_dtype, int batch,
                     int T, int C, float dropout_p, uint32_t seed, float* part, void* stream);
/* part (optional): f32 workspace of min(B*T, 2048) * C floats: dembed's per-workgroup sums are
 * then added in a fixed order (deterministic) instead of by f32 atomics */
/* out[i] = in[i] * dropout_mask(seed, p)[i] (cast); in f32, out f32/bf16 */
int nrse_dropout_cast(const float* in, void* out, int out_dtype, long long n, float dropout_p, uint32_t seed,
                      void* stream);
/* out[r, c] = in[r, c] * dropout_mask(seed, p)[r*C + c] (cast) and colsum[c] += sum_r out[r, c]
 * in one pass (the nn.Dropout backward feeding a Linear: its input gradient and bias gradient,
 * [TF]modeling_wavlm.py:294, 482). C % 8 == 0, 16-byte aligned. */
int nrse_dropout_cast_colsum(const float* in, void* out, int out_dtype, long long rows, int C, float dropout_p,
                             uint32_t seed, float* colsum, float* part, void* stream);
/* colsum[c] += sum_r x[r, c]. part: optional f32 workspace of nrse_colsum_workspace(rows, C) floats
 * (also for nrse_dropout_cast_colsum): the row-chunk sums are then added in a fixed order
 * (deterministic) instead of by f32 atomics. */
int nrse_colsum(const void* x, int dtype, float* colsum, long long rows, int C, float* part, void* stream);
long long nrse_colsum_workspace(long long rows, int C);
/* y = x cast (f32 <-> bf16), n elements */
int nrse_cast(const void* x, int x_dtype, void* y, int y_dtype, long long n, void* stream);
/* split-bf16 pair of an f32 tensor: hi = bf16(x), lo = bf16(x - hi) (the split-weight mode's GEMM
 * operand planes: x @ (hi + lo) carries the f32 weight to ~2^-17 relative) */
int nrse_split_bf16(const float* x, void* hi, void* lo, long long n, void* stream);
/* ABI 6: the fp8 correction plane of the same split: lo8[i] = fp8((x[i] - bf16(x[i])) * 2^lo8_exp)
 * (NRSE_FP8, saturated), as nrse_adamw_params.p_shadow_lo8 writes it */
int nrse_split_lo8(const float* x, void* lo8, int lo8_exp, long long n, unsigned int* sat_count, void* stream);
/* (ABI 10: sat_count optional, += the saturated conversions, as nrse_adamw_params.sat_count) */
/* ABI 6: y8[i] = fp8(x[i]) of a bf16 / f32 tensor (NRSE_FP8, saturated at +-448), n elements */
int nrse_cast_fp8(const void* x, int x_dtype, void* y8, long long n, void* stream);
/* ABI 6: dst[i] = 0 for i < n floats (the step's small accumulators: no torch fill kernel) */
int nrse_zero(float* dst, long long n, void* stream);
/* Split-K reduction of a weight gradient (the Linear wgrads of the backward, train_byol.py:65):
 * dst[i] (+)= sum_s slabs[s * n + i], s = 0 .. splits-1, in split order (deterministic); f32;
 * accumulate = 0 overwrites dst. The partial slabs are written by nrse_gemm with c_split = n. */
int nrse_splitk_reduce(float* dst, const float* slabs, int splits, long long n, int accumulate, void* stream);
/* Ordered reduction of per-workgroup partial rows (the deterministic form of the gradient
 * column sums and accumulators): a slab row is [d0: n0 | d1: n1 | d2: n2] (d1, d2 optional, in
 * order); d_j[b * n_j + c] (+)= sum_{s < S} slab[(b * S + s) * n + off_j + c] in s order, for
 * b < batch (16-byte vectors when every n_j % 4 == 0 and the pointers are aligned). */
int nrse_rows_reduce(float* d0, long long n0, float* d1, long long n1, float* d2, long long n2, const float* slab, int S,
                     int batch, int accumulate, void* stream);
/* ABI 9: deferred reductions. nrse_reduce_defer(1) makes every later nrse_rows_reduce -- including
 * the ones the LayerNorm / attention / gate backward, GEMM column-sum and colsum entry points end
 * with -- queue its reduction (up to 256) instead of launching it; nrse_reduce_flush(stream) runs
 * the queue on `stream` (batched, up to 12 reductions per launch, bitwise the sums of the
 * immediate form) and empties it. The caller keeps each queued slab and destination alive and
 * unchanged until the flush's work has run on that stream (the step's backward queues a layer's
 * reductions on the dX chain's stream and flushes them on the weight-gradient stream:
 * engine.py encoder_backward). Returns the previous setting; process-wide, not thread-safe
 * (one engine per process). Replaces nothing in the reference (its reductions are ATen's). */
int nrse_reduce_defer(int on);
int nrse_reduce_pending(void);
int nrse_reduce_flush(void* stream);
/* ABI 10: drop the queued reductions without running them and turn deferral off (error recovery:
 * a caller whose backward raised mid-layer must not flush jobs whose workspaces it has released) */
int nrse_reduce_discard(void);
/* dst[a][c][b] (+)= src[a][b][c]  (conv weight [co][ci][k] <-> implicit-GEMM layout [co][k][ci]) */
int nrse_swap12(const void* src, int src_dtype, void* dst, int dst_dtype, int d0, int d1, int d2, int accumulate,
                void* stream);
/* out[b, pad_front + t, c] = dy[b, t, c] * gelu'(pre[b, t, c]); pad rows zeroed */
int nrse_gelu_bwd_pad(const float* dy, const void* pre, int pre_dtype, void* out, int out_dtype, int batch, int T,
                      int C, int pad_front, int pad_back, void* stream);

/* ------------------------------------------------------------------------------------------
 * Heads + loss: BatchNorm1d (train: batch stats, running stats momentum / unbiased var;
 * eval: running stats) with optional fused ReLU (multi_layer_heads.py:16-20, 39-45) and the
 * BYOL loss forward+backward (src/models/byol.py:104-128).
 * ------------------------------------------------------------------------------------------ */
int nrse_bn_fwd(const float* x, const float* w, const float* b, float* y, float* run_mean, float* run_var,
                float* save_mean, float* save_invstd, int rows, int C, float momentum, float eps, int train, int relu,
                void* stream);
int nrse_bn_bwd(const float* dy, const float* x, const float* y, const float* w, const float* save_mean,
                const float* save_invstd, float* dx, float* dw, float* db, int rows, int C, int relu, void* stream);
/* SyncBatchNorm for data-parallel heads (torch.nn.SyncBatchNorm semantics over the reference's
 * BatchNorm1d, src/models/multi_layer_heads.py:16-20, 39-45): phase 1 per-column local sums
 * (f64 sum x, sum x^2 -> sums[2C]), the caller all-reduces them, phase 2 normalises with the global
 * statistics over nglobal rows; backward: local (sum dy, sum dy*xhat) -> sums[2C], all-reduced by
 * the caller into global_sums; dw/db accumulate the local share. */
int nrse_bn_stats(const float* x, double* sums, int rows, int C, void* stream);
int nrse_bn_fwd_global(const float* x, const float* w, const float* b, float* y, float* run_mean, float* run_var,
                       float* save_mean, float* save_invstd, const double* global_sums, long long nglobal, int rows,
                       int C, float momentum, float eps, int relu, void* stream);
int nrse_bn_bwd_sums(const float* dy, const float* x, const float* y, const float* save_mean,
                     const float* save_invstd, float* sums, int rows, int C, int relu, void* stream);
int nrse_bn_bwd_global(const float* dy, const float* x, const float* y, const float* w, const float* save_mean,
                       const float* save_invstd, const float* local_sums, const float* global_sums, long long nglobal,
                       float* dx, float* dw, float* db, int rows, int C, int relu, void* stream);
/* loss[0] = 2 - 2 mean_b clamp(<p_b/|p_b|, z_b/|z_b|>, -1, 1) (+1e-10 offsets, eps 1e-10);
 * dp = dloss/dp (scaled by grad_scale); stats[0..1] = NaN flags before/after normalisation. */
int nrse_byol_loss(const float* p, const float* z, float* loss, float* dp, float* stats, int rows, int D,
                   float grad_scale, float* part, void* stream);
/* part (optional): f32 workspace of rows * (stats ? 3 : 1) floats; the per-row loss terms (and
 * NaN flags) are then added in row order (deterministic) instead of by f32 atomics */

/* ------------------------------------------------------------------------------------------
 * Downstream emotion head (BASELINE configs[3]; src/models/emotion.py over the frozen encoder).
 * Attentive statistics pooling (src/models/pool.py:25-58) per utterance b over its first
 * lens[b] frames (feat_len = (wav_len - 1) // 320 + 1, pool.py:11-19):
 *   x [B, T, C] encoder output (f32/bf16), h [B, T, C] f32 = tanh(sap_linear(x)) (nrse_gemm with
 *   NRSE_EPI_TANH), att [C]; w = softmax_t(h . att); pooled [B, 2C] = [sum w x,
 *   sqrt(max(sum w x^2 - mu^2, 1e-5))]; w_out [B, T] and var_out [B, C] are saved for backward.
 * Backward: dpre [B, T, C] = d(sap pre-activation) (zero past lens[b]; dtype dpre_dtype),
 *   datt [C] accumulated; the encoder is frozen (no dx). C % 256 == 0, C <= 2048.
 * CCC loss (src/train/dimentional_emotions.py:427-450): loss[0] = mean_d (1 - CCC_d) over pred,
 *   target [rows, D]; dpred (optional) = dloss/dpred; 0 when rows <= 1.
 * ------------------------------------------------------------------------------------------ */
int nrse_asp_fwd(const void* x, int x_dtype, const float* h, const float* att, const int* lens, int batch, int T,
                 int C, float* w_out, float* var_out, float* pooled, void* stream);
int nrse_asp_bwd(const void* x, int x_dtype, const float* h, const float* att, const int* lens, int batch, int T,
                 int C, const float* w_in, const float* var_in, const float* pooled, const float* dpooled, void* dpre,
                 int dpre_dtype, float* datt, void* stream);
int nrse_ccc_loss(const float* pred, int ld, const float* target, float* loss, float* dpred, int rows, int D,
                  void* stream);   /* pred / dpred rows of stride ld >= D, target [rows, D] */

/* ------------------------------------------------------------------------------------------
 * Optimiser tail over the flat f32 parameter / gradient buffers (train_byol.py:67-71,
 * src/models/byol.py:62-73): sum of squares (f64 accumulation), clip + AdamW, target EMA.
 * ------------------------------------------------------------------------------------------ */
int nrse_sumsq(const float* x, long long n, double* out, double* part, void* stream);
/* part (optional): f64 workspace of 4096 doubles; the per-workgroup sums are then added in a
 * fixed order (deterministic) instead of by f64 atomics */
typedef struct {
  uint32_t struct_size;  /* ABI 10: sizeof(nrse_adamw_params), checked by every entry point taking it */
  float* p; const float* g; float* m; float* v; void* p_shadow; int shadow_dtype;
  long long n;
  float lr, beta1, beta2, eps, weight_decay; int step;
  float max_norm; const double* sumsq;    /* clip coefficient min(1, max_norm/(sqrt(sumsq)+1e-6)) */
  float grad_scale;                       /* extra multiplier on g (e.g. 1/world_size) */
  void* p_shadow_lo;                      /* optional (bf16 shadow only): lo = bf16(p - shadow), the
                                             split-weight mode's second weight plane */
  /* optional target EMA fused into the update (src/models/byol.py:62-73, as nrse_ema on the
   * updated p): for i < ema_n, ema_t[i] = ema_decay * ema_t[i] + (1 - ema_decay) * p_new[i], its
   * shadow (ema_shadow_dtype, and the bf16 lo plane) written alongside; saves nrse_ema's re-read
   * of p and its launch. ema_t null: no EMA. ema_n <= n. */
  float* ema_t;
  void* ema_shadow;
  void* ema_shadow_lo;
  int ema_shadow_dtype;
  float ema_decay;
  long long ema_n;
  /* ABI 6, optional: the split-weight mode's fp8 correction planes (NRSE_FP8, one byte per weight):
   * p_shadow_lo8[i] = fp8((p_new[i] - bf16(p_new[i])) * 2^lo8_exp), ema_shadow_lo8 likewise for the
   * EMA target (i < ema_n); the nrse_gemm b8 operand with b8_exp = lo8_exp */
  void* p_shadow_lo8;
  void* ema_shadow_lo8;
  int lo8_exp;
  /* ABI 6, optional: nonzero stores 0 to every g[i] after reading it, so the gradient buffer is
   * zeroed for the next step's accumulation inside this pass (no separate fill over g) */
  int zero_grad;
  int lo8_dtype;                  /* 0 or NRSE_FP8 (fp8); anything else is refused */
  /* ABI 10, optional: sat_count[0] += the number of fp8 correction values (p_shadow_lo8 and
   * ema_shadow_lo8) that saturated, |(w - bf16 w) 2^lo8_exp| > 448: lo8_exp no longer has headroom
   * for the weights (they grew in training); the caller re-derives it (see nrse_ln_fwd_params).
   * sat_ranges (optional, device memory): sat_nranges sorted [start, end) pairs of flat indices,
   * p[i] being flat index sat_offset + i; only saturations inside them count (the planes of the
   * weights no GEMM reads -- norms, biases, heads -- may saturate harmlessly). Checked only on the
   * saturating path (a binary search per saturated element): free in normal operation */
  unsigned int* sat_count;
  const long long* sat_ranges;
  int sat_nranges;
  long long sat_offset;
} nrse_adamw_params;
int nrse_adamw(const nrse_adamw_params* p, void* stream);
/* t_shadow_lo: optional, as nrse_adamw_params.p_shadow_lo */
int nrse_ema(float* target, const float* online, void* t_shadow, int shadow_dtype, long long n, float decay,
             void* t_shadow_lo, void* stream);
/* health check (train_byol.py:52-59 / debugging_utils.py:4-30): accumulates into the caller-zeroed
 * stats[0..3] = NaN count, Inf count, sum|x| over finite x, max|x| over finite x (decisions on the
 * host, nrse_amd/health.py, in check_audio_tensor's order) */
int nrse_health(const void* x, int dtype, long long n, float* stats, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused on-GPU SNR mix (src/data/augment.py:4-66 + noisy_speech_dataset.py:88-129):
 * per pair b: tile/truncate noise to L, k = sqrt(Ps / (Pn * 10^(snr/10))), y = s + k n,
 * peak-normalise both, optional zero-mean/unit-var (feature extractor do_normalize).
 * mode (`do_normalize` argument): 0 = raw mix y = s + k n (add_noise_to_speech), 1 = + peak
 * normalisation, 2 = + feature-extractor normalisation. noise_len[b] <= noise_stride.
 * status[b] follows oracle/snr_mix.py codes (0 = ok); outputs of failed pairs are zeroed.
 * scratch: batch * NRSE_SNR_SCRATCH_PER_PAIR doubles -> the chunked form (16 workgroups per pair,
 * four launches, per-chunk f64 partials folded in chunk order); null -> one workgroup per pair.
 * ------------------------------------------------------------------------------------------ */
#define NRSE_SNR_SCRATCH_PER_PAIR 256
int nrse_snr_mix(const float* clean, const float* noise, const int* noise_len, long long noise_stride,
                 const float* snr_db, float* clean_out, float* noisy_out, int* status, float* kscale, double* scratch,
                 int batch, int L, int do_normalize, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NRSE_HIP_H */
