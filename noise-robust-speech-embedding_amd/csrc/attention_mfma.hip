// MFMA flash-attention kernels for the gated relative-position attention (bf16).
// Placeholder dispatch until the MFMA kernels land: the exact-f32 kernels of attention.hip run.
#include "common.h"

int nrse_attn_use_mfma(int dtype, int head_dim) { return 0; }
int nrse_attn_fwd_mfma(const nrse_attn_fwd_params* p, hipStream_t st) { return NRSE_ERR_UNSUPPORTED; }
int nrse_attn_bwd_mfma(const nrse_attn_bwd_params* p, hipStream_t st) { return NRSE_ERR_UNSUPPORTED; }
