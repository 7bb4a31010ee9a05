/*
 * bsmr_rocsparse.h — vendor SDDMM baseline (rocSPARSE) on the same device buffers as the engine
 * (libbsmr_rocsparse.so). A baseline, not the product: it is what the reference's cuSPARSE
 * baseline is on NVIDIA hardware.
 *
 * Replaces (paths relative to the reference repository root):
 *   cuSparseSDDMM(A, B, P, logger)   include/cuSparseSDDMM.cuh:27-145
 *   baselines/cuSPARSE_SDDMM/src/cuSPARSE-main.cu (the standalone baseline program)
 * Same operation and operand layouts: P = (A · B) ∘ spy(S), alpha = 1, beta = 0, non-transposed
 * operands, A M×K row-major (ld K), B K×N column-major (ld K), S/P CSR with 32-bit indices,
 * base 0, fp32 compute (CUSPARSE_SDDMM_ALG_DEFAULT -> rocsparse_sddmm_alg_default).
 * fp16/bf16 A/B use rocSPARSE's mixed precision (A/B half, C fp32, compute fp32).
 */
#ifndef BSMR_ROCSPARSE_H
#define BSMR_ROCSPARSE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bsmr_rocsparse bsmr_rocsparse;

/* d_rowptr/d_colidx: DEVICE arrays of S (caller-owned, must outlive the handle).
 * dtype: 0 fp32, 1 fp16, 2 bf16 (bsmr_dtype). alg: 0 default (pattern dot products),
 * 1 dense (rocsparse_sddmm_alg_dense). stream: hipStream_t (NULL = default stream).
 * Runs rocsparse_sddmm_buffer_size + preprocess once (the reference calls preprocess once
 * before its timed loop, cuSparseSDDMM.cuh:115-121). Returns 0 or a bsmr_status code. */
int bsmr_rocsparse_create(uint32_t M, uint32_t N, uint32_t K, uint32_t nnz,
                          const uint32_t* d_rowptr, const uint32_t* d_colidx, int dtype, int alg,
                          void* stream, bsmr_rocsparse** out);
/* One rocsparse_sddmm over device A, B into device P (nnz fp32, CSR order), async on the
 * handle's stream. rocSPARSE reads P even with beta = 0, so P must hold finite values (the
 * reference passes S's values, cuSparseSDDMM.cuh:98-101). */
int bsmr_rocsparse_sddmm(bsmr_rocsparse* h, const void* dA, const void* dB, float* dP);
void bsmr_rocsparse_destroy(bsmr_rocsparse* h);
/* Last error of the calling thread ("" if none). */
const char* bsmr_rocsparse_last_error(void);

#ifdef __cplusplus
}
#endif

#endif
