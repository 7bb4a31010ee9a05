/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference BSMR-SDDMM hot path (CX9898/sddmm-gpu @ 2025-08-01).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline. The product (sddmm-gpu_amd/) never
 * links or calls it.
 *
 * Parity pinning: the reference cannot be built here (every translation unit pulls
 * cuda_runtime.h / mma.h through TensorCoreConfig.cuh), and it ships no tests or golden
 * vectors. This restatement is pinned against the reference's OWN published logs
 * (scripts/results_suiteSparse_dataset/BSMR_results/ logs) for the matrices of those logs
 * that can be rebuilt exactly from their published definition (Trefethen_20000,
 * Trefethen_20000b, mycielskian14/15/16): every reorder statistic the reference printed
 * (NumRowPanel, bsmr_numClusters, bsmr_numDenseBlock, bsmr_averageDensity,
 * original_numDenseBlock, thread-block and data counts) over the full alpha x delta sweep.
 * See tests/golden/ and DESIGN.md "Oracle".
 */
#pragma once
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_csr orc_csr;
typedef struct orc_plan orc_plan;

/* ---- Matrix Market loader (Matrix.cpp:279-294, 373-480; util.hpp:182-197) ---- */
/* Returns NULL on any rejection the reference makes; prints the reference messages. */
orc_csr* orc_load_mtx(const char* path, int verbose);
orc_csr* orc_load_smtx(const char* path, int verbose);  // Matrix.cpp:296-371
orc_csr* orc_load_snap(const char* path, int verbose);  // Matrix.cpp:482-575
orc_csr* orc_load(const char* path, int verbose);       // suffix dispatch, Matrix.cpp:279-294
orc_csr* orc_csr_from_arrays(uint32_t M, uint32_t N, uint32_t nnz, const uint32_t* rowptr,
                             const uint32_t* colidx);
void orc_csr_info(const orc_csr* c, uint32_t* M, uint32_t* N, uint32_t* nnz);
void orc_csr_copy(const orc_csr* c, uint32_t* rowptr, uint32_t* colidx, float* values);
void orc_csr_free(orc_csr* c);

/* ---- makeData (Matrix.cpp:117-138, util.hpp:71-73): default-seeded mt19937, U[0,2) ---- */
void orc_make_data(uint64_t n, float* out);

/* ---- calculateBlockSize (rowReordering.cu:1009-1025) with free memory as an input ---- */
uint32_t orc_block_size(uint32_t M, uint32_t N, uint64_t free_mem_bytes);
/* clustering block dim B(nbpr) (rowReordering.cu:911-920) */
uint32_t orc_cluster_block_dim(uint32_t nbpr);

/* ---- BSMR row reordering (rowReordering.cu:49-93, 215-432, 893-1095) ----
 * out_rows: capacity M; *out_len = number of non-zero rows kept. exact_all != 0 disables the
 * guard-band fast path and evaluates every similarity with the exact fp32 warp-tree. */
int orc_row_reorder(const orc_csr* c, float alpha, uint32_t block_size, int exact_all,
                    uint32_t* out_rows, uint32_t* out_len, int32_t* out_num_clusters,
                    uint64_t* out_exact_evals, uint64_t* out_total_evals);
/* encodings/dispersion of one row set (for unit tests of the dispersion kernel) */
void orc_dispersion(const orc_csr* c, uint32_t block_size, uint32_t* disp /* M */);

/* ---- column reordering + RPHM + evaluation (colReordering.cu:244-404, BSMR.cpp:83-265, 826-994) */
orc_plan* orc_plan_from_rows(const orc_csr* c, const uint32_t* rows, uint32_t nrows,
                             int32_t num_clusters, float delta);

typedef struct {
    int32_t numRowPanels;
    int32_t numClusters;
    int32_t numDenseBlock;          /* evaluationReordering */
    float averageDensity;
    int32_t originalNumDenseBlock;
    float originalAverageDensity;
    int32_t numDenseThreadBlocks;
    int32_t numSparseThreadBlocks;
    int32_t numDenseData;
    int32_t numSparseData;
    uint32_t maxNumDenseColBlocksInRowPanel;
    uint32_t numDenseBlocksTotal;      /* blockOffsets.back() */
    uint32_t rphmNumSparseThreadBlocks; /* RPHM::numSparseThreadBlocks_ */
} orc_stats;

int orc_plan_stats(const orc_plan* p, orc_stats* s);

enum {
    ORC_REORDERED_ROWS = 0,
    ORC_DENSE_COLS = 1,
    ORC_DENSE_COL_OFFSETS = 2,
    ORC_SPARSE_COLS = 3,
    ORC_SPARSE_COL_OFFSETS = 4,
    ORC_SPARSE_VALUE_OFFSETS = 5,
    ORC_BLOCK_OFFSETS = 6,
    ORC_BLOCK_VALUES = 7,
    ORC_SPARSE_VALUES = 8,
    ORC_SPARSE_RELATIVE_ROWS = 9,
    ORC_SPARSE_COL_INDICES = 10
};
/* returns the array length; copies into out when out != NULL */
uint64_t orc_plan_array(const orc_plan* p, int which, uint32_t* out);
void orc_plan_free(orc_plan* p);

/* ---- host SDDMM (host.cpp:45-76): P[idx] = sum_k A[r*K+k]*B[c*K+k], fp32, k ascending ---- */
void orc_sddmm_cpu(const orc_csr* c, uint32_t K, const float* A, const float* B, float* P,
                   int num_threads);
/* same, but only the rows [row_begin,row_end) (bounded CPU-baseline samples) */
void orc_sddmm_cpu_rows(const orc_csr* c, uint32_t K, const float* A, const float* B, float* P,
                        uint32_t row_begin, uint32_t row_end, int num_threads);
/* the same with thread t pinned to cpus[t % ncpus] (OMP_PROC_BIND=close done explicitly); the
 * caller's mask is restored; returns the number of threads pinned */
int orc_sddmm_cpu_rows_bound(const orc_csr* c, uint32_t K, const float* A, const float* B, float* P,
                             uint32_t row_begin, uint32_t row_end, int nthreads, const int* cpus,
                             int ncpus);

/* ---- checkData (checkData.hpp:14-79) ---- */
int orc_check_one(float a, float b);
/* returns number of mismatches; prints the reference report when verbose */
uint64_t orc_check_data(uint64_t n, const float* a, const float* b, int verbose);

#ifdef __cplusplus
}
#endif
