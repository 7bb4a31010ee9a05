/*
 * bsmr.h — C ABI of the MI355X-native BSMR-SDDMM engine (libbsmr_amd.so).
 *
 * Drop-in boundary for the reference BSMR-SDDMM hot path (CX9898/sddmm-gpu): plain pointers and
 * sizes, int status codes, no exceptions, plan-owned device memory, caller-owned streams.
 * Each entry point names the reference interface it replaces (paths relative to the reference
 * repository root). Reference-side bindings a maintainer would add: INTEGRATION.md.
 *
 * Layouts (same as the reference):
 *   S : CSR, rowptr[M+1] and colidx[nnz] (uint32), column order inside a row = file order.
 *   A : M x K row-major            A[r*K + k]        (Matrix<float>(M,K,row_major), main.cu:23)
 *   B : K x N column-major         B[c*K + k]        (Matrix<float>(K,N,col_major), main.cu:26)
 *   P : nnz values in CSR order    P[idx] = sum_k A[row(idx)*K+k] * B[col(idx)*K+k]
 */
#ifndef BSMR_AMD_H
#define BSMR_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSMR_ABI_VERSION 13 /* 2: bsmr_plan_shard_dtype, layout stats; 3: 128-byte rows (5 sizes);
                              4: dense_sampled_tiles, rb_orig_rows; 5: row-stage export/import,
                              bsmr_sddmm_panels_local, host SDDMM + checkData; 6: bsmr_tuning in
                              the plan options (no environment reads in the library);
                              7: bsmr_tuning.out_packed; 8: bsmr_tuning.sweep*, rb_sweep;
                              9: bsmr_tuning.cluster_filter, filter stats;
                              10: bsmr_plan_check, bsmr_check_rphm_arrays, BSMR_ERR_CHECK,
                              bsmr_tuning.pair_min_items, stats rb_pairs;
                              11: bsmr_tuning.batches, stats rb_batches;
                              12: bsmr_tuning.ptile / ptile_tpi (panel-grouped fp16/bf16 tile
                              launch), piece_balance, stats ptile_items, bsmr_cost_cuts; removed the dropped experiments'
                              knobs piece_order, seg_items, sweep* and stats rb_sweep;
                              13: bsmr_tuning.col_blocks (column-block launch of wide patterns),
                              stats rb_col_blocks */

typedef enum {
    BSMR_OK = 0,
    BSMR_ERR_INVALID = 1,     /* bad argument / shape */
    BSMR_ERR_IO = 2,          /* file cannot be opened or parsed */
    BSMR_ERR_REJECTED = 3,    /* matrix rejected by the reference loader rules */
    BSMR_ERR_HIP = 4,         /* HIP runtime error (message via bsmr_last_error) */
    BSMR_ERR_TIMEOUT = 5,     /* a persistent reorder kernel gave up waiting (never expected) */
    BSMR_ERR_UNSUPPORTED = 6, /* e.g. K not a multiple of 16, dtype not built */
    BSMR_ERR_CHECK = 7        /* bsmr_plan_check found a structural error (bsmr_last_error) */
} bsmr_status;

typedef enum { BSMR_F32 = 0, BSMR_F16 = 1, BSMR_BF16 = 2 } bsmr_dtype;

/* Last error message of the calling thread ("" if none). */
const char* bsmr_last_error(void);
int bsmr_abi_version(void);

/* ------------------------------------------------------------------ host matrix input ---- */
typedef struct bsmr_csr bsmr_csr;

/* Replaces sparseMatrix::CSR<float>::initializeFromMtxFile (src/Matrix.cpp:398-480): .mtx/.mmio
 * only. Same acceptance/rejection rules and messages; verbose != 0 prints
 * "sparseMatrix::CSR initialize from file : <f>" like the reference. */
int bsmr_csr_load_mtx(const char* path, int verbose, bsmr_csr** out);
/* Replaces CSR::initializeFromSmtxFile (Matrix.cpp:296-371), the DLMC .smtx format: header
 * "rows cols nnz", one line of row offsets, one line of column indices; values 1. */
int bsmr_csr_load_smtx(const char* path, int verbose, bsmr_csr** out);
/* Replaces CSR::initializeFromGraphDataset (Matrix.cpp:482-575), SNAP edge lists (.txt): node ids
 * renumbered by first appearance, rows = cols = "Nodes:", nnz = "Edges:". */
int bsmr_csr_load_snap(const char* path, int verbose, bsmr_csr** out);
/* Replaces CSR::initializeFromMatrixFile (Matrix.cpp:279-294): dispatch on the last '.' suffix
 * (.mtx/.mmio, .smtx, .txt); any other suffix prints "Error, file format is not supported". */
int bsmr_csr_load(const char* path, int verbose, bsmr_csr** out);
/* Wrap caller arrays (copied). */
int bsmr_csr_create(uint32_t M, uint32_t N, uint32_t nnz, const uint32_t* rowptr,
                    const uint32_t* colidx, bsmr_csr** out);
void bsmr_csr_info(const bsmr_csr* s, uint32_t* M, uint32_t* N, uint32_t* nnz);
const uint32_t* bsmr_csr_rowptr(const bsmr_csr* s);
const uint32_t* bsmr_csr_colidx(const bsmr_csr* s);
const float* bsmr_csr_values(const bsmr_csr* s);
void bsmr_csr_free(bsmr_csr* s);

/* Replaces Matrix<T>::makeData (src/Matrix.cpp:117-138): n values of a fresh default-seeded
 * std::mt19937 through uniform_real_distribution<float>(0,2), generated single-threaded
 * (the reference's OpenMP loop shares one engine across threads). */
void bsmr_make_data(uint64_t n, float* out);

/* ------------------------------------------------------------------------ the plan ---- */
typedef struct bsmr_plan bsmr_plan;

/* Launch-layout tuning knobs of the SDDMM engine (measurement, A/B experiments, tests). Every
 * field's "auto" value (-1, or < 0 for the floats; diag 0) keeps the measured default. Results
 * are identical for every setting (checkData tolerance) except `diag`, whose profiling ablations
 * drop work on purpose. The library never reads the environment: a caller that wants the
 * BSMR_<FIELD> variables (the tools/ A/B scripts) copies them in with bsmr_tuning_from_env. */
typedef struct {
    uint32_t diag;             /* BSMR_DIAG ablation bits (sddmm.hip; results WRONG); 0 = off */
    int32_t tile_min_f32;      /* BSMR_TILE_MIN_F32: fp32 tiles with fewer entries run as residual
                                  entries on the row-block launch; -1 = 257 (all demoted) */
    int32_t tile_min_half;     /* BSMR_TILE_MIN_HALF: the same for fp16/bf16; -1 = 128 */
    int32_t piece_max;         /* BSMR_PIECE_MAX: entries per column-run piece, 1..16; -1 = 16 */
    float piece_weight;        /* BSMR_PIECE_WEIGHT: item cost of a piece in entries; < 0 = 4 */
    float shard_piece_weight;  /* BSMR_SHARD_PIECE_WEIGHT: the same for shard cuts; < 0 = 4 */
    float dense_min;           /* BSMR_DENSE_MIN: density from which fp16/bf16 patterns take the
                                  dense-sampled launch; < 0 = 0.05 */
    int32_t orig_rows;         /* BSMR_ORIG_ROWS: original-order row blocks 0 never, 1 always,
                                  -1 auto */
    int32_t orig_contig;       /* BSMR_ORIG_CONTIG: their XCD deal, 0 round robin, 1 contiguous
                                  eighths; -1 = 1 */
    int32_t dense_ks;          /* BSMR_DENSE_KS: dense-sampled waves per tile, 1 = four, 2 = eight,
                                  0 = by tile count; -1 = 0 */
    int32_t dense_ns;          /* BSMR_DENSE_NS: dense-sampled LDS stages 2..5; -1 = 2 */
    int32_t out_staged;        /* BSMR_OUT_STAGED: results through LDS in CSR order, 0 never,
                                  1 always, -1 auto (P > 8 MiB) */
    int32_t l2_range_kb;       /* BSMR_L2_RANGE_KB: B bytes per XCD column range (>= 64);
                                  -1 = auto */
    int32_t stage_nt;          /* BSMR_STAGE_NT: row-block A staging with the nt cache policy, 0
                                  never, 1 always, -1 auto */
    int32_t rb_rows;           /* BSMR_RB_ROWS: rows per row block of the row-block launch (a
                                  multiple of 16 within 160 KiB of LDS); -1 = by the LDS budget */
    int32_t late_b;            /* BSMR_LATE_B: 1 = row-block phase-0 B columns loaded after the
                                  staging barrier instead of behind the LDS-DMAs (0 = behind them);
                                  -1 = 1 */
    float item_cap;            /* BSMR_ITEM_CAP: no row-block item above this multiple of one
                                  workgroup slot's share of the launch's cost (0 = no cap);
                                  < 0 = auto: the multiple in {2, 1.5, 1.25, 1} whose item
                                  lists a slot model runs fastest */
    int32_t item_sched;        /* BSMR_ITEM_SCHED: 1 = chunk cuts by cost, unsplit items list-
                                  scheduled heaviest first onto the XCD where they start earliest,
                                  and sparse-row patterns with fewer row blocks than slots sized
                                  to one block per slot; 0 = entry-even cuts, fewest-items deal,
                                  LDS-budget blocks (the item_cap still applies: with item_cap
                                  = 0 as well this is the round-2 layout); -1 = 1 */
    int32_t out_packed;        /* BSMR_OUT_PACKED: unstaged row-block layouts carry each entry's CSR
                                  position in its metadata word (one 4-byte load per entry instead
                                  of two), 0 never, else whenever nnz <= 2^22; -1 = auto */
    int32_t cluster_filter;    /* BSMR_CLUSTER_FILTER: bound every pair's similarity on the matrix
                                  cores before the clustering chain and skip the pairs that cannot
                                  reach alpha (same permutation), 0 never, 1 when
                                  alpha >= 0.01 and its buffers fit a quarter of the free memory,
                                  -1 = auto (the same, from 32768 rows) */
    int32_t pair_min_items;    /* BSMR_PAIR_MIN_ITEMS: staged-output row-block layouts of rows >= 512 B
                                  with at least this many list items run two items per workgroup
                                  (k_sddmm_rb_pair, the second item's staging under the first's
                                  stores); -1 = 4096 */
    int32_t batches;           /* BSMR_BATCHES: row-block launches of rows <= 512 B deal column-run
                                  pieces to waves in batches from an LDS counter instead of fixed
                                  phases; 0 never, 1 always, -1 = auto (512-byte rows, items of
                                  >= 2 pieces per row-group) */
    int32_t ptile;             /* BSMR_PTILE: panel-grouped tile launch for fp16/bf16 K in {64, 128,
                                  256, 512} (every BSMR tile on MFMA, a panel's A rows staged once
                                  per item): 0 never, 1 whenever dtype and K allow, -1 = auto
                                  (tile-dominated plans, e.g. 16 x 16 block masks) */
    int32_t ptile_tpi;         /* BSMR_PTILE_TPI: 0 = equal tile runs, one per CU, of up to two
                                  panels each; 1..64 = items of at most that many tiles of one
                                  panel; -1 = 0 */
    int32_t piece_balance;     /* BSMR_PIECE_BALANCE: row-block items without dynamic batches place
                                  their pieces so that the waves' phase costs even out (runs of
                                  the longest-first list dealt to the least-loaded wave) instead of
                                  longest first in position order; 0 never, 1 always, -1 = auto */
    int32_t col_blocks;        /* BSMR_COL_BLOCKS: column-block launch (blocks of original columns,
                                  B rows staged, A rows gathered per row run) for the whole plan: 0
                                  never, 1 always, 2 = wide patterns (N >= 2 M) with fewer than 0.9 x
                                  the pieces of the row-block layout; -1 = 0 */
} bsmr_tuning;

void bsmr_tuning_default(bsmr_tuning* t);
/* Debug helper: overwrite the fields whose BSMR_<FIELD> environment variable is set (names in
 * the comments above). Returns the number of fields taken from the environment. */
int bsmr_tuning_from_env(bsmr_tuning* t);

typedef struct {
    float alpha;              /* similarity threshold  (Options -a, default 0.3) */
    float delta;              /* tile density threshold (Options -d, default 0.3) */
    uint64_t free_mem_bytes;  /* calculateBlockSize input; 0 = query the device (hipMemGetInfo) */
    int device;               /* HIP device ordinal */
    uint32_t cluster_batch;   /* clusters per persistent launch; 0 = default */
    int exact_similarity;     /* !=0: evaluate every similarity with the exact fp32 tree */
    int layout;               /* SDDMM launch layout: BSMR_LAYOUT_AUTO / _ROWBLOCK / _COLMAJOR */
    uint32_t lds_budget_kb;   /* LDS per row-block workgroup, 16..160 KiB; 0 = default (144) */
    const bsmr_tuning* tuning;  /* launch-layout knobs (copied at plan creation); NULL = auto */
} bsmr_plan_options;

/* AUTO: A rows staged in LDS per row block for rows of 256 B .. 2 KiB (fp32 K = 64..512,
 * fp16/bf16 K = 128..1024), unless dense tiles carry over 3/4 of the work (then one tile per
 * wave, column-major residual slots); the column-major path for other K. ROWBLOCK: row blocks
 * whenever the row size allows. COLMAJOR: column-major slots for every K. Results are identical
 * up to fp32 summation order (checkData tolerance). */
enum { BSMR_LAYOUT_AUTO = 0, BSMR_LAYOUT_ROWBLOCK = 1, BSMR_LAYOUT_COLMAJOR = 2 };

void bsmr_plan_options_default(bsmr_plan_options* o);

/* Replaces BSMR::BSMR(alpha, delta, S) + RPHM::RPHM(S, bsmr) (src/BSMR.cpp:16-265;
 * include/BSMR.hpp:25-28, 83-159): row reordering (rowReordering.cu:1027-1095), column
 * reordering (colReordering.cu:274-404) and the dense-tile / residual layout, all built on the
 * GPU. Host CSR in, device-resident plan out. */
int bsmr_plan_create(const uint32_t* rowptr, const uint32_t* colidx, uint32_t M, uint32_t N,
                     uint32_t nnz, const bsmr_plan_options* opt, bsmr_plan** out);
/* Row stage of a plan (BSMR::rowReordering, BSMR.cpp:27-50 / rowReordering.cu:1027-1095): the
 * clustering result that multi-GPU runs compute once and broadcast (a bit-exact
 * permutation needs the global first-fit over all rows). */
typedef struct {
    uint32_t M, N, nnz;
    uint32_t block_size, num_blocks_per_row, cluster_block_dim;
    uint32_t num_zero_rows;        /* rows dropped before the panels (rowReordering.cu:1081-1090) */
    uint32_t num_reordered_rows;   /* R = M - num_zero_rows: length of the rows array */
    int32_t num_clusters;          /* bsmr_numClusters */
    float alpha;                   /* the similarity threshold the rows were clustered with */
    float row_reorder_ms;
    uint64_t exact_similarity_evals, total_similarity_evals;
} bsmr_row_stage;

/* Copy the row stage out: hdr always, the reordered rows (num_reordered_rows uint32) into `rows`
 * when non-NULL; `rows` may be host or device memory (e.g. the buffer a broadcast sends). */
int bsmr_plan_export_rows(const bsmr_plan* plan, bsmr_row_stage* hdr, uint32_t* rows);
/* Build a plan from an exported row stage without clustering again: the same CSR, the header and
 * rows (host or device memory; checked to be the non-empty rows of S, each once), then the
 * column reordering and tile layout for opt->delta (alpha is the header's). The result is
 * identical to bsmr_plan_create's plan for (alpha, delta); parity arrays DISPERSION/ASCENDING
 * are not kept (length 0). */
int bsmr_plan_import_rows(const uint32_t* rowptr, const uint32_t* colidx,
                          const bsmr_row_stage* hdr, const uint32_t* rows,
                          const bsmr_plan_options* opt, bsmr_plan** out);

/* Test-mode split (sddmm.cu:62-118): keep the row reordering, redo the column split for delta. */
int bsmr_plan_recolumn(bsmr_plan* plan, float delta);
void bsmr_plan_destroy(bsmr_plan* plan);

typedef struct {
    uint32_t M, N, nnz;
    uint32_t block_size;             /* calculateBlockSize */
    uint32_t num_blocks_per_row;     /* nbpr */
    uint32_t cluster_block_dim;      /* B(nbpr) of bsa_clustering */
    int32_t num_clusters;            /* bsmr_numClusters (incl. the reference quirk) */
    uint32_t num_row_panels;         /* NumRowPanel */
    uint32_t num_reordered_rows;
    uint32_t num_dense_tiles;        /* blockOffsets.back() */
    uint32_t max_dense_tiles_per_panel;
    uint32_t num_residual;           /* sparseValueOffsets.back() */
    uint32_t num_dense_thread_blocks;   /* reference launch shape numbers, for the log */
    uint32_t num_sparse_thread_blocks;
    uint64_t exact_similarity_evals;
    uint64_t total_similarity_evals;
    float row_reorder_ms;            /* bsmr_rowReordering */
    float col_reorder_ms;            /* bsmr_colReordering (incl. tile layout) */
    uint32_t dense_items, residual_items;  /* work-list sizes of the SDDMM launch */
    /* row-block layouts built so far (index 0..4: rows of 128/256/512/1024/2048 bytes; 0 = not
     * built): rows per block, workgroup items (incl. per-XCD padding), column-run pieces */
    uint32_t rb_rows[5], rb_items[5], rb_pieces[5];
    /* the same layouts: residual entries (incl. entries of demoted tiles), MFMA tiles kept,
     * non-padding items */
    uint32_t rb_entries[5], rb_tiles[5], rb_work_items[5];
    /* fp16/bf16 dense-sampled launch (whole 128 x 128 MFMA tiles of P, patterns >= 5 % dense):
     * tiles holding at least one stored entry, 0 = not built */
    uint32_t dense_sampled_tiles;
    /* bit i set: row-block layout i (as rb_rows) uses original-order row blocks (banded patterns
     * whose reordering scatters the band) */
    uint32_t rb_orig_rows;
    /* panel-grouped tile launch (bsmr_tuning.ptile): item slots of its list, 0 = not built */
    uint32_t ptile_items;
    /* clustering candidate filter (bsmr_tuning.cluster_filter): 1 when it ran, and its time
     * (included in row_reorder_ms) */
    uint32_t cluster_filter_used;
    float cluster_filter_ms;
    /* bit i set: row-block layout i (as rb_rows) launches two items per workgroup (pairs) */
    uint32_t rb_pairs;
    /* bit i set: row-block layout i (as rb_rows) deals its pieces in dynamic batches */
    uint32_t rb_batches;
    /* bit i set: row-block layout i (as rb_rows) is the column-block launch (bsmr_tuning.col_blocks) */
    uint32_t rb_col_blocks;
} bsmr_plan_stats;

int bsmr_plan_get_stats(const bsmr_plan* plan, bsmr_plan_stats* out);

/* Parity dumps: copy one plan array to host. *len receives the element count; host_out may be
 * NULL to query the length. Arrays are the reference RPHM/BSMR members. */
typedef enum {
    BSMR_ARR_REORDERED_ROWS = 0,
    BSMR_ARR_DENSE_COLS = 1,
    BSMR_ARR_DENSE_COL_OFFSETS = 2,
    BSMR_ARR_SPARSE_COLS = 3,
    BSMR_ARR_SPARSE_COL_OFFSETS = 4,
    BSMR_ARR_SPARSE_VALUE_OFFSETS = 5,
    BSMR_ARR_BLOCK_OFFSETS = 6,
    BSMR_ARR_BLOCK_VALUES = 7,
    BSMR_ARR_SPARSE_VALUES = 8,
    BSMR_ARR_SPARSE_RELATIVE_ROWS = 9,
    BSMR_ARR_SPARSE_COL_INDICES = 10,
    BSMR_ARR_DISPERSION = 11,      /* per original row */
    BSMR_ARR_ASCENDING = 12        /* rows stably sorted by dispersion */
} bsmr_array;
int bsmr_plan_get_array(const bsmr_plan* plan, int which, uint32_t* host_out, uint64_t* len);

/* Reorder-quality statistics printed by the reference log (evaluationReordering,
 * BSMR.cpp:826-994), evaluated on the host from the plan arrays (log only, not timed). */
typedef struct {
    int32_t num_dense_block;          /* bsmr_numDenseBlock */
    float average_density;            /* bsmr_averageDensity */
    int32_t original_num_dense_block; /* original_numDenseBlock */
    float original_average_density;   /* original_averageDensity */
    int32_t num_dense_data;           /* bsmr_numDenseData */
    int32_t num_sparse_data;          /* bsmr_numSparseData */
} bsmr_eval_stats;
int bsmr_plan_evaluate(const bsmr_plan* plan, bsmr_eval_stats* out);

/* Replaces check_rphm(matrix, bsmr, rphm, delta) (src/BSMR.cpp:932-953, with check_rowReordering
 * 444-486, check_colReordering 488-637 and check_rphm 639-824), which the reference runs under
 * VALIDATE before checkSddmm (src/sddmm.cu:34-38). Host check of the plan against its S:
 *   row reordering: every non-empty row exactly once, no empty row;
 *   column reordering: per panel the dense / sparse column lists are the panel's columns, each
 *     once, in descending count order, padded with the sentinel N, the dense prefix exactly the
 *     16-column groups reaching ceil(delta * 256) entries, the sparse data in order and counted;
 *   RPHM: every blockValues slot the CSR index of its (row, column) or NULL, every sparse value in
 *     its row and column, every stored entry in exactly one of blockValues / sparseValues;
 *   launch layout (K > 0): the layout bsmr_sddmm runs for (K, dtype) computes every stored entry
 *     exactly once (kept MFMA tile, column-run piece or residual slot) with its row, column and
 *     output position consistent with S.
 * verbose != 0 prints the reference's messages on stderr ("Error! Row is duplicated! ...", then
 * "Error! The row reordering is incorrect!" / "... col reordering ..." / "... rphm ..." / "Error!
 * The launch layout is incorrect! ..."). Returns BSMR_OK when every check passes, BSMR_ERR_CHECK
 * when one fails (bsmr_last_error names the first failure). Not timed; O(nnz) host work. */
int bsmr_plan_check(const bsmr_plan* plan, uint32_t K, int dtype, int verbose);
/* The same row / column / RPHM checks over caller host arrays (S in CSR, and the plan arrays as
 * bsmr_plan_get_array returns them: R reordered rows, P = ceil(R / 16) panels), e.g. a plan dumped
 * by another build or the reference's own RPHM copied to the host. No device needed. */
int bsmr_check_rphm_arrays(uint32_t M, uint32_t N, uint32_t nnz, const uint32_t* rowptr,
                           const uint32_t* colidx, uint32_t R, const uint32_t* rows,
                           const uint32_t* denseColOffsets, const uint32_t* denseCols,
                           const uint32_t* sparseColOffsets, const uint32_t* sparseCols,
                           const uint32_t* sparseValueOffsets, const uint32_t* blockOffsets,
                           const uint32_t* blockValues, const uint32_t* sparseValues,
                           const uint32_t* sparseRelativeRows, const uint32_t* sparseColIndices,
                           float delta, int verbose);

/* ------------------------------------------------------------------------- SDDMM ---- */
/* Replaces sddmm_gpu(M, N, K, dA, dB, rphm, dP, logger) (include/sddmmKernel.cuh:25-30,
 * src/sddmmKernel.cu:2540-2762): device pointers, dA row-major M x K, dB column-major K x N,
 * dP (fp32, nnz, CSR order) overwritten. dtype selects the A/B element type (fp32, or fp16/bf16
 * with fp32 accumulation). stream: a hipStream_t (NULL = default stream). Asynchronous. */
int bsmr_sddmm(const bsmr_plan* plan, const void* dA, const void* dB, uint32_t K, int dtype,
               float* dP, void* stream);
/* Replaces sddmm_gpu_batch(numBatch, M, N, K, nnz, dA, dB, rphm, dP, time)
 * (include/sddmmKernel.cuh:41-47, src/sddmmKernel.cu:2764-2850): the same plan over num_batch
 * (A, B) pairs, batch b at dA + b*M*K, dB + b*N*K elements, writing dP + b*nnz (the reference's
 * batch strides, sddmmKernel.cu:1281-1283). One launch per 65535 batches. Asynchronous. */
int bsmr_sddmm_batch(const bsmr_plan* plan, uint32_t num_batch, const void* dA, const void* dB,
                     uint32_t K, int dtype, float* dP, void* stream);

/* Row-panel sharding for multi-GPU runs: rank's contiguous panel range [p0, p1)
 * of `world`; bsmr_sddmm_panels computes only the outputs of those panels (any dtype on the
 * row-block launch). When (K, dtype) runs the row-block launch the cuts fall on its row-block
 * boundaries, balanced by the layout's item costs (entries, column-run pieces, tiles, staged
 * rows; builds the layout on first use); otherwise by the per-panel model of bsmr_shard_cuts.
 * bsmr_plan_shard = bsmr_plan_shard_dtype(..., BSMR_F32, ...). */
int bsmr_plan_shard(const bsmr_plan* plan, uint32_t K, int rank, int world, uint32_t* p0,
                    uint32_t* p1);
int bsmr_plan_shard_dtype(const bsmr_plan* plan, uint32_t K, int dtype, int rank, int world,
                          uint32_t* p0, uint32_t* p1);
/* Measured-cost rebalancing of the row-block cut: prev_cuts[world+1] are the panel cuts the ranks
 * ran (bsmr_plan_shard_dtype's, or an earlier rebalance) and shard_ms[world] the time each shard
 * took; every row block's model cost is scaled by its shard's measured / predicted ratio and the
 * plan is cut again (cuts[world+1], row-block boundaries). A shard whose time is 0, NaN or inf
 * counts as unmeasured: its row blocks keep their model cost (scaled by the measured shards' mean
 * factor). Deterministic in its inputs, so every
 * rank derives the same cuts from the same gathered times. Row-block launches of reordered
 * plans only, else BSMR_ERR_UNSUPPORTED. */
int bsmr_plan_shard_rebalance(const bsmr_plan* plan, uint32_t K, int dtype, int world,
                              const uint32_t* prev_cuts, const float* shard_ms, uint32_t* cuts);
/* Per-panel cost model on host offset arrays (no device): cuts[world+1], cuts[0]=0,
 * cuts[world]=P. */
int bsmr_shard_cuts(const uint32_t* blockOffsets, const uint32_t* sparseValueOffsets, uint32_t P,
                    uint32_t K, int world, uint32_t* cuts);
/* Host-only form of the row-block cuts behind bsmr_plan_shard_dtype / bsmr_plan_shard_rebalance
 * (no plan, no device): nblocks blocks of panels_per_block panels (the last may be short; P panels
 * in all) with model costs block_cost[b]; cuts[0..world] at the block boundary nearest each equal
 * share of the cumulative cost. With prev_cuts and shard_ms (both or neither): each block's cost
 * scaled by its previous shard's measured / predicted time first (unmeasured shards keep the mean
 * factor). Deterministic in its inputs, so every rank derives the same cuts. */
int bsmr_cost_cuts(const double* block_cost, uint32_t nblocks, uint32_t panels_per_block, uint32_t P,
                   int world, const uint32_t* prev_cuts, const float* shard_ms, uint32_t* cuts);
int bsmr_sddmm_panels(const bsmr_plan* plan, const void* dA, const void* dB, uint32_t K,
                      int dtype, float* dP, uint32_t p0, uint32_t p1, void* stream);

/* The same shard launch with a shard-local A: dA_local holds only the A rows of reordered
 * positions [16 p0, min(16 p1, R)) in that order (row j = A row reorderedRows[16 p0 + j]), so a
 * rank receives just its panels' rows ("A partitioned"). dB and dP as in
 * bsmr_sddmm (whole B, P in CSR order; only the shard's outputs are written). Row-block launches
 * only (rows of 128 B .. 2 KiB), else BSMR_ERR_UNSUPPORTED. */
int bsmr_sddmm_panels_local(const bsmr_plan* plan, const void* dA_local, const void* dB,
                            uint32_t K, int dtype, float* dP, uint32_t p0, uint32_t p1,
                            void* stream);

/* Timing: run `iters` back-to-back SDDMMs on `stream`, timing each kernel with HIP events on
 * that stream. Outputs average ms per launch of the dense-tile kernel, the residual kernel and
 * the whole SDDMM. */
int bsmr_sddmm_profile(const bsmr_plan* plan, const void* dA, const void* dB, uint32_t K,
                       int dtype, float* dP, int iters, void* stream, float* ms_dense,
                       float* ms_residual, float* ms_total);

/* ------------------------------------------------------------------- validation ---- */
/* Replaces sddmm_cpu(A, B, S, P) (src/host.cpp:45-76): host SDDMM in the reference's loop order
 * (per stored entry a serial fp32 `val += A[r*K+k] * B[c*K+k]`, k ascending, no FMA), rows split
 * over nthreads host threads (0 = all cores); P receives nnz values in CSR order. */
int bsmr_sddmm_cpu(const uint32_t* rowptr, const uint32_t* colidx, uint32_t M, uint32_t N,
                   uint32_t K, const float* A, const float* B, float* P, int nthreads);
/* Replaces checkOneData<float> (include/checkData.hpp:21-30): 1 if |a-b| < 1e-5 or
 * |a-b| / max(|a|, |b|, 1e-3) < 1e-3. */
int bsmr_check_one(float data1, float data2);
/* Replaces checkDataFunction (include/checkData.hpp:44-79): returns the number of mismatches;
 * verbose != 0 prints the reference's framed report (first 9 errors, error rate) on stdout. */
uint64_t bsmr_check_data(uint64_t n, const float* data1, const float* data2, int verbose);

#ifdef __cplusplus
}
#endif
#endif /* BSMR_AMD_H */
