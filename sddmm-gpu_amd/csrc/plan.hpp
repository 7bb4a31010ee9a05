// plan.hpp — the device-resident BSMR plan (reference BSMR + RPHM, include/BSMR.hpp:21-159).
#pragma once

#include <algorithm>
#include <memory>
#include <mutex>
#include <vector>

#include "common.hpp"

namespace bsmr {

// SDDMM work-list granularity
constexpr u32 TILES_PER_ITEM = 1;   // dense tiles per wave item
constexpr u32 RES_PER_ITEM = 256;   // residual entries per panel-major wave item (panel ranges)
constexpr u32 CM_PER_ITEM = 64;     // residual entries per column-major wave item (full launch)
constexpr u32 RB_PIECE_MAX = 16;    // entries per column-run piece (row-block layout)
constexpr u32 XCD_BUCKETS = 8;      // MI355X XCDs: column bucket -> workgroups b with b % 8

struct Plan;
// fp16/bf16 SDDMM launch (sddmm_half.hip); mode: 1 dense tiles, 2 residual, 3 both
int launch_half(const Plan& p, const void* dA, const void* dB, u32 K, int dtype, float* dP,
                u32 mode, hipStream_t s, u32 nb = 1);
// fp16/bf16 dense-sampled launch (sddmm_dense.hip): K a multiple of 64
int launch_dense(const Plan& p, const void* dA, const void* dB, u32 K, int dtype, float* dP,
                 hipStream_t s, u32 nb = 1);
// fp16/bf16 panel-grouped tile launch (sddmm_half.hip): K in {64, 128, 256, 512}; mode as above
int launch_ptile(const Plan& p, const void* dA, const void* dB, u32 K, int dtype, float* dP,
                 u32 mode, hipStream_t s, u32 nb = 1);

// clustering candidate filter (cluster_filter.hip): the bit triangle of pairs (leader q,
// position p > q) whose similarity bound may reach alpha; W = words per full row
int build_sim_filter(const uint4* pmeta, const u32* enc, u32 M, u32 nbpr, u32 B, u32 keptMask, float alpha,
                     DevBuf<u32>& bits, u32& W, hipStream_t s);
u64 sim_filter_words(u32 M);

u32 block_size_for(u32 M, u32 N, u64 free_mem);
u32 cluster_block_dim(u32 nbpr);
u32 kept_warp_mask(u32 B);

struct Plan {
    int device = 0;
    hipStream_t stream = nullptr;
    u32 M = 0, N = 0, nnz = 0;
    u32 bs = 16, nbpr = 1, B = 32, keptMask = 1;
    float alpha = 0.3f, delta = 0.3f;
    int exact_all = 0;
    // launch layout (bsmr_plan_options.layout): row-block LDS items for K in {64, 128, 256, 512}
    // unless BSMR_LAYOUT_COLMAJOR; the column-major residual slots for every other K
    bool use_rowblock = true;
    bool force_rowblock = false;  // BSMR_LAYOUT_ROWBLOCK: also for tile-dominated plans
    u32 rb_lds_kb = 144;  // LDS budget of a row-block workgroup (bsmr_plan_options.lds_budget_kb)
    bool rb_lds_user = false;  // set by the caller: then also for staged layouts
    // staged-output layouts (below) default to a 120 KiB image and 4 MiB column ranges: the
    // 40 KiB tail holds 10240 results, so items are cut less, and each row block is staged for
    // half as many ranges. C4 reddit-like x0.5 sweep (profiles/r02abl/C4_sweep*.txt): 1.305 ms at
    // (144 KiB, 2 MiB) -> 1.128 ms at (120 KiB, 4 MiB); C3 unchanged (72.9-73.2 us)
    u32 rb_lds_kb_staged = 120, l2_range_kb_staged = 4096;
    u32 diag = 0;  // BSMR_DIAG profiling ablations (wrong results; never set in normal use)
    // L2 budget of one column range of the row-block layout (KiB; BSMR_L2_RANGE_KB)
    u32 l2_range_kb = 2048;
    bool l2_range_user = false;  // BSMR_L2_RANGE_KB given: then also for staged layouts
    // entries per column-run piece of the row-block layout (<= RB_PIECE_MAX; BSMR_PIECE_MAX)
    u32 piece_max = RB_PIECE_MAX;
    // a column-run piece's weight in the item cost model, in entries (BSMR_PIECE_WEIGHT): each
    // piece gathers a whole B row. Measured (profiles/r02c/piece_weight.txt): C2 11.60 us at 1,
    // 11.05 at 4, 11.15 at 8 (items of the short last row block, all short pieces, were the
    // launch's tail); C4 x0.5 -0.8 %; C3 unchanged
    double piece_weight = 4.0;
    // the same weight in the row-panel shard cost (RowBlockLayout::rbCost, bsmr_plan_shard):
    // BSMR_SHARD_PIECE_WEIGHT
    double shard_piece_weight = 4.0;
    // row-block results staged in LDS and written in CSR order per item, for P larger than
    // out_staged_min bytes (BSMR_OUT_STAGED: 0 never, 1 always, else auto). Measured
    // (profiles/r02ab1): C3 cop20k-like (P 10 MB) 77.0 -> 72.0 us, C4 reddit-like x0.5 (232 MB)
    // 1.394 -> 1.305 ms; C2 nips-like (3 MB, P stays in L2 and its scattered stores merge there)
    // 11.86 -> 12.60 us, so it stays on one store per entry
    int out_staged = -1;
    // BSMR_OUT_PACKED: unstaged row-block layouts carry the CSR position in the metadata word
    // (0 never, else whenever nnz <= 2^22)
    int out_packed = -1;
    // A staging with the nt cache policy (BSMR_STAGE_NT: 0 never, 1 always, else auto = staged
    // output layouts when stage_nt_auto)
    int stage_nt = -1;
    int rb_rows_force = -1;  // BSMR_RB_ROWS: rows per row block (tuning / experiments)
    // BSMR_LATE_B: phase-0 B loads after the staging barrier (0 = behind the LDS-DMAs, else on).
    // Measured (profiles/r03d/ab_lateb): C2 11.05 -> 10.86 us, C3 72.0 -> 68.9, C4 x0.5 1.012 ->
    // 0.998 ms, C5 unchanged
    int late_b = -1;
    // item cost cap (multiple of one slot's share of a round; 0 = none), cost-even chunk cuts and
    // list-scheduled (heaviest-first) unsplit items; item_fixed = an item's fixed cost in entries
    // beside its staged rows (piece_weight each). BSMR_ITEM_CAP / BSMR_ITEM_SCHED
    double item_cap = -1.0;  // < 0: auto (build_rowblock_layout), 0: no cap
    bool item_cost_cuts = true, item_lpt = true;
    double item_fixed = 1024.0;
    // sparse-row patterns with fewer row blocks than slots: one block per workgroup slot
    bool small_sparse_rb = true;
    bool stage_nt_auto = false;
    u64 out_staged_min = 8ull << 20;
    // fp16/bf16 patterns with at least this fraction of M x N stored run the dense-sampled
    // launch (whole 128 x 128 MFMA tiles; BSMR_DENSE_MIN; > 1 = never). Measured crossover
    // (tools/dense_sweep.py, 2048^2 bf16 K=512): gathered faster at 3 %, dense from 5 %
    float dense_min = 0.05f;
    // clusters per persistent clustering launch (bsmr_plan_options.cluster_batch); r01k timing
    // on reddit_like x0.25: 512 -> 9.7 s, 4096 -> 4.6 s, 16384 -> 2.3 s (fewer host round trips, more in flight)
    u32 cluster_batch = 16384;
    // clustering candidate filter (cluster_filter.hip; bsmr_tuning.cluster_filter): -1 auto (M >=
    // filter_min_rows, alpha >= 0.01, the filter's buffers fit a quarter of the free memory), 0
    // never, 1 whenever alpha >= 0.01 and it fits
    int cluster_filter = -1;
    u32 filter_min_rows = 32768;
    bool filter_used = false;
    // staged-output row-block layouts (rows >= 512 B) of at least this many items run in pairs
    // (k_sddmm_rb_pair; bsmr_tuning.pair_min_items)
    u32 pair_min_items = 4096;
    // dynamic piece batches of the row-block launch (rows of <= 512 B; bsmr_tuning.batches): 1
    // always, 0 never, -1 for 512-byte rows whose items hold >= batch_min_phases pieces per
    // row-group on average
    int batches = -1;
    double batch_min_phases = 2.0;
    // static piece order of row-block items without dynamic batches (plan.hip balance_pieces;
    // bsmr_tuning.piece_balance): 1 = runs dealt to the least-loaded wave, 0 = longest first in
    // position order
    int piece_balance = 0;
    float filter_ms = 0.f;

    // input
    DevBuf<u32> rowptr, colidx;
    // row stage
    DevBuf<u32> enc, nblk, disp, SC, S1C, asc;
    DevBuf<u32> rows;  // reorderedRows_
    u32 z = 0, R = 0, P = 0;
    int32_t numClusters = 1;
    u64 exact_evals = 0, total_evals = 0;
    float row_ms = 0.f, col_ms = 0.f;

    // column stage (the sorted panel segments do not depend on delta and are kept)
    bool segments_ready = false;
    DevBuf<u32> roff, skeys, svals, ent_idx, seg_begin, seg_end;
    DevBuf<uint8_t> ent_lr;
    DevBuf<u32> denseCols, denseColOffsets, sparseCols, sparseColOffsets, sparseValueOffsets;
    DevBuf<u32> blockOffsets, blockValues, sparseValues, sparseRel, sparseColIdx;
    u32 numDenseTiles = 0, nres = 0, maxTilesPerPanel = 0, numDenseTB = 0, numSparseTB = 0;
    std::vector<u32> h_blockOffsets, h_sparseValueOffsets;

    // work lists
    DevBuf<uint4> denseItems, resItems;
    u32 nDenseItems = 0, nResItems = 0;
    DevBuf<u32> tileRows;  // [tile][16] A-row index of each tile row (NULLV = none)
    // column-major residual execution list (same entries as the reference residual arrays,
    // ordered by (column % 8, column), stable): A row, column, output index; and the
    // XCD-interleaved slots {e0, e1} of the full launch
    DevBuf<u32> cmRow, cmCol, cmOut;
    DevBuf<uint2> cmSlots;
    u32 nSlots = 0;

    // Row-block launch layout for one K (built on first use): the A rows of RB consecutive
    // reordered positions are staged in LDS once per workgroup; residual entries are sorted by
    // (row block, column) so one B read serves a column run. The columns are cut into 8 ranges of
    // equal residual count, one per XCD; item i {rb, t0, t1, e0} (+ itemEnd[i]) holds a chunk of
    // row block rb's entries in column range i % 8 (so its B columns sit in that XCD's L2) and a
    // share of rb's dense tiles; about one item per workgroup slot of the chip.
    // Residual entries of an item are cut into column-run pieces of <= RB_PIECE_MAX entries; the
    // 4-lane row-groups of a workgroup take one piece each per phase, so every group loads its B
    // column in the same (full-width) instruction. items[i].w / itemEnd[i] delimit its pieces.
    struct RowBlockLayout {
        u32 rowBytes = 0, RB = 0, NT = 1024, nRB = 0, nItems = 0, nPieces = 0;
        // panels [pa, pb) covered (the whole plan: 0, P); row block b starts at reordered
        // position 16 * pa + b * RB; rows at or past rowEnd = min(R, 16 * pb) are not staged
        u32 pa = 0, pb = 0, rowEnd = 0;
        // dense tiles run as MFMA tiles only with >= tileMin stored entries; the entries of the
        // others join the residual entries (fp32 MFMA has no rate advantage over vector FMA, so a
        // sparse fp32 tile costs more than its entries' dot products)
        u32 tileMin = 0, nTilesKept = 0, nDemoted = 0, nEntries = 0, nWorkItems = 0;
        DevBuf<u32> tileIds;  // kept tile ids; item tile ranges index this list
        size_t lds = 0;
        DevBuf<u32> meta;   // local row << 22 | column (staged output: local row << 22 | slot)
        DevBuf<u32> out;    // output index (CSR position); released when the output is staged
        // staged output (outLds != 0): an item's results go to LDS at byte offset outLds, slot =
        // the entry's rank by CSR position inside its item, and the workgroup writes them at the
        // end in CSR order (P[sortedPos[ea + t]] = slot t: runs of consecutive positions become
        // full-line stores instead of one scattered 4-byte store per entry). itemEnt[i] = {ea,
        // number of entries} of item i; entries of an item never exceed the LDS tail past the
        // A image (outCap floats)
        u32 outLds = 0, outCap = 0;
        // packed output (unstaged layouts of plans with nnz <= 2^22): the entry metadata's low 22
        // bits hold the CSR position itself, so an entry costs one 4-byte metadata load (no out)
        bool outPacked = false;
        DevBuf<u32> sortedPos;
        DevBuf<uint2> itemEnt;
        // run table (staged output, outRuns): the item's slots in CSR order cut into runs of
        // consecutive positions (one per row it touches when rows are column-sorted): runs[j] =
        // {first position, first slot | length << 16}, itemRuns[i] = {first run, number of runs}
        // (<= NT, one per lane); the store pass then reads 8 bytes per run instead of a position
        // per result, and sortedPos is released
        bool outRuns = false;
        DevBuf<uint2> runs, itemRuns;
        DevBuf<uint4> items;
        DevBuf<u32> itemEnd;
        DevBuf<uint2> pieces;  // {first entry, column | (length - 1) << 22}
        // per row block: Σ over its items of (entries + pieces + 16 tiles + RB staged rows), the
        // shard cost model of bsmr_plan_shard
        std::vector<double> rbCost;
        // per item slot (launch order): {row block, kept tiles, entries, pieces}; padding zeros
        std::vector<uint4> itemStat;
        // original-order row blocks (banded / FEM patterns whose reordering scatters the band):
        // row block b = original rows [b RB, (b + 1) RB), staged through rowIds (identity), every
        // entry residual; whole-plan launches only (shards cut reordered panels)
        bool orig = false;
        // column blocks (wide patterns, Plan::col_blocks): the roles of A and B swapped — block b
        // = original COLUMNS [b RB, (b + 1) RB), their B rows staged through rowIds (identity over
        // N), and each piece a run of one A row (an original row of S) over the block's columns;
        // the metadata's "column" is that row, the output the entry's CSR position. The launch
        // passes B as the staged operand and A as the gathered one; whole-plan launches only
        bool cols = false;
        DevBuf<u32> rowIds;
        // dynamic piece batches (k_sddmm_rb / k_sddmm_rb_pair<.., true>; Plan::batches)
        bool dynBatches = false;
    };
    // rows of 128, 256, 512, 1024 and 2048 bytes, for fp32 [0, 5) and fp16/bf16 [5, 10) (tileMin)
    static constexpr int N_RB_SIZES = 5;
    static constexpr int N_RB_LAYOUTS = 2 * N_RB_SIZES;
    mutable RowBlockLayout rbl[N_RB_LAYOUTS];
    // whole-plan original-order candidates (built for sparse-row patterns) and, per slot, whether
    // the launch uses it: its column-run pieces are below 0.9 x the reordered layout's pieces +
    // 16 per MFMA tile. BSMR_ORIG_ROWS: 0 = never, 1 = always, else auto
    mutable RowBlockLayout rblo[N_RB_LAYOUTS];
    mutable bool rb_use_orig[N_RB_LAYOUTS] = {};
    int orig_rows = -1;
    // whole-plan column-block layouts and whether the launch uses them. BSMR_COL_BLOCKS: 0 =
    // never (default: on C2, the one wide BASELINE pattern, 19 % fewer pieces measured 1 % slower
    // at steady state and 0-4 % faster from a standing start), 1 = always, 2 = for
    // wide patterns (N >= 2 M) whose column-block pieces are below 0.9 x the chosen layout's
    mutable RowBlockLayout rblc[N_RB_LAYOUTS];
    mutable bool rb_use_cols[N_RB_LAYOUTS] = {};
    int col_blocks = 0;
    // BSMR_ORIG_CONTIG: unsplit original-order blocks dealt as contiguous eighths per XCD (1)
    // or to the shortest list (0); C3: 78.6 -> 76.8 us (profiles/r01s)
    int orig_contig = 1;
    // stored entries a dense tile needs to run on MFMA in the row-block launch (BSMR_TILE_MIN_F32
    // / BSMR_TILE_MIN_HALF); 0 = every tile. Measured (r01k sweep, profiles/r01k/tile_min.json):
    // fp32 MFMA (16x16x4) runs at the vector-FMA rate on gfx950 and a tile pays its empty slots,
    // so every fp32 tile is cheaper as residual entries (257: none kept; C2 14.4 -> 12.9 us);
    // fp16/bf16 MFMA is 8x the v_dot2 rate, so half tiles stay unless under half full
    u32 tile_min_f32 = 257, tile_min_half = 128;
    // layouts of panel ranges (row-panel shards, bsmr_sddmm_panels), most recent last
    static constexpr size_t MAX_SHARD_LAYOUTS = 16;
    // shared: a caller keeps its layout alive while another thread's request evicts it
    mutable std::vector<std::shared_ptr<RowBlockLayout>> shard_rbl;
    int build_rowblock_layout(RowBlockLayout& L, u32 rowBytes, u32 pa, u32 pb, u32 tileMin,
                              bool orig = false, bool cols = false) const;
    // the whole-plan layout a launch of this slot uses (rbl, rblo or rblc)
    const RowBlockLayout& rb_whole(int slot) const {
        return rb_use_cols[slot] ? rblc[slot] : rb_use_orig[slot] ? rblo[slot] : rbl[slot];
    }
    // the (cached) layout for rows of rowBytes over panels [pa, pb) for fp32 (half = false) or
    // fp16/bf16 operands; null on error. Call with layout_mu held; the whole-plan layouts are
    // plan members (non-owning pointer), a shard layout is shared with the cache
    std::shared_ptr<const RowBlockLayout> rowblock_layout(u32 rowBytes, bool half, u32 pa, u32 pb,
                                                          int* err) const;

    mutable DevBuf<uint8_t> tmp;  // scan/sort scratch
    // BSMR_DIAG & 32 debug timeline (4 u64 per wave of the last launch)
    mutable DevBuf<unsigned long long> trace;
    mutable size_t traceN = 0;
    int prepare_trace(size_t waves, hipStream_t s) const {
        if (trace.size() < waves * 4) BSMR_CHECK(trace.alloc(waves * 4));
        BSMR_HIP(hipMemsetAsync(trace.data(), 0, waves * 4 * sizeof(unsigned long long), s));
        traceN = waves;
        return BSMR_OK;
    }
    mutable std::mutex layout_mu;
    // identity over reordered positions (built on first use): the row list of launches whose A
    // holds the shard's rows in reordered order (bsmr_sddmm_panels_local)
    mutable DevBuf<u32> iotaR;

    // dense-sampled launch: per 128 x 128 tile of P (original index space) its stored entries
    struct DenseLayout {
        bool built = false;
        u32 ntn = 0, ntiles = 0, nonempty = 0;
        DevBuf<u32> off, loc, out;  // loc = local row << 7 | local column; out = CSR position
    };
    mutable DenseLayout dense;
    // BSMR_DENSE_KS: dense-sampled workgroups of 1 = four waves (64 x 64 quadrants), 2 = eight
    // waves (64 x 32 blocks), else eight below 512 non-empty tiles
    int dense_ks = 0;
    int dense_ns = 2;  // BSMR_DENSE_NS: LDS stages of the eight-wave dense launch (2..5)
    int build_dense_layout() const;

    // panel-grouped tile launch (sddmm_half.hip k_sddmm_ptile): tile-dominated fp16/bf16 plans,
    // K in {64, 128, 256, 512}; items {panel, first tile, tiles <= tpi, 0} in launch order
    struct PtileLayout {
        bool built = false;
        u32 tpi = 0, nItems = 0, nListed = 0, waves = 8, stride = 0;
        // per item slot {first panel, first tile, tiles, second panel + 1 (0: one panel)}
        DevBuf<uint4> items;
        // per item slot (stride u32): 32 A rows (the first panel's 16, then the second's, or the
        // first's again), {first tile, tiles, tiles of the first panel, panels}, 12 zeros, 16
        // columns per tile (a block for every tile and at least one per wave)
        DevBuf<u32> desc;
        static u32 desc_waves(u32 tpi) { return tpi > 0 && tpi <= 4 ? 4u : 8u; }
        static u32 desc_stride(u32 tiles) { return 48 + 16 * tiles; }
    };
    mutable PtileLayout ptile;
    int ptile_mode = -1;  // BSMR_PTILE: 0 never, 1 whenever it applies, -1 auto
    // BSMR_PTILE_TPI: 0 = equal tile runs, one per CU (up to two panels each); n > 0 = items of
    // at most n tiles of one panel (C5 block: 4 -> 5.93 us, 2 -> 7.5, 5 -> 7.7)
    u32 ptile_tpi = 0;
    int build_ptile_layout(u32 tpi) const;

    int build_rows(const u32* h_rowptr, const u32* h_col);
    int build_columns();
    ~Plan() {
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// the whole plan's row-block layout for (K, dtype) (sddmm.hip); *out = null for column-major
int whole_rb_layout(const Plan& p, u32 K, int dtype, const Plan::RowBlockLayout** out,
                    bool reordered = false);
// whether a full launch of layout L runs two items per workgroup (k_sddmm_rb_pair; sddmm.hip)
bool rb_uses_pairs(const Plan& p, const Plan::RowBlockLayout& L);

}  // namespace bsmr

struct bsmr_plan {
    bsmr::Plan p;
};
