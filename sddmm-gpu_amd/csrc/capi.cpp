// capi.cpp — plan lifecycle, parity dumps, reorder statistics and sharding of the C ABI.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "plan.hpp"

using namespace bsmr;

extern "C" void bsmr_plan_options_default(bsmr_plan_options* o) {
    o->alpha = 0.3f;   // Options.hpp:40
    o->delta = 0.3f;   // Options.hpp:41
    o->free_mem_bytes = 0;
    o->device = 0;
    o->cluster_batch = 0;
    o->exact_similarity = 0;
    o->layout = BSMR_LAYOUT_AUTO;
    o->lds_budget_kb = 0;
    o->tuning = nullptr;
}

extern "C" void bsmr_tuning_default(bsmr_tuning* t) {
    t->diag = 0;
    t->tile_min_f32 = t->tile_min_half = t->piece_max = -1;
    t->piece_weight = t->shard_piece_weight = t->dense_min = -1.0f;
    t->orig_rows = t->orig_contig = t->dense_ks = t->dense_ns = t->out_staged = -1;
    t->l2_range_kb = -1;
    t->stage_nt = -1;
    t->rb_rows = -1;
    t->late_b = -1;
    t->item_cap = -1.0f;
    t->item_sched = -1;
    t->out_packed = -1;
    t->cluster_filter = -1;
    t->pair_min_items = -1;
    t->batches = -1;
    t->ptile = t->ptile_tpi = -1;
    t->piece_balance = -1;
    t->col_blocks = -1;
}

extern "C" int bsmr_tuning_from_env(bsmr_tuning* t) {
    int n = 0;
    auto geti = [&](const char* name, int32_t& f) {
        if (const char* v = std::getenv(name)) {
            f = std::atoi(v);
            ++n;
        }
    };
    auto getf = [&](const char* name, float& f) {
        if (const char* v = std::getenv(name)) {
            f = static_cast<float>(std::atof(v));
            ++n;
        }
    };
    // tri-state switches: "0" never, "1" always, anything else auto
    auto get3 = [&](const char* name, int32_t& f) {
        if (const char* v = std::getenv(name)) {
            f = v[0] == '0' ? 0 : v[0] == '1' ? 1 : -1;
            ++n;
        }
    };
    if (const char* v = std::getenv("BSMR_DIAG")) {
        t->diag = static_cast<uint32_t>(std::atoi(v));
        ++n;
    }
    geti("BSMR_TILE_MIN_F32", t->tile_min_f32);
    geti("BSMR_TILE_MIN_HALF", t->tile_min_half);
    geti("BSMR_PIECE_MAX", t->piece_max);
    getf("BSMR_PIECE_WEIGHT", t->piece_weight);
    getf("BSMR_SHARD_PIECE_WEIGHT", t->shard_piece_weight);
    getf("BSMR_DENSE_MIN", t->dense_min);
    get3("BSMR_ORIG_ROWS", t->orig_rows);
    geti("BSMR_ORIG_CONTIG", t->orig_contig);
    geti("BSMR_DENSE_KS", t->dense_ks);
    geti("BSMR_DENSE_NS", t->dense_ns);
    get3("BSMR_OUT_STAGED", t->out_staged);
    geti("BSMR_L2_RANGE_KB", t->l2_range_kb);
    get3("BSMR_STAGE_NT", t->stage_nt);
    geti("BSMR_RB_ROWS", t->rb_rows);
    geti("BSMR_LATE_B", t->late_b);
    getf("BSMR_ITEM_CAP", t->item_cap);
    get3("BSMR_ITEM_SCHED", t->item_sched);
    get3("BSMR_OUT_PACKED", t->out_packed);
    get3("BSMR_CLUSTER_FILTER", t->cluster_filter);
    geti("BSMR_PAIR_MIN_ITEMS", t->pair_min_items);
    get3("BSMR_BATCHES", t->batches);
    get3("BSMR_PTILE", t->ptile);
    geti("BSMR_PTILE_TPI", t->ptile_tpi);
    get3("BSMR_PIECE_BALANCE", t->piece_balance);
    geti("BSMR_COL_BLOCKS", t->col_blocks);
    return n;
}

namespace {

// device, stream and the launch / tuning options shared by bsmr_plan_create and
// bsmr_plan_import_rows
int init_plan(Plan& p, const bsmr_plan_options& o) {
    p.device = o.device;
    if (hipSetDevice(o.device) != hipSuccess) {
        set_error("bsmr_plan: hipSetDevice failed");
        return BSMR_ERR_HIP;
    }
    if (hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking) != hipSuccess) {
        set_error("bsmr_plan: hipStreamCreate failed");
        return BSMR_ERR_HIP;
    }
    p.alpha = o.alpha;
    p.delta = o.delta;
    p.exact_all = o.exact_similarity;
    if (o.cluster_batch) p.cluster_batch = o.cluster_batch;
    if (o.layout < BSMR_LAYOUT_AUTO || o.layout > BSMR_LAYOUT_COLMAJOR ||
        (o.lds_budget_kb && (o.lds_budget_kb < 16 || o.lds_budget_kb > 160))) {
        set_error("bsmr_plan: bad layout or lds_budget_kb");
        return BSMR_ERR_INVALID;
    }
    p.use_rowblock = o.layout != BSMR_LAYOUT_COLMAJOR;
    p.force_rowblock = o.layout == BSMR_LAYOUT_ROWBLOCK;
    if (o.lds_budget_kb) {
        p.rb_lds_kb = o.lds_budget_kb;
        p.rb_lds_user = true;
    }
    if (const bsmr_tuning* t = o.tuning) {  // launch-layout knobs; "auto" keeps the defaults
        p.diag = t->diag;
        if (t->tile_min_f32 >= 0) p.tile_min_f32 = static_cast<u32>(t->tile_min_f32);
        if (t->tile_min_half >= 0) p.tile_min_half = static_cast<u32>(t->tile_min_half);
        if (t->piece_max >= 0) p.piece_max = std::min<u32>(RB_PIECE_MAX, std::max(1, t->piece_max));
        if (t->piece_weight >= 0) p.piece_weight = t->piece_weight;
        if (t->shard_piece_weight >= 0) p.shard_piece_weight = t->shard_piece_weight;
        if (t->dense_min >= 0) p.dense_min = t->dense_min;
        if (t->orig_rows >= 0) p.orig_rows = t->orig_rows ? 1 : 0;
        if (t->orig_contig >= 0) p.orig_contig = t->orig_contig;
        if (t->dense_ks >= 0) p.dense_ks = t->dense_ks;
        if (t->dense_ns >= 0) p.dense_ns = t->dense_ns;
        if (t->out_staged >= 0) p.out_staged = t->out_staged ? 1 : 0;
        if (t->out_packed >= 0) p.out_packed = t->out_packed ? 1 : 0;
        if (t->stage_nt >= 0) p.stage_nt = t->stage_nt ? 1 : 0;
        if (t->rb_rows > 0) p.rb_rows_force = t->rb_rows;
        if (t->late_b >= 0) p.late_b = t->late_b;
        if (t->item_cap >= 0) p.item_cap = t->item_cap;
        if (t->item_sched >= 0)
            p.item_cost_cuts = p.item_lpt = p.small_sparse_rb = t->item_sched != 0;
        if (t->cluster_filter >= 0) p.cluster_filter = t->cluster_filter ? 1 : 0;
        if (t->pair_min_items >= 0) p.pair_min_items = static_cast<u32>(t->pair_min_items);
        if (t->batches >= 0) p.batches = t->batches ? 1 : 0;
        if (t->ptile >= 0) p.ptile_mode = t->ptile ? 1 : 0;
        if (t->ptile_tpi >= 0) p.ptile_tpi = static_cast<u32>(std::min(64, t->ptile_tpi));
        if (t->piece_balance >= 0) p.piece_balance = t->piece_balance ? 1 : 0;
        if (t->col_blocks >= 0) p.col_blocks = std::min(2, t->col_blocks);
        if (t->l2_range_kb >= 0) {
            p.l2_range_kb = static_cast<u32>(std::max(64, t->l2_range_kb));
            p.l2_range_user = true;
        }
    }
    return BSMR_OK;
}

bool valid_csr(const uint32_t* rowptr, const uint32_t* colidx, uint32_t M, uint32_t N,
               uint32_t nnz) {
    return rowptr && colidx && M != 0 && N != 0 && rowptr[M] == nnz && nnz >= 2;
}

}  // namespace

extern "C" int bsmr_plan_create(const uint32_t* rowptr, const uint32_t* colidx, uint32_t M,
                                uint32_t N, uint32_t nnz, const bsmr_plan_options* opt,
                                bsmr_plan** out) {
    *out = nullptr;
    if (!valid_csr(rowptr, colidx, M, N, nnz)) {
        set_error("bsmr_plan_create: invalid CSR (need rowptr[M] == nnz >= 2)");
        return BSMR_ERR_INVALID;
    }
    bsmr_plan_options o;
    if (opt)
        o = *opt;
    else
        bsmr_plan_options_default(&o);
    auto* h = new bsmr_plan;
    Plan& p = h->p;
    auto fail = [&](int st) {
        delete h;
        return st;
    };
    p.M = M;
    p.N = N;
    p.nnz = nnz;
    int st = init_plan(p, o);
    if (st != BSMR_OK) return fail(st);
    u64 free_mem = o.free_mem_bytes;
    if (free_mem == 0) {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
            set_error("bsmr_plan_create: hipMemGetInfo failed");
            return fail(BSMR_ERR_HIP);
        }
        free_mem = fr;
    }
    p.bs = block_size_for(M, N, free_mem);
    if (p.bs > 65535) {
        set_error("bsmr_plan_create: column block size exceeds 16-bit encoding");
        return fail(BSMR_ERR_UNSUPPORTED);
    }
    p.nbpr = static_cast<u32>(std::ceil(static_cast<float>(N) / static_cast<float>(p.bs)));  // rowReordering.cu:1035
    p.B = cluster_block_dim(p.nbpr);
    p.keptMask = kept_warp_mask(p.B);
    st = p.build_rows(rowptr, colidx);
    if (st != BSMR_OK) return fail(st);
    st = p.build_columns();
    if (st != BSMR_OK) return fail(st);
    *out = h;
    return BSMR_OK;
}

extern "C" int bsmr_plan_export_rows(const bsmr_plan* plan, bsmr_row_stage* hdr, uint32_t* rows) {
    if (!plan || !hdr) {
        set_error("bsmr_plan_export_rows: bad arguments");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    std::memset(hdr, 0, sizeof(*hdr));
    hdr->M = p.M;
    hdr->N = p.N;
    hdr->nnz = p.nnz;
    hdr->block_size = p.bs;
    hdr->num_blocks_per_row = p.nbpr;
    hdr->cluster_block_dim = p.B;
    hdr->num_zero_rows = p.z;
    hdr->num_reordered_rows = p.R;
    hdr->num_clusters = p.numClusters;
    hdr->alpha = p.alpha;
    hdr->row_reorder_ms = p.row_ms;
    hdr->exact_similarity_evals = p.exact_evals;
    hdr->total_similarity_evals = p.total_evals;
    if (rows && p.R) {
        BSMR_HIP(hipSetDevice(p.device));
        BSMR_HIP(hipMemcpyAsync(rows, p.rows.data(), static_cast<size_t>(p.R) * sizeof(u32),
                                hipMemcpyDefault, p.stream));
        BSMR_HIP(hipStreamSynchronize(p.stream));
    }
    return BSMR_OK;
}

extern "C" int bsmr_plan_import_rows(const uint32_t* rowptr, const uint32_t* colidx,
                                     const bsmr_row_stage* hdr, const uint32_t* rows,
                                     const bsmr_plan_options* opt, bsmr_plan** out) {
    *out = nullptr;
    if (!hdr || !valid_csr(rowptr, colidx, hdr->M, hdr->N, hdr->nnz) ||
        hdr->num_reordered_rows > hdr->M || hdr->num_zero_rows > hdr->M ||
        hdr->num_reordered_rows + hdr->num_zero_rows != hdr->M ||
        (hdr->num_reordered_rows && !rows)) {
        set_error("bsmr_plan_import_rows: invalid CSR or row-stage header");
        return BSMR_ERR_INVALID;
    }
    bsmr_plan_options o;
    if (opt)
        o = *opt;
    else
        bsmr_plan_options_default(&o);
    o.alpha = hdr->alpha;  // the row stage was built for this alpha; delta comes from opt
    auto* h = new bsmr_plan;
    Plan& p = h->p;
    auto fail = [&](int st) {
        delete h;
        return st;
    };
    const u32 M = hdr->M, R = hdr->num_reordered_rows;
    p.M = M;
    p.N = hdr->N;
    p.nnz = hdr->nnz;
    int st = init_plan(p, o);
    if (st != BSMR_OK) return fail(st);
    // the column-stage geometry must be the one bsmr_plan_create derives from (M, N, bs)
    // (rowReordering.cu:1035, 911-920); bs itself depends on the exporter's free memory
    if (hdr->block_size < 16 || hdr->block_size > 65535 ||
        hdr->num_blocks_per_row !=
            static_cast<u32>(std::ceil(static_cast<float>(hdr->N) / static_cast<float>(hdr->block_size))) ||
        hdr->cluster_block_dim != cluster_block_dim(hdr->num_blocks_per_row)) {
        set_error("bsmr_plan_import_rows: block_size / num_blocks_per_row / cluster_block_dim "
                  "inconsistent with N");
        return fail(BSMR_ERR_INVALID);
    }
    // the rows must be the non-empty rows of S, each once (they index rowptr on the device):
    // num_zero_rows equal to S's empty-row count, R distinct non-empty rows, R + z == M
    u32 empty = 0;
    for (u32 r = 0; r < M; ++r) empty += rowptr[r] == rowptr[r + 1];
    if (empty != hdr->num_zero_rows) {
        set_error("bsmr_plan_import_rows: num_zero_rows differs from the empty rows of S");
        return fail(BSMR_ERR_INVALID);
    }
    std::vector<u32> hrows(R);
    if (R && hipMemcpy(hrows.data(), rows, static_cast<size_t>(R) * sizeof(u32), hipMemcpyDefault) !=
                 hipSuccess) {
        set_error("bsmr_plan_import_rows: cannot read rows");
        return fail(BSMR_ERR_HIP);
    }
    std::vector<uint8_t> seen(M, 0);
    for (u32 r : hrows) {
        if (r >= M || seen[r] || rowptr[r] == rowptr[r + 1]) {
            set_error("bsmr_plan_import_rows: rows are not the non-empty rows of S, each once");
            return fail(BSMR_ERR_INVALID);
        }
        seen[r] = 1;
    }
    p.bs = hdr->block_size;
    p.nbpr = hdr->num_blocks_per_row;
    p.B = hdr->cluster_block_dim;
    p.keptMask = kept_warp_mask(p.B);
    p.z = hdr->num_zero_rows;
    p.R = R;
    p.P = (R + 15) / 16;
    p.numClusters = hdr->num_clusters;
    p.row_ms = hdr->row_reorder_ms;
    p.exact_evals = hdr->exact_similarity_evals;
    p.total_evals = hdr->total_similarity_evals;
    st = p.rowptr.upload(rowptr, M + 1ull, p.stream);
    if (st == BSMR_OK) st = p.colidx.upload(colidx, p.nnz, p.stream);
    if (st == BSMR_OK) st = p.rows.upload(hrows.data(), R, p.stream);  // R >= 1: nnz >= 2
    if (st == BSMR_OK) st = p.build_columns();
    if (st != BSMR_OK) return fail(st);
    *out = h;
    return BSMR_OK;
}

extern "C" int bsmr_plan_recolumn(bsmr_plan* plan, float delta) {
    if (!plan) return BSMR_ERR_INVALID;
    plan->p.delta = delta;
    return plan->p.build_columns();
}

extern "C" void bsmr_plan_destroy(bsmr_plan* plan) { delete plan; }

extern "C" int bsmr_plan_get_stats(const bsmr_plan* plan, bsmr_plan_stats* s) {
    if (!plan || !s) return BSMR_ERR_INVALID;
    const Plan& p = plan->p;
    std::memset(s, 0, sizeof(*s));
    s->M = p.M;
    s->N = p.N;
    s->nnz = p.nnz;
    s->block_size = p.bs;
    s->num_blocks_per_row = p.nbpr;
    s->cluster_block_dim = p.B;
    s->num_clusters = p.numClusters;
    s->num_row_panels = p.P;
    s->num_reordered_rows = p.R;
    s->num_dense_tiles = p.numDenseTiles;
    s->max_dense_tiles_per_panel = p.maxTilesPerPanel;
    s->num_residual = p.nres;
    s->num_dense_thread_blocks = p.numDenseTB;
    s->num_sparse_thread_blocks = p.numSparseTB;
    s->exact_similarity_evals = p.exact_evals;
    s->total_similarity_evals = p.total_evals;
    s->row_reorder_ms = p.row_ms;
    s->cluster_filter_used = p.filter_used ? 1u : 0u;
    s->cluster_filter_ms = p.filter_ms;
    s->col_reorder_ms = p.col_ms;
    s->dense_items = p.nDenseItems;
    s->residual_items = p.nResItems;
    for (int i = 0; i < Plan::N_RB_SIZES; ++i) {  // per row size: the fp32 layout, else the half one
        const Plan::RowBlockLayout& L = p.rbl[i].rowBytes ? p.rb_whole(i) : p.rb_whole(i + Plan::N_RB_SIZES);
        s->rb_rows[i] = L.rowBytes ? L.RB : 0;
        s->rb_items[i] = L.rowBytes ? L.nItems : 0;
        s->rb_pieces[i] = L.rowBytes ? L.nPieces : 0;
        s->rb_entries[i] = L.rowBytes ? L.nEntries : 0;
        s->rb_tiles[i] = L.rowBytes ? L.nTilesKept : 0;
        s->rb_work_items[i] = L.rowBytes ? L.nWorkItems : 0;
        if (L.rowBytes && L.orig) s->rb_orig_rows |= 1u << i;
        if (L.rowBytes && L.cols) s->rb_col_blocks |= 1u << i;
        if (L.rowBytes && rb_uses_pairs(p, L)) s->rb_pairs |= 1u << i;
        if (L.rowBytes && L.dynBatches) s->rb_batches |= 1u << i;
    }
    s->dense_sampled_tiles = p.dense.built ? p.dense.nonempty : 0;
    s->ptile_items = p.ptile.built ? p.ptile.nItems : 0;
    return BSMR_OK;
}

extern "C" int bsmr_plan_get_array(const bsmr_plan* plan, int which, uint32_t* host_out,
                                   uint64_t* len) {
    if (!plan) return BSMR_ERR_INVALID;
    const Plan& p = plan->p;
    const DevBuf<u32>* b = nullptr;
    size_t n = 0;
    switch (which) {
        case BSMR_ARR_REORDERED_ROWS: b = &p.rows; n = p.R; break;
        case BSMR_ARR_DENSE_COLS: b = &p.denseCols; n = p.denseCols.n; break;
        case BSMR_ARR_DENSE_COL_OFFSETS: b = &p.denseColOffsets; n = p.P + 1; break;
        case BSMR_ARR_SPARSE_COLS: b = &p.sparseCols; n = p.sparseCols.n; break;
        case BSMR_ARR_SPARSE_COL_OFFSETS: b = &p.sparseColOffsets; n = p.P + 1; break;
        case BSMR_ARR_SPARSE_VALUE_OFFSETS: b = &p.sparseValueOffsets; n = p.P + 1; break;
        case BSMR_ARR_BLOCK_OFFSETS: b = &p.blockOffsets; n = p.P + 1; break;
        case BSMR_ARR_BLOCK_VALUES: b = &p.blockValues; n = p.blockValues.n; break;
        case BSMR_ARR_SPARSE_VALUES: b = &p.sparseValues; n = p.nres; break;
        case BSMR_ARR_SPARSE_RELATIVE_ROWS: b = &p.sparseRel; n = p.nres; break;
        case BSMR_ARR_SPARSE_COL_INDICES: b = &p.sparseColIdx; n = p.nres; break;
        // (not kept by plans imported from a row stage: length 0)
        case BSMR_ARR_DISPERSION: b = &p.disp; n = p.disp.n ? p.M : 0; break;
        case BSMR_ARR_ASCENDING: b = &p.asc; n = p.asc.n ? p.M : 0; break;
        default:
            set_error("bsmr_plan_get_array: unknown array");
            return BSMR_ERR_INVALID;
    }
    if (len) *len = n;
    if (host_out && n) {
        BSMR_HIP(hipSetDevice(p.device));
        BSMR_HIP(hipMemcpy(host_out, b->data(), n * sizeof(u32), hipMemcpyDeviceToHost));
    }
    return BSMR_OK;
}

// evaluationReordering + calculateNumDenseBlocksAndAverageDensityInOriginalMatrix
// (BSMR.cpp:826-930, 955-994), evaluated on the host from the plan arrays (log statistics only;
// not on the timed path). Float accumulation order follows the reference loops.
extern "C" int bsmr_plan_evaluate(const bsmr_plan* plan, bsmr_eval_stats* out) {
    if (!plan || !out) return BSMR_ERR_INVALID;
    const Plan& p = plan->p;
    BSMR_HIP(hipSetDevice(p.device));
    std::vector<u32> rowptr, col, rows, dco, dcols, sco, scols;
    BSMR_CHECK(p.rowptr.download(rowptr, p.stream));
    BSMR_CHECK(p.colidx.download(col, p.stream));
    BSMR_CHECK(p.rows.download(rows, p.stream));
    BSMR_CHECK(p.denseColOffsets.download(dco, p.stream));
    BSMR_CHECK(p.denseCols.download(dcols, p.stream));
    BSMR_CHECK(p.sparseColOffsets.download(sco, p.stream));
    BSMR_CHECK(p.sparseCols.download(scols, p.stream));
    rows.resize(p.R);
    const u32 N = p.N;
    int numDense = 0, numSparseData = 0;
    float total = 0.f;
    std::vector<u32> blockOf(N + 1, NULLV);
    std::vector<char> isSparse(N + 1, 0);
    for (u32 q = 0; q < p.P; ++q) {
        const u32 d0 = dco[q], d1 = dco[q + 1], s0 = sco[q], s1 = sco[q + 1];
        const u32 nDB = (d1 - d0 + 15) / 16;
        for (u32 j = d0; j < d1; ++j) blockOf[dcols[j]] = (j - d0) / 16;
        for (u32 j = s0; j < s1; ++j) isSparse[scols[j]] = 1;
        std::vector<u32> cnt(nDB, 0);
        const u32 r1 = std::min(q * 16 + 16, p.R);
        for (u32 x = q * 16; x < r1; ++x)
            for (u32 k = rowptr[rows[x]]; k < rowptr[rows[x] + 1]; ++k) {
                if (blockOf[col[k]] != NULLV) ++cnt[blockOf[col[k]]];
                if (isSparse[col[k]]) ++numSparseData;
            }
        for (u32 b = 0; b < nDB; ++b)
            if (cnt[b] > 0) {
                const float density = static_cast<float>(cnt[b]) / 256.0f;
                total += density;
                if (density >= p.delta) ++numDense;
            }
        for (u32 j = d0; j < d1; ++j) blockOf[dcols[j]] = NULLV;
        for (u32 j = s0; j < s1; ++j) isSparse[scols[j]] = 0;
    }
    out->num_dense_block = numDense;
    const float avg = total / static_cast<float>(numDense);
    out->average_density = avg > 0 ? avg : 0.0f;
    out->num_sparse_data = numSparseData;
    out->num_dense_data = static_cast<int32_t>(p.nnz) - numSparseData;
    // original-order tiles
    const u32 OP = (p.M + 15) / 16;
    u32 onum = 0;
    float ototal = 0.f;
    std::vector<u32> cb;
    for (u32 q = 0; q < OP; ++q) {
        cb.clear();
        const u32 r0 = q * 16, r1 = std::min(r0 + 16, p.M);
        for (u32 r = r0; r < r1; ++r)
            for (u32 k = rowptr[r]; k < rowptr[r + 1]; ++k) cb.push_back(col[k] / 16);
        std::sort(cb.begin(), cb.end());
        for (size_t k = 0; k < cb.size();) {
            size_t j = k;
            while (j < cb.size() && cb[j] == cb[k]) ++j;
            const u32 c0 = cb[k] * 16, c1 = std::min(c0 + 16, N);
            const float bsz = static_cast<float>((r1 - r0) * (c1 - c0));
            const float density = static_cast<float>(j - k) / bsz;
            if (density >= p.delta) {
                ototal += density;
                ++onum;
            }
            k = j;
        }
    }
    out->original_num_dense_block = static_cast<int32_t>(onum);
    out->original_average_density = onum > 0 ? ototal / static_cast<float>(onum) : 0.0f;
    return BSMR_OK;
}

// Contiguous panel ranges balanced by a cost model: a dense tile costs 256*K MACs on the matrix
// core, priced at 1/4 of a residual MAC (fp32 MFMA vs. gathered scalar FMA); a residual entry
// costs K; every panel costs 1 (its A rows). cuts[0] = 0, cuts[world] = P, non-decreasing.
extern "C" int bsmr_shard_cuts(const uint32_t* blockOffsets, const uint32_t* sparseValueOffsets,
                               uint32_t P, uint32_t K, int world, uint32_t* cuts) {
    if (!blockOffsets || !sparseValueOffsets || !cuts || world <= 0) {
        set_error("bsmr_shard_cuts: bad arguments");
        return BSMR_ERR_INVALID;
    }
    std::vector<double> cum(P + 1ull, 0.0);
    for (u32 q = 0; q < P; ++q) {
        const double tiles = blockOffsets[q + 1] - blockOffsets[q];
        const double res = sparseValueOffsets[q + 1] - sparseValueOffsets[q];
        cum[q + 1] = cum[q] + tiles * 64.0 * K + res * K + 1.0;
    }
    cuts[0] = 0;
    for (int r = 1; r < world; ++r) {
        const double target = cum[P] * r / world;
        u32 c = static_cast<u32>(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        c = std::min(std::max(c, cuts[r - 1]), P);
        cuts[r] = c;
    }
    cuts[world] = P;
    return BSMR_OK;
}

extern "C" int bsmr_plan_shard(const bsmr_plan* plan, uint32_t K, int rank, int world,
                               uint32_t* p0, uint32_t* p1) {
    return bsmr_plan_shard_dtype(plan, K, BSMR_F32, rank, world, p0, p1);
}

namespace {
// cut [0, nRB) row blocks of cumulative cost cum (size nRB + 1) into `world` contiguous ranges,
// each cut at the row-block boundary closest to its target; cuts are panel indices
void cut_row_blocks(const std::vector<double>& cum, u32 nRB, u32 ppr, u32 P, int world, u32* cuts) {
    cuts[0] = 0;
    for (int r = 1; r < world; ++r) {
        const double target = cum[nRB] * r / world;
        u32 b = static_cast<u32>(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        if (b > 0 && target - cum[b - 1] < cum[std::min(b, nRB)] - target) --b;
        cuts[r] = std::max(cuts[r - 1], std::min(b * ppr, P));
    }
    cuts[world] = P;
}
}  // namespace

extern "C" int bsmr_cost_cuts(const double* block_cost, uint32_t nblocks, uint32_t panels_per_block,
                              uint32_t P, int world, const uint32_t* prev_cuts,
                              const float* shard_ms, uint32_t* cuts) {
    if ((!block_cost && nblocks) || world <= 0 || !cuts || panels_per_block == 0 ||
        (!prev_cuts) != (!shard_ms)) {
        set_error("bsmr_cost_cuts: bad arguments");
        return BSMR_ERR_INVALID;
    }
    const u32 nRB = nblocks, ppr = panels_per_block;
    std::vector<double> scale(nRB, 1.0);
    double norm = 1.0;
    if (prev_cuts) {
        if (prev_cuts[0] != 0 || prev_cuts[world] != P) {
            set_error("bsmr_plan_shard_rebalance: previous cuts must span [0, P]");
            return BSMR_ERR_INVALID;
        }
        // each block's model cost scaled by its shard's measured / predicted time
        std::vector<char> measured(nRB, 0);
        for (int r = 0; r < world; ++r) {
            if (prev_cuts[r + 1] < prev_cuts[r] || (prev_cuts[r] % ppr && prev_cuts[r] != P)) {
                set_error("bsmr_plan_shard_rebalance: previous cuts are not row-block boundaries");
                return BSMR_ERR_INVALID;
            }
            const u32 b0 = prev_cuts[r] / ppr, b1 = std::min(nRB, (prev_cuts[r + 1] + ppr - 1) / ppr);
            double pred = 0.0;
            for (u32 b = b0; b < b1; ++b) pred += block_cost[b];
            if (pred <= 0.0 || !(shard_ms[r] > 0.0f) || !std::isfinite(shard_ms[r])) continue;
            const double f = static_cast<double>(shard_ms[r]) / pred;
            for (u32 b = b0; b < b1; ++b) {
                scale[b] = f;
                measured[b] = 1;
            }
        }
        // normalise the factors of measured blocks to their mean; unmeasured blocks (a shard
        // whose time is 0 / NaN / inf) take the mean factor, i.e. keep their model cost
        double fs = 0.0;
        u32 nf = 0;
        for (u32 b = 0; b < nRB; ++b)
            if (measured[b]) {
                fs += scale[b];
                ++nf;
            }
        norm = nf ? fs / nf : 1.0;
        for (u32 b = 0; b < nRB; ++b)
            if (!measured[b]) scale[b] = norm;
    }
    std::vector<double> cum(nRB + 1ull, 0.0);
    for (u32 b = 0; b < nRB; ++b) cum[b + 1] = cum[b] + block_cost[b] * (scale[b] / norm);
    cut_row_blocks(cum, nRB, ppr, P, world, cuts);
    return BSMR_OK;
}

extern "C" int bsmr_plan_shard_rebalance(const bsmr_plan* plan, uint32_t K, int dtype, int world,
                                         const uint32_t* prev_cuts, const float* shard_ms,
                                         uint32_t* cuts) {
    if (!plan || world <= 0 || !prev_cuts || !shard_ms || !cuts || K == 0 || K % 16 ||
        (dtype != BSMR_F32 && dtype != BSMR_F16 && dtype != BSMR_BF16)) {
        set_error("bsmr_plan_shard_rebalance: bad arguments");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    const Plan::RowBlockLayout* L = nullptr;
    BSMR_CHECK(whole_rb_layout(p, K, dtype, &L, true));
    if (!L || L->nRB == 0 || L->orig) {
        set_error("bsmr_plan_shard_rebalance: needs the row-block launch of the reordered plan");
        return BSMR_ERR_UNSUPPORTED;
    }
    return bsmr_cost_cuts(L->rbCost.data(), L->nRB, L->RB / 16, p.P, world, prev_cuts, shard_ms, cuts);
}

extern "C" int bsmr_plan_shard_dtype(const bsmr_plan* plan, uint32_t K, int dtype, int rank,
                                     int world, uint32_t* p0, uint32_t* p1) {
    if (!plan || world <= 0 || rank < 0 || rank >= world || !p0 || !p1 || K == 0 || K % 16 ||
        (dtype != BSMR_F32 && dtype != BSMR_F16 && dtype != BSMR_BF16)) {
        set_error("bsmr_plan_shard: bad arguments");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    std::vector<u32> cuts(world + 1);
    // row-block launches: cut at row-block boundaries of the whole plan's layout by its measured
    // item costs (entries, column-run pieces, tiles, staged rows), so each shard's own layout has
    // the same row blocks; otherwise the per-panel model of bsmr_shard_cuts
    const Plan::RowBlockLayout* L = nullptr;
    BSMR_CHECK(whole_rb_layout(p, K, dtype, &L, true));
    if (L && L->nRB > 0 && !L->orig) {  // (original-order row blocks do not map to panels)
        BSMR_CHECK(bsmr_cost_cuts(L->rbCost.data(), L->nRB, L->RB / 16, p.P, world, nullptr, nullptr,
                                  cuts.data()));
    } else {
        BSMR_CHECK(bsmr_shard_cuts(p.h_blockOffsets.data(), p.h_sparseValueOffsets.data(), p.P, K,
                                   world, cuts.data()));
    }
    *p0 = cuts[rank];
    *p1 = cuts[rank + 1];
    return BSMR_OK;
}
