// plan_check.cpp — structural self-check of a BSMR plan and of the launch layout built from it.
//
// The reference runs check_rphm(matrix, bsmr, rphm, delta) under VALIDATE before checkSddmm
// (src/sddmm.cu:34-38): check_rowReordering (src/BSMR.cpp:444-486), check_colReordering
// (488-637) and check_rphm (639-824), driven by BSMR.cpp:932-953, each printing its own error
// line and then "Error! The <stage> is incorrect!" on stderr. bsmr_plan_check restates those
// checks on the host over the plan's device arrays, with the reference's messages, and makes them
// complete where the reference's are partial:
//   rows     every non-empty row of S exactly once, no empty row, none out of range;
//   columns  per panel: the dense and sparse column lists are the panel's distinct columns, each
//            once, in descending count order (ties in ascending column order: the stable sort of
//            colReordering.cu:333-336), padded with the sentinel column N to a multiple of 16
//            (colReordering.cu:338-343) and nowhere else, the dense prefix exactly the 16-column
//            groups with >= ceil(delta * 256) entries (colReordering.cu:244-271), and the sparse
//            data in (sparse column, panel row) order with the right count;
//   RPHM     every blockValues slot holds the CSR index of its (row, column) or NULL where that
//            entry is not stored / the row or column is padding; every sparse entry's CSR index
//            lies in its row and column; every stored entry in exactly one of blockValues /
//            sparseValues;
//   launch   (K > 0) the layout bsmr_sddmm runs for (K, dtype): every stored entry computed by
//            exactly one kept MFMA tile, column-run piece entry or residual slot, and each entry's
//            staged row, gathered column and output position agree with S.
// Deliberate difference: the reference's check_colReordering reports its own sentinel padding
// (column N, not a column of the panel) as an error (BSMR.cpp:547-550, 577-582); here the sentinel
// is accepted exactly where colReordering_cpu puts it. Not on any timed path.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "plan.hpp"

namespace bsmr {

bool sddmm_uses_dense(const Plan& p, u32 K, int dtype);  // sddmm.hip
bool sddmm_uses_ptile(const Plan& p, u32 K, int dtype);  // sddmm.hip

namespace {

constexpr u32 CM22 = (1u << 22) - 1;

std::string fmt(const char* f, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, f);
    std::vsnprintf(buf, sizeof(buf), f, ap);
    va_end(ap);
    return buf;
}

// the first failure of a parallel pass: the lowest index wins, so the report does not depend on
// the thread split
struct FirstErr {
    std::mutex mu;
    std::atomic<u64> idx{~0ull};
    std::string msg;
    void put(u64 i, std::string m) {
        std::lock_guard<std::mutex> g(mu);
        if (i < idx.load()) {
            idx.store(i);
            msg = std::move(m);
        }
    }
    bool any() const { return idx.load() != ~0ull; }
};

// f(begin, end) over [0, n) on up to 16 host threads
template <class F>
void par_range(size_t n, F&& f) {
    const unsigned T = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (n < 4096 || T == 1) {
        f(size_t{0}, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t chunk = (n + T - 1) / T;
    for (unsigned t = 0; t < T; ++t) {
        const size_t a = t * chunk, b = std::min(n, a + chunk);
        if (a < b) th.emplace_back([&f, a, b]() { f(a, b); });
    }
    for (auto& x : th) x.join();
}

inline u32 bump(uint8_t* c) { return __atomic_fetch_add(c, uint8_t{1}, __ATOMIC_RELAXED); }

struct Host {
    u32 M = 0, N = 0, nnz = 0, R = 0, P = 0;
    std::vector<u32> rowptr, col, rows, dcols, dco, scols, sco, svo, bo, bv, sval, srel, scol;
};

class Checker {
public:
    // p: the plan (device arrays, launch layouts); null for a check of host arrays (h())
    Checker(const Plan* p, float delta, int verbose) : pp_(p), delta_(delta), verbose_(verbose) {}

    Host& h() { return h_; }

    int load() {
        const Plan& p_ = *pp_;
        Host& h = h_;
        h.M = p_.M;
        h.N = p_.N;
        h.nnz = p_.nnz;
        h.R = p_.R;
        h.P = p_.P;
        hipStream_t s = p_.stream;
        BSMR_CHECK(p_.rowptr.download(h.rowptr, s));
        BSMR_CHECK(p_.colidx.download(h.col, s));
        BSMR_CHECK(p_.rows.download(h.rows, s));
        BSMR_CHECK(p_.denseCols.download(h.dcols, s));
        BSMR_CHECK(p_.denseColOffsets.download(h.dco, s));
        BSMR_CHECK(p_.sparseCols.download(h.scols, s));
        BSMR_CHECK(p_.sparseColOffsets.download(h.sco, s));
        BSMR_CHECK(p_.sparseValueOffsets.download(h.svo, s));
        BSMR_CHECK(p_.blockOffsets.download(h.bo, s));
        BSMR_CHECK(p_.blockValues.download(h.bv, s));
        BSMR_CHECK(p_.sparseValues.download(h.sval, s));
        BSMR_CHECK(p_.sparseRel.download(h.srel, s));
        BSMR_CHECK(p_.sparseColIdx.download(h.scol, s));
        h.rows.resize(std::min<size_t>(h.rows.size(), h.R));
        h.dcols.resize(std::min<size_t>(h.dcols.size(), p_.denseCols.n));
        h.scols.resize(std::min<size_t>(h.scols.size(), p_.sparseCols.n));
        h.sval.resize(std::min<size_t>(h.sval.size(), p_.nres));
        h.srel.resize(std::min<size_t>(h.srel.size(), p_.nres));
        h.scol.resize(std::min<size_t>(h.scol.size(), p_.nres));
        return BSMR_OK;
    }

    // check_rowReordering (BSMR.cpp:444-486)
    bool rows() {
        const Host& h = h_;
        if (h.rows.size() != h.R) return fail(fmt("Error! reorderedRows holds %zu rows, expected %u",
                                                  h.rows.size(), h.R));
        for (u32 q = 0; q < h.R; ++q)
            if (h.rows[q] >= h.M) return fail(fmt("Error! Row is out of range! Row: %u", h.rows[q]));
        rowsInRange_ = true;
        std::vector<u32> at(h.M, NULLV);
        for (u32 q = 0; q < h.R; ++q) {
            const u32 r = h.rows[q];
            if (at[r] != NULLV) return fail(fmt("Error! Row is duplicated! Duplicated row: %u", r));
            at[r] = q;
        }
        for (u32 r = 0; r < h.M; ++r) {
            const bool empty = h.rowptr[r + 1] == h.rowptr[r];
            if (empty && at[r] != NULLV) return fail(fmt("Error! Empty row is stored! Row: %u", r));
            if (!empty && at[r] == NULLV) return fail(fmt("Error! Row is missing! Row: %u", r));
        }
        rowsOk_ = true;
        return true;
    }

    // check_colReordering (BSMR.cpp:488-637), completed (see the file header)
    bool columns() {
        const Host& h = h_;
        const u32 P = h.P, N = h.N;
        if (!rowsInRange_) return fail("Error! The columns cannot be checked: reorderedRows holds rows outside S");
        if (h.dco.size() < P + 1 || h.sco.size() < P + 1 || h.svo.size() < P + 1 || h.dco[0] ||
            h.sco[0] || h.svo[0] || h.dco[P] != h.dcols.size() || h.sco[P] != h.scols.size() ||
            h.svo[P] != h.sval.size())
            return fail("Error! The column offsets of the row panels are incorrect!");
        for (u32 q = 0; q < P; ++q)
            if (h.dco[q + 1] < h.dco[q] || h.sco[q + 1] < h.sco[q] || h.svo[q + 1] < h.svo[q])
                return fail(fmt("Error! The column offsets of the row panels are incorrect! rowPanelId: %u", q));
        if (P != (h.R + 15) / 16) return fail(fmt("Error! The number of row panels is incorrect: %u", P));
        const u32 thr = static_cast<u32>(std::ceil(delta_ * 256.0f));
        FirstErr fe;
        par_range(P, [&](size_t q0, size_t q1) {
            std::vector<u32> cnt(N + 1, 0), rank(N + 1, NULLV);
            std::vector<uint8_t> flag(N + 1, 0);
            std::vector<u32> touched, list;
            for (u32 q = static_cast<u32>(q0); q < q1 && q < fe.idx; ++q) {
                std::string err = panel(q, thr, cnt, rank, flag, touched, list);
                for (u32 c : touched) {
                    cnt[c] = 0;
                    flag[c] = 0;
                }
                for (u32 c : list) rank[c] = NULLV;
                touched.clear();
                list.clear();
                if (!err.empty()) fe.put(q, std::move(err));
            }
        });
        if (fe.any()) return fail(fe.msg);
        colsOk_ = true;
        return true;
    }

    // check_rphm (BSMR.cpp:639-824), completed (see the file header)
    bool rphm() {
        const Host& h = h_;
        const u32 P = h.P, N = h.N;
        if (h.bo.size() < P + 1 || h.bo[0] != 0)
            return fail("Error! The number of blocks in the row panel is incorrect! rowPanelId: 0");
        for (u32 q = 0; q < P; ++q) {
            const u32 nb = h.bo[q + 1] - h.bo[q];
            if (h.bo[q + 1] < h.bo[q] || (colsOk_ && nb * 16 != h.dco[q + 1] - h.dco[q]))
                return fail(fmt("Error! The number of blocks in the row panel is incorrect! rowPanelId: %u", q));
        }
        if (h.bv.size() != static_cast<size_t>(h.bo[P]) * TILE)
            return fail(fmt("Error! blockValues holds %zu values, expected %llu", h.bv.size(),
                            static_cast<unsigned long long>(h.bo[P]) * TILE));
        if (!rowsOk_ || !colsOk_) return fail("Error! The rphm cannot be checked without a valid row and column reordering");
        // every slot of every tile against S (by position)
        FirstErr fe;
        par_range(P, [&](size_t q0, size_t q1) {
            std::vector<u32> posOf(N + 1, NULLV);
            for (u32 q = static_cast<u32>(q0); q < q1 && q < fe.idx; ++q) {
                const u32 nt = h.bo[q + 1] - h.bo[q];
                for (u32 lr = 0; lr < 16 && nt; ++lr) {
                    const u32 x = q * 16 + lr;
                    const u32 row = x < h.R ? h.rows[x] : NULLV;
                    if (row != NULLV)
                        for (u32 k = h.rowptr[row]; k < h.rowptr[row + 1]; ++k) posOf[h.col[k]] = k;
                    std::string err;
                    for (u32 j = 0; j < nt && err.empty(); ++j)
                        for (u32 lc = 0; lc < 16; ++lc) {
                            const u32 c = h.dcols[h.dco[q] + 16 * j + lc];
                            const u64 idx = static_cast<u64>(h.bo[q] + j) * TILE + lr * 16 + lc;
                            const u32 v = h.bv[idx];
                            const u32 want = row != NULLV && c < N ? posOf[c] : NULLV;
                            if (v == want) continue;
                            if (row == NULLV || c >= N)
                                err = fmt("Error! The value is incorrect!(Check based on the blockValues) idxOfBlockValues: %llu",
                                          static_cast<unsigned long long>(idx));
                            else if (v == NULLV)
                                err = fmt("Error! Missing value!(Check based on the blockValues) row: %u, col: %u, "
                                          "idxOfBlockValues: %llu, idxOfOriginalMatrix: %u",
                                          row, c, static_cast<unsigned long long>(idx), want);
                            else if (want == NULLV)
                                err = fmt("Error! A non-existent value appeared in blockValues! idxOfBlockValues: %llu",
                                          static_cast<unsigned long long>(idx));
                            else
                                err = fmt("Error! The block value is incorrect!(Check based on the blockValues) row: %u, "
                                          "col: %u, idxOfBlockValues: %llu, idxOfOriginalMatrix: %u",
                                          row, c, static_cast<unsigned long long>(idx), want);
                            break;
                        }
                    if (row != NULLV)
                        for (u32 k = h.rowptr[row]; k < h.rowptr[row + 1]; ++k) posOf[h.col[k]] = NULLV;
                    if (!err.empty()) {
                        fe.put(q, std::move(err));
                        break;
                    }
                }
                // the panel's sparse entries: CSR index in its row, at its column
                for (u32 i = h.svo[q]; i < h.svo[q + 1]; ++i) {
                    const u32 row = h.rows[q * 16 + h.srel[i]];  // srel checked by columns()
                    const u32 v = h.sval[i];
                    if (v < h.rowptr[row] || v >= h.rowptr[row + 1] || h.col[v] != h.scol[i]) {
                        fe.put(q, fmt("Error! The sparse value is incorrect! rowPanelId: %u, sparseValues[%u]: %u", q, i, v));
                        break;
                    }
                }
            }
        });
        if (fe.any()) return fail(fe.msg);
        // every stored entry in exactly one of blockValues / sparseValues
        std::vector<uint8_t> hit(h.nnz, 0);
        for (size_t i = 0; i < h.bv.size(); ++i) {
            const u32 v = h.bv[i];
            if (v == NULLV) continue;
            if (v >= h.nnz || hit[v]) return fail(fmt("Error! The block value is duplicated! val: %u", v));
            hit[v] = 1;
        }
        for (size_t i = 0; i < h.sval.size(); ++i) {
            const u32 v = h.sval[i];
            if (v >= h.nnz || hit[v] == 2)
                return fail(fmt("Error! The original matrix index is duplicated in sparseValues! originalMatrixIndex: %u, "
                                "sparseValues[%zu]", v, i));
            if (hit[v] == 1)
                return fail(fmt("Error! The original matrix index is in both blockValues and sparseValues! "
                                "originalMatrixIndex: %u, sparseValues[%zu]", v, i));
            hit[v] = 2;
        }
        for (u32 k = 0; k < h.nnz; ++k)
            if (!hit[k])
                return fail(fmt("Error! The original matrix index is in neither blockValues nor sparseValues! "
                                "originalMatrixIndex: %u", k));
        return true;
    }

    // the launch layout bsmr_sddmm runs for (K, dtype)
    int layout(u32 K, int dtype, bool* ok) {
        const Plan& p_ = *pp_;
        *ok = true;
        if (!rowsOk_) {
            *ok = fail("Error! The launch layout cannot be checked without a valid row reordering");
            return BSMR_OK;
        }
        if (sddmm_uses_dense(p_, K, dtype)) {
            {
                std::lock_guard<std::mutex> g(p_.layout_mu);
                if (!p_.dense.built) BSMR_CHECK(p_.build_dense_layout());
            }
            *ok = dense_layout();
            return BSMR_OK;
        }
        if (sddmm_uses_ptile(p_, K, dtype)) {
            {
                std::lock_guard<std::mutex> g(p_.layout_mu);
                if (!p_.ptile.built || p_.ptile.tpi != p_.ptile_tpi) BSMR_CHECK(p_.build_ptile_layout(p_.ptile_tpi));
            }
            bool r = false;
            BSMR_CHECK(ptile_layout(&r));
            *ok = r;
            return BSMR_OK;
        }
        const Plan::RowBlockLayout* L = nullptr;
        BSMR_CHECK(whole_rb_layout(p_, K, dtype, &L));
        if (L) {
            bool r = false;
            BSMR_CHECK(rb_layout(*L, &r));
            *ok = r;
            return BSMR_OK;
        }
        bool r = false;
        BSMR_CHECK(cm_layout(&r));
        *ok = r;
        return BSMR_OK;
    }

    const std::string& first() const { return first_; }

private:
    bool fail(const std::string& msg) {
        if (verbose_) std::fprintf(stderr, "%s\n", msg.c_str());
        if (first_.empty()) first_ = msg;
        return false;
    }

    // one panel of columns(); "" = correct
    std::string panel(u32 q, u32 thr, std::vector<u32>& cnt, std::vector<u32>& rank,
                      std::vector<uint8_t>& flag, std::vector<u32>& touched, std::vector<u32>& list) {
        const Host& h = h_;
        const u32 N = h.N;
        const u32 x0 = q * 16, x1 = std::min(x0 + 16, h.R);
        for (u32 x = x0; x < x1; ++x) {
            const u32 r = h.rows[x];
            for (u32 k = h.rowptr[r]; k < h.rowptr[r + 1]; ++k)
                if (cnt[h.col[k]]++ == 0) touched.push_back(h.col[k]);
        }
        const u32 d0 = h.dco[q], d1 = h.dco[q + 1], s0 = h.sco[q], s1 = h.sco[q + 1];
        if ((d1 - d0) % 16)
            return fmt("Error! The number of dense columns in the row panel is not a multiple of 16! rowPanelId: %u", q);
        // the whole list: dense prefix then sparse rest
        u32 real = 0, pad = 0;
        for (u32 j = d0; j < d1; ++j) {
            const u32 c = h.dcols[j];
            if (c == N) {
                ++pad;
                continue;
            }
            if (c > N || pad) return fmt("Error! Column indexes in the row panel is incorrect! rowPanelId: %u", q);
            if (flag[c]) return "Error! Column indexes are duplicated";
            if (!cnt[c]) return fmt("Error! Column indexes in the row panel is incorrect! rowPanelId: %u", q);
            flag[c] = 1;
            rank[c] = static_cast<u32>(list.size());
            list.push_back(c);
            ++real;
        }
        for (u32 j = s0; j < s1; ++j) {
            const u32 c = h.scols[j];
            if (c == N) {
                ++pad;
                continue;
            }
            if (c > N || pad)
                return fmt("Error! Column index not in current row panel! rowPanelId: %u, col: %u", q, c);
            if (flag[c] == 2) return "Error! Column indexes are duplicated";
            if (flag[c] == 1)
                return fmt(" Error! Dense column index is also in sparse column segment! rowPanelId: %u, denseCol: %u", q, c);
            if (!cnt[c]) return fmt("Error! Column index not in current row panel! rowPanelId: %u, col: %u", q, c);
            flag[c] = 2;
            rank[c] = static_cast<u32>(list.size());
            list.push_back(c);
            ++real;
        }
        if (real != touched.size())
            return fmt("Error! The number of column indexes in the row panel is incorrect! Row panel : %u", q);
        const u32 total = (d1 - d0) + (s1 - s0);
        if (total % 16 || total - real >= 16)
            return fmt("Error! The sentinel padding of the row panel's column list is incorrect! rowPanelId: %u", q);
        for (size_t i = 1; i < list.size(); ++i) {
            const u32 a = list[i - 1], b = list[i];
            if (cnt[a] < cnt[b] || (cnt[a] == cnt[b] && a > b))
                return fmt("Error! The order of column indexes in the row panel is incorrect! rowPanelId: %u", q);
        }
        // the dense prefix = the 16-column groups reaching thr (colReordering.cu:244-271)
        const u32 nd = (d1 - d0) / 16;
        for (u32 g = 0; g * 16 < total; ++g) {
            u32 sum = 0;
            for (u32 t = g * 16; t < g * 16 + 16 && t < list.size(); ++t) sum += cnt[list[t]];
            if ((g < nd) != (sum >= thr))
                return fmt("Error! The dense column segment does not match delta! rowPanelId: %u, group: %u", q, g);
            if (g >= nd) break;  // sums are non-increasing: the first sparse group decides
        }
        // sparse data: count, then (sparse column, panel row) order of BSMR.cpp:177-219
        u64 want = 0;
        for (size_t i = 0; i < list.size(); ++i)
            if (flag[list[i]] == 2) want += cnt[list[i]];
        const u32 v0 = h.svo[q], v1 = h.svo[q + 1];
        if (v1 - v0 != want)
            return fmt("Error! The number of sparse data in the row panel is incorrect! rowPanelId: %u", q);
        u64 prev = 0;
        for (u32 i = v0; i < v1; ++i) {
            const u32 rel = h.srel[i], c = h.scol[i];
            if (rel >= 16 || x0 + rel >= x1)
                return fmt("Error! Row not in current row panel! rowPanelId: %u, sparseValues[%u]", q, i);
            if (c >= N || flag[c] != 2)
                return fmt("Error! Column not in current row panel! rowPanelId: %u, sparseValues[%u]", q, i);
            const u64 key = (static_cast<u64>(rank[c]) << 5 | rel) + 1;
            if (key <= prev)
                return fmt("Error! The order of sparse data in the row panel is incorrect! rowPanelId: %u, sparseValues[%u]", q, i);
            prev = key;
        }
        return std::string();
    }

    // an entry (row, column, output position) against S
    bool entry_ok(u32 row, u32 c, u32 pos) const {
        return row < h_.M && pos < h_.nnz && pos >= h_.rowptr[row] && pos < h_.rowptr[row + 1] &&
               h_.col[pos] == c;
    }

    // every stored entry hit exactly once (tiles + entries); "" = correct
    std::string coverage(const std::vector<uint8_t>& hit) const {
        for (u32 k = 0; k < h_.nnz; ++k)
            if (hit[k] != 1)
                return fmt("stored entry %u (row of CSR position) computed %u times", k, static_cast<u32>(hit[k]));
        return std::string();
    }

    bool layout_fail(const std::string& what) {
        fail("Error! The launch layout is incorrect! " + what);
        return false;
    }

    bool dense_layout() {
        const Plan& p_ = *pp_;
        const Plan::DenseLayout& D = p_.dense;
        std::vector<u32> off, loc, out;
        if (D.off.download(off, p_.stream) || D.loc.download(loc, p_.stream) || D.out.download(out, p_.stream))
            return layout_fail("(dense-sampled lists unreadable)");
        const u32 T = 128;
        if (off.size() != static_cast<size_t>(D.ntiles) + 1 || off[0] != 0 || off[D.ntiles] != h_.nnz)
            return layout_fail("dense-sampled tile offsets");
        std::vector<uint8_t> hit(h_.nnz, 0);
        for (u32 t = 0; t < D.ntiles; ++t) {
            const u32 ti = t / D.ntn, tj = t % D.ntn;
            for (u32 k = off[t]; k < off[t + 1]; ++k) {
                const u32 row = ti * T + (loc[k] >> 7), c = tj * T + (loc[k] & 127u);
                if (!entry_ok(row, c, out[k]))
                    return layout_fail(fmt("dense-sampled tile %u entry %u: row %u col %u -> position %u", t, k, row, c, out[k]));
                if (hit[out[k]]++) return layout_fail(fmt("dense-sampled position %u written twice", out[k]));
            }
        }
        const std::string e = coverage(hit);
        return e.empty() ? true : layout_fail(e);
    }

    // kept / all MFMA tiles: a tile id's stored entries into hit; "" = correct
    std::string tile_hits(u32 g, std::vector<uint8_t>& hit) const {
        if (static_cast<u64>(g) * TILE >= h_.bv.size()) return fmt("tile id %u out of range", g);
        for (u32 i = 0; i < TILE; ++i) {
            const u32 v = h_.bv[static_cast<size_t>(g) * TILE + i];
            if (v == NULLV) continue;
            if (v >= h_.nnz) return fmt("tile %u value %u", g, v);
            if (bump(&hit[v])) return fmt("position %u computed twice (tile %u)", v, g);
        }
        return std::string();
    }

    int rb_layout(const Plan::RowBlockLayout& L, bool* ok) {
        hipStream_t s = pp_->stream;
        std::vector<uint4> items;
        std::vector<u32> iend, meta, out, tileIds, sortedPos, rowIds;
        std::vector<uint2> pieces, itemEnt, runs, itemRuns;
        BSMR_CHECK(L.items.download(items, s));
        BSMR_CHECK(L.itemEnd.download(iend, s));
        BSMR_CHECK(L.pieces.download(pieces, s));
        BSMR_CHECK(L.meta.download(meta, s));
        BSMR_CHECK(L.tileIds.download(tileIds, s));
        if (L.out.size()) BSMR_CHECK(L.out.download(out, s));
        if (L.sortedPos.size()) BSMR_CHECK(L.sortedPos.download(sortedPos, s));
        if (L.itemEnt.size()) BSMR_CHECK(L.itemEnt.download(itemEnt, s));
        if (L.outRuns) {
            BSMR_CHECK(L.runs.download(runs, s));
            BSMR_CHECK(L.itemRuns.download(itemRuns, s));
        }
        if (L.orig || L.cols) BSMR_CHECK(L.rowIds.download(rowIds, s));
        items.resize(L.nItems);
        iend.resize(L.nItems);
        pieces.resize(L.nPieces);
        tileIds.resize(L.nTilesKept);
        const bool staged = L.outLds != 0;
        const u32 nE = L.nEntries;
        *ok = false;
        if (meta.size() < nE) return layout_fail("entry metadata shorter than the entries"), BSMR_OK;
        if (staged && itemEnt.size() < L.nItems) return layout_fail("staged item table"), BSMR_OK;
        if (staged && !L.outRuns && sortedPos.size() < nE) return layout_fail("staged positions"), BSMR_OK;
        if (!staged && !L.outPacked && out.size() < nE) return layout_fail("output positions"), BSMR_OK;
        const u32 nRB = L.nRB, RB = L.RB;
        const u32 qbase = (L.orig || L.cols) ? 0 : 16 * L.pa;
        // column blocks: the image rows are S's columns (identity over N) and a piece's
        // "column" is a row of S; every check below then runs on (row, column) swapped back
        const u32 nStream = L.cols ? h_.M : h_.N;
        if ((L.orig || L.cols) && rowIds.size() < L.rowEnd)
            return layout_fail("original-order row list shorter than the staged rows"), BSMR_OK;
        {
            // the workgroup's LDS (launch_rb: 160 KiB at 1024 threads, 80 KiB at 512) holds the
            // image and, for staged output, the largest item's result slots past it; rows of
            // <= 512 B keep the last 16 bytes for the piece-batch counter
            const u64 dyn = (L.NT == 1024 ? 160u : 80u) * 1024u, img = static_cast<u64>(RB) * L.rowBytes;
            u64 maxEnt = 0;
            if (staged)
                for (u32 i = 0; i < L.nItems; ++i) maxEnt = std::max<u64>(maxEnt, itemEnt[i].y);
            const u64 used = (staged ? std::max<u64>(L.outLds, img) + 4 * maxEnt : img) +
                             (L.rowBytes <= 512 ? 16u : 0u);
            if (used > dyn || (staged && L.outLds < img))
                return layout_fail(fmt("LDS layout: image %llu B, %llu result slots at %u, %llu B per workgroup",
                                       static_cast<unsigned long long>(img),
                                       static_cast<unsigned long long>(maxEnt), L.outLds,
                                       static_cast<unsigned long long>(dyn))),
                       BSMR_OK;
        }
        std::vector<uint8_t> hit(h_.nnz, 0), ehit(std::max<u32>(nE, 1), 0), thit(std::max<size_t>(h_.bv.size() / TILE, 1), 0);
        FirstErr fe;
        par_range(L.nItems, [&](size_t i0, size_t i1) {
            std::vector<u32> slotPos;
            for (size_t i = i0; i < i1 && i < fe.idx; ++i) {
                const uint4 it = items[i];
                const u32 pw = it.w, pe = iend[i];
                if (pe < pw || pe > L.nPieces || it.z < it.y || it.z > L.nTilesKept) {
                    fe.put(i, fmt("item %zu: piece range [%u, %u) / tile range [%u, %u)", i, pw, pe, it.y, it.z));
                    break;
                }
                if (pw == pe && it.y == it.z) continue;  // padding
                if (it.x >= nRB) {
                    fe.put(i, fmt("item %zu: row block %u of %u", i, it.x, nRB));
                    break;
                }
                const u64 base = qbase + static_cast<u64>(it.x) * RB;
                std::string err;
                // kept tiles: in the item's row block
                for (u32 t = it.y; t < it.z && err.empty(); ++t) {
                    const u32 g = tileIds[t];
                    if (g >= thit.size()) {
                        err = fmt("item %zu: tile id %u", i, g);
                        break;
                    }
                    const u32 q = static_cast<u32>(std::upper_bound(h_.bo.begin(), h_.bo.begin() + h_.P + 1, g) - h_.bo.begin()) - 1;
                    if (16ull * q < base || 16ull * q >= base + RB) err = fmt("item %zu: tile %u (panel %u) outside row block %u", i, g, q, it.x);
                    else if (bump(&thit[g])) err = fmt("item %zu: tile %u run twice", i, g);
                    else err = tile_hits(g, hit);
                }
                // staged: slot -> CSR position of this item
                u32 ea = 0, ne = 0;
                if (staged) {
                    ea = itemEnt[i].x;
                    ne = itemEnt[i].y;
                    if (static_cast<u64>(ea) + ne > nE) err = fmt("item %zu: staged entries [%u, +%u)", i, ea, ne);
                    slotPos.assign(ne, NULLV);
                    if (err.empty() && L.outRuns) {
                        const uint2 ir = itemRuns[i];
                        for (u32 r = ir.x; r < ir.x + ir.y && err.empty(); ++r) {
                            const u32 first = runs[r].y & 0xFFFFu, len = runs[r].y >> 16;
                            for (u32 t = 0; t < len; ++t) {
                                if (first + t >= ne || slotPos[first + t] != NULLV) {
                                    err = fmt("item %zu: run %u slots", i, r);
                                    break;
                                }
                                slotPos[first + t] = runs[r].x + t;
                            }
                        }
                    } else if (err.empty()) {
                        for (u32 t = 0; t < ne; ++t) slotPos[t] = sortedPos[ea + t];
                    }
                }
                u32 seen = 0;
                for (u32 k = pw; k < pe && err.empty(); ++k) {
                    const u32 e0 = pieces[k].x, c = pieces[k].y & CM22, len = (pieces[k].y >> 22) + 1;
                    if (static_cast<u64>(e0) + len > nE || c >= nStream ||
                        (staged && (e0 < ea || e0 + len > ea + ne))) {
                        err = fmt("item %zu piece %u: entries [%u, +%u) column %u", i, k, e0, len, c);
                        break;
                    }
                    for (u32 e = e0; e < e0 + len; ++e) {
                        const u32 m = meta[e], lr = m >> 22;
                        if (lr >= RB || base + lr >= (L.orig ? h_.M : L.rowEnd)) {
                            err = fmt("item %zu entry %u: local row %u", i, e, lr);
                            break;
                        }
                        const u32 img = (L.orig || L.cols) ? rowIds[base + lr] : h_.rows[base + lr];
                        u32 pos;
                        if (staged) {
                            const u32 slot = m & CM22;
                            pos = slot < ne ? slotPos[slot] : NULLV;
                        } else if (L.outPacked) {
                            pos = m & CM22;
                        } else {
                            if ((m & CM22) != c) {
                                err = fmt("item %zu entry %u: column %u in a piece of column %u", i, e, m & CM22, c);
                                break;
                            }
                            pos = out[e];
                        }
                        const u32 row = L.cols ? c : img, col = L.cols ? img : c;
                        if (!entry_ok(row, col, pos)) {
                            err = fmt("item %zu entry %u: row %u col %u -> position %u", i, e, row, col, pos);
                            break;
                        }
                        if (bump(&ehit[e])) {
                            err = fmt("item %zu entry %u in two pieces", i, e);
                            break;
                        }
                        if (bump(&hit[pos])) {
                            err = fmt("item %zu entry %u: position %u computed twice", i, e, pos);
                            break;
                        }
                        ++seen;
                    }
                }
                if (err.empty() && staged && seen != ne) err = fmt("item %zu: %u entries in pieces, %u slots", i, seen, ne);
                if (!err.empty()) fe.put(i, std::move(err));
            }
        });
        if (fe.any()) return layout_fail(fe.msg), BSMR_OK;
        for (u32 e = 0; e < nE; ++e)
            if (ehit[e] != 1) return layout_fail(fmt("entry %u in no piece", e)), BSMR_OK;
        for (u32 t = 0; t < L.nTilesKept; ++t)
            if (thit[tileIds[t]] != 1) return layout_fail(fmt("kept tile %u in no item", tileIds[t])), BSMR_OK;
        const std::string e = coverage(hit);
        if (!e.empty()) return layout_fail(e), BSMR_OK;
        *ok = true;
        return BSMR_OK;
    }

    // column-major launch (k_sddmm_f32 / k_sddmm_half): every tile + residual slots
    // the panel-grouped tile launch: every tile id in exactly one item; an item's tiles are one
    // contiguous run inside its first panel, or inside its first and second panel with no tile of
    // a third between them (its A rows are those panels' 16 reordered rows each), at most tpi
    // tiles of one panel when tpi > 0; the descriptors the kernel reads agree; then the residual
    // slots as in the column-major launch
    int ptile_layout(bool* ok) {
        const Plan& p_ = *pp_;
        const Plan::PtileLayout& PL = p_.ptile;
        std::vector<uint4> items;
        BSMR_CHECK(PL.items.download(items, p_.stream));
        items.resize(PL.nItems);
        std::vector<u32> desc;
        BSMR_CHECK(PL.desc.download(desc, p_.stream));
        *ok = false;
        const u32 nt = static_cast<u32>(h_.bv.size() / TILE), ds = PL.stride;
        std::vector<uint8_t> thit(std::max<u32>(nt, 1), 0);
        if (PL.nItems % XCD_BUCKETS)
            return layout_fail(fmt("panel-tile launch: %u item slots, not a multiple of 8", PL.nItems)), BSMR_OK;
        if (desc.size() < static_cast<size_t>(PL.nItems) * ds || ds < 48)
            return layout_fail("panel-tile descriptors missing"), BSMR_OK;
        for (u32 i = 0; i < PL.nItems; ++i) {
            const uint4 it = items[i];
            const u32* d = desc.data() + static_cast<size_t>(i) * ds;
            if (it.z == 0) {
                if (d[33] != 0) return layout_fail(fmt("panel-tile descriptor %u: tiles in a padding slot", i)), BSMR_OK;
                continue;
            }
            const u32 q0 = it.x, two = it.w != 0, q1 = two ? it.w - 1 : q0;
            const u32 t0 = it.y, t1 = it.y + it.z;
            const bool inside = q0 < h_.P && q1 < h_.P && t0 >= h_.bo[q0] &&
                                (two ? q1 > q0 && h_.bo[q0 + 1] == h_.bo[q1] && t0 < h_.bo[q0 + 1] &&
                                           t1 > h_.bo[q1] && t1 <= h_.bo[q1 + 1]
                                     : t1 <= h_.bo[q0 + 1]);
            if (!inside || (PL.tpi > 0 && (two || it.z > PL.tpi)) || 48 + 16 * it.z > ds)
                return layout_fail(fmt("panel-tile item %u {panels %u..%u, tiles [%u, %u)} outside its panels", i, q0, q1, t0, t1)), BSMR_OK;
            for (u32 t = t0; t < t1; ++t)
                if (thit[t]++) return layout_fail(fmt("panel-tile: tile %u in two items", t)), BSMR_OK;
            // the descriptor
            const u32 n0 = two ? h_.bo[q0 + 1] - t0 : it.z;
            if (d[32] != t0 || d[33] != it.z || d[34] != n0 || d[35] != (two ? 2u : 1u))
                return layout_fail(fmt("panel-tile descriptor %u: tiles [%u, +%u) split %u panels %u for item [%u, +%u)", i, d[32], d[33], d[34], d[35], t0, it.z)), BSMR_OK;
            for (u32 r = 0; r < 32; ++r) {
                const u32 x = 16 * (r < 16 ? q0 : q1) + (r & 15), want = x < h_.R ? h_.rows[x] : h_.rows[0];
                if (d[r] != want)
                    return layout_fail(fmt("panel-tile descriptor %u: row %u is %u, panel row %u", i, r, d[r], want)), BSMR_OK;
            }
            for (u32 j = 0; j < it.z; ++j)
                for (u32 c = 0; c < 16; ++c)
                    if (d[48 + 16 * j + c] != h_.dcols[static_cast<size_t>(t0 + j) * 16 + c])
                        return layout_fail(fmt("panel-tile descriptor %u: column %u of tile %u", i, c, t0 + j)), BSMR_OK;
        }
        for (u32 t = 0; t < nt; ++t)
            if (!thit[t]) return layout_fail(fmt("panel-tile: tile %u in no item", t)), BSMR_OK;
        return cm_layout(ok);
    }

    int cm_layout(bool* ok) {
        const Plan& p_ = *pp_;
        hipStream_t s = p_.stream;
        std::vector<u32> cr, cc, co;
        std::vector<uint2> slots;
        BSMR_CHECK(p_.cmRow.download(cr, s));
        BSMR_CHECK(p_.cmCol.download(cc, s));
        BSMR_CHECK(p_.cmOut.download(co, s));
        BSMR_CHECK(p_.cmSlots.download(slots, s));
        slots.resize(p_.nSlots);
        const u32 n = p_.nres;
        *ok = false;
        std::vector<uint8_t> hit(h_.nnz, 0), ehit(std::max<u32>(n, 1), 0);
        const u32 nt = static_cast<u32>(h_.bv.size() / TILE);
        if (p_.nDenseItems != nt) return layout_fail(fmt("%u dense items for %u tiles", p_.nDenseItems, nt)), BSMR_OK;
        for (u32 g = 0; g < nt; ++g) {
            const std::string e = tile_hits(g, hit);
            if (!e.empty()) return layout_fail(e), BSMR_OK;
        }
        for (u32 sl = 0; sl < p_.nSlots; ++sl) {
            const uint2 r = slots[sl];
            if (r.y < r.x || r.y > n) return layout_fail(fmt("residual slot %u [%u, %u)", sl, r.x, r.y)), BSMR_OK;
            for (u32 e = r.x; e < r.y; ++e) {
                if (ehit[e]++) return layout_fail(fmt("residual entry %u in two slots", e)), BSMR_OK;
                if (!entry_ok(cr[e], cc[e], co[e]))
                    return layout_fail(fmt("residual entry %u: row %u col %u -> position %u", e, cr[e], cc[e], co[e])), BSMR_OK;
                if (hit[co[e]]++) return layout_fail(fmt("position %u computed twice", co[e])), BSMR_OK;
            }
        }
        for (u32 e = 0; e < n; ++e)
            if (!ehit[e]) return layout_fail(fmt("residual entry %u in no slot", e)), BSMR_OK;
        const std::string e = coverage(hit);
        if (!e.empty()) return layout_fail(e), BSMR_OK;
        *ok = true;
        return BSMR_OK;
    }

    const Plan* pp_;
    float delta_;
    int verbose_;
    Host h_;
    bool rowsInRange_ = false, rowsOk_ = false, colsOk_ = false;
    std::string first_;
};

int run_checks(Checker& c, u32 K, int dtype, int verbose);
}  // namespace
}  // namespace bsmr

using namespace bsmr;

extern "C" int bsmr_plan_check(const bsmr_plan* plan, uint32_t K, int dtype, int verbose) {
    if (!plan) {
        set_error("bsmr_plan_check: null plan");
        return BSMR_ERR_INVALID;
    }
    if (K > 0 && (dtype < BSMR_F32 || dtype > BSMR_BF16)) {
        set_error("bsmr_plan_check: bad dtype");
        return BSMR_ERR_INVALID;
    }
    const Plan& p = plan->p;
    BSMR_HIP(hipSetDevice(p.device));
    Checker c(&p, p.delta, verbose);
    BSMR_CHECK(c.load());
    return run_checks(c, K, dtype, verbose);
}

extern "C" int bsmr_check_rphm_arrays(uint32_t M, uint32_t N, uint32_t nnz, const uint32_t* rowptr,
                                      const uint32_t* colidx, uint32_t R, const uint32_t* rows,
                                      const uint32_t* denseColOffsets, const uint32_t* denseCols,
                                      const uint32_t* sparseColOffsets, const uint32_t* sparseCols,
                                      const uint32_t* sparseValueOffsets, const uint32_t* blockOffsets,
                                      const uint32_t* blockValues, const uint32_t* sparseValues,
                                      const uint32_t* sparseRelativeRows,
                                      const uint32_t* sparseColIndices, float delta, int verbose) {
    if (!rowptr || !colidx || (R && !rows) || !denseColOffsets || !sparseColOffsets ||
        !sparseValueOffsets || !blockOffsets || rowptr[M] != nnz) {
        set_error("bsmr_check_rphm_arrays: bad arguments");
        return BSMR_ERR_INVALID;
    }
    // the checks index per-column and per-entry vectors with S itself: an untrusted S must be a
    // well-formed CSR first (rowptr non-decreasing from 0 to nnz, every column < N)
    if (rowptr[0] != 0) {
        set_error("bsmr_check_rphm_arrays: rowptr[0] != 0");
        return BSMR_ERR_INVALID;
    }
    for (u32 r = 0; r < M; ++r)
        if (rowptr[r + 1] < rowptr[r] || rowptr[r + 1] > nnz) {
            set_error("bsmr_check_rphm_arrays: rowptr is not non-decreasing within [0, nnz] at row " +
                      std::to_string(r));
            return BSMR_ERR_INVALID;
        }
    for (u32 k = 0; k < nnz; ++k)
        if (colidx[k] >= N) {
            set_error("bsmr_check_rphm_arrays: colidx[" + std::to_string(k) + "] = " +
                      std::to_string(colidx[k]) + " is not below N");
            return BSMR_ERR_INVALID;
        }
    const u32 P = (R + 15) / 16;
    Checker c(nullptr, delta, verbose);
    Host& h = c.h();
    h.M = M;
    h.N = N;
    h.nnz = nnz;
    h.R = R;
    h.P = P;
    auto take = [](std::vector<u32>& v, const uint32_t* a, size_t n) {
        v.assign(a, a + (a ? n : 0));
    };
    take(h.rowptr, rowptr, M + 1ull);
    take(h.col, colidx, nnz);
    take(h.rows, rows, R);
    take(h.dco, denseColOffsets, P + 1ull);
    take(h.sco, sparseColOffsets, P + 1ull);
    take(h.svo, sparseValueOffsets, P + 1ull);
    take(h.bo, blockOffsets, P + 1ull);
    take(h.dcols, denseCols, h.dco[P]);
    take(h.scols, sparseCols, h.sco[P]);
    take(h.bv, blockValues, static_cast<size_t>(h.bo[P]) * TILE);
    take(h.sval, sparseValues, h.svo[P]);
    take(h.srel, sparseRelativeRows, h.svo[P]);
    take(h.scol, sparseColIndices, h.svo[P]);
    if ((h.dco[P] && !denseCols) || (h.sco[P] && !sparseCols) || (h.bo[P] && !blockValues) ||
        (h.svo[P] && (!sparseValues || !sparseRelativeRows || !sparseColIndices))) {
        set_error("bsmr_check_rphm_arrays: missing array");
        return BSMR_ERR_INVALID;
    }
    return run_checks(c, 0, BSMR_F32, verbose);
}

namespace bsmr {
namespace {
int run_checks(Checker& c, u32 K, int dtype, int verbose) {
    bool ok = true;
    // the reference's three checks, each followed by its summary line (BSMR.cpp:936-952)
    if (!c.rows()) {
        if (verbose) std::fprintf(stderr, "Error! The row reordering is incorrect!\n");
        ok = false;
    }
    if (!c.columns()) {
        if (verbose) std::fprintf(stderr, "Error! The col reordering is incorrect!\n");
        ok = false;
    }
    if (!c.rphm()) {
        if (verbose) std::fprintf(stderr, "Error! The rphm is incorrect!\n");
        ok = false;
    }
    if (K > 0) {
        bool lok = true;
        BSMR_CHECK(c.layout(K, dtype, &lok));
        ok = ok && lok;
    }
    if (!ok) {
        set_error("bsmr_plan_check: " + c.first());
        return BSMR_ERR_CHECK;
    }
    return BSMR_OK;
}
}  // namespace
}  // namespace bsmr

// Test hook (not in the header; tests/test_gpu_plan_check.py): overwrite element `index` of one
// plan array (which = a bsmr_array value 0..10) or of the launch layout bsmr_sddmm runs for
// (K, dtype) (100: row-block entry metadata, 101: row-block piece words {first entry, column |
// (length - 1) << 22} as 2 u32 per piece, 102: column-major residual output positions, 103: the
// panel-tile launch's item descriptors), so a
// test can show that bsmr_plan_check catches the corruption. *old receives the previous value.
extern "C" int bsmr_debug_plan_poke(bsmr_plan* plan, int which, uint64_t index, uint32_t value,
                                    uint32_t K, int dtype, uint32_t* old) {
    if (!plan) return BSMR_ERR_INVALID;
    Plan& p = plan->p;
    BSMR_HIP(hipSetDevice(p.device));
    u32* base = nullptr;
    size_t n = 0;
    switch (which) {
        case BSMR_ARR_REORDERED_ROWS: base = p.rows.data(); n = p.R; break;
        case BSMR_ARR_DENSE_COLS: base = p.denseCols.data(); n = p.denseCols.n; break;
        case BSMR_ARR_DENSE_COL_OFFSETS: base = p.denseColOffsets.data(); n = p.P + 1; break;
        case BSMR_ARR_SPARSE_COLS: base = p.sparseCols.data(); n = p.sparseCols.n; break;
        case BSMR_ARR_SPARSE_COL_OFFSETS: base = p.sparseColOffsets.data(); n = p.P + 1; break;
        case BSMR_ARR_SPARSE_VALUE_OFFSETS: base = p.sparseValueOffsets.data(); n = p.P + 1; break;
        case BSMR_ARR_BLOCK_OFFSETS: base = p.blockOffsets.data(); n = p.P + 1; break;
        case BSMR_ARR_BLOCK_VALUES: base = p.blockValues.data(); n = p.blockValues.n; break;
        case BSMR_ARR_SPARSE_VALUES: base = p.sparseValues.data(); n = p.nres; break;
        case BSMR_ARR_SPARSE_RELATIVE_ROWS: base = p.sparseRel.data(); n = p.nres; break;
        case BSMR_ARR_SPARSE_COL_INDICES: base = p.sparseColIdx.data(); n = p.nres; break;
        case 100:
        case 101: {
            const Plan::RowBlockLayout* L = nullptr;
            BSMR_CHECK(whole_rb_layout(p, K, dtype, &L));
            if (!L) {
                set_error("bsmr_debug_plan_poke: (K, dtype) runs no row-block layout");
                return BSMR_ERR_UNSUPPORTED;
            }
            if (which == 100) {
                base = L->meta.data();
                n = L->nEntries;
            } else {
                base = reinterpret_cast<u32*>(L->pieces.data());
                n = 2ull * L->nPieces;
            }
            break;
        }
        case 102: base = p.cmOut.data(); n = p.nres; break;
        case 103:  // the panel-tile launch's item descriptors (built by the launch or the check)
            base = p.ptile.built ? p.ptile.desc.data() : nullptr;
            n = p.ptile.built ? p.ptile.desc.n : 0;
            break;
        default:
            set_error("bsmr_debug_plan_poke: unknown array");
            return BSMR_ERR_INVALID;
    }
    if (index >= n || !base) {
        set_error("bsmr_debug_plan_poke: index out of range");
        return BSMR_ERR_INVALID;
    }
    u32 prev = 0;
    BSMR_HIP(hipMemcpy(&prev, base + index, 4, hipMemcpyDeviceToHost));
    BSMR_HIP(hipMemcpy(base + index, &value, 4, hipMemcpyHostToDevice));
    if (old) *old = prev;
    return BSMR_OK;
}
