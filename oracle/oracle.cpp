// oracle.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h for the scope rule and how it is pinned).
//
// A CPU restatement of the reference BSMR-SDDMM path. Each function cites the reference
// file:line it restates (paths relative to the reference repository root). Nothing here is
// copied; it re-derives the same arithmetic so that the row permutation, column split and tile
// layout come out bit-for-bit identical, and the SDDMM values follow the host loop order.
//
// Build: oracle/Makefile (g++ -O2 -fopenmp -ffp-contract=off; no fast-math: the clustering
// similarity is IEEE fp32 division/sqrt, compared with '> alpha').

#include "oracle.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <random>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include <omp.h>
#include <pthread.h>
#include <sched.h>

namespace {

using u32 = uint32_t;
using u64 = uint64_t;
constexpr u32 NULLV = 0xFFFFFFFFu;            // TensorCoreConfig.cuh:11-12
constexpr u32 PANEL = 16;                     // ROW_PANEL_SIZE, BSMR.hpp:8
constexpr u32 BCOL = 16;                      // BLOCK_COL_SIZE, BSMR.hpp:9
constexpr u32 TILE = PANEL * BCOL;            // BLOCK_SIZE, BSMR.hpp:10
constexpr u32 DENSE_BLOCKS_PER_TB = 4;        // sddmmKernel.cuh:11
constexpr u32 SPARSE_DATA_PER_TB = 128;       // sddmmKernel.cuh:14-17
constexpr u32 MAX_SHMEM = 49152;              // TensorCoreConfig.cuh:14

}  // namespace

struct orc_csr {
    u32 M = 0, N = 0, nnz = 0;
    std::vector<u32> rowptr, col;
    std::vector<float> val;
};

struct orc_plan {
    const orc_csr* csr = nullptr;
    float delta = 0.f;
    int32_t numClusters = 1;
    u32 numRowPanels = 0;
    std::vector<u32> rows;  // reorderedRows_
    std::vector<u32> denseCols, denseColOffsets, sparseCols, sparseColOffsets, sparseValueOffsets;
    std::vector<u32> blockOffsets, blockValues, sparseValues, sparseRelativeRows, sparseColIndices;
    orc_stats stats{};
};

namespace {

// ------------------------------------------------------------------------------------------
// Loader. util.hpp:182-197 splits words on ' ', '\t', '\r'. Matrix.cpp:373-396 parses
// "first second [third]" with stoi/stoi/stod; a missing third word is 0, an out-of-range one
// is 0 with a warning. The reference throws (and so aborts) on a non-numeric first/second
// word; this restatement rejects the file instead (documented deviation).
// ------------------------------------------------------------------------------------------
std::string next_word(const std::string& line, size_t& it) {
    const size_t begin = it;
    while (it < line.size() && line[it] != ' ' && line[it] != '\t' && line[it] != '\r') ++it;
    const size_t end = it;
    while (it < line.size() && (line[it] == ' ' || line[it] == '\t' || line[it] == '\r')) ++it;
    return end > begin ? line.substr(begin, end - begin) : std::string();
}

bool parse_int(const std::string& w, long& out) {
    // std::stoi: strtol base 10, needs at least one digit, throws if out of int range.
    if (w.empty()) return false;
    errno = 0;
    char* endp = nullptr;
    const long v = std::strtol(w.c_str(), &endp, 10);
    if (endp == w.c_str()) return false;
    if (errno == ERANGE || v < INT32_MIN || v > INT32_MAX) return false;
    out = v;
    return true;
}

// returns 0 = blank line, 1 = ok, -1 = unparsable (reference would throw)
template <typename T>
int three_words(const std::string& line, u32& a, u32& b, T& c) {
    if (line.empty()) return 0;  // Matrix.cpp:375-377
    size_t it = 0;
    long x, y;
    if (!parse_int(next_word(line, it), x)) return -1;
    if (!parse_int(next_word(line, it), y)) return -1;
    a = static_cast<u32>(static_cast<int>(x));
    b = static_cast<u32>(static_cast<int>(y));
    const std::string w = next_word(line, it);
    if (w.empty()) {
        c = static_cast<T>(0);
        return 1;
    }
    errno = 0;
    char* endp = nullptr;
    const double d = std::strtod(w.c_str(), &endp);
    if (endp == w.c_str()) return -1;  // stod invalid_argument
    if (errno == ERANGE) {
        // libstdc++ std::stod throws out_of_range whenever strtod sets ERANGE
        std::cout << "Warning: valueStr out of range: " << w << std::endl;
        c = static_cast<T>(0);
        return 1;
    }
    c = static_cast<T>(d);
    return 1;
}

// CSR row offsets from row-sorted indices (Matrix.cpp:236-250).
void csr_offsets(u32 M, const std::vector<u32>& rowIdx, std::vector<u32>& off) {
    off.assign(static_cast<size_t>(M) + 1, 0);
    std::vector<u32> cnt(M, 0);
    for (u32 r : rowIdx) ++cnt[r];
    for (u32 r = 0; r < M; ++r) off[r + 1] = off[r] + cnt[r];
}

}  // namespace

extern "C" orc_csr* orc_load_mtx(const char* path, int verbose) {
    const std::string file(path);
    const size_t dot = file.find_last_of('.');
    const std::string suffix = dot == std::string::npos ? std::string() : file.substr(dot);
    if (suffix != ".mtx" && suffix != ".mmio") {  // Matrix.cpp:279-294 (.smtx/.txt: orc_load)
        std::cerr << "Error, file format is not supported : " << file << std::endl;
        return nullptr;
    }
    std::ifstream in(file);
    if (!in.is_open()) {
        std::cerr << "Error, file cannot be opened : " << file << std::endl;
        return nullptr;
    }
    if (verbose) std::cout << "sparseMatrix::CSR initialize from file : " << file << std::endl;
    std::string line;
    bool got = false;
    while (std::getline(in, line)) {  // Matrix.cpp:410: skip lines whose first char is '%'
        got = true;
        if (line.empty() || line[0] != '%') break;
    }
    u32 M = 0, N = 0, nnz = 0;
    if (!got || three_words(line, M, N, nnz) != 1 || M == NULLV || N == NULLV || nnz == NULLV) {
        std::cerr << "Error, file " << file << " format is incorrect!" << std::endl;
        return nullptr;
    }
    std::vector<u32> ri, ci;
    std::vector<float> vv;
    ri.reserve(nnz);
    ci.reserve(nnz);
    vv.reserve(nnz);
    u64 idx = 0;
    while (std::getline(in, line)) {
        u32 r = NULLV, c = NULLV;
        float v = 0.f;
        const int st = three_words(line, r, c, v);
        if (st == 0) continue;
        if (st < 0) {
            std::cerr << "Error, file " << file << " format is incorrect!" << std::endl;
            return nullptr;
        }
        if (idx >= nnz) {
            std::cerr << "Error, file " << file << " too many elements, exceeding the number nnz!"
                      << std::endl;
            return nullptr;
        }
        ri.push_back(r - 1);
        ci.push_back(c - 1);
        vv.push_back(v);
        ++idx;
    }
    if (idx < nnz) {
        std::cerr << "Error, file " << file << " elements is not enough!" << std::endl;
        return nullptr;
    }
    std::set<std::pair<u32, u32>> seen;  // Matrix.cpp:447-461
    for (u64 i = 0; i < nnz; ++i) {
        if (ri[i] >= M || ci[i] >= N) {
            std::cerr << "Error, file " << file << " row or col is too big!" << std::endl;
            return nullptr;
        }
        if (!seen.insert({ri[i], ci[i]}).second) {
            std::cerr << "Error, matrix has duplicate data!" << std::endl;
            return nullptr;
        }
    }
    if (nnz <= 1) {  // Matrix.cpp:462-465
        std::cerr << "Warning, file " << file << " nnz is 1, this is not a valid matrix!"
                  << std::endl;
        return nullptr;
    }
    // stable sort by row (thrust host sort_by_key is stable): file order kept inside a row.
    std::vector<u32> order(nnz);
    for (u32 i = 0; i < nnz; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](u32 a, u32 b) { return ri[a] < ri[b]; });
    auto* c = new orc_csr;
    c->M = M;
    c->N = N;
    c->nnz = nnz;
    c->col.resize(nnz);
    c->val.resize(nnz);
    std::vector<u32> rs(nnz);
    for (u32 i = 0; i < nnz; ++i) {
        rs[i] = ri[order[i]];
        c->col[i] = ci[order[i]];
        c->val[i] = vv[order[i]];
    }
    csr_offsets(M, rs, c->rowptr);
    return c;
}

// .smtx (DLMC), Matrix.cpp:296-371: '%' lines skipped; header "rows cols nnz"; nnz == 0 is
// rejected; the next line holds rows+1 row offsets, the line after it nnz column indices, both
// word-split as above; values are 1; a column repeated inside a row is rejected. Column order in a
// row = file order. The reference throws on a missing or non-numeric word (that is how a short
// line ends there) and does not validate the offsets or the column range; this restatement rejects
// all of those with the messages below (documented deviations).
extern "C" orc_csr* orc_load_smtx(const char* path, int verbose) {
    const std::string file(path);
    std::ifstream in(file);
    if (!in.is_open()) {
        std::cerr << "Error, file cannot be opened : " << file << std::endl;
        return nullptr;
    }
    if (verbose) std::cout << "sparseMatrix::CSR initialize From file : " << file << std::endl;
    std::string line;
    bool got = false;
    while (std::getline(in, line)) {
        got = true;
        if (line.empty() || line[0] != '%') break;
    }
    long hdr[3];
    size_t it = 0;
    for (long& h : hdr)
        if (!got || !parse_int(next_word(line, it), h) || h < 0) {
            std::cerr << "Error, file " << file << " format is incorrect!" << std::endl;
            return nullptr;
        }
    const u32 M = static_cast<u32>(hdr[0]), N = static_cast<u32>(hdr[1]), nnz = static_cast<u32>(hdr[2]);
    if (nnz == 0) {
        std::cerr << "Error, file " << file << " nnz is 0!" << std::endl;
        return nullptr;
    }
    auto* c = new orc_csr;
    c->M = M;
    c->N = N;
    c->nnz = nnz;
    c->rowptr.resize(static_cast<size_t>(M) + 1);
    c->col.resize(nnz);
    c->val.assign(nnz, 1.f);
    auto fail = [&](const std::string& msg) {
        std::cerr << msg << std::endl;
        delete c;
        return static_cast<orc_csr*>(nullptr);
    };
    auto read_ints = [&](std::vector<u32>& dst) {
        if (!std::getline(in, line)) return false;
        size_t w = 0;
        for (u32& v : dst) {
            long x;
            if (!parse_int(next_word(line, w), x) || x < 0) return false;
            v = static_cast<u32>(x);
        }
        return true;
    };
    if (!read_ints(c->rowptr)) return fail("Error, file " + file + " rowOffsets is not enough!");
    if (!read_ints(c->col)) return fail("Error, file " + file + " nnz is not enough!");
    if (c->rowptr[0] != 0 || c->rowptr[M] != nnz) return fail("Error, file " + file + " format is incorrect!");
    for (u32 r = 0; r < M; ++r)
        if (c->rowptr[r] > c->rowptr[r + 1]) return fail("Error, file " + file + " format is incorrect!");
    for (u32 r = 0; r < M; ++r) {
        std::set<u32> seen;
        for (u32 k = c->rowptr[r]; k < c->rowptr[r + 1]; ++k) {
            if (c->col[k] >= N) return fail("Error, file " + file + " row or col is too big!");
            if (!seen.insert(c->col[k]).second) return fail("Error, matrix has duplicate data!");
        }
    }
    return c;
}

// SNAP edge list (.txt), Matrix.cpp:482-575: leading '#' lines, of which one carries
// "Nodes: <n>" and one "Edges: <e>" (possibly the same line); rows = cols = n, nnz = e. Then one
// "from to [value]" per line (blank lines skipped); node ids are renumbered 0, 1, .. in order of
// first appearance (from before to); more than e edges, fewer, an id >= n or a repeated
// (from, to) pair is rejected, the first offending edge in file order deciding the message; the
// edges are then stably sorted by row (file order inside a row). No mirroring.
extern "C" orc_csr* orc_load_snap(const char* path, int verbose) {
    const std::string file(path);
    std::ifstream in(file);
    if (!in.is_open()) {
        std::cerr << "Error, file cannot be opened : " << file << std::endl;
        return nullptr;
    }
    if (verbose) std::cout << "sparseMatrix::CSR initialize From file : " << file << std::endl;
    std::string line;
    long nodes = 0, edges = 0;
    bool data = false;  // `line` holds the first data line
    while (std::getline(in, line)) {
        if (line.empty() || line[0] != '#') {
            data = true;
            break;
        }
        for (const char* key : {"Nodes: ", "Edges: "}) {
            const size_t at = line.find(key);
            if (at == std::string::npos) continue;
            size_t w = at + 7;
            long v;
            if (!parse_int(next_word(line, w), v) || v < 0) {
                std::cerr << "Error, file " << file << " format is incorrect!" << std::endl;
                return nullptr;
            }
            (key[0] == 'N' ? nodes : edges) = v;
        }
    }
    if (!nodes || !edges) {
        std::cerr << "Error, file " << file << " row or col or nnz not initialized!" << std::endl;
        return nullptr;
    }
    const u32 n = static_cast<u32>(nodes), e = static_cast<u32>(edges);
    std::vector<u32> ri, ci;
    std::vector<float> vv;
    std::unordered_map<u32, u32> id;
    auto renum = [&](u32 node) {
        auto f = id.find(node);
        if (f != id.end()) return f->second;
        const u32 k = static_cast<u32>(id.size());
        id.emplace(node, k);
        return k;
    };
    for (bool have = data; have; have = static_cast<bool>(std::getline(in, line))) {
        u32 a, b;
        float v = 0.f;
        const int st = three_words(line, a, b, v);
        if (st == 0) continue;
        if (st < 0) {
            std::cerr << "Error, file " << file << " format is incorrect!" << std::endl;
            return nullptr;
        }
        const u32 ra = renum(a), rb = renum(b);
        if (ri.size() >= e) {
            std::cerr << "Error, file " << file << " too many elements, exceeding the number nnz!"
                      << std::endl;
            return nullptr;
        }
        ri.push_back(ra);
        ci.push_back(rb);
        vv.push_back(v);
    }
    if (ri.size() < e) {
        std::cerr << "Error, file " << file << " elements is not enough!" << std::endl;
        return nullptr;
    }
    std::set<std::pair<u32, u32>> seen;
    for (u32 i = 0; i < e; ++i) {
        if (ri[i] >= n || ci[i] >= n) {
            std::cerr << "Error, file " << file << " row or col is too big!" << std::endl;
            return nullptr;
        }
        if (!seen.insert({ri[i], ci[i]}).second) {
            std::cerr << "Error, matrix has duplicate data!" << std::endl;
            return nullptr;
        }
    }
    std::vector<u32> order(e);
    for (u32 i = 0; i < e; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](u32 x, u32 y) { return ri[x] < ri[y]; });
    auto* c = new orc_csr;
    c->M = n;
    c->N = n;
    c->nnz = e;
    c->col.resize(e);
    c->val.resize(e);
    std::vector<u32> rs(e);
    for (u32 i = 0; i < e; ++i) {
        rs[i] = ri[order[i]];
        c->col[i] = ci[order[i]];
        c->val[i] = vv[order[i]];
    }
    csr_offsets(n, rs, c->rowptr);
    return c;
}

// CSR::initializeFromMatrixFile (Matrix.cpp:279-294): dispatch on the last '.' suffix
extern "C" orc_csr* orc_load(const char* path, int verbose) {
    const std::string file(path);
    const size_t dot = file.find_last_of('.');
    const std::string suffix = dot == std::string::npos ? std::string() : file.substr(dot);
    if (suffix == ".mtx" || suffix == ".mmio") return orc_load_mtx(path, verbose);
    if (suffix == ".smtx") return orc_load_smtx(path, verbose);
    if (suffix == ".txt") return orc_load_snap(path, verbose);
    std::cerr << "Error, file format is not supported : " << file << std::endl;
    return nullptr;
}

extern "C" orc_csr* orc_csr_from_arrays(uint32_t M, uint32_t N, uint32_t nnz,
                                        const uint32_t* rowptr, const uint32_t* colidx) {
    auto* c = new orc_csr;
    c->M = M;
    c->N = N;
    c->nnz = nnz;
    c->rowptr.assign(rowptr, rowptr + M + 1);
    c->col.assign(colidx, colidx + nnz);
    c->val.assign(nnz, 0.f);
    return c;
}

extern "C" void orc_csr_info(const orc_csr* c, uint32_t* M, uint32_t* N, uint32_t* nnz) {
    *M = c->M;
    *N = c->N;
    *nnz = c->nnz;
}

extern "C" void orc_csr_copy(const orc_csr* c, uint32_t* rowptr, uint32_t* colidx,
                             float* values) {
    if (rowptr) std::memcpy(rowptr, c->rowptr.data(), (c->M + 1) * sizeof(u32));
    if (colidx) std::memcpy(colidx, c->col.data(), c->nnz * sizeof(u32));
    if (values) std::memcpy(values, c->val.data(), c->nnz * sizeof(float));
}

extern "C" void orc_csr_free(orc_csr* c) { delete c; }

// makeData: a fresh default-constructed std::mt19937 per matrix, uniform_real_distribution<float>
// (0,2) (Matrix.cpp:128-137). libstdc++'s generate_canonical<float,24> with a 32-bit engine is
// one draw: float(u) / 2^32, clamped below 1, then *2 + 0 — restated here explicitly.
extern "C" void orc_make_data(uint64_t n, float* out) {
    std::mt19937 gen;  // seed 5489
    const float scale = 4294967296.0f;
    const float below_one = std::nextafter(1.0f, 0.0f);
    for (u64 i = 0; i < n; ++i) {
        float u = static_cast<float>(static_cast<u32>(gen())) / scale;
        if (u >= 1.0f) u = below_one;
        out[i] = u * (2.0f - 0.0f) + 0.0f;
    }
}

// calculateBlockSize (rowReordering.cu:1009-1025)
extern "C" uint32_t orc_block_size(uint32_t M, uint32_t N, uint64_t free_mem) {
    const u32 gmem = static_cast<u32>(std::ceil(
        static_cast<float>(static_cast<u64>(M) * M * sizeof(u32)) / static_cast<float>(free_mem / 2)));
    const u32 smem = static_cast<u32>(std::ceil(static_cast<float>(static_cast<u64>(N) * sizeof(u32)) /
                                                static_cast<float>(MAX_SHMEM / 2)));
    const u32 bs = std::max(gmem, smem);
    return bs > 16 ? bs : 16;
}

// bsa_clustering block size (rowReordering.cu:911-920)
extern "C" uint32_t orc_cluster_block_dim(uint32_t nbpr) {
    if (nbpr < 32) return 32;
    int cand = static_cast<int>(32 * std::ceil(static_cast<float>(static_cast<int>(nbpr) / 4) / 32.0f));
    cand = cand > 32 ? cand : 32;
    return static_cast<u32>(1024 < cand ? 1024 : cand);
}

namespace {

// ------------------------------------------------------------------------------------------
// Block reduction shape (cudaUtil.cuh:13-45): xor butterfly inside each 32-lane warp, then
// `for (stride = blockDim/64; stride >= 1; stride >>= 1) s[w] += s[w+stride] (w < stride)`.
// For a warp count that is not a power of two some warps never reach s[0]; `kept` marks the
// ones that do.
// ------------------------------------------------------------------------------------------
struct Shape {
    u32 B = 32, W = 1;
    std::vector<char> kept;  // per warp
    std::vector<char> keptIdx;  // per encoding index i < nbpr: warp((i mod B)) kept
};

Shape make_shape(u32 B, u32 nbpr) {
    Shape s;
    s.B = B;
    s.W = B / 32;
    std::vector<std::vector<char>> reach(s.W, std::vector<char>(s.W, 0));
    for (u32 w = 0; w < s.W; ++w) reach[w][w] = 1;
    for (u32 stride = B / 64; stride >= 1; stride >>= 1)
        for (u32 w = 0; w < stride; ++w)
            for (u32 x = 0; x < s.W; ++x) reach[w][x] |= reach[w + stride][x];
    s.kept = reach[0];
    s.keptIdx.resize(nbpr);
    for (u32 i = 0; i < nbpr; ++i) s.keptIdx[i] = s.kept[(i % B) / 32];
    return s;
}

float tree_reduce(const std::vector<float>& partial, const Shape& sh) {
    std::vector<float> s(sh.W);
    float v[32];
    for (u32 w = 0; w < sh.W; ++w) {
        for (u32 l = 0; l < 32; ++l) v[l] = partial[w * 32 + l];
        for (u32 step = 1; step < 32; step <<= 1)
            for (u32 l = 0; l < 32; l += 2 * step) v[l] = v[l] + v[l + step];
        s[w] = v[0];
    }
    for (u32 stride = sh.B / 64; stride >= 1; stride >>= 1)
        for (u32 w = 0; w < stride; ++w) s[w] = s[w] + s[w + stride];
    return s[0];
}

inline u32 sq(u32 e) { return e * e; }  // (int)e*(int)e with 32-bit wrap, as unsigned bits

// calculate_similarity_norm_weighted_jaccard, u32 version (rowReordering.cu:235-293): exact.
float similarity_exact(const u32* rep, const u32* cmp, u32 nbpr, const Shape& sh) {
    const u32 B = sh.B;
    u32 SR = 0, SC = 0;
    for (u32 t = 0; t < B; ++t) {
        if (!sh.kept[t / 32]) continue;
        for (u32 i = t; i < nbpr; i += B) {
            SR += sq(rep[i]);
            SC += sq(cmp[i]);
        }
    }
    if (SR == 0 && SC == 0) return 1.0f;
    if (SR == 0 || SC == 0) return 0.0f;
    const float nr = std::sqrt(static_cast<float>(SR));
    const float nc = std::sqrt(static_cast<float>(SC));
    std::vector<float> mn(B, 0.f), mx(B, 0.f);
    for (u32 t = 0; t < B; ++t) {
        float a = 0.f, b = 0.f;
        for (u32 i = t; i < nbpr; i += B) {
            const float x = static_cast<float>(rep[i]) / nr;
            const float y = static_cast<float>(cmp[i]) / nc;
            a += std::fmin(x, y);
            b += std::fmax(x, y);
        }
        mn[t] = a;
        mx[t] = b;
    }
    const float MN = tree_reduce(mn, sh);
    const float MX = tree_reduce(mx, sh);
    return MN / MX;
}

struct SparseRow {
    u32 begin, end;  // into blk/cnt arrays
    u32 SC;          // kept sum of squares (u32 wrap)
    u64 S1C;         // kept sum of counts
};

}  // namespace

// kernel::calculateDispersion (rowReordering.cu:49-93): e[b] = #{c in row : c/bs == b};
// disp = sum_{b: e>0} (bs - e_b) + nnz * #{b: e>0}, all in u32.
extern "C" void orc_dispersion(const orc_csr* c, uint32_t bs, uint32_t* disp) {
    const int nbpr = static_cast<int>(std::ceil(static_cast<float>(c->N) / static_cast<float>(bs)));
    (void)nbpr;
#pragma omp parallel
    {
        std::unordered_map<u32, u32> h;
#pragma omp for schedule(dynamic, 64)
        for (long r = 0; r < static_cast<long>(c->M); ++r) {
            const u32 b0 = c->rowptr[r], b1 = c->rowptr[r + 1];
            const u32 n = b1 - b0;
            if (n == 0) {
                disp[r] = 0;
                continue;
            }
            h.clear();
            for (u32 k = b0; k < b1; ++k) ++h[c->col[k] / bs];
            u32 d = 0;
            for (auto& kv : h) d += bs - kv.second;
            d += n * static_cast<u32>(h.size());
            disp[r] = d;
        }
    }
}

// Row reordering = bsa_rowReordering_gpu (rowReordering.cu:1027-1095) + get_permutation_gpu
// (893-1007). The device mutex chain of bsa_clustering (325-432) makes cluster c examine
// position i only after cluster c-1 has; cluster c+1 is spawned at c's first rejection. That is
// sequential first-fit (SURVEY.md §8a spec 6b), restated here directly.
//
// Speed: each similarity is first evaluated in double from the sparse row (exact integer norms
// and the same fp32 norms as the device code); only when it lies within GUARD of alpha is the
// exact fp32 warp-tree evaluated. The fp32 tree differs from the real value by < 3e-6 (≤ 16
// rounding levels), so outside the guard band the '> alpha' decision is the same.
extern "C" int orc_row_reorder(const orc_csr* c, float alpha, uint32_t bs, int exact_all,
                               uint32_t* out_rows, uint32_t* out_len, int32_t* out_num_clusters,
                               uint64_t* out_exact, uint64_t* out_total) {
    const u32 M = c->M;
    const u32 nbpr = static_cast<u32>(std::ceil(static_cast<float>(c->N) / static_cast<float>(bs)));
    const u32 B = orc_cluster_block_dim(nbpr);
    const Shape sh = make_shape(B, nbpr);

    // sparse encodings per row (sorted block ids) + dispersion
    std::vector<u32> disp(M, 0);
    std::vector<SparseRow> srow(M);
    std::vector<u32> blk(c->nnz), cnt(c->nnz);
#pragma omp parallel
    {
        std::vector<u32> tmp;
#pragma omp for schedule(dynamic, 64)
        for (long r = 0; r < static_cast<long>(M); ++r) {
            const u32 b0 = c->rowptr[r], b1 = c->rowptr[r + 1];
            tmp.clear();
            for (u32 k = b0; k < b1; ++k) tmp.push_back(c->col[k] / bs);
            std::sort(tmp.begin(), tmp.end());
            u32 w = b0, nb = 0, d = 0;
            u32 SC = 0;
            u64 S1 = 0;
            for (size_t k = 0; k < tmp.size();) {
                size_t j = k;
                while (j < tmp.size() && tmp[j] == tmp[k]) ++j;
                const u32 e = static_cast<u32>(j - k);
                blk[w] = tmp[k];
                cnt[w] = e;
                ++w;
                ++nb;
                d += bs - e;
                if (sh.keptIdx[tmp[k]]) {
                    SC += sq(e);
                    S1 += e;
                }
                k = j;
            }
            const u32 n = b1 - b0;
            disp[r] = n == 0 ? 0 : d + n * nb;
            srow[r] = SparseRow{b0, w, SC, S1};
        }
    }

    // ascending = [0..M) stably sorted by dispersion (rowReordering.cu:1055-1062)
    std::vector<u32> asc(M);
    for (u32 i = 0; i < M; ++i) asc[i] = i;
    std::stable_sort(asc.begin(), asc.end(), [&](u32 a, u32 b) { return disp[a] < disp[b]; });

    // zero rows -> cluster 0 (rowReordering.cu:939-949)
    std::vector<u32> ids(M, NULLV);
    u32 z = 0;
    while (z < M && disp[asc[z]] == 0) {
        ids[z] = 0;
        ++z;
    }

    struct Cluster {
        std::vector<u32> rep;
        u32 SR = 0;
        u64 S1R = 0;
    };
    std::vector<Cluster> cl;
    std::vector<u32> dense_cmp(nbpr, 0);
    const double GUARD = 1e-5;
    const double alpha_d = static_cast<double>(alpha);
    u64 nexact = 0, ntotal = 0;

    auto add_row = [&](Cluster& C, const SparseRow& s) {
        for (u32 k = s.begin; k < s.end; ++k) {
            const u32 i = blk[k];
            if (sh.keptIdx[i]) {
                C.SR -= sq(C.rep[i]);
                C.S1R -= C.rep[i];
            }
            C.rep[i] += cnt[k];
            if (sh.keptIdx[i]) {
                C.SR += sq(C.rep[i]);
                C.S1R += C.rep[i];
            }
        }
    };

    for (u32 pos = z; pos < M; ++pos) {
        const u32 row = asc[pos];
        const SparseRow& s = srow[row];
        bool placed = false;
        for (u32 ci = 0; ci < cl.size(); ++ci) {
            Cluster& C = cl[ci];
            ++ntotal;
            bool accept;
            bool need_exact = exact_all != 0;
            double sim_d = 0.0;
            if (!need_exact) {
                if (C.SR == 0 && s.SC == 0) {
                    sim_d = 1.0;
                } else if (C.SR == 0 || s.SC == 0) {
                    sim_d = 0.0;
                } else {
                    const float nr = std::sqrt(static_cast<float>(C.SR));
                    const float nc = std::sqrt(static_cast<float>(s.SC));
                    double mn = 0.0;
                    for (u32 k = s.begin; k < s.end; ++k) {
                        const u32 i = blk[k];
                        if (!sh.keptIdx[i] || C.rep[i] == 0) continue;
                        mn += std::min(static_cast<double>(C.rep[i]) / nr,
                                       static_cast<double>(cnt[k]) / nc);
                    }
                    const double mx = static_cast<double>(C.S1R) / nr +
                                      static_cast<double>(s.S1C) / nc - mn;
                    sim_d = mn / mx;
                    if (std::fabs(sim_d - alpha_d) <= GUARD) need_exact = true;
                }
            }
            if (need_exact) {
                ++nexact;
                for (u32 k = s.begin; k < s.end; ++k) dense_cmp[blk[k]] = cnt[k];
                const float sim = similarity_exact(C.rep.data(), dense_cmp.data(), nbpr, sh);
                for (u32 k = s.begin; k < s.end; ++k) dense_cmp[blk[k]] = 0;
                accept = sim > alpha;
            } else {
                accept = sim_d > alpha_d;
            }
            if (accept) {
                ids[pos] = ci + 1;
                add_row(C, s);
                placed = true;
                break;
            }
        }
        if (!placed) {
            cl.emplace_back();
            Cluster& C = cl.back();
            C.rep.assign(nbpr, 0);
            add_row(C, s);
            ids[pos] = static_cast<u32>(cl.size());
        }
    }

    // stable sort of positions by cluster id; permutation[k] = asc[indices[k]] (988-995)
    std::vector<u32> indices(M);
    for (u32 i = 0; i < M; ++i) indices[i] = i;
    std::stable_sort(indices.begin(), indices.end(), [&](u32 a, u32 b) { return ids[a] < ids[b]; });
    std::vector<u32> sorted_ids(M);
    for (u32 k = 0; k < M; ++k) sorted_ids[k] = ids[indices[k]];
    // numClusters reads the already-sorted ids at indices[M-1] (rowReordering.cu:996, quirk)
    const int32_t ncl = static_cast<int32_t>(sorted_ids[indices[M - 1]]) + (z != 0 ? 1 : 0);

    // drop leading zero rows (1081-1090)
    u32 k0 = 0;
    while (k0 < M && c->rowptr[asc[indices[k0]] + 1] - c->rowptr[asc[indices[k0]]] == 0) ++k0;
    u32 n = 0;
    for (u32 k = k0; k < M; ++k) out_rows[n++] = asc[indices[k]];
    *out_len = n;
    *out_num_clusters = ncl;
    if (out_exact) *out_exact = nexact;
    if (out_total) *out_total = ntotal;
    return 0;
}

namespace {

// colReordering_cpu (colReordering.cu:274-404) + analysisDescendingOrderColSegment (244-271).
void col_reorder(orc_plan& p) {
    const orc_csr& c = *p.csr;
    const u32 P = p.numRowPanels;
    const u32 R = static_cast<u32>(p.rows.size());
    const u32 thr = static_cast<u32>(std::ceil(p.delta * static_cast<float>(TILE)));
    std::vector<std::vector<u32>> cols(P);
    std::vector<u32> nd(P), ns(P), sdata(P);
#pragma omp parallel
    {
        std::vector<u32> count(c.N, 0);
        std::vector<u32> touched;
#pragma omp for schedule(dynamic)
        for (long pp = 0; pp < static_cast<long>(P); ++pp) {
            const u32 r0 = static_cast<u32>(pp) * PANEL, r1 = std::min(r0 + PANEL, R);
            touched.clear();
            for (u32 q = r0; q < r1; ++q) {
                const u32 row = p.rows[q];
                for (u32 k = c.rowptr[row]; k < c.rowptr[row + 1]; ++k) {
                    if (count[c.col[k]]++ == 0) touched.push_back(c.col[k]);
                }
            }
            // columns with cnt>0 in ascending order, then stable sort by count descending
            std::sort(touched.begin(), touched.end());
            std::stable_sort(touched.begin(), touched.end(),
                             [&](u32 a, u32 b) { return count[a] > count[b]; });
            std::vector<u32> cnts(touched.size());
            for (size_t k = 0; k < touched.size(); ++k) cnts[k] = count[touched[k]];
            if (touched.size() % BCOL != 0) {  // pad with sentinel N (338-343)
                const size_t pad = BCOL - touched.size() % BCOL;
                touched.insert(touched.end(), pad, c.N);
                cnts.insert(cnts.end(), pad, 0);
            }
            u32 dense = 0;
            for (size_t g = 0; g + BCOL <= cnts.size(); g += BCOL) {
                u32 s = 0;
                for (u32 k = 0; k < BCOL; ++k) s += cnts[g + k];
                if (s >= thr) dense += BCOL;
            }
            const u32 sparse = static_cast<u32>(cnts.size()) - dense;
            u32 sd = 0;
            for (u32 k = dense; k < dense + sparse; ++k) sd += cnts[k];
            nd[pp] = dense;
            ns[pp] = sparse;
            sdata[pp] = sd;
            for (u32 col : touched)
                if (col < c.N) count[col] = 0;
            cols[pp] = std::move(touched);
        }
    }
    p.denseColOffsets.assign(P + 1, 0);
    p.sparseColOffsets.assign(P + 1, 0);
    p.sparseValueOffsets.assign(P + 1, 0);
    for (u32 q = 0; q < P; ++q) {
        p.denseColOffsets[q + 1] = p.denseColOffsets[q] + nd[q];
        p.sparseColOffsets[q + 1] = p.sparseColOffsets[q] + ns[q];
        p.sparseValueOffsets[q + 1] = p.sparseValueOffsets[q] + sdata[q];
    }
    p.denseCols.resize(p.denseColOffsets[P]);
    p.sparseCols.resize(p.sparseColOffsets[P]);
    for (u32 q = 0; q < P; ++q) {
        std::copy(cols[q].begin(), cols[q].begin() + nd[q], p.denseCols.begin() + p.denseColOffsets[q]);
        std::copy(cols[q].begin() + nd[q], cols[q].end(), p.sparseCols.begin() + p.sparseColOffsets[q]);
    }
}

// RPHM::RPHM (BSMR.cpp:83-265): dense tiles (BELL-like, 256 CSR indices per 16x16 tile, NULL
// where absent) and the per-panel residual in sparseCols order.
void build_rphm(orc_plan& p) {
    const orc_csr& c = *p.csr;
    const u32 P = p.numRowPanels;
    const u32 R = static_cast<u32>(p.rows.size());
    p.blockOffsets.assign(P + 1, 0);
    for (u32 q = 0; q < P; ++q) {
        const u32 ncol = p.denseColOffsets[q + 1] - p.denseColOffsets[q];
        p.blockOffsets[q + 1] = p.blockOffsets[q] +
                                static_cast<u32>(std::ceil(static_cast<float>(ncol) / BCOL));
    }
    p.blockValues.assign(static_cast<size_t>(p.blockOffsets[P]) * TILE, NULLV);
#pragma omp parallel
    {
        std::unordered_map<u32, u32> colToIdx;
#pragma omp for schedule(dynamic, 16)
        for (long q = 0; q < static_cast<long>(R); ++q) {
            const u32 row = p.rows[q];
            colToIdx.clear();
            for (u32 k = c.rowptr[row]; k < c.rowptr[row + 1]; ++k) colToIdx[c.col[k]] = k;
            const u32 panel = static_cast<u32>(q) / PANEL, lr = static_cast<u32>(q) % PANEL;
            const size_t base = static_cast<size_t>(p.blockOffsets[panel]) * TILE;
            u32 count = 0;
            for (u32 j = p.denseColOffsets[panel]; j < p.denseColOffsets[panel + 1]; ++j, ++count) {
                auto it = colToIdx.find(p.denseCols[j]);
                if (it != colToIdx.end())
                    p.blockValues[base + (count / BCOL) * TILE + lr * BCOL + count % BCOL] = it->second;
            }
        }
    }
    const u32 nres = p.sparseValueOffsets[P];
    p.sparseValues.assign(nres, 0);
    p.sparseRelativeRows.assign(nres, 0);
    p.sparseColIndices.assign(nres, 0);
#pragma omp parallel
    {
        std::unordered_map<u32, std::vector<std::pair<u32, u32>>> m;
#pragma omp for schedule(dynamic)
        for (long q = 0; q < static_cast<long>(P); ++q) {
            m.clear();
            const u32 r0 = static_cast<u32>(q) * PANEL, r1 = std::min(r0 + PANEL, R);
            for (u32 x = r0; x < r1; ++x) {
                const u32 row = p.rows[x];
                for (u32 k = c.rowptr[row]; k < c.rowptr[row + 1]; ++k)
                    m[c.col[k]].push_back({x % PANEL, k});
            }
            u32 w = p.sparseValueOffsets[q];
            for (u32 j = p.sparseColOffsets[q]; j < p.sparseColOffsets[q + 1]; ++j) {
                const u32 col = p.sparseCols[j];
                auto it = m.find(col);
                if (it == m.end()) continue;
                for (auto& e : it->second) {
                    p.sparseRelativeRows[w] = e.first;
                    p.sparseValues[w] = e.second;
                    p.sparseColIndices[w] = col;
                    ++w;
                }
            }
        }
    }
}

// calculateNumDenseBlocksAndAverageDensityInOriginalMatrix (BSMR.cpp:955-994): 16x16 tiles of
// the ORIGINAL order (edge tiles smaller), float density, summed in (panel, colBlock) order.
std::pair<u32, float> original_dense_blocks(const orc_csr& c, float delta) {
    const u32 P = static_cast<u32>(std::ceil(static_cast<float>(c.M) / PANEL));
    u32 num = 0;
    float total = 0.f;
    std::vector<std::vector<std::pair<u32, u32>>> per(P);  // (colBlock, count) sorted
#pragma omp parallel for schedule(dynamic)
    for (long q = 0; q < static_cast<long>(P); ++q) {
        std::vector<u32> cb;
        const u32 r0 = static_cast<u32>(q) * PANEL, r1 = std::min(r0 + PANEL, c.M);
        for (u32 r = r0; r < r1; ++r)
            for (u32 k = c.rowptr[r]; k < c.rowptr[r + 1]; ++k) cb.push_back(c.col[k] / BCOL);
        std::sort(cb.begin(), cb.end());
        auto& v = per[q];
        for (size_t k = 0; k < cb.size();) {
            size_t j = k;
            while (j < cb.size() && cb[j] == cb[k]) ++j;
            v.push_back({cb[k], static_cast<u32>(j - k)});
            k = j;
        }
    }
    for (u32 q = 0; q < P; ++q) {
        const u32 r0 = q * PANEL, r1 = std::min(r0 + PANEL, c.M);
        for (auto& e : per[q]) {
            const u32 c0 = e.first * BCOL, c1 = std::min(c0 + BCOL, c.N);
            const float bsz = static_cast<float>((r1 - r0) * (c1 - c0));
            const float density = static_cast<float>(e.second) / bsz;
            if (density >= delta) {
                total += density;
                ++num;
            }
        }
    }
    const float avg = num > 0 ? total / static_cast<float>(num) : 0.0f;
    return {num, avg};
}

// evaluationReordering (BSMR.cpp:826-930)
void evaluate(orc_plan& p) {
    const orc_csr& c = *p.csr;
    const u32 P = p.numRowPanels;
    const u32 R = static_cast<u32>(p.rows.size());
    int numDense = 0, numDenseTB = 0, numSparseTB = 0, numSparseData = 0;
    float totalDensity = 0.f;
    std::vector<u32> blockOfCol(c.N + 1, NULLV);
    std::vector<char> isSparse(c.N + 1, 0);
    for (u32 q = 0; q < P; ++q) {
        const u32 d0 = p.denseColOffsets[q], d1 = p.denseColOffsets[q + 1];
        const u32 s0 = p.sparseColOffsets[q], s1 = p.sparseColOffsets[q + 1];
        const int nDB = static_cast<int>(std::ceil((d1 - d0) / static_cast<float>(BCOL)));
        numDenseTB += static_cast<int>(std::ceil(static_cast<float>(nDB) / DENSE_BLOCKS_PER_TB));
        numSparseTB += static_cast<int>(std::ceil(
            static_cast<float>(p.sparseValueOffsets[q + 1] - p.sparseValueOffsets[q]) / SPARSE_DATA_PER_TB));
        for (u32 j = d0; j < d1; ++j) blockOfCol[p.denseCols[j]] = (j - d0) / BCOL;
        for (u32 j = s0; j < s1; ++j) isSparse[p.sparseCols[j]] = 1;
        std::vector<u32> nnzIn(nDB, 0);
        const u32 r0 = q * PANEL, r1 = std::min(r0 + PANEL, R);
        for (u32 x = r0; x < r1; ++x) {
            const u32 row = p.rows[x];
            for (u32 k = c.rowptr[row]; k < c.rowptr[row + 1]; ++k) {
                const u32 col = c.col[k];
                if (blockOfCol[col] != NULLV) ++nnzIn[blockOfCol[col]];
                if (isSparse[col]) ++numSparseData;
            }
        }
        for (int b = 0; b < nDB; ++b) {
            if (nnzIn[b] > 0) {
                const float density = static_cast<float>(nnzIn[b]) / static_cast<float>(PANEL * BCOL);
                totalDensity += density;
                if (density >= p.delta) ++numDense;
            }
        }
        for (u32 j = d0; j < d1; ++j) blockOfCol[p.denseCols[j]] = NULLV;
        for (u32 j = s0; j < s1; ++j) isSparse[p.sparseCols[j]] = 0;
    }
    const auto orig = original_dense_blocks(c, p.delta);
    orc_stats& s = p.stats;
    s.numRowPanels = static_cast<int32_t>(P);
    s.numClusters = p.numClusters;
    s.numDenseBlock = numDense;
    const float avg = totalDensity / static_cast<float>(numDense);  // inf / nan as the reference
    s.averageDensity = avg > 0 ? avg : 0.0f;
    s.originalNumDenseBlock = static_cast<int32_t>(orig.first);
    s.originalAverageDensity = orig.second;
    s.numDenseThreadBlocks = numDenseTB;
    s.numSparseThreadBlocks = numSparseTB;
    s.numSparseData = numSparseData;
    s.numDenseData = static_cast<int32_t>(c.nnz) - numSparseData;
    u32 maxDense = 0, rphmSparseTB = 0;
    for (u32 q = 0; q < P; ++q) {
        maxDense = std::max(maxDense, p.blockOffsets[q + 1] - p.blockOffsets[q]);
        rphmSparseTB += static_cast<u32>(std::ceil(
            static_cast<float>(p.sparseValueOffsets[q + 1] - p.sparseValueOffsets[q]) / SPARSE_DATA_PER_TB));
    }
    s.maxNumDenseColBlocksInRowPanel = maxDense;
    s.numDenseBlocksTotal = p.blockOffsets[P];
    s.rphmNumSparseThreadBlocks = rphmSparseTB;
}

}  // namespace

extern "C" orc_plan* orc_plan_from_rows(const orc_csr* c, const uint32_t* rows, uint32_t nrows,
                                        int32_t num_clusters, float delta) {
    auto* p = new orc_plan;
    p->csr = c;
    p->delta = delta;
    p->numClusters = num_clusters;
    p->rows.assign(rows, rows + nrows);
    p->numRowPanels = static_cast<u32>(std::ceil(static_cast<float>(nrows) / PANEL));  // BSMR.cpp:48
    col_reorder(*p);
    build_rphm(*p);
    evaluate(*p);
    return p;
}

extern "C" int orc_plan_stats(const orc_plan* p, orc_stats* s) {
    *s = p->stats;
    return 0;
}

extern "C" uint64_t orc_plan_array(const orc_plan* p, int which, uint32_t* out) {
    const std::vector<u32>* v = nullptr;
    switch (which) {
        case ORC_REORDERED_ROWS: v = &p->rows; break;
        case ORC_DENSE_COLS: v = &p->denseCols; break;
        case ORC_DENSE_COL_OFFSETS: v = &p->denseColOffsets; break;
        case ORC_SPARSE_COLS: v = &p->sparseCols; break;
        case ORC_SPARSE_COL_OFFSETS: v = &p->sparseColOffsets; break;
        case ORC_SPARSE_VALUE_OFFSETS: v = &p->sparseValueOffsets; break;
        case ORC_BLOCK_OFFSETS: v = &p->blockOffsets; break;
        case ORC_BLOCK_VALUES: v = &p->blockValues; break;
        case ORC_SPARSE_VALUES: v = &p->sparseValues; break;
        case ORC_SPARSE_RELATIVE_ROWS: v = &p->sparseRelativeRows; break;
        case ORC_SPARSE_COL_INDICES: v = &p->sparseColIndices; break;
        default: return 0;
    }
    if (out && !v->empty()) std::memcpy(out, v->data(), v->size() * sizeof(u32));
    return v->size();
}

extern "C" void orc_plan_free(orc_plan* p) { delete p; }

// sddmm_cpu (host.cpp:45-76): OpenMP over rows; serial fp32 `val += a*b`, k ascending. Built with
// -ffp-contract=off so no FMA is formed (the reference's g++ -O3 x86-64 build has none).
extern "C" void orc_sddmm_cpu_rows(const orc_csr* c, uint32_t K, const float* A, const float* B,
                                   float* P, uint32_t row_begin, uint32_t row_end, int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
    for (long row = row_begin; row < static_cast<long>(row_end); ++row) {
        const float* a = A + static_cast<size_t>(row) * K;
        for (u32 idx = c->rowptr[row]; idx < c->rowptr[row + 1]; ++idx) {
            const float* b = B + static_cast<size_t>(c->col[idx]) * K;
            float val = 0.0f;
            for (u32 k = 0; k < K; ++k) val += a[k] * b[k];
            P[idx] = val;
        }
    }
}

// The same loop with its OpenMP team pinned "close" (BASELINE.md §2's OMP_PROC_BIND=close, done
// here so that only this team is bound, whatever OpenMP runtime the host process started first):
// thread t runs on cpus[t % ncpus] (the caller passes its affinity set in order); the calling
// thread's own mask is restored afterwards. Returns the threads that took their CPU.
extern "C" int orc_sddmm_cpu_rows_bound(const orc_csr* c, uint32_t K, const float* A, const float* B,
                                        float* P, uint32_t row_begin, uint32_t row_end, int nthreads,
                                        const int* cpus, int ncpus) {
    cpu_set_t saved;
    CPU_ZERO(&saved);
    const bool have = pthread_getaffinity_np(pthread_self(), sizeof(saved), &saved) == 0;
    int pinned = 0;
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel reduction(+ : pinned)
    {
        if (cpus && ncpus > 0) {
            cpu_set_t one;
            CPU_ZERO(&one);
            CPU_SET(cpus[omp_get_thread_num() % ncpus], &one);
            pinned += pthread_setaffinity_np(pthread_self(), sizeof(one), &one) == 0;
        }
#pragma omp for schedule(static)
        for (long row = row_begin; row < static_cast<long>(row_end); ++row) {
            const float* a = A + static_cast<size_t>(row) * K;
            for (u32 idx = c->rowptr[row]; idx < c->rowptr[row + 1]; ++idx) {
                const float* b = B + static_cast<size_t>(c->col[idx]) * K;
                float val = 0.0f;
                for (u32 k = 0; k < K; ++k) val += a[k] * b[k];
                P[idx] = val;
            }
        }
    }
    if (have) pthread_setaffinity_np(pthread_self(), sizeof(saved), &saved);
    return pinned;
}

extern "C" void orc_sddmm_cpu(const orc_csr* c, uint32_t K, const float* A, const float* B,
                              float* P, int nthreads) {
    orc_sddmm_cpu_rows(c, K, A, B, P, 0, c->M, nthreads);
}

// checkOneData<float> (checkData.hpp:21-30)
extern "C" int orc_check_one(float a, float b) {
    const float absDiff = std::fabs(a - b);
    if (absDiff < 1e-5f) return 1;
    const float eps = 1e-3f;
    const float maxVal = std::max(std::max(std::fabs(a), std::fabs(b)), eps);
    return (absDiff / maxVal) < eps;
}

// checkDataFunction (checkData.hpp:44-79)
extern "C" uint64_t orc_check_data(uint64_t n, const float* a, const float* b, int verbose) {
    if (verbose) {
        printf("|---------------------------check data---------------------------|\n");
        printf("| Data size : %ld\n", static_cast<long>(n));
        printf("| Error threshold epsilon : %f\n", static_cast<double>(1e-3f));
        printf("| Checking results...\n");
    }
    u64 errors = 0;
    for (u64 i = 0; i < n; ++i) {
        if (!orc_check_one(a[i], b[i])) {
            ++errors;
            if (verbose && errors < 10)
                printf("| Error : idx = %d, data1 = %f, data2 = %f, difference = %f\n",
                       static_cast<int>(i), static_cast<double>(a[i]), static_cast<double>(b[i]),
                       static_cast<double>(a[i] - b[i]));
        }
    }
    if (verbose) {
        if (errors > 0)
            printf("| No Pass! Inconsistent data! %zu errors! Error rate : %2.2f%%\n",
                   static_cast<size_t>(errors),
                   static_cast<double>(static_cast<float>(errors) / static_cast<float>(n) * 100));
        else
            printf("| Pass! Result validates successfully.\n");
        printf("|----------------------------------------------------------------|\n");
        fflush(stdout);
    }
    return errors;
}
