// csr_io.cpp — host-side input boundary: Matrix Market loader, makeData, error plumbing.
//
// Loader semantics follow sparseMatrix::CSR<T>::initializeFromMtxFile (src/Matrix.cpp:398-480)
// and its helpers (Matrix.cpp:373-396, include/util.hpp:182-197):
//   * lines starting with '%' before the header are skipped; header "M N nnz";
//   * entries "r c [v]" 1-based, words split on ' ', '\t', '\r'; missing value = 0, a value
//     std::stod reports out of range = 0 with a warning; blank lines skipped;
//   * symmetric/pattern/complex qualifiers are NOT interpreted (no mirroring);
//   * reject: more entries than nnz, fewer, out-of-range index, duplicate (the first offending
//     entry in file order decides the message, as the reference's sequential loop), nnz <= 1;
//   * stable sort by row, so the column order inside a row is the file order.
// Deviation: the reference throws (aborts) on a non-numeric row/col word; we reject the file.

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <numeric>
#include <random>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.hpp"

struct bsmr_csr {
    uint32_t M = 0, N = 0, nnz = 0;
    std::vector<uint32_t> rowptr, colidx;
    std::vector<float> values;
};

namespace bsmr {

static thread_local std::string g_error;
void set_error(const std::string& msg) { g_error = msg; }
const char* get_error() { return g_error.c_str(); }

namespace {

inline bool is_sep(char ch) { return ch == ' ' || ch == '\t' || ch == '\r'; }

// Word iterator equivalent to util::iterateOneWordFromLine.
struct Words {
    const char* p;
    const char* e;
    bool next(std::string& w) {
        const char* b = p;
        while (p < e && !is_sep(*p)) ++p;
        w.assign(b, p - b);
        while (p < e && is_sep(*p)) ++p;
        return !w.empty();
    }
};

// std::stoi semantics: strtol, at least one digit consumed, int range.
bool to_int(const std::string& w, long& out) {
    if (w.empty()) return false;
    errno = 0;
    char* endp = nullptr;
    const long v = std::strtol(w.c_str(), &endp, 10);
    if (endp == w.c_str() || errno == ERANGE || v < INT_MIN || v > INT_MAX) return false;
    out = v;
    return true;
}

// 1 = parsed, 0 = blank line, -1 = unparsable
template <typename T>
int parse_line(const char* b, const char* e, uint32_t& x, uint32_t& y, T& v) {
    if (b == e) return 0;
    Words it{b, e};
    std::string w;
    long a, c;
    it.next(w);
    if (!to_int(w, a)) return -1;
    it.next(w);
    if (!to_int(w, c)) return -1;
    x = static_cast<uint32_t>(static_cast<int>(a));
    y = static_cast<uint32_t>(static_cast<int>(c));
    it.next(w);
    if (w.empty()) {
        v = static_cast<T>(0);
        return 1;
    }
    errno = 0;
    char* endp = nullptr;
    const double d = std::strtod(w.c_str(), &endp);
    if (endp == w.c_str()) return -1;
    if (errno == ERANGE) {
        std::cout << "Warning: valueStr out of range: " << w << std::endl;
        v = static_cast<T>(0);
        return 1;
    }
    v = static_cast<T>(d);
    return 1;
}

}  // namespace
}  // namespace bsmr

using namespace bsmr;

extern "C" const char* bsmr_last_error(void) { return get_error(); }
extern "C" int bsmr_abi_version(void) { return BSMR_ABI_VERSION; }

extern "C" int bsmr_csr_load_mtx(const char* path, int verbose, bsmr_csr** out) {
    *out = nullptr;
    const std::string file(path ? path : "");
    const size_t dot = file.find_last_of('.');
    const std::string suffix = dot == std::string::npos ? std::string() : file.substr(dot);
    if (suffix != ".mtx" && suffix != ".mmio") {
        std::cerr << "Error, file format is not supported : " << file << std::endl;
        set_error("unsupported file suffix: " + file);
        return BSMR_ERR_UNSUPPORTED;
    }
    std::ifstream in(file, std::ios::binary);
    if (!in.is_open()) {
        std::cerr << "Error, file cannot be opened : " << file << std::endl;
        set_error("cannot open " + file);
        return BSMR_ERR_IO;
    }
    if (verbose) std::cout << "sparseMatrix::CSR initialize from file : " << file << std::endl;
    std::string buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    const char* p = buf.data();
    const char* end = p + buf.size();
    auto next_line = [&](const char*& lb, const char*& le) -> bool {
        if (p >= end) return false;
        lb = p;
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', end - p));
        le = nl ? nl : end;
        p = nl ? nl + 1 : end;
        return true;
    };
    auto reject = [&](const std::string& msg, int code) {
        std::cerr << msg << std::endl;
        set_error(msg);
        return code;
    };
    const char *lb = nullptr, *le = nullptr;
    bool got = false;
    while (next_line(lb, le)) {
        got = true;
        if (lb == le || *lb != '%') break;
    }
    uint32_t M = 0, N = 0, nnz = 0;
    if (!got || parse_line(lb, le, M, N, nnz) != 1 || M == NULLV || N == NULLV || nnz == NULLV)
        return reject("Error, file " + file + " format is incorrect!", BSMR_ERR_IO);

    std::vector<uint32_t> ri, ci;
    std::vector<float> vv;
    ri.reserve(nnz);
    ci.reserve(nnz);
    vv.reserve(nnz);
    uint64_t count = 0;
    while (next_line(lb, le)) {
        uint32_t r = NULLV, c = NULLV;
        float v = 0.f;
        const int st = parse_line(lb, le, r, c, v);
        if (st == 0) continue;
        if (st < 0) return reject("Error, file " + file + " format is incorrect!", BSMR_ERR_IO);
        if (count >= nnz)
            return reject("Error, file " + file + " too many elements, exceeding the number nnz!",
                          BSMR_ERR_REJECTED);
        ri.push_back(r - 1);
        ci.push_back(c - 1);
        vv.push_back(v);
        ++count;
    }
    if (count < nnz)
        return reject("Error, file " + file + " elements is not enough!", BSMR_ERR_REJECTED);

    // First offending entry in file order: out of range vs. repeat of an earlier (r, c).
    uint64_t first_oob = UINT64_MAX;
    for (uint64_t i = 0; i < nnz; ++i)
        if (ri[i] >= M || ci[i] >= N) {
            first_oob = i;
            break;
        }
    uint64_t first_dup = UINT64_MAX;
    {
        const uint64_t lim = std::min<uint64_t>(first_oob, nnz);
        std::vector<uint32_t> ord(lim);
        std::iota(ord.begin(), ord.end(), 0u);
        std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
            if (ri[a] != ri[b]) return ri[a] < ri[b];
            if (ci[a] != ci[b]) return ci[a] < ci[b];
            return a < b;
        });
        for (uint64_t k = 1; k < lim; ++k)
            if (ri[ord[k]] == ri[ord[k - 1]] && ci[ord[k]] == ci[ord[k - 1]])
                first_dup = std::min<uint64_t>(first_dup, ord[k]);
    }
    if (first_oob != UINT64_MAX && first_oob < first_dup)
        return reject("Error, file " + file + " row or col is too big!", BSMR_ERR_REJECTED);
    if (first_dup != UINT64_MAX) return reject("Error, matrix has duplicate data!", BSMR_ERR_REJECTED);
    if (nnz <= 1)
        return reject("Warning, file " + file + " nnz is 1, this is not a valid matrix!",
                      BSMR_ERR_REJECTED);

    auto* s = new bsmr_csr;
    s->M = M;
    s->N = N;
    s->nnz = nnz;
    // stable counting sort by row (== thrust host stable sort_by_key)
    s->rowptr.assign(static_cast<size_t>(M) + 1, 0);
    for (uint64_t i = 0; i < nnz; ++i) ++s->rowptr[ri[i] + 1];
    for (uint32_t r = 0; r < M; ++r) s->rowptr[r + 1] += s->rowptr[r];
    std::vector<uint32_t> fill(s->rowptr.begin(), s->rowptr.end() - 1);
    s->colidx.resize(nnz);
    s->values.resize(nnz);
    for (uint64_t i = 0; i < nnz; ++i) {
        const uint32_t dst = fill[ri[i]]++;
        s->colidx[dst] = ci[i];
        s->values[dst] = vv[i];
    }
    *out = s;
    return BSMR_OK;
}

namespace {

// whole-file line reader ('\n'-separated; '\r' is a word separator as in the reference)
struct Lines {
    std::string buf;
    const char* p = nullptr;
    const char* end = nullptr;
    bool open(const std::string& file) {
        std::ifstream in(file, std::ios::binary);
        if (!in.is_open()) return false;
        buf.assign((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
        p = buf.data();
        end = p + buf.size();
        return true;
    }
    bool next(const char*& lb, const char*& le) {
        if (p >= end) return false;
        lb = p;
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', end - p));
        le = nl ? nl : end;
        p = nl ? nl + 1 : end;
        return true;
    }
};

int reject_msg(const std::string& msg, int code) {
    std::cerr << msg << std::endl;
    set_error(msg);
    return code;
}

// stable counting sort of (row, col, value) triples into CSR (file order kept inside a row)
bsmr_csr* to_csr(uint32_t M, uint32_t N, const std::vector<uint32_t>& ri,
                 const std::vector<uint32_t>& ci, const std::vector<float>& vv) {
    auto* s = new bsmr_csr;
    s->M = M;
    s->N = N;
    s->nnz = static_cast<uint32_t>(ri.size());
    s->rowptr.assign(static_cast<size_t>(M) + 1, 0);
    for (uint32_t r : ri) ++s->rowptr[r + 1];
    for (uint32_t r = 0; r < M; ++r) s->rowptr[r + 1] += s->rowptr[r];
    std::vector<uint32_t> fill(s->rowptr.begin(), s->rowptr.end() - 1);
    s->colidx.resize(ri.size());
    s->values.resize(ri.size());
    for (size_t i = 0; i < ri.size(); ++i) {
        const uint32_t dst = fill[ri[i]]++;
        s->colidx[dst] = ci[i];
        s->values[dst] = vv[i];
    }
    return s;
}

// index of the first entry (in file order) that repeats an earlier (row, col) pair, or n
size_t first_duplicate(const std::vector<uint32_t>& ri, const std::vector<uint32_t>& ci, size_t n) {
    std::vector<uint32_t> ord(n);
    std::iota(ord.begin(), ord.end(), 0u);
    std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
        if (ri[a] != ri[b]) return ri[a] < ri[b];
        if (ci[a] != ci[b]) return ci[a] < ci[b];
        return a < b;
    });
    size_t first = n;
    for (size_t k = 1; k < n; ++k)
        if (ri[ord[k]] == ri[ord[k - 1]] && ci[ord[k]] == ci[ord[k - 1]]) first = std::min<size_t>(first, ord[k]);
    return first;
}

}  // namespace

// .smtx (DLMC) — CSR::initializeFromSmtxFile (src/Matrix.cpp:296-371): '%' lines skipped, header
// "rows cols nnz" (nnz == 0 rejected), one line of rows+1 row offsets, one line of nnz column
// indices, values 1, a column repeated inside a row rejected, column order = file order.
// Deviations (the reference throws on a short or non-numeric line and does not validate the
// offsets or the column range): all rejected with the messages below.
extern "C" int bsmr_csr_load_smtx(const char* path, int verbose, bsmr_csr** out) {
    *out = nullptr;
    const std::string file(path ? path : "");
    Lines L;
    if (!L.open(file)) return reject_msg("Error, file cannot be opened : " + file, BSMR_ERR_IO);
    if (verbose) std::cout << "sparseMatrix::CSR initialize From file : " << file << std::endl;
    const char *lb = nullptr, *le = nullptr;
    bool got = false;
    while (L.next(lb, le)) {
        got = true;
        if (lb == le || *lb != '%') break;
    }
    long hdr[3];
    {
        Words it{lb, le};
        std::string w;
        for (long& h : hdr) {
            it.next(w);
            if (!got || !to_int(w, h) || h < 0)
                return reject_msg("Error, file " + file + " format is incorrect!", BSMR_ERR_IO);
        }
    }
    const uint32_t M = static_cast<uint32_t>(hdr[0]), N = static_cast<uint32_t>(hdr[1]);
    const uint32_t nnz = static_cast<uint32_t>(hdr[2]);
    if (nnz == 0) return reject_msg("Error, file " + file + " nnz is 0!", BSMR_ERR_REJECTED);
    auto read_ints = [&](std::vector<uint32_t>& dst) {
        if (!L.next(lb, le)) return false;
        Words it{lb, le};
        std::string w;
        for (uint32_t& v : dst) {
            long x;
            it.next(w);
            if (!to_int(w, x) || x < 0) return false;
            v = static_cast<uint32_t>(x);
        }
        return true;
    };
    auto* s = new bsmr_csr;
    s->M = M;
    s->N = N;
    s->nnz = nnz;
    s->rowptr.resize(static_cast<size_t>(M) + 1);
    s->colidx.resize(nnz);
    s->values.assign(nnz, 1.f);
    auto fail = [&](const std::string& msg, int code) {
        delete s;
        return reject_msg(msg, code);
    };
    if (!read_ints(s->rowptr)) return fail("Error, file " + file + " rowOffsets is not enough!", BSMR_ERR_IO);
    if (!read_ints(s->colidx)) return fail("Error, file " + file + " nnz is not enough!", BSMR_ERR_IO);
    if (s->rowptr[0] != 0 || s->rowptr[M] != nnz)
        return fail("Error, file " + file + " format is incorrect!", BSMR_ERR_IO);
    for (uint32_t r = 0; r < M; ++r)
        if (s->rowptr[r] > s->rowptr[r + 1]) return fail("Error, file " + file + " format is incorrect!", BSMR_ERR_IO);
    std::vector<uint32_t> mark(N, NULLV);  // last row that used column c
    for (uint32_t r = 0; r < M; ++r)
        for (uint32_t k = s->rowptr[r]; k < s->rowptr[r + 1]; ++k) {
            const uint32_t c = s->colidx[k];
            if (c >= N) return fail("Error, file " + file + " row or col is too big!", BSMR_ERR_REJECTED);
            if (mark[c] == r) return fail("Error, matrix has duplicate data!", BSMR_ERR_REJECTED);
            mark[c] = r;
        }
    *out = s;
    return BSMR_OK;
}

// SNAP edge list (.txt) — CSR::initializeFromGraphDataset (src/Matrix.cpp:482-575): leading '#'
// lines carry "Nodes: n" and "Edges: e" (rows = cols = n, nnz = e); then "from to [value]" lines
// (blank skipped); node ids renumbered 0, 1, .. by first appearance (from, then to); more than e
// edges, fewer, an id >= n or a repeated pair rejected (first offending edge in file order
// decides); stable sort by row. No mirroring (directed edges as listed).
extern "C" int bsmr_csr_load_snap(const char* path, int verbose, bsmr_csr** out) {
    *out = nullptr;
    const std::string file(path ? path : "");
    Lines L;
    if (!L.open(file)) return reject_msg("Error, file cannot be opened : " + file, BSMR_ERR_IO);
    if (verbose) std::cout << "sparseMatrix::CSR initialize From file : " << file << std::endl;
    const char *lb = nullptr, *le = nullptr;
    long nodes = 0, edges = 0;
    bool data = false;
    while (L.next(lb, le)) {
        if (lb == le || *lb != '#') {
            data = true;
            break;
        }
        const std::string line(lb, le);
        for (const char* key : {"Nodes: ", "Edges: "}) {
            const size_t at = line.find(key);
            if (at == std::string::npos) continue;
            Words it{line.data() + at + 7, line.data() + line.size()};
            std::string w;
            it.next(w);
            long v;
            if (!to_int(w, v) || v < 0) return reject_msg("Error, file " + file + " format is incorrect!", BSMR_ERR_IO);
            (key[0] == 'N' ? nodes : edges) = v;
        }
    }
    if (!nodes || !edges)
        return reject_msg("Error, file " + file + " row or col or nnz not initialized!", BSMR_ERR_REJECTED);
    const uint32_t n = static_cast<uint32_t>(nodes), e = static_cast<uint32_t>(edges);
    std::vector<uint32_t> ri, ci;
    std::vector<float> vv;
    ri.reserve(e);
    ci.reserve(e);
    vv.reserve(e);
    std::unordered_map<uint32_t, uint32_t> id;
    auto renum = [&](uint32_t node) {
        const auto ins = id.emplace(node, static_cast<uint32_t>(id.size()));
        return ins.first->second;
    };
    for (bool have = data; have; have = L.next(lb, le)) {
        uint32_t a = 0, b = 0;
        float v = 0.f;
        const int st = parse_line(lb, le, a, b, v);
        if (st == 0) continue;
        if (st < 0) return reject_msg("Error, file " + file + " format is incorrect!", BSMR_ERR_IO);
        const uint32_t ra = renum(a), rb = renum(b);
        if (ri.size() >= e)
            return reject_msg("Error, file " + file + " too many elements, exceeding the number nnz!",
                              BSMR_ERR_REJECTED);
        ri.push_back(ra);
        ci.push_back(rb);
        vv.push_back(v);
    }
    if (ri.size() < e) return reject_msg("Error, file " + file + " elements is not enough!", BSMR_ERR_REJECTED);
    size_t first_oob = e;
    for (size_t i = 0; i < e; ++i)
        if (ri[i] >= n || ci[i] >= n) {
            first_oob = i;
            break;
        }
    // a repeat before the first out-of-range edge decides first (== first_oob: no repeat there)
    if (first_duplicate(ri, ci, first_oob) < first_oob)
        return reject_msg("Error, matrix has duplicate data!", BSMR_ERR_REJECTED);
    if (first_oob < e) return reject_msg("Error, file " + file + " row or col is too big!", BSMR_ERR_REJECTED);
    *out = to_csr(n, n, ri, ci, vv);
    return BSMR_OK;
}

// CSR::initializeFromMatrixFile (src/Matrix.cpp:279-294): dispatch on the last '.' suffix
extern "C" int bsmr_csr_load(const char* path, int verbose, bsmr_csr** out) {
    *out = nullptr;
    const std::string file(path ? path : "");
    const size_t dot = file.find_last_of('.');
    const std::string suffix = dot == std::string::npos ? std::string() : file.substr(dot);
    if (suffix == ".mtx" || suffix == ".mmio") return bsmr_csr_load_mtx(path, verbose, out);
    if (suffix == ".smtx") return bsmr_csr_load_smtx(path, verbose, out);
    if (suffix == ".txt") return bsmr_csr_load_snap(path, verbose, out);
    std::cerr << "Error, file format is not supported : " << file << std::endl;
    set_error("unsupported file suffix: " + file);
    return BSMR_ERR_UNSUPPORTED;
}

extern "C" int bsmr_csr_create(uint32_t M, uint32_t N, uint32_t nnz, const uint32_t* rowptr,
                               const uint32_t* colidx, bsmr_csr** out) {
    *out = nullptr;
    if (!rowptr || !colidx || rowptr[M] != nnz) {
        set_error("bsmr_csr_create: rowptr[M] != nnz or null arrays");
        return BSMR_ERR_INVALID;
    }
    auto* s = new bsmr_csr;
    s->M = M;
    s->N = N;
    s->nnz = nnz;
    s->rowptr.assign(rowptr, rowptr + M + 1);
    s->colidx.assign(colidx, colidx + nnz);
    s->values.assign(nnz, 0.f);
    *out = s;
    return BSMR_OK;
}

extern "C" void bsmr_csr_info(const bsmr_csr* s, uint32_t* M, uint32_t* N, uint32_t* nnz) {
    if (M) *M = s->M;
    if (N) *N = s->N;
    if (nnz) *nnz = s->nnz;
}
extern "C" const uint32_t* bsmr_csr_rowptr(const bsmr_csr* s) { return s->rowptr.data(); }
extern "C" const uint32_t* bsmr_csr_colidx(const bsmr_csr* s) { return s->colidx.data(); }
extern "C" const float* bsmr_csr_values(const bsmr_csr* s) { return s->values.data(); }
extern "C" void bsmr_csr_free(bsmr_csr* s) { delete s; }

// Matrix<T>::makeData (src/Matrix.cpp:117-138): fresh default-seeded std::mt19937 and
// uniform_real_distribution<float>(0, 2) from the same libstdc++; single-threaded, so the
// stream is deterministic (the reference shares one engine across OpenMP threads).
extern "C" void bsmr_make_data(uint64_t n, float* out) {
    std::mt19937 gen;
    std::uniform_real_distribution<float> dist(0.0f, 2.0f);
    for (uint64_t i = 0; i < n; ++i) out[i] = dist(gen);
}
