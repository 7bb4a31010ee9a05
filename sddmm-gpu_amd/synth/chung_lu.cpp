// chung_lu.cpp — synthetic power-law graph for the C4 (reddit-like) workload (bench/test input
// generation only; not part of the SDDMM engine). Built as lib/libbsmr_synth.so, called from
// bsmr/synth.py.
//
// Model (Chung-Lu, as SURVEY.md §8d C4): endpoints drawn with probability proportional to
// w_i = (i+1)^(-1/(exponent-1)) (alias method) over a seeded random relabelling of the nodes, self loops
// dropped, each undirected edge kept once, until `target` distinct edges exist; exactly `target`
// of them are kept (the smallest seeded 64-bit hashes), then both directions are stored with
// ascending columns per row. Every random number comes from a fixed (seed, round, chunk) stream,
// so the pattern does not depend on the thread count.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <parallel/algorithm>
#include <vector>

namespace {

uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Xoshiro {  // xoshiro256**
    uint64_t s[4];
    explicit Xoshiro(uint64_t seed) {
        for (auto& v : s) v = splitmix64(seed);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
};

uint64_t mix(uint64_t a, uint64_t b) {
    uint64_t x = a ^ (b * 0x9E3779B97F4A7C15ull);
    return splitmix64(x);
}

constexpr int CHUNKS = 512;  // fixed work split: the streams do not depend on the thread count

}  // namespace

extern "C" int bsmr_synth_chung_lu(uint32_t n, uint64_t nnz_target, uint64_t seed, double exponent,
                                   uint32_t* rowptr, uint32_t* colidx) {
    if (n < 2 || nnz_target < 2) return 1;
    const uint64_t target = nnz_target / 2;
    if (target > static_cast<uint64_t>(n) * (n - 1) / 2) return 1;
    // node weights -> Walker/Vose alias table (one uniform index + one compare per draw), with
    // the node relabelling folded into the table
    std::vector<double> w(n);
    double acc = 0.0;
    for (uint32_t i = 0; i < n; ++i) acc += (w[i] = std::pow(static_cast<double>(i + 1), -1.0 / (exponent - 1.0)));
    std::vector<uint32_t> perm(n);
    std::iota(perm.begin(), perm.end(), 0u);
    {
        Xoshiro g(mix(seed, 0xA11CEull));
        for (uint32_t i = n - 1; i > 0; --i) std::swap(perm[i], perm[g.next() % (i + 1ull)]);
    }
    struct Slot {
        double p;
        uint32_t self, alias;
    };
    std::vector<Slot> tab(n);
    {
        std::vector<uint32_t> small, large;
        std::vector<double> q(n);
        for (uint32_t i = 0; i < n; ++i) {
            q[i] = w[i] * n / acc;
            (q[i] < 1.0 ? small : large).push_back(i);
        }
        while (!small.empty() && !large.empty()) {
            const uint32_t s = small.back(), l = large.back();
            small.pop_back();
            tab[s] = {q[s], perm[s], perm[l]};
            q[l] = (q[l] + q[s]) - 1.0;
            if (q[l] < 1.0) {
                large.pop_back();
                small.push_back(l);
            }
        }
        for (uint32_t i : large) tab[i] = {1.0, perm[i], perm[i]};
        for (uint32_t i : small) tab[i] = {1.0, perm[i], perm[i]};
    }
    auto node = [&](Xoshiro& g) {
        const uint64_t r = g.next();
        const Slot& t = tab[static_cast<uint32_t>(((r >> 32) * n) >> 32)];
        return static_cast<double>(r & 0xFFFFFFFFull) * 0x1.0p-32 < t.p ? t.self : t.alias;
    };
    std::vector<uint64_t> edges;
    // one round usually suffices: the hub pairs repeat, ~1/4 of the draws are duplicates
    uint64_t draw = target + target * 2 / 5, drawn_total = 0;
    for (uint64_t round = 0;; ++round) {
        std::vector<std::vector<uint64_t>> part(CHUNKS);
#pragma omp parallel for schedule(dynamic, 1)
        for (int c = 0; c < CHUNKS; ++c) {
            const uint64_t lo = draw * c / CHUNKS, hi = draw * (c + 1) / CHUNKS;
            Xoshiro g(mix(mix(seed, round + 1), static_cast<uint64_t>(c)));
            auto& v = part[c];
            v.reserve(hi - lo);
            for (uint64_t d = lo; d < hi; ++d) {
                const uint32_t i = node(g), j = node(g);
                if (i != j) v.push_back(static_cast<uint64_t>(std::min(i, j)) * n + std::max(i, j));
            }
        }
        size_t total = edges.size();
        for (auto& v : part) total += v.size();
        edges.reserve(total);
        for (auto& v : part) {
            edges.insert(edges.end(), v.begin(), v.end());
            std::vector<uint64_t>().swap(v);
        }
        __gnu_parallel::sort(edges.begin(), edges.end());
        edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
        drawn_total += draw;
        if (edges.size() >= target) break;
        // distinct edges per draw fall as the graph fills: ask for the shortfall at the current
        // yield, plus a margin
        draw = std::max<uint64_t>(1000000, static_cast<uint64_t>(
                                               (target - edges.size()) * 1.5 * drawn_total /
                                               std::max<size_t>(edges.size(), 1)));
    }
    if (edges.size() > target) {  // keep the `target` edges of smallest seeded hash
        const size_t E = edges.size();
        std::vector<uint64_t> h(E);
        const uint64_t hs = mix(seed, 0x5E1EC7ull);
#pragma omp parallel for
        for (size_t e = 0; e < E; ++e) h[e] = mix(edges[e], hs);
        std::vector<uint64_t> hc(h);
        __gnu_parallel::nth_element(hc.begin(), hc.begin() + (target - 1), hc.end());
        const uint64_t thr = hc[target - 1];
        std::vector<uint64_t>().swap(hc);
        size_t k = 0, below = 0;
        for (size_t e = 0; e < E; ++e) below += h[e] < thr;
        size_t at_thr = target - below;  // ties at the threshold: the first ones in key order
        for (size_t e = 0; e < E; ++e)
            if (h[e] < thr || (h[e] == thr && at_thr && at_thr--)) edges[k++] = edges[e];
        edges.resize(k);
    }
    // CSR of both directions: row r = [lo of edges (lo, r)] ++ [hi of edges (r, hi)], each part
    // ascending because the edges are sorted by (lo, hi)
    std::vector<uint32_t> lower(n, 0), upper(n, 0);
    for (uint64_t e : edges) {
        ++upper[e / n];
        ++lower[e % n];
    }
    rowptr[0] = 0;
    for (uint32_t r = 0; r < n; ++r) rowptr[r + 1] = rowptr[r] + lower[r] + upper[r];
    std::vector<uint32_t> lcur(n), ucur(n);
    for (uint32_t r = 0; r < n; ++r) {
        lcur[r] = rowptr[r];
        ucur[r] = rowptr[r] + lower[r];
    }
    for (uint64_t e : edges) {
        const uint32_t lo = static_cast<uint32_t>(e / n), hi = static_cast<uint32_t>(e % n);
        colidx[ucur[lo]++] = hi;
        colidx[lcur[hi]++] = lo;
    }
    return 0;
}
