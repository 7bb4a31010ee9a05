// cluster_filter.hip — the clustering's candidate filter: an upper bound of every pairwise
// similarity, computed on the matrix cores before the first-fit chain runs (plan.hip k_cluster).
//
// Similarity (rowReordering.cu:235-293; oracle.cpp similarity_exact): for a representative with
// kept block counts a_i and norm nr = sqrt(sum a_i^2), a row with counts b_i and norm nc,
//     mn = sum_i min(a_i / nr, b_i / nc),   S = S1R / nr + S1C / nc,   sim = mn / (S - mn),
// and sim > alpha  <=>  mn (1 + alpha) > alpha S. Since min(x, y) <= sqrt(x y) for x, y >= 0,
//     mn <= sum_i sqrt(a_i b_i) / sqrt(nr nc) = G / (sqrt(nr) sqrt(nc)),   G = <sqrt a, sqrt b>,
// exact for 0/1 counts (graph rows: most blocks hold one entry). G of every pair of rows is one
// GEMM X X^T over the block dimension, X[p][i] = sqrt(b_i) of the row at position p (fp16,
// rounded up, non-kept blocks 0). A pair whose bound cannot reach the accept threshold,
//     G (1 + alpha) 1.01 <= alpha (u_q + u_p) sq_q sq_p     (u = S1 / n, sq = sqrt(n)),
// is a certain reject; the 1 % margin covers the fp16 rounding (upwards), the fp32 accumulation
// and the < 3e-6 error of the exact fp32 tree the chain decides with. The chain (k_cluster) skips
// a cluster for a position when the cluster is still its leader row alone and the pair's bit is
// clear; clusters that took more rows, and every pair whose bit is set, are evaluated as before,
// so the permutation is the same.
//
// Bits: positions are the dispersion-ascending order the chain walks (pmeta); row q of the
// triangle holds 32-bit words [q / 32, W) (W = ceil(M / 32)), bit p of word p / 32 set when the
// pair (leader q, position p > q) may accept (plan_kernels.hpp fbits_row_offset).
//
// GEMM: 128 x 128 tiles of the upper triangle (tm <= tn), one 256-thread workgroup each, the
// 64-wide k-chunks of the two 128-row panels streamed through a 2-stage LDS ring by LDS-DMA (the
// structure of sddmm_dense.hip), `v_mfma_f32_16x16x32_f16`, each wave a 64 x 64 quadrant; the
// epilogue compares in registers and ballots the bits. XCD x takes a contiguous range of tiles,
// so the tile row's A panel stays in its L2.
#include <algorithm>
#include <cmath>

#include "common.hpp"
#include "plan.hpp"
#include "plan_kernels.hpp"

namespace bsmr {
namespace {

using dev::fbits_row_offset;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));

constexpr u32 FT = 128;                 // output tile edge
constexpr u32 FKC = 64;                 // k-chunk (halves) per stage
constexpr u32 FCB = FT * FKC * 2;       // one operand chunk image (16 KiB)
constexpr u32 FNW = 4;                  // waves per workgroup (64 x 64 quadrant each)
constexpr u32 FND = FKC / 16 * 4 / FNW; // LDS-DMAs per wave and operand per chunk (4)

struct FilterArgs {
    const _Float16* X;  // [M][Kp]
    const float2* us;   // per position {u, sq}; u = -1e30 marks "always a candidate"
    u32* bits;
    u32 M, Kp, W, ntm, ntiles;
    float c1, alpha;    // (1 + alpha) * 1.01, alpha
};

// slot of (row r, 16-byte group g) in a chunk image: XOR-permuted so the 16 lanes of a
// ds_read_b128 lane group (rows l & 15, one group) hit distinct bank groups (sddmm_dense.hip)
__device__ __forceinline__ u32 fslot(u32 r, u32 g) { return (FKC / 8) * r + (g ^ ((r >> 1) & 7)); }

__device__ __forceinline__ void lds_dma16(const char* g, char* l) {
    const u32 m0 = __builtin_amdgcn_readfirstlane(static_cast<u32>(
        reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)l)));
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0)
                 : "memory", "m0");
}

__device__ __forceinline__ void fstage(const FilterArgs& a, const u32 r0, const u32 c0, const u32 kc,
                                       const u32 ws, const u32 lane, char* sa, char* sb) {
    constexpr u32 GP = FKC / 8;
    const size_t rowB = static_cast<size_t>(a.Kp) * 2;
#pragma unroll
    for (u32 i = 0; i < FND; ++i) {
        const u32 s = 64 * (FND * ws + i) + lane, r = s / GP, g = (s % GP) ^ ((r >> 1) & 7);
        const u32 ra = min(r0 + r, a.M - 1), rb = min(c0 + r, a.M - 1);
        const size_t ko = static_cast<size_t>(kc) * (FKC * 2) + 16 * g;
        const char* X = reinterpret_cast<const char*>(a.X);
        lds_dma16(X + ra * rowB + ko, sa + 1024 * (FND * ws + i));
        lds_dma16(X + rb * rowB + ko, sb + 1024 * (FND * ws + i));
    }
}

// tile t of the upper triangle, row-major: row tm holds tiles tn = tm .. ntm - 1
__device__ __forceinline__ void tile_of(u32 t, u32 ntm, u32& tm, u32& tn) {
    const double b = 2.0 * ntm + 1.0;
    u32 r = static_cast<u32>((b - sqrt(b * b - 8.0 * t)) / 2.0);
    auto start = [&](u32 x) { return static_cast<u64>(x) * ntm - static_cast<u64>(x) * (x - 1) / 2; };
    while (r > 0 && start(r) > t) --r;
    while (r + 1 < ntm && start(r + 1) <= t) ++r;
    tm = r;
    tn = r + static_cast<u32>(t - start(r));
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void k_sim_filter(FilterArgs a) {
    __shared__ __attribute__((aligned(16))) char st[2 * 2 * FCB];
    const u32 per = (a.ntiles + XCD_BUCKETS - 1) / XCD_BUCKETS;
    const u32 t = (blockIdx.x % XCD_BUCKETS) * per + blockIdx.x / XCD_BUCKETS;
    if (t >= a.ntiles) return;
    u32 tm, tn;
    tile_of(t, a.ntm, tm, tn);
    const u32 r0 = FT * tm, c0 = FT * tn;
    const u32 tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const u32 ws = __builtin_amdgcn_readfirstlane(w);
    const u32 wy = ws >> 1, wx = ws & 1;
    f32x4 acc[4][4];
#pragma unroll
    for (u32 i = 0; i < 4; ++i)
#pragma unroll
        for (u32 j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const u32 nk = a.Kp / FKC;
    fstage(a, r0, c0, 0, ws, lane, st, st + FCB);
    const u32 rr = lane & 15, g4 = lane >> 4;
    for (u32 kc = 0; kc < nk; ++kc) {
        // this wave's LDS-DMAs of chunk kc have landed; the barrier makes everyone's visible and
        // ends every read of the stage the next chunk overwrites
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if (kc + 1 < nk) {
            char* const sn = st + ((kc + 1) & 1) * (2 * FCB);
            fstage(a, r0, c0, kc + 1, ws, lane, sn, sn + FCB);
        }
        const char* const sa = st + (kc & 1) * (2 * FCB);
        const char* const sb = sa + FCB;
#pragma unroll
        for (u32 ks = 0; ks < FKC / 32; ++ks) {
            f32x4 av[4], bv[4];
#pragma unroll
            for (u32 i = 0; i < 4; ++i)
                av[i] = *reinterpret_cast<const f32x4*>(sa + 16 * fslot(64 * wy + 16 * i + rr, 4 * ks + g4));
#pragma unroll
            for (u32 j = 0; j < 4; ++j)
                bv[j] = *reinterpret_cast<const f32x4*>(sb + 16 * fslot(64 * wx + 16 * j + rr, 4 * ks + g4));
#pragma unroll
            for (u32 i = 0; i < 4; ++i)
#pragma unroll
                for (u32 j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                        __builtin_bit_cast(h16x8, av[i]), __builtin_bit_cast(h16x8, bv[j]), acc[i][j], 0, 0, 0);
        }
    }
    // epilogue: accumulator (i, j) reg r of lane l = G[64 wy + 16 i + 4 (l >> 4) + r][64 wx + 16 j + (l & 15)]
    float2 cu[4];
#pragma unroll
    for (u32 j = 0; j < 4; ++j) cu[j] = a.us[min(c0 + 64 * wx + 16 * j + rr, a.M - 1)];
    __syncthreads();  // every image read done: the stage memory takes the tile's bits
    unsigned long long* bt = reinterpret_cast<unsigned long long*>(st);  // [128 rows][2 halves]
#pragma unroll
    for (u32 i = 0; i < 4; ++i) {
#pragma unroll
        for (u32 r = 0; r < 4; ++r) {
            const u32 R = 64 * wy + 16 * i + 4 * g4 + r;
            const float2 ur = a.us[min(r0 + R, a.M - 1)];
            unsigned long long rb = 0;
#pragma unroll
            for (u32 j = 0; j < 4; ++j) {
                const float rhs = a.alpha * (ur.x + cu[j].x) * ur.y * cu[j].y;
                const bool cand = acc[i][j][r] * a.c1 > rhs;
                const unsigned long long m = __ballot(cand);
                rb |= ((m >> (16 * g4)) & 0xFFFFull) << (16 * j);
            }
            if (rr == 0) bt[2 * R + wx] = rb;
        }
    }
    __syncthreads();
    // rows q = r0 + R, words c0 / 32 + k (k < 4) that the triangle stores (>= q / 32, < W)
    const u32 R = tid >> 1, q = r0 + R;
    if (q < a.M) {
        const u64 base = fbits_row_offset(q, a.W);
        const u32 qw = q >> 5;
#pragma unroll
        for (u32 h = 0; h < 2; ++h) {
            const u32 k = 2 * (tid & 1) + h;
            const u32 wd = c0 / 32 + k;
            const unsigned long long v = bt[2 * R + (k >> 1)];
            const u32 word = static_cast<u32>(v >> (32 * (k & 1)));
            if (wd >= qw && wd < a.W) a.bits[base + (wd - qw)] = word;
        }
    }
}

// X rows (sqrt of the kept block counts, fp16 rounded up) and the per-position scalars
__global__ __launch_bounds__(64) void k_filter_x(const uint4* __restrict__ pmeta, const u32* __restrict__ enc,
                                                 u32 Kp, u32 B, u32 keptMask, _Float16* X, float2* us) {
    const u32 p = blockIdx.x, l = threadIdx.x;
    const uint4 m = pmeta[p];
    for (u32 e = l; e < m.y; e += 64) {
        const u32 ent = enc[m.x + e];
        const u32 blk = ent & 0xFFFFu, cnt = ent >> 16;
        if (!((keptMask >> ((blk % B) >> 5)) & 1u)) continue;
        const float f = sqrtf(static_cast<float>(cnt)) * 1.000001f;
        _Float16 h = static_cast<_Float16>(f);
        if (static_cast<float>(h) < f) {  // round up: the next fp16 (positive, finite)
            unsigned short b = __builtin_bit_cast(unsigned short, h);
            h = __builtin_bit_cast(_Float16, static_cast<unsigned short>(b + 1));
        }
        X[static_cast<size_t>(p) * Kp + blk] = h;
    }
    if (l == 0) {
        // SC = 0 (no kept entry): the chain's special cases decide; always a candidate
        float2 v = make_float2(-1e30f, 1.0f);
        if (m.z != 0) {
            const float nr = sqrtf(static_cast<float>(m.z));
            v = make_float2(static_cast<float>(m.w) / nr, sqrtf(nr));
        }
        us[p] = v;
    }
}

}  // namespace

u64 sim_filter_words(u32 M) {
    const u32 W = (M + 31) / 32;
    return dev::fbits_row_offset(M, W);
}

int build_sim_filter(const uint4* pmeta, const u32* enc, u32 M, u32 nbpr, u32 B, u32 keptMask, float alpha,
                     DevBuf<u32>& bits, u32& W, hipStream_t s) {
    const u32 Kp = (nbpr + FKC - 1) / FKC * FKC;
    W = (M + 31) / 32;
    DevBuf<_Float16> X;
    DevBuf<float2> us;
    BSMR_CHECK(X.alloc(static_cast<size_t>(M) * Kp));
    BSMR_CHECK(us.alloc(M));
    BSMR_CHECK(bits.alloc(std::max<u64>(sim_filter_words(M), 1)));
    BSMR_HIP(hipMemsetAsync(X.data(), 0, static_cast<size_t>(M) * Kp * sizeof(_Float16), s));
    hipLaunchKernelGGL(k_filter_x, dim3(M), dim3(64), 0, s, pmeta, enc, Kp, B, keptMask, X.data(), us.data());
    BSMR_HIP(hipGetLastError());
    FilterArgs a{};
    a.X = X.data();
    a.us = us.data();
    a.bits = bits.data();
    a.M = M;
    a.Kp = Kp;
    a.W = W;
    a.ntm = (M + FT - 1) / FT;
    a.ntiles = static_cast<u32>(static_cast<u64>(a.ntm) * (a.ntm + 1) / 2);
    a.alpha = alpha;
    a.c1 = (1.0f + alpha) * 1.01f;
    const u32 per = (a.ntiles + XCD_BUCKETS - 1) / XCD_BUCKETS;
    hipLaunchKernelGGL(k_sim_filter, dim3(per * XCD_BUCKETS), dim3(256), 0, s, a);
    BSMR_HIP(hipGetLastError());
    // X and us are freed on return: wait for the kernels that read them
    BSMR_HIP(hipStreamSynchronize(s));
    return BSMR_OK;
}

}  // namespace bsmr
