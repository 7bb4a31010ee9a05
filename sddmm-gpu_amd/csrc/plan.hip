// plan.hip — BSMR reordering and tile layout, built on the GPU (gfx950).
//
// Pipeline (reference functions in brackets; file:line relative to the reference root):
//   1. k_encode        per-row LDS histogram of col/bs -> sparse encoding, dispersion, norms
//                      [kernel::calculateDispersion, rowReordering.cu:49-93, 478-501]
//   2. radix sort      rows stably by dispersion [host::sort_by_key, rowReordering.cu:1055-1062]
//   3. k_cluster       similarity clustering as a persistent chain of cluster tiles
//                      [bsa_clustering + get_permutation_gpu, rowReordering.cu:215-432, 893-1007]
//   4. radix sort      positions stably by cluster id -> reorderedRows [rowReordering.cu:988-996,
//                      1081-1090]
//   5. k_gather + segmented radix sort + k_panel_pass1/2: per-16-row-panel column histogram,
//                      count-descending order, dense/sparse split and the RPHM tile/residual
//                      arrays [colReordering_cpu, colReordering.cu:244-404; RPHM::RPHM,
//                      BSMR.cpp:83-265]
//   6. k_items         compact work lists for the SDDMM launch (replaces the reference's 2-D
//                      panels x maxBlocks grid, sddmmKernel.cu:2570-2581)
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <queue>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "plan.hpp"
#include "plan_kernels.hpp"

namespace bsmr {
namespace {

using namespace dev;

// ------------------------------------------------------------------------------------------
// 1. Row encodings. One 256-thread workgroup per row: LDS histogram over the nbpr column
// blocks, then an ordered compaction (ascending block id) into enc[rowptr[r] ...] as
// (count << 16 | block). Also: #blocks, dispersion (u32, as the reference's sum), and the
// "kept" integer norms used by the clustering similarity.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ bool kept_idx(u32 i, u32 B, u32 keptMask) {
    return (keptMask >> ((i % B) >> 5)) & 1u;
}

__global__ __launch_bounds__(256) void k_encode(const u32* __restrict__ rowptr,
                                                const u32* __restrict__ col, u32 M, u32 bs,
                                                u32 nbpr, u32 B, u32 keptMask,
                                                u32* __restrict__ enc, u32* __restrict__ nblk,
                                                u32* __restrict__ disp, u32* __restrict__ SC,
                                                u32* __restrict__ S1C) {
    extern __shared__ __attribute__((aligned(16))) u32 smem[];
    u32* hist = smem;                 // nbpr
    u32* red = smem + ((nbpr + 3) & ~3u);  // 4 waves x 4 values
    const u32 r = blockIdx.x;
    const u32 t = threadIdx.x, lane = t & 63, w = t >> 6;
    const u32 b0 = rowptr[r], n = rowptr[r + 1] - b0;
    if (n == 0) {
        if (t == 0) {
            nblk[r] = 0;
            disp[r] = 0;
            SC[r] = 0;
            S1C[r] = 0;
        }
        return;
    }
    for (u32 i = t; i < nbpr; i += 256) hist[i] = 0;
    __syncthreads();
    for (u32 k = t; k < n; k += 256) atomicAdd(&hist[col[b0 + k] / bs], 1u);
    __syncthreads();
    const u32 chunk = (nbpr + 255) / 256;
    const u32 i0 = min(t * chunk, nbpr), i1 = min(i0 + chunk, nbpr);
    u32 cnz = 0, dsum = 0, sq = 0, s1 = 0;
    for (u32 i = i0; i < i1; ++i) {
        const u32 e = hist[i];
        if (e) {
            ++cnz;
            dsum += bs - e;
            if (kept_idx(i, B, keptMask)) {
                sq += e * e;
                s1 += e;
            }
        }
    }
    const u32 incl = wave_incl_scan(cnz);
    const u32 wd = wave_sum(dsum), wq = wave_sum(sq), ws = wave_sum(s1);
    if (lane == 63) {
        red[w * 4 + 0] = incl;
        red[w * 4 + 1] = wd;
        red[w * 4 + 2] = wq;
        red[w * 4 + 3] = ws;
    }
    __syncthreads();
    u32 base = 0, tot = 0;
    for (u32 j = 0; j < 4; ++j) {
        if (j < w) base += red[j * 4];
        tot += red[j * 4];
    }
    u32 off = b0 + base + incl - cnz;
    for (u32 i = i0; i < i1; ++i) {
        const u32 e = hist[i];
        if (e) enc[off++] = (e << 16) | i;
    }
    if (t == 0) {
        u32 d = 0, q = 0, s = 0;
        for (u32 j = 0; j < 4; ++j) {
            d += red[j * 4 + 1];
            q += red[j * 4 + 2];
            s += red[j * 4 + 3];
        }
        nblk[r] = tot;
        disp[r] = d + n * tot;  // sum_{b}(bs - e_b) + nnz * #b, u32 wrap like the reference
        SC[r] = q;
        S1C[r] = s;
    }
}

__global__ void k_iota(u32* p, u32 n) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = i;
}

// number of leading zeros in the sorted dispersion keys = number of empty rows
__global__ void k_count_zero(const u32* __restrict__ sorted, u32 M, u32* out) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M && sorted[i] == 0 && (i + 1 == M || sorted[i + 1] != 0)) *out = i + 1;
}

// state[pos] = ASSIGNED|0 for empty rows (cluster 0, rowReordering.cu:939-949), else 0 =
// "rejected by virtual cluster 0"; st[0] = z + 1 so cluster 1 scans from position z.
// per position of the ascending order: {encoding offset, #blocks, SC, S1C} of its row, so the
// clustering reads a candidate's metadata in one 16-byte load instead of asc -> row -> 4 loads
__global__ void k_pmeta(const u32* asc, const u32* rowptr, const u32* nblk, const u32* SC,
                        const u32* S1C, u32 M, uint4* pmeta) {
    const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < M) {
        const u32 row = asc[p];
        pmeta[p] = make_uint4(rowptr[row], nblk[row], SC[row], S1C[row]);
    }
}

__global__ void k_init_state(u32* state, u32* st, u32 M, u32 z) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) state[i] = i < z ? ASSIGNED : 0u;
    if (i == 0) st[0] = z + 1;
}

// ------------------------------------------------------------------------------------------
// 3. Clustering. The reference runs one single-block kernel per cluster and chains them with
// per-row device mutexes and device-side launches; the result is sequential first-fit (cluster
// c examines position i only after c-1 has, and takes it when the similarity to its
// representative exceeds alpha). Here one 1024-thread workgroup runs a TILE of T consecutive
// clusters (T representatives side by side in LDS): every candidate position's encoding is read
// once per tile instead of once per cluster, and the 16 waves evaluate 16 positions at a time
// against all T representatives. A leader wave then walks the sub-batch in position order and
// applies the sequential rule: position p goes to the first tile cluster whose similarity
// exceeds alpha; while the tile has fewer than T clusters, a position no cluster takes starts
// the next one; once it is full, a position every cluster rejects is passed on. An accept or a
// new cluster changes a representative, so the positions after it are evaluated again (both
// are rare next to rejects). Tiles follow each other through the per-position state word:
//     state[i] = ASSIGNED | c   row assigned to cluster c (sticky)
//     state[i] = c              unassigned, rejected by clusters 1..c
// and cluster c publishes its start in st[c] (start + 2; ST_NONE = no such cluster). A launch
// runs R = T x (tiles) consecutive clusters; the next launch continues from the last one.
//
// Similarity: calculate_similarity_norm_weighted_jaccard (rowReordering.cu:235-293) with the
// reference's reduce_sum tree (cudaUtil.cuh:13-45) for block size B: each logical thread t<B
// sums i = t, t+B, ... in order; xor-butterfly inside 32-lane warps; then the strided warp
// tree that drops warps when B/32 is not a power of two (keptMask). The integer norms are kept
// incrementally (u32 wrap, order-free). A double-precision estimate from the sparse row decides
// whenever it is further than GUARD from alpha (fp32 tree error < 3e-6); otherwise
// the exact fp32 emulation below decides.
// ------------------------------------------------------------------------------------------
struct ClusterArgs {
    const uint4* pmeta;  // per position: encoding offset (= CSR row offset), #blocks, SC, S1C
    const u32* enc;
    u32* state;
    u32* st;
    u32* ctrl;          // [0] abort, [1] timeout, [2..3] exact evals (u64), [4..5] total evals,
                        // [6] the launch's tile ticket counter
    u32* cmpScratch;    // [tiles][nbpr] zeros: dense row image of the exact path
    u32 M, nbpr, NP, B, keptMask, c0, T;
    u32 allKept;  // every warp of the reduction tree kept (B / 32 a power of two): no kept test
    float alpha;
    int exact_all;
    u64 timeout_ticks;  // s_memrealtime ticks (100 MHz)
    // candidate filter (cluster_filter.hip), or null: bit p of row q set when position p may
    // join the cluster led by position q while it is that row alone; fW = words per full row
    const u32* fbits;
    u32 fW;
    // BSMR_DIAG & 2048: per tile (global index (first cluster - 1) / T) 16 u64: kernel entry,
    // start found, end (s_memrealtime), windows, empty windows, sub-batch rounds, evaluations,
    // ticket, ticks in window scans (spins included), in evaluation, in the leader's resolution,
    // exact evaluations, ticks wave 0 spent on its own rows, encoding entries wave 0 read, rows
    // evaluated (the candidate filter's survivors), clusters holding more than their leader; else
    // null
    unsigned long long* ctrace;
};

constexpr double GUARD = 1e-5;
constexpr u32 CL_TMAX = 8;      // clusters per tile (register arrays)
#ifndef BSMR_CL_WAVES
#define BSMR_CL_WAVES 16
#endif
constexpr u32 CL_WAVES = BSMR_CL_WAVES;  // waves per tile workgroup
#ifndef BSMR_CL_SUB
#define BSMR_CL_SUB 64
#endif
constexpr u32 CL_SUB = BSMR_CL_SUB;  // positions per evaluation sub-batch (4 per wave)
constexpr u32 CL_WIN = 256;     // ready positions per window
constexpr u32 CL_LDS_BUDGET = 148 * 1024;  // representatives (the control block follows)
// accept chains the leader resolves alone (re-evaluating one position at a time) before it
// hands the rest of a sub-batch back to all waves
constexpr u32 CL_LEADER_EVALS = 16;
// encoding loads per lane the leader keeps in flight when it fills or updates a representative
constexpr u32 CL_ENC_B = 8;
// encoding chunks (256 entries) of a row whose loads are issued together (registers: 4 per chunk)
#ifndef BSMR_CL_PRE_CH
#define BSMR_CL_PRE_CH 2
#endif
constexpr u32 CL_PRE_CH = BSMR_CL_PRE_CH;

__device__ __forceinline__ u64 now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// control block after the representatives
struct ClusterCtl {
    u32 todo[CL_WIN];      // unassigned ready positions of the window
    u32 res[CL_WIN];       // verdict masks per todo slot (eval_row; current sub-batch)
    uint4 meta[CL_WIN];    // per todo slot: encoding offset, #blocks, SC, S1C of its row
    float inrf[CL_TMAX];   // 1 / nr per tile cluster (0 for an empty or zero-norm slot)
    float nr[CL_TMAX];     // sqrtf(SR)
    u32 SR[CL_TMAX];       // kept-block sum of squares of the representative (u32 wrap)
    u64 S1R[CL_TMAX];      // kept-block sum of the representative
    u32 scanL[CL_WIN / 64], scanN[CL_WIN / 64];  // window scan: ready prefix, unassigned count
    u32 ntodo, t, nact, done, i, nact_eval;
    u32 lead[CL_TMAX];  // position that started each tile cluster (candidate filter)
    u32 multi;          // bit c: cluster c holds more than its leader row (the filter cannot skip it)
    u32 nev;            // rows of the sub-batch the filter keeps, in evl (position order)
    u32 evl[CL_WIN];
    // the candidate bits of the window for each tile cluster: words wb0 .. wb0 + CL_WB - 1 of its
    // leader's row (~0 where the row stores no word: positions before the leader)
    u32 wb0;
    u32 wbits[CL_TMAX][CL_WIN / 32 + 1];
    u32 nxt;  // the sub-batch's next row for a free wave (rows t .. t + 15 go to waves 0 .. 15)
    u64 nexact, ntotal;
    u64 tr_begin, tr_started;  // BSMR_DIAG & 2048 timeline (ClusterArgs::ctrace)
    u64 tr_t0, tr_scan, tr_eval, tr_lead, tr_own, tr_ent, tr_nev;
    u32 tr_win, tr_idle, tr_sub;
};

// exact fp32 similarity of a tile cluster (LDS, element i at rep[i * TS]) with the row whose
// dense image is cmp (global scratch), one wave; the warp partials live in lanes 0..31 and the
// strided tree is applied lane-parallel (each level reads only indices the level does not write)
template <u32 TS>
__device__ float sim_exact_wave(const u32* rep, const u32* cmp, u32 nbpr, u32 B, float nr,
                                float nc) {
    const u32 l = lane_id();
    const u32 J = (B + 63) / 64;
    float wmn = 0.0f, wmx = 0.0f;
    for (u32 j = 0; j < J; ++j) {
        const u32 t = l + 64 * j;
        float pm = 0.0f, px = 0.0f;
        if (t < B) {
            for (u32 i = t; i < nbpr; i += B) {
                const float x = static_cast<float>(rep[i * TS]) / nr;
                const float y = static_cast<float>(cmp[i]) / nc;
                pm = pm + fminf(x, y);
                px = px + fmaxf(x, y);
            }
        }
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
            pm = pm + __shfl_xor(pm, o);
            px = px + __shfl_xor(px, o);
        }
        // warp 2j = lanes 0-31, warp 2j+1 = lanes 32-63
        const float m0 = __shfl(pm, 0), m1 = __shfl(pm, 32);
        const float x0 = __shfl(px, 0), x1 = __shfl(px, 32);
        if (l == 2 * j) {
            wmn = m0;
            wmx = x0;
        }
        if (l == 2 * j + 1) {
            wmn = m1;
            wmx = x1;
        }
    }
    for (u32 stride = B / 64; stride >= 1; stride >>= 1) {
        const float on = __shfl(wmn, (l + stride) & 63), ox = __shfl(wmx, (l + stride) & 63);
        if (l < stride) {
            wmn = wmn + on;
            wmx = wmx + ox;
        }
    }
    const float mn0 = __shfl(wmn, 0), mx0 = __shfl(wmx, 0);
    return mn0 / mx0;
}

__device__ __forceinline__ double readlane_f64(double v, u32 lane) {
    const u64 b = __builtin_bit_cast(u64, v);
    const u32 lo = __builtin_amdgcn_readlane(static_cast<u32>(b), lane);
    const u32 hi = __builtin_amdgcn_readlane(static_cast<u32>(b >> 32), lane);
    return __builtin_bit_cast(double, (static_cast<u64>(hi) << 32) | lo);
}

// the 8 per-lane partial sums reduced over the wave together (transposed butterfly: each xor
// step halves the values a lane keeps); cluster c's total ends in lanes 8c .. 8c + 7
__device__ __forceinline__ double wave_sum8(const double (&v)[CL_TMAX]) {
    const u32 l = lane_id();
    double a4[4], a2[2];
    const bool b5 = (l & 32) != 0, b4 = (l & 16) != 0, b3 = (l & 8) != 0;
#pragma unroll
    for (u32 i = 0; i < 4; ++i) {
        const double keep = b5 ? v[4 + i] : v[i], send = b5 ? v[i] : v[4 + i];
        a4[i] = keep + __shfl_xor(send, 32);
    }
#pragma unroll
    for (u32 i = 0; i < 2; ++i) {
        const double keep = b4 ? a4[2 + i] : a4[i], send = b4 ? a4[i] : a4[2 + i];
        a2[i] = keep + __shfl_xor(send, 16);
    }
    double s;
    {
        const double keep = b3 ? a2[1] : a2[0], send = b3 ? a2[0] : a2[1];
        s = keep + __shfl_xor(send, 8);
    }
    s += __shfl_xor(s, 4);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 1);
    return s;
}

// verdict bits of tile clusters [0, nact) on the row with metadata m (see eval_row), from the
// estimate's min-sum of cluster c (mnc_of(c); only read when est)
template <class F>
__device__ __forceinline__ u32 cl_verdict(const ClusterArgs& a, const ClusterCtl& C, uint4 m,
                                          u32 nact, bool est, F mnc_of) {
    const u32 scr = m.z, s1c = m.w;
    const float nc = sqrtf(static_cast<float>(scr));
    u32 acc = 0, ex = 0;
    for (u32 c = 0; c < nact; ++c) {
        const u32 SR = C.SR[c];
        if (SR == 0 && scr == 0) {
            if (1.0f > a.alpha) acc |= 1u << c;
            continue;
        }
        if (SR == 0 || scr == 0) {
            if (0.0f > a.alpha) acc |= 1u << c;
            continue;
        }
        if (!est) {
            ex |= 1u << c;
            continue;
        }
        const double mnc = mnc_of(c);
        const double mx = static_cast<double>(C.S1R[c]) / C.nr[c] + static_cast<double>(s1c) / nc - mnc;
        const double sim = mnc / mx;
        const double ad = static_cast<double>(a.alpha);
        if (fabs(sim - ad) > GUARD) {
            if (sim > ad) acc |= 1u << c;
        } else {
            ex |= 1u << c;
        }
    }
    return acc | (ex << 8);
}

// one wave: the verdicts of tile clusters [0, nact) on the row with metadata m (encoding offset,
// #blocks, SC, S1C) and first encoding chunk pre (entries l + 64u, 0 past the row), from the
// estimate: bit c of the low byte = accept, of the second byte = guard band (the exact emulation
// must decide c); neither = reject. Estimate: fp32 products and minima (relative error <= 2 ulp
// each), summed in fp32 over 4 entries and in double beyond: < 5e-7 relative in total, far
// inside GUARD.
template <u32 TS>
__device__ u32 eval_row(const ClusterArgs& a, const u32* reps, const ClusterCtl& C, uint4 m,
                        const u32 (&pre)[4], u32 nact) {
    const u32 l = lane_id();
    const u32 b0 = m.x, nb = m.y, scr = m.z, s1c = m.w;
    const float nc = sqrtf(static_cast<float>(scr));
    const bool est = !a.exact_all && scr != 0;
    double red = 0.0;
    if (est) {
        double mn[CL_TMAX];
        float inr[TS];
#pragma unroll
        for (u32 c = 0; c < CL_TMAX; ++c) mn[c] = 0.0;
#pragma unroll
        for (u32 c = 0; c < TS; ++c) inr[c] = C.inrf[c];
        const float incf = 1.0f / nc;
        // one chunk of 4 entries per lane (entries l + 64u): fp32 minima summed over the chunk
        auto chunk = [&](const u32 e0, const u32 e1, const u32 e2, const u32 e3) {
            const u32 ent[4] = {e0, e1, e2, e3};
            float s[TS];
#pragma unroll
            for (u32 c = 0; c < TS; ++c) s[c] = 0.0f;
#pragma unroll
            for (u32 u = 0; u < 4; ++u) {
                const u32 blk = ent[u] & 0xFFFFu;
                // a padding (count 0) or non-kept entry contributes min(x, 0) = 0; the kept test
                // (a division by B per entry) only when some warp of the tree is dropped
                const float yr = static_cast<float>(ent[u] >> 16) * incf;
                const float y = (a.allKept || kept_idx(blk, a.B, a.keptMask)) ? yr : 0.0f;
                const u32* rp = reps + blk * TS;
                u32 rv[TS];
                if constexpr (TS % 4 == 0) {
#pragma unroll
                    for (u32 q = 0; q < TS; q += 4) {
                        const uint4 v4 = *reinterpret_cast<const uint4*>(rp + q);
                        rv[q] = v4.x;
                        rv[q + 1] = v4.y;
                        rv[q + 2] = v4.z;
                        rv[q + 3] = v4.w;
                    }
                } else {
#pragma unroll
                    for (u32 q = 0; q < TS; q += 2) {
                        const uint2 v2 = *reinterpret_cast<const uint2*>(rp + q);
                        rv[q] = v2.x;
                        rv[q + 1] = v2.y;
                    }
                }
#pragma unroll
                for (u32 c = 0; c < TS; ++c)
                    s[c] += fminf(static_cast<float>(rv[c]) * inr[c], y);
            }
#pragma unroll
            for (u32 c = 0; c < TS; ++c) mn[c] += static_cast<double>(s[c]);
        };
        // the row's first CL_PRE_CH chunks: chunk 0 was prefetched (pre), the next ones are all
        // issued now, so such a row pays one load round trip instead of one per chunk
        // (T = 8 keeps chunk 0 only: its 8 representatives' partial sums fill the registers)
        constexpr u32 NX = TS <= 6 || CL_WAVES <= 8 ? 4 * (CL_PRE_CH - 1) : 0;
        u32 ent[NX > 0 ? NX : 1];
#pragma unroll
        for (u32 u = 0; u < NX; ++u) {  // clamped loads, no branch per load
            const u32 e = l + 256 + 64 * u;
            const u32 v = a.enc[b0 + min(e, nb - 1)];
            ent[u] = e < nb ? v : 0u;
        }
        chunk(pre[0], pre[1], pre[2], pre[3]);
#pragma unroll
        for (u32 q = 0; q < NX / 4; ++q)
            if (256 * (q + 1) < nb) chunk(ent[4 * q], ent[4 * q + 1], ent[4 * q + 2], ent[4 * q + 3]);
        // longer rows: one chunk in flight ahead of the one computed (the loop used to load a
        // chunk and wait for it, one round trip per 256 entries)
        auto load4 = [&](u32 (&x)[4], const u32 e0) {
#pragma unroll
            for (u32 u = 0; u < 4; ++u) {  // clamped loads, no branch per load
                const u32 e = e0 + 64 * u;
                const u32 v = a.enc[b0 + min(e, nb - 1)];
                x[u] = e < nb ? v : 0u;
            }
        };
        constexpr u32 C1 = 256 + 64 * NX;  // first entry past the prefetched chunks
        if constexpr (TS > 4 && CL_WAVES > 8) {  // (the pipelined loop spills at T = 6 / 8, 16 waves)
            for (u32 e0 = l + C1; e0 < nb; e0 += 256) {
                u32 x[4];
                load4(x, e0);
                chunk(x[0], x[1], x[2], x[3]);
            }
        } else if (C1 < nb) {
            u32 x[4];
            load4(x, l + C1);
            for (u32 c0 = C1; c0 < nb; c0 += 256) {  // wave-uniform chunk base
                u32 y[4] = {0u, 0u, 0u, 0u};
                const bool more = c0 + 256 < nb;
                if (more) load4(y, l + c0 + 256);
                chunk(x[0], x[1], x[2], x[3]);
#pragma unroll
                for (u32 u = 0; u < 4; ++u) x[u] = y[u];
            }
        }
        red = wave_sum8(mn);
    }
    (void)s1c;
    return cl_verdict(a, C, m, nact, est, [&](u32 c) { return readlane_f64(red, 8 * c); });
}

__device__ __forceinline__ void load_chunk0(const ClusterArgs& a, uint4 m, u32 (&ent)[4]) {
    const u32 l = lane_id();
#pragma unroll
    for (u32 u = 0; u < 4; ++u) {  // clamped (rows hold >= 1 entry; m.y = 0: no row, no load)
        const u32 e = l + 64 * u;
        u32 v = 0;
        if (m.y) v = a.enc[m.x + min(e, m.y - 1)];
        ent[u] = e < m.y ? v : 0u;
    }
}

template <u32 TS>
__global__ __launch_bounds__(64 * CL_WAVES) void k_cluster(ClusterArgs a) {
    extern __shared__ __attribute__((aligned(16))) u32 smem[];
    constexpr u32 T = TS;
    u32* reps = smem;  // [NP][TS]: block b of tile cluster c at reps[b * TS + c]
    ClusterCtl& C = *reinterpret_cast<ClusterCtl*>(smem + a.NP * TS);
    const u32 tid = threadIdx.x, l = lane_id(), w = tid >> 6;
    __shared__ u32 s_ticket;
    if (tid == 0) s_ticket = atomicAdd(&a.ctrl[6], 1u);
    for (u32 x = tid; x < a.NP * TS; x += blockDim.x) reps[x] = 0;
    if (tid == 0) {
        C.tr_begin = a.ctrace ? now_ticks() : 0ull;
        C.tr_started = 0;
        C.tr_scan = C.tr_eval = C.tr_lead = C.tr_own = C.tr_ent = C.tr_nev = 0;
        C.tr_win = C.tr_idle = C.tr_sub = 0;
    }
    if (tid == 0) {
        C.multi = 0;
        C.wb0 = 0;
    }
    if (tid < CL_TMAX) {
        C.lead[tid] = 0;
        C.inrf[tid] = 0.0f;
        C.nr[tid] = 0.0f;
        C.SR[tid] = 0;
        C.S1R[tid] = 0;
    }
    __syncthreads();
    const u32 ticket = s_ticket;
    const u32 kfirst = a.c0 + ticket * T, klast = kfirst + T - 1, pred = kfirst - 1;
    u32* cmp = a.cmpScratch + static_cast<size_t>(ticket) * a.nbpr;  // zero between uses
    const u32 M = a.M;

    auto check_abort = [&](u64 t_start) -> bool {
        u32 ab = 0;
        if (l == 0) {
            ab = ld_agent(&a.ctrl[0]);
            if (!ab && now_ticks() - t_start > a.timeout_ticks) {
                st_agent(&a.ctrl[1], 1u);
                st_agent(&a.ctrl[0], 1u);
                ab = 1;
            }
        }
        return __shfl(ab, 0) != 0;
    };
    auto set_norm = [&](u32 c, u32 sr) {  // lane 0
        C.SR[c] = sr;
        const float nr = sqrtf(static_cast<float>(sr));
        C.nr[c] = nr;
        C.inrf[c] = sr ? 1.0f / nr : 0.0f;
    };
    // candidate filter: lanes k < CL_WIN / 32 + 1 load the window's words of the row of leader q
    // (cluster c) into LDS; wbit(c, p): may position p (in the window) join cluster c's leader
    constexpr u32 CL_WB = CL_WIN / 32 + 1;
    auto load_wbits = [&](u32 c, u32 q) {
        if (l < CL_WB) {
            const u32 wd = C.wb0 + l, qw = q >> 5;
            C.wbits[c][l] = wd >= qw && wd < a.fW ? a.fbits[fbits_row_offset(q, a.fW) + (wd - qw)] : ~0u;
        }
    };
    auto wbit = [&](u32 c, u32 p) -> bool { return (C.wbits[c][(p >> 5) - C.wb0] >> (p & 31)) & 1u; };
    // leader: start a new tile cluster (index C.nact) at position p (metadata m)
    // leader: the row's encoding entries (metadata m), CL_ENC_B loads per lane in flight per
    // round trip, each handed to body in turn (a load -> LDS store loop paid one round trip per 64
    // entries, and new clusters are the chain's critical path once the candidate filter skips
    // the evaluations)
    auto for_enc = [&](uint4 m, auto&& body) {
        for (u32 e0 = 0; e0 < m.y; e0 += 64 * CL_ENC_B) {
            u32 v[CL_ENC_B];
#pragma unroll
            for (u32 k = 0; k < CL_ENC_B; ++k) {  // clamped, unconditional (m.y >= 1 here)
                const u32 e = e0 + l + 64 * k;
                const u32 x = a.enc[m.x + min(e, m.y - 1)];
                v[k] = x;
            }
#pragma unroll
            for (u32 k = 0; k < CL_ENC_B; ++k)
                if (e0 + l + 64 * k < m.y) body(v[k]);
        }
    };
    auto new_cluster = [&](u32 p, uint4 m) {
        const u32 c = C.nact;
        if (a.fbits) load_wbits(c, p);
        for_enc(m, [&](u32 ent) { reps[(ent & 0xFFFFu) * TS + c] = ent >> 16; });
        if (l == 0) {
            set_norm(c, m.z);
            C.S1R[c] = m.w;
            C.lead[c] = p;
            C.nact = c + 1;
            st_agent(&a.state[p], ASSIGNED | (kfirst + c));
            st_agent(&a.st[kfirst + c], p + 2);
        }
    };
    // leader: position p (metadata m) joins tile cluster c
    auto accept = [&](u32 p, uint4 m, u32 c) {
        u32 dsr = 0, ds1 = 0;
        for_enc(m, [&](u32 ent) {  // (a row's blocks are distinct: no two lanes update one slot)
            const u32 blk = ent & 0xFFFFu, cnt = ent >> 16;
            const u32 o = reps[blk * TS + c], nv = o + cnt;
            reps[blk * TS + c] = nv;
            if (kept_idx(blk, a.B, a.keptMask)) {
                dsr += nv * nv - o * o;
                ds1 += cnt;
            }
        });
        dsr = wave_sum(dsr);
        ds1 = wave_sum(ds1);
        if (l == 0) {
            set_norm(c, C.SR[c] + dsr);
            C.S1R[c] += ds1;
            C.multi |= 1u << c;
            st_agent(&a.state[p], ASSIGNED | (kfirst + c));
        }
    };
    // leader: exact similarity of tile cluster c with the row of metadata m
    auto exact = [&](uint4 m, u32 c) -> bool {
        for (u32 e = l; e < m.y; e += 64) {
            const u32 ent = a.enc[m.x + e];
            cmp[ent & 0xFFFFu] = ent >> 16;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        const float nc = sqrtf(static_cast<float>(m.z));
        const float sim = sim_exact_wave<TS>(reps + c, cmp, a.nbpr, a.B, C.nr[c], nc);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        for (u32 e = l; e < m.y; e += 64) cmp[a.enc[m.x + e] & 0xFFFFu] = 0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        return sim > a.alpha;
    };
    auto row_meta = [&](u32 p) -> uint4 { return a.pmeta[p]; };

    // ---- leader: wait for the predecessor tile's last start, find the first cluster's start
    if (w == 0) {
        u32 start = M;
        bool aborted = false;
        u32 sprev = 0;
        u64 t0 = now_ticks();
        while (true) {
            u32 v = 0;
            if (l == 0) v = ld_agent(&a.st[pred]);
            v = __shfl(v, 0);
            if (v != 0) {
                sprev = v;
                break;
            }
            if (check_abort(t0)) {
                aborted = true;
                break;
            }
            __builtin_amdgcn_s_sleep(4);
        }
        if (!aborted && sprev != ST_NONE) {
            u32 i = sprev - 1;
            t0 = now_ticks();
            while (i < M) {
                const u32 idx = i + l;
                const u32 v = idx < M ? ld_agent(&a.state[idx]) : ASSIGNED;
                const bool ready = (v & ASSIGNED) || v == pred;
                const u64 notready = __ballot(!ready);
                const u32 L = notready ? __builtin_ctzll(notready) : 64u;
                const u64 cand = __ballot(ready && !(v & ASSIGNED) && l < L);
                if (cand) {
                    start = i + __builtin_ctzll(cand);
                    break;
                }
                if (L == 0) {
                    if (check_abort(t0)) {
                        aborted = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                } else {
                    i += L;
                    t0 = now_ticks();
                }
            }
        }
        if (l == 0) {
            C.nact = 0;
            C.nexact = 0;
            C.ntotal = 0;
            C.done = (aborted || start >= M) ? 1u : 0u;
            C.i = start + 1;
        }
        if (!aborted && start < M) {
            const uint4 m = row_meta(start);
            new_cluster(start, m);
        }
        if (a.ctrace && l == 0) C.tr_started = now_ticks();
        if (aborted && l == 0) C.nact = T;  // no ST_NONE on abort: the host reports the timeout
    }
    __syncthreads();

    u64 t_idle = now_ticks();
    while (!C.done) {
        __syncthreads();  // every wave has read the previous window's control words
        if (a.ctrace && tid == 0) C.tr_t0 = now_ticks();
        // ---- next window of ready positions (rejected by the predecessor tile or assigned):
        // the longest ready prefix of [C.i, C.i + CL_WIN), read by CL_WIN / 64 waves at once
        // (state word and metadata of every position in one round trip); the unassigned ones and
        // their rows' metadata go to C.todo / C.meta in position order
        constexpr u32 SW = CL_WIN / 64;  // scanning waves
        u32 sc_idx = 0;
        uint4 sc_m = make_uint4(0, 0, 0, 0);
        u64 sc_mm = 0;
        if (w < SW) {
            sc_idx = C.i + 64 * w + l;
            const bool in = sc_idx < M;
            const u32 v = in ? ld_agent(&a.state[sc_idx]) : ASSIGNED;
            if (in) sc_m = row_meta(sc_idx);
            const bool ready = (v & ASSIGNED) || v == pred;
            const u64 notready = __ballot(!ready || !in);
            const u32 L = notready ? __builtin_ctzll(notready) : 64u;
            sc_mm = __ballot(!(v & ASSIGNED) && l < L);
            if (l == 0) {
                C.scanL[w] = L;
                C.scanN[w] = static_cast<u32>(__builtin_popcountll(sc_mm));
            }
        }
        __syncthreads();
        if (w < SW) {
            // wave w's chunk counts when every chunk before it was fully ready
            u32 n0 = 0;
            bool live = true;
            for (u32 k = 0; k < w; ++k) {
                live = live && C.scanL[k] == 64u;
                n0 += C.scanN[k];
            }
            if (live && ((sc_mm >> l) & 1ull)) {
                const u32 slot = n0 + __builtin_amdgcn_mbcnt_hi(
                                          static_cast<u32>(sc_mm >> 32),
                                          __builtin_amdgcn_mbcnt_lo(static_cast<u32>(sc_mm), 0u));
                C.todo[slot] = sc_idx;
                C.meta[slot] = sc_m;
            }
        }
        if (w == 0) {
            const u32 i = C.i;
            u32 n = 0, total = 0;
            for (u32 k = 0; k < SW; ++k) {
                n += C.scanN[k];
                total += C.scanL[k];
                if (C.scanL[k] < 64u) break;
            }
            bool aborted = false;
            if (l == 0) ++C.tr_win;
            if (total == 0 && i < M) {
                if (l == 0) ++C.tr_idle;
                if (check_abort(t_idle)) aborted = true;
                else __builtin_amdgcn_s_sleep(1);
            } else {
                t_idle = now_ticks();
            }
            if (l == 0) {
                C.ntodo = n;
                C.t = 0;
                C.nxt = CL_WAVES;
                C.i = i + total;
                C.wb0 = i >> 5;
                if (aborted) {
                    C.done = 1;
                    C.nact = T;
                }
                if (i + total >= M && n == 0) C.done = 1;
            }
        }
        __syncthreads();
        if (a.fbits && w == 0) {
            // the window's candidate bits of every tile cluster (x = CL_WB c + k; T = 8 takes two
            // passes of the wave)
            const u32 na = C.nact;
            for (u32 x = l; x < na * CL_WB; x += 64) {
                const u32 c = x / CL_WB, k = x - c * CL_WB;
                const u32 q = C.lead[c], wd = C.wb0 + k, qw = q >> 5;
                C.wbits[c][k] = wd >= qw && wd < a.fW ? a.fbits[fbits_row_offset(q, a.fW) + (wd - qw)] : ~0u;
            }
        }
        if (a.ctrace && tid == 0) C.tr_scan += now_ticks() - C.tr_t0;
        if (C.done && C.ntodo == 0) break;
        // ---- evaluate / resolve sub-batches
        while (true) {
            const u32 t = C.t, ntodo = C.ntodo, nact = C.nact;
            if (t >= ntodo) break;
            if (tid == 0) {
                ++C.tr_sub;
                if (a.ctrace) C.tr_t0 = now_ticks();
            }
            // with the candidate filter a sub-batch is the whole window while every tile cluster
            // is its leader row alone (skipped rows cost a bit test, not an evaluation); once one
            // holds more rows, accepts are common and short sub-batches re-evaluate less
            const u32 tend = min(ntodo, t + (a.fbits && C.multi == 0 ? CL_WIN : CL_SUB));
            u32 nev = tend - t;
            if (a.fbits) {
                // a row needs its evaluation only if some tile cluster holds more than its leader
                // row, or the bound of (leader, row) may reach alpha (the window's bits in LDS);
                // the others are rejected by every tile cluster (res 0)
                if (w == 0) {
                    // (every row needs its evaluation while a tile cluster holds several rows;
                    // the bit tests without short-circuit branches, so their LDS reads overlap)
                    const bool anyMulti = (C.multi & ((1u << nact) - 1u)) != 0;
                    const u32 wb0 = C.wb0;
                    u32 n = 0;
                    for (u32 j0 = t; j0 < tend; j0 += 64) {
                        const u32 j = j0 + l;
                        bool need = false;
                        if (j < tend) {
                            const u32 p = C.todo[j], k = (p >> 5) - wb0;
                            u32 bits = 0;
                            for (u32 c = 0; c < nact; ++c) bits |= C.wbits[c][k];
                            need = anyMulti || ((bits >> (p & 31)) & 1u);
                            C.res[j] = 0;
                        }
                        const u64 b = __ballot(need);
                        if (need)
                            C.evl[n + __builtin_amdgcn_mbcnt_hi(static_cast<u32>(b >> 32),
                                                                __builtin_amdgcn_mbcnt_lo(static_cast<u32>(b), 0u))] = j;
                        n += static_cast<u32>(__builtin_popcountll(b));
                    }
                    if (l == 0) {
                        C.nev = n;
                        C.nxt = t + CL_WAVES;
                    }
                }
                __syncthreads();
                nev = C.nev;
            }
            if (a.ctrace && tid == 0) C.tr_nev += nev;
            {
                // row k of the sub-batch's evaluation list (whichever wave is free takes the next)
                auto row_at = [&](u32 k) { return a.fbits ? C.evl[k] : t + k; };
                u32 k = w;
                u32 pre[4];
                uint4 m = make_uint4(0, 0, 0, 0);
                if (k < nev) {
                    m = C.meta[row_at(k)];
                    load_chunk0(a, m, pre);
                }
                while (k < nev) {
                    // the next row comes from the sub-batch's counter: rows go to whichever wave
                    // is free, so a long row no longer holds a fixed three others behind it
                    // (wave 0 spent 40 % of the evaluation phase waiting at the barrier on
                    // reddit-like x1; profiles/r03j/cltrace)
                    u32 kn = 0;
                    if (l == 0) kn = atomicAdd(&C.nxt, 1u) - t;
                    kn = __builtin_amdgcn_readfirstlane(kn);
                    const u32 cur[4] = {pre[0], pre[1], pre[2], pre[3]};
                    const uint4 mc = m;
                    if (kn < nev) {  // the next row's first chunk in flight while this one runs
                        m = C.meta[row_at(kn)];
                        load_chunk0(a, m, pre);
                    }
                    const u32 r = eval_row<TS>(a, reps, C, mc, cur, nact);
                    if (l == 0) C.res[row_at(k)] = r;
                    if (a.ctrace && tid == 0) C.tr_ent += mc.y;
                    k = kn;
                }
            }
            if (a.ctrace && tid == 0) C.tr_own += now_ticks() - C.tr_t0;  // wave 0's own rows
            __syncthreads();
            if (a.ctrace && tid == 0) {
                const u64 tn = now_ticks();
                C.tr_eval += tn - C.tr_t0;
                C.tr_t0 = tn;
            }
            if (w == 0) {
                // the sequential rule over the sub-batch. Verdicts of clusters whose
                // representative changed since the evaluation (dirty: accepts, new clusters)
                // are stale: a position whose walk reaches one is evaluated again by this wave
                // (accept chains), up to CL_LEADER_EVALS times; after a new cluster (unless the
                // candidate filter runs), or past that budget, the rest goes back to all waves
                u32 j = t, dirty = 0, budget = CL_LEADER_EVALS;
                u64 nex = 0, ntot = 0;
                while (j < tend) {
                    if (dirty == 0) {
                        // plain rejects of a full tile up to the first other verdict, stored
                        // lane-parallel
                        const u32 n = tend - j;
                        const u32 r = l < n ? C.res[j + l] : 0u;
                        // (filter: clusters started since the evaluation are the leader rows
                        // alone here; a set bit makes the row an event)
                        bool newc = false;
                        if (a.fbits && l < n) {
                            const u32 p = C.todo[j + l], k = (p >> 5) - C.wb0, na = C.nact;
                            u32 bits = 0;
                            for (u32 c = nact; c < na; ++c) bits |= C.wbits[c][k];
                            newc = (bits >> (p & 31)) & 1u;
                        }
                        const u64 ev = __ballot(l < n && (r != 0u || C.nact < T || newc));
                        const u32 e = ev ? static_cast<u32>(__builtin_ctzll(ev)) : min(n, 64u);  // (one wave: 64 at a time)
                        if (l < e) st_agent(&a.state[C.todo[j + l]], klast);
                        ntot += static_cast<u64>(e) * C.nact;
                        j += e;
                        if (j >= tend) break;
                    }
                    const u32 p = C.todo[j];
                    const uint4 m = C.meta[j];
                    u32 r = C.res[j];
                    bool fresh = false;
                    const u32 na = C.nact;
                    u32 c = 0, take = ~0u, nex_p = 0;  // exact evaluations of this walk
                    bool stop = false;  // the rest to all waves
                    for (; c < na; ++c) {
                        if (!fresh && (((dirty >> c) & 1u) || c >= nact)) {
                            // filter: a cluster started since the evaluation and still its leader
                            // row alone rejects without an evaluation when the pair's bit is clear
                            if (a.fbits && !((dirty >> c) & 1u) && !((C.multi >> c) & 1u) && !wbit(c, p))
                                continue;
                            if (budget == 0) {
                                stop = true;
                                break;
                            }
                            --budget;
                            u32 pre[4];
                            load_chunk0(a, m, pre);
                            r = eval_row<TS>(a, reps, C, m, pre, na);
                            fresh = true;
                        }
                        if ((r >> c) & 1u) {
                            take = c;
                            break;
                        }
                        if ((r >> (8 + c)) & 1u) {
                            ++nex_p;
                            if (exact(m, c)) {
                                take = c;
                                break;
                            }
                        }
                    }
                    if (stop) break;  // this position is walked again by the next round
                    nex += nex_p;
                    ++j;
                    if (take != ~0u) {
                        ntot += take + 1;
                        accept(p, m, take);
                        dirty |= 1u << take;
                        continue;
                    }
                    ntot += na;
                    if (na < T) {
                        new_cluster(p, m);
                        // a new cluster: without the filter the rest of the sub-batch goes back
                        // to all waves; with it the walk goes on (its bits are in LDS)
                        if (!a.fbits) break;
                        continue;
                    }
                    if (l == 0) st_agent(&a.state[p], klast);
                }
                if (l == 0) {
                    C.t = j;
                    C.nxt = j + CL_WAVES;
                    C.nexact += nex;
                    C.ntotal += ntot;
                }
            }
            __syncthreads();
            if (a.ctrace && tid == 0) C.tr_lead += now_ticks() - C.tr_t0;
        }
        if (C.done) break;
    }
    if (w == 0 && l == 0) {
        for (u32 c = C.nact; c < T; ++c) st_agent(&a.st[kfirst + c], ST_NONE);
        atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctrl[2]), C.nexact);
        atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctrl[4]), C.ntotal);
        if (a.ctrace) {
            unsigned long long* tr = a.ctrace + 16ull * ((kfirst - 1) / T);
            tr[0] = C.tr_begin;
            tr[1] = C.tr_started;
            tr[2] = now_ticks();
            tr[3] = C.tr_win;
            tr[4] = C.tr_idle;
            tr[5] = C.tr_sub;
            tr[6] = C.ntotal;
            tr[7] = ticket;
            tr[8] = C.tr_scan;
            tr[9] = C.tr_eval;
            tr[10] = C.tr_lead;
            tr[11] = C.nexact;
            tr[12] = C.tr_own;
            tr[13] = C.tr_ent;
            tr[14] = C.tr_nev;
            tr[15] = static_cast<u64>(__builtin_popcount(C.multi));
        }
    }
}

__global__ void k_ids(const u32* state, u32* ids, u32 M) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) ids[i] = state[i] & ~ASSIGNED;
}

// reorderedRows[q] = asc[indices[z + q]]
__global__ void k_perm(const u32* asc, const u32* indices, u32 z, u32 R, u32* rows) {
    const u32 q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < R) rows[q] = asc[indices[z + q]];
}

// ------------------------------------------------------------------------------------------
// 5. Column split.
// ------------------------------------------------------------------------------------------
__global__ void k_row_nnz(const u32* rowptr, const u32* rows, u32 R, u32* rn) {
    const u32 q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < R) rn[q] = rowptr[rows[q] + 1] - rowptr[rows[q]];
}

// one wave per reordered row: copy its columns into the panel segment (row order inside the
// panel, file order inside the row, so a stable sort by column keeps row order per column)
__global__ __launch_bounds__(256) void k_gather(const u32* __restrict__ rowptr,
                                                const u32* __restrict__ col,
                                                const u32* __restrict__ rows,
                                                const u32* __restrict__ roff, u32 R,
                                                u32* __restrict__ keys, u32* __restrict__ vals,
                                                uint8_t* __restrict__ ent_lr,
                                                u32* __restrict__ ent_idx) {
    const u32 q = blockIdx.x * 4 + (threadIdx.x >> 6);
    const u32 l = threadIdx.x & 63;
    if (q >= R) return;
    const u32 row = rows[q];
    const u32 s = rowptr[row], n = rowptr[row + 1] - s, d = roff[q];
    for (u32 j = l; j < n; j += 64) {
        keys[d + j] = col[s + j];
        vals[d + j] = d + j;
        ent_lr[d + j] = static_cast<uint8_t>(q & 15u);
        ent_idx[d + j] = s + j;
    }
}

__global__ void k_segments(const u32* roff, u32 R, u32 P, u32* seg_begin, u32* seg_end) {
    const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < P) {
        seg_begin[p] = roff[p * 16];
        seg_end[p] = roff[min(p * 16 + 16, R)];
    }
}

// F(x) = sum of counts over sorted positions < x, with hist[b] distinct columns of count 16-b
// placed at bstart[b] (count-descending order).
__device__ __forceinline__ u32 prefix_counts(u32 x, const u32* hist, const u32* bstart) {
    u32 s = 0;
#pragma unroll
    for (u32 b = 0; b < 16; ++b) {
        const u32 lo = bstart[b];
        const u32 take = x > lo ? min(x - lo, hist[b]) : 0u;
        s += take * (16u - b);
    }
    return s;
}

__device__ __forceinline__ u32 run_length(const u32* keys, u32 e, u32 end) {
    const u32 key = keys[e];
    u32 c = 1;
    while (e + c < end && c < 16 && keys[e + c] == key) ++c;
    return c;
}

// pass 1: per panel, count distinct columns per count bucket; dense groups; totals.
__global__ __launch_bounds__(256) void k_panel_pass1(const u32* __restrict__ seg_begin,
                                                     const u32* __restrict__ seg_end,
                                                     const u32* __restrict__ skeys, u32 thr,
                                                     u32* __restrict__ phist, u32* __restrict__ pnd,
                                                     u32* __restrict__ pns, u32* __restrict__ psd) {
    __shared__ u32 hist[16], bstart[16], dense_cnt;
    const u32 p = blockIdx.x, t = threadIdx.x;
    const u32 s0 = seg_begin[p], s1 = seg_end[p];
    if (t < 16) hist[t] = 0;
    if (t == 0) dense_cnt = 0;
    __syncthreads();
    for (u32 e = s0 + t; e < s1; e += 256) {
        const bool head = e == s0 || skeys[e - 1] != skeys[e];
        if (head) atomicAdd(&hist[16 - run_length(skeys, e, s1)], 1u);
    }
    __syncthreads();
    if (t == 0) {
        u32 acc = 0;
        for (u32 b = 0; b < 16; ++b) {
            bstart[b] = acc;
            acc += hist[b];
        }
    }
    __syncthreads();
    const u32 ndist = bstart[15] + hist[15];
    const u32 L = (ndist + 15) & ~15u;
    u32 dense = 0;
    for (u32 g = t; g < L / 16; g += 256) {
        const u32 sum = prefix_counts(16 * g + 16, hist, bstart) - prefix_counts(16 * g, hist, bstart);
        if (sum >= thr) ++dense;
    }
    dense = wave_sum(dense);
    if ((t & 63) == 0 && dense) atomicAdd(&dense_cnt, dense);
    __syncthreads();
    if (t < 16) phist[p * 16 + t] = hist[t];
    if (t == 0) {
        const u32 nd = 16 * dense_cnt;
        pnd[p] = nd;
        pns[p] = L - nd;
        psd[p] = (s1 - s0) - prefix_counts(nd, hist, bstart);
    }
}

// pass 2: rank every distinct column inside its count bucket (column-ascending), place it,
// and scatter its entries into the dense tiles or the residual lists.
__global__ __launch_bounds__(256) void k_panel_pass2(
    const u32* __restrict__ seg_begin, const u32* __restrict__ seg_end,
    const u32* __restrict__ skeys, const u32* __restrict__ svals,
    const uint8_t* __restrict__ ent_lr, const u32* __restrict__ ent_idx,
    const u32* __restrict__ phist, const u32* __restrict__ pnd,
    const u32* __restrict__ dcoff, const u32* __restrict__ scoff, const u32* __restrict__ sdoff,
    u32 N, u32* __restrict__ denseCols, u32* __restrict__ sparseCols,
    u32* __restrict__ blockValues, u32* __restrict__ sparseValues,
    u32* __restrict__ sparseRel, u32* __restrict__ sparseColIdx) {
    __shared__ u32 hist[16], bstart[16], base[16], wcnt[4][16];
    const u32 p = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const u32 s0 = seg_begin[p], s1 = seg_end[p];
    if (t < 16) {
        hist[t] = phist[p * 16 + t];
        base[t] = 0;
    }
    __syncthreads();
    if (t == 0) {
        u32 acc = 0;
        for (u32 b = 0; b < 16; ++b) {
            bstart[b] = acc;
            acc += hist[b];
        }
    }
    __syncthreads();
    const u32 nd = pnd[p];
    const u32 dOff = dcoff[p], sOff = scoff[p], sdOff = sdoff[p];
    const u64 tile0 = dcoff[p] / 16;
    const u32 Fnd = prefix_counts(nd, hist, bstart);
    const u64 lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (u32 c0 = s0; c0 < s1; c0 += 256) {
        const u32 e = c0 + t;
        bool head = false;
        u32 b = 0, c = 0;
        if (e < s1) {
            head = e == s0 || skeys[e - 1] != skeys[e];
            if (head) {
                c = run_length(skeys, e, s1);
                b = 16 - c;
            }
        }
        u32 rank = 0;
#pragma unroll
        for (u32 bb = 0; bb < 16; ++bb) {
            const u64 m = __ballot(head && b == bb);
            if (head && b == bb) rank = __popcll(m & lt);
            if (lane == 0) wcnt[w][bb] = __popcll(m);
        }
        __syncthreads();
        if (head) {
            for (u32 j = 0; j < w; ++j) rank += wcnt[j][b];
            rank += base[b];
            const u32 pos = bstart[b] + rank;
            const u32 colv = skeys[e];
            if (pos < nd) {
                denseCols[dOff + pos] = colv;
                const u64 tb = (tile0 + pos / 16) * 256ull + (pos % 16);
                for (u32 j = 0; j < c; ++j) {
                    const u32 ent = svals[e + j];
                    blockValues[tb + 16ull * ent_lr[ent]] = ent_idx[ent];
                }
            } else {
                sparseCols[sOff + pos - nd] = colv;
                const u32 rb = sdOff + prefix_counts(pos, hist, bstart) - Fnd;
                for (u32 j = 0; j < c; ++j) {
                    const u32 ent = svals[e + j];
                    sparseValues[rb + j] = ent_idx[ent];
                    sparseRel[rb + j] = ent_lr[ent];
                    sparseColIdx[rb + j] = colv;
                }
            }
        }
        __syncthreads();
        if (t < 16) {
            u32 s = 0;
            for (u32 j = 0; j < 4; ++j) s += wcnt[j][t];
            base[t] += s;
        }
        __syncthreads();
    }
    // sentinel padding (column N) up to a multiple of 16 (colReordering.cu:338-343)
    const u32 ndist = bstart[15] + hist[15];
    const u32 L = (ndist + 15) & ~15u;
    for (u32 pos = ndist + t; pos < L; pos += 256) {
        if (pos < nd)
            denseCols[dOff + pos] = N;
        else
            sparseCols[sOff + pos - nd] = N;
    }
}

__global__ void k_div16(const u32* in, u32* out, u32 n) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] / 16;
}

// ------------------------------------------------------------------------------------------
// 6. Work lists: dense items {panel, first tile, tiles} of <= TILES_PER_ITEM tiles, residual
// items {panel, first entry, end entry} of <= RES_PER_ITEM entries.
// ------------------------------------------------------------------------------------------
__global__ void k_item_counts(const u32* pnd, const u32* psd, u32 P, u32 tpi, u32 rpi, u32* dc,
                              u32* rc) {
    const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < P) {
        dc[p] = (pnd[p] / 16 + tpi - 1) / tpi;
        rc[p] = (psd[p] + rpi - 1) / rpi;
    }
}

__global__ void k_item_fill(const u32* dcoff, const u32* sdoff, const u32* doffs,
                            const u32* roffs, u32 P, u32 tpi, u32 rpi, uint4* ditems,
                            uint4* ritems) {
    const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const u32 t0 = dcoff[p] / 16, t1 = dcoff[p + 1] / 16;
    u32 o = doffs[p];
    for (u32 t = t0; t < t1; t += tpi) ditems[o++] = make_uint4(p, t, min(tpi, t1 - t), 0);
    const u32 e0 = sdoff[p], e1 = sdoff[p + 1];
    o = roffs[p];
    for (u32 e = e0; e < e1; e += rpi) ritems[o++] = make_uint4(p, e, min(e + rpi, e1), 0);
}

// A-row index of every dense tile row (NULLV past the last reordered row), so a dense-tile wave
// needs one dependent round trip less (tile -> rows directly, not tile -> panel -> rows).
__global__ void k_tile_rows(const uint4* __restrict__ items, u32 nitems,
                            const u32* __restrict__ rows, u32 R, u32* __restrict__ tileRows) {
    const u32 i = blockIdx.x * 16 + (threadIdx.x >> 4), r = threadIdx.x & 15;
    if (i >= nitems) return;
    const uint4 it = items[i];
    const u32 q = it.x * 16 + r;
    const u32 row = q < R ? rows[q] : NULLV;
    for (u32 j = 0; j < it.z; ++j) tileRows[(it.y + j) * 16ull + r] = row;
}

// Column-major residual execution list: key = (col % 8) * N + col keeps each XCD bucket's
// columns together (the launch deals bucket x to blocks b with b % 8 == x, so one XCD's L2 holds
// 1/8 of B) and, within a column, the reference's panel-major entry order.
__global__ __launch_bounds__(256) void k_cm_keys(const u32* __restrict__ sdoff,
                                                 const u32* __restrict__ rows,
                                                 const u32* __restrict__ sparseRel,
                                                 const u32* __restrict__ sparseColIdx, u32 N,
                                                 u32* __restrict__ keys, u32* __restrict__ vals,
                                                 u32* __restrict__ rowOf) {
    const u32 p = blockIdx.x;
    const u32 e0 = sdoff[p], e1 = sdoff[p + 1];
    for (u32 e = e0 + threadIdx.x; e < e1; e += 256) {
        const u32 c = sparseColIdx[e];
        keys[e] = (c % XCD_BUCKETS) * N + c;
        vals[e] = e;
        rowOf[e] = rows[p * 16 + sparseRel[e]];
    }
}

__global__ void k_cm_gather(const u32* __restrict__ order, const u32* __restrict__ rowOf,
                            const u32* __restrict__ sparseColIdx,
                            const u32* __restrict__ sparseValues, const u32* __restrict__ skeys,
                            u32 n, u32 N, u32* __restrict__ cmRow, u32* __restrict__ cmCol,
                            u32* __restrict__ cmOut, u32* __restrict__ bucketCount) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 e = order[i];
    cmRow[i] = rowOf[e];
    cmCol[i] = sparseColIdx[e];
    cmOut[i] = sparseValues[e];
    if (i + 1 == n || skeys[i] / N != skeys[i + 1] / N) bucketCount[skeys[i] / N] = i + 1;
}

// Row-block layout: key = rowblock(q) * N + col (u64), q = reordered position of the entry's row.
// Panel range [pa, pa + gridDim.x): entry e is stored at i = e - sdoff[pa], q relative to 16 pa.
__global__ __launch_bounds__(256) void k_rb_keys(const u32* __restrict__ sdoff,
                                                 const u32* __restrict__ sparseRel,
                                                 const u32* __restrict__ sparseColIdx, u32 pa,
                                                 u32 RB, u32 N,
                                                 unsigned long long* __restrict__ keys,
                                                 u32* __restrict__ vals, u32* __restrict__ qOf) {
    const u32 p = pa + blockIdx.x;
    const u32 base = sdoff[pa];
    const u32 e0 = sdoff[p], e1 = sdoff[p + 1];
    for (u32 e = e0 + threadIdx.x; e < e1; e += 256) {
        const u32 q = blockIdx.x * 16 + sparseRel[e];
        keys[e - base] = static_cast<unsigned long long>(q / RB) * N + sparseColIdx[e];
        vals[e - base] = e - base;
        qOf[e - base] = q;
    }
}

// original-order row blocks: key = (row / RB) * N + col for every stored entry (thread per row)
__global__ __launch_bounds__(256) void k_rb_keys_csr(const u32* __restrict__ rowptr,
                                                     const u32* __restrict__ colidx, u32 M, u32 RB,
                                                     u32 N, unsigned long long* __restrict__ keys,
                                                     u32* __restrict__ vals, u32* __restrict__ qOf) {
    const u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= M) return;
    for (u32 e = rowptr[r]; e < rowptr[r + 1]; ++e) {
        keys[e] = static_cast<unsigned long long>(r / RB) * N + colidx[e];
        vals[e] = e;
        qOf[e] = r;
    }
}

// column blocks: key = (col / RB) * M + row for every stored entry (thread per row); qOf = the
// entry's column (its image row), rowOf = its row (the gathered A row)
__global__ __launch_bounds__(256) void k_rb_keys_cols(const u32* __restrict__ rowptr,
                                                      const u32* __restrict__ colidx, u32 M, u32 RB,
                                                      unsigned long long* __restrict__ keys,
                                                      u32* __restrict__ vals, u32* __restrict__ qOf,
                                                      u32* __restrict__ rowOf) {
    const u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= M) return;
    for (u32 e = rowptr[r]; e < rowptr[r + 1]; ++e) {
        const u32 c = colidx[e];
        keys[e] = static_cast<unsigned long long>(c / RB) * M + r;
        vals[e] = e;
        qOf[e] = c;
        rowOf[e] = r;
    }
}

// stored entries of tiles [t0, t0 + gridDim.x) (one 256-thread block per tile)
__global__ __launch_bounds__(256) void k_tile_nnz(const u32* __restrict__ blockValues, u32 t0,
                                                  u32* __restrict__ cnt) {
    __shared__ u32 wsum[4];
    const u32 t = t0 + blockIdx.x;
    const bool v = blockValues[static_cast<size_t>(t) * TILE + threadIdx.x] != NULLV;
    const u64 m = __ballot(v);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// entries of the demoted tiles (doff[i] != NULLV: their first slot among the demoted entries)
// become residual-style entries n0 + doff[i] + k in slot order: q relative to qa, column, output
__global__ __launch_bounds__(256) void k_tile_demote(const u32* __restrict__ blockValues,
                                                     const uint4* __restrict__ tilePanel,
                                                     const u32* __restrict__ denseCols, u32 t0,
                                                     const u32* __restrict__ doff, u32 qa, u32 RB,
                                                     u32 N, u32 n0,
                                                     unsigned long long* __restrict__ keys,
                                                     u32* __restrict__ vals, u32* __restrict__ qOf,
                                                     u32* __restrict__ dcol, u32* __restrict__ dout) {
    __shared__ u32 wsum[4];
    const u32 off = doff[blockIdx.x];
    if (off == NULLV) return;  // kept tile (uniform)
    const u32 t = t0 + blockIdx.x;
    const u32 slot = threadIdx.x, w = slot >> 6, l = slot & 63;
    const u32 idx = blockValues[static_cast<size_t>(t) * TILE + slot];
    const bool v = idx != NULLV;
    const u64 m = __ballot(v);
    if (l == 0) wsum[w] = __popcll(m);
    __syncthreads();
    if (!v) return;
    u32 r = __popcll(m & ((1ull << l) - 1));
    for (u32 k = 0; k < w; ++k) r += wsum[k];
    const u32 j = off + r;  // among the demoted entries
    const u32 q = tilePanel[t].x * 16 + slot / 16 - qa;
    const u32 c = denseCols[static_cast<size_t>(t) * 16 + slot % 16];
    keys[n0 + j] = static_cast<unsigned long long>(q / RB) * N + c;
    vals[n0 + j] = n0 + j;
    qOf[n0 + j] = q;
    dcol[j] = c;
    dout[j] = idx;
}

// local entry e < n0: residual entry e (arrays offset to the range); else demoted entry e - n0
__global__ void k_rb_gather(const u32* __restrict__ order, const u32* __restrict__ qOf,
                            const u32* __restrict__ sparseColIdx,
                            const u32* __restrict__ sparseValues, const u32* __restrict__ dcol,
                            const u32* __restrict__ dout, u32 n0, u32 n, u32 RB,
                            u32* __restrict__ meta, u32* __restrict__ out, u32* __restrict__ rbEnd) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 e = order[i];
    const u32 q = qOf[e];
    meta[i] = ((q % RB) << 22) | (e < n0 ? sparseColIdx[e] : dcol[e - n0]);
    out[i] = e < n0 ? sparseValues[e] : dout[e - n0];
    const u32 rb = q / RB;
    if (i + 1 == n || qOf[order[i + 1]] / RB != rb) rbEnd[rb] = i + 1;
}

// k_rb_gather for original-order row blocks: entry e is CSR position e
__global__ void k_rb_gather_csr(const u32* __restrict__ order, const u32* __restrict__ qOf,
                                const u32* __restrict__ colidx, u32 n, u32 RB,
                                u32* __restrict__ meta, u32* __restrict__ out,
                                u32* __restrict__ rbEnd) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 e = order[i];
    const u32 q = qOf[e];
    meta[i] = ((q % RB) << 22) | colidx[e];
    out[i] = e;
    const u32 rb = q / RB;
    if (i + 1 == n || qOf[order[i + 1]] / RB != rb) rbEnd[rb] = i + 1;
}

inline u32 grid_for(u64 n, u32 b) { return static_cast<u32>((n + b - 1) / b); }

// packed output: metadata word = local row << 22 | CSR position (the column bits are only read
// on the host, to cut the pieces, before this)
__global__ void k_pack_out(u32* __restrict__ meta, const u32* __restrict__ out, u32 n) {
    const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) meta[e] = (meta[e] & ~0x3FFFFFu) | out[e];
}

// staged output: item i's entries [ea, ea + E) sorted by CSR position (keys = positions, vals =
// index inside the item): slot t of the sorted order -> the entry's metadata low bits, and the
// position into sortedPos[ea + t]
__global__ __launch_bounds__(256) void k_item_slots(const uint2* __restrict__ itemEnt,
                                                    const u32* __restrict__ skeys,
                                                    const u32* __restrict__ svals,
                                                    u32* __restrict__ meta,
                                                    u32* __restrict__ sortedPos) {
    const uint2 ie = itemEnt[blockIdx.x];
    for (u32 t = threadIdx.x; t < ie.y; t += blockDim.x) {
        const u32 j = ie.x + t, e = ie.x + svals[j];
        meta[e] = (meta[e] & ~0x3FFFFFu) | t;
        sortedPos[j] = skeys[j];
    }
}

// exclusive scan of n values into out[0..n] (out[n] = total)
int excl_scan(const u32* in, u32* out, u32 n, DevBuf<uint8_t>& tmp, hipStream_t s) {
    BSMR_HIP(hipMemsetAsync(out, 0, sizeof(u32), s));
    if (n == 0) return BSMR_OK;
    size_t bytes = 0;
    BSMR_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, bytes, in, out + 1, static_cast<int>(n), s));
    if (bytes > tmp.size()) BSMR_CHECK(tmp.alloc(bytes));
    BSMR_HIP(hipcub::DeviceScan::InclusiveSum(tmp.data(), bytes, in, out + 1, static_cast<int>(n), s));
    return BSMR_OK;
}

int sort_pairs(const u32* kin, u32* kout, const u32* vin, u32* vout, u32 n, int end_bit,
               DevBuf<uint8_t>& tmp, hipStream_t s) {
    if (n == 0) return BSMR_OK;
    size_t bytes = 0;
    BSMR_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, kin, kout, vin, vout,
                                                static_cast<int>(n), 0, end_bit, s));
    if (bytes > tmp.size()) BSMR_CHECK(tmp.alloc(bytes));
    BSMR_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.data(), bytes, kin, kout, vin, vout,
                                                static_cast<int>(n), 0, end_bit, s));
    return BSMR_OK;
}

template <typename T>
int read_one(const T* dptr, T& h, hipStream_t s) {
    BSMR_HIP(hipMemcpyAsync(&h, dptr, sizeof(T), hipMemcpyDeviceToHost, s));
    BSMR_HIP(hipStreamSynchronize(s));
    return BSMR_OK;
}

int sort_pairs64(const unsigned long long* kin, unsigned long long* kout, const u32* vin, u32* vout,
                 u32 n, int end_bit, DevBuf<uint8_t>& tmp, hipStream_t s) {
    if (n == 0) return BSMR_OK;
    size_t bytes = 0;
    BSMR_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, kin, kout, vin, vout,
                                                static_cast<int>(n), 0, end_bit, s));
    if (bytes > tmp.size()) BSMR_CHECK(tmp.alloc(bytes));
    BSMR_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.data(), bytes, kin, kout, vin, vout,
                                                static_cast<int>(n), 0, end_bit, s));
    return BSMR_OK;
}

int bits_for(u64 maxval) {
    int b = 1;
    while (b < 64 && (1ull << b) <= maxval) ++b;
    return b;
}

}  // namespace

// calculateBlockSize (rowReordering.cu:1009-1025); free memory is an explicit input.
u32 block_size_for(u32 M, u32 N, u64 free_mem) {
    const u32 gmem = static_cast<u32>(std::ceil(static_cast<float>(static_cast<u64>(M) * M * 4ull) /
                                                static_cast<float>(free_mem / 2)));
    const u32 smem = static_cast<u32>(
        std::ceil(static_cast<float>(static_cast<u64>(N) * 4ull) / static_cast<float>(REF_MAX_SHMEM / 2)));
    const u32 bs = std::max(gmem, smem);
    return bs > 16 ? bs : 16;
}

// bsa_clustering block size (rowReordering.cu:911-920)
u32 cluster_block_dim(u32 nbpr) {
    if (nbpr < 32) return 32;
    int cand = static_cast<int>(32 * std::ceil(static_cast<float>(static_cast<int>(nbpr) / 4) / 32.0f));
    cand = cand > 32 ? cand : 32;
    return static_cast<u32>(1024 < cand ? 1024 : cand);
}

// warps whose partial sums reach s[0] in cuUtil::reduce_sum (cudaUtil.cuh:27-45)
u32 kept_warp_mask(u32 B) {
    const u32 W = B / 32;
    std::vector<u32> reach(W);
    for (u32 w = 0; w < W; ++w) reach[w] = 1u << w;
    for (u32 stride = B / 64; stride >= 1; stride >>= 1)
        for (u32 w = 0; w < stride; ++w) reach[w] |= reach[w + stride];
    return reach[0];
}

// Rows per row block for rows of rowBytes: a multiple of 16 with RB * rowBytes within the LDS
// budget, at most 1024 (10-bit local row in the entry metadata) and no more than the matrix needs.
u32 rowblock_rows(u32 rowBytes, u32 lds_kb, u32 R) {
    // (rows of <= 512 B: the workgroup's last LDS word is the piece-batch counter of k_sddmm_rb /
    // k_sddmm_rb_pair, so a whole-LDS budget leaves it out; an 80 KiB image is caught where the
    // block size is final)
    u64 bytes = static_cast<u64>(lds_kb) * 1024;
    if (rowBytes <= 512 && bytes >= 160u * 1024u) bytes = 160u * 1024u - 16u;
    u32 rb = static_cast<u32>(bytes / rowBytes / 16 * 16);
    rb = std::min<u32>(std::max<u32>(rb, 16), 1024);
    return std::min<u32>(rb, std::max<u32>((R + 15) / 16 * 16, 16));
}

namespace {
// split q chunks over segments by cost (largest remainder); every non-empty segment gets >= 1,
// and >= ceil(cost / cap) when cap > 0 (no chunk above cap; the total may then exceed q)
std::vector<u32> apportion(const std::vector<double>& cost, u32 q, double cap = 0.0) {
    const size_t n = cost.size();
    std::vector<u32> out(n, 0);
    double tot = 0;
    for (double c : cost) tot += c;
    if (tot <= 0) return out;
    std::vector<std::pair<double, size_t>> frac;
    u32 used = 0;
    for (size_t i = 0; i < n; ++i) {
        if (cost[i] <= 0) continue;
        const double ideal = q * cost[i] / tot;
        out[i] = std::max<u32>(1, static_cast<u32>(std::floor(ideal)));
        if (cap > 0) out[i] = std::max<u32>(out[i], static_cast<u32>(std::ceil(cost[i] / cap)));
        used += out[i];
        // capped: rank by what is still missing; uncapped: by the fractional part (the round-2
        // rule, so BSMR_ITEM_SCHED=0 BSMR_ITEM_CAP=0 reproduces the round-2 item lists)
        frac.push_back({cap > 0 ? ideal - out[i] : ideal - std::floor(ideal), i});
    }
    std::stable_sort(frac.begin(), frac.end(),
                     [](const auto& a, const auto& b) { return a.first > b.first; });
    for (size_t k = 0; used < q && k < frac.size(); ++k, ++used) ++out[frac[k].second];
    return out;
}
}  // namespace

// a candidate layout the launch does not use: its device arrays freed (its counts stay)
static void release_layout(Plan::RowBlockLayout& L) {
    L.meta.release();
    L.out.release();
    L.items.release();
    L.itemEnd.release();
    L.pieces.release();
    L.tileIds.release();
    L.rowIds.release();
    L.sortedPos.release();
    L.itemEnt.release();
    L.runs.release();
    L.itemRuns.release();
}

std::shared_ptr<const Plan::RowBlockLayout> Plan::rowblock_layout(u32 rowBytes, bool half,
                                                                  u32 pa, u32 pb, int* err) const {
    *err = BSMR_OK;
    const u32 tmin = half ? tile_min_half : tile_min_f32;
    if (pa == 0 && pb == P) {
        const int slot = (rowBytes == 128 ? 0 : rowBytes == 256 ? 1 : rowBytes == 512 ? 2 : rowBytes == 1024 ? 3 : 4) +
                         (half ? Plan::N_RB_SIZES : 0);
        RowBlockLayout& L = rbl[slot];
        if (L.rowBytes != rowBytes || L.tileMin != tmin) {
            rb_use_orig[slot] = false;
            rb_use_cols[slot] = false;
            *err = build_rowblock_layout(L, rowBytes, 0, P, tmin);
            if (*err != BSMR_OK) return nullptr;
            // sparse rows (the same < 64 entries per row rule as the row-block sizing): try
            // original-order row blocks and keep the cheaper layout by the shard cost model
            const bool sparse = R && static_cast<u64>(nres) + static_cast<u64>(numDenseTiles) * 16 <
                                         64ull * R;
            if (orig_rows == 1 || (orig_rows != 0 && sparse)) {
                RowBlockLayout& Lo = rblo[slot];
                *err = build_rowblock_layout(Lo, rowBytes, 0, P, tmin, true);
                if (*err != BSMR_OK) return nullptr;
                // column-run pieces (one B row gathered each) and MFMA tiles decide: the entries
                // are the same, and their LDS dot products cost far less than a gathered row
                // (C3 cop20k-like: 1.03 M -> 0.80 M pieces, 109 -> 78 us)
                const double c = L.nPieces + 16.0 * L.nTilesKept, co = Lo.nPieces;
                rb_use_orig[slot] = orig_rows == 1 || co < 0.9 * c;
                if (!rb_use_orig[slot]) release_layout(Lo);  // keep the decision, free the candidate
            }
            // column blocks, B rows staged and A rows gathered (the roles swapped): always (1),
            // or (2) for wide patterns (N >= 2 M) when their pieces are below 0.9 x the chosen
            // layout's (C2 nips-like 1,500 x 12,419: 93.5 K -> 75.8 K pieces, the same time)
            rb_use_cols[slot] = false;
            if (col_blocks == 1 || (col_blocks == 2 && static_cast<u64>(N) >= 2ull * M)) {
                RowBlockLayout& Lc = rblc[slot];
                *err = build_rowblock_layout(Lc, rowBytes, 0, P, tmin, false, true);
                if (*err != BSMR_OK) return nullptr;
                const RowBlockLayout& Lw = rb_use_orig[slot] ? rblo[slot] : L;
                const double cw = Lw.nPieces + 16.0 * Lw.nTilesKept;
                rb_use_cols[slot] = col_blocks == 1 || Lc.nPieces < 0.9 * cw;
                if (!rb_use_cols[slot]) release_layout(Lc);
            }
        }
        return std::shared_ptr<const RowBlockLayout>(std::shared_ptr<void>(), &rb_whole(slot));
    }
    for (const auto& L : shard_rbl)
        if (L->rowBytes == rowBytes && L->pa == pa && L->pb == pb && L->tileMin == tmin) return L;
    auto L = std::make_shared<RowBlockLayout>();
    *err = build_rowblock_layout(*L, rowBytes, pa, pb, tmin);
    if (*err != BSMR_OK) return nullptr;
    if (shard_rbl.size() >= MAX_SHARD_LAYOUTS) shard_rbl.erase(shard_rbl.begin());
    shard_rbl.push_back(L);
    return L;
}

// Row-block launch layout over panels [pa, pb) (the whole plan, or one row-panel shard).
// the layout's host passes over [0, n) on up to 16 threads: f(thread, begin, end), contiguous
// ranges, each index visited once (results written per index are independent of the split)
template <class F>
static void par_for(size_t n, F&& f, size_t serial_below = 2048) {
    const unsigned T = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (n < serial_below || T == 1) {
        f(0u, size_t{0}, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t chunk = (n + T - 1) / T;
    for (unsigned t = 0; t < T; ++t) {
        const size_t a = t * chunk, b = std::min(n, a + chunk);
        if (a < b) th.emplace_back([&f, t, a, b]() { f(t, a, b); });
    }
    for (auto& x : th) x.join();
}

// Static piece order of one row-block item (Plan::piece_balance). The kernel deals phase ph's
// pieces [ph NG, (ph + 1) NG) to row-groups gr, reversed in odd phases (sddmm.hip: piece
// ph NG + (ph odd ? NG - 1 - gr : gr)); a wave's 64 / G row-groups run a phase in lockstep, so a
// wave pays per phase its longest piece plus one gather (w entry-steps, the item cost model's
// piece weight). With the pieces longest first in position order, the waves that also run the
// short last phase end last. Here the same pieces, sorted longest first, go out in runs — one
// run per (wave, phase) bucket, as many pieces as that bucket has positions — always to the wave
// whose running cost is lowest (LPT over the buckets), so waves with two phases get shorter runs.
static void balance_pieces(std::vector<uint2>& pcs, u32 NT, u32 G, double w) {
    const u32 NG = NT / G, GW = 64 / G, NW = NT / 64;
    const u32 np = static_cast<u32>(pcs.size());
    if (np <= NG) return;  // one phase: every wave has one bucket already in cost order
    const u32 nph = (np + NG - 1) / NG;
    struct Bucket {
        u32 ph, cap;
        std::vector<u32> pos;  // the positions (piece indices) of its row-groups
    };
    std::vector<std::vector<Bucket>> wb(NW);
    for (u32 ph = 0; ph < nph; ++ph)
        for (u32 wv = 0; wv < NW; ++wv) {
            Bucket bk{ph, 0, {}};
            for (u32 gr = wv * GW; gr < (wv + 1) * GW; ++gr) {
                const u32 pos = ph * NG + ((ph & 1) ? NG - 1 - gr : gr);
                if (pos < np) bk.pos.push_back(pos);
            }
            bk.cap = static_cast<u32>(bk.pos.size());
            if (bk.cap) wb[wv].push_back(std::move(bk));
        }
    // buckets of a wave largest first
    for (auto& v : wb)
        std::stable_sort(v.begin(), v.end(), [](const Bucket& a, const Bucket& b) { return a.cap > b.cap; });
    std::vector<double> cost(NW, 0.0);
    std::vector<u32> next(NW, 0);
    std::vector<uint2> out(np);
    u32 k = 0;  // pcs sorted longest first
    while (k < np) {
        u32 best = NW;
        for (u32 wv = 0; wv < NW; ++wv)
            if (next[wv] < wb[wv].size() && (best == NW || cost[wv] < cost[best])) best = wv;
        const Bucket& bk = wb[best][next[best]++];
        cost[best] += static_cast<double>((pcs[k].y >> 22) + 1) + w;
        for (u32 pos : bk.pos) out[pos] = pcs[k++];
    }
    pcs.swap(out);
}

int Plan::build_rowblock_layout(RowBlockLayout& L, u32 rowBytes, u32 pa, u32 pb, u32 tileMin,
                                bool orig, bool cols) const {
    L.rowBytes = 0;
    L.orig = orig && !cols;
    L.cols = cols;
    orig = orig && !cols;
    // whole: original-order blocks of rows (orig) or of columns (cols), every entry residual
    const bool whole = orig || cols;
    // the gathered index space: columns of S, or (column blocks) its rows
    const u32 NS = cols ? M : N;
    hipStream_t s = stream;
    if (NS > (1u << 22)) {
        set_error(cols ? "column-block layout needs M <= 2^22" : "row-block layout needs N <= 2^22");
        return BSMR_ERR_UNSUPPORTED;
    }
    if (whole && (pa != 0 || pb != P)) {
        set_error("original-order row / column blocks cover the whole plan only");
        return BSMR_ERR_INVALID;
    }
    // BSMR_DIAG & 524288: section times of this build to stderr (host-side layout cost)
    auto lap_t = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!(diag & 524288)) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[rb layout %u B] %-12s %8.1f ms\n", rowBytes, what,
                     std::chrono::duration<double, std::milli>(t - lap_t).count());
        lap_t = t;
    };
    const u32 qa = whole ? 0 : 16 * pa, qend = orig ? M : cols ? N : std::min(R, 16 * pb);
    const u32 Rs = qend > qa ? qend - qa : 0;  // (reordered) rows of the range
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
        cus = 256;
    const u32 ebase = whole ? 0 : h_sparseValueOffsets[pa];
    // residual entries of the range (original order: every stored entry)
    const u32 n0 = whole ? nnz : h_sparseValueOffsets[pb] - ebase;
    // staged output (results through LDS, written per item in CSR order) for large P
    const bool stagedWanted = out_staged == 1 || (out_staged == -1 && 4ull * nnz > out_staged_min);
    // staged-output budget by row size (item_sched): 1 KiB rows take an 80 KiB image (two
    // workgroups per CU, results stored directly), 2 KiB rows the whole 160 KiB (mycielskian K =
    // 256 / 512: 379 -> 358 us and 896 -> 771 us against the 120 KiB staged image;
    // profiles/r03f/itemcal); 512-byte rows keep the tuned 120 KiB staged image (C4)
    const u32 stagedKb = !item_cost_cuts || rowBytes <= 512 ? rb_lds_kb_staged : rowBytes <= 1024 ? 80u : 160u;
    // 2 KiB rows (fp32 K = 512, fp16/bf16 K = 1024) take the whole-LDS image and 8 MiB column
    // ranges whatever P's size: an item's A image is 80 rows x 2 KiB, and fewer, wider ranges
    // restage it less (mycielskian14 / 15 / 16 K = 512: 100 -> 87, 253 -> 238, 735 -> 716 us;
    // 1 KiB rows lose with 8 MiB ranges: mycielskian16 K = 256 358 -> 468 us; profiles/r03u).
    // Sparse rows (< 64 stored entries per row) keep the small-row-block rule below (Trefethen
    // K = 512: 48-row blocks 48.1 us, 80-row blocks 51.5 us; profiles/r03v)
    const bool bigRows = item_cost_cuts && rowBytes >= 2048 && n0 >= 64ull * Rs;
    const u32 ldsKb = (stagedWanted || bigRows) && !rb_lds_user ? stagedKb : rb_lds_kb;
    // staged 512-byte rows (C4 reddit-like x1 fp32 K = 128): 8 MiB ranges too, half the A
    // restaging for a B range twice the L2 (4.01 -> 3.89 ms over three alternating runs,
    // profiles/r03y; C3 fp16 K = 256 neutral)
    // ... but at least two ranges per XCD when its B share exceeds its 4 MiB L2: one range of the
    // whole share ran C4 x0.5 (7.5 MiB per XCD) at 1.33 ms against 1.00 ms with two
    // (profiles/r04x); x1 keeps two 7.5 MiB ranges; a share that fits the L2 stays one range
    // (mycielskian16 K = 128, 3 MiB per XCD: 166 us against 181 us with two; profiles/r04zr)
    const bool staged512 = stagedWanted && item_cost_cuts && rowBytes == 512;
    const double shareKb = static_cast<double>(NS) * rowBytes / XCD_BUCKETS / 1024.0;
    const u32 l2Kb = l2_range_user ? l2_range_kb
                     : staged512 ? (shareKb > 4096.0 ? std::min<u32>(8192u, static_cast<u32>(std::ceil(shareKb / 2)) + 1)
                                                     : 8192u)
                     : bigRows ? 8192u
                     : stagedWanted ? l2_range_kb_staged : l2_range_kb;
    u32 RBr = rowblock_rows(rowBytes, ldsKb, Rs);
    {
        // sparse rows (< 64 stored entries per row: banded / FEM patterns) keep their row blocks
        // whole, one item each; when there are more row blocks than workgroup slots, use the
        // smallest row block that needs no more rounds of slots, so the last round is full
        // (cop20k-like C3: 421 blocks of 288 rows = 1.6 rounds -> 505 blocks of 240 rows)
        const size_t lds0 = static_cast<size_t>(RBr) * rowBytes;
        const u32 slots = static_cast<u32>(cus) * (lds0 > 80 * 1024 ? 1u : 2u);
        const u32 nRB0 = (Rs + RBr - 1) / std::max<u32>(RBr, 1);
        // (column blocks keep the whole image: their point is long row runs per block)
        if (cols) {
        } else if (Rs && n0 < 64ull * Rs && nRB0 > slots) {
            const u32 rounds = (nRB0 + slots - 1) / slots;
            const u32 rb = (Rs + rounds * slots - 1) / (rounds * slots);
            RBr = std::min(RBr, std::max<u32>(16, (rb + 15) / 16 * 16));
        } else if (Rs && n0 < 64ull * Rs && small_sparse_rb) {
            // fewer row blocks than slots: a block would be cut into chunks that each restage
            // its whole image for a few entries (Trefethen_20000 K = 64: 35 blocks of 576 rows in
            // 257 items, 15.2 us). One block per slot instead, at two workgroups per CU when the
            // image fits 80 KiB (48-row blocks in 512 items: 8.9 us; profiles/r03e/itemcal)
            const u32 s2 = static_cast<u32>(cus) * 2u;
            const u32 rb2 = std::max<u32>(16, ((Rs + s2 - 1) / s2 + 15) / 16 * 16);
            const u32 rb1 = std::max<u32>(16, ((Rs + cus - 1) / cus + 15) / 16 * 16);
            if (static_cast<size_t>(rb2) * rowBytes <= 80 * 1024) RBr = std::min(RBr, rb2);
            else RBr = std::min(RBr, rb1);
        }
    }
    if (Rs && (cols || n0 >= 64ull * Rs) && !(diag & 32768)) {
        // non-sparse rows: the same number of row blocks, of equal size (a multiple of 16), so
        // no short last block and every item stages the smallest image that count allows (C2
        // nips-like: 5 x 288 + 60 rows -> 5 x 256 + 220, 10.80 -> 10.63 us; BSMR_DIAG & 32768
        // keeps the LDS-budget size)
        const u32 nb0 = (Rs + RBr - 1) / RBr;
        RBr = std::min(RBr, std::max<u32>(16, ((Rs + nb0 - 1) / nb0 + 15) / 16 * 16));
    }
    // column blocks: the largest image the workgroup's LDS takes (fewer blocks, longer row runs:
    // C2 nips-like 288 -> 304 columns, 78.7 K -> 75.8 K pieces)
    // (staged output keeps its budget: the result slots live past the image)
    if (cols && !rb_lds_user && !stagedWanted && Rs) {
        // (batches never: no piece-batch counter to keep free, so the image may fill the LDS)
        const u32 rfull = std::min<u32>(std::min<u32>(160u * 1024u / rowBytes / 16 * 16, 1024),
                                        std::max<u32>((Rs + 15) / 16 * 16, 16));
        const u32 rmax = batches == 0 ? rfull : rowblock_rows(rowBytes, 160, Rs), nb0 = (Rs + rmax - 1) / rmax;
        RBr = std::min(rmax, std::max<u32>(16, ((Rs + nb0 - 1) / nb0 + 15) / 16 * 16));
    }
    if (rb_rows_force > 0)  // tuning: rows per block (a multiple of 16 within the LDS budget)
        RBr = std::min(rowblock_rows(rowBytes, 160, Rs),
                       std::max<u32>(16, (static_cast<u32>(rb_rows_force) + 15) / 16 * 16));
    // rows of <= 512 B: an image of exactly 80 KiB would fill a 512-thread workgroup's LDS, whose
    // last word is the piece-batch counter (160 KiB images are excluded by rowblock_rows)
    if (rowBytes <= 512 && static_cast<size_t>(RBr) * rowBytes == 80u * 1024u && RBr > 16) RBr -= 16;
    const u32 nRB = std::max<u32>(1, (Rs + RBr - 1) / RBr);
    const size_t lds = static_cast<size_t>(RBr) * rowBytes;
    const u32 NT = lds > 80 * 1024 ? 1024 : 512;
    // k_sddmm_rb takes 160 KiB (1024 threads) or 80 KiB (512) of LDS per workgroup
    const u32 wgPerCU = NT == 1024 ? 1 : 2;
    const u32 perBucket = std::max<u32>(1, static_cast<u32>(cus) * wgPerCU / XCD_BUCKETS);
    // dense tiles of the range: kept (>= tileMin stored entries) or demoted to entries
    const u32 T0 = h_blockOffsets[pa], nT = whole ? 0 : h_blockOffsets[pb] - T0;
    std::vector<u32> tcnt(nT, 0), doff(nT, NULLV), keptPos(nT + 1ull, 0), hkept;
    u32 nd = 0;
    if (nT && tileMin > 0) {
        DevBuf<u32> dcnt;
        BSMR_CHECK(dcnt.alloc(nT));
        hipLaunchKernelGGL(k_tile_nnz, dim3(nT), dim3(256), 0, s, blockValues.data(), T0, dcnt.data());
        BSMR_HIP(hipGetLastError());
        BSMR_HIP(hipMemcpyAsync(tcnt.data(), dcnt.data(), nT * sizeof(u32), hipMemcpyDeviceToHost, s));
        BSMR_HIP(hipStreamSynchronize(s));
    }
    for (u32 t = 0; t < nT; ++t) {
        keptPos[t] = static_cast<u32>(hkept.size());
        if (tileMin > 0 && tcnt[t] < tileMin) {
            doff[t] = nd;
            nd += tcnt[t];
        } else {
            hkept.push_back(T0 + t);
        }
    }
    keptPos[nT] = static_cast<u32>(hkept.size());
    const u32 n = n0 + nd;
    if (hkept.empty())
        BSMR_CHECK(L.tileIds.alloc(1));
    else
        BSMR_CHECK(L.tileIds.upload(hkept.data(), hkept.size(), s));
    BSMR_CHECK(L.meta.alloc(std::max<u32>(n, 1)));
    BSMR_CHECK(L.out.alloc(std::max<u32>(n, 1)));
    std::vector<u32> rbEnd(nRB, 0), hmeta(n);
    if (n) {
        DevBuf<unsigned long long> keys, skeys;
        DevBuf<u32> vals, order, qOf, dEnd, ddoff, dcol, dout, rowOf;
        BSMR_CHECK(keys.alloc(n));
        BSMR_CHECK(skeys.alloc(n));
        BSMR_CHECK(vals.alloc(n));
        BSMR_CHECK(order.alloc(n));
        BSMR_CHECK(qOf.alloc(n));
        BSMR_CHECK(dEnd.alloc(nRB));
        BSMR_CHECK(dcol.alloc(std::max<u32>(nd, 1)));
        BSMR_CHECK(dout.alloc(std::max<u32>(nd, 1)));
        BSMR_HIP(hipMemsetAsync(dEnd.data(), 0, nRB * sizeof(u32), s));
        if (cols) {
            BSMR_CHECK(rowOf.alloc(n));
            hipLaunchKernelGGL(k_rb_keys_cols, dim3(grid_for(M, 256)), dim3(256), 0, s, rowptr.data(),
                               colidx.data(), M, RBr, keys.data(), vals.data(), qOf.data(), rowOf.data());
        } else if (orig)
            hipLaunchKernelGGL(k_rb_keys_csr, dim3(grid_for(M, 256)), dim3(256), 0, s, rowptr.data(),
                               colidx.data(), M, RBr, N, keys.data(), vals.data(), qOf.data());
        else if (pb > pa)
            hipLaunchKernelGGL(k_rb_keys, dim3(pb - pa), dim3(256), 0, s, sparseValueOffsets.data(),
                               sparseRel.data(), sparseColIdx.data(), pa, RBr, N, keys.data(),
                               vals.data(), qOf.data());
        if (nd) {
            BSMR_CHECK(ddoff.upload(doff.data(), nT, s));
            hipLaunchKernelGGL(k_tile_demote, dim3(nT), dim3(256), 0, s, blockValues.data(),
                               denseItems.data(), denseCols.data(), T0, ddoff.data(), qa, RBr, N, n0,
                               keys.data(), vals.data(), qOf.data(), dcol.data(), dout.data());
        }
        BSMR_HIP(hipGetLastError());
        BSMR_CHECK(sort_pairs64(keys.data(), skeys.data(), vals.data(), order.data(), n,
                                bits_for(static_cast<u64>(nRB) * NS), tmp, s));
        if (whole)  // vals = CSR positions: the output index is the entry itself
            hipLaunchKernelGGL(k_rb_gather_csr, dim3(grid_for(n, 256)), dim3(256), 0, s, order.data(),
                               qOf.data(), cols ? rowOf.data() : colidx.data(), n, RBr, L.meta.data(),
                               L.out.data(), dEnd.data());
        else
            hipLaunchKernelGGL(k_rb_gather, dim3(grid_for(n, 256)), dim3(256), 0, s, order.data(),
                               qOf.data(), sparseColIdx.data() + ebase, sparseValues.data() + ebase,
                               dcol.data(), dout.data(), n0, n, RBr, L.meta.data(), L.out.data(),
                               dEnd.data());
        BSMR_HIP(hipGetLastError());
        BSMR_HIP(hipMemcpyAsync(rbEnd.data(), dEnd.data(), nRB * sizeof(u32), hipMemcpyDeviceToHost, s));
        BSMR_HIP(hipMemcpyAsync(hmeta.data(), L.meta.data(), n * sizeof(u32), hipMemcpyDeviceToHost, s));
        BSMR_HIP(hipStreamSynchronize(s));
        for (u32 b = 1; b < nRB; ++b) rbEnd[b] = std::max(rbEnd[b], rbEnd[b - 1]);
    }
    lap("sort+meta");
    // column ranges: NCR = 8 m ranges of (nearly) equal residual count; XCD x owns ranges
    // [x m, (x + 1) m). m makes one range's B columns (N rowBytes / NCR) fit an L2 budget: the
    // items of an XCD are ordered by range, so the B columns an item gathers were brought into
    // that XCD's L2 by the items before it (graph matrices: B is gathered once per row block and
    // column run, from L2 instead of the Infinity Cache)
    constexpr u32 CM = (1u << 22) - 1;
    const u32 rangeKb = l2Kb;
    const u32 m = std::max<u32>(1, static_cast<u32>(std::ceil(
        static_cast<double>(NS) * rowBytes / XCD_BUCKETS / (static_cast<double>(rangeKb) * 1024.0))));
    const u32 NCR = XCD_BUCKETS * m;
    std::vector<u32> cuts(NCR + 1, NS);
    cuts[0] = 0;
    {
        // column weight: its entries, plus (item_sched) piece_weight per column-run piece it
        // heads, so the XCDs' ranges carry equal modeled cost rather than equal entry counts
        // (mycielskian: the last XCD's range carried 10 % more piece work and ended 10 % later)
        // (integer counts per column — entries, and column-run starts = ceil(run / piece_max) per
        // row block — then cnt = entries + piece_weight x starts: exact whatever the host's thread
        // count, so every rank of a multi-GPU run derives the same layout. Each host thread takes a
        // stripe of columns and finds its part of every row block's column-sorted entries by
        // binary search: N + 1 counters in all, not one vector per row-block chunk)
        std::vector<u32> ecount(NS + 1, 0), scount(NS + 1, 0);
        const u32 NSTR = 64;
        par_for(NSTR, [&](unsigned, size_t s0, size_t s1) {
            for (size_t st = s0; st < s1; ++st) {
                const u32 c0 = static_cast<u32>(static_cast<u64>(NS) * st / NSTR);
                const u32 c1 = static_cast<u32>(static_cast<u64>(NS) * (st + 1) / NSTR);
                if (c0 == c1) continue;
                for (u32 b = 0; b < nRB; ++b) {
                    const u32* lo = hmeta.data() + (b ? rbEnd[b - 1] : 0u);
                    const u32* hi = hmeta.data() + rbEnd[b];
                    const auto byCol = [](u32 m, u32 c) { return (m & CM) < c; };
                    const u32* p = std::lower_bound(lo, hi, c0, byCol);
                    const u32* q = std::lower_bound(p, hi, c1, byCol);
                    for (const u32* i = p; i < q;) {
                        const u32 c = *i & CM;
                        const u32* j = i + 1;
                        while (j < q && (*j & CM) == c) ++j;
                        const u32 n = static_cast<u32>(j - i);
                        ecount[c] += n;
                        scount[c] += (n + piece_max - 1) / piece_max;
                        i = j;
                    }
                }
            }
        }, 1);
        std::vector<double> cnt(NS + 1, 0.0);
        for (u32 c = 0; c < NS; ++c)
            cnt[c] = static_cast<double>(ecount[c]) + (item_cost_cuts ? piece_weight * scount[c] : 0.0);
        double tot = 0;
        for (u32 c = 0; c < NS; ++c) tot += cnt[c];
        double run = 0;
        u32 x = 1;
        for (u32 c = 0; c < NS && x < NCR; ++c) {
            while (x < NCR && run >= tot * x / NCR) cuts[x++] = c;
            run += cnt[c];
        }
        for (; x < NCR; ++x) cuts[x] = NS;
    }
    lap("cuts");
    // segments (rb, range k): entries of rb in range k + 1/NCR of rb's tiles; cost = entries +
    // column-run pieces (one B column each) + 16 per tile
    const size_t nseg = static_cast<size_t>(nRB) * NCR;
    std::vector<u32> se0(nseg), se1(nseg), st0(nseg), st1(nseg), spc(nseg, 0);
    std::vector<double> cost(nseg);
    std::vector<u64> piecesRB(nRB, 0);
    par_for(nRB, [&](unsigned, size_t bb0, size_t bb1) {
    for (u32 b = static_cast<u32>(bb0); b < bb1; ++b) {
        const u32 eb0 = b ? rbEnd[b - 1] : 0, eb1 = rbEnd[b];
        const u32 p0 = std::min(pa + b * (RBr / 16), pb), p1 = std::min(pa + (b + 1) * (RBr / 16), pb);
        // kept tiles of the row block: positions [t0, t0 + nt) of the kept list
        const u32 t0 = whole ? 0 : keptPos[h_blockOffsets[p0] - T0];
        const u32 nt = whole ? 0 : keptPos[h_blockOffsets[p1] - T0] - t0;
        u32 lo = eb0;
        for (u32 k = 0; k < NCR; ++k) {
            const size_t i = static_cast<size_t>(b) * NCR + k;
            const u32 hi = k + 1 < NCR
                               ? static_cast<u32>(std::lower_bound(hmeta.begin() + lo, hmeta.begin() + eb1,
                                                                   cuts[k + 1],
                                                                   [](u32 v, u32 c) { return (v & CM) < c; }) -
                                                  hmeta.begin())
                               : eb1;
            se0[i] = lo;
            se1[i] = hi;
            for (u32 e = lo; e < hi;) {  // column runs cut every piece_max entries
                const u32 col = hmeta[e] & CM;
                u32 f = e + 1;
                while (f < hi && f - e < piece_max && (hmeta[f] & CM) == col) ++f;
                ++spc[i];
                e = f;
            }
            piecesRB[b] += spc[i];
            lo = hi;
            st0[i] = t0 + static_cast<u32>(static_cast<u64>(nt) * k / NCR);
            st1[i] = t0 + static_cast<u32>(static_cast<u64>(nt) * (k + 1) / NCR);
            cost[i] = (se1[i] - se0[i]) + piece_weight * spc[i] + 16.0 * (st1[i] - st0[i]);
        }
    }
    }, 16);
    lap("segments");
    // chunks. A row block is split by the column ranges (its items then read B from their own
    // XCD's L2) when it is big enough for >= 8 items of a one-round launch, or (m > 1) when its
    // column runs would gather more B rows than NCR restagings of its A rows cost; a smaller one
    // (e.g. banded matrices: many row blocks of few entries) is cut along its whole column-sorted
    // entry list, and its items balance the XCD list lengths. Item counts come from
    // largest-remainder apportionment; Q is one round of workgroup slots (fewer if items would
    // drop below ~128 cost units), or whole rounds when the split segments need more items.
    std::vector<std::vector<uint4>> lists(XCD_BUCKETS);
    std::vector<std::vector<u32>> lends(XCD_BUCKETS);
    double total = 0;
    for (double c : cost) total += c;
    const u32 Q1 = perBucket * XCD_BUCKETS;
    u32 Q = std::max<u32>(1, std::min<u32>(Q1, static_cast<u32>(total / 128.0)));
    const double target = total / Q;
    // no chunk above item_cap x one slot's share of a round (0: off): a row block of one hub row
    // (mycielskian: 8 K single-entry pieces in one item against a 6 K-entry median) otherwise
    // outlasts the whole launch (profiles/r03e/itemcal). 1x would force extra items into a
    // second round wherever a segment sits just above the mean (C2: 11 -> 17 us)
    const double cap = (item_cap < 0 ? 2.0 : item_cap) * total / Q1;
    std::vector<double> cb(nRB, 0.0);
    std::vector<char> split(nRB, 0);
    double splitTotal = 0;
    std::vector<u32> segX(XCD_BUCKETS, 0);  // non-empty split segments per XCD
    // column blocks whose whole gathered operand (A) fits half an XCD's L2 (C2: 768 KiB): no
    // block is split by range, so each block's items run on one XCD (contiguous eighths) and its
    // B image comes into that L2 once — split by range, every XCD would pull every block's image
    // from the Infinity Cache (8 x B per launch) to save gathers of an A that is L2-resident anyway
    const bool colsLocal = cols && static_cast<u64>(NS) * rowBytes <= (2ull << 20) && !(diag & 4096);
    for (u32 b = 0; b < nRB; ++b) {
        for (u32 k = 0; k < NCR; ++k) cb[b] += cost[static_cast<size_t>(b) * NCR + k];
        split[b] = !colsLocal && (cb[b] >= XCD_BUCKETS * target ||
                                  (m > 1 && piecesRB[b] >= static_cast<u64>(NCR) * RBr));
        if (!split[b]) continue;
        splitTotal += cb[b];
        for (u32 k = 0; k < NCR; ++k)
            segX[k / m] += cost[static_cast<size_t>(b) * NCR + k] > 0;
    }
    // the same quota for every XCD (the column cuts balance them): an extra item in one list
    // would start another round of slots on that XCD
    const u32 segMax = *std::max_element(segX.begin(), segX.end());
    if (segMax * XCD_BUCKETS > Q) Q = (segMax * XCD_BUCKETS + Q1 - 1) / Q1 * Q1;
    const u32 qEach = std::max<u32>(segMax, static_cast<u32>(std::llround(
        static_cast<double>(Q / XCD_BUCKETS) * (total > 0 ? splitTotal / total : 0.0))));
    const u32 qSplit = qEach * XCD_BUCKETS;
    std::vector<double> cu(nRB, 0.0);
    for (u32 b = 0; b < nRB; ++b) cu[b] = split[b] ? 0.0 : cb[b];
    std::vector<u32> nu;
    // staged output: the LDS past the A image (the launch takes 160 / 80 KiB) holds an item's
    // results when it has room for >= 1024 of them; larger items are cut to fit
    const size_t ldsDyn = (NT == 1024 ? 160u : 80u) * 1024u;
    // (the last 16 bytes: the piece-batch counter)
    const u32 outCap = ldsDyn > lds + 16 ? static_cast<u32>((ldsDyn - lds - 16) / 4) : 0u;
    const bool staged = stagedWanted && outCap >= 1024;
    // chunk k of an entry range: cut where the running cost (1 per entry + piece_weight per
    // column-run piece start) crosses k / nch of the range's cost, so chunks of single-entry
    // pieces get fewer entries than chunks of long runs; a chunk above the staged-output
    // capacity is then cut entry-evenly into as many as it needs (an entry-even cut of the whole
    // range would put a hub row's single-entry run into one chunk of 5x the others' cost)
    std::vector<u32> ecut, ecut2;
    // tot = the range's entries + piece_weight per piece (known from its segments' costs), so
    // one pass finds the cuts; ccost = the chunks' costs (entries + pieces) for the slot model
    std::vector<double> ccost, ccost2;
    auto cuts_by_cost = [&](u32 e0, u32 ne, u32 nch, double tot) {
        ecut.assign(nch + 1, e0 + ne);
        ecut[0] = e0;
        ccost.assign(nch, nch ? tot / nch : 0.0);
        if (nch > 1 && !item_cost_cuts) {
            for (u32 k = 1; k < nch; ++k) ecut[k] = e0 + static_cast<u32>(static_cast<u64>(ne) * k / nch);
        } else if (nch > 1) {
            double acc = 0, last = 0;
            u32 k = 1, run = 0;
            for (u32 e = e0; e < e0 + ne && k < nch; ++e) {
                const bool start = e == e0 || (hmeta[e] & CM) != (hmeta[e - 1] & CM) || run >= piece_max;
                run = start ? 1 : run + 1;
                while (k < nch && acc >= tot * k / nch) {
                    ecut[k] = e;
                    ccost[k - 1] = acc - last;
                    last = acc;
                    ++k;
                }
                acc += 1.0 + (start ? piece_weight : 0.0);
            }
            // the chunk from the last cut runs to the range's end; cuts never reached (k < nch)
            // leave empty chunks behind it
            for (u32 j = k; j < nch; ++j) ccost[j] = 0.0;
            ccost[k - 1] = std::max(0.0, tot - last);
        }
        if (!staged) return;
        ecut2.assign(1, e0);
        ccost2.clear();
        for (u32 j = 0; j < nch; ++j) {
            const u32 a = ecut[j], len = ecut[j + 1] - a, parts = std::max<u32>(1, (len + outCap - 1) / outCap);
            for (u32 q = 1; q <= parts; ++q) {
                ecut2.push_back(a + static_cast<u32>(static_cast<u64>(len) * q / parts));
                ccost2.push_back(ccost[j] / parts);
            }
        }
        ecut.swap(ecut2);
        ccost.swap(ccost2);
    };
    // lcost: each item's modeled cost (its entries + pieces + 16 per kept tile + staging
    // (piece_weight per row) + item_fixed), for the slot model
    std::vector<std::vector<double>> lcost(XCD_BUCKETS);
    auto emit = [&](u32 xl, u32 b, u32 e0, u32 ne, u32 t0, u32 nt, u32 nch, double rcost) {
        if (staged) nch = std::max<u32>(nch, (ne + outCap - 1) / outCap);
        cuts_by_cost(e0, ne, nch, rcost);
        nch = static_cast<u32>(ecut.size() - 1);
        for (u32 k = 0; k < nch; ++k) {
            const u32 ea = ecut[k];
            const u32 eb = ecut[k + 1];
            const u32 ta = t0 + static_cast<u32>(static_cast<u64>(nt) * k / nch);
            const u32 tb = t0 + static_cast<u32>(static_cast<u64>(nt) * (k + 1) / nch);
            if (ea == eb && ta == tb) continue;
            lists[xl].push_back(make_uint4(b, ta, tb, ea));
            lends[xl].push_back(eb);
            lcost[xl].push_back(ccost[k] + 16.0 * (tb - ta) + piece_weight * RBr + item_fixed);
        }
    };
    using Slot = std::priority_queue<double, std::vector<double>, std::greater<double>>;
    // the XCD lists for one cost cap (0: none); returns the modeled makespan: each XCD runs its
    // list on perBucket slots, an item starting when a slot frees (in list order)
    auto build_lists = [&](const double capv) -> double {
    lists.assign(XCD_BUCKETS, {});
    lends.assign(XCD_BUCKETS, {});
    lcost.assign(XCD_BUCKETS, {});
    nu = apportion(cu, Q > qSplit ? Q - qSplit : 0u, capv);
    for (u32 x = 0; x < XCD_BUCKETS; ++x) {
        // XCD x's segments in (range, row block) order
        std::vector<double> c(static_cast<size_t>(m) * nRB, 0.0);
        for (u32 j = 0; j < m; ++j)
            for (u32 b = 0; b < nRB; ++b)
                c[static_cast<size_t>(j) * nRB + b] =
                    split[b] ? cost[static_cast<size_t>(b) * NCR + x * m + j] : 0.0;
        const std::vector<u32> nch = apportion(c, qEach, capv);
        for (u32 j = 0; j < m; ++j)
            for (u32 b = 0; b < nRB; ++b) {
                const size_t i = static_cast<size_t>(b) * NCR + x * m + j;
                const u32 q = nch[static_cast<size_t>(j) * nRB + b];
                if (q)
                    emit(x, b, se0[i], se1[i] - se0[i], st0[i], st1[i] - st0[i], q,
                         (se1[i] - se0[i]) + piece_weight * spc[i]);
            }
    }
    // unsplit row blocks: their items, in row-block order, go to the list with the fewest items,
    // so no XCD runs an extra round (a contiguous range of blocks per XCD, for L2 sharing of
    // banded columns, measured 7 % slower on the cop20k-like C3 pattern)
    const u32 spare = XCD_BUCKETS;  // staging list index
    lists.resize(XCD_BUCKETS + 1);
    lends.resize(XCD_BUCKETS + 1);
    lcost.resize(XCD_BUCKETS + 1);
    for (u32 b = 0; b < nRB; ++b) {
        if (!nu[b]) continue;
        const size_t i0 = static_cast<size_t>(b) * NCR, i1 = i0 + NCR - 1;
        double rc = 0.0;
        for (size_t i = i0; i <= i1; ++i) rc += (se1[i] - se0[i]) + piece_weight * spc[i];
        emit(spare, b, se0[i0], se1[i1] - se0[i0], st0[i0], st1[i1] - st0[i0], nu[b], rc);
    }
    {
        const size_t nsp = lists[spare].size();
        const bool contig = whole && orig_contig && qSplit == 0;
        if (item_lpt && !contig && nsp) {
            // list scheduling: each XCD runs its list on perBucket slots, an item starting when a
            // slot frees (in list order). The XCD lists' split items are simulated first; then
            // the unsplit items, heaviest first, each go to the XCD where it starts earliest
            // (ties: fewer items, lower index), appended to that list, which keeps every list in
            // descending order of its unsplit items' cost
            std::vector<Slot> free(XCD_BUCKETS);
            for (u32 x = 0; x < XCD_BUCKETS; ++x) {
                for (u32 k = 0; k < perBucket; ++k) free[x].push(0.0);
                for (size_t j = 0; j < lists[x].size(); ++j) {
                    const double t = free[x].top();
                    free[x].pop();
                    free[x].push(t + lcost[x][j]);
                }
            }
            std::vector<std::pair<double, size_t>> ord(nsp);
            for (size_t i = 0; i < nsp; ++i) ord[i] = {lcost[spare][i], i};
            std::stable_sort(ord.begin(), ord.end(),
                             [](const auto& a, const auto& b) { return a.first > b.first; });
            for (const auto& [c, i] : ord) {
                u32 x = 0;
                for (u32 y = 1; y < XCD_BUCKETS; ++y) {
                    const double ty = free[y].top(), tx = free[x].top();
                    if (ty < tx || (ty == tx && lists[y].size() < lists[x].size())) x = y;
                }
                const double t = free[x].top();
                free[x].pop();
                free[x].push(t + c);
                lists[x].push_back(lists[spare][i]);
                lends[x].push_back(lends[spare][i]);
                lcost[x].push_back(c);
            }
        } else {
            for (size_t next = 0; next < nsp; ++next) {
                u32 x = 0;  // the list with the fewest items (ties: lowest index)
                for (u32 y = 1; y < XCD_BUCKETS; ++y)
                    if (lists[y].size() < lists[x].size()) x = y;
                // original-order blocks (orig_contig): XCD x takes the x-th contiguous eighth, so
                // the band's B rows of neighbouring blocks stay in one L2
                if (contig) x = static_cast<u32>(next * XCD_BUCKETS / nsp);
                lists[x].push_back(lists[spare][next]);
                lends[x].push_back(lends[spare][next]);
                lcost[x].push_back(lcost[spare][next]);
            }
        }
        lists.resize(XCD_BUCKETS);
        lends.resize(XCD_BUCKETS);
        lcost.resize(XCD_BUCKETS);
    }
    double ms = 0.0;
    for (u32 x = 0; x < XCD_BUCKETS; ++x) {
        Slot fr;
        for (u32 k = 0; k < perBucket; ++k) fr.push(0.0);
        double end = 0.0;
        for (size_t j = 0; j < lists[x].size(); ++j) {
            const double t = fr.top() + lcost[x][j];
            fr.pop();
            fr.push(t);
            end = std::max(end, t);
        }
        ms = std::max(ms, end);
    }
    return ms;
    };
    // the cap: item_cap x one slot's share, or (auto, item_sched, up to 32 M entries) the
    // multiple in {2, 1.5, 1.25, 1} whose lists the slot model runs fastest (a one-round launch
    // ends with its longest item: mycielskian15 K = 256, 2x cap 144 us; C2's segments sit just
    // above the mean, where 1x would open a second round)
    double capUse = cap;
    if (item_lpt && item_cap < 0 && n <= (1u << 25)) {
        double best = -1.0;
        for (const double f : {2.0, 1.5, 1.25, 1.0}) {
            const double msf = build_lists(f * total / Q1);
            if (best < 0 || msf < 0.995 * best) {
                best = msf;
                capUse = f * total / Q1;
            }
        }
    }
    const double msUse = build_lists(capUse);
    if (diag & 1024) {  // layout debug (host stderr)
        std::fprintf(stderr, "[rb layout] RB %u NT %u nRB %u m %u Q1 %u Q %u total %.0f target %.0f cap %.0f (used %.0f, model makespan %.0f) "
                     "splitTotal %.0f qEach %u segMax %u\n", RBr, NT, nRB, m, Q1, Q, total, target, cap, capUse, msUse,
                     splitTotal, qEach, segMax);
        for (u32 b = 0; b < nRB; ++b)
            if (cb[b] > 2 * target)
                std::fprintf(stderr, "[rb layout]   block %u cost %.0f split %d nu %u\n", b, cb[b], split[b], nu[b]);
    }
    lap("chunks");
    std::vector<uint4> items;
    std::vector<u32> ends;
    size_t nmax = 0;
    for (const auto& l : lists) nmax = std::max(nmax, l.size());
    // staged layouts: an even number of list positions, so the launch can pair them (k_sddmm_rb)
    if (staged) nmax = (nmax + 1) & ~static_cast<size_t>(1);
    items.assign(nmax * XCD_BUCKETS, make_uint4(0, 0, 0, 0));
    ends.assign(nmax * XCD_BUCKETS, 0);
    for (u32 x = 0; x < XCD_BUCKETS; ++x)
        for (size_t j = 0; j < lists[x].size(); ++j) {
            items[j * XCD_BUCKETS + x] = lists[x][j];
            ends[j * XCD_BUCKETS + x] = lends[x][j];
        }
    lap("items");
    // column-run pieces: each item's entries [e0, e1) cut at column changes and every
    // piece_max (<= RB_PIECE_MAX) entries; piece {first entry, column | (length - 1) << 22}. A workgroup's NG
    // row-groups take one piece each per phase, so phase ph runs the item's pieces
    // [ph NG, (ph + 1) NG). Longest first over the whole item, so the 16 row-groups of a wave get
    // pieces of similar length
    std::vector<uint2> ient(items.size());
    for (size_t i = 0; i < items.size(); ++i)
        ient[i] = make_uint2(items[i].w, (items[i].y == items[i].z && items[i].w == ends[i]) ? 0u
                                                                                          : ends[i] - items[i].w);
    // (per item on the host threads, then placed in item order)
    std::vector<std::vector<uint2>> ipc(items.size());
    par_for(items.size(), [&](unsigned, size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            std::vector<uint2>& mine = ipc[i];
            const u32 ea = items[i].w, eb = ends[i];
            for (u32 e = ea; e < eb;) {
                const u32 col = hmeta[e] & CM;
                u32 f = e + 1;
                while (f < eb && f - e < piece_max && (hmeta[f] & CM) == col) ++f;
                mine.push_back(make_uint2(e, col | ((f - e - 1) << 22)));
                e = f;
            }
            std::stable_sort(mine.begin(), mine.end(),
                             [](const uint2& a, const uint2& b) { return (a.y >> 22) > (b.y >> 22); });
        }
    });
    // dynamic piece batches (Plan::batches; kernels for rows of <= 512 B): after its first batch
    // of 64 / G pieces a wave takes the next from an LDS counter, which balances the waves of
    // items with several pieces per row-group. Measured (profiles/r05bt, forced on against off):
    // 512-byte rows with 2.4 / 6.5 / 6.8 pieces per row-group (mycielskian14 K = 128, C3, C4
    // x0.5) -4.5 / -2.4 / -2.2 %, C2's 1.4 +5 %; 128- and 256-byte rows (mycielskian15 K = 32,
    // Trefethen K = 64: little work per entry behind each counter round trip) +2 to +8 %. Auto:
    // 512-byte rows from batch_min_phases pieces per row-group
    bool dyn = false;
    {
        u64 npAll = 0;
        u32 nWork = 0;
        for (size_t i = 0; i < items.size(); ++i) {
            npAll += ipc[i].size();
            nWork += !(items[i].y == items[i].z && items[i].w == ends[i]);
        }
        const u32 NGl = NT / 4;  // row-groups (G = 4 for rows of <= 512 B)
        const double perItem = nWork ? static_cast<double>(npAll) / nWork : 0.0;
        dyn = rowBytes <= 512 &&
              (batches == 1 || (batches < 0 && rowBytes == 512 && perItem >= batch_min_phases * NGl));
    }
    // static phases (no batches): the item's pieces placed so that its waves end together
    // (balance_pieces; items with kept MFMA tiles keep the longest-first order, whose shortest
    // pieces sit with the tile waves)
    if (!dyn && piece_balance == 1) {
        const u32 G = rowBytes >= 2048 ? 16 : rowBytes >= 1024 ? 8 : 4;  // sddmm.hip RowGeom
        par_for(items.size(), [&](unsigned, size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; ++i)
                if (items[i].y == items[i].z) balance_pieces(ipc[i], NT, G, piece_weight);
        });
    }
    std::vector<size_t> poff(items.size() + 1, 0);
    for (size_t i = 0; i < items.size(); ++i) poff[i + 1] = poff[i] + ipc[i].size();
    std::vector<uint2> pieces(poff.back());
    L.itemStat.assign(items.size(), make_uint4(0, 0, 0, 0));
    std::vector<u64> ientc(items.size(), 0);
    std::vector<char> ipad(items.size(), 0);
    par_for(items.size(), [&](unsigned, size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            const bool pad = items[i].y == items[i].z && items[i].w == ends[i];
            std::copy(ipc[i].begin(), ipc[i].end(), pieces.begin() + poff[i]);
            std::vector<uint2>().swap(ipc[i]);
            items[i].w = static_cast<u32>(poff[i]);
            ends[i] = static_cast<u32>(poff[i + 1]);
            ipad[i] = pad;
            if (pad) continue;
            u64 ent = 0;
            for (u32 k = items[i].w; k < ends[i]; ++k) ent += (pieces[k].y >> 22) + 1;
            ientc[i] = ent;
            L.itemStat[i] = make_uint4(items[i].x, items[i].z - items[i].y, static_cast<u32>(ent),
                                       ends[i] - items[i].w);
        }
    });
    L.rbCost.assign(nRB, 0.0);
    L.nWorkItems = 0;
    for (size_t i = 0; i < items.size(); ++i) {
        const uint4 it = items[i];
        if (ipad[i]) continue;  // padding
        ++L.nWorkItems;
        L.rbCost[it.x] += static_cast<double>(ientc[i]) + shard_piece_weight * (ends[i] - it.w) +
                          16.0 * (it.z - it.y) + RBr;
    }
    L.nItems = static_cast<u32>(items.size());
    L.nPieces = static_cast<u32>(pieces.size());
    L.outLds = 0;
    L.outCap = 0;
    L.outPacked = false;
    L.outRuns = false;
    L.sortedPos.release();
    L.itemEnt.release();
    L.runs.release();
    L.itemRuns.release();
    lap("pieces");
    if (staged && n) {
        // slots: per item, its entries sorted by CSR position (segmented radix sort on the device)
        BSMR_CHECK(L.itemEnt.upload(ient.data(), ient.size(), s));
        std::vector<u32> segb(ient.size()), sege(ient.size());
        for (size_t i = 0; i < ient.size(); ++i) {
            segb[i] = ient[i].x;
            sege[i] = ient[i].x + ient[i].y;
        }
        DevBuf<u32> dsb, dse, lidx, skeys, svals;
        BSMR_CHECK(dsb.upload(segb.data(), segb.size(), s));
        BSMR_CHECK(dse.upload(sege.data(), sege.size(), s));
        std::vector<u32> hl(n);
        par_for(ient.size(), [&](unsigned, size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; ++i)
                for (u32 t = 0; t < ient[i].y; ++t) hl[ient[i].x + t] = t;
        });
        BSMR_CHECK(lidx.upload(hl.data(), n, s));
        BSMR_CHECK(skeys.alloc(n));
        BSMR_CHECK(svals.alloc(n));
        // entries outside every item (none) keep their place: pre-fill the outputs with the input
        BSMR_HIP(hipMemcpyAsync(skeys.data(), L.out.data(), n * sizeof(u32), hipMemcpyDeviceToDevice, s));
        BSMR_HIP(hipMemcpyAsync(svals.data(), lidx.data(), n * sizeof(u32), hipMemcpyDeviceToDevice, s));
        size_t bytes = 0;
        const int endbit = bits_for(nnz);
        BSMR_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(
            nullptr, bytes, L.out.data(), skeys.data(), lidx.data(), svals.data(), static_cast<int>(n),
            static_cast<int>(ient.size()), dsb.data(), dse.data(), 0, endbit, s));
        if (bytes > tmp.size()) BSMR_CHECK(tmp.alloc(bytes));
        BSMR_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(
            tmp.data(), bytes, L.out.data(), skeys.data(), lidx.data(), svals.data(),
            static_cast<int>(n), static_cast<int>(ient.size()), dsb.data(), dse.data(), 0, endbit, s));
        BSMR_CHECK(L.sortedPos.alloc(n));
        hipLaunchKernelGGL(k_item_slots, dim3(static_cast<u32>(ient.size())), dim3(256), 0, s,
                           L.itemEnt.data(), skeys.data(), svals.data(), L.meta.data(),
                           L.sortedPos.data());
        BSMR_HIP(hipGetLastError());
        BSMR_HIP(hipStreamSynchronize(s));
        L.out.release();
        L.outLds = static_cast<u32>(lds);
        L.outCap = outCap;
        // run table (BSMR_DIAG & 8192: keep the per-result positions): up to 64 consecutive CSR
        // positions of an item's sorted slots form one run; used when no item has more runs
        // than the workgroup has lanes (one descriptor per lane, loaded in the last phase)
        L.outRuns = false;
        L.runs.release();
        L.itemRuns.release();
        if (!(diag & 8192) && outCap < 65536) {
            std::vector<u32> hpos(n);
            BSMR_HIP(hipMemcpyAsync(hpos.data(), L.sortedPos.data(), n * sizeof(u32),
                                    hipMemcpyDeviceToHost, s));
            BSMR_HIP(hipStreamSynchronize(s));
            // two passes on the host threads: count each item's runs, then (offsets by a scan)
            // write them in item order into one flat table (no per-item vectors: C4 x1 holds
            // ~60 M runs)
            // a run is one wave store: at most 64 consecutive positions (an unsplit original-order
            // item is one long run, which would leave all but one wave idle in the store pass)
            auto runs_of = [&](size_t i, uint2* dst) {
                const u32 e0 = ient[i].x, len = ient[i].y;
                u32 nrun = 0;
                for (u32 t = 0; t < len;) {
                    u32 u = t + 1;
                    while (u < len && u - t < 64 && hpos[e0 + u] == hpos[e0 + u - 1] + 1) ++u;
                    if (dst) dst[nrun] = make_uint2(hpos[e0 + t], t | ((u - t) << 16));
                    ++nrun;
                    t = u;
                }
                return nrun;
            };
            std::vector<uint2> hir(ient.size(), make_uint2(0, 0));
            par_for(ient.size(), [&](unsigned, size_t i0, size_t i1) {
                for (size_t i = i0; i < i1; ++i) hir[i].y = runs_of(i, nullptr);
            });
            bool fits = true;
            size_t nr = 0;
            for (size_t i = 0; i < ient.size(); ++i) {
                fits = fits && hir[i].y <= NT;
                hir[i].x = static_cast<u32>(nr);
                nr += hir[i].y;
            }
            std::vector<uint2> hr(fits ? nr : 0);
            if (fits)
                par_for(ient.size(), [&](unsigned, size_t i0, size_t i1) {
                    for (size_t i = i0; i < i1; ++i) runs_of(i, hr.data() + hir[i].x);
                });
            if (fits) {
                BSMR_CHECK(L.runs.upload(hr.data(), std::max<size_t>(hr.size(), 1), s));
                BSMR_CHECK(L.itemRuns.upload(hir.data(), std::max<size_t>(hir.size(), 1), s));
                BSMR_HIP(hipStreamSynchronize(s));
                L.sortedPos.release();
                L.outRuns = true;
            }
        }
    } else if (n && out_packed != 0 && nnz <= (1u << 22)) {
        hipLaunchKernelGGL(k_pack_out, dim3((n + 255) / 256), dim3(256), 0, s, L.meta.data(),
                           L.out.data(), n);
        BSMR_HIP(hipGetLastError());
        BSMR_HIP(hipStreamSynchronize(s));
        L.out.release();
        L.outPacked = true;
    }
    lap("staged");
    L.dynBatches = dyn;  // (decided with the piece order above)
    BSMR_CHECK(L.items.upload(items.data(), std::max<size_t>(items.size(), 1), s));
    BSMR_CHECK(L.itemEnd.upload(ends.data(), std::max<size_t>(ends.size(), 1), s));
    BSMR_CHECK(L.pieces.upload(pieces.data(), std::max<size_t>(pieces.size(), 1), s));
    BSMR_HIP(hipStreamSynchronize(s));
    L.RB = RBr;
    L.NT = NT;
    L.lds = lds;
    L.nRB = nRB;
    L.pa = pa;
    L.pb = pb;
    L.rowEnd = qend;
    if (whole) {  // identity over the staged rows (S's rows, or for column blocks its columns)
        std::vector<u32> ids(qend);
        for (u32 r = 0; r < qend; ++r) ids[r] = r;
        BSMR_CHECK(L.rowIds.upload(ids.data(), std::max<u32>(qend, 1), s));
        BSMR_HIP(hipStreamSynchronize(s));
    }
    lap("upload");
    L.tileMin = tileMin;
    L.nTilesKept = static_cast<u32>(hkept.size());
    L.nDemoted = nd;
    L.nEntries = n;
    L.rowBytes = rowBytes;
    return BSMR_OK;
}

int Plan::build_rows(const u32* h_rowptr, const u32* h_col) {
    hipStream_t s = stream;
    hipEvent_t e0, e1;
    BSMR_HIP(hipEventCreate(&e0));
    BSMR_HIP(hipEventCreate(&e1));
    BSMR_CHECK(rowptr.upload(h_rowptr, M + 1ull, s));
    BSMR_CHECK(colidx.upload(h_col, nnz, s));
    BSMR_HIP(hipEventRecord(e0, s));

    // 1. encodings
    BSMR_CHECK(enc.alloc(std::max<u32>(nnz, 1)));
    BSMR_CHECK(nblk.alloc(M));
    BSMR_CHECK(disp.alloc(M));
    BSMR_CHECK(SC.alloc(M));
    BSMR_CHECK(S1C.alloc(M));
    const size_t lds_enc = (((nbpr + 3) & ~3u) + 16) * sizeof(u32);
    hipLaunchKernelGGL(k_encode, dim3(M), dim3(256), lds_enc, s, rowptr.data(), colidx.data(), M,
                       bs, nbpr, B, keptMask, enc.data(), nblk.data(), disp.data(), SC.data(),
                       S1C.data());
    BSMR_HIP(hipGetLastError());

    // 2. ascending = rows stably sorted by dispersion
    DevBuf<u32> keys_sorted, iota;
    BSMR_CHECK(keys_sorted.alloc(M));
    BSMR_CHECK(iota.alloc(M));
    BSMR_CHECK(asc.alloc(M));
    hipLaunchKernelGGL(k_iota, dim3(grid_for(M, 256)), dim3(256), 0, s, iota.data(), M);
    BSMR_CHECK(sort_pairs(disp.data(), keys_sorted.data(), iota.data(), asc.data(), M, 32, tmp, s));
    DevBuf<u32> zdev;
    BSMR_CHECK(zdev.alloc(1));
    BSMR_HIP(hipMemsetAsync(zdev.data(), 0, sizeof(u32), s));
    hipLaunchKernelGGL(k_count_zero, dim3(grid_for(M, 256)), dim3(256), 0, s, keys_sorted.data(), M,
                       zdev.data());
    BSMR_CHECK(read_one(zdev.data(), z, s));

    // 3. clustering
    DevBuf<u32> state, st, ctrl;
    BSMR_CHECK(state.alloc(M));
    BSMR_CHECK(st.alloc(M + 2ull + CL_TMAX));  // the last tile may name up to T - 1 ids past M
    BSMR_CHECK(ctrl.alloc(8));
    BSMR_HIP(hipMemsetAsync(st.data(), 0, (M + 2ull + CL_TMAX) * sizeof(u32), s));
    BSMR_HIP(hipMemsetAsync(ctrl.data(), 0, 8 * sizeof(u32), s));
    hipLaunchKernelGGL(k_init_state, dim3(grid_for(M, 256)), dim3(256), 0, s, state.data(), st.data(),
                       M, z);
    BSMR_HIP(hipGetLastError());
    DevBuf<uint4> pmeta;
    BSMR_CHECK(pmeta.alloc(M));
    hipLaunchKernelGGL(k_pmeta, dim3(grid_for(M, 256)), dim3(256), 0, s, asc.data(), rowptr.data(),
                       nblk.data(), SC.data(), S1C.data(), M, pmeta.data());
    BSMR_HIP(hipGetLastError());
    // candidate filter: an MFMA pass over every pair of rows bounds their similarity, so the
    // chain skips the pairs that cannot reach alpha (cluster_filter.hip)
    // cluster_filter = 1: from the start; auto (-1, from filter_min_rows rows): after a first
    // launch of about 1,536 clusters without it, when those took at least one position in four
    // (most positions then start their own cluster and the chain compares nearly every pair;
    // patterns whose rows join a few clusters finish cheaply without it: cop20k-like alpha 0.1
    // 87 ms unfiltered against a 125 ms filter pass, profiles/r04ze)
    DevBuf<u32> fbits;
    u32 fW = 0;
    filter_used = false;
    filter_ms = 0.f;
    const bool filter_ok = cluster_filter != 0 && !exact_all && alpha >= 0.01f && M - z >= 2 &&
                           (cluster_filter == 1 || M >= filter_min_rows);
    auto build_filter = [&]() -> int {
        size_t fr = 0, tot = 0;
        BSMR_HIP(hipMemGetInfo(&fr, &tot));
        const u64 Kp = (nbpr + 63ull) / 64 * 64;
        const u64 need = static_cast<u64>(M) * Kp * 2 + sim_filter_words(M) * 4 + static_cast<u64>(M) * 8;
        if (need > fr / 4) return BSMR_OK;  // (the chain runs unfiltered)
        hipEvent_t f0, f1;
        BSMR_HIP(hipEventCreate(&f0));
        BSMR_HIP(hipEventCreate(&f1));
        BSMR_HIP(hipEventRecord(f0, s));
        BSMR_CHECK(build_sim_filter(pmeta.data(), enc.data(), M, nbpr, B, keptMask, alpha, fbits, fW, s));
        BSMR_HIP(hipEventRecord(f1, s));
        BSMR_HIP(hipEventSynchronize(f1));
        BSMR_HIP(hipEventElapsedTime(&filter_ms, f0, f1));
        BSMR_HIP(hipEventDestroy(f0));
        BSMR_HIP(hipEventDestroy(f1));
        filter_used = true;
        return BSMR_OK;
    };
    if (filter_ok && cluster_filter == 1) BSMR_CHECK(build_filter());
    bool probe = filter_ok && cluster_filter != 1;
    ClusterArgs ca{};
    ca.fbits = filter_used ? fbits.data() : nullptr;
    ca.fW = fW;
    ca.pmeta = pmeta.data();
    ca.enc = enc.data();
    ca.state = state.data();
    ca.st = st.data();
    ca.ctrl = ctrl.data();
    ca.M = M;
    ca.nbpr = nbpr;
    ca.B = B;
    ca.keptMask = keptMask;
    ca.allKept = keptMask == (B / 32 >= 32 ? 0xFFFFFFFFu : (1u << (B / 32)) - 1u) ? 1u : 0u;
    ca.alpha = alpha;
    ca.exact_all = exact_all;
    ca.timeout_ticks = 100ull * 1000 * 1000 * 20;  // 20 s without progress
    // tile of T clusters: as many representatives as fit the LDS budget, at most CL_TMAX, an
    // even number (block b of cluster c at reps[b * T + c]: 8- or 16-byte LDS reads of all T)
    const u32 NP = (nbpr + 3) & ~3u;
    u32 T = std::max<u32>(2, std::min<u32>(CL_TMAX, CL_LDS_BUDGET / (NP * 4)) & ~1u);
    if (diag & 65536) T = std::min<u32>(T, 4);  // (experiment: 4 clusters per tile)
    ca.NP = NP;
    ca.T = T;
    const size_t lds_cl = static_cast<size_t>(T) * NP * 4 + sizeof(ClusterCtl);
    // clusters per launch (a multiple of T): each tile takes the next T cluster ids from a
    // ticket counter and waits only for its predecessor tile, which therefore has always started,
    // so more tiles than fit on the chip at once cannot deadlock (later ones start as earlier
    // ones finish); capped by the exact path's scratch (<= 256 MiB)
    const u32 Rcap = static_cast<u32>(std::max<u64>(
        T, std::min<u64>(cluster_batch, (64ull << 20) / std::max<u32>(nbpr, 1)) / T * T));
    const u32 tilesMax = Rcap / T;
    DevBuf<u32> cmpScratch;
    BSMR_CHECK(cmpScratch.alloc(static_cast<size_t>(tilesMax) * nbpr));
    BSMR_HIP(hipMemsetAsync(cmpScratch.data(), 0, static_cast<size_t>(tilesMax) * nbpr * sizeof(u32), s));
    ca.cmpScratch = cmpScratch.data();
    ca.ctrace = nullptr;
    if (diag & 2048) {  // clustering timeline (tools/cluster_trace.py): 16 u64 per tile
        BSMR_CHECK(prepare_trace((static_cast<size_t>(M) / T + 2) * 4, s));
        ca.ctrace = trace.data();
    }
    u32 c0 = 1;
    u32 last_valid = 0;
    while (c0 <= M) {  // at most M - z clusters
        // (the probe launch too stays within tilesMax: the exact path's scratch has tilesMax rows)
        const u32 tiles = std::min<u32>(probe ? std::min<u32>(tilesMax, std::max<u32>(1, 1536 / T)) : tilesMax,
                                        (M + 1 - c0 + T - 1) / T);
        const u32 R = tiles * T;
        ca.c0 = c0;
        BSMR_HIP(hipMemsetAsync(ctrl.data() + 6, 0, sizeof(u32), s));  // ticket counter
        switch (T) {
            case 2: hipLaunchKernelGGL(k_cluster<2>, dim3(tiles), dim3(64 * CL_WAVES), lds_cl, s, ca); break;
            case 4: hipLaunchKernelGGL(k_cluster<4>, dim3(tiles), dim3(64 * CL_WAVES), lds_cl, s, ca); break;
            case 6: hipLaunchKernelGGL(k_cluster<6>, dim3(tiles), dim3(64 * CL_WAVES), lds_cl, s, ca); break;
            default: hipLaunchKernelGGL(k_cluster<8>, dim3(tiles), dim3(64 * CL_WAVES), lds_cl, s, ca); break;
        }
        BSMR_HIP(hipGetLastError());
        std::vector<u32> hst(R);
        BSMR_HIP(hipMemcpyAsync(hst.data(), st.data() + c0, R * sizeof(u32), hipMemcpyDeviceToHost, s));
        u32 hctrl[8];
        BSMR_HIP(hipMemcpyAsync(hctrl, ctrl.data(), sizeof(hctrl), hipMemcpyDeviceToHost, s));
        BSMR_HIP(hipStreamSynchronize(s));
        if (hctrl[0]) {
            set_error("clustering kernel aborted (timeout waiting for predecessor)");
            return BSMR_ERR_TIMEOUT;
        }
        bool done = false;
        for (u32 j = 0; j < R; ++j) {
            if (hst[j] == ST_NONE) {
                done = true;
                break;
            }
            last_valid = c0 + j;
        }
        exact_evals = (static_cast<u64>(hctrl[3]) << 32) | hctrl[2];
        total_evals = (static_cast<u64>(hctrl[5]) << 32) | hctrl[4];
        if (done) break;
        if (probe) {
            // the probe launch's last cluster started at position hst[R - 1] - 2
            probe = false;
            const u32 pos = hst[R - 1] - 2;
            if (pos >= z && 4ull * R >= static_cast<u64>(pos - z + 1)) {
                BSMR_CHECK(build_filter());
                ca.fbits = filter_used ? fbits.data() : nullptr;
                ca.fW = fW;
            }
        }
        c0 += R;
    }
    (void)last_valid;

    // 4. stable sort of positions by cluster id
    DevBuf<u32> ids, sorted_ids, indices;
    BSMR_CHECK(ids.alloc(M));
    BSMR_CHECK(sorted_ids.alloc(M));
    BSMR_CHECK(indices.alloc(M));
    hipLaunchKernelGGL(k_ids, dim3(grid_for(M, 256)), dim3(256), 0, s, state.data(), ids.data(), M);
    BSMR_CHECK(sort_pairs(ids.data(), sorted_ids.data(), iota.data(), indices.data(), M,
                          bits_for(M + 1ull), tmp, s));
    R = M - z;
    BSMR_CHECK(rows.alloc(std::max<u32>(R, 1)));
    hipLaunchKernelGGL(k_perm, dim3(grid_for(R, 256)), dim3(256), 0, s, asc.data(), indices.data(), z,
                       R, rows.data());
    BSMR_HIP(hipGetLastError());
    // numClusters = sorted_ids[indices[M-1]] + (zero rows ? 1 : 0) (rowReordering.cu:996)
    u32 last_index = 0, id_at = 0;
    BSMR_CHECK(read_one(indices.data() + (M - 1), last_index, s));
    BSMR_CHECK(read_one(sorted_ids.data() + last_index, id_at, s));
    numClusters = static_cast<int32_t>(id_at) + (z != 0 ? 1 : 0);
    P = (R + 15) / 16;  // ceil(float(R)/16) (BSMR.cpp:48)

    BSMR_HIP(hipEventRecord(e1, s));
    BSMR_HIP(hipEventSynchronize(e1));
    BSMR_HIP(hipEventElapsedTime(&row_ms, e0, e1));
    BSMR_HIP(hipEventDestroy(e0));
    BSMR_HIP(hipEventDestroy(e1));
    // the encodings are only needed by the clustering
    enc.release();
    SC.release();
    S1C.release();
    return BSMR_OK;
}

int Plan::build_columns() {
    hipStream_t s = stream;
    hipEvent_t e0, e1;
    BSMR_HIP(hipEventCreate(&e0));
    BSMR_HIP(hipEventCreate(&e1));
    BSMR_HIP(hipEventRecord(e0, s));
    if (!segments_ready) {
        DevBuf<u32> rn;
        BSMR_CHECK(rn.alloc(std::max<u32>(R, 1)));
        BSMR_CHECK(roff.alloc(R + 1ull));
        hipLaunchKernelGGL(k_row_nnz, dim3(grid_for(R, 256)), dim3(256), 0, s, rowptr.data(),
                           rows.data(), R, rn.data());
        BSMR_CHECK(excl_scan(rn.data(), roff.data(), R, tmp, s));
        DevBuf<u32> keys, vals;
        BSMR_CHECK(keys.alloc(nnz));
        BSMR_CHECK(vals.alloc(nnz));
        BSMR_CHECK(skeys.alloc(nnz));
        BSMR_CHECK(svals.alloc(nnz));
        BSMR_CHECK(ent_lr.alloc(nnz));
        BSMR_CHECK(ent_idx.alloc(nnz));
        hipLaunchKernelGGL(k_gather, dim3(grid_for(R, 4)), dim3(256), 0, s, rowptr.data(),
                           colidx.data(), rows.data(), roff.data(), R, keys.data(), vals.data(),
                           ent_lr.data(), ent_idx.data());
        BSMR_CHECK(seg_begin.alloc(P));
        BSMR_CHECK(seg_end.alloc(P));
        hipLaunchKernelGGL(k_segments, dim3(grid_for(P, 256)), dim3(256), 0, s, roff.data(), R, P,
                           seg_begin.data(), seg_end.data());
        BSMR_HIP(hipGetLastError());
        size_t bytes = 0;
        const int endbit = bits_for(N);
        BSMR_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(
            nullptr, bytes, keys.data(), skeys.data(), vals.data(), svals.data(),
            static_cast<int>(nnz), static_cast<int>(P), seg_begin.data(), seg_end.data(), 0, endbit,
            s));
        if (bytes > tmp.size()) BSMR_CHECK(tmp.alloc(bytes));
        BSMR_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(
            tmp.data(), bytes, keys.data(), skeys.data(), vals.data(), svals.data(),
            static_cast<int>(nnz), static_cast<int>(P), seg_begin.data(), seg_end.data(), 0, endbit,
            s));
        segments_ready = true;
    }
    for (auto& L : rbl) L.rowBytes = 0;  // launch layouts depend on the column split
    shard_rbl.clear();
    // pass 1
    const u32 thr =static_cast<u32>(std::ceil(delta * static_cast<float>(TILE)));  // colReordering.cu:246
    DevBuf<u32> phist, pnd, pns, psd;
    BSMR_CHECK(phist.alloc(16ull * P));
    BSMR_CHECK(pnd.alloc(P));
    BSMR_CHECK(pns.alloc(P));
    BSMR_CHECK(psd.alloc(P));
    hipLaunchKernelGGL(k_panel_pass1, dim3(P), dim3(256), 0, s, seg_begin.data(), seg_end.data(),
                       skeys.data(), thr, phist.data(), pnd.data(), pns.data(), psd.data());
    BSMR_HIP(hipGetLastError());
    BSMR_CHECK(denseColOffsets.alloc(P + 1ull));
    BSMR_CHECK(sparseColOffsets.alloc(P + 1ull));
    BSMR_CHECK(sparseValueOffsets.alloc(P + 1ull));
    BSMR_CHECK(blockOffsets.alloc(P + 1ull));
    BSMR_CHECK(excl_scan(pnd.data(), denseColOffsets.data(), P, tmp, s));
    BSMR_CHECK(excl_scan(pns.data(), sparseColOffsets.data(), P, tmp, s));
    BSMR_CHECK(excl_scan(psd.data(), sparseValueOffsets.data(), P, tmp, s));
    hipLaunchKernelGGL(k_div16, dim3(grid_for(P + 1ull, 256)), dim3(256), 0, s, denseColOffsets.data(),
                       blockOffsets.data(), P + 1);
    u32 nDenseCols = 0, nSparseCols = 0;
    BSMR_CHECK(read_one(denseColOffsets.data() + P, nDenseCols, s));
    BSMR_CHECK(read_one(sparseColOffsets.data() + P, nSparseCols, s));
    BSMR_CHECK(read_one(sparseValueOffsets.data() + P, nres, s));
    numDenseTiles = nDenseCols / 16;
    BSMR_CHECK(denseCols.alloc(std::max<u32>(nDenseCols, 1)));
    BSMR_CHECK(sparseCols.alloc(std::max<u32>(nSparseCols, 1)));
    BSMR_CHECK(blockValues.alloc(std::max<u64>(static_cast<u64>(numDenseTiles) * TILE, 1)));
    BSMR_CHECK(sparseValues.alloc(std::max<u32>(nres, 1)));
    BSMR_CHECK(sparseRel.alloc(std::max<u32>(nres, 1)));
    BSMR_CHECK(sparseColIdx.alloc(std::max<u32>(nres, 1)));
    denseCols.n = nDenseCols;
    sparseCols.n = nSparseCols;
    blockValues.n = static_cast<size_t>(numDenseTiles) * TILE;
    sparseValues.n = sparseRel.n = sparseColIdx.n = nres;
    if (blockValues.n)
        BSMR_HIP(hipMemsetAsync(blockValues.data(), 0xFF, blockValues.n * sizeof(u32), s));
    hipLaunchKernelGGL(k_panel_pass2, dim3(P), dim3(256), 0, s, seg_begin.data(), seg_end.data(),
                       skeys.data(), svals.data(), ent_lr.data(), ent_idx.data(), phist.data(),
                       pnd.data(), denseColOffsets.data(), sparseColOffsets.data(),
                       sparseValueOffsets.data(), N, denseCols.data(), sparseCols.data(),
                       blockValues.data(), sparseValues.data(), sparseRel.data(),
                       sparseColIdx.data());
    BSMR_HIP(hipGetLastError());

    // column-major residual execution list + XCD-interleaved slots
    {
        const u32 n = nres;
        BSMR_CHECK(cmRow.alloc(std::max<u32>(n, 1)));
        BSMR_CHECK(cmCol.alloc(std::max<u32>(n, 1)));
        BSMR_CHECK(cmOut.alloc(std::max<u32>(n, 1)));
        std::vector<u32> ends(XCD_BUCKETS, 0);
        if (n) {
            DevBuf<u32> keys, vals, skeys2, order, rowOf, bcount;
            BSMR_CHECK(keys.alloc(n));
            BSMR_CHECK(vals.alloc(n));
            BSMR_CHECK(skeys2.alloc(n));
            BSMR_CHECK(order.alloc(n));
            BSMR_CHECK(rowOf.alloc(n));
            BSMR_CHECK(bcount.alloc(XCD_BUCKETS));
            BSMR_HIP(hipMemsetAsync(bcount.data(), 0, XCD_BUCKETS * sizeof(u32), s));
            hipLaunchKernelGGL(k_cm_keys, dim3(P), dim3(256), 0, s, sparseValueOffsets.data(),
                               rows.data(), sparseRel.data(), sparseColIdx.data(), N, keys.data(),
                               vals.data(), rowOf.data());
            BSMR_CHECK(sort_pairs(keys.data(), skeys2.data(), vals.data(), order.data(), n,
                                  bits_for(static_cast<u64>(XCD_BUCKETS) * N), tmp, s));
            hipLaunchKernelGGL(k_cm_gather, dim3(grid_for(n, 256)), dim3(256), 0, s, order.data(),
                               rowOf.data(), sparseColIdx.data(), sparseValues.data(),
                               skeys2.data(), n, N, cmRow.data(), cmCol.data(), cmOut.data(),
                               bcount.data());
            BSMR_HIP(hipGetLastError());
            BSMR_HIP(hipMemcpyAsync(ends.data(), bcount.data(), XCD_BUCKETS * sizeof(u32),
                                    hipMemcpyDeviceToHost, s));
            BSMR_HIP(hipStreamSynchronize(s));
            for (u32 b = 1; b < XCD_BUCKETS; ++b) ends[b] = std::max(ends[b], ends[b - 1]);
        }
        u32 rmax = 0;
        std::vector<u32> begins(XCD_BUCKETS, 0);
        for (u32 b = 0; b < XCD_BUCKETS; ++b) {
            begins[b] = b ? ends[b - 1] : 0;
            rmax = std::max(rmax, (ends[b] - begins[b] + CM_PER_ITEM - 1) / CM_PER_ITEM);
        }
        // the launch runs 4 waves (slots) per workgroup and deals workgroups round-robin over
        // the 8 XCDs: slot s lives in workgroup s / 4, on XCD (s / 4) % 8 = its bucket
        rmax = (rmax + 3) & ~3u;
        nSlots = rmax * XCD_BUCKETS;
        std::vector<uint2> slots(std::max<u32>(nSlots, 1), make_uint2(0, 0));
        for (u32 b = 0; b < XCD_BUCKETS; ++b)
            for (u32 j = 0; j < rmax; ++j) {
                const u32 e0 = std::min(begins[b] + j * CM_PER_ITEM, ends[b]);
                const u32 s = ((j / 4) * XCD_BUCKETS + b) * 4 + (j % 4);
                slots[s] = make_uint2(e0, std::min(e0 + CM_PER_ITEM, ends[b]));
            }
        BSMR_CHECK(cmSlots.upload(slots.data(), slots.size(), s));
        BSMR_HIP(hipStreamSynchronize(s));  // `slots` is pageable host memory
    }

    // 6. work lists
    DevBuf<u32> dc, rc, doffs, roffs;
    BSMR_CHECK(dc.alloc(P));
    BSMR_CHECK(rc.alloc(P));
    BSMR_CHECK(doffs.alloc(P + 1ull));
    BSMR_CHECK(roffs.alloc(P + 1ull));
    hipLaunchKernelGGL(k_item_counts, dim3(grid_for(P, 256)), dim3(256), 0, s, pnd.data(), psd.data(),
                       P, TILES_PER_ITEM, RES_PER_ITEM, dc.data(), rc.data());
    BSMR_CHECK(excl_scan(dc.data(), doffs.data(), P, tmp, s));
    BSMR_CHECK(excl_scan(rc.data(), roffs.data(), P, tmp, s));
    BSMR_CHECK(read_one(doffs.data() + P, nDenseItems, s));
    BSMR_CHECK(read_one(roffs.data() + P, nResItems, s));
    BSMR_CHECK(denseItems.alloc(std::max<u32>(nDenseItems, 1)));
    BSMR_CHECK(resItems.alloc(std::max<u32>(nResItems, 1)));
    hipLaunchKernelGGL(k_item_fill, dim3(grid_for(P, 256)), dim3(256), 0, s, denseColOffsets.data(),
                       sparseValueOffsets.data(), doffs.data(), roffs.data(), P, TILES_PER_ITEM,
                       RES_PER_ITEM, denseItems.data(), resItems.data());
    BSMR_HIP(hipGetLastError());
    BSMR_CHECK(tileRows.alloc(std::max<u64>(static_cast<u64>(numDenseTiles) * 16, 1)));
    if (nDenseItems)
        hipLaunchKernelGGL(k_tile_rows, dim3(grid_for(nDenseItems, 16)), dim3(256), 0, s,
                           denseItems.data(), nDenseItems, rows.data(), R, tileRows.data());
    BSMR_HIP(hipGetLastError());

    // host copies of the small per-panel arrays (shard cost model, stats)
    BSMR_CHECK(blockOffsets.download(h_blockOffsets, s));
    BSMR_CHECK(sparseValueOffsets.download(h_sparseValueOffsets, s));
    maxTilesPerPanel = 0;
    numSparseTB = 0;
    numDenseTB = 0;
    for (u32 p = 0; p < P; ++p) {
        const u32 nt = h_blockOffsets[p + 1] - h_blockOffsets[p];
        maxTilesPerPanel = std::max(maxTilesPerPanel, nt);
        numDenseTB += static_cast<u32>(std::ceil(static_cast<float>(nt) / REF_DENSE_BLOCKS_PER_TB));
        numSparseTB += static_cast<u32>(std::ceil(
            static_cast<float>(h_sparseValueOffsets[p + 1] - h_sparseValueOffsets[p]) /
            REF_SPARSE_DATA_PER_TB));
    }

    BSMR_HIP(hipEventRecord(e1, s));
    BSMR_HIP(hipEventSynchronize(e1));
    BSMR_HIP(hipEventElapsedTime(&col_ms, e0, e1));
    BSMR_HIP(hipEventDestroy(e0));
    BSMR_HIP(hipEventDestroy(e1));
    return BSMR_OK;
}

}  // namespace bsmr
