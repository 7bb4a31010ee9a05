// sddmm_dense.hip — dense-sampled SDDMM for fp16/bf16 operands on patterns dense enough that
// computing whole 128 x 128 output tiles on the matrix cores beats gathering entry by entry
// (DLMC-like 90 %-sparse masks, BASELINE.json C5: "MFMA-utilisation stress").
//
// Tile (tm, tn) = rows [128 tm, +128) x columns [128 tn, +128) of P = A B^T in the ORIGINAL index
// space (the reordering does not change which dot products exist). One 256-thread workgroup per
// non-empty tile: the K loop streams 64-wide k-chunks of the tile's 128 A rows and 128 B rows
// (128 bytes each) into LDS by LDS-DMA through a ring of NS stages (NS - 1 chunks in flight while
// one computes; NS = 2 fits two workgroups per CU, so one tile's prologue and epilogue overlap
// another's MFMAs); wave (wy, wx) owns a 64 x 64 quadrant as
// 4 x 4 `v_mfma_f32_16x16x32_{f16,bf16}` accumulators (fp32). The finished tile goes through LDS
// (fp32) and the workgroup writes exactly the tile's stored entries to P, in CSR order positions
// (Plan::DenseLayout: per-tile entry lists of local row << 7 | local column and output index).
// Tiles are dealt so that XCD x works on a contiguous band of tile rows (A panels and all of B
// stay in its L2).
#include <algorithm>
#include <vector>

#include "common.hpp"
#include "plan.hpp"

namespace bsmr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));

constexpr u32 DT_TILE = 128;   // output tile edge
// k-chunk per barrier KC: 64 (two MFMA k-steps of 32; 128-byte rows) or 32 (one; 64-byte rows)
template <u32 KC>
constexpr u32 chunk_bytes() { return DT_TILE * KC * 2; }  // one operand chunk image

struct DenseArgs {
    const char* A;  // M x K halves, row-major
    const char* B;  // N x K halves (B column-major)
    float* P;
    const u32* off;  // [tiles + 1] entry ranges per tile
    const u32* loc;  // local row << 7 | local column
    const u32* out;  // CSR position
    u32 M, N, K, ntn, ntiles;
    unsigned long long bA, bB, bP;  // batched launch: A/B byte strides, P element stride
    unsigned long long* trace;      // BSMR_DIAG & 32: per workgroup {start, chunk 0 landed,
                                    // end, xcc << 60 | k-loop end} (s_memrealtime); else null
};

// 16-byte slot of (row r, k-group g) in a chunk image of KC/8 groups per row: the groups of a
// row permuted by a row-dependent XOR so the 16 lanes of each ds_read_b128 lane group (rows
// l & 15, one group) hit 16 distinct 16-byte bank groups
template <u32 KC>
__device__ __forceinline__ u32 dswz(u32 r) {
    return KC == 64 ? (r >> 1) & 7 : (r >> 2) & 3;
}
template <u32 KC>
__device__ __forceinline__ u32 dslot(u32 r, u32 g) { return (KC / 8) * r + (g ^ dswz<KC>(r)); }

// one wave-wide 16-byte-per-lane LDS-DMA (lane l lands at l*16 past the wave-uniform l).
// Issued by inline asm on purpose: the compiler's wait-count pass loses track of LDS-DMA
// stores across the k-loop's back edge and would put a vmcnt(0) at its head; these DMAs are
// instead ordered by the kernel's own vmcnt waits + barriers.
__device__ __forceinline__ void lds_dma16(const char* g, char* l) {
    const u32 m0 = __builtin_amdgcn_readfirstlane(static_cast<u32>(
        reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)l)));
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0)
                 : "memory", "m0");
}

// LDS-DMAs per wave and operand for one chunk (16 KiB images of 1 KiB wave-instructions)
template <u32 KC, u32 NWAV>
constexpr u32 dense_nd() { return KC / 16 * 4 / NWAV; }

// chunk kc of the tile's A and B rows into (sa, sb), spread over NWAV waves; no branches (rows
// past M / N read the last row; they are never sampled)
template <u32 KC, u32 NWAV>
__device__ __forceinline__ void dense_stage(const DenseArgs& a, const u32 r0, const u32 c0,
                                            const u32 kc, const u32 ws, const u32 lane, char* sa,
                                            char* sb) {
    constexpr u32 ND = dense_nd<KC, NWAV>(), GP = KC / 8;
    const size_t rowB = static_cast<size_t>(a.K) * 2;
#pragma unroll
    for (u32 i = 0; i < ND; ++i) {
        const u32 s = 64 * (ND * ws + i) + lane, r = s / GP, g = (s % GP) ^ dswz<KC>(r);
        const u32 ra = min(r0 + r, a.M - 1), rb = min(c0 + r, a.N - 1);
        const size_t ko = static_cast<size_t>(kc) * (KC * 2) + 16 * g;
        lds_dma16(a.A + ra * rowB + ko, sa + 1024 * (ND * ws + i));
        lds_dma16(a.B + rb * rowB + ko, sb + 1024 * (ND * ws + i));
    }
}

template <int DT>
__device__ __forceinline__ f32x4 mfma16x16x32(const f32x4 x, const f32x4 y, const f32x4 c) {
    if constexpr (DT == 1)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h16x8, x),
                                                      __builtin_bit_cast(h16x8, y), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b16x8, x),
                                                       __builtin_bit_cast(b16x8, y), c, 0, 0, 0);
}

// one k-chunk of the wave's 64 x (16 NJ) block of the tile from the images (sa, sb): rows
// [64 wy, +64) of A, rows [16 NJ wx, +16 NJ) of B, every k-step
template <int DT, u32 KC, u32 NJ>
__device__ __forceinline__ void dense_chunk(const char* sa, const char* sb, const u32 wy,
                                            const u32 wx, const u32 lane, f32x4 (&acc)[4][NJ]) {
    const u32 rr = lane & 15, g4 = lane >> 4;
#pragma unroll
    for (u32 ks = 0; ks < KC / 32; ++ks) {
        f32x4 av[4], bv[NJ];
#pragma unroll
        for (u32 i = 0; i < 4; ++i) {
            const u32 ra = 64 * wy + 16 * i + rr;
            av[i] = *reinterpret_cast<const f32x4*>(sa + 16 * dslot<KC>(ra, 4 * ks + g4));
        }
#pragma unroll
        for (u32 j = 0; j < NJ; ++j) {
            const u32 rb = 16 * NJ * wx + 16 * j + rr;
            bv[j] = *reinterpret_cast<const f32x4*>(sb + 16 * dslot<KC>(rb, 4 * ks + g4));
        }
#pragma unroll
        for (u32 i = 0; i < 4; ++i)
#pragma unroll
            for (u32 j = 0; j < NJ; ++j) acc[i][j] = mfma16x16x32<DT>(av[i], bv[j], acc[i][j]);
    }
}

template <u32 KC, u32 NS>
constexpr u32 dense_lds() { return NS * 2 * chunk_bytes<KC>(); }
// workgroups per CU the LDS allows (160 KiB), capped at 4 (VGPR budget 128)
template <u32 KC, u32 NS>
constexpr u32 dense_wgs() { return 160u * 1024 / dense_lds<KC, NS>() < 4 ? 160u * 1024 / dense_lds<KC, NS>() : 4; }

// NW = 4: four waves, a 64 x 64 quadrant each. NW = 8: eight waves, a 64 x 32 block each (two
// waves per SIMD, so one wave's LDS reads run under the other's MFMAs when the tiles give one
// workgroup per CU)
template <int DT, u32 KC, u32 NS, u32 NW>
__global__ __launch_bounds__(64 * NW)
__attribute__((amdgpu_waves_per_eu(dense_wgs<KC, NS>() * NW / 4 < 4 ? dense_wgs<KC, NS>() * NW / 4 : 4)))
void k_sddmm_dense(DenseArgs a) {
    constexpr u32 NT = 64 * NW, ND = dense_nd<KC, NW>(), NJ = 16 / NW;
    constexpr u32 CB = chunk_bytes<KC>(), LDS = dense_lds<KC, NS>();
    static_assert(LDS >= DT_TILE * DT_TILE * 4, "the fp32 tile fits the stage images");
    __shared__ __attribute__((aligned(16))) char st[LDS];
    if (blockIdx.y) {
        a.A += blockIdx.y * a.bA;
        a.B += blockIdx.y * a.bB;
        a.P += blockIdx.y * a.bP;
    }
    // XCD x = blockIdx % 8 takes the x-th contiguous eighth of the tiles (tile rows together)
    const u32 per = (a.ntiles + XCD_BUCKETS - 1) / XCD_BUCKETS;
    const u32 t = (blockIdx.x % XCD_BUCKETS) * per + blockIdx.x / XCD_BUCKETS;
    if (t >= a.ntiles) return;
    const u32 e0 = a.off[t], e1 = a.off[t + 1];
    if (e0 == e1) return;  // no stored entry in this tile (uniform)
    const u32 tm = t / a.ntn, tn = t - tm * a.ntn;
    const u32 r0 = DT_TILE * tm, c0 = DT_TILE * tn;
    const u32 tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const u32 ws = __builtin_amdgcn_readfirstlane(w);
    const u32 wy = NW == 4 ? ws >> 1 : ws >> 2, wx = NW == 4 ? ws & 1 : ws & 3;
    f32x4 acc[4][NJ];
#pragma unroll
    for (u32 i = 0; i < 4; ++i)
#pragma unroll
        for (u32 jj = 0; jj < NJ; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned long long t_start = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    unsigned long long t_first = 0;
    const u32 nk = a.K / KC;  // launch_dense: K a multiple of KC
    // chunk kc lands in stage kc % NS. Before a stage is read every wave waits for its own
    // LDS-DMAs into it (2 ND per chunk; those of the younger chunks already issued may stay in
    // flight) and the workgroup barrier then makes everyone's visible; the same barrier ends all
    // reads of the stage the next prefetch overwrites. No chunk past the last is staged.
    auto stage = [&](const u32 kc) {
        char* const sa = st + (kc % NS) * (2 * CB);
        dense_stage<KC, NW>(a, r0, c0, kc, ws, lane, sa, sa + CB);
    };
#pragma unroll
    for (u32 j = 0; j + 1 < NS; ++j)
        if (j < nk) stage(j);
    for (u32 kc = 0; kc < nk; ++kc) {
        if (NS > 2 && kc + NS - 2 < nk)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * ND * (NS > 2 ? NS - 2 : 0)) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if (a.trace && kc == 0) t_first = __builtin_amdgcn_s_memrealtime();
        if (kc + NS - 1 < nk) stage(kc + NS - 1);
        const char* const sa = st + (kc % NS) * (2 * CB);
        dense_chunk<DT, KC, NJ>(sa, sa + CB, wy, wx, lane, acc);
    }
    // the first PF entries of each thread's share of the tile's stored entries (local offset,
    // CSR position), loaded right after the k-loop (after every LDS-DMA, so no chunk wait
    // includes them): their latency runs under the tile's LDS pass instead of after it
    constexpr u32 PF = 4;
    u32 pl[PF], po[PF];
#pragma unroll
    for (u32 q = 0; q < PF; ++q) {  // unconditional (clamped) loads: all 2 PF in flight at once
        const u32 e = e0 + tid + NT * q, ec = min(e, e1 - 1);
        const u32 lv = a.loc[ec], ov = a.out[ec];
        pl[q] = e < e1 ? lv : NULLV;
        po[q] = ov;
    }
    // every read of the images done (every LDS-DMA landed at the last chunk's wait): they
    // become the fp32 tile, element (r, c) at ((r >> 2) * 128 + c) * 4 + (r & 3), so a lane's
    // four accumulator rows are one 16-byte store
    __syncthreads();
    const unsigned long long t_loop = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    float* const ct = reinterpret_cast<float*>(st);
    // accumulator (i, jj) reg r of lane l = D[64 wy + 16 i + 4 (l >> 4) + r][16 NJ wx + 16 jj + (l & 15)]
#pragma unroll
    for (u32 i = 0; i < 4; ++i)
#pragma unroll
        for (u32 jj = 0; jj < NJ; ++jj) {
            const u32 rq = 16 * wy + 4 * i + (lane >> 4), col = 16 * NJ * wx + 16 * jj + (lane & 15);
            *reinterpret_cast<f32x4*>(ct + (rq * DT_TILE + col) * 4) = acc[i][jj];
        }
    __syncthreads();
    auto at = [&](u32 lc) {  // loc = local row << 7 | local column
        return ct[((lc >> 9) * DT_TILE + (lc & 127)) * 4 + ((lc >> 7) & 3)];
    };
#pragma unroll
    for (u32 q = 0; q < PF; ++q)
        if (pl[q] != NULLV) a.P[po[q]] = at(pl[q]);
    // denser tiles: the rest PF entries at a time, loads unconditional so they overlap
    for (u32 eb = e0 + tid + NT * PF; eb < e1; eb += NT * PF) {
        u32 lv[PF], ov[PF];
#pragma unroll
        for (u32 q = 0; q < PF; ++q) {
            const u32 ec = min(eb + NT * q, e1 - 1);
            lv[q] = a.loc[ec];
            ov[q] = a.out[ec];
        }
#pragma unroll
        for (u32 q = 0; q < PF; ++q)
            if (eb + NT * q < e1) a.P[ov[q]] = at(lv[q]);
    }
    if (a.trace && tid == 0) {
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        const u32 xcc = __builtin_amdgcn_s_getreg(0xF814);  // HW_REG_XCC_ID
        unsigned long long* tr = a.trace + 4ull * (blockIdx.y * gridDim.x + blockIdx.x);
        tr[0] = t_start;
        tr[1] = t_first;
        tr[2] = t_end;
        tr[3] = (static_cast<unsigned long long>(xcc) << 60) | t_loop;
    }
}

}  // namespace

// Per-tile entry lists of the dense-sampled launch (built on first use).
int Plan::build_dense_layout() const {
    DenseLayout& D = dense;
    std::vector<u32> hrp, hci;
    BSMR_CHECK(rowptr.download(hrp, stream));
    BSMR_CHECK(colidx.download(hci, stream));
    const u32 ntm = (M + DT_TILE - 1) / DT_TILE, ntn = (N + DT_TILE - 1) / DT_TILE;
    const size_t ntiles = static_cast<size_t>(ntm) * ntn;
    std::vector<u32> off(ntiles + 1, 0), loc(std::max<u32>(nnz, 1)), out(std::max<u32>(nnz, 1));
    for (u32 r = 0; r < M; ++r)
        for (u32 e = hrp[r]; e < hrp[r + 1]; ++e) ++off[(r / DT_TILE) * static_cast<size_t>(ntn) + hci[e] / DT_TILE + 1];
    for (size_t t = 0; t < ntiles; ++t) off[t + 1] += off[t];
    std::vector<u32> pos(off.begin(), off.end() - 1);
    for (u32 r = 0; r < M; ++r)
        for (u32 e = hrp[r]; e < hrp[r + 1]; ++e) {
            const u32 c = hci[e];
            const u32 k = pos[(r / DT_TILE) * static_cast<size_t>(ntn) + c / DT_TILE]++;
            loc[k] = ((r % DT_TILE) << 7) | (c % DT_TILE);
            out[k] = e;
        }
    BSMR_CHECK(D.off.upload(off.data(), off.size(), stream));
    BSMR_CHECK(D.loc.upload(loc.data(), loc.size(), stream));
    BSMR_CHECK(D.out.upload(out.data(), out.size(), stream));
    BSMR_HIP(hipStreamSynchronize(stream));
    D.ntn = ntn;
    D.ntiles = static_cast<u32>(ntiles);
    D.nonempty = 0;
    for (size_t t = 0; t < ntiles; ++t) D.nonempty += off[t + 1] > off[t];
    D.built = true;
    return BSMR_OK;
}

// fp16/bf16, K a multiple of 64: the whole product in 128 x 128 MFMA tiles, sampled
int launch_dense(const Plan& p, const void* dA, const void* dB, u32 K, int dtype, float* dP,
                 hipStream_t s, u32 nb) {
    {
        std::lock_guard<std::mutex> g(p.layout_mu);
        if (!p.dense.built) BSMR_CHECK(p.build_dense_layout());
    }
    const Plan::DenseLayout& D = p.dense;
    DenseArgs a{};
    a.A = static_cast<const char*>(dA);
    a.B = static_cast<const char*>(dB);
    a.P = dP;
    a.off = D.off.data();
    a.loc = D.loc.data();
    a.out = D.out.data();
    a.M = p.M;
    a.N = p.N;
    a.K = K;
    a.ntn = D.ntn;
    a.ntiles = D.ntiles;
    a.bA = static_cast<unsigned long long>(p.M) * K * 2;
    a.bB = static_cast<unsigned long long>(p.N) * K * 2;
    a.bP = p.nnz;
    const u32 per = (D.ntiles + XCD_BUCKETS - 1) / XCD_BUCKETS;
    const u32 grid = per * XCD_BUCKETS;
    const dim3 g(grid, nb);
    a.trace = nullptr;
    if (p.diag & 32) {
        BSMR_CHECK(p.prepare_trace(static_cast<size_t>(grid) * nb, s));
        a.trace = p.trace.data();
    }
    // (KC, NS) = (64, 2): two workgroups per CU. Measured (tools/gpu_dense_stages.sh history,
    // r01q): 4 stages at one workgroup per CU and KC = 32 at 2-4 stages / 2-4 workgroups were
    // all slower (C5 uniform 10.6-12.1 us vs 8.8-9.8)
    // eight waves (64 x 32 blocks, two per SIMD) when the tiles fill at most one workgroup per CU
    // (C5: 256 tiles)
    const bool ks2 = p.dense_ks == 2 || (p.dense_ks != 1 && D.nonempty < 512);
    if (ks2) {
        const bool f16 = dtype == BSMR_F16;
        switch (p.dense_ns) {
            case 3:
                if (f16) hipLaunchKernelGGL((k_sddmm_dense<1, 64, 3, 8>), g, dim3(512), 0, s, a);
                else hipLaunchKernelGGL((k_sddmm_dense<2, 64, 3, 8>), g, dim3(512), 0, s, a);
                break;
            case 4:
                if (f16) hipLaunchKernelGGL((k_sddmm_dense<1, 64, 4, 8>), g, dim3(512), 0, s, a);
                else hipLaunchKernelGGL((k_sddmm_dense<2, 64, 4, 8>), g, dim3(512), 0, s, a);
                break;
            case 5:
                if (f16) hipLaunchKernelGGL((k_sddmm_dense<1, 64, 5, 8>), g, dim3(512), 0, s, a);
                else hipLaunchKernelGGL((k_sddmm_dense<2, 64, 5, 8>), g, dim3(512), 0, s, a);
                break;
            default:
                if (f16) hipLaunchKernelGGL((k_sddmm_dense<1, 64, 2, 8>), g, dim3(512), 0, s, a);
                else hipLaunchKernelGGL((k_sddmm_dense<2, 64, 2, 8>), g, dim3(512), 0, s, a);
        }
    } else if (dtype == BSMR_F16) {
        hipLaunchKernelGGL((k_sddmm_dense<1, 64, 2, 4>), g, dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL((k_sddmm_dense<2, 64, 2, 4>), g, dim3(256), 0, s, a);
    }
    BSMR_HIP(hipGetLastError());
    return BSMR_OK;
}

}  // namespace bsmr
