// sddmm_dense.hip — dense-sampled SDDMM for fp16/bf16 operands on patterns dense enough that
// computing whole 128 x 128 output tiles on the matrix cores beats gathering entry by entry
// (DLMC-like 90 %-sparse masks, BASELINE.json C5: "MFMA-utilisation stress").
//
// Tile (tm, tn) = rows [128 tm, +128) x columns [128 tn, +128) of P = A B^T in the ORIGINAL index
// space (the reordering does not change which dot products exist). One 256-thread workgroup per
// non-empty tile: the K loop streams 64-wide k-chunks of the tile's 128 A rows and 128 B rows
// (128 bytes each) into LDS by LDS-DMA, double-buffered in two static images so a chunk's
// LDS-DMA is in flight while the previous chunk's MFMAs run; wave (wy, wx) owns a 64 x 64 quadrant as
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
constexpr u32 DT_KC = 64;      // k-chunk per barrier (two MFMA k-steps of 32)
constexpr u32 DT_CHUNK = DT_TILE * DT_KC * 2;  // bytes of one operand chunk image (16 KiB)
constexpr u32 DT_CS = DT_TILE + 4;             // fp32 output image row stride (floats)

struct DenseArgs {
    const char* A;  // M x K halves, row-major
    const char* B;  // N x K halves (B column-major)
    float* P;
    const u32* off;  // [tiles + 1] entry ranges per tile
    const u32* loc;  // local row << 7 | local column
    const u32* out;  // CSR position
    u32 M, N, K, ntn, ntiles;
    unsigned long long bA, bB, bP;  // batched launch: A/B byte strides, P element stride
};

__shared__ __attribute__((aligned(16))) char g_da0[DT_CHUNK];
__shared__ __attribute__((aligned(16))) char g_db0[DT_CHUNK];
__shared__ __attribute__((aligned(16))) char g_da1[DT_CHUNK];
__shared__ __attribute__((aligned(16))) char g_db1[DT_CHUNK];
__shared__ __attribute__((aligned(16))) float g_dc[DT_TILE * DT_CS];

// 16-byte slot of (row r, k-group g < 8) in a chunk image: rows of 128 bytes, the eight groups of
// a row permuted by (r >> 1) & 7, so the 16 lanes of each ds_read_b128 lane group (rows l & 15,
// group 4 s + (l >> 4)) hit 16 distinct 16-byte bank groups
__device__ __forceinline__ u32 dslot(u32 r, u32 g) { return 8 * r + (g ^ ((r >> 1) & 7)); }

// chunk kc of the tile's A and B rows into (sa, sb): 1024 slots each, 4 LDS-DMAs per wave and
// operand, no branches (rows past M / N read the last row; they are never sampled)
__device__ __forceinline__ void dense_stage(const DenseArgs& a, const u32 r0, const u32 c0,
                                            const u32 kc, const u32 ws, const u32 lane, char* sa,
                                            char* sb) {
    const size_t rowB = static_cast<size_t>(a.K) * 2;
#pragma unroll
    for (u32 i = 0; i < 4; ++i) {
        const u32 s = 64 * (4 * ws + i) + lane, r = s >> 3, g = (s & 7) ^ ((r >> 1) & 7);
        const u32 ra = min(r0 + r, a.M - 1), rb = min(c0 + r, a.N - 1);
        const size_t ko = static_cast<size_t>(kc) * (DT_KC * 2) + 16 * g;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(a.A + ra * rowB + ko),
            (__attribute__((address_space(3))) void*)(sa + 1024 * (4 * ws + i)), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(a.B + rb * rowB + ko),
            (__attribute__((address_space(3))) void*)(sb + 1024 * (4 * ws + i)), 16, 0, 0);
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

// one k-chunk of the wave's 64 x 64 quadrant from the images (sa, sb)
template <int DT>
__device__ __forceinline__ void dense_chunk(const char* sa, const char* sb, const u32 wy,
                                            const u32 wx, const u32 lane, f32x4 (&acc)[4][4]) {
    const u32 rr = lane & 15, g4 = lane >> 4;
#pragma unroll
    for (u32 ks = 0; ks < DT_KC / 32; ++ks) {
        f32x4 av[4], bv[4];
#pragma unroll
        for (u32 i = 0; i < 4; ++i) {
            const u32 ra = 64 * wy + 16 * i + rr, rb = 64 * wx + 16 * i + rr;
            av[i] = *reinterpret_cast<const f32x4*>(sa + 16 * dslot(ra, 4 * ks + g4));
            bv[i] = *reinterpret_cast<const f32x4*>(sb + 16 * dslot(rb, 4 * ks + g4));
        }
#pragma unroll
        for (u32 i = 0; i < 4; ++i)
#pragma unroll
            for (u32 jj = 0; jj < 4; ++jj) acc[i][jj] = mfma16x16x32<DT>(av[i], bv[jj], acc[i][jj]);
    }
}

template <int DT>
__global__ __launch_bounds__(256) void k_sddmm_dense(DenseArgs a) {
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
    const u32 ws = __builtin_amdgcn_readfirstlane(w), wy = ws >> 1, wx = ws & 1;
    f32x4 acc[4][4];
#pragma unroll
    for (u32 i = 0; i < 4; ++i)
#pragma unroll
        for (u32 jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    const u32 nk = a.K / DT_KC;  // even (launch_dense: K a multiple of 128)
    dense_stage(a, r0, c0, 0, ws, lane, g_da0, g_db0);
    __syncthreads();
    for (u32 kc = 0; kc < nk; kc += 2) {
        // chunk kc + 1 lands in image 1 while chunk kc computes from image 0, and so on; the
        // last prefetch re-reads chunk nk - 1 (no branch around an LDS-DMA)
        dense_stage(a, r0, c0, kc + 1, ws, lane, g_da1, g_db1);
        dense_chunk<DT>(g_da0, g_db0, wy, wx, lane, acc);
        __syncthreads();
        dense_stage(a, r0, c0, min(kc + 2, nk - 1), ws, lane, g_da0, g_db0);
        dense_chunk<DT>(g_da1, g_db1, wy, wx, lane, acc);
        __syncthreads();
    }
    // accumulator (i, jj) reg r of lane l = D[64 wy + 16 i + 4 (l >> 4) + r][64 wx + 16 jj + (l & 15)]
#pragma unroll
    for (u32 i = 0; i < 4; ++i)
#pragma unroll
        for (u32 jj = 0; jj < 4; ++jj)
#pragma unroll
            for (u32 r = 0; r < 4; ++r)
                g_dc[(64 * wy + 16 * i + 4 * (lane >> 4) + r) * DT_CS + 64 * wx + 16 * jj + (lane & 15)] =
                    acc[i][jj][r];
    __syncthreads();
    for (u32 e = e0 + tid; e < e1; e += 256) {
        const u32 lc = a.loc[e];
        a.P[a.out[e]] = g_dc[(lc >> 7) * DT_CS + (lc & 127)];
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
    D.built = true;
    return BSMR_OK;
}

// fp16/bf16, K a multiple of 128: the whole product in 128 x 128 MFMA tiles, sampled
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
    if (dtype == BSMR_F16)
        hipLaunchKernelGGL(k_sddmm_dense<1>, dim3(grid, nb), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_sddmm_dense<2>, dim3(grid, nb), dim3(256), 0, s, a);
    BSMR_HIP(hipGetLastError());
    return BSMR_OK;
}

}  // namespace bsmr
