// sddmm_half.hip — SDDMM with fp16 / bf16 A and B, fp32 accumulation and fp32 P (configs C3
// cop20k_A fp16 K=256 and C5 DLMC bf16 K=512 of BASELINE.json; the reference builds TF32 only).
//
// Same plan, same launch structure as the fp32 column-major path (sddmm.hip):
//   * dense tile: `v_mfma_f32_16x16x32_{f16,bf16}`; lane l holds A[row l&15][32kk + 8(l>>4) + j]
//     and B[k = 32kk + 8(l>>4) + j][col l&15], j = 0..7 (one 16-byte load each); K/32 MFMAs.
//   * residual slot: one 16-lane row per entry, lane s holds W consecutive halves s, s+16, ... of
//     A[row] and B[col]; products of two halves are exact in fp32 and summed in fp32; DPP row sum.
#include <algorithm>

#include "common.hpp"
#include "plan.hpp"

namespace bsmr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));

struct HalfArgs {
    const uint16_t* A;
    const uint16_t* B;
    float* P;
    u32 nd, nslots;
    const u32* tileRows;
    const u32* denseCols;
    const u32* blockValues;
    const uint2* slots;
    const u32* cmRow;
    const u32* cmCol;
    const u32* cmOut;
    u32 N, K;
    unsigned long long bA, bB, bP;  // batched launch (grid.y = batch), element strides
};

template <bool BF16>
__device__ __forceinline__ float h2f(uint16_t h) {
    if constexpr (BF16) {
        return __builtin_bit_cast(float, static_cast<u32>(h) << 16);
    } else {
        return static_cast<float>(__builtin_bit_cast(_Float16, h));
    }
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                                 CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float v) {
    v += dppf<0xB1>(v);
    v += dppf<0x4E>(v);
    v += dppf<0x141>(v);
    v += dppf<0x140>(v);
    return v;
}

template <bool BF16>
__device__ __forceinline__ f32x4 mfma32(s16x8 a, s16x8 b, f32x4 c) {
    if constexpr (BF16)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b16x8, a),
                                                       __builtin_bit_cast(b16x8, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h16x8, a),
                                                      __builtin_bit_cast(h16x8, b), c, 0, 0, 0);
}

// one dense tile; K multiple of 32
template <bool BF16>
__device__ __forceinline__ void dense_tile_h(const HalfArgs& a, const u32 tile) {
    const u32 l = __lane_id(), rr = l & 15, g = l >> 4;
    const u32 row = a.tileRows[tile * 16 + rr];
    const u32 c = a.denseCols[tile * 16 + rr];
    const u32* bvals = a.blockValues + static_cast<size_t>(tile) * 256 + 64 * g + rr;
    u32 idx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) idx[r] = bvals[16 * r];
    const bool rvalid = row != NULLV;
    const bool cvalid = c < a.N;
    const uint16_t* arow = a.A + static_cast<size_t>(rvalid ? row : 0) * a.K + 8 * g;
    const uint16_t* bcol = a.B + static_cast<size_t>(cvalid ? c : 0) * a.K + 8 * g;
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    const s16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
    u32 k = 0;
    for (; k + 64 <= a.K; k += 64) {
        const s16x8 a0 = rvalid ? *reinterpret_cast<const s16x8*>(arow + k) : zero;
        const s16x8 b0 = cvalid ? *reinterpret_cast<const s16x8*>(bcol + k) : zero;
        const s16x8 a1 = rvalid ? *reinterpret_cast<const s16x8*>(arow + k + 32) : zero;
        const s16x8 b1 = cvalid ? *reinterpret_cast<const s16x8*>(bcol + k + 32) : zero;
        acc0 = mfma32<BF16>(a0, b0, acc0);
        acc1 = mfma32<BF16>(a1, b1, acc1);
    }
    if (k < a.K) {
        const s16x8 a0 = rvalid ? *reinterpret_cast<const s16x8*>(arow + k) : zero;
        const s16x8 b0 = cvalid ? *reinterpret_cast<const s16x8*>(bcol + k) : zero;
        acc0 = mfma32<BF16>(a0, b0, acc0);
    }
    const f32x4 acc = acc0 + acc1;
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (idx[r] != NULLV) a.P[idx[r]] = acc[r];
}

// residual slot: each 16-lane row takes a contiguous share; lane s reads 2 halves (4 bytes) at
// k = 2s + 32j, j = 0 .. K/32-1, for A and B; up to U entries in flight per row
template <bool BF16>
__device__ __forceinline__ void residual_h(const HalfArgs& a, const uint2 sl) {
    constexpr int U = 4;
    const u32 l = __lane_id(), sub = l & 15, grp = l >> 4;
    const u32 n = sl.y - sl.x;
    const u32 share = (n + 3) / 4;
    const u32 gs = sl.x + min(grp * share, n), ge = sl.x + min(grp * share + share, n);
    const u32 K = a.K;
    for (u32 base = gs; base < ge; base += U) {
        float acc[U];
        u32 out[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32 e = base + u;
            ok[u] = e < ge;
            const u32 ee = ok[u] ? e : gs;
            out[u] = a.cmOut[ee];
            const uint16_t* ap = a.A + static_cast<size_t>(a.cmRow[ee]) * K + 2 * sub;
            const uint16_t* bp = a.B + static_cast<size_t>(a.cmCol[ee]) * K + 2 * sub;
            float s = 0.f;
            for (u32 k = 0; k < K; k += 32) {
                const u32 av = *reinterpret_cast<const u32*>(ap + k);
                const u32 bv = *reinterpret_cast<const u32*>(bp + k);
                s += h2f<BF16>(static_cast<uint16_t>(av)) * h2f<BF16>(static_cast<uint16_t>(bv));
                s += h2f<BF16>(static_cast<uint16_t>(av >> 16)) *
                     h2f<BF16>(static_cast<uint16_t>(bv >> 16));
            }
            acc[u] = s;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float t = row_sum16(acc[u]);
            if (sub == 0 && ok[u]) a.P[out[u]] = t;
        }
    }
}

template <bool BF16>
__global__ __launch_bounds__(64) void k_sddmm_half(HalfArgs a) {
    if (blockIdx.y) {
        a.A += blockIdx.y * a.bA;
        a.B += blockIdx.y * a.bB;
        a.P += blockIdx.y * a.bP;
    }
    const u32 b = blockIdx.x;
    if (b < a.nd) {
        dense_tile_h<BF16>(a, b);
        return;
    }
    const u32 ndpad = (a.nd + 7) & ~7u;
    if (b < ndpad) return;
    const u32 s = b - ndpad;
    if (s < a.nslots) {
        const uint2 sl = a.slots[s];
        if (sl.x < sl.y) residual_h<BF16>(a, sl);
    }
}

// ---------------------------------------------------------------------------------------------
// Panel-grouped tile launch (tile-dominated fp16 / bf16 plans, e.g. the 16 x 16 block masks of
// BASELINE.json C5): the reference's design — every BSMR dense tile on the tensor cores
// (sddmmKernel.cu:213-351, launched per row panel at 2570-2581) — with the panel's A rows staged
// ONCE per workgroup instead of once per tile.
//
// Item i = {panel q, first tile t0, tiles nt} (<= PtileLayout::tpi tiles of one panel), read from
// its descriptor (the panel's 16 rows and the tiles' columns inline, so A and B addresses are one
// load away from the workgroup id). One 256-thread workgroup per item: the panel's 16 A rows (16 x 2K bytes) go to LDS through
// registers, chunk c of row r at 16-byte slot 4NK r + (c ^ swz(r)) so the 16 rows of a
// ds_read_b128 lane group hit 16 distinct bank groups; wave w takes tiles t0 + w, t0 + w + 4, ...
// Lane (rr, g) = (l & 15, l >> 4) holds B[col rr][32 s + 8 g, +8) of every k-step s in registers
// (NK = K / 32 16-byte loads straight from L2, the next tile's in flight while this one runs its
// NK `v_mfma_f32_16x16x32_{f16,bf16}`), reads A[row rr][32 s + 8 g, +8) from LDS and scatters
// D[4 g + r][rr] to P[blockValues[256 t + 16 (4 g + r) + rr]] (NULLV = no stored entry: rows past
// the last reordered row, sentinel columns, empty slots). Ingest per tile: 16 B rows; per item:
// 16 A rows — against 16 + 16 rows per tile when each tile loads its own A (k_sddmm_half) and
// 128 + 128 rows per 128 x 128 tile of the dense-sampled launch.
// Workgroups past the items run 4 residual slots each (residual_h, one per wave; the column-major
// slots' XCD deal holds because the item count is a multiple of 8).
struct PtileArgs {
    HalfArgs h;
    const u32* desc;     // per item slot in launch order (PtileLayout::desc); tiles = 0: padding
    u32 dstride;
    u32 nItems;          // item slots (a multiple of 8)
    // BSMR_DIAG & 32: per workgroup {start, A staged (after the barrier), end, xcc << 60 | wave 0's
    // first tile's MFMAs done} (s_memrealtime, 100 MHz); else null
    unsigned long long* trace;
};

template <u32 NK>
__device__ __forceinline__ u32 ptile_slot(u32 r, u32 c) {
    // 4 NK 16-byte chunks per row; rows of >= 16 chunks XOR the low 4 bits with the row
    return 4 * NK * r + (c ^ (NK >= 4 ? (r & 15) : (r & 7)));
}

template <bool BF16, u32 NK, u32 NW>
__global__ __launch_bounds__(64 * NW) void k_sddmm_ptile(PtileArgs a) {
    static_assert(NK == 2 || NK == 4 || NK == 8 || NK == 16, "K / 32 in {2, 4, 8, 16}");
    constexpr u32 NT = 64 * NW;
    // the A image: up to two panels (32 rows) of the item
    __shared__ __attribute__((aligned(16))) s16x8 sa[32 * 4 * NK];
    if (blockIdx.y) {
        a.h.A += blockIdx.y * a.h.bA;
        a.h.B += blockIdx.y * a.h.bB;
        a.h.P += blockIdx.y * a.h.bP;
    }
    const u32 b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const u32 w = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (b >= a.nItems) {  // residual slots: 4 per workgroup (the column-major slots' XCD deal)
        const u32 s = (b - a.nItems) * 4 + w;
        if (w < 4 && s < a.h.nslots) {
            const uint2 sl = a.h.slots[s];
            if (sl.x < sl.y) residual_h<BF16>(a.h, sl);
        }
        return;
    }
    const unsigned long long t_start = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // the item's descriptor (PtileLayout): rows d[0..32) (panel 0's 16, then panel 1's), {first
    // tile, tiles, tiles of panel 0, panels} at d[32..36), columns d[48 + 16 j + c]
    const u32* const d = a.desc + static_cast<size_t>(b) * a.dstride;
    const u32 rr = lane & 15, g = lane >> 4;
    constexpr u32 CPR = 4 * NK, NCH = 32 * CPR, PER = (NCH + NT - 1) / NT;
    // round trip 1, every descriptor load at once: the rows of this thread's A chunks, the
    // columns of the wave's first tile, the tile range (a padding slot's descriptor is zeros)
    u32 arow[PER];
#pragma unroll
    for (u32 i = 0; i < PER; ++i) {
        const u32 f = tid + NT * i;
        arow[i] = (NCH % NT == 0 || f < NCH) ? d[f / CPR] : 0u;
    }
    const u32 cfirst = d[48 + 16 * w + rr];
    const uint4 hd = *reinterpret_cast<const uint4*>(d + 32);
    const u32 t0 = __builtin_amdgcn_readfirstlane(hd.x), nt = __builtin_amdgcn_readfirstlane(hd.y);
    const u32 n0 = __builtin_amdgcn_readfirstlane(hd.z), np = __builtin_amdgcn_readfirstlane(hd.w);
    // (no early return for a padding slot, nt = 0: a branch here would hold every other load of
    // the prologue behind the tile count's round trip; it loads row 0 and tile t0 = 0 and stores
    // nothing)
    const u32 K = 32 * NK;
    const size_t rowB = static_cast<size_t>(K) * 2;
    const char* const Ab = reinterpret_cast<const char*>(a.h.A);
    const char* const Bb = reinterpret_cast<const char*>(a.h.B);
    // the wave's tile j: B fragments (one 16-byte load per k-step) and its four output positions
    s16x8 bf[NK];
    u32 idx[4];
    auto load_tile = [&](const u32 j, const u32 c) {
        // (a wave past the item's tiles, or of a padding slot, loads a real tile and stores nothing)
        const u32 tile = t0 + min(j, max(nt, 1u) - 1);
        const char* bp = Bb + static_cast<size_t>(c < a.h.N ? c : 0) * rowB + 16 * g;
#pragma unroll
        for (u32 s = 0; s < NK; ++s) bf[s] = *reinterpret_cast<const s16x8*>(bp + 64 * s);
        const u32* bv = a.h.blockValues + static_cast<size_t>(tile) * 256 + 64 * g + rr;
#pragma unroll
        for (u32 r = 0; r < 4; ++r) idx[r] = bv[16 * r];
    };
    // round trip 2: the item's A rows (chunks of the second panel only when it has one; thread tid
    // takes chunks tid, tid + NT, ...), then the first tile's B fragments and output positions;
    // the A data's wait leaves the B loads in flight across the barrier
    const u32 lim = (np > 1 ? 32u : 16u) * CPR;
    s16x8 av[PER];
#pragma unroll
    for (u32 i = 0; i < PER; ++i) {
        const u32 f = tid + NT * i;
        if (f < lim)
            av[i] = *reinterpret_cast<const s16x8*>(Ab + static_cast<size_t>(arow[i]) * rowB + 16 * (f % CPR));
    }
    load_tile(w, cfirst);
#pragma unroll
    for (u32 i = 0; i < PER; ++i) {
        const u32 f = tid + NT * i;
        if (f < lim) sa[ptile_slot<NK>(f / CPR, f % CPR)] = av[i];
    }
    __syncthreads();
    const unsigned long long t_mid = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    unsigned long long t_mfma = 0;
    // one tile per wave at a time (NK 16-byte B loads in flight per lane): NK MFMAs with A
    // fragments from its panel's rows in LDS, then the scatter
    for (u32 j = w; j < nt; j += NW) {
        if (j != w) load_tile(j, d[48 + 16 * j + rr]);
        const u32 ra = (j < n0 ? 0u : 16u) + rr;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (u32 s = 0; s < NK; ++s) acc = mfma32<BF16>(sa[ptile_slot<NK>(ra, 4 * s + g)], bf[s], acc);
        if (a.trace && j == w)  // (reads the result: after the last MFMA)
            t_mfma = __builtin_amdgcn_s_memrealtime() + (acc[0] != acc[0] ? 1ull : 0ull);
#pragma unroll
        for (u32 r = 0; r < 4; ++r)
            if (idx[r] != NULLV) a.h.P[idx[r]] = acc[r];
    }
    if (a.trace && tid == 0) {
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        const u32 xcc = __builtin_amdgcn_s_getreg(0xF814);  // HW_REG_XCC_ID
        unsigned long long* tr = a.trace + 4ull * (blockIdx.y * gridDim.x + blockIdx.x);
        tr[0] = t_start;
        tr[1] = t_mid;
        tr[2] = t_end;
        tr[3] = (static_cast<unsigned long long>(xcc) << 60) | (t_mfma & ((1ull << 60) - 1));
    }
}

}  // namespace

// Items of the panel-grouped tile launch (built on first use). By default (tpi = 0) the tiles,
// in plan order, are cut into as many equal runs as the chip has CUs (runs of at most 8 tiles
// when there are more), a run crossing a panel boundary taking both panels' A rows (a run that
// would need a third panel is split): every CU then stages about the same bytes — 16 B rows per
// tile plus 16 A rows per panel — in one round. With tpi > 0 (BSMR_PTILE_TPI) every panel's tiles
// are cut into ceil(n / tpi) near-equal items of one panel. The list is dealt as contiguous
// eighths per XCD (slot b on XCD b % 8 takes list position (b % 8) per + b / 8).
int Plan::build_ptile_layout(u32 tpi) const {
    PtileLayout& L = ptile;
    struct It {
        u32 q0, q1, t0, nt, n0;  // panels q0 (and q1 when n0 < nt), tiles [t0, t0 + nt)
    };
    std::vector<It> list;
    const u32 T = h_blockOffsets[P];
    const auto panel_of = [&](u32 t) {  // the panel holding tile t (empty panels skipped)
        return static_cast<u32>(std::upper_bound(h_blockOffsets.begin(), h_blockOffsets.begin() + P + 1, t) -
                                h_blockOffsets.begin()) - 1;
    };
    u32 maxTiles = 0;
    if (tpi > 0) {
        for (u32 q = 0; q < P; ++q) {
            const u32 a = h_blockOffsets[q], n = h_blockOffsets[q + 1] - a, k = (n + tpi - 1) / tpi;
            for (u32 i = 0; i < k; ++i) {
                const u32 t0 = a + static_cast<u32>(static_cast<u64>(n) * i / k);
                const u32 t1 = a + static_cast<u32>(static_cast<u64>(n) * (i + 1) / k);
                list.push_back({q, q, t0, t1 - t0, t1 - t0});
            }
        }
    } else if (T > 0) {
        int cus = 256;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
            cus = 256;
        const u32 nb = std::max<u32>(static_cast<u32>(cus), (T + 7) / 8);
        for (u32 k = 0; k < nb; ++k) {
            const u32 a = static_cast<u32>(static_cast<u64>(T) * k / nb);
            const u32 e = static_cast<u32>(static_cast<u64>(T) * (k + 1) / nb);
            for (u32 t = a; t < e;) {
                const u32 q0 = panel_of(t), e0 = std::min(h_blockOffsets[q0 + 1], e);
                if (e0 == e) {
                    list.push_back({q0, q0, t, e - t, e - t});
                    t = e;
                } else {
                    const u32 q1 = panel_of(e0), e1 = std::min(h_blockOffsets[q1 + 1], e);
                    list.push_back({q0, q1, t, e1 - t, e0 - t});
                    t = e1;
                }
            }
        }
    }
    for (const It& it : list) maxTiles = std::max(maxTiles, it.nt);
    const u32 n = static_cast<u32>(list.size());
    const u32 per = (n + XCD_BUCKETS - 1) / XCD_BUCKETS;
    const u32 nslots = per * XCD_BUCKETS;
    // the descriptors (PtileArgs::desc): per item slot its rows, header and tile columns
    std::vector<u32> hrows, hcols;
    BSMR_CHECK(rows.download(hrows, stream));
    BSMR_CHECK(denseCols.download(hcols, stream));
    const u32 waves = PtileLayout::desc_waves(tpi);
    const u32 ds = PtileLayout::desc_stride(std::max(maxTiles, waves));
    std::vector<u32> desc(static_cast<size_t>(nslots) * ds, 0);
    std::vector<uint4> items(std::max<u32>(nslots, 1), make_uint4(0, 0, 0, 0));
    for (u32 b = 0; b < nslots; ++b) {
        const u32 pos = (b % XCD_BUCKETS) * per + b / XCD_BUCKETS;
        if (pos >= n) continue;
        const It& it = list[pos];
        items[b] = make_uint4(it.q0, it.t0, it.nt, it.n0 < it.nt ? it.q1 + 1 : 0u);
        u32* d = desc.data() + static_cast<size_t>(b) * ds;
        for (u32 r = 0; r < 32; ++r) {
            const u32 x = 16 * (r < 16 || it.n0 == it.nt ? it.q0 : it.q1) + (r & 15);
            d[r] = x < R ? hrows[x] : hrows[0];
        }
        d[32] = it.t0;
        d[33] = it.nt;
        d[34] = it.n0;
        d[35] = it.n0 < it.nt ? 2u : 1u;
        for (u32 j = 0; j < it.nt; ++j)
            for (u32 c = 0; c < 16; ++c) d[48 + 16 * j + c] = hcols[(it.t0 + j) * 16 + c];
    }
    BSMR_CHECK(L.items.upload(items.data(), items.size(), stream));
    BSMR_CHECK(L.desc.upload(desc.data(), std::max<size_t>(desc.size(), 1), stream));
    BSMR_HIP(hipStreamSynchronize(stream));  // host vectors are pageable memory
    L.nItems = nslots;
    L.nListed = n;
    L.tpi = tpi;
    L.waves = waves;
    L.stride = ds;
    L.built = true;
    return BSMR_OK;
}

// tile-dominated fp16/bf16 plans, K in {64, 128, 256, 512}: the panel-grouped tile launch (mode: 1
// tiles, 2 residual slots, 3 both)
int launch_ptile(const Plan& p, const void* dA, const void* dB, u32 K, int dtype, float* dP,
                 u32 mode, hipStream_t s, u32 nb) {
    const u32 NK = K / 32;
    if (K % 32 != 0 || (NK != 2 && NK != 4 && NK != 8 && NK != 16)) {
        set_error("bsmr_sddmm: the panel-tile launch needs K in {64, 128, 256, 512}");
        return BSMR_ERR_UNSUPPORTED;
    }
    {
        std::lock_guard<std::mutex> g(p.layout_mu);
        if (!p.ptile.built || p.ptile.tpi != p.ptile_tpi) BSMR_CHECK(p.build_ptile_layout(p.ptile_tpi));
    }
    PtileArgs a{};
    a.h.A = static_cast<const uint16_t*>(dA);
    a.h.B = static_cast<const uint16_t*>(dB);
    a.h.P = dP;
    a.h.nslots = (mode & 2) ? p.nSlots : 0;
    a.h.denseCols = p.denseCols.data();
    a.h.blockValues = p.blockValues.data();
    a.h.slots = p.cmSlots.data();
    a.h.cmRow = p.cmRow.data();
    a.h.cmCol = p.cmCol.data();
    a.h.cmOut = p.cmOut.data();
    a.h.N = p.N;
    a.h.K = K;
    a.h.bA = static_cast<unsigned long long>(p.M) * K;
    a.h.bB = static_cast<unsigned long long>(p.N) * K;
    a.h.bP = p.nnz;
    a.desc = p.ptile.desc.data();
    a.dstride = p.ptile.stride;
    a.nItems = (mode & 1) ? p.ptile.nItems : 0;
    a.trace = nullptr;
    u32 grid = a.nItems + (a.h.nslots + 3) / 4;
    if (grid == 0) {
        if (mode == 3) return BSMR_OK;
        grid = 1;  // a profiling split with nothing to run (no residual) still dispatches once
    }
    if (p.diag & 32) {
        BSMR_CHECK(p.prepare_trace(static_cast<size_t>(grid) * nb, s));
        a.trace = p.trace.data();
    }
    const bool bf = dtype == BSMR_BF16;
    const dim3 gd(grid, nb);
    // waves per workgroup: one per tile of an item up to 8 (items of more tiles loop)
    const bool w8 = p.ptile.waves == 8;
#define BSMR_PT(NKV) (w8 ? (bf ? k_sddmm_ptile<true, NKV, 8> : k_sddmm_ptile<false, NKV, 8>) \
                         : (bf ? k_sddmm_ptile<true, NKV, 4> : k_sddmm_ptile<false, NKV, 4>))
    void (*fn)(PtileArgs) = NK == 2 ? BSMR_PT(2) : NK == 4 ? BSMR_PT(4) : NK == 8 ? BSMR_PT(8) : BSMR_PT(16);
#undef BSMR_PT
    hipLaunchKernelGGL(fn, gd, dim3(w8 ? 512 : 256), 0, s, a);
    BSMR_HIP(hipGetLastError());
    return BSMR_OK;
}

// dtype: BSMR_F16 or BSMR_BF16; K a positive multiple of 32. mode: 1 dense, 2 residual, 3 both
int launch_half(const Plan& p, const void* dA, const void* dB, u32 K, int dtype, float* dP,
                u32 mode, hipStream_t s, u32 nb) {
    if (K == 0 || K % 32 != 0) {
        set_error("bsmr_sddmm: fp16/bf16 inputs need K to be a positive multiple of 32");
        return BSMR_ERR_UNSUPPORTED;
    }
    HalfArgs a{};
    a.A = static_cast<const uint16_t*>(dA);
    a.B = static_cast<const uint16_t*>(dB);
    a.P = dP;
    a.nd = (mode & 1) ? p.nDenseItems : 0;
    a.nslots = (mode & 2) ? p.nSlots : 0;
    a.tileRows = p.tileRows.data();
    a.denseCols = p.denseCols.data();
    a.blockValues = p.blockValues.data();
    a.slots = p.cmSlots.data();
    a.cmRow = p.cmRow.data();
    a.cmCol = p.cmCol.data();
    a.cmOut = p.cmOut.data();
    a.N = p.N;
    a.K = K;
    a.bA = static_cast<unsigned long long>(p.M) * K;
    a.bB = static_cast<unsigned long long>(p.N) * K;
    a.bP = p.nnz;
    const u32 grid = a.nslots ? ((a.nd + 7) & ~7u) + a.nslots : a.nd;
    if (grid == 0) return BSMR_OK;
    if (dtype == BSMR_BF16)
        hipLaunchKernelGGL(k_sddmm_half<true>, dim3(grid, nb), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL(k_sddmm_half<false>, dim3(grid, nb), dim3(64), 0, s, a);
    BSMR_HIP(hipGetLastError());
    return BSMR_OK;
}

}  // namespace bsmr
