// knn_fused16.hip -- the fused-norm filter on v_mfma_f32_16x16x32_bf16 (round 6; gfx950).
// DESIGN.md "k_gemm_fused16".
//
// The same filter as k_gemm_fused (knn_fused.hip: operands, certificate, fast test, lane-parallel
// slow path, schedule) with the 16x16 output tile of the K = 32 bf16 MFMA instead of the 32x32
// tile of the K = 16 one, for the register-list shapes (k <= 32, d = 64 / 128):
//   * same train tile blocks (k_tn_rows: bn rows rn(t) | bn norms | tile statistics), same
//     blocks of 8 waves and the same queries per block, so the host plan, the LDS image, the
//     DMA pieces and the schedule are those of the 32x32 shape with the same tile and block;
//   * QG 16-query groups per wave x RG 16-row groups per tile: the 32-query shape (QG = 2,
//     RG = 4, 64-row tiles) and the 64-query shape (QG = 4, RG = 2, 32-row tiles);
//   * lane (j, g4) = (lane & 15, lane >> 4) holds query j of each query group and rows
//     16 rg + 4 g4 + r (r < 4) of each row group (the MFMA's C/D map: col = lane & 15,
//     row = 4 (lane >> 4) + reg); its A fragment (train) is row 16 rg + j, bytes 64 s + 16 g4,
//     its B fragment (query) the same bytes of query row j -- one ds_read_b128 each;
//   * each accumulator starts from its 4 rows' norms: ONE broadcast ds_read_b128 per 16-row
//     group (the 32x32 tile needs four per 32-row group: half the norm reads per MFMA cycle);
//   * a query's values sit in four lanes (quarters) instead of two (halves): each quarter keeps
//     the ceil(k/4) smallest U of its own rows (lists of 4 for k <= 16, 8 for k <= 32) and the
//     bound is the largest of the four quarters' ceil(k/4)-th smallest (>= 4 ceil(k/4) >= k kept
//     rows have U <= it); candidates go to sub-slice 4 seg + g4 of the query's list.
// Why: MI355X holds a higher clock on the 16x16x32 shape in MFMA loops (MI355X_MICROARCH.md,
// DVFS give-back (7): 1.12-1.15x the FLOP/s of 32x32x16 on random data) and the filter runs
// clock-limited (A: 1.71-1.82 GHz at 62-66 % MFMA busy); against it, the 16x16x32 MFMA holds
// the SIMD's vector issue for 8 of its 16 cycles (32x32x16: 8 of 32), so the fast test and the
// slow path have half the issue room per FLOP.  Selected by the plan only when forced
// (KNN_FUSED_MFMA16=1, a study switch read at knn_create) until the same-box comparison says
// otherwise.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "knn_device.h"
#include "knn_kernels.h"
#include "knn_study.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

#ifndef KNN_FUSED16_LIST_FIRST
#define KNN_FUSED16_LIST_FIRST 31  // first list exchange after this tile (then doubling), as k_gemm_fused
#endif
constexpr int F16_SHARE_EVERY = 64;  // tiles between threshold exchanges of a query's pieces (gthr)

// the word of lane ^ 16 (v_permlane16_swap: one of the swap's two results is the partner row's word)
__device__ __forceinline__ uint32_t lane_xor16(uint32_t v) {
    const auto sw = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane_id() & 16) ? sw[0] : sw[1];
}
__device__ __forceinline__ uint32_t lane_xor32(uint32_t v) {
    const auto sw = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane_id() & 32) ? sw[0] : sw[1];
}
// the largest of a word over the four quarters of a query (lanes j, j + 16, j + 32, j + 48)
__device__ __forceinline__ float quarter_max(float x) {
    const float inf = __uint_as_float(0x7f800000u);
    const float m = __builtin_amdgcn_fmed3f(x, __uint_as_float(lane_xor16(__float_as_uint(x))), inf);
    return __builtin_amdgcn_fmed3f(m, __uint_as_float(lane_xor32(__float_as_uint(m))), inf);
}

// slow-path scans of one query group's NV values (v = 4 rg + r, value of row 16 rg + 4 g4 + r)
// in one asm block each (no hazard padding between the values):
//   mask: bit v of m = (y_v <= tf), built from v = NV-1 down to 0 by v_addc (m = 2m + VCC);
//   eq:   bit v of e = (y_v == yv);
//   sel:  yv = y_idx.
#define F16_LE(n) "v_cmp_le_f32_e32 vcc, %" #n ", %1\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
#define F16_SEL(i, n) "v_cmp_eq_u32_e32 vcc, " #i ", %1\n\tv_cndmask_b32_e32 %0, %0, %" #n ", vcc\n\t"
#define F16_Y(v) "v"(Y[g * RG + ((v) >> 2)][(v)&3])

}  // namespace

template <int RB, int NBUF, int NW, int QG, int RG, int KR>
__device__ __forceinline__ void fused16_piece(const GemmFilterArgs& a, const int qt, const int seg,
                                              const int64_t row_begin, const int64_t row_end) {
    static_assert((QG == 2 && RG == 4) || (QG == 4 && RG == 2), "shapes: 32 queries x 64 rows, 64 x 32");
    static_assert(KR == 8 || KR == 32, "register lists (k <= 16, k <= 32)");
    static_assert(RB % 64 == 0, "tile blocks with a norm header (RB = 2d, d = 64 / 128)");
    static_assert(NBUF == 8 || NBUF == 16, "quads or octets");
    constexpr int BN = 16 * RG;     // train rows per tile
    constexpr int HS = BN / 4 + 1;  // header slots: BN fp32 norms + the statistics
    // the LDS image and DMA geometry of the 32x32 shape with the same tile and block
    typedef FilterTile<RB, NW, QG / 2, RG / 2, HS> FT;
    static_assert(FT::BN == BN && FT::BM == 16 * QG * NW, "geometry");
    constexpr int BM = FT::BM, STRIDE = FT::STRIDE, SLOTS = FT::SLOTS;
    constexpr int DMA_INS = FT::DMA_INS, TILE = FT::TILE, HDR = FT::HDR;
    constexpr int64_t TB = (int64_t)BN * RB + 16 * HS;  // operand bytes per tile block
    constexpr int DMA_PER_WAVE = (DMA_INS + NW - 1) / NW;
    constexpr int NS = RB / 64;        // k-steps of K = 32
    constexpr int NACC = QG * RG;      // 16x16 accumulators per wave per tile (c = g RG + rg)
    constexpr int NV = 4 * RG;         // values per query group per lane
    constexpr int VPK = (NV + NS - 1) / NS;  // fast-test values folded per k-step per group
    constexpr int GRP = NBUF / 2;      // tiles per barrier
    constexpr int AHEAD = GRP;         // tiles between a step and the tile it DMAs
    constexpr int PFK = 1;                // k-steps of A fragments read ahead (a k-step is 8 MFMAs)
    constexpr int LL = KR == 8 ? 4 : 8;   // list entries per quarter
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* tiles = smem;  // [NBUF][TILE]
    const int cap_sub = a.cap_seg / 4;  // candidate sub-slice of one quarter of a query

    const int lane = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = lane & 15;
    const int g4 = lane >> 4;
    const int k = a.k;
    const float INF = __uint_as_float(0x7f800000u);
    const float coef = a.coef, eta = a.eta;
    const unsigned char* trainb = reinterpret_cast<const unsigned char*>(a.train);

    // this lane's queries, one per query group (the four quarters hold the same queries):
    // query group g's is q0 + 16 g
    const int64_t q0 = (int64_t)qt * BM + wave * QG * 16 + j;
    auto q = [&](int g) __attribute__((always_inline)) -> int64_t { return q0 + 16 * g; };
    // (per-group state kept small: the 64-query shape at d = 128 holds 64 operand and 64
    // accumulator registers; validity is recomputed, a piece publishes its bound without a
    // "published" copy -- compared with the shared word it reads anyway)
    auto qvalid_of = [&](int g) __attribute__((always_inline)) { return q(g) < a.nq; };
    uint4 qf[QG][NS];
    float qn[QG], thr[QG], tfb[QG], qe2[QG], eq2[QG];
    int ccnt[QG];
#pragma unroll
    for (int g = 0; g < QG; g++) {
        const bool qvalid = qvalid_of(g);
        const unsigned char* qrow = reinterpret_cast<const unsigned char*>(a.test) +
                                    (qvalid ? q(g) : 0) * (int64_t)a.ld_q * 2;
#pragma unroll
        for (int s = 0; s < NS; s++)
            qf[g][s] = qvalid ? *reinterpret_cast<const uint4*>(qrow + 64 * s + 16 * g4) : make_uint4(0u, 0u, 0u, 0u);
        qn[g] = qvalid ? a.qnorm[q(g)] : 0.0f;
        thr[g] = qvalid ? o2f(a.gthr[q(g)]) : -INF;
        ccnt[g] = 0;
        qe2[g] = eq2[g] = 0.0f;
        if (qvalid) {
            const float2 qs = a.qstat[q(g)];
            qe2[g] = 2.0f * qs.x * (1.0f + 0x1p-17f);
            eq2[g] = 2.0f * qs.y * (1.0f + 0x1p-17f);
        }
    }
    // tf without the tile term (k_gemm_fused's fast test, unchanged)
    auto make_tfb = [&](int g) __attribute__((always_inline)) {
        tfb[g] = qvalid_of(g) ? ((thr[g] - qn[g]) + fmaf(coef, qn[g], eta)) + 0x1p-18f * (fabsf(thr[g]) + qn[g]) : -INF;
    };
#pragma unroll
    for (int g = 0; g < QG; g++) make_tfb(g);
    // tile terms: the tile's maximum norm (shared by the query groups) and each group's
    // operand-rounding bound against the tile
    // (the tile's statistics: max norm, max |t - rt|, max |rt|; each group's rounding bound
    // rho = 2 (|q| max|t - rt| + |q - rq| max|rt|) (1 + 2^-17) is formed where it is used)
    struct TQ { float tmax, ty, tz; };
    auto rho_of = [&](int g, const TQ& tq) __attribute__((always_inline)) { return fmaf(qe2[g], tq.ty, eq2[g] * tq.tz); };
    auto tf_of = [&](int g, const TQ& tq) __attribute__((always_inline)) {
        return fmaf(coef + 0x1p-18f, tq.tmax, tfb[g]) + rho_of(g, tq);
    };
    auto tile_q = [&](int buf) __attribute__((always_inline)) -> TQ {
        const float4 w = *reinterpret_cast<const float4*>(tiles + buf * TILE + HDR + 4 * BN);
        return TQ{w.x, w.y, w.z};
    };

    // tiles of the piece: a multiple of the group (static tile places; the extra tiles read the
    // next rows or the pad blocks past the grid, which row_end rejects)
    const int ntiles = (row_end > row_begin) ? ((int)((row_end - row_begin + BN - 1) / BN) + GRP - 1) / GRP * GRP : 0;
    // scan rotation by the per-XCD cursor (the multi-segment schedule), as k_gemm_fused
    const int xcd = blockIdx.x & 7;
    int* blk_rot = reinterpret_cast<int*>(smem + NBUF * TILE);
    if (threadIdx.x == 0) {
        int r0 = 0;
        if (a.cursor && ntiles > 0) {
            const int64_t cu = (int64_t)__hip_atomic_load(&a.cursor[xcd], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 64;
            if (cu > row_begin && cu < row_end) r0 = (int)((cu - row_begin) / BN);
        }
        *blk_rot = r0;
    }
    int rot = 0;
    auto tile_row = [&](int t) __attribute__((always_inline)) -> int64_t {
        int pt = t + rot;
        pt = pt >= ntiles ? pt - ntiles : pt;
        return row_begin + (int64_t)pt * BN;
    };

    // ---- LDS-DMA of tiles (k_gemm_fused's pieces: slot P -> row P / SLOTS, the header past the
    // rows), with the row's 16-B slots swizzled: LDS slot p of row r holds column slot p ^ sw(r),
    // sw(r) = bit 2 ^ bit 3 of r.  The A-fragment read of this shape (lane l: row l & 15, slot
    // 4 s + (l >> 4)) on the padded rows (272 B at d = 128) is 2-way bank-conflicted in
    // ds_read_b128's lane groups {0-3, 12-15, 20-27}, ... (MI355X_MICROARCH.md, LDS; profiled:
    // SQ_LDS_BANK_CONFLICT 1.6e9 cycles per A launch, r06d16); with the swizzle every group
    // reads 64 distinct banks.  (The 32x32 shapes' reads are conflict-free unswizzled.)
    auto sw = [](int r) __attribute__((always_inline)) { return ((r >> 2) ^ (r >> 3)) & 1; };
    uint32_t doff[DMA_PER_WAVE];
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; i++) {
        const int P = (wave + NW * i) * 64 + lane;
        if (P >= BN * SLOTS) {
            doff[i] = (uint32_t)(BN * RB + 16 * min(P - BN * SLOTS, HS - 1));
        } else {
            const int row = min(P / SLOTS, BN - 1), sl = P % SLOTS;
            doff[i] = (uint32_t)(row * RB + 16 * (sl == SLOTS - 1 ? 0 : sl ^ sw(row)));
        }
    }
    const uint32_t lds_tiles = __builtin_amdgcn_readfirstlane(lds_addr(tiles));
    struct DmaTile { const unsigned char* src; uint32_t lds; };
    const unsigned char* piece_src = trainb + (row_begin / BN) * TB;
    auto dma_desc = [&](int buf, int t) -> DmaTile {
        int pt = t + rot;
        pt = pt >= ntiles ? pt - ntiles : pt;
        return DmaTile{piece_src + (int64_t)pt * TB, lds_tiles + (uint32_t)(buf * TILE)};
    };
    auto dma_piece = [&](int i, const DmaTile& d) __attribute__((always_inline)) {
        const int ins = wave + NW * i;
        if (NW * (i + 1) <= DMA_INS || ins < DMA_INS) dma16s(doff[i], d.src, d.lds + (uint32_t)ins * 1024u);
    };
    auto dma_at = [&](int s, bool on, const DmaTile& d) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < DMA_PER_WAVE; i++)
            if (on && (i * NS) / DMA_PER_WAVE == s) dma_piece(i, d);
    };

    // ---- one tile's MFMAs into X; between them the fast test of the previous tile (Y): per query
    // group the minimum of its NV values (a v_min3 chain pinned to the k-steps); returns bit g when
    // some lane of query group g holds a value <= tf[g]
    uint4 pa[PFK][RG];  // the next tile's first A fragments, read before the slow path
    const int aoff = j * STRIDE + 16 * (g4 ^ sw(j));  // this lane's A-fragment slot (swizzled rows)
    auto afrag = [&](const unsigned char* tile, int rg, int s) __attribute__((always_inline)) -> uint4 {
        return *reinterpret_cast<const uint4*>(tile + 16 * rg * STRIDE + aoff + 64 * s);
    };
    auto prefetch = [&](int buf) __attribute__((always_inline)) {
        const unsigned char* tile = tiles + buf * TILE;
#pragma unroll
        for (int s = 0; s < PFK && s < NS; s++)
#pragma unroll
            for (int rg = 0; rg < RG; rg++) pa[s][rg] = afrag(tile, rg, s);
    };
    auto step = [&](floatx4 (&X)[NACC], floatx4 (&Y)[NACC], int buf, bool dma_on, const DmaTile& dd,
                    const float (&tf)[QG], bool pre, float (&mn_out)[QG]) -> uint32_t {
        const unsigned char* tile = tiles + buf * TILE;
        // the norms of rows 16 rg + 4 g4 .. + 3 (one broadcast ds_read_b128 per row group) into
        // query group 0's accumulator; at k-step 0 the other groups' MFMAs read them there first
#pragma unroll
        for (int rg = 0; rg < RG; rg++) {
            if constexpr (KNN_STUDY_NO_NORM) {
                X[rg] = floatx4{1.0f, 1.0f, 1.0f, 1.0f} * ((float)a.d * (1.0f / 3.0f));
            } else {
                const float4 v = *reinterpret_cast<const float4*>(tile + HDR + 4 * (16 * rg + 4 * g4));
                X[rg] = floatx4{v.x, v.y, v.z, v.w};
            }
        }
        float mn[QG];
#pragma unroll
        for (int g = 0; g < QG; g++) mn[g] = INF;
        uint4 xa[NS][RG];
#pragma unroll
        for (int s = 0; s < PFK && s < NS; s++)
#pragma unroll
            for (int rg = 0; rg < RG; rg++) xa[s][rg] = pre ? pa[s][rg] : afrag(tile, rg, s);
#pragma unroll
        for (int s = 0; s < NS; s++) {
            dma_at(s, dma_on, dd);
            if (s + PFK < NS) {
#pragma unroll
                for (int rg = 0; rg < RG; rg++) xa[s + PFK][rg] = afrag(tile, rg, s + PFK);
            }
#pragma unroll
            for (int gg = 0; gg < QG; gg++) {
                const int g = s == 0 ? QG - 1 - gg : gg;  // (k-step 0: query group 0 last)
#pragma unroll
                for (int rg = 0; rg < RG; rg++) {
                    const int c = g * RG + rg;
                    X[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xa[s][rg]),
                                                                   __builtin_bit_cast(bf16x8, qf[g][s]),
                                                                   s == 0 ? X[rg] : X[c], 0, 0, 0);
                }
                if (!KNN_STUDY_NO_EPI) {
#pragma unroll
                    for (int v = s * VPK; v < (s + 1) * VPK && v < NV; v++)
                        mn[g] = fminf(mn[g], Y[g * RG + (v >> 2)][v & 3]);
                    if (s * VPK < NV) asm volatile("" : "+v"(mn[g]));
                }
            }
        }
        uint32_t u = 0u;
#pragma unroll
        for (int g = 0; g < QG; g++) u |= __ballot(mn[g] <= tf[g]) != 0ull ? (1u << g) : 0u;
#pragma unroll
        for (int g = 0; g < QG; g++) mn_out[g] = mn[g];
        return u;
    };

    auto store_cand = [&](int g, float L, float U, int64_t t) __attribute__((always_inline)) {
        if (ccnt[g] < cap_sub) {
            const int64_t o = q(g) * (int64_t)a.cap + (int64_t)(4 * seg + g4) * cap_sub + ccnt[g];
            a.cand[o] = CandRec{(int32_t)t, L, U};
        }
        ccnt[g]++;
    };
    auto bounds = [&](int g, float y, const TQ& tq, float& L, float& U) __attribute__((always_inline)) {
        const float G = qn[g] + y;
        const float dl = fmaf(coef, qn[g] + tq.tmax, eta) + rho_of(g, tq);
        L = G - dl;
        U = G + dl;
    };

    // per-quarter register lists: ascending, the first LL - ceil(k/4) entries -inf pads
    float lst[QG][LL];
    {
        const int pads = LL - (k + 3) / 4;
#pragma unroll
        for (int g = 0; g < QG; g++)
#pragma unroll
            for (int i = 0; i < LL; i++) lst[g][i] = i < pads ? -INF : INF;
    }
    float ninf_op;  // (an opaque -inf: min as v_med3, see k_gemm_fused)
    asm("s_mov_b32 %0, 0xff800000" : "=s"(ninf_op));
    auto fmin_op = [&](float x, float y) __attribute__((always_inline)) { return __builtin_amdgcn_fmed3f(x, y, ninf_op); };
    auto list_insert = [&](int g, float w) __attribute__((always_inline)) {
#pragma unroll
        for (int i = LL - 1; i >= 1; i--) lst[g][i] = __builtin_amdgcn_fmed3f(lst[g][i - 1], w, lst[g][i]);
        lst[g][0] = fmin_op(lst[g][0], w);
    };

    // lane-parallel slow path of query group g: every lane scans ITS OWN NV values once (the
    // passing mask, the value = the group minimum when the lane passes once), then handles one
    // passing value per round, all lanes together
    auto slow = [&](floatx4 (&Y)[NACC], int tp, const float (&tf)[QG], const TQ& tq, const float (&mnY)[QG],
                    uint32_t u) {
        const int64_t tbase = tile_row(tp);
        auto visit = [&](int g, int idx, float yv) __attribute__((always_inline)) {
            const int row = 16 * (idx >> 2) + 4 * g4 + (idx & 3);
            const int64_t t = tbase + row;
            float L, U;
            bounds(g, yv, tq, L, U);
            const bool keep = idx >= 0 && t < row_end && L <= thr[g];
            if (keep) store_cand(g, L, U, t);
            const float w = (keep && U < lst[g][LL - 1]) ? U : INF;
            if (__ballot(w < INF)) {
                list_insert(g, w);
                thr[g] = fmin_op(thr[g], quarter_max(lst[g][LL - 1]));
            }
        };
        auto pick = [](uint32_t mm) __attribute__((always_inline)) { return __ffs((int)mm) - 1; };
#pragma unroll
        for (int g = 0; g < QG; g++) {
            if (!((u >> g) & 1u)) continue;  // (wave-uniform)
            const float tfc = tf[g];
            uint32_t m = 0u;
            if constexpr (NV == 16) {
                asm volatile(F16_LE(17) F16_LE(16) F16_LE(15) F16_LE(14) F16_LE(13) F16_LE(12) F16_LE(11) F16_LE(10)
                             F16_LE(9) F16_LE(8) F16_LE(7) F16_LE(6) F16_LE(5) F16_LE(4) F16_LE(3) F16_LE(2)
                             : "+v"(m)
                             : "v"(tfc), F16_Y(0), F16_Y(1), F16_Y(2), F16_Y(3), F16_Y(4), F16_Y(5), F16_Y(6), F16_Y(7),
                               F16_Y(8), F16_Y(9), F16_Y(10), F16_Y(11), F16_Y(12), F16_Y(13), F16_Y(14), F16_Y(15)
                             : "vcc");
            } else {
                asm volatile(F16_LE(9) F16_LE(8) F16_LE(7) F16_LE(6) F16_LE(5) F16_LE(4) F16_LE(3) F16_LE(2)
                             : "+v"(m)
                             : "v"(tfc), F16_Y(0), F16_Y(1), F16_Y(2), F16_Y(3), F16_Y(4), F16_Y(5), F16_Y(6), F16_Y(7)
                             : "vcc");
            }
            float yv = mnY[g];
            int idx;
            if (__ballot((m & (m - 1u)) != 0u)) {
                // some lane passes twice: the minimum's position from a second mask
                uint32_t e = 0u;
                if constexpr (NV == 16) {
                    asm volatile(F16_LE(17) F16_LE(16) F16_LE(15) F16_LE(14) F16_LE(13) F16_LE(12) F16_LE(11) F16_LE(10)
                                 F16_LE(9) F16_LE(8) F16_LE(7) F16_LE(6) F16_LE(5) F16_LE(4) F16_LE(3) F16_LE(2)
                                 : "+v"(e)
                                 : "v"(yv), F16_Y(0), F16_Y(1), F16_Y(2), F16_Y(3), F16_Y(4), F16_Y(5), F16_Y(6), F16_Y(7),
                                   F16_Y(8), F16_Y(9), F16_Y(10), F16_Y(11), F16_Y(12), F16_Y(13), F16_Y(14), F16_Y(15)
                                 : "vcc");
                } else {
                    asm volatile(F16_LE(9) F16_LE(8) F16_LE(7) F16_LE(6) F16_LE(5) F16_LE(4) F16_LE(3) F16_LE(2)
                                 : "+v"(e)
                                 : "v"(yv), F16_Y(0), F16_Y(1), F16_Y(2), F16_Y(3), F16_Y(4), F16_Y(5), F16_Y(6), F16_Y(7)
                                 : "vcc");
                }
                // (y <= min holds at the minimum's positions only: e marks them)
                idx = pick(m & e);
            } else {
                idx = pick(m);
            }
            visit(g, idx, yv);
            if (__ballot((m & (m - 1u)) != 0u)) {
                m = idx >= 0 ? m ^ (1u << idx) : 0u;
#pragma unroll 1
                for (int round = 1; round < NV; round++) {
                    if (!__ballot(m != 0u)) break;
                    idx = pick(m);
                    yv = INF;
                    if constexpr (NV == 16) {
                        asm volatile(F16_SEL(0, 2) F16_SEL(1, 3) F16_SEL(2, 4) F16_SEL(3, 5) F16_SEL(4, 6) F16_SEL(5, 7)
                                     F16_SEL(6, 8) F16_SEL(7, 9) F16_SEL(8, 10) F16_SEL(9, 11) F16_SEL(10, 12)
                                     F16_SEL(11, 13) F16_SEL(12, 14) F16_SEL(13, 15) F16_SEL(14, 16) F16_SEL(15, 17)
                                     : "+v"(yv)
                                     : "v"(idx), F16_Y(0), F16_Y(1), F16_Y(2), F16_Y(3), F16_Y(4), F16_Y(5), F16_Y(6),
                                       F16_Y(7), F16_Y(8), F16_Y(9), F16_Y(10), F16_Y(11), F16_Y(12), F16_Y(13), F16_Y(14),
                                       F16_Y(15)
                                     : "vcc");
                    } else {
                        asm volatile(F16_SEL(0, 2) F16_SEL(1, 3) F16_SEL(2, 4) F16_SEL(3, 5) F16_SEL(4, 6) F16_SEL(5, 7)
                                     F16_SEL(6, 8) F16_SEL(7, 9)
                                     : "+v"(yv)
                                     : "v"(idx), F16_Y(0), F16_Y(1), F16_Y(2), F16_Y(3), F16_Y(4), F16_Y(5), F16_Y(6),
                                       F16_Y(7)
                                     : "vcc");
                    }
                    visit(g, idx, yv);
                    m = idx >= 0 ? m ^ (1u << idx) : 0u;
                }
            }
        }
#pragma unroll
        for (int g = 0; g < QG; g++) make_tfb(g);
    };

    // list exchange between the pieces of a query (the 32-query shape, a.lshare): each quarter
    // publishes its list at [q][piece][LL g4 ..] and merges the same quarter's lists of the other
    // pieces (disjoint rows), the bound the largest of the four quarters' merged ceil(k/4)-th
    auto exchange_lists = [&]() __attribute__((always_inline)) {
        const int W = a.lshare_w;
        const int pads = LL - (k + 3) / 4;
#pragma unroll
        for (int g = 0; g < QG; g++) {
            float* base = a.lshare + ((qvalid_of(g) ? q(g) : 0) * (int64_t)a.nseg) * W + LL * g4;
            if (qvalid_of(g)) {
                uint32_t* dst = reinterpret_cast<uint32_t*>(base + (int64_t)seg * W);
#pragma unroll
                for (int i = 0; i < LL; i++)
                    __hip_atomic_store(dst + i, __float_as_uint(lst[g][i] == -INF ? INF : lst[g][i]), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            float tmp[LL];
#pragma unroll
            for (int i = 0; i < LL; i++) tmp[i] = lst[g][i];
            for (int p = 0; p < a.nseg; p++) {
                if (p == seg) continue;
                const uint32_t* src = reinterpret_cast<const uint32_t*>(base + (int64_t)p * W);
#pragma unroll 1
                for (int i0 = pads & ~3; i0 < LL; i0 += 4) {
                    float w[4];
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        w[i] = qvalid_of(g) ? __uint_as_float(__hip_atomic_load(src + i0 + i, __ATOMIC_RELAXED,
                                                                             __HIP_MEMORY_SCOPE_AGENT))
                                         : INF;
                    const float wmin = fmin_fast(fmin_fast(w[0], w[1]), fmin_fast(w[2], w[3]));
                    if (!__ballot(wmin < tmp[LL - 1])) break;
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const float wi = w[i] < tmp[LL - 1] ? w[i] : INF;
#pragma unroll
                        for (int e = LL - 1; e >= 1; e--) tmp[e] = __builtin_amdgcn_fmed3f(tmp[e - 1], wi, tmp[e]);
                        tmp[0] = fmin_fast(tmp[0], wi);
                    }
                }
            }
            const float ub = quarter_max(tmp[LL - 1]);
            if (qvalid_of(g) && ub < thr[g]) {
                thr[g] = ub;
                make_tfb(g);
            }
        }
    };

    floatx4 accA[NACC], accB[NACC];
#pragma unroll
    for (int c = 0; c < NACC; c++) accA[c] = accB[c] = floatx4{};
    __syncthreads();  // blk_rot is written
    rot = __builtin_amdgcn_readfirstlane(*blk_rot);
#pragma unroll
    for (int p = 0; p < AHEAD; p++)
        if (p < ntiles) {
            const DmaTile d0 = dma_desc(p, p);
#pragma unroll
            for (int i = 0; i < DMA_PER_WAVE; i++) dma_piece(i, d0);
        }
    TQ tm_prev{0.0f, 0.0f, 0.0f};
    auto share_now = [&](int it) __attribute__((always_inline)) {
        return (it & (F16_SHARE_EVERY - 1)) == F16_SHARE_EVERY - 1;
    };
    auto list_share_now = [&](int it) __attribute__((always_inline)) {
        return it >= KNN_FUSED16_LIST_FIRST && ((it + 1) & it) == 0;
    };
    auto iter = [&](auto posc, floatx4 (&X)[NACC], floatx4 (&Y)[NACC], int it) {
        constexpr int POS = decltype(posc)::value;
        if constexpr (QG == 2) {
            if (a.lshare && list_share_now(it)) exchange_lists();
        }
        if (share_now(it)) {
            if (a.cursor && threadIdx.x == 0)
                __hip_atomic_store(&a.cursor[xcd], (uint32_t)(tile_row(it) >> 6), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            if (a.nseg > 1) {
#pragma unroll
                for (int g = 0; g < QG; g++) {
                    if (!qvalid_of(g)) continue;
                    const float gv = o2f(__hip_atomic_load(&a.gthr[q(g)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    if (g4 == 0 && thr[g] < gv) atomicMin(&a.gthr[q(g)], f2o(thr[g]));  // publish this bound
                    if (gv < thr[g]) { thr[g] = gv; make_tfb(g); }
                }
            }
        }
        if (POS == 0) {
            if constexpr (KNN_STUDY_NO_BARRIER) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            else wait_dma_barrier();
        }
        const TQ tm_cur = tile_q(it % NBUF);
        const bool dma_on = !KNN_STUDY_NO_DMA && it + AHEAD < ntiles;
        const DmaTile dd = dma_desc((it + AHEAD) % NBUF, it + AHEAD);
        float tf[QG];
#pragma unroll
        for (int g = 0; g < QG; g++) tf[g] = it > 0 ? tf_of(g, tm_prev) : -INF;
        float mnY[QG];
        const uint32_t uY = step(X, Y, it % NBUF, dma_on, dd, tf, POS != 0, mnY);
        if (POS != GRP - 1 && it + 1 < ntiles) prefetch((it + 1) % NBUF);
        if (!KNN_STUDY_NO_SLOW) {
            if (uY) slow(Y, it - 1, tf, tm_prev, mnY, uY);
        } else {
            asm volatile("" ::"s"(uY));
        }
        tm_prev = tm_cur;
    };
    if constexpr (GRP == 8) {
        for (int it = 0; it < ntiles; it += 8) {
            iter(std::integral_constant<int, 0>{}, accA, accB, it);
            iter(std::integral_constant<int, 1>{}, accB, accA, it + 1);
            iter(std::integral_constant<int, 2>{}, accA, accB, it + 2);
            iter(std::integral_constant<int, 3>{}, accB, accA, it + 3);
            iter(std::integral_constant<int, 4>{}, accA, accB, it + 4);
            iter(std::integral_constant<int, 5>{}, accB, accA, it + 5);
            iter(std::integral_constant<int, 6>{}, accA, accB, it + 6);
            iter(std::integral_constant<int, 7>{}, accB, accA, it + 7);
        }
    } else {
        for (int it = 0; it < ntiles; it += 4) {
            iter(std::integral_constant<int, 0>{}, accA, accB, it);
            iter(std::integral_constant<int, 1>{}, accB, accA, it + 1);
            iter(std::integral_constant<int, 2>{}, accA, accB, it + 2);
            iter(std::integral_constant<int, 3>{}, accB, accA, it + 3);
        }
    }
    if (ntiles > 0) {
        // drain: the last tile's accumulators (ntiles is even: accB)
        const int last = ntiles - 1;
        float tf[QG], mnB[QG];
#pragma unroll
        for (int g = 0; g < QG; g++) {
            tf[g] = tf_of(g, tm_prev);
            mnB[g] = INF;
#pragma unroll
            for (int v = 0; v < NV; v++) mnB[g] = fminf(mnB[g], accB[g * RG + (v >> 2)][v & 3]);
        }
        slow(accB, last, tf, tm_prev, mnB, (1u << QG) - 1u);
    }
#pragma unroll
    for (int g = 0; g < QG; g++)
        if (qvalid_of(g) && g4 == 0) atomicMin(&a.gthr[q(g)], f2o(thr[g]));
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < QG; g++)
        if (qvalid_of(g)) a.cnt[(int64_t)(4 * seg + g4) * a.nq + q(g)] = ccnt[g];
}

// the grid of k_gemm_fused (knn_fused_schedule: whole query tiles, then balanced ranges run from
// their end; or the segment schedule), one piece function per block
template <int RB, int MINW, int NBUF, int NW, int QG, int RG, int KR>
__global__ __launch_bounds__(64 * NW, MINW) void k_gemm_fused16(GemmFilterArgs a) {
    if ((a.gate && *a.gate == 0) || (*a.status & KNN_STATUS_GEMM_UNSAFE)) return;
    const int64_t T = a.tiles64;
    const int b = blockIdx.x;
    const bool segmode = a.g2 < 0;
    const bool p1 = !segmode && b < a.p1_blocks;
    const int64_t b2 = b - a.p1_blocks;
    auto lo = [&](int64_t bb) { return bb * a.w2 / a.g2; };
    int64_t x = 0, x1 = 1;
    if (!segmode) {
        x = p1 ? (int64_t)b * T : lo(b2);
        x1 = p1 ? x + T : lo(b2 + 1);
    }
    const int qbase = p1 ? 0 : a.p1_blocks;
    for (bool first = true; x < x1; first = false) {
        int qt, seg;
        int64_t rb, re, adv;
        if (segmode) {
            qt = b % a.n_qtiles;
            seg = b / a.n_qtiles;
            rb = (int64_t)seg * a.seg_len;
            re = min(a.nt, rb + a.seg_len);
            adv = 1;
        } else {
            const int64_t ql = (x1 - 1) / T;
            const int64_t t0 = max(x, ql * T) - ql * T, t1 = x1 - ql * T;
            qt = qbase + (int)ql;
            seg = p1 ? 0 : (int)(b2 - ((ql * T + 1) * a.g2 - 1) / a.w2);
            rb = t0 * 64;
            re = min(a.nt, t1 * 64);
            adv = t1 - t0;
        }
        if (!first) __syncthreads();
        fused16_piece<RB, NBUF, NW, QG, RG, KR>(a, qt, seg, rb, re);
        if (segmode) x += adv;
        else x1 -= adv;
    }
}

// the 16x16x32 kernel of a register-list plan (knn_fused_plan with force.m16): plan (qg, rg) in
// 32-units -> (2 qg, 2 rg) 16-groups; nullptr when the plan has no 16x16x32 form
const void* knn_fused16_ptr(int d, const FilterPlan& f) {
    if (!(f.kr == 8 || f.kr == 32) || f.nw != 8) return nullptr;
#define KNN_F16(RB, NB, QG, RG, KR) reinterpret_cast<const void*>(&k_gemm_fused16<RB, 2, NB, 8, QG, RG, KR>)
#define KNN_F16_D(RB)                                                                              \
    do {                                                                                           \
        if (f.qg == 2 && f.rg == 1 && f.nbuf == 16) return f.kr == 8 ? KNN_F16(RB, 16, 4, 2, 8) : KNN_F16(RB, 16, 4, 2, 32); \
        if (f.qg == 1 && f.rg == 2 && f.nbuf == 8) return f.kr == 8 ? KNN_F16(RB, 8, 2, 4, 8) : KNN_F16(RB, 8, 2, 4, 32);   \
    } while (0)
    if (d == 64) KNN_F16_D(128);
    if (d == 128) KNN_F16_D(256);
#undef KNN_F16_D
#undef KNN_F16
    return nullptr;
}
