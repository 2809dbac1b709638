// knn_fused.hip -- the GEMM-form candidate filter on the bf16 MFMA with the train norm
// folded into the MFMA (gfx950).  DESIGN.md "Fused-norm filter".
//
// Rows are augmented by 16 bf16 columns (k_aug_rows):
//   train  [ rn(t_0) .. rn(t_{d-1}) | tn_hi tn_mid tn_lo 0 x 13 ]   (tn = ||t||^2, fp32)
//   query  [ -2 rn(q_0) .. -2 rn(q_{d-1}) | 1 1 1 0 x 13 ]
// so one chain of v_mfma_f32_32x32x16_bf16 over d/16 + 1 k-steps leaves
//   y = tn - 2 rn(q).rn(t)
// in the accumulators: the fast test is a v_min3 chain over the 16 values of an
// accumulator against one per-(query, tile) threshold, with no per-value norm read or
// fma; the slow path walks the values in a runtime loop with a wave-uniform index (a
// scalar-indexed register read, no scratch), computes the exact certificate bounds
//   G = qn + y,  Delta = coef (qn + tn) + eta,  L = G - Delta <= D <= U = G + Delta
// (D: the reference's direct-form distance, main.cpp:14-23) and keeps (row, L, U) for
// the exact rescore (k_rescore) exactly like k_gemm_filter.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "knn_device.h"
#include "knn_kernels.h"
#include "knn_study.h"

#ifndef KNN_FUSED_PF
#define KNN_FUSED_PF 6  // A-fragment prefetch depth in MFMAs
#endif
#ifndef KNN_FUSED_DEFER
#define KNN_FUSED_DEFER 1  // 8-wave shapes: queue passing values, flush all waves together
#endif
#ifndef KNN_FUSED_DEFER_EVERY
#define KNN_FUSED_DEFER_EVERY 64  // tiles between flushes of the deferred queues
#endif
#ifndef KNN_FUSED_PSTEP
#define KNN_FUSED_PSTEP 0  // 1 (study): the in-step pass set for d >= 128
#endif
#ifndef KNN_FUSED_PRIO
#define KNN_FUSED_PRIO 0  // 1 (study): s_setprio 1 for the second half of the waves
#endif
#ifndef KNN_FUSED_LATE_DMA
#define KNN_FUSED_LATE_DMA 0
#endif
#ifndef KNN_FUSED_DMA_OFS
#define KNN_FUSED_DMA_OFS 0  // k-steps the tile's DMA pieces are shifted by within the step (study)
#endif
#ifndef KNN_FUSED_SHARE_EVERY
#define KNN_FUSED_SHARE_EVERY 64  // tiles between threshold exchanges of a query's pieces (gthr)
#endif
#ifndef KNN_FUSED_GROUP_SET
#define KNN_FUSED_GROUP_SET 1  // the lazy pass set by groups of 4 values first (B 703 -> 674 ms, A same)
#endif
#ifndef KNN_FUSED_ROW_NORM
#define KNN_FUSED_ROW_NORM 0  // 1: the slow path's bounds use each row's norm (an LDS ring filled by DMA)
#endif
#ifndef KNN_FUSED_RQ
#define KNN_FUSED_RQ 4  // deferred-queue depth per lane
#endif


// ---------------------------------------------------------------------------------
// k_aug_rows<E>: rows of the fused filter, [n][d + 16] bf16.  Element c < d is
// rn(scale * x[r][c]) (scale = 1: train, -2: queries; exact scaling by a power of two);
// the augmented block is the three-term bf16 split of norms[r] (train: tn = hi + mid +
// lo + r, |r| <= 2^-24 tn, each subtraction exact by Sterbenz) or (1, 1, 1) (queries,
// norms == NULL), then zeros.  One thread per 4 elements: a float4 (or 4 bf16) in, one
// 8-byte bf16 quad out.
// ---------------------------------------------------------------------------------
template <typename E>
__global__ __launch_bounds__(256) void k_aug_rows(const E* __restrict__ x, int64_t n, int ld, int d,
                                                  const float* __restrict__ norms, float scale,
                                                  bf16_t* __restrict__ out, const int32_t* __restrict__ gate) {
    if (gate && *gate == 0) return;
    const int per_row = (d + 16) >> 2;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n * per_row) return;
    const int64_t r = i / per_row;
    const int c = (int)(i - r * per_row) * 4;
    uint32_t w0 = 0u, w1 = 0u;
    if (c < d) {
        const float4 v = load4(x + r * ld + c);
        w0 = bf16_rne(scale * v.x) | (bf16_rne(scale * v.y) << 16);
        w1 = bf16_rne(scale * v.z) | (bf16_rne(scale * v.w) << 16);
    } else if (c == d) {
        if (norms) {
            const float t = norms[r];
            const uint32_t hi = bf16_rne(t);
            const float r1 = t - __uint_as_float(hi << 16);
            const uint32_t mid = bf16_rne(r1);
            const uint32_t lo = bf16_rne(r1 - __uint_as_float(mid << 16));
            w0 = hi | (mid << 16);
            w1 = lo;
        } else {
            w0 = 0x3f803f80u;  // bf16 1.0, 1.0
            w1 = 0x00003f80u;  // 1.0, 0
        }
    }
    *reinterpret_cast<uint2*>(out + r * (int64_t)(d + 16) + c) = make_uint2(w0, w1);
}

hipError_t knn_launch_aug_rows(const void* x, int elem, int64_t n, int ld, int d, const float* norms, float scale,
                               uint16_t* out, hipStream_t st, const int32_t* gate) {
    const int64_t total = n * ((d + 16) / 4);
    if (total <= 0) return hipSuccess;
    if (d % 4 || ld % 4) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((total + 255) / 256));
    if (elem == ELEM_BF16)
        hipLaunchKernelGGL(k_aug_rows<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, n, ld, d, norms, scale,
                           (bf16_t*)out, gate);
    else
        hipLaunchKernelGGL(k_aug_rows<float>, grid, dim3(256), 0, st, (const float*)x, n, ld, d, norms, scale,
                           (bf16_t*)out, gate);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

// ---------------------------------------------------------------------------------
// k_gemm_fused<RB, MINW, NBUF, NW, RG>: the filter (RB = bytes per augmented row,
// 2d + 32).  Block = NW waves x 32 queries; a train tile has BN = 32 RG rows, copied
// global -> LDS by LDS-DMA (NBUF buffers, one barrier per tile, pieces issued between
// the MFMAs) with each row padded to RB + 16 bytes (conflict-free ds_read_b128 of the A
// fragments).  Lane (j, h) holds 16 bytes of its query's augmented row per k-step in
// VGPRs (the B fragment) for the whole scan; register r of accumulator c holds train
// row 32c + (r & 3) + 8 (r >> 2) + 4h of the tile against query j.  Per tile each wave
// issues the MFMAs of tile it into X while the fast test of tile it-1 (Y) runs in
// between (software pipelining).
//
// Fast test: the tile passes for query q when min_r y_r <= tf(q, tile), with
//   tf = (thr - qn) + coef qn + eta + 2^-18 (|thr| + qn) + (coef + 2^-18) tmax_tile,
// tmax_tile >= tn of every row of the tile (k_row_norms' per-64-row maxima): a superset
// of the exact test L <= thr (2^-18 (...) covers the few fp32 roundings between the two
// forms, <= 2^-21 of the same magnitudes).
// Threshold thr: the k-th smallest U among rows this block kept (per-query 4-ary
// max-heap in LDS, as k_gemm_filter), or a smaller bound published by another segment
// (gthr).  Every row of the exact top-k has L <= D <= D_(k) <= thr, so it is kept.
// ---------------------------------------------------------------------------------
// fused_piece: one piece of work -- query tile qt against train rows [row_begin, row_end),
// piece (segment) id seg of that query tile (its candidate sub-slices, 2 seg + h)
template <int RB, int NBUF, int NW, int RG, bool PSTEP, int KR>
__device__ __forceinline__ void fused_piece(const GemmFilterArgs& a, const int qt, const int seg,
                                            const int64_t row_begin, const int64_t row_end) {
    typedef FilterTile<RB, NW, 1, RG> FT;
    constexpr int NACC = RG, BN = FT::BN, BM = FT::BM, STRIDE = FT::STRIDE, SLOTS = FT::SLOTS;
    constexpr int DMA_INS = FT::DMA_INS, TILE = FT::TILE;
    constexpr int NT = 64 * NW;
    constexpr int DMA_PER_WAVE = (DMA_INS + NW - 1) / NW;
    constexpr int NS = RB / 32;                  // k-steps: d/16 feature steps + the norm step
    constexpr int VPS = (16 + NS - 1) / NS;      // fast-test values per k-step per accumulator
    constexpr int NR = NBUF + 1;                 // norm ring slots: tiles it-1 .. it+NBUF-1
    constexpr int RS = BN;                       // ring slot: BN row norms
    static_assert(NBUF == 2 || NBUF == 3 || NBUF == 4 || NBUF == 6, "tile buffers");
    // NBUF = 2 GRP (4, 6): tiles go in groups of GRP -- one barrier per group; the DMA of tile
    // it + GRP is issued during step it into the buffer tile it - GRP used (read before this
    // group's barrier)
    constexpr int GRP = (NBUF == 4 || NBUF == 6) ? NBUF / 2 : 1;
    constexpr bool PAIR = GRP > 1;
    constexpr int AHEAD = PAIR ? GRP : NBUF - 1;  // tiles between a step and the tile it DMAs
    static_assert(RG == 1 || RG == 2, "row groups");
    static_assert(KR == 0 || KR == 16 || KR == 32, "register lists: k <= 16, k <= 32, or LDS heaps");
    constexpr bool RL = KR > 0;       // thresholds from per-lane register lists (else LDS heaps)
    constexpr bool HALVES = KR == 32;  // k <= 32: one 16-entry list per lane half (below)
    constexpr int LL = 16;             // register list length
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* tiles = smem;                                     // [NBUF][TILE]
    float* ring = reinterpret_cast<float*>(smem + NBUF * TILE);      // [NR][RS] train norms tn
    const int hs = heap_stride(a.k);
    float* topU = ring + NR * RS;                                    // [BM][hs] max-heaps of U
    const int cap_sub = a.cap_seg / 2;  // candidate sub-slice of one lane half (h) of a query

    const int lane = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = lane & 31;
    const int h = lane >> 5;
    if (KNN_FUSED_PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    const int k = a.k;
    const float INF = __uint_as_float(0x7f800000u);
    const float coef = a.coef, eta = a.eta;
    const int64_t ldb = (int64_t)a.ld_t * 2;  // augmented train row pitch, bytes
    const unsigned char* trainb = reinterpret_cast<const unsigned char*>(a.train);

    if constexpr (!RL) {
        for (int i = threadIdx.x; i < BM * hs; i += NT) {
            const int e = i % hs;
            topU[i] = (e == hs - 1 || e <= k - 2) ? INF : -INF;  // root, nodes 1..k-1: +inf
        }
    }
    for (int i = threadIdx.x; i < NR * RS; i += NT) ring[i] = INF;

    // this lane's query (both lane halves hold the same query, different rows)
    const int jl = wave * 32 + j;
    const int64_t q = (int64_t)qt * BM + jl;
    const bool qvalid = q < a.nq;
    uint4 qf[NS];
    {
        const unsigned char* qrow = reinterpret_cast<const unsigned char*>(a.test) +
                                    (qvalid ? q : 0) * (int64_t)a.ld_q * 2;
#pragma unroll
        for (int s = 0; s < NS; s++)
            qf[s] = qvalid ? *reinterpret_cast<const uint4*>(qrow + 32 * s + 16 * h) : make_uint4(0u, 0u, 0u, 0u);
    }
    const float qn = qvalid ? a.qnorm[q] : 0.0f;
    float thr = qvalid ? o2f(a.gthr[q]) : -INF;
    float published = thr;
    float root = INF;  // this query's heap root, mirrored in both lanes
    int ccnt = 0;      // candidates this lane half kept
    float tfb;         // tf without the tile term
    auto make_tfb = [&]() __attribute__((always_inline)) {
        tfb = qvalid ? ((thr - qn) + fmaf(coef, qn, eta)) + 0x1p-18f * (fabsf(thr) + qn) : -INF;
    };
    make_tfb();
    // tile term: tq = {the tile's maximum norm tmax, the operand-rounding bound of this query
    // against the tile's rows, 2 (|q| max|t - rt| + |q - rq| max|rt|) (1 + 2^-17)}
    auto tf_of = [&](float2 tq) __attribute__((always_inline)) { return fmaf(coef + 0x1p-18f, tq.x, tfb) + tq.y; };
    float qe2 = 0.0f, eq2 = 0.0f;  // 2 |q| and 2 |q - rq|, rounded up
    if (qvalid) {
        const float2 qs = a.qstat[q];
        qe2 = 2.0f * qs.x * (1.0f + 0x1p-17f);
        eq2 = 2.0f * qs.y * (1.0f + 0x1p-17f);
    }
    // the tile's stats by a scalar load (constant address space, wave-uniform index): counted
    // by lgkmcnt, so using them never waits on the vector-memory count the tile DMAs share
    auto tile_q = [&](int64_t tile) __attribute__((always_inline)) -> float2 {
        const int ti = __builtin_amdgcn_readfirstlane((int)tile);
#ifdef __HIP_DEVICE_COMPILE__
        typedef __attribute__((address_space(4))) const float* cfloatp;
        const cfloatp p = (cfloatp)(a.tstat + ti);
        const float4 t = make_float4(p[0], p[1], p[2], p[3]);
#else
        const float4 t = a.tstat[ti];  // (the host pass only parses device code)
#endif
        return make_float2(t.x, fmaf(qe2, t.y, eq2 * t.z));
    };

    const int ntiles = (row_end > row_begin) ? (int)((row_end - row_begin + BN - 1) / BN) : 0;

    // ---- LDS-DMA of tiles (same image as k_gemm_filter: slot P -> row P / SLOTS, slot P % SLOTS,
    // the pad slot duplicates slot 0; rows past nt read row nt-1 and are rejected by index)
    uint32_t doff[DMA_PER_WAVE];
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; i++) {
        const int P = (wave + NW * i) * 64 + lane;
        const int row = min(P / SLOTS, BN - 1), sl = P % SLOTS;
        doff[i] = (uint32_t)(row * ldb + 16 * (sl == SLOTS - 1 ? 0 : sl));
    }
    // this wave's vector-memory ops per tile: its DMA pieces (+ the norm ring load of the
    // last wave) and the tile-max load
    int n_dma_wave = (KNN_FUSED_ROW_NORM && wave == NW - 1) ? 2 : 1;
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; i++) n_dma_wave += (wave + NW * i < DMA_INS) ? 1 : 0;
    constexpr int NPIECE = DMA_PER_WAVE + (KNN_FUSED_ROW_NORM ? 1 : 0);
    const uint32_t lds_tiles = __builtin_amdgcn_readfirstlane(lds_addr(tiles));
    const uint32_t lds_ring = __builtin_amdgcn_readfirstlane(lds_addr(ring));
    struct DmaTile { const unsigned char* src; uint32_t lds, lring; int64_t r0; bool full; };
    auto dma_desc = [&](int buf, int slot, int64_t r0) -> DmaTile {
        return DmaTile{trainb + r0 * ldb, lds_tiles + (uint32_t)(buf * TILE), lds_ring + (uint32_t)(slot * RS * 4), r0,
                       r0 + BN <= a.nt};
    };
    auto dma_piece = [&](int i, const DmaTile& d) __attribute__((always_inline)) {
        if (i < DMA_PER_WAVE) {
            const int ins = wave + NW * i;
            if (ins < DMA_INS) {
                if (i == DMA_PER_WAVE - 1 && ins == DMA_INS - 1 && lane >= FT::LAST_LANES) return;
                const uint32_t dst = d.lds + (uint32_t)ins * 1024u;
                if (d.full) {
                    dma16s(doff[i], d.src, dst);
                } else {
                    const int P = ins * 64 + lane;
                    const int row = P / SLOTS, sl = P % SLOTS;
                    const int64_t t = min(d.r0 + row, a.nt - 1);
                    dma16(trainb + t * ldb + 16 * (sl == SLOTS - 1 ? 0 : sl), dst);
                }
            }
        } else if (wave == NW - 1 && lane < BN) {
            dma4s(4u * lane, a.tnorm + d.r0, d.lring);
        }
    };
    auto dma_tile = [&](int buf, int slot, int64_t r0) __attribute__((always_inline)) {
        const DmaTile d = dma_desc(buf, slot, r0);
#pragma unroll
        for (int i = 0; i < NPIECE; i++) dma_piece(i, d);
    };
    auto dma_at = [&](int s, bool on, const DmaTile& d) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NPIECE; i++)
            if (on && ((i * NS) / NPIECE + KNN_FUSED_DMA_OFS) % NS == s) dma_piece(i, d);
    };

    // ---- one tile's MFMAs into X; in between, the fast test of the previous tile (Y): bit
    // 16c + r of the returned set is 1 iff value r of accumulator c passes (y <= tf) in some
    // lane (one v_cmp per value into an SGPR pair; the scalar ops issue beside the MFMAs --
    // measured faster on A than a v_min3 chain plus a separate pass over the values)
    constexpr int PF = KNN_FUSED_PF / NACC;  // k-steps of A fragments read ahead
    uint4 pa[PF], pb[PF];                    // PAIR: the odd step's first fragments, read early
    auto prefetch = [&](int buf) __attribute__((always_inline)) {
        const unsigned char* tile = tiles + buf * TILE;
        const unsigned char* a0p = tile + j * STRIDE + 16 * h;
        const unsigned char* a1p = tile + ((RG == 2 ? 32 : 0) + j) * STRIDE + 16 * h;
#pragma unroll
        for (int s = 0; s < PF && s < NS; s++) {
            pa[s] = *reinterpret_cast<const uint4*>(a0p + 32 * s);
            if (RG == 2) pb[s] = *reinterpret_cast<const uint4*>(a1p + 32 * s);
        }
    };
    auto step = [&](floatx16 (&X)[NACC], floatx16 (&Y)[NACC], int buf, bool dma_on, const DmaTile& dd,
                    float tf, bool pre) -> uint32_t {
        const unsigned char* tile = tiles + buf * TILE;
        const unsigned char* a0p = tile + j * STRIDE + 16 * h;
        const unsigned char* a1p = tile + ((RG == 2 ? 32 : 0) + j) * STRIDE + 16 * h;
        KNN_STUDY_STEP_HEAD();
#pragma unroll
        for (int c = 0; c < NACC; c++) X[c] = floatx16{};
        uint32_t u = 0u;
        float mn[NACC];
#pragma unroll
        for (int c = 0; c < NACC; c++) mn[c] = INF;
        uint4 xa[NS], xb[NS];
#pragma unroll
        for (int s = 0; s < PF && s < NS; s++) {
            if (pre) {
                xa[s] = pa[s];
                if (RG == 2) xb[s] = pb[s];
            } else {
                xa[s] = *reinterpret_cast<const uint4*>(a0p + 32 * s);
                if (RG == 2) xb[s] = *reinterpret_cast<const uint4*>(a1p + 32 * s);
            }
        }
#pragma unroll
        for (int s = 0; s < NS; s++) {
            dma_at(s, dma_on, dd);
            if (s + PF < NS) {
                xa[s + PF] = *reinterpret_cast<const uint4*>(a0p + 32 * (s + PF));
                if (RG == 2) xb[s + PF] = *reinterpret_cast<const uint4*>(a1p + 32 * (s + PF));
            }
#pragma unroll
            for (int c = 0; c < NACC; c++) {
                const bf16x8 A = __builtin_bit_cast(bf16x8, (RG == 2 && c) ? xb[s] : xa[s]);
                X[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, __builtin_bit_cast(bf16x8, qf[s]), X[c], 0, 0, 0);
#ifndef KNN_ABLATE_NO_EPI
                if constexpr (PSTEP) {
#pragma unroll
                    for (int v = s * VPS; v < (s + 1) * VPS && v < 16; v++)
                        u |= (__ballot(Y[c][v] <= tf) != 0ull ? 1u : 0u) << (16 * c + v);
                } else {
#pragma unroll
                    for (int v = s * VPS; v < (s + 1) * VPS && v < 16; v++) mn[c] = fminf(mn[c], Y[c][v]);
                }
#endif
            }
            // keep this k-step's order (prefetch, MFMA, VALU): load-bearing -- relaxed, the
            // filter runs 11 % faster and drops true neighbours (DESIGN.md "Next" 1)
            KNN_STUDY_KSTEP_BARRIER(s);
        }
        if constexpr (!PSTEP) {
            // which accumulators hold a passing value; the slow path builds their value sets
            // (pass_set) -- usually one of the two
#pragma unroll
            for (int c = 0; c < NACC; c++) u |= __ballot(mn[c] <= tf) != 0ull ? (0xffffu << (16 * c)) : 0u;
        }
        return u;
    };

#ifdef KNN_FILTER_TIMING
    unsigned long long tph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define KNN_TSTAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define KNN_TSTAMP(v)
#endif

    // append candidate (L, U) of global row t to this lane half's sub-slice (past its
    // capacity: counted only, the rescore then sends the query to the exact scan)
    auto store_cand = [&](float L, float U, int64_t t) __attribute__((always_inline)) {
        if (ccnt < cap_sub) {
            const int64_t o = q * (int64_t)a.cap + (int64_t)(2 * seg + h) * cap_sub + ccnt;
            a.cand[o] = CandRec{(int32_t)t, L, U};
        }
        ccnt++;
    };
    // keep candidate (L, U) of global row t: the exact test against the current threshold,
    // the candidate store into this lane half's sub-slice, and, if U beats the heap root, a
    // sift-down of the query's 4-ary max-heap (node n >= 1 in H[n-1], the root in H[hs-1]:
    // the four children of node i are one aligned 16-byte read at H[4i]).  Only one lane of
    // a query runs it at a time.
    auto accept = [&](float L, float U, int64_t t) __attribute__((always_inline)) {
        if (!(L <= thr)) return;
        store_cand(L, U, t);
        if (U < root) {
            float* H = topU + jl * hs;
            int i = 0;
            float newroot = U;
            for (;;) {
                if (4 * i + 1 > k - 1) break;
                const float4 cc = *reinterpret_cast<const float4*>(H + 4 * i);
                const float cm = fmaxf(fmaxf(cc.x, cc.y), fmaxf(cc.z, cc.w));
                if (cm <= U) break;
                const int ci = cm == cc.x ? 0 : cm == cc.y ? 1 : cm == cc.z ? 2 : 3;
                H[i == 0 ? hs - 1 : i - 1] = cm;
                if (i == 0) newroot = cm;
                i = 4 * i + 1 + ci;
            }
            H[i == 0 ? hs - 1 : i - 1] = U;
            root = newroot;
            thr = fminf(thr, root);
        }
    };
    auto sync_roots = [&](int hh) __attribute__((always_inline)) {
        const float other = __shfl_xor(root, 32);
        if (h != hh) root = other;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    };
    auto publish = [&]() __attribute__((always_inline)) {
        if (qvalid) {
            thr = fminf(thr, root);
            if (a.nseg > 1 && h == 0 && thr < published) {
                atomicMin(&a.gthr[q], f2o(thr));
                published = thr;
            }
            make_tfb();
        }
    };
    // certified bounds L <= D <= U of value y of row `row` of tile tp: Delta = coef (qn + tn)
    // + eta with tn the row's norm (KNN_FUSED_ROW_NORM, from the ring) or, by default, the
    // tile's maximum norm tm >= tn -- a slightly wider band (still L <= D <= U), and no LDS
    // read and wait per visited value
    auto bounds = [&](float y, int row, int tp, float2 tq, float& L, float& U) __attribute__((always_inline)) {
        const float G = qn + y;
        const float tn = KNN_FUSED_ROW_NORM ? ring[(tp % NR) * RS + row] : tq.x;
        const float dl = fmaf(coef, qn + tn, eta) + tq.y;
        L = G - dl;
        U = G + dl;
    };

    // value v (wave-uniform) of accumulators Y: a scalar-indexed register read (v_movrels),
    // so the walk below is a runtime loop with one copy of its body -- a static walk over
    // the 16 NACC values replicates accept() per value, and the code no longer fits the
    // instruction cache (measured 10x slower on B)
    auto yval = [&](floatx16 (&Y)[NACC], int v) __attribute__((always_inline)) -> float {
        if constexpr (NACC == 1) return Y[0][v & 15];
        else return (v >> 4) ? Y[1][v & 15] : Y[0][v & 15];
    };
    // the values of Y some lane passes (bit 16c + r): one v_cmp per value into an SGPR pair,
    // then scalar ops (the !PSTEP variant builds it only on tiles some value passes).
    // Measured (same box): sets by groups of 4 values (a min of 4 per ballot) are slower on A
    // and B -- the extra slow-path visits cost more than the scalar ops they save.
    auto pass_set = [&](floatx16 (&Y)[NACC], float tf, uint32_t acc = 0xffffffffu) __attribute__((always_inline)) -> uint32_t {
        uint32_t u = 0u;
#pragma unroll
        for (int c = 0; c < NACC; c++)
            if ((acc >> (16 * c)) & 1u) {  // (wave-uniform) only the accumulators that pass
#if KNN_FUSED_GROUP_SET
                // then only the groups of 4 values (rows 8g .. 8g+3 of the lane half) whose
                // minimum passes
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const float gm = fminf(fminf(Y[c][4 * g], Y[c][4 * g + 1]), fminf(Y[c][4 * g + 2], Y[c][4 * g + 3]));
                    if (__ballot(gm <= tf)) {
#pragma unroll
                        for (int r = 4 * g; r < 4 * g + 4; r++)
                            u |= (__ballot(Y[c][r] <= tf) != 0ull ? 1u : 0u) << (16 * c + r);
                    }
                }
#else
#pragma unroll
                for (int r = 0; r < 16; r++) u |= (__ballot(Y[c][r] <= tf) != 0ull ? 1u : 0u) << (16 * c + r);
#endif
            }
        return u;
    };
    // immediate slow path: the passing values of tile tp, visited by index; the two lanes
    // of a query take turns (one heap writer at a time)
    auto slow = [&](floatx16 (&Y)[NACC], int tp, float tf, float2 tq, uint32_t u) {
        const int64_t tbase = row_begin + (int64_t)tp * BN;
        if constexpr (!PSTEP) u = pass_set(Y, tf, u);
        while (u) {
            const int v = __builtin_ctz(u);
            u &= u - 1u;
            const float y = yval(Y, v);
            const bool p = y <= tf;
            const int r = v & 15;
            const int row = 32 * (v >> 4) + (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t t = tbase + row;
#pragma unroll 1
            for (int hh = 0; hh < 2; hh++) {
                if (!__ballot(p && h == hh)) continue;
                if (p && h == hh && t < row_end) {
                    float L, U;
                    bounds(y, row, tp, tq, L, U);
                    accept(L, U, t);
                }
                sync_roots(hh);
            }
        }
        publish();
    };

    // register-list slow path (KR > 0), k <= 16: both lanes of a query (its two row halves)
    // keep the same ascending list lst[] of the 16 smallest U of the query's kept candidates
    // -- the first 16 - k entries are -inf pads, so lst[15] is the k-th smallest real U, an
    // upper bound on D_(k) (k rows with D <= U <= it).  Per passing value the two lanes swap
    // their candidate U (v_permlane32_swap) and both insert both (32 v_med3, the multiset and
    // so the list come out the same in either order): the query's exact k-th smallest, like
    // the heap, for all 32 queries of the wave at once -- no LDS, no lane takes turns.
    // HALVES (16 < k <= 32): each lane keeps its own half's ceil(k/2) smallest U (16 - ceil(k/2)
    // pads) and inserts only its own values (16 v_med3); the bound is the larger of the two
    // halves' ceil(k/2)-th smallest -- at least 2 ceil(k/2) >= k kept rows have U <= it.  A
    // little looser than the exact k-th smallest, with no LDS heap and no turn-taking.
    float lst[RL ? LL : 1];
    if constexpr (RL) {
        const int pads = LL - (HALVES ? (k + 1) / 2 : k);
#pragma unroll
        for (int i = 0; i < LL; i++) lst[i] = i < pads ? -INF : INF;
    }
    auto list_insert = [&](float w) __attribute__((always_inline)) {
#pragma unroll
        for (int i = LL - 1; i >= 1; i--) lst[i] = __builtin_amdgcn_fmed3f(lst[i - 1], w, lst[i]);
        lst[0] = fminf(lst[0], w);
    };
    // the other lane half's copy of a word (v_permlane32_swap: one result of the swap is this
    // lane's own word, the other its partner's)
    auto partner = [&](float x) __attribute__((always_inline)) -> float {
        const uint32_t xb = __float_as_uint(x);
        const auto sw = __builtin_amdgcn_permlane32_swap(xb, xb, false, false);
        return __uint_as_float(sw[0] == xb ? sw[1] : sw[0]);
    };
    auto slow_rl = [&](floatx16 (&Y)[NACC], int tp, float tf, float2 tq, uint32_t u) {
        if constexpr (RL) {
            const int64_t tbase = row_begin + (int64_t)tp * BN;
            if constexpr (!PSTEP) u = pass_set(Y, tf, u);
            while (u) {
                const int v = __builtin_ctz(u);
                u &= u - 1u;
                const float y = yval(Y, v);
                const int r = v & 15;
                const int row = 32 * (v >> 4) + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int64_t t = tbase + row;
                float L, U;
                bounds(y, row, tp, tq, L, U);
                const bool keep = y <= tf && t < row_end && L <= thr;
                if (keep) store_cand(L, U, t);
                const float w = (keep && U < lst[LL - 1]) ? U : INF;
                if constexpr (HALVES) {
                    if (__ballot(w < INF)) {
                        list_insert(w);
                        thr = fminf(thr, fmaxf(lst[LL - 1], partner(lst[LL - 1])));
                    }
                } else {
                    // (no lane inserting means no partner inserting: the swap waits for one)
                    if (__ballot(w < INF)) {
                        const float wp = partner(w);  // the other half's candidate
                        list_insert(w);
                        list_insert(wp);
                        thr = fminf(thr, lst[LL - 1]);
                    }
                }
            }
            make_tfb();
        }
    };

    // deferred slow path (8-wave shapes): passing values with L <= thr are queued -- (L, U,
    // row) in registers -- and flushed through accept() every DEFER_EVERY tiles by all waves
    // together, or when some lane's queue is full.  A threshold waiting for the flush is
    // stale but still valid (it only ever tightens).
    // the queue is three register vectors read with a wave-uniform index (v_movrels), so
    // the flush is a runtime loop with one copy of accept()
    bool dirty = false;  // this wave issued vector-memory ops after the newest DMA
    constexpr int RQ = KNN_FUSED_RQ;
    static_assert(RQ == 2 || RQ == 4 || RQ == 8, "queue depth");
    typedef float qvecf __attribute__((ext_vector_type(RQ)));
    typedef int qveci __attribute__((ext_vector_type(RQ)));
    qvecf qL = qvecf{}, qU = qvecf{};
    qveci qT = qveci{};
    int qcnt = 0;
    auto flush = [&]() __attribute__((always_inline)) {
#ifdef KNN_FILTER_TIMING
        const unsigned long long tf0 = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll 1
        for (int hh = 0; hh < 2; hh++) {
#pragma unroll 1
            for (int i = 0; i < RQ; i++) {
                const bool mine = h == hh && i < qcnt;
                if (!__ballot(mine)) break;
                if (mine) accept(qL[i], qU[i], (int64_t)qT[i]);
            }
            sync_roots(hh);
        }
        qcnt = 0;
        publish();
#ifdef KNN_FILTER_TIMING
        tph[6] += 1;
        tph[7] += __builtin_amdgcn_s_memtime() - tf0;
#endif
    };
    auto record = [&](floatx16 (&Y)[NACC], int tp, float tf, float2 tq, uint32_t u) {
        const int64_t tbase = row_begin + (int64_t)tp * BN;
        if constexpr (!PSTEP) u = pass_set(Y, tf, u);
#ifdef KNN_FILTER_TIMING
        tph[4] += 1;
        tph[5] += __builtin_popcount(u);
#endif
        while (u) {
            const int v = __builtin_ctz(u);
            u &= u - 1u;
            const float y = yval(Y, v);
            const bool p = y <= tf;
            if (__ballot(p && qcnt >= RQ)) flush();
            const int r = v & 15;
            const int row = 32 * (v >> 4) + (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t t = tbase + row;
            if (p && t < row_end) {
                float L, U;
                bounds(y, row, tp, tq, L, U);
                if (L <= thr) {
#pragma unroll
                    for (int i = 0; i < RQ; i++) {
                        qL[i] = i == qcnt ? L : qL[i];
                        qU[i] = i == qcnt ? U : qU[i];
                        qT[i] = i == qcnt ? (int)t : qT[i];
                    }
                    qcnt++;
                }
            }
        }
    };

    floatx16 accA[NACC], accB[NACC];
#pragma unroll
    for (int c = 0; c < NACC; c++) accA[c] = accB[c] = floatx16{};
    __syncthreads();  // LDS init is complete before any DMA lands
#pragma unroll
    for (int p = 0; p < AHEAD; p++)
        if (p < ntiles) dma_tile(p, p, row_begin + (int64_t)p * BN);
#ifndef KNN_FUSED_EARLY_DMA
#define KNN_FUSED_EARLY_DMA 0
#endif
    // KNN_FUSED_LATE_DMA (study): tiles in groups also issue their DMA after the step
    constexpr bool LATE_DMA = (NBUF == 3 && !KNN_FUSED_EARLY_DMA) || (NBUF >= 4 && KNN_FUSED_LATE_DMA);
    constexpr bool DEFER = NW == 8 && KNN_FUSED_DEFER && !RL;
    constexpr int DEFER_EVERY = KNN_FUSED_DEFER_EVERY;
    // per-64-row maximum train norm of the tile in the pipeline (tile it) and of tile it-1
    const int64_t tile0 = row_begin >> 6;
    float2 tm_prev = make_float2(0.0f, 0.0f);
    float2 tmg[GRP];  // PAIR: the group's tile terms, loaded after its barrier
    auto iter = [&](floatx16 (&X)[NACC], floatx16 (&Y)[NACC], int it) {
        if ((it & (KNN_FUSED_SHARE_EVERY - 1)) == KNN_FUSED_SHARE_EVERY - 1) {
            if (a.nseg > 1 && qvalid) {
                if constexpr (RL) {  // publish this query's bound (the heap path does it per accept)
                    if (h == 0 && thr < published) {
                        atomicMin(&a.gthr[q], f2o(thr));
                        published = thr;
                    }
                }
                // thresholds published by other segments of this query
                const float gv = o2f(__hip_atomic_load(&a.gthr[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (gv < thr) { thr = gv; make_tfb(); }
            }
        }
        KNN_TSTAMP(t0);
        if constexpr (PAIR) {
            // pair (it, it + 1) starts: both tiles have landed (every wave's pieces), and
            // every wave is done with the previous pair's buffers
            if (it % GRP == 0) wait_dma_barrier(0);
        } else {
            const bool keep_next = NBUF == 3 && it + 1 < ntiles && (LATE_DMA || !dirty);
            wait_dma_barrier(keep_next ? n_dma_wave : 0);
        }
        dirty = false;
        // this tile's maximum train norm, for its fast test in the next iteration: issued after
        // the barrier, it lands under this step (the next barrier's wait covers it)
        float2 tm_cur;
        if constexpr (PAIR) {
            // both tiles' maxima after the pair's barrier: no compiler wait on a load issued
            // before the DMA of the second step (it would wait for that DMA too)
            const int gi = it % GRP;
            if (gi == 0) {
#pragma unroll
                for (int g = 0; g < GRP; g++) tmg[g] = tile_q(tile0 + ((min(it + g, ntiles - 1) * BN) >> 6));
            }
            tm_cur = tmg[0];
#pragma unroll
            for (int g = 1; g < GRP; g++) tm_cur = gi == g ? tmg[g] : tm_cur;
        } else {
            tm_cur = tile_q(tile0 + ((it * BN) >> 6));
        }
        KNN_TSTAMP(t1);
#ifndef KNN_ABLATE_NO_DMA
        const bool dma_on = it + AHEAD < ntiles;
#else
        const bool dma_on = false;
#endif
        const DmaTile dd = dma_desc((it + AHEAD) % NBUF, (it + AHEAD) % NR, row_begin + (int64_t)(it + AHEAD) * BN);
        const float tf = it > 0 ? tf_of(tm_prev) : -INF;
        // (measured slower: both tiles of the next pair DMA'd in one burst after the even step,
        // A 28.0 -> 28.5 ms, B 752 -> 802 ms)
        const uint32_t uY = step(X, Y, it % NBUF, dma_on && !LATE_DMA, dd, tf, PAIR && it % GRP != 0);
        // PAIR: the group's next tile is resident since its barrier -- its first fragments
        // are read now, so their latency hides under the slow path below
        if (PAIR && it % GRP != GRP - 1 && it + 1 < ntiles) prefetch((it + 1) % NBUF);
        KNN_TSTAMP(t2);
#ifndef KNN_ABLATE_NO_SLOW
        if (uY) {
            if constexpr (RL) { slow_rl(Y, it - 1, tf, tm_prev, uY); dirty = true; }
            else if constexpr (DEFER) record(Y, it - 1, tf, tm_prev, uY);
            else { slow(Y, it - 1, tf, tm_prev, uY); dirty = true; }
        }
        if constexpr (DEFER) {
            if ((it & (DEFER_EVERY - 1)) == DEFER_EVERY - 1 && __ballot(qcnt > 0)) {
                flush();
                dirty = true;
            }
        }
#else
        asm volatile("" ::"s"(uY));
#endif
        if (LATE_DMA && dma_on) {
#pragma unroll
            for (int i = 0; i < NPIECE; i++) dma_piece(i, dd);
        }
        tm_prev = tm_cur;
#ifdef KNN_FILTER_TIMING
        KNN_TSTAMP(t3);
        tph[0] += t1 - t0; tph[2] += t2 - t1; tph[3] += t3 - t2;
#endif
    };
    for (int it = 0; it < ntiles; it += 2) {
        iter(accA, accB, it);
        if (it + 1 < ntiles) iter(accB, accA, it + 1);
    }
    if (ntiles > 0) {
        // drain: the last tile's accumulators are in accA (ntiles odd) or accB (even)
        const int last = ntiles - 1;
        auto drain = [&](floatx16 (&Lc)[NACC]) {
            KNN_STUDY_STEP_HEAD();
            const float tf = tf_of(tm_prev);
            uint32_t u = pass_set(Lc, tf);
            if (u) {
                if constexpr (!PSTEP) u = 0xffffffffu;  // the slow paths rebuild the set per accumulator
                if constexpr (RL) slow_rl(Lc, last, tf, tm_prev, u);
                else if constexpr (DEFER) record(Lc, last, tf, tm_prev, u);
                else slow(Lc, last, tf, tm_prev, u);
            }
        };
        if (last & 1) drain(accB);
        else drain(accA);
    }
    if constexpr (DEFER) {
        if (__ballot(qcnt > 0)) flush();
    }
    if constexpr (RL) {  // the final bound of this segment, for the other segments' rescore
        if (a.nseg > 1 && qvalid && h == 0 && thr < published) atomicMin(&a.gthr[q], f2o(thr));
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (qvalid) a.cnt[(int64_t)(2 * seg + h) * a.nq + q] = ccnt;
#ifdef KNN_FILTER_TIMING
    if (a.timing && lane == 0) {
        atomicAdd(&a.timing[0], tph[0]);
        atomicAdd(&a.timing[2], tph[2]);
        atomicAdd(&a.timing[3], tph[3]);
        atomicAdd(&a.timing[4], 1ull);
        atomicAdd(&a.timing[6], tph[4]);  // record calls
        atomicAdd(&a.timing[7], tph[5]);  // passing value indices visited
        atomicAdd(&a.timing[8], tph[6]);  // flushes
        atomicAdd(&a.timing[5], tph[7]);  // flush clocks
    }
#endif
#undef KNN_TSTAMP
}

// The grid (knn_fused_schedule): blocks [0, p1) take one whole query tile each (qt = block,
// every train row) -- whole rounds of the resident blocks, all sweeping the train rows from
// row 0 together (one L2 stream per XCD); the remaining query tiles' (qtile, 64-row tile)
// work is one linear space of w2 units cut into g2 equal ranges, one per block [p1, p1+g2):
// a range covers the tail of one query tile and the head of the next (a piece each), so the
// last round of blocks ends together instead of a partial wave of whole query tiles.
// Pieces of one query tile share thresholds through gthr like segments (piece id = block -
// the first block of that query tile).  One call site of fused_piece (instruction cache).
template <int RB, int MINW, int NBUF, int NW, int RG, bool PSTEP, int KR>
__global__ __launch_bounds__(64 * NW, MINW) void k_gemm_fused(GemmFilterArgs a) {
    if ((a.gate && *a.gate == 0) || (*a.status & KNN_STATUS_GEMM_UNSAFE)) return;  // not taken / exact path
    const int64_t T = a.tiles64;  // 64-row units per query tile
    const int b = blockIdx.x;
    // g2 < 0: segment mode -- block = (segment b / n_qtiles, query tile b % n_qtiles), one piece
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
            const int64_t ql = x / T, t0 = x - ql * T;
            const int64_t t1 = min(T, t0 + (x1 - x));
            qt = qbase + (int)ql;
            // the block whose range holds the query tile's first unit: largest bb with lo(bb) <= ql T
            seg = p1 ? 0 : (int)(b2 - ((ql * T + 1) * a.g2 - 1) / a.w2);
            rb = t0 * 64;
            re = min(a.nt, t1 * 64);
            adv = t1 - t0;
        }
        if (!first) __syncthreads();  // every wave is done with the previous piece's LDS
        fused_piece<RB, NBUF, NW, RG, PSTEP, KR>(a, qt, seg, rb, re);
        x += adv;
    }
}

// Balanced schedule (see k_gemm_fused): whole rounds of query tiles, the rest cut into g2 equal
// ranges of 64-row units (at least min(T, 256) units each).  Returns the grid and sets *nseg
// to the most pieces one query tile gets (its candidate sub-slices).
int knn_fused_schedule(GemmFilterArgs& a, int slots, int* nseg) {
    const int64_t T = (a.nt + 63) / 64;
    const int64_t nqt = a.n_qtiles;
    a.tiles64 = T;
    const int64_t R = nqt / slots, r = nqt - R * slots;
    a.p1_blocks = (int)(R * slots);
    *nseg = 1;
    if (r == 0) {
        a.g2 = 0;  // whole rounds only
        a.w2 = 0;
        return a.p1_blocks;
    }
    const int64_t W = r * T;
    const int64_t minp = std::min<int64_t>(T, 256);
    const int64_t g2 = std::max<int64_t>(1, std::min<int64_t>(slots, W / minp));
    a.g2 = (int)g2;
    a.w2 = W;
    auto blk = [&](int64_t xx) { return ((xx + 1) * g2 - 1) / W; };
    for (int64_t ql = 0; ql < r; ql++) *nseg = std::max<int>(*nseg, (int)(blk((ql + 1) * T - 1) - blk(ql * T) + 1));
    return a.p1_blocks + (int)g2;
}

// ---------------------------------------------------------------------------------
// plan and launch
// ---------------------------------------------------------------------------------
static size_t fused_lds_of(int row_bytes, int k, int nw, int rg, int nbuf, bool heaps) {
    const int bn = 32 * rg, bm = 32 * nw;
    const int ins = (bn * (row_bytes / 16 + 1) + 63) / 64;
    return (size_t)nbuf * ins * 1024 + ((size_t)(nbuf + 1) * bn + (heaps ? (size_t)bm * heap_stride(k) : 0)) * sizeof(float);
}

bool knn_fused_supported(int d) { return d == 64 || d == 128 || d == 256; }

// Shapes (d = features; rows of 2d + 32 bytes):
//  d = 64:   4 waves x 32 queries, 64-row tiles, two blocks per CU (short rows: the per-tile
//            barrier and fast test outweigh 5 MFMAs per 32x32 block; the other block hides them)
//  d >= 128: 8 waves x 32 queries (two waves per SIMD), 64-row tiles, double-buffered; 32-row
//            tiles when the per-query heaps of a large k leave no room for 64-row tiles.
// Thresholds: k <= 16 keeps per-query register lists (KR = 16), k <= 32 per-half lists
// (KR = 32, 16 entries: exact 32-entry lists cost a block per CU of occupancy and 9 % of
// time on B), larger k the LDS heaps.
FilterPlan knn_fused_plan(int d, int k, const FilterStudy* fs) {
    const int rb = 2 * d + 32;
    const size_t cap = 160 * 1024 - 256;  // room for the kernel's static LDS (the start tile)
    // pass-set variant (FilterPlan.qg): the v_min3 chain and a lazy pass set for every d --
    // measured on A (same box, with the rounding certificate): 29.8 (in-step set) -> 28.8 ms
    const int pstep = (d >= 128 && KNN_FUSED_PSTEP) ? 1 : 0;
    int kr = k <= 16 ? 16 : k <= 32 ? 32 : 0;
    if (fs && fs->kr == 0) kr = 0;  // study: the heaps for every k
    auto make = [&](int nw, int rg, int minw, int nbuf) {
        FilterPlan f{nw, pstep, rg, minw, nbuf, 32 * nw, fused_lds_of(rb, k, nw, rg, nbuf, kr == 0)};
        f.kr = kr;
        return f;
    };
    const bool force8 = fs && fs->shape[0] == 'w' && fs->shape[1] == '8';
    // study: 3 buffers or pairs (4); triples (6) measured slower (A 28.0 -> 31.9 ms, B 749 -> 995)
    const int nb = fs && (fs->nbuf == 3 || fs->nbuf == 4) ? fs->nbuf : 2;
    const bool force4 = fs && fs->shape[0] == 'w' && fs->shape[1] == '4';
    // d = 64 with register lists: 8-wave blocks in pairs like d >= 128 (B, same box: 765 ms
    // with 4-wave blocks in pairs, 743 with 8-wave) -- 256 queries share each tile's DMA
    if ((d == 64 || force4) && !force8 && kr == 0 && fused_lds_of(rb, k, 4, 2, nb, true) <= cap / 2) return make(4, 2, 2, nb);
    if (force4 && fused_lds_of(rb, k, 4, 2, nb, kr == 0) <= cap / 2) return make(4, 2, 2, nb);
    // d >= 128: tiles in pairs (one barrier per two tiles) when four buffers fit -- measured
    // on A (same box): filter 33.4 -> 31.3 ms; B's d = 64 shape loses occupancy with them
    const bool study_nb = fs && fs->nbuf > 0;
    if (!study_nb && fused_lds_of(rb, k, 8, 2, 4, kr == 0) <= cap) return make(8, 2, 2, 4);
    if (fused_lds_of(rb, k, 8, 2, nb, kr == 0) <= cap) return make(8, 2, 2, nb);
    if (fused_lds_of(rb, k, 8, 1, 2, kr == 0) <= cap) return make(8, 1, 2, 2);
    return FilterPlan{0, 0, 0, 0, 0, 0, 0};  // k too large for the LDS heaps: not supported
}

// FilterPlan.qg carries the pass-set variant of the fused kernel: 1 = built in the step
// (PSTEP: a v_cmp per value between the MFMAs; d >= 128, where the MFMAs hide it), 0 = a
// v_min3 chain in the step and the set built on passing tiles only (d = 64: 10 MFMAs per
// tile leave no room).  Measured on one box: A (d = 128) PSTEP faster, B (d = 64) slower.
template <int RB, bool P, int KR>
static const void* fused_fn_p(const FilterPlan& f) {
#define KNN_FUSED_FN(NB, NW, RG) reinterpret_cast<const void*>(&k_gemm_fused<RB, 2, NB, NW, RG, P, KR>)
    if (f.nw == 4) return f.nbuf == 4 ? KNN_FUSED_FN(4, 4, 2) : f.nbuf == 3 ? KNN_FUSED_FN(3, 4, 2) : KNN_FUSED_FN(2, 4, 2);
    if (f.rg == 2) return f.nbuf == 4 ? KNN_FUSED_FN(4, 8, 2) : f.nbuf == 3 ? KNN_FUSED_FN(3, 8, 2) : KNN_FUSED_FN(2, 8, 2);
    return KNN_FUSED_FN(2, 8, 1);
#undef KNN_FUSED_FN
}
template <int RB, bool P>
static const void* fused_fn_k(const FilterPlan& f) {
    return f.kr == 16 ? fused_fn_p<RB, P, 16>(f) : f.kr == 32 ? fused_fn_p<RB, P, 32>(f) : fused_fn_p<RB, P, 0>(f);
}
template <int RB>
static const void* fused_fn(const FilterPlan& f) {
    return fused_fn_k<RB, (RB >= 288) && KNN_FUSED_PSTEP>(f);  // the pass-set variant (knn_fused_plan)
}

static const void* fused_ptr(int d, const FilterPlan& f) {
    return d == 64 ? fused_fn<160>(f) : d == 128 ? fused_fn<288>(f) : fused_fn<544>(f);
}

hipError_t knn_fused_occupancy(int d, int k, int* blocks_per_cu, const FilterStudy* fs) {
    const FilterPlan f = knn_fused_plan(d, k, fs);
    if (!knn_fused_supported(d) || f.nw == 0) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fused_ptr(d, f), 64 * f.nw, f.lds);
}

hipError_t knn_launch_fused(const GemmFilterArgs& a, hipStream_t st, const FilterStudy* fs) {
    const FilterPlan f = knn_fused_plan(a.d, a.k, fs);
    if (!knn_fused_supported(a.d) || f.nw == 0 || a.ld_t != a.d + 16 || a.ld_q != a.d + 16 || !a.tstat || !a.qstat)
        return hipErrorInvalidValue;
    void* args[] = {const_cast<GemmFilterArgs*>(&a)};
    const dim3 grid((unsigned)(a.g2 < 0 ? (int64_t)a.n_qtiles * a.nseg : (int64_t)a.p1_blocks + a.g2));
    hipError_t e = hipLaunchKernel(fused_ptr(a.d, f), grid, dim3(64 * f.nw), args, f.lds, st);
    if (e != hipSuccess) return e;
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}
