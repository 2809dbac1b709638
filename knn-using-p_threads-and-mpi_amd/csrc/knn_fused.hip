// knn_fused.hip -- the GEMM-form candidate filter on the bf16 MFMA with the train norm
// folded into the MFMA (gfx950).  DESIGN.md "k_gemm_fused".
//
// Train operand: tile blocks (k_tn_rows), one per tile of bn rows,
//   [ bn rows x d bf16 rn(t) | bn fp32 norms tn = ||t||^2 | {max tn, max |t - rt|, max |rt|, 0} ]
// -- exactly the bytes one tile's LDS-DMA copies.  Query operand: [nq][d] bf16 rn(-2 q).
// Each accumulator starts from its rows' norms (the first MFMA's C operand), so one chain of
// v_mfma_f32_32x32x16_bf16 over d/16 k-steps leaves
//   y = tn - 2 rn(q).rn(t)
// in the accumulators: the fast test is a v_min3 chain over the 16 values of an
// accumulator against one per-(query, tile) threshold, with no per-value norm read or
// fma; the slow path takes each lane's passing values, computes the certificate bounds
//   G = qn + y,  Delta = coef (qn + tmax_tile) + eta + rho,  L = G - Delta <= D <= U = G + Delta
// (D: the reference's direct-form distance, main.cpp:14-23) and keeps (row, L, U) for
// the exact rescore (k_rescore).  (The KNN_STUDY_AUG64 build keeps the round-2 layout at
// d = 64: rows augmented by 16 bf16 columns carrying the norm split, k_aug_rows.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "knn_device.h"
#include "knn_kernels.h"
#include "knn_study.h"

// Constants of the filter (each measured against its alternatives; DESIGN.md "Filter studies")
#ifndef KNN_STUDY_PF
static constexpr int FUSED_PF = 6;            // A-fragment prefetch depth, in MFMAs
#else
static constexpr int FUSED_PF = KNN_STUDY_PF;  // (study builds pf4 / pf8)
#endif
static constexpr int FUSED_DEFER_EVERY = 64;  // 8-wave heap shapes: tiles between flushes of the queued values
static constexpr int FUSED_SHARE_EVERY = 64;  // tiles between threshold exchanges of a query's pieces (gthr)
static constexpr int FUSED_RQ = 4;            // queued passing values per lane (heap shapes)
#ifndef KNN_FUSED_LIST_SHARE
#define KNN_FUSED_LIST_SHARE 1                // pieces exchange threshold lists (a.lshare; QG = 1)
#endif
#ifndef KNN_FUSED_FORWARD
#define KNN_FUSED_FORWARD 0                   // balanced ranges in range order (study; default: from the end)
#endif
#ifndef KNN_FUSED_LIST_FIRST
#define KNN_FUSED_LIST_FIRST 31               // first list exchange after this tile (then doubling)
#endif
#ifndef KNN_FUSED_TF_GLOBAL
#define KNN_FUSED_TF_GLOBAL 1                 // fast-test tile term from the maxima over all tiles (a.tsmax)
#endif
#ifndef KNN_FUSED_IDLE_SKIP
#define KNN_FUSED_IDLE_SKIP 1                 // a wave with no valid query issues its tile DMAs and barriers only
#endif
#ifndef KNN_FUSED_DMA_FRONT
#define KNN_FUSED_DMA_FRONT 0                 // (study) a group's tile DMAs all issued right after its barrier
#endif
#ifndef KNN_FUSED_LIST_EVERY
#define KNN_FUSED_LIST_EVERY (1 << 30)        // list exchanges: tiles 32, 64, 128, ... (+ every this many)
#endif

// ---------------------------------------------------------------------------------
// k_aug_rows<E>: rows of the fused filter, [n][d + 16] bf16.  Element c < d is
// rn(scale * x[r][c]) (scale = 1: train, -2: queries; exact scaling by a power of two);
// the augmented block is the three-term bf16 split of norms[r] (train: tn = hi + mid +
// lo + r, |r| <= 2^-24 tn, each subtraction exact by Sterbenz) or (1, 1, 1) (queries,
// norms == NULL), then zeros.  One thread per 4 elements: a float4 (or 4 bf16) in, one
// 8-byte bf16 quad out.
// ---------------------------------------------------------------------------------
// bf16 bits of the smallest bf16 >= x (x >= 0 finite): an upper bound stays one
__device__ __forceinline__ uint32_t bf16_up(float x) {
    const uint32_t b = __float_as_uint(x);
    return (b >> 16) + ((b & 0xffffu) ? 1u : 0u);
}

template <typename E>
__global__ __launch_bounds__(256) void k_aug_rows(const E* __restrict__ x, int64_t n, int64_t n_valid, int ld,
                                                  int d, const float* __restrict__ norms, float scale,
                                                  bf16_t* __restrict__ out, const float4* __restrict__ tstat,
                                                  const int32_t* __restrict__ gate) {
    if (gate && *gate == 0) return;
    const int per_row = (d + 16) >> 2;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n * per_row; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / per_row;
    const int c = (int)(i - r * per_row) * 4;
    uint32_t w0 = 0u, w1 = 0u;
    if (c == d + 8 && tstat && (r & 31) == 0 && (r >> 6) < (n_valid + 63) >> 6) {
        // the 64-row tile's statistics (k_row_norms, over its valid rows), rounded up
        const float4 t = tstat[r >> 6];
        w0 = bf16_up(t.x) | (bf16_up(t.y) << 16);
        w1 = bf16_up(t.z);
    } else if (r >= n_valid) {
        // pad rows up to the 64-row tile grid (train only): zero features and tn_hi = 0x1.fep127,
        // so y = tn - 2 q.t ~ 1.7e38 never passes a fast test; their indices are past row_end
        if (c == d && norms) w0 = 0x7f7fu;
    } else if (c < d) {
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
}

hipError_t knn_launch_aug_rows(const void* x, int elem, int64_t n, int64_t n_valid, int ld, int d, const float* norms,
                               float scale, uint16_t* out, const float4* tstat, hipStream_t st, const int32_t* gate) {
    const int64_t total = n * ((d + 16) / 4);
    if (total <= 0) return hipSuccess;
    if (d % 4 || ld % 4) return hipErrorInvalidValue;
    const dim3 grid(gated_grid(elementwise_grid(total), gate));
    if (elem == ELEM_BF16)
        hipLaunchKernelGGL(k_aug_rows<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, n, n_valid, ld, d, norms, scale,
                           (bf16_t*)out, tstat, gate);
    else
        hipLaunchKernelGGL(k_aug_rows<float>, grid, dim3(256), 0, st, (const float*)x, n, n_valid, ld, d, norms, scale,
                           (bf16_t*)out, tstat, gate);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

// ---------------------------------------------------------------------------------
// k_tn_rows<E>: operand rows of the filter (no augmented columns).
//   queries (norms == NULL): [n][d] bf16 = rn(scale * x)
//   train: blocks of bn rows, [bn][d] bf16 = rn(x) | bn fp32 norms | {max tn, max |t - rt|,
//   max |rt|, 0} of the enclosing 64-row tile (k_row_norms) -- the image one tile's LDS-DMA
//   copies, header included.  Rows n_valid .. n-1 (padding past the tile grid): zero features
//   and norm 0x1.fep127, so y = tn - 2 q.t never passes a fast test.  n % bn == 0.
// ---------------------------------------------------------------------------------
template <typename E>
__global__ __launch_bounds__(256) void k_tn_rows(const E* __restrict__ x, int64_t n, int64_t n_valid, int ld, int d,
                                                 const float* __restrict__ norms, float scale,
                                                 unsigned char* __restrict__ out, const float4* __restrict__ tstat,
                                                 int bn, const int32_t* __restrict__ gate) {
    if (gate && *gate == 0) return;
    const int per_row = d >> 2;
    auto quad = [&](int64_t r, int c) -> uint2 {
        if (r >= n_valid) return make_uint2(0u, 0u);
        const float4 v = load4(x + r * ld + c);
        return make_uint2(bf16_rne(scale * v.x) | (bf16_rne(scale * v.y) << 16),
                          bf16_rne(scale * v.z) | (bf16_rne(scale * v.w) << 16));
    };
    if (!norms) {
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n * per_row; i += (int64_t)gridDim.x * 256) {
            const int64_t r = i / per_row;
            const int c = (int)(i - r * per_row) * 4;
            *reinterpret_cast<uint2*>(out + (r * d + c) * 2) = quad(r, c);
        }
        return;
    }
    const int64_t per_tile = (int64_t)bn * per_row + bn + 1;
    const int64_t tb = (int64_t)bn * d * 2 + 4 * bn + 16;
    const int64_t nvt = (n_valid + 63) >> 6;  // 64-row tiles with statistics
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < (n / bn) * per_tile; i += (int64_t)gridDim.x * 256) {
        const int64_t T = i / per_tile;
        const int64_t l = i - T * per_tile;
        const int64_t r0 = T * bn;
        unsigned char* blk = out + T * tb;
        if (l < (int64_t)bn * per_row) {
            const int rr = (int)(l / per_row);
            const int c = (int)(l - (int64_t)rr * per_row) * 4;
            *reinterpret_cast<uint2*>(blk + ((int64_t)rr * d + c) * 2) = quad(r0 + rr, c);
        } else if (l < (int64_t)bn * per_row + bn) {
            const int rr = (int)(l - (int64_t)bn * per_row);
            const int64_t r = r0 + rr;
            *reinterpret_cast<float*>(blk + (int64_t)bn * d * 2 + 4 * rr) = r < n_valid ? norms[r] : 0x1.fep127f;
        } else {
            const int64_t t64 = r0 >> 6;
            *reinterpret_cast<float4*>(blk + (int64_t)bn * d * 2 + 4 * bn) =
                t64 < nvt ? tstat[t64] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
    }
}

hipError_t knn_launch_tn_rows(const void* x, int elem, int64_t n, int64_t n_valid, int ld, int d, const float* norms,
                              float scale, void* out, const float4* tstat, int bn, hipStream_t st,
                              const int32_t* gate) {
    if (n <= 0) return hipSuccess;
    if (d % 4 || ld % 4 || (norms && (bn <= 0 || n % bn))) return hipErrorInvalidValue;
    const int64_t total = norms ? (n / bn) * ((int64_t)bn * (d / 4) + bn + 1) : n * (d / 4);
    const dim3 grid(gated_grid(elementwise_grid(total), gate));
    if (elem == ELEM_BF16)
        hipLaunchKernelGGL(k_tn_rows<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, n, n_valid, ld, d, norms, scale,
                           (unsigned char*)out, tstat, bn, gate);
    else
        hipLaunchKernelGGL(k_tn_rows<float>, grid, dim3(256), 0, st, (const float*)x, n, n_valid, ld, d, norms, scale,
                           (unsigned char*)out, tstat, bn, gate);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

// ---------------------------------------------------------------------------------
// k_tile_stat_max: out = {max tn, max |t - rt|, max |rt|, 0} over the n 64-row tile statistics
// (k_row_norms' tstat): the fused filter's fast-test tile term (a.tsmax).  One block.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tile_stat_max(const float4* __restrict__ t, int64_t n, float4* __restrict__ out) {
    __shared__ float4 part[4];
    float4 m = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // (the statistics are >= 0)
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        const float4 v = t[i];
        m.x = fmaxf(m.x, v.x); m.y = fmaxf(m.y, v.y); m.z = fmaxf(m.z, v.z);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        m.x = fmaxf(m.x, __shfl_xor(m.x, o)); m.y = fmaxf(m.y, __shfl_xor(m.y, o)); m.z = fmaxf(m.z, __shfl_xor(m.z, o));
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float4 r = part[0];
        for (int w = 1; w < 4; w++) { r.x = fmaxf(r.x, part[w].x); r.y = fmaxf(r.y, part[w].y); r.z = fmaxf(r.z, part[w].z); }
        *out = r;
    }
}

hipError_t knn_launch_tile_stat_max(const float4* tstat, int64_t n, float4* out, hipStream_t st) {
    if (n <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_tile_stat_max, dim3(1), dim3(256), 0, st, tstat, n, out);
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
#if KNN_FUSED_STAMPS
// per-wave sums over the launch: barrier wait, step, slow path, piece cycles, tiles with a
// slow path, tiles, pieces (read by knn_debug_stamps; study build only)
__device__ unsigned long long g_knn_stamps[8];
extern "C" int knn_debug_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_knn_stamps), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_knn_stamps), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

template <int RB, int NBUF, int NW, int QG, int RG, int KR>
__device__ __forceinline__ void fused_piece(const GemmFilterArgs& a, const int qt, const int seg,
                                            const int64_t row_begin, const int64_t row_end) {
    // TN (RB = 2d, the product): train tiles carry their rows' norms in a header, and each
    // accumulator starts from them (the MFMA's C operand) -- no augmented k-step.  Otherwise
    // (RB = 2d + 32, the KNN_STUDY_AUG64 build at d = 64) the norm rides in 16 augmented columns
    // (one more k-step).
    constexpr bool TN = RB % 64 == 0;
    constexpr int BN_ = 32 * RG;
    constexpr int HS = TN ? BN_ / 4 + 1 : 0;  // header slots: BN fp32 norms + the statistics
    // QG 32-query groups per wave (QG = 2: 64 queries per wave on 32-row tiles, the register-list
    // shapes only): accumulator c holds row group c % RG against query group c / RG, so each A
    // fragment read from LDS feeds QG MFMAs and each tile copy serves 32 QG NW queries
    typedef FilterTile<RB, NW, QG, RG, HS> FT;
    constexpr int NACC = FT::NACC, BN = FT::BN, BM = FT::BM, STRIDE = FT::STRIDE, SLOTS = FT::SLOTS;
    constexpr int DMA_INS = FT::DMA_INS, TILE = FT::TILE, HDR = FT::HDR;
    // bytes of one tile in the train operand (TN: a block of rows + header; else rows of pitch RB)
    constexpr int64_t TB = (int64_t)BN * RB + 16 * HS;
    constexpr int NT = 64 * NW;
    constexpr int DMA_PER_WAVE = (DMA_INS + NW - 1) / NW;
    constexpr int NS = RB / 32;                  // k-steps: d/16 feature steps (+ the norm step)
    constexpr int VPS = (16 + NS - 1) / NS;      // fast-test values per k-step per accumulator
    static_assert(NBUF == 2 || NBUF == 4 || NBUF == 8 || NBUF == 16, "tile buffers: two, four (pairs), eight (quads), 16 (octets)");
    // NBUF = 4: tiles go in pairs -- one barrier per pair; the DMA of tile it + 2 is issued
    // during step it into the buffer tile it - 2 used (read before this pair's barrier)
    // NBUF = 8: quads -- one barrier per four tiles; NBUF = 16: octets (the QG = 2 default,
    // knn_fused_plan: eight 32-row tiles per barrier; the code of eight static tile places is
    // ~50 KB)
    constexpr int GRP = NBUF >= 4 ? NBUF / 2 : 1;  // tiles per barrier
    constexpr bool PAIR = GRP > 1;
    constexpr int AHEAD = PAIR ? GRP : NBUF - 1;  // tiles between a step and the tile it DMAs
    static_assert(RG == 1 || RG == 2, "row groups");
    static_assert(KR == 0 || KR == 8 || KR == 32 || KR == 104, "register lists: k <= 16, 32, 104, or LDS heaps");
    constexpr bool RL = KR > 0;                   // thresholds from per-lane register lists (else LDS heaps)
    // (QG = 2 on 64-row tiles, four accumulators, was tried at d = 64: 1.5 KB of scratch spills)
    static_assert(QG == 1 || (QG == 2 && RG == 1 && RL), "64-query waves: 32-row tiles, register lists");
    constexpr int LL = KR == 104 ? 52 : KR == 8 ? 8 : 16;  // register list length (one per lane half)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* tiles = smem;                                     // [NBUF][TILE]
    const int hs = heap_stride(a.k);
    float* topU = reinterpret_cast<float*>(smem + NBUF * TILE);      // [BM][hs] max-heaps of U
    const int cap_sub = a.cap_seg / 2;  // candidate sub-slice of one lane half (h) of a query

    const int lane = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = lane & 31;
    const int h = lane >> 5;
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

    // this lane's queries, one per query group g (both lane halves hold the same queries,
    // different rows): query jl[g] of the block
    int jl[QG];
    int64_t q[QG];
    bool qvalid[QG];
    uint4 qf[QG][NS];
    float qn[QG], thr[QG], published[QG];
    int ccnt[QG];  // candidates this lane half kept, per query
#pragma unroll
    for (int g = 0; g < QG; g++) {
        jl[g] = (wave * QG + g) * 32 + j;
        q[g] = (int64_t)qt * BM + jl[g];
        qvalid[g] = q[g] < a.nq;
        const unsigned char* qrow = reinterpret_cast<const unsigned char*>(a.test) +
                                    (qvalid[g] ? q[g] : 0) * (int64_t)a.ld_q * 2;
#pragma unroll
        for (int s = 0; s < NS; s++)
            qf[g][s] = qvalid[g] ? *reinterpret_cast<const uint4*>(qrow + 32 * s + 16 * h)
                                 : make_uint4(0u, 0u, 0u, 0u);
        qn[g] = qvalid[g] ? a.qnorm[q[g]] : 0.0f;
        thr[g] = qvalid[g] ? o2f(a.gthr[q[g]]) : -INF;
        published[g] = thr[g];
        ccnt[g] = 0;
    }
    // a wave whose queries all lie past nq (the last query tile; a few-query call's seven other
    // waves) keeps the block's tile DMAs and barriers but runs no MFMAs or tests, so its SIMD
    // partner has the matrix pipe to itself
    bool any_q = false;
#pragma unroll
    for (int g = 0; g < QG; g++) any_q = any_q || qvalid[g];
    const bool wave_live = !KNN_FUSED_IDLE_SKIP || KNN_FUSED_DMA_FRONT || __ballot(any_q) != 0ull;
    float root = INF;  // (heap shapes, QG = 1) this query's heap root, mirrored in both lanes
    float qe2[QG], eq2[QG];  // 2 |q| and 2 |q - rq|, rounded up
#pragma unroll
    for (int g = 0; g < QG; g++) {
        qe2[g] = eq2[g] = 0.0f;
        if (qvalid[g]) {
            const float2 qs = a.qstat[q[g]];
            qe2[g] = 2.0f * qs.x * (1.0f + 0x1p-17f);
            eq2[g] = 2.0f * qs.y * (1.0f + 0x1p-17f);
        }
    }
    // Fast-test tile term (round 6, TFG): from the maxima over ALL tiles of the tile statistics
    // (a.tsmax = {max tn, max |t - rt|, max |rt|} over the train set's 64-row tiles) instead of
    // each tile's own: one threshold tfc per query group, rebuilt only when the threshold moves
    // (make_tfb) -- no header read and two FMAs per group and tile.  The maxima bound every
    // tile's, so the test passes a superset of what the per-tile test passed (the 2^-18 slack
    // covers the reordered additions); the slow path still bounds L, U with the tile's own
    // statistics, read when it runs (the tile's buffer is not rewritten before the next group's
    // DMA: PAIR shapes, AHEAD = GRP).  On uniform rows the tile maxima vary by a few 1e-4 of the
    // band.  KNN_FUSED_TF_GLOBAL=0: the per-tile term (round 5).
    constexpr bool TFG = KNN_FUSED_TF_GLOBAL && PAIR && TN;
    float tk[QG], tfc[QG];  // (TFG) the tile term and the fast-test threshold, per query group
    if constexpr (TFG) {
        const float4 smax = *a.tsmax;
#pragma unroll
        for (int g = 0; g < QG; g++) tk[g] = fmaf(coef + 0x1p-18f, smax.x, fmaf(qe2[g], smax.y, eq2[g] * smax.z));
    }
    float tfb[QG];     // tf without the tile term
    auto make_tfb = [&](int g) __attribute__((always_inline)) {
        tfb[g] = qvalid[g] ? ((thr[g] - qn[g]) + fmaf(coef, qn[g], eta)) + 0x1p-18f * (fabsf(thr[g]) + qn[g]) : -INF;
        if constexpr (TFG) tfc[g] = tfb[g] + tk[g];
    };
#pragma unroll
    for (int g = 0; g < QG; g++) make_tfb(g);
    // tile term: tq = {the tile's maximum norm tmax, the operand-rounding bound of this query
    // against the tile's rows, 2 (|q| max|t - rt| + |q - rq| max|rt|) (1 + 2^-17)}
    auto tf_of = [&](int g, float2 tq) __attribute__((always_inline)) {
        return fmaf(coef + 0x1p-18f, tq.x, tfb[g]) + tq.y;
    };
    // the tile's statistics, from its LDS image (TN: the header's last slot, fp32; the
    // KNN_STUDY_AUG64 layout: augmented columns d+8..d+10 of row 0, bf16): one broadcast read,
    // in order with the fragment reads -- no scalar memory load in the loop
    struct TQ { float2 v[QG]; };
    auto tile_q = [&](int buf) __attribute__((always_inline)) -> TQ {
        float tx, ty, tz;
        if constexpr (TN) {
            const float4 w = *reinterpret_cast<const float4*>(tiles + buf * TILE + HDR + 4 * BN);
            tx = w.x; ty = w.y; tz = w.z;
        } else {
            const uint2 w = *reinterpret_cast<const uint2*>(tiles + buf * TILE + (RB - 16));
            tx = __uint_as_float(w.x << 16); ty = __uint_as_float(w.x & 0xffff0000u);
            tz = __uint_as_float(w.y << 16);
        }
        TQ r;
#pragma unroll
        for (int g = 0; g < QG; g++) r.v[g] = make_float2(tx, fmaf(qe2[g], ty, eq2[g] * tz));
        return r;
    };

    // tiles of the piece, rounded up to an even count: the scan loop below runs tiles in twos
    // with no exit between them, so only accB is live out of it (with an odd tail the compiler
    // copies both accumulator sets -- 32 v_mov -- at every back edge).  The extra tile reads the
    // next BN rows (another piece's, or the padding the train tile blocks carry past the
    // 64-row grid, run_gemm), which the row_end test rejects.
    // (quads / octets: a multiple of four / eight -- the loop runs whole groups, so every tile's
    // place in its group is a compile-time constant; up to 7 extra 32-row tiles, within the 256
    // pad rows past the train grid, run_gemm)
    constexpr int TSTEP = GRP > 2 ? GRP : 2;
    const int ntiles = (row_end > row_begin) ? ((int)((row_end - row_begin + BN - 1) / BN) + TSTEP - 1) / TSTEP * TSTEP : 0;
    // Scan order (a.cursor set: the host does so for the multi-segment schedule): the piece's
    // tiles rotated to start where this XCD's other blocks are (per XCD: the 64-row unit the last
    // block to publish was at, if inside this piece) -- so the blocks one XCD runs at once
    // stream the same rows through its L2 instead of drifting apart (blocks are dispatched to
    // the XCDs round-robin).  Correctness does not depend on the order: every tile is scanned
    // once and the threshold logic is order-free.
    // All waves of the block must use the same order (they DMA pieces of the same tiles): thread
    // 0 reads the cursor and hands the rotation to the others through LDS (blk_rot, written
    // before the block barrier below, read after it).
    const int xcd = blockIdx.x & 7;
    int* blk_rot = reinterpret_cast<int*>(smem + NBUF * TILE + (RL ? 0 : BM * hs * (int)sizeof(float)));
    if (threadIdx.x == 0) {
        int r0 = 0;
        if (a.cursor && ntiles > 0) {
            const int64_t cu =
                (int64_t)__hip_atomic_load(&a.cursor[xcd], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 64;
            if (cu > row_begin && cu < row_end) r0 = (int)((cu - row_begin) / BN);
        }
        *blk_rot = r0;
    }
    int rot = 0;  // (set after the barrier)
    // the first row of logical tile t (t < ntiles): physical tile (t + rot) mod ntiles
    auto tile_row = [&](int t) __attribute__((always_inline)) -> int64_t {
        int pt = t + rot;
        pt = pt >= ntiles ? pt - ntiles : pt;
        return row_begin + (int64_t)pt * BN;
    };

    // ---- LDS-DMA of tiles (same image as k_gemm_filter: slot P -> row P / SLOTS, slot P % SLOTS,
    // the pad slot duplicates slot 0; rows past row_end are read (padding or the next piece's
    // rows) and rejected by index).  Every tile is whole: the train tile blocks are padded to
    // the 64-row grid (run_gemm), so a piece is always the scalar tile base + this lane's fixed
    // offset -- no per-tile address arithmetic in VGPRs.
    // (piece ins = wave + NW i; rotating the DMA_INS % NW remainder pieces between even and odd
    // tiles, so no wave issues two more per pair than another, measured no faster: r03r)
    uint32_t doff[DMA_PER_WAVE];
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; i++) {
        const int P = (wave + NW * i) * 64 + lane;
        if (TN && P >= BN * SLOTS) {  // header slot: norms, then the statistics
            doff[i] = (uint32_t)(BN * RB + 16 * min(P - BN * SLOTS, HS - 1));
        } else {
            const int row = min(P / SLOTS, BN - 1), sl = P % SLOTS;
            doff[i] = (uint32_t)(row * ldb + 16 * (sl == SLOTS - 1 ? 0 : sl));
        }
    }
    const uint32_t lds_tiles = __builtin_amdgcn_readfirstlane(lds_addr(tiles));
    struct DmaTile { const unsigned char* src; uint32_t lds; };
    // the source of a tile: its block in the train operand (the piece's first row is a multiple
    // of 64, BN divides 64)
    const int64_t TBR = TN ? TB : (int64_t)BN * ldb;  // operand bytes per tile
    const unsigned char* piece_src = trainb + (row_begin / BN) * TBR;
    auto dma_desc = [&](int buf, int t) -> DmaTile {  // logical tile t of the piece
        int pt = t + rot;
        pt = pt >= ntiles ? pt - ntiles : pt;
        return DmaTile{piece_src + (int64_t)pt * TBR, lds_tiles + (uint32_t)(buf * TILE)};
    };
    // The last piece of a tile is issued whole: its lanes past the header re-read the header's
    // last slot into the buffer's slack (TILE = DMA_INS KiB), so no piece needs an exec mask.
    auto dma_piece = [&](int i, const DmaTile& d) __attribute__((always_inline)) {
        const int ins = wave + NW * i;
        if (NW * (i + 1) <= DMA_INS || ins < DMA_INS) dma16s(doff[i], d.src, d.lds + (uint32_t)ins * 1024u);
    };
    // piece i goes out in k-step (i NS) / DMA_PER_WAVE of the step
    auto dma_at = [&](int s, bool on, const DmaTile& d) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < DMA_PER_WAVE; i++)
            if (on && (i * NS) / DMA_PER_WAVE == s) dma_piece(i, d);
    };

    // ---- one tile's MFMAs into X; in between, the fast test of the previous tile (Y): a v_min3
    // chain per accumulator; returns bit 16c (x 0xffff) when some lane of accumulator c holds a
    // passing value (the slow path builds the value set, pass_set)
    [[maybe_unused]] floatx16 cnorm;  // (KNN_ABLATE_NO_NORM only)
    if constexpr (KNN_STUDY_NO_NORM) {
#pragma unroll
        for (int r = 0; r < 16; r++) cnorm[r] = (float)a.d * (1.0f / 3.0f);
    }
    constexpr int PF = FUSED_PF / NACC;  // k-steps of A fragments read ahead
    uint4 pa[PF], pb[PF];                // PAIR: the odd step's first fragments, read early
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
                    const float (&tf)[QG], bool pre, float (&mn_out)[NACC]) -> uint32_t {
        const unsigned char* tile = tiles + buf * TILE;
        const unsigned char* a0p = tile + j * STRIDE + 16 * h;
        const unsigned char* a1p = tile + ((RG == 2 ? 32 : 0) + j) * STRIDE + 16 * h;
        // each accumulator's chain starts from its rows' norms: register r of row group rg is row
        // 32 rg + (r & 3) + 8 (r >> 2) + 4h (four broadcast ds_read_b128 per row group; the QG
        // accumulators of a row group share them as the first MFMA's C operand)
        // (the norms land in row group rg's query-group-0 accumulator X[rg]; at k-step 0 the other
        // query groups' MFMAs take them as their C operand first, then X[rg]'s own -- no copy)
        if constexpr (TN && !KNN_STUDY_NO_NORM) {
            const unsigned char* hn = tile + HDR + 4 * (4 * h);
#pragma unroll
            for (int rg = 0; rg < RG; rg++) {
#pragma unroll
                for (int g4 = 0; g4 < 4; g4++) {
                    const float4 v = *reinterpret_cast<const float4*>(hn + 4 * (32 * rg + 8 * g4));
                    X[rg][4 * g4] = v.x;
                    X[rg][4 * g4 + 1] = v.y;
                    X[rg][4 * g4 + 2] = v.z;
                    X[rg][4 * g4 + 3] = v.w;
                }
            }
        } else if constexpr (TN) {
            // (ablation KNN_ABLATE_NO_NORM: every accumulator starts from the mean row norm d/3 of
            // the uniform generator instead of its rows' norms -- no norm reads; results invalid)
#pragma unroll
            for (int rg = 0; rg < RG; rg++) X[rg] = cnorm;
        } else {
#pragma unroll
            for (int rg = 0; rg < RG; rg++) X[rg] = floatx16{};
        }
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
            for (int cc = 0; cc < NACC; cc++) {
                const int c = s == 0 ? NACC - 1 - cc : cc;  // (k-step 0: query group 0 last)
                const int rg = c % RG, g = c / RG;
                const bf16x8 A = __builtin_bit_cast(bf16x8, (RG == 2 && rg) ? xb[s] : xa[s]);
                X[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, __builtin_bit_cast(bf16x8, qf[g][s]),
                                                               s == 0 ? X[rg] : X[c], 0, 0, 0);
                if (!KNN_STUDY_NO_EPI) {
#pragma unroll
                    for (int v = s * VPS; v < (s + 1) * VPS && v < 16; v++) mn[c] = fminf(mn[c], Y[c][v]);
                    // computed here, beside this k-step's MFMAs: without the opaque use the
                    // compiler sinks the whole v_min3 chain into the last k-step, where it
                    // runs exposed after the final MFMA
                    if (s * VPS < 16) asm volatile("" : "+v"(mn[c]));
                }
            }
            KNN_FUSED_KSTEP_ORDER();
        }
        // which accumulators hold a passing value; the slow path builds their value sets
        // (pass_set) -- usually one of the two
        uint32_t u = 0u;
#pragma unroll
        for (int c = 0; c < NACC; c++) u |= __ballot(mn[c] <= tf[c / RG]) != 0ull ? (0xffffu << (16 * c)) : 0u;
#pragma unroll
        for (int c = 0; c < NACC; c++) mn_out[c] = mn[c];
        return u;
    };

    // append candidate (L, U) of global row t to query group g's sub-slice of this lane half
    // (past its capacity: counted only, the rescore then sends the query to the exact scan)
    auto store_cand32 = [&](int g, float L, float U, int32_t t) __attribute__((always_inline)) {
#ifndef KNN_STUDY_NO_STORE
        if (ccnt[g] < cap_sub) {
            const int64_t o = q[g] * (int64_t)a.cap + (int64_t)(2 * seg + h) * cap_sub + ccnt[g];
            a.cand[o] = CandRec{t, L, U};
        }
        ccnt[g]++;
#else  // (ablation build: no candidate stores, nothing counted -- every query takes the exact scan)
        asm volatile("" ::"v"(L), "v"(U), "v"(t));
#endif
    };
    auto store_cand = [&](int g, float L, float U, int64_t t) __attribute__((always_inline)) {
        store_cand32(g, L, U, (int32_t)t);
    };
    // (heap shapes, QG = 1) keep candidate (L, U) of global row t: the exact test against the
    // current threshold, the candidate store into this lane half's sub-slice, and, if U beats
    // the heap root, a sift-down of the query's 4-ary max-heap (node n >= 1 in H[n-1], the root
    // in H[hs-1]: the four children of node i are one aligned 16-byte read at H[4i]).  Only one
    // lane of a query runs it at a time.
    auto accept = [&](float L, float U, int64_t t) __attribute__((always_inline)) {
        if (!(L <= thr[0])) return;
        store_cand(0, L, U, t);
        if (U < root) {
            float* H = topU + jl[0] * hs;
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
            thr[0] = fminf(thr[0], root);
        }
    };
    auto sync_roots = [&](int hh) __attribute__((always_inline)) {
        const float other = __shfl_xor(root, 32);
        if (h != hh) root = other;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    };
    auto publish = [&]() __attribute__((always_inline)) {  // (heap shapes)
        if (qvalid[0]) {
            thr[0] = fminf(thr[0], root);
            if (a.nseg > 1 && h == 0 && thr[0] < published[0]) {
                atomicMin(&a.gthr[q[0]], f2o(thr[0]));
                published[0] = thr[0];
            }
            make_tfb(0);
        }
    };
    // certified bounds L <= D <= U of value y of query group g against tile stats tq: Delta =
    // coef (qn + tmax) + eta + rho -- the tile's maximum norm tmax >= the row's norm, a slightly
    // wider band (still L <= D <= U) for no per-value norm read
    auto bounds = [&](int g, float y, float2 tq, float& L, float& U) __attribute__((always_inline)) {
        const float G = qn[g] + y;
        const float dl = fmaf(coef, qn[g] + tq.x, eta) + tq.y;
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
    // (heap shapes) the values of Y some lane passes (bit 16c + r), for the accumulators set in
    // acc: per group of 4 values (rows 8g .. 8g+3 of the lane half) one ballot of their minimum,
    // then one v_cmp + ballot per value of the passing groups only
    auto pass_set = [&](floatx16 (&Y)[NACC], float tf, uint32_t acc) __attribute__((always_inline)) -> uint32_t {
        uint32_t u = 0u;
#pragma unroll
        for (int c = 0; c < NACC; c++)
            if ((acc >> (16 * c)) & 1u) {  // (wave-uniform) only the accumulators that pass
#pragma unroll
                for (int g4 = 0; g4 < 4; g4++) {
                    const float gm = fminf(fminf(Y[c][4 * g4], Y[c][4 * g4 + 1]), fminf(Y[c][4 * g4 + 2], Y[c][4 * g4 + 3]));
                    if (__ballot(gm <= tf)) {
#pragma unroll
                        for (int r = 4 * g4; r < 4 * g4 + 4; r++)
                            u |= (__ballot(Y[c][r] <= tf) != 0ull ? 1u : 0u) << (16 * c + r);
                    }
                }
            }
        return u;
    };
    // immediate slow path (4-wave heap shapes): the passing values of tile tp, visited by
    // index; the two lanes of a query take turns (one heap writer at a time)
    auto slow = [&](floatx16 (&Y)[NACC], int tp, float tf, float2 tq, uint32_t u) {
        const int64_t tbase = tile_row(tp);
        u = pass_set(Y, tf, u);
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
                    bounds(0, y, tq, L, U);
                    accept(L, U, t);
                }
                sync_roots(hh);
            }
        }
        publish();
    };

    // register-list slow path (KR > 0): the two lanes of a query (its two row halves) each keep
    // an ascending list lst[] of their own half's ceil(k/2) smallest U (k <= 16: KR = 8, LL = 8;
    // k <= 32: KR = 32, LL = 16; 32 < k <= 104: KR = 104, LL = 52; the first LL - ceil(k/2)
    // entries are -inf pads) and insert only their own values (LL v_med3); the bound is the
    // larger of the two halves' ceil(k/2)-th smallest -- at least 2 ceil(k/2) >= k kept rows
    // have U <= it.  A little looser than the exact k-th smallest, with no LDS heap and no lane
    // taking turns, for all queries of the wave at once.  (Until round 5, k <= 16 kept one exact
    // 16-entry list in both lanes, each inserting both lanes' values: 32 v_med3 and a lane swap
    // per insert; the halves keep ~20 % more candidates and measured A 20.05 -> 19.84 ms, its
    // 8-GPU share 3.05 -> 2.97 ms, same box, r05v.)  (QG = 2: one list per query group.)
    float lst[QG][RL ? LL : 1];
    if constexpr (RL) {
        const int pads = LL - (k + 1) / 2;
#pragma unroll
        for (int g = 0; g < QG; g++)
#pragma unroll
            for (int i = 0; i < LL; i++) lst[g][i] = i < pads ? -INF : INF;
    }
    // min as v_med3 against a -inf the compiler cannot see: with a literal -inf it folds the
    // med3 back into v_min_f32 and canonicalises both inputs (two more v_max per min)
    float ninf_op;
    asm("s_mov_b32 %0, 0xff800000" : "=s"(ninf_op));
    auto fmin_op = [&](float a, float b) __attribute__((always_inline)) {
        return __builtin_amdgcn_fmed3f(a, b, ninf_op);
    };
    auto list_insert = [&](int g, float w) __attribute__((always_inline)) {
#pragma unroll
        for (int i = LL - 1; i >= 1; i--) lst[g][i] = __builtin_amdgcn_fmed3f(lst[g][i - 1], w, lst[g][i]);
        lst[g][0] = fmin_op(lst[g][0], w);
    };
    // the other lane half's copy of a word (v_permlane32_swap: one of the swap's two results
    // is this lane's own word, the other its partner's)
    auto partner = [&](float x) __attribute__((always_inline)) -> float {
        return __uint_as_float(lane_xor(__float_as_uint(x), 32));
    };
    // Lane-parallel slow path.  Passes are sparse (A: a wave-tile has one in about 8 tiles,
    // usually one query, one value), so instead of visiting the passing positions one
    // wave-wide step at a time, every lane takes ITS OWN passing values, one per round, all
    // lanes at once: one scan of the lane's 16 values of a passing accumulator yields its
    // passing set (a 16-bit mask) and the value of the lowest passing index; later rounds take
    // the next set bit; fn(c, idx, y) then handles every lane's candidate together
    // (idx < 0: none).  Rounds = the most passing values of one lane in the accumulator (1
    // unless the threshold is still loose).  Any processing order keeps every true neighbour:
    // a row is kept iff L <= the threshold at its turn, and the threshold is always the k-th
    // smallest U of kept rows.
    auto lane_rounds = [&](floatx16 (&Y)[NACC], const float (&tf)[QG], const float (&mnY)[NACC], uint32_t u,
                           auto&& fn) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < NACC; c++) {
            if (!((u >> (16 * c)) & 1u)) continue;  // (wave-uniform) no lane passes in c
            const float tfc = tf[c / RG];
            // round 1, one scan of the lane's 16 values from r = 15 down to 0: the passing set as
            // a 16-bit mask m = 2m + (y_r <= tf) (v_addc_co_u32 with the compare's VCC as
            // carry-in) and the value of the LOWEST passing index (v_cndmask on the same VCC) --
            // three VALU per value in one asm block (no hazard padding between values), no SGPR
            // mask pairs held.  The lowest passing index is ffs(m) - 1 and "passes twice" is
            // m & (m - 1); later rounds take the next lowest set bit.  Same box (r05n) against the
            // compiler's scan (compare + index, value and count selects: ~4.5 VALU per value):
            // A filter 19.94 -> 19.55 ms, B 465.3 -> 456.7, C1 1683.6 -> 1643.6.
            // (Scanning the highest passing group of four, found by the group minima, measured
            // 4-8 % slower: r03q; the count from the compares' wave masks by scalar ops, 2.7 %
            // slower on B: r03s.)
            uint32_t m = 0u;
            float yv = INF;
            int idx;
            auto pick = [](uint32_t mm) __attribute__((always_inline)) { return __ffs((int)mm) - 1; };  // lowest set bit
            if constexpr (KR <= 32) {
                // k <= 32 (lists of 16): the value is the fast test's minimum -- a lane with ONE
                // passing value passes with its minimum, so the scan only builds the passing mask
                // (compare + add-with-carry, 2 VALU per value); only when some lane passes twice, a
                // second mask of the positions equal to the minimum picks its index.  Same box (r05p):
                // A filter 20.07 -> 19.85 ms, B 466.7 -> 463.3; C1 (k = 100: more lanes pass twice,
                // each paying the second mask) 1677 -> 1687, so KR = 104 keeps the value scan
                asm volatile("v_cmp_le_f32_e32 vcc, %17, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %16, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %15, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %14, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %13, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %12, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %11, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %10, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %9, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %8, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %7, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %6, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %5, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %4, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %3, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %2, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             : "+v"(m)
                             : "v"(tfc), "v"(Y[c][0]), "v"(Y[c][1]), "v"(Y[c][2]), "v"(Y[c][3]), "v"(Y[c][4]), "v"(Y[c][5]), "v"(Y[c][6]), "v"(Y[c][7]), "v"(Y[c][8]), "v"(Y[c][9]), "v"(Y[c][10]), "v"(Y[c][11]), "v"(Y[c][12]), "v"(Y[c][13]), "v"(Y[c][14]), "v"(Y[c][15])
                             : "vcc");
                yv = mnY[c];
                if (__ballot((m & (m - 1u)) != 0u)) {
                    uint32_t e = 0u;
                    asm volatile("v_cmp_eq_f32_e32 vcc, %17, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %16, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %15, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %14, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %13, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %12, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %11, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %10, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %9, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %8, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %7, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %6, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %5, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %4, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %3, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_eq_f32_e32 vcc, %2, %1\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                                 : "+v"(e)
                                 : "v"(yv), "v"(Y[c][0]), "v"(Y[c][1]), "v"(Y[c][2]), "v"(Y[c][3]), "v"(Y[c][4]), "v"(Y[c][5]), "v"(Y[c][6]), "v"(Y[c][7]), "v"(Y[c][8]), "v"(Y[c][9]), "v"(Y[c][10]), "v"(Y[c][11]), "v"(Y[c][12]), "v"(Y[c][13]), "v"(Y[c][14]), "v"(Y[c][15])
                                 : "vcc");
                    idx = pick(m & e);
                } else {
                    idx = pick(m);
                }
            } else {
                asm volatile("v_cmp_le_f32_e32 vcc, %18, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %18, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %17, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %17, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %16, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %16, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %15, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %15, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %14, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %14, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %13, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %13, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %12, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %12, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %11, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %11, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %10, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %10, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %9, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %9, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %8, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %8, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %7, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %7, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %6, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %6, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %5, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %5, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %4, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %4, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             "v_cmp_le_f32_e32 vcc, %3, %2\n\t"
                             "v_cndmask_b32_e32 %1, %1, %3, vcc\n\t"
                             "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
                             : "+v"(m), "+v"(yv)
                             : "v"(tfc), "v"(Y[c][0]), "v"(Y[c][1]), "v"(Y[c][2]), "v"(Y[c][3]), "v"(Y[c][4]), "v"(Y[c][5]), "v"(Y[c][6]), "v"(Y[c][7]), "v"(Y[c][8]), "v"(Y[c][9]), "v"(Y[c][10]), "v"(Y[c][11]), "v"(Y[c][12]), "v"(Y[c][13]), "v"(Y[c][14]), "v"(Y[c][15])
                             : "vcc");
                idx = pick(m);  // -1 when nothing passes
            }
            fn(c, idx, yv);
            if (__ballot((m & (m - 1u)) != 0u)) {
                m = idx >= 0 ? m ^ (1u << idx) : 0u;
#pragma unroll 1
                for (int round = 1; round < 16; round++) {
                    if (!__ballot(m != 0u)) break;
                    idx = pick(m);
                    yv = INF;
                    // the value at idx: compare + select per value in one asm block (the
                    // compiler's form pads each pair with a hazard s_nop)
                    asm volatile("v_cmp_eq_u32_e32 vcc, 0, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %2, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 1, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %3, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 2, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %4, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 3, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %5, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 4, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %6, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 5, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %7, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 6, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %8, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 7, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %9, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 8, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %10, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 9, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %11, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 10, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %12, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 11, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %13, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 12, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %14, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 13, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %15, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 14, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %16, vcc\n\t"
                                 "v_cmp_eq_u32_e32 vcc, 15, %1\n\t"
                                 "v_cndmask_b32_e32 %0, %0, %17, vcc\n\t"
                                 : "+v"(yv)
                                 : "v"(idx), "v"(Y[c][0]), "v"(Y[c][1]), "v"(Y[c][2]), "v"(Y[c][3]), "v"(Y[c][4]), "v"(Y[c][5]), "v"(Y[c][6]), "v"(Y[c][7]), "v"(Y[c][8]), "v"(Y[c][9]), "v"(Y[c][10]), "v"(Y[c][11]), "v"(Y[c][12]), "v"(Y[c][13]), "v"(Y[c][14]), "v"(Y[c][15])
                                 : "vcc");
                    fn(c, idx, yv);
                    m = idx >= 0 ? m ^ (1u << idx) : 0u;
                }
            }
        }
    };
    // a kept row into this lane's list and candidate sub-slice (register lists).  (Round 6: these
    // inserts deferred -- kept rows queued two per lane, flushed for all lanes together every
    // 16 / 64 tiles or when a queue filled -- measured A 19.59 -> 19.98 / 19.65 ms, B 469.8 ->
    // 471.2, A's 8-GPU share equal, same box, r06l: the sparse late visits' cost is the lane
    // scan and its latency, not the insert)
    auto keep_row = [&](int g, bool keep, float L, float U, int64_t t) __attribute__((always_inline)) {
        if constexpr (RL) {
            if (keep) store_cand(g, L, U, t);
            const float w = (keep && U < lst[g][LL - 1]) ? U : INF;
            if (__ballot(w < INF)) {
                list_insert(g, w);
                thr[g] = fmin_op(thr[g], __builtin_amdgcn_fmed3f(lst[g][LL - 1], partner(lst[g][LL - 1]), INF));
            }
        }
    };
    auto slow_rl = [&](floatx16 (&Y)[NACC], int tp, const float (&tf)[QG], const TQ& tq, const float (&mnY)[NACC],
                       uint32_t u) {
        if constexpr (RL) {
            const int64_t tbase = tile_row(tp);
            // (the band's half-width hoisted per tile and 32-bit row compares measured no faster:
            // r05q)
            auto visit = [&](int c, int idx, float yv) __attribute__((always_inline)) {
                const int g = c / RG;
                const int row = 32 * (c % RG) + (idx & 3) + 8 * (idx >> 2) + 4 * h;
                const int64_t t = tbase + row;
                float L, U;
                bounds(g, yv, tq.v[g], L, U);
                keep_row(g, idx >= 0 && t < row_end && L <= thr[g], L, U, t);
            };
            lane_rounds(Y, tf, mnY, u, visit);
#pragma unroll
            for (int g = 0; g < QG; g++) make_tfb(g);
        }
    };

    // deferred slow path (8-wave heap shapes): passing values with L <= thr are queued -- (L,
    // U, row) in registers -- and flushed through accept() every FUSED_DEFER_EVERY tiles by all
    // waves together, or when some lane's queue is full.  A threshold waiting for the flush is
    // stale but still valid (it only ever tightens).  The queue is three register vectors read
    // with a wave-uniform index (v_movrels), so the flush is a runtime loop with one copy of
    // accept()
    constexpr int RQ = FUSED_RQ;
    typedef float qvecf __attribute__((ext_vector_type(RQ)));
    typedef int qveci __attribute__((ext_vector_type(RQ)));
    qvecf qL = qvecf{}, qU = qvecf{};
    qveci qT = qveci{};
    int qcnt = 0;
    auto flush = [&]() __attribute__((always_inline)) {
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
    };
    // (the heap shapes visit the passing positions wave-wide: per value only a queue append,
    // so the lane-parallel scan would cost more than it saves -- C1 259.8 vs 273.3 ms, r03p)
    auto record = [&](floatx16 (&Y)[NACC], int tp, float tf, float2 tq, uint32_t u) {
        const int64_t tbase = tile_row(tp);
        u = pass_set(Y, tf, u);
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
                bounds(0, y, tq, L, U);
                if (L <= thr[0]) {
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
    __syncthreads();  // LDS init is complete before any DMA lands; blk_rot is written
    rot = __builtin_amdgcn_readfirstlane(*blk_rot);
#pragma unroll
    for (int p = 0; p < AHEAD; p++)
        if (p < ntiles) {
            const DmaTile d0 = dma_desc(p, p);
#pragma unroll
            for (int i = 0; i < DMA_PER_WAVE; i++) dma_piece(i, d0);
        }
    constexpr bool DEFER = NW == 8 && !RL;
    // tile terms (max norm, rounding bound) of the tile in the pipeline (it) and of tile it-1
    TQ tm_prev;
#pragma unroll
    for (int g = 0; g < QG; g++) tm_prev.v[g] = make_float2(0.0f, 0.0f);
    // study build KNN_STUDY_STAMPS: shader-clock stamps per wave (barrier wait, step, slow path)
    [[maybe_unused]] uint64_t st_bar = 0, st_step = 0, st_slow = 0, st_visits = 0;
    [[maybe_unused]] const uint64_t st_start = KNN_FUSED_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    auto now = [&]() __attribute__((always_inline)) -> uint64_t {
        return KNN_FUSED_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    };
    // threshold exchanges between the pieces of a query (gthr): every FUSED_SHARE_EVERY tiles
    // (also after tiles 2, 4, ..., 32 measured no fewer kept rows and B 3 % slower: r04d)
    auto share_now = [&](int it) __attribute__((always_inline)) {
        return (it & (FUSED_SHARE_EVERY - 1)) == FUSED_SHARE_EVERY - 1;
    };
    // List exchange between the pieces of a query (register-list shapes, a.lshare): a piece's
    // own list holds the k smallest U of ITS rows only, so the k-th value other pieces publish
    // through gthr is the k-th best of 1/P of the rows -- with P pieces the threshold trails a
    // single scan's by a factor P in rank (A's 8-GPU share, P ~ 5: 599 kept rows per query
    // against 172).  At tiles 32, 64, 128, ... each piece publishes its list (pads as +inf) and
    // takes the k-th smallest U of the union of every piece's list: a valid bound, as the
    // pieces' rows are disjoint and every published value is the U of a kept row.  Any value
    // read may be stale or from a list being rewritten: a list only ever lowers its entries
    // position by position, so a stale mix counts no more rows below a bound than the current
    // list holds (a looser bound, never a wrong one).  Per lane half (its rows), the
    // bound the larger of the two halves' union values.
    auto list_share_now = [&](int it) __attribute__((always_inline)) {
        return (it >= KNN_FUSED_LIST_FIRST && ((it + 1) & it) == 0) || (it & (KNN_FUSED_LIST_EVERY - 1)) == KNN_FUSED_LIST_EVERY - 1;
    };
    auto exchange_lists = [&]() __attribute__((always_inline)) {
        if constexpr (RL) {
            const int W = a.lshare_w;
#pragma unroll
            for (int g = 0; g < QG; g++) {
                float* base = a.lshare + ((qvalid[g] ? q[g] : 0) * (int64_t)a.nseg) * W + LL * h;
                if (qvalid[g]) {
                    uint32_t* dst = reinterpret_cast<uint32_t*>(base + (int64_t)seg * W);
#pragma unroll
                    for (int i = 0; i < LL; i++)
                        __hip_atomic_store(dst + i, __float_as_uint(lst[g][i] == -INF ? INF : lst[g][i]), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
                float tmp[LL];
#pragma unroll
                for (int i = 0; i < LL; i++) tmp[i] = lst[g][i];
                // a published list: +inf at the pad positions [0, pads), then its real values
                // ascending (+inf where not filled yet) -- reading starts at the chunk holding the
                // first real value, and a chunk whose smallest value no lane can take ends it
                const int pads = LL - (k + 1) / 2;
                for (int p = 0; p < a.nseg; p++) {
                    if (p == seg) continue;
                    const uint32_t* src = reinterpret_cast<const uint32_t*>(base + (int64_t)p * W);
#pragma unroll 1
                    for (int i0 = pads & ~3; i0 < LL; i0 += 4) {
                        float w[4];
#pragma unroll
                        for (int i = 0; i < 4; i++)
                            w[i] = qvalid[g] ? __uint_as_float(__hip_atomic_load(src + i0 + i, __ATOMIC_RELAXED,
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
                const float ub = __builtin_amdgcn_fmed3f(tmp[LL - 1], partner(tmp[LL - 1]), INF);
                if (qvalid[g] && ub < thr[g]) {
                    thr[g] = ub;
                    make_tfb(g);
                }
            }
        }
    };
    // one tile of the scan; posc: the tile's place in its barrier group (it % GRP), static
    auto iter = [&](auto posc, floatx16 (&X)[NACC], floatx16 (&Y)[NACC], int it) {
        constexpr int POS = decltype(posc)::value;
        if constexpr (RL && QG == 1 && KR <= 32 && KNN_FUSED_LIST_SHARE) {
            if (a.lshare && list_share_now(it)) exchange_lists();
        }
        if (share_now(it)) {
            if (a.cursor && threadIdx.x == 0)
                __hip_atomic_store(&a.cursor[xcd], (uint32_t)(tile_row(it) >> 6), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            if (a.nseg > 1) {
#pragma unroll
                for (int g = 0; g < QG; g++) {
                    if (!qvalid[g]) continue;
                    if constexpr (RL) {  // publish this query's bound (the heap path does it per accept)
                        if (h == 0 && thr[g] < published[g]) {
                            atomicMin(&a.gthr[q[g]], f2o(thr[g]));
                            published[g] = thr[g];
                        }
                    }
                    // thresholds published by other segments of this query
                    const float gv = o2f(__hip_atomic_load(&a.gthr[q[g]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    if (gv < thr[g]) { thr[g] = gv; make_tfb(g); }
                }
            }
        }
        // the tiles of this step (both of a pair) have landed -- every wave's pieces: each wave
        // waits for all of its own vector-memory ops, then the barrier -- and every wave is done
        // with the buffers the next DMAs overwrite
        const uint64_t t0 = now();
        if (POS == 0) {
            if constexpr (KNN_STUDY_NO_BARRIER) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            else wait_dma_barrier();
        }
        const uint64_t t1 = now();
        // this tile's terms, for its fast test in the next iteration (the tile is resident:
        // landed before this step's barrier, not overwritten before the next one)
        TQ tm_cur;
        if constexpr (!TFG) tm_cur = tile_q(it % NBUF);
        // Tile DMAs.  Spread (the round-4 order): step it issues tile it + AHEAD's pieces between
        // its MFMAs -- so the next group's last tile goes out in the last step before the
        // barrier that waits for it (vmcnt(0)), and its whole memory latency is exposed at every
        // group barrier.  Front (KNN_FUSED_DMA_FRONT, groups of GRP >= 2 tiles): right after a
        // group's barrier, when the previous group's buffers are free, every tile of the NEXT
        // group is issued at once, so each has a whole group's compute to land.  Measured slower
        // everywhere (r05d, same box: A 20.56 -> 21.03 ms, B 479.6 -> 493.2, C1 1729 -> 1796, A's
        // 8-GPU share 3.27 -> 3.39): the barrier wait is the waves' slow-path skew, not the last
        // DMA's latency, and the burst lands on the group's first fragment reads.  A study build.
        constexpr bool FRONT = KNN_FUSED_DMA_FRONT && PAIR;
        if constexpr (FRONT) {
            if (POS == 0 && !KNN_STUDY_NO_DMA) {
#pragma unroll
                for (int p = 0; p < GRP; p++) {
                    const int tn = it + GRP + p;
                    if (tn < ntiles) {
                        const DmaTile dp = dma_desc(tn % NBUF, tn);
#pragma unroll
                        for (int i = 0; i < DMA_PER_WAVE; i++) dma_piece(i, dp);
                    }
                }
            }
        }
        const bool dma_on = !FRONT && !KNN_STUDY_NO_DMA && it + AHEAD < ntiles;
        const DmaTile dd = dma_desc((it + AHEAD) % NBUF, it + AHEAD);
        float tf[QG];
#pragma unroll
        for (int g = 0; g < QG; g++) tf[g] = it > 0 ? (TFG ? tfc[g] : tf_of(g, tm_prev.v[g])) : -INF;
        float mnY[NACC];
        const uint32_t uY = step(X, Y, it % NBUF, dma_on, dd, tf, POS != 0, mnY);
        // PAIR: the pair's next tile is resident since its barrier -- its first fragments are
        // read now, so their latency hides under the slow path below
        if (POS != GRP - 1 && it + 1 < ntiles) prefetch((it + 1) % NBUF);
        const uint64_t t2 = now();
        if (!KNN_STUDY_NO_SLOW) {
            if (uY) {
                // (TFG: the previous tile's own statistics, for the bounds, from its buffer now)
                const TQ tq = TFG ? tile_q((it - 1) % NBUF) : tm_prev;
                if constexpr (RL) slow_rl(Y, it - 1, tf, tq, mnY, uY);
                else if constexpr (DEFER) record(Y, it - 1, tf[0], tq.v[0], uY);
                else slow(Y, it - 1, tf[0], tq.v[0], uY);
            }
            if constexpr (DEFER) {
                if ((it & (FUSED_DEFER_EVERY - 1)) == FUSED_DEFER_EVERY - 1 && __ballot(qcnt > 0)) flush();
            }
        } else {
            asm volatile("" ::"s"(uY));
        }
        if constexpr (KNN_FUSED_STAMPS) {
            const uint64_t t3 = now();
            st_bar += t1 - t0;
            st_step += t2 - t1;
            st_slow += t3 - t2;
            st_visits += uY ? 1 : 0;
        }
        if constexpr (!TFG) tm_prev = tm_cur;
    };
    typedef std::integral_constant<int, 0> P0;
    typedef std::integral_constant<int, 1 % GRP> P1;
    if (!wave_live) {
        // (no valid query) the same barriers, and this wave's pieces of every tile's DMA
        for (int it = 0; it < ntiles; it++) {
            if (it % GRP == 0) wait_dma_barrier();
            if (!KNN_STUDY_NO_DMA && it + AHEAD < ntiles) {
                const DmaTile dd = dma_desc((it + AHEAD) % NBUF, it + AHEAD);
#pragma unroll
                for (int i = 0; i < DMA_PER_WAVE; i++) dma_piece(i, dd);
            }
        }
    } else if constexpr (GRP == 8) {  // octets (the 64-query shape's default)
        for (int it = 0; it < ntiles; it += 8) {
            iter(P0{}, accA, accB, it);
            iter(P1{}, accB, accA, it + 1);
            iter(std::integral_constant<int, 2>{}, accA, accB, it + 2);
            iter(std::integral_constant<int, 3>{}, accB, accA, it + 3);
            iter(std::integral_constant<int, 4>{}, accA, accB, it + 4);
            iter(std::integral_constant<int, 5>{}, accB, accA, it + 5);
            iter(std::integral_constant<int, 6>{}, accA, accB, it + 6);
            iter(std::integral_constant<int, 7>{}, accB, accA, it + 7);
        }
    } else if constexpr (GRP == 4) {
        for (int it = 0; it < ntiles; it += 4) {
            iter(P0{}, accA, accB, it);
            iter(P1{}, accB, accA, it + 1);
            iter(std::integral_constant<int, 2>{}, accA, accB, it + 2);
            iter(std::integral_constant<int, 3>{}, accB, accA, it + 3);
        }
    } else {
        for (int it = 0; it < ntiles; it += 2) {
            iter(P0{}, accA, accB, it);
            iter(P1{}, accB, accA, it + 1);
        }
    }
    if (ntiles > 0 && wave_live) {
        // drain: the last tile's accumulators (ntiles is even: accB)
        const int last = ntiles - 1;
        if constexpr (TFG) tm_prev = tile_q(last % NBUF);  // (no DMA since: the buffer holds it)
        float tf[QG];
#pragma unroll
        for (int g = 0; g < QG; g++) tf[g] = TFG ? tfc[g] : tf_of(g, tm_prev.v[g]);
        if constexpr (RL) {
            float mnB[NACC];
#pragma unroll
            for (int c = 0; c < NACC; c++) {
                mnB[c] = INF;
#pragma unroll
                for (int v = 0; v < 16; v++) mnB[c] = fminf(mnB[c], accB[c][v]);
            }
            slow_rl(accB, last, tf, tm_prev, mnB, 0xffffffffu);
        } else {
            if (pass_set(accB, tf[0], 0xffffffffu)) {
                if constexpr (DEFER) record(accB, last, tf[0], tm_prev.v[0], 0xffffffffu);
                else slow(accB, last, tf[0], tm_prev.v[0], 0xffffffffu);
            }
        }
    }
    if constexpr (DEFER) {
        if (__ballot(qcnt > 0)) flush();
    }
    // the final bound of this piece, any segment count: k_rescore stages only the candidates
    // with L <= gthr (every value there is a k-th smallest U of kept rows, so >= the k-th
    // smallest U of all of them)
    if constexpr (!RL) {
        if (qvalid[0]) thr[0] = fminf(thr[0], root);
    }
#pragma unroll
    for (int g = 0; g < QG; g++)
        if (qvalid[g] && h == 0 && thr[g] < published[g]) atomicMin(&a.gthr[q[g]], f2o(thr[g]));
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < QG; g++)
        if (qvalid[g]) a.cnt[(int64_t)(2 * seg + h) * a.nq + q[g]] = ccnt[g];
#if KNN_FUSED_STAMPS
    {
        if (lane == 0) {
            atomicAdd(&g_knn_stamps[0], (unsigned long long)st_bar);
            atomicAdd(&g_knn_stamps[1], (unsigned long long)st_step);
            atomicAdd(&g_knn_stamps[2], (unsigned long long)st_slow);
            atomicAdd(&g_knn_stamps[3], (unsigned long long)(now() - st_start));
            atomicAdd(&g_knn_stamps[4], (unsigned long long)st_visits);
            atomicAdd(&g_knn_stamps[5], (unsigned long long)ntiles);
            atomicAdd(&g_knn_stamps[6], 1ull);
        }
    }
#endif
}

// The grid (knn_fused_schedule): blocks [0, p1) take one whole query tile each (qt = block,
// every train row) -- whole rounds of the resident blocks, all sweeping the train rows from
// row 0 together (one L2 stream per XCD); the remaining query tiles' (qtile, 64-row tile)
// work is one linear space of w2 units cut into g2 equal ranges, one per block [p1, p1+g2):
// a range covers the tail of one query tile and the head of the next (a piece each), so the
// last round of blocks ends together instead of a partial wave of whole query tiles.
// Pieces of one query tile share thresholds through gthr like segments (piece id = block -
// the first block of that query tile).  One call site of fused_piece (instruction cache).
template <int RB, int MINW, int NBUF, int NW, int QG, int RG, int KR>
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
    // A range runs from its END: the head of its later query tile first (from train row 0),
    // then the tail of the earlier one.  At time tau every block of the balanced schedule is
    // then near train tile tau (or tau + T - W after its switch), so the blocks stream the
    // train rows together through the L2s and the Infinity Cache; in range order each would
    // start from its own row, all 260 MB of A's train operand in use at once, cycling through
    // a 256 MiB cache.  (KNN_FUSED_FORWARD=1: range order, a study build.)
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
#if KNN_FUSED_FORWARD
            const int64_t ql = x / T, t0 = x - ql * T;
            const int64_t t1 = min(T, t0 + (x1 - x));
#else
            const int64_t ql = (x1 - 1) / T;
            const int64_t t0 = max(x, ql * T) - ql * T, t1 = x1 - ql * T;
#endif
            qt = qbase + (int)ql;
            // the block whose range holds the query tile's first unit: largest bb with lo(bb) <= ql T
            seg = p1 ? 0 : (int)(b2 - ((ql * T + 1) * a.g2 - 1) / a.w2);
            rb = t0 * 64;
            re = min(a.nt, t1 * 64);
            adv = t1 - t0;
        }
        if (!first) __syncthreads();  // every wave is done with the previous piece's LDS
        fused_piece<RB, NBUF, NW, QG, RG, KR>(a, qt, seg, rb, re);
        if (KNN_FUSED_FORWARD || segmode) x += adv;
        else x1 -= adv;
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
static size_t fused_lds_of(int row_bytes, int k, int nw, int rg, int nbuf, bool heaps, int qg = 1) {
    const int bn = 32 * rg, bm = 32 * qg * nw;
    const int hs = row_bytes % 64 == 0 ? bn / 4 + 1 : 0;  // (k_gemm_fused: TN header slots)
    const int ins = (bn * (row_bytes / 16 + 1) + hs + 63) / 64;
    // (+ 16 bytes: the block's scan rotation, k_gemm_fused)
    return (size_t)nbuf * ins * 1024 + (heaps ? (size_t)bm * heap_stride(k) * sizeof(float) : 0) + 16;
}

int knn_fused_list_share_width(const FilterPlan& f) {
    if (!KNN_FUSED_LIST_SHARE || !f.ls || !(f.kr == 8 || f.kr == 32)) return 0;
    return f.kr == 32 ? 32 : 16;  // (two lane halves' lists)
}

bool knn_fused_supported(int d) { return d == 64 || d == 128 || d == 256; }

// bytes per operand row in the tile image: 2d -- the accumulators start from the norms in the
// tile header (B, d = 64: 614 -> 586 ms against the augmented k-step, r03q); the augmented block
// (2d + 32) stays as the study build KNN_STUDY_AUG64
int knn_fused_row_bytes(int d) { return d == 64 && KNN_FUSED_AUG64 ? 2 * d + 32 : 2 * d; }

// Shapes (d = features; rows of 2d bytes).  Block = NW waves x 32 QG queries:
//  * k <= 32 (register lists, KR = 8 / 32): 8 waves; 64 queries per wave on 32-row tiles in
//    octets for large query counts (below), else 32 per wave on 64-row tiles -- in quads when
//    eight buffers fit (d <= 128), else in pairs (four buffers, one barrier per two tiles:
//    A 33.4 -> 31.3 ms against two buffers, round 2; 8-wave blocks: B 765 -> 743 ms).
//  * d = 256, 32 < k <= 104 (KR = 104): 8 waves, 32-row tiles in quads.
//  * k > 32 otherwise (LDS heaps, KR = 0): d = 64 in 4-wave blocks, two buffers, two blocks per
//    CU (the other block hides the per-tile barrier and fast test of 5-step tiles); d >= 128 in
//    8-wave blocks: pairs when they fit beside the heaps, else two buffers, else 32-row tiles.
// Register lists, one per lane half: k <= 16 8 entries (KR = 8), k <= 32 16 (KR = 32: exact
// 32-entry lists cost a block per CU of occupancy and 9 % of time on B).
FilterPlan knn_fused_plan(int d, int k, int64_t nq, int num_cus, const FusedForce& force, int max_pieces) {
    const int rb = knn_fused_row_bytes(d);
    const size_t cap = 160 * 1024 - 256;  // room for the kernel's static LDS
    // d = 256, 32 < k <= 104 (C): per-half 52-entry register lists instead of LDS heaps, so
    // the tile buffers get the LDS the heaps held -- 32-row tiles in quads (one barrier per 128
    // rows) instead of one barrier per 32-row tile (force.heaps: the heap shape).  (64-row
    // tiles in pairs, the other way to the same barrier count, spill: two more accumulators.)
    const int kr = k <= 16 ? 8 : k <= 32 ? 32 : (k <= 104 && d == 256 && !force.heaps) ? 104 : 0;
    auto make = [&](int nw, int rg, int minw, int nbuf, int qg = 1) {
        FilterPlan f{nw, qg, rg, minw, nbuf, 32 * qg * nw, fused_lds_of(rb, k, nw, rg, nbuf, kr == 0, qg)};
        f.kr = kr;
        return f;
    };
    // Register-list shapes: 64 queries per wave on 32-row tiles (QG = 2: each A fragment read
    // from LDS feeds two MFMAs, the two accumulators share one norm read, and each tile copy
    // serves 512 queries -- half the LDS reads and DMA per MFMA) when the 512-query blocks fill
    // a round of CUs: at least 384 queries per CU, or (round 6) when the query tiles times the
    // most pieces a query's candidate list allows (max_pieces, the caller's capacity rule)
    // reach 80 % of the CUs (one such block per CU: 8 waves at ~240 VGPRs).  Fewer queries
    // would leave CUs idle (pieces beyond max_pieces overflow the lists) or cut each query
    // tile into many pieces (each piece starts its thresholds from +inf), so they keep 32 per
    // wave on 64-row tiles (with the list exchange).  Same box (profiles/r04c): A 24.08 -> 23.19
    // ms, B 575.9 -> 550.9 ms; A's 8-GPU share (12,500 queries) 3.40 -> 6.33 ms with QG = 2.
    // The fill rule (profiles/r06_studies/r06qg, r06qh; filter ms, QG = 1 -> 2, A's rows, d and
    // k): 18,750 queries (37 tiles x 5 pieces = 71 % of the CUs) 4.57 -> 4.83, 21,875 (84 %)
    // 5.21 -> 5.02, 25,000 5.73 -> 5.19, 50,000 11.02 -> 10.10, 75,000 16.49 -> 14.50, 90,000
    // 18.27 -> 16.83; B's rows (2 pieces): 31,250 (48 %) 17.2 -> 29.1, 62,500 (96 %) 31.9 -> 30.7.
    // force.qg = 1|2 forces the choice (a study override, snapshot at knn_create).
    // (d = 256 keeps 32 queries per wave: two query groups' operands alone are 128 VGPRs)
    const bool fills = (nq + 511) / 512 * (int64_t)std::max(max_pieces, 1) * 5 >= (int64_t)4 * num_cus;
    const bool qg2 = d <= 128 && (force.qg == 2 || (force.qg != 1 && (nq >= (int64_t)384 * num_cus || fills)));
    // tiles in octets: 16 buffers, one barrier per eight 32-row tiles, the loop running whole
    // groups so each tile's place is static (pairs -> quads: B 557.2 -> 501.1 ms, A 22.61 ->
    // 21.67 ms, r04i; quads -> octets: A 21.49 -> 20.80 ms, B 504.6 -> 483.8 ms, r04y).
    // force.nbuf = 4|8 forces pairs or quads (a study override).
    // the v_mfma_f32_16x16x32_bf16 form of a register-list shape (k_gemm_fused16: same tiles,
    // blocks, LDS image and schedule; a study switch until measured)
    auto m16 = [&](FilterPlan f) {
        if (force.m16 && knn_fused16_ptr(d, f)) f.m16 = 1;
        return f;
    };
    if (kr > 0 && qg2) {
        const int nb = force.nbuf == 4 || force.nbuf == 8 ? force.nbuf : 16;
        return m16(make(8, 1, 2, fused_lds_of(rb, k, 8, 1, nb, false, 2) <= cap ? nb : 8, 2));
    }
    if (kr == 104) return make(8, 1, 2, 8);
    // list exchange between a query's pieces (a.lshare, knn_capi.cpp): the QG = 1 shapes only
    // (QG = 2 with it: A 21.81 -> 22.84 ms; on A's 8-GPU share, 10 pieces, 3.55 ms against
    // QG = 1's 3.38 -- more pieces, more kept rows: r04l, r04p)
    if (kr > 0) {
        // 64-row tiles in quads when eight buffers fit (d <= 128): A's 8-GPU share 3.08 -> 2.96 ms,
        // A at QG = 1 23.05 -> 22.31 (r04u); force.nbuf = 4 forces pairs (a study override)
        const bool q8 = force.nbuf != 4 && fused_lds_of(rb, k, 8, 2, 8, false) <= cap;
        FilterPlan f = make(8, 2, 2, q8 ? 8 : 4);
        f.ls = 1;
        return m16(f);
    }
    if (kr == 0 && d == 64 && fused_lds_of(rb, k, 4, 2, 2, true) <= cap / 2) return make(4, 2, 2, 2);
    if (fused_lds_of(rb, k, 8, 2, 4, kr == 0) <= cap) return make(8, 2, 2, 4);
    if (fused_lds_of(rb, k, 8, 2, 2, kr == 0) <= cap) return make(8, 2, 2, 2);
    if (fused_lds_of(rb, k, 8, 1, 2, kr == 0) <= cap) return make(8, 1, 2, 2);
    return FilterPlan{0, 0, 0, 0, 0, 0, 0};  // k too large for the LDS heaps: not supported
}

template <int RB, int KR>
static const void* fused_fn_k(const FilterPlan& f) {
#define KNN_FUSED_FN(NB, NW, QG, RG) reinterpret_cast<const void*>(&k_gemm_fused<RB, 2, NB, NW, QG, RG, KR>)
    if constexpr (KR == 104) {
        return KNN_FUSED_FN(8, 8, 1, 1);
    } else if constexpr (KR > 0) {
        // register lists always fit the pairs shape
        if constexpr (RB <= 256) {  // (QG = 2: d <= 128, knn_fused_plan)
            if (f.qg == 2)
                return f.nbuf == 16 ? KNN_FUSED_FN(16, 8, 2, 1) : f.nbuf == 8 ? KNN_FUSED_FN(8, 8, 2, 1) : KNN_FUSED_FN(4, 8, 2, 1);
        }
        if constexpr (RB <= 256) {  // (quads of 64-row tiles: d <= 128, knn_fused_plan)
            if (f.nbuf == 8) return KNN_FUSED_FN(8, 8, 1, 2);
        }
        return KNN_FUSED_FN(4, 8, 1, 2);
    } else {
        if (f.nw == 4) return KNN_FUSED_FN(2, 4, 1, 2);
        if (f.rg == 2) return f.nbuf == 4 ? KNN_FUSED_FN(4, 8, 1, 2) : KNN_FUSED_FN(2, 8, 1, 2);
        return KNN_FUSED_FN(2, 8, 1, 1);
    }
#undef KNN_FUSED_FN
}
template <int RB>
static const void* fused_fn(const FilterPlan& f) {
    if constexpr (RB == 512)
        if (f.kr == 104) return fused_fn_k<RB, 104>(f);
    return f.kr == 8 ? fused_fn_k<RB, 8>(f) : f.kr == 32 ? fused_fn_k<RB, 32>(f) : fused_fn_k<RB, 0>(f);
}

static const void* fused_ptr(int d, const FilterPlan& f) {
    if (f.m16) return knn_fused16_ptr(d, f);
    if (d == 64) {
        if constexpr (KNN_FUSED_AUG64) return fused_fn<160>(f);
        else return fused_fn<128>(f);
    }
    return d == 128 ? fused_fn<256>(f) : fused_fn<512>(f);
}

hipError_t knn_fused_occupancy(int d, const FilterPlan& f, int* blocks_per_cu) {
    if (!knn_fused_supported(d) || f.nw == 0) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fused_ptr(d, f), 64 * f.nw, f.lds);
}

hipError_t knn_launch_fused(const GemmFilterArgs& a, const FilterPlan& f, hipStream_t st) {
    const int ld = knn_fused_row_bytes(a.d) / 2;  // operand row pitch in elements
    if (!knn_fused_supported(a.d) || f.nw == 0 || a.ld_t != ld || a.ld_q != ld || !a.qstat)
        return hipErrorInvalidValue;
    if (f.m16 && !knn_fused16_ptr(a.d, f)) return hipErrorInvalidValue;
    if (f.kr > 0 && !(f.nw == 8 && (((f.nbuf == 4 || f.nbuf == 8) && f.qg == 1 && f.rg == 2 && f.kr <= 32) ||
                                     ((f.nbuf == 4 || f.nbuf == 8 || f.nbuf == 16) && f.qg == 2 && f.rg == 1 && f.kr <= 32) ||
                                     (f.nbuf == 8 && f.qg == 1 && f.rg == 1 && f.kr == 104 && a.d == 256))))
        return hipErrorInvalidValue;  // (fused_fn_k)
    void* args[] = {const_cast<GemmFilterArgs*>(&a)};
    const dim3 grid((unsigned)(a.g2 < 0 ? (int64_t)a.n_qtiles * a.nseg : (int64_t)a.p1_blocks + a.g2));
    hipError_t e = hipLaunchKernel(fused_ptr(a.d, f), grid, dim3(64 * f.nw), args, f.lds, st);
    if (e != hipSuccess) return e;
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}
