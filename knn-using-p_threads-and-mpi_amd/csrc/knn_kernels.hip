// knn_kernels.hip -- CDNA4 (gfx950) kernels of the KNN hot path.
//
// Reference semantics (srna99/KNN-using-p_threads-and-MPI):
//   distance(): fp32 sum of (a_i-b_i)^2, i ascending, no FMA        main.cpp:14-23
//   insertion queue: strict '<', lower train index wins ties          main.cpp:45-61
//   vote: bincount, argmax with ties to the smallest label            main.cpp:64-78
//
// Neighbour order is encoded as one 64-bit key (distance bits << 32 | train index):
// distances are >= +0, so unsigned order of the float bits is numeric order, and the
// index in the low word reproduces the reference's stable (lower index first) ties.
// A distance that is not < FLT_MAX (inf, NaN, FLT_MAX) gets KEY_NONE and never
// qualifies, exactly like `dist < candidates[2c]` against the FLT_MAX sentinel.
//
// Feature rows are fp32 or bf16 (ELEM_*).  bf16 values widen exactly to fp32, so every
// distance is the reference's fp32 direct form on the widened values.
//
// Kernels
//   k_exact_scan   fused direct-form distance + wave-resident top-k + vote (low d,
//                  ARFF inputs, and the per-query fallback of the GEMM path)
//   k_row_norms    ||x||^2 per row (for the GEMM form)
//   k_gemm_filter  q.t on MFMA (fp32: v_mfma_f32_32x32x2_f32, bf16:
//                  v_mfma_f32_32x32x16_bf16), certified candidate filter with a
//                  running per-query threshold
//   k_rescore      exact direct-form rescore of the surviving candidates + top-k + vote
//   k_merge_vote   merge of per-train-shard neighbour lists (train-sharded runs) + vote
//   k_generate     counter-based synthetic rows (same formula as oracle/knn_oracle.c)
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <type_traits>

#include "knn_kernels.h"
#include "knn_study.h"

#include "knn_device.h"

// ---------------------------------------------------------------------------------
// Direct-form distance, restated from main.cpp:14-23 with contraction disabled so
// every diff*diff and += rounds to fp32 exactly like the reference.  q is the query
// row already widened to fp32 (LDS); t is a train row of element type E.
// ---------------------------------------------------------------------------------
#pragma clang fp contract(off)
template <typename E>
__device__ __forceinline__ float direct_dist(const float* q, const E* __restrict__ t, int d) {
    float sum = 0.0f;
    int i = 0;
    if ((((uintptr_t)t) & (4 * sizeof(E) - 1)) == 0) {
        for (; i + 4 <= d; i += 4) {
            const float4 v = load4(t + i);
            float d0 = q[i + 0] - v.x; sum = sum + d0 * d0;
            float d1 = q[i + 1] - v.y; sum = sum + d1 * d1;
            float d2 = q[i + 2] - v.z; sum = sum + d2 * d2;
            float d3 = q[i + 3] - v.w; sum = sum + d3 * d3;
        }
    }
    for (; i < d; i++) {
        float df = q[i] - widen(t[i]);
        sum = sum + df * df;
    }
    return sum;
}
// The same distance with the train row read in batches of 8 independent float4 loads
// (one memory round trip per 32 features instead of one per 4): for the rescore's
// scattered survivor rows.  Summation order and roundings are direct_dist's.
template <typename E>
__device__ __forceinline__ float direct_dist_batched(const float* q, const E* __restrict__ t, int d) {
    if ((((uintptr_t)t) & (4 * sizeof(E) - 1)) != 0) return direct_dist(q, t, d);
    float sum = 0.0f;
    int i = 0;
    // 8 loads in flight, then the in-order sum over them (16 in flight: 64 more VGPRs, a
    // wave per SIMD less in k_rescore -- measured A 0.50 -> 0.39 ms, B 9.1 -> 7.1 ms with 8)
    for (; i + 32 <= d; i += 32) {
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = load4(t + i + 4 * j);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int b = i + 4 * j;
            float d0 = q[b + 0] - v[j].x; sum = sum + d0 * d0;
            float d1 = q[b + 1] - v[j].y; sum = sum + d1 * d1;
            float d2 = q[b + 2] - v[j].z; sum = sum + d2 * d2;
            float d3 = q[b + 3] - v[j].w; sum = sum + d3 * d3;
        }
    }
    for (; i + 4 <= d; i += 4) {
        const float4 v = load4(t + i);
        float d0 = q[i + 0] - v.x; sum = sum + d0 * d0;
        float d1 = q[i + 1] - v.y; sum = sum + d1 * d1;
        float d2 = q[i + 2] - v.z; sum = sum + d2 * d2;
        float d3 = q[i + 3] - v.w; sum = sum + d3 * d3;
    }
    for (; i < d; i++) {
        float df = q[i] - widen(t[i]);
        sum = sum + df * df;
    }
    return sum;
}
// The same distance with G lanes per row (the rescore when m * G <= 64 survivors, G = d / 32):
// lane p of a group loads features [32p, 32p + 32) in one batch and squares them, then the sum
// runs through the group in order -- lane p continues lane p-1's partial sum -- so every
// addition happens in direct_dist's order and the total (in lane G-1 of the group) has its
// bits.  One memory round trip per row instead of d / 32.  Every lane of the wave calls it
// (the hand-off is a shuffle); t is 4-element aligned.
template <typename E>
__device__ __forceinline__ float direct_dist_grouped(const float* q, const E* __restrict__ t, bool act,
                                                     int p, int G) {
    float sq[32];  // unset in an inactive group, whose sum nobody reads
    if (act) {
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = load4(t + 32 * p + 4 * j);
        const float* qp = q + 32 * p;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            float d0 = qp[4 * j + 0] - v[j].x; sq[4 * j + 0] = d0 * d0;
            float d1 = qp[4 * j + 1] - v[j].y; sq[4 * j + 1] = d1 * d1;
            float d2 = qp[4 * j + 2] - v[j].z; sq[4 * j + 2] = d2 * d2;
            float d3 = qp[4 * j + 3] - v[j].w; sq[4 * j + 3] = d3 * d3;
        }
    }
    float sum = 0.0f;
    for (int j = 0; j < G; j++) {
        const float in = __shfl_up(sum, 1);
        if (p == j) {
            float s = j ? in : 0.0f;
#pragma unroll
            for (int i = 0; i < 32; i++) s = s + sq[i];
            sum = s;
        }
    }
    return sum;
}
#pragma clang fp contract(on)

// ---------------------------------------------------------------------------------
// The vote of main.cpp:64-78 without a C-sized table (any class count): the argmax of
// the label counts over the list entries, ties to the smallest label.  lab[r] is the
// label of list element 64r + lane (-1: none / outside the list).  k rounds of one
// broadcast + R ballots.  Returns (count << 32) | (0xffffffff - label), 0 if empty.
// ---------------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ u64 vote_ballot(const int (&lab)[R], int k) {
    u64 best = 0;
    for (int e = 0; e < k; e++) {
        int le = lab[0];
#pragma unroll
        for (int r = 1; r < R; r++)
            if (r == (e >> 6)) le = lab[r];
        le = __shfl(le, e & 63);
        if (le < 0) continue;
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < R; r++) cnt += __popcll(__ballot(lab[r] == le));
        best = umax64(best, ((u64)(uint32_t)cnt << 32) | (u64)(0xffffffffu - (uint32_t)le));
    }
    return best;
}

// ---------------------------------------------------------------------------------
// Outputs for one query from a finished wave list: the neighbour list (dist, idx_base +
// idx, label) and, when o.pred is set, the vote of main.cpp:64-78.
// counts: wave-private LDS array of C ints, or NULL for the table-free vote_ballot
// (class counts above KNN_VOTE_LDS_MAX_C).  Runs on one wave.
// lab0 (optional): the label of element `lane` of T[0], already loaded by the caller.
// ---------------------------------------------------------------------------------
template <int R>
__device__ void finish_query(const u64 (&T)[R], int k, int C, const int32_t* __restrict__ labels,
                             int* counts, int64_t q, const QueryOut& o, int32_t* __restrict__ status,
                             const int* lab0 = nullptr) {
    const int lane = lane_id();
    const bool vote = o.pred != nullptr;
    const bool lds_vote = vote && counts != nullptr;
    if (lds_vote) {
        for (int c = lane; c < C; c += 64) counts[c] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    u64 kth = list_at(T, k - 1);
    bool bad = (kth == KEY_NONE);
    int labr[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        labr[r] = -1;
        int e = 64 * r + lane;
        if (e < k) {
            const u64 key = T[r];
            const int64_t off = q * o.stride + e;
            if (key != KEY_NONE) {
                int32_t idx = (int32_t)(uint32_t)(key & 0xffffffffull);
                const int lab = (r == 0 && lab0) ? *lab0 : labels[idx];
                if (o.dist) o.dist[off] = __uint_as_float((uint32_t)(key >> 32));
                if (o.idx) o.idx[off] = (int32_t)(o.idx_base + idx);
                if (o.label) o.label[off] = lab;
                if (lab >= 0 && lab < C) {
                    labr[r] = lab;
                    if (lds_vote) atomicAdd(&counts[lab], 1);
                } else {
                    atomicOr(status, KNN_STATUS_BAD_LABEL);
                }
            } else {
                if (o.dist) o.dist[off] = FLT_MAX;
                if (o.idx) o.idx[off] = -1;
                if (o.label) o.label[off] = -1;
            }
        }
    }
    if (!vote) return;
    u64 best = 0;
    if (lds_vote) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // argmax, strict '>' scanning 0..C-1 == max count, smallest label on ties
        for (int c = lane; c < C; c += 64) {
            u64 v = ((u64)(uint32_t)counts[c] << 32) | (u64)(0xffffffffu - (uint32_t)c);
            best = umax64(best, v);
        }
#pragma unroll
        for (int j = 32; j > 0; j >>= 1) best = umax64(best, __shfl_xor(best, j));
    } else {
        best = vote_ballot<R>(labr, k);
    }
    if (lane == 0) {
        o.pred[q] = bad ? 0 : (int32_t)(0xffffffffu - (uint32_t)(best & 0xffffffffull));
        if (bad && !KNN_STUDY_RESULTS_INVALID) atomicOr(status, KNN_STATUS_TOO_FEW);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------------------------
// k_exact_scan: one 256-thread block per query (grid-stride over the query list).
// Wave w scans train rows in 64-row batches b = w, w+4, ...; each lane computes one
// direct-form distance; batches with any key below the running k-th key are merged
// into the wave list.  The four wave lists are then merged by wave 0, which votes.
// LDS: q row [ld_pad] f32 | 4 wave lists [4][64R] u64 | counts [C] i32
// ---------------------------------------------------------------------------------
template <int R, typename E>
__global__ __launch_bounds__(256) void k_exact_scan(ExactScanArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* qs = reinterpret_cast<float*>(smem);
    u64* lists = reinterpret_cast<u64*>(smem + a.q_lds_bytes);
    int* counts = reinterpret_cast<int*>(smem + a.q_lds_bytes + 4 * 64 * R * sizeof(u64));
    if (a.C > KNN_VOTE_LDS_MAX_C) counts = nullptr;  // table-free vote (vote_ballot)
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    KNN_STUDY_SKIP_FALLBACK(a.qlist);
    const int64_t n_work = a.qlist ? (int64_t)(*a.qcount) : a.nq;
    const E* train = reinterpret_cast<const E*>(a.train);
    const E* test = reinterpret_cast<const E*>(a.test);

    for (int64_t w = blockIdx.x; w < n_work; w += gridDim.x) {
        const int64_t q = a.qlist ? (int64_t)a.qlist[w] : w;
        __syncthreads();
        for (int i = threadIdx.x; i < a.d; i += 256) qs[i] = widen(test[q * a.ld_q + i]);
        __syncthreads();

        u64 T[R];
#pragma unroll
        for (int r = 0; r < R; r++) T[r] = KEY_NONE;
        u64 thr = KEY_NONE;
        for (int64_t base = (int64_t)wave * 64; base < a.nt; base += 256) {
            const int64_t t = base + lane;
            u64 key = KEY_NONE;
            if (t < a.nt) key = make_key(direct_dist(qs, train + t * a.ld_t, a.d), (uint32_t)t);
            bool pass = key < thr;
            if (__ballot(pass)) {
                topk_merge<R>(T, pass ? key : KEY_NONE);
                thr = list_at(T, a.k - 1);
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) lists[(wave * R + r) * 64 + lane] = T[r];
        __syncthreads();
        if (wave == 0) {
            for (int ow = 1; ow < 4; ow++) {
#pragma unroll
                for (int r = 0; r < R; r++) {
                    u64 x = lists[(ow * R + r) * 64 + lane];
                    bool pass = x < thr;
                    if (__ballot(pass)) {
                        topk_merge<R>(T, pass ? x : KEY_NONE);
                        thr = list_at(T, a.k - 1);
                    }
                }
            }
            finish_query<R>(T, a.k, a.C, a.labels, counts, q, a.out, a.status);
        }
    }
}

// ---------------------------------------------------------------------------------
// k_direct_tile<QW, R, E>: the direct form (main.cpp:14-23), tiled for throughput.
// A block of DT_NW = 8 waves owns 8*QW queries: wave w owns QW of them, and lane l
// computes the distances of train row r0 + l to each of its wave's queries.
//  * Train tiles (64 rows x DC dims, widened to fp32) are staged once per block in LDS,
//    double-buffered, and read by all 8 waves: 8*QW queries share every staged byte.
//    Rows are padded to an odd number of 16-B slots, so the per-lane ds_read_b128 of a
//    row is conflict-free.  Rows wider than DC are staged in DC-dim chunks; a tile's
//    partial sums carry over the chunks in ascending dim order.
//  * Query values are wave-uniform and reach the VALU from scalar loads, so the inner
//    loop is v_sub (SGPR operand), v_mul, v_add per dim per pair: the reference's
//    unfused fp32 order, bit for bit (contract(off) below).  VALU-bound: 3 ops per dim
//    per pair, 128 ops/clk/CU with >= 2 waves per SIMD.
//  * After each tile every query runs k_exact_scan's selection on its 64 new distances:
//    a ballot against its running k-th distance (rows of a wave arrive in ascending
//    order, so `D < k-th distance` is exactly main.cpp:47's strict test), and a wave
//    bitonic merge only when some lane passes.
//  * SH (k <= 16): the list lives in lanes 0..k-1 of T[i][0], and a tile with at most
//    DT_SHIFT_MAX passing rows inserts them one at a time, in row order, by a lane shift
//    (shift_insert: two DPP row_shr:1 moves and a few selects per row) instead of a 64-key
//    bitonic sort + merge (~300 instructions).  After a segment's first tiles the threshold
//    is tight and a tile has one or two passing rows per query at most (config L, k = 5:
//    about 34 insertions per query over a 27-tile segment); the sort remains for the dense
//    first tiles.
//  * Segments: blockIdx = seg * n_qblocks + qb (co-resident blocks stream the same
//    rows).  With nseg > 1 each block writes its segment's exact top-k as records
//    (dist bits, local row, label) [nseg][nq][3][k], merged by k_merge_vote.
// LDS: 2 tile buffers [64][stride] f32 | per-wave class counts [8][Cpad] (vote_lds)
// ---------------------------------------------------------------------------------
// Insert key y into the ascending list held in lanes 0..15 of T (lanes >= k hold KEY_NONE and
// are left alone: in_list = lane < k).  y's train index is above every listed one (rows are
// visited in ascending order), so `T > y` on the 64-bit keys is main.cpp:47's strict `<` on the
// distance.  Lane e takes lane e-1's key (row_shr:1; lane 0 of a row reads 0 <= y) when both
// are above y, y itself when only its own is: the first key above y moves up one lane and the
// k-th falls off.  Needs k <= 16 (one DPP row).
__device__ __forceinline__ void shift_insert(u64& T, u64 y, bool in_list) {
    const uint32_t phi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(T >> 32), 0x111, 0xF, 0xF, true);
    const uint32_t plo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)T, 0x111, 0xF, 0xF, true);
    const u64 prev = ((u64)phi << 32) | (u64)plo;
    const bool gt = in_list && T > y;
    T = gt ? (prev > y ? prev : y) : T;
}
// distance of list element k-1 (wave-uniform): the insertion threshold, FLT_MAX while the list
// has fewer than k keys (main.cpp:33's sentinel)
__device__ __forceinline__ float kth_dist(u64 T, int k) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(T >> 32), k - 1);
    return hi == 0xffffffffu ? FLT_MAX : __uint_as_float(hi);
}
#ifndef DT_SHIFT_MAX
#define DT_SHIFT_MAX 8  // passing rows per tile and query up to which the lane shift beats the sort
#endif
#pragma clang fp contract(off)
template <int QW, int R, typename E, bool SH>
__global__ __launch_bounds__(64 * DT_NW, 4) void k_direct_tile(DirectTileArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NT = 64 * DT_NW;
    const int lane = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tile_floats = 64 * a.stride;
    float* bufs = reinterpret_cast<float*>(smem);
    int* counts = a.vote_lds ? reinterpret_cast<int*>(smem + 2 * (size_t)tile_floats * 4) + wave * ((a.C + 3) & ~3)
                             : nullptr;
    const int qb = blockIdx.x % a.n_qblocks;
    const int seg = blockIdx.x / a.n_qblocks;
    const int64_t row_begin = (int64_t)seg * a.seg_len;
    const int64_t row_end = min(a.nt, row_begin + a.seg_len);
    const E* __restrict__ train = reinterpret_cast<const E*>(a.train);
    const E* __restrict__ test = reinterpret_cast<const E*>(a.test);
    const int d = a.d, k = a.k;

    int64_t qi[QW];
    const E* qrow[QW];
    u64 T[QW][R];
    float thr[QW];
#pragma unroll
    for (int i = 0; i < QW; i++) {
        qi[i] = (int64_t)qb * (DT_NW * QW) + wave * QW + i;
        qrow[i] = test + (qi[i] < a.nq ? qi[i] : a.nq - 1) * (int64_t)a.ld_q;
#pragma unroll
        for (int r = 0; r < R; r++) T[i][r] = KEY_NONE;
        thr[i] = FLT_MAX;  // main.cpp:33: the FLT_MAX sentinel
    }
    const int ngr = (d + 3) >> 2;          // 4-dim groups per row
    const int gpc = a.dc >> 2;             // groups per chunk
    const int nchunk = (ngr + gpc - 1) / gpc;
    const int pieces = 64 * gpc;           // 4-element pieces per staged chunk
    const int64_t nrows = row_end > row_begin ? row_end - row_begin : 0;
    const int64_t nsteps = ((nrows + 63) >> 6) * nchunk;

    float4 st[DT_MAXP];
    auto load_chunk = [&](int64_t s) __attribute__((always_inline)) {
        const int64_t r0 = row_begin + (s / nchunk) * 64;
        const int c0 = (int)(s % nchunk) * a.dc;
#pragma unroll
        for (int j = 0; j < DT_MAXP; j++) {
            const int p = threadIdx.x + j * NT;
            const int row = p / gpc, g = p - row * gpc;
            if (p < pieces && c0 + 4 * g < 4 * ngr) {
                const int64_t t = min(r0 + row, row_end - 1);
                st[j] = load4(train + t * a.ld_t + c0 + 4 * g);
            }
        }
    };
    auto store_chunk = [&](int64_t s) __attribute__((always_inline)) {
        float* b = bufs + (s & 1) * tile_floats;
        const int c0 = (int)(s % nchunk) * a.dc;
#pragma unroll
        for (int j = 0; j < DT_MAXP; j++) {
            const int p = threadIdx.x + j * NT;
            const int row = p / gpc, g = p - row * gpc;
            if (p < pieces && c0 + 4 * g < 4 * ngr) *reinterpret_cast<float4*>(b + row * a.stride + 4 * g) = st[j];
        }
    };

    float acc[QW];
#pragma unroll
    for (int i = 0; i < QW; i++) acc[i] = 0.0f;
    if (nsteps > 0) {
        load_chunk(0);
        store_chunk(0);
    }
    __syncthreads();
    for (int64_t s = 0; s < nsteps; s++) {
        if (s + 1 < nsteps) load_chunk(s + 1);  // in flight during this chunk's compute
        const int ch = (int)(s % nchunk);
        const int c0 = ch * a.dc;
        const float* tb = bufs + (s & 1) * tile_floats + lane * a.stride;
        const int gend = min(gpc, ngr - ch * gpc);
        for (int g = 0; g < gend; g++) {
            const float4 t = *reinterpret_cast<const float4*>(tb + 4 * g);
            const int col = c0 + 4 * g;
            if (col + 4 <= d) {
#pragma unroll
                for (int i = 0; i < QW; i++) {
                    const float4 qv = load4(qrow[i] + col);  // wave-uniform: scalar loads
                    float s0 = acc[i];
                    float df;
                    df = qv.x - t.x; s0 = s0 + df * df;
                    df = qv.y - t.y; s0 = s0 + df * df;
                    df = qv.z - t.z; s0 = s0 + df * df;
                    df = qv.w - t.w; s0 = s0 + df * df;
                    acc[i] = s0;
                }
            } else {
                const int rem = d - col;  // 1..3 trailing dims
#pragma unroll
                for (int i = 0; i < QW; i++) {
                    const float4 qv = load4(qrow[i] + col);
                    float s0 = acc[i];
                    float df;
                    df = qv.x - t.x; s0 = s0 + df * df;
                    if (rem > 1) { df = qv.y - t.y; s0 = s0 + df * df; }
                    if (rem > 2) { df = qv.z - t.z; s0 = s0 + df * df; }
                    acc[i] = s0;
                }
            }
        }
        if (ch == nchunk - 1) {
            // the tile's distances are final: selection (main.cpp:45-61)
            const int64_t row = row_begin + (s / nchunk) * 64 + lane;
            const bool valid = row < row_end;
#pragma unroll
            for (int i = 0; i < QW; i++) {
                const bool pass = valid && acc[i] < thr[i];
                u64 m = __ballot(pass);
                if (m) {
                    if (SH && __popcll(m) <= DT_SHIFT_MAX) {
                        // one row at a time, ascending: each re-tested against the threshold
                        // the previous insertions left (main.cpp:45-61 in row order)
                        const uint32_t row0 = (uint32_t)(row - lane);
                        do {
                            const int b = __builtin_ctzll(m);
                            m &= m - 1;
                            const float x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc[i]), b));
                            if (x < thr[i]) {
                                shift_insert(T[i][0], ((u64)__float_as_uint(x) << 32) | (u64)(row0 + (uint32_t)b),
                                             lane < k);
                                thr[i] = kth_dist(T[i][0], k);
                            }
                        } while (m);
                    } else {
                        topk_merge<R>(T[i], pass ? make_key(acc[i], (uint32_t)row) : KEY_NONE);
                        if constexpr (SH) {
                            thr[i] = kth_dist(T[i][0], k);
                        } else {
                            const u64 kth = list_at(T[i], k - 1);
                            thr[i] = kth == KEY_NONE ? FLT_MAX : __uint_as_float((uint32_t)(kth >> 32));
                        }
                    }
                }
                acc[i] = 0.0f;
            }
        }
        if (s + 1 < nsteps) store_chunk(s + 1);
        __syncthreads();
    }
    if (a.nseg == 1) {
#pragma unroll
        for (int i = 0; i < QW; i++)
            if (qi[i] < a.nq) finish_query<R>(T[i], k, a.C, a.labels, counts, qi[i], a.out, a.status);
        return;
    }
    // segment records: k (dist bits, local row, label), ascending (KEY_NONE: FLT_MAX, -1, -1)
#pragma unroll
    for (int i = 0; i < QW; i++) {
        if (qi[i] >= a.nq) continue;
        int32_t* rec = a.rec + ((int64_t)seg * a.nq + qi[i]) * 3 * (int64_t)k;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int e = 64 * r + lane;
            if (e < k) {
                const u64 key = T[i][r];
                const bool none = key == KEY_NONE;
                const int32_t idx = (int32_t)(uint32_t)(key & 0xffffffffull);
                rec[e] = none ? (int32_t)__float_as_uint(FLT_MAX) : (int32_t)(uint32_t)(key >> 32);
                rec[k + e] = none ? -1 : idx;
                rec[2 * k + e] = none ? -1 : a.labels[idx];
            }
        }
    }
}

// ---------------------------------------------------------------------------------
// k_direct_rows<NG, QW, E>: the direct form for d <= 16 and k <= 16 (NG = ceil(d / 4) groups of
// four features; config L: d = 11, k = 5).  Such rows are 16-64 bytes, so the tile kernel's LDS
// staging and per-tile block barrier cost more than the arithmetic they feed.  Here every wave
// is independent -- no LDS, no barrier: lane = train row, each lane loads its own row (NG
// float4; the rows of a tile are contiguous across the lanes, one coalesced read) two tiles
// ahead of its use, and the wave's QW queries are loop-invariant registers.  The arithmetic
// runs on query PAIRS in packed fp32 (v_pk_add_f32 / v_pk_mul_f32: two lanes of IEEE fp32 per
// instruction, each rounded exactly like the scalar op), so the sub, mul, add of
// main.cpp:14-23 cost 1.5 instructions per dimension per query instead of 3 -- the same bits.
// Selection: the lane-shift insert of k_direct_tile's SH path.  Work unit = one wave = (QW
// queries, one train segment): wave u of the grid takes query group u % n_qb and segment
// u / n_qb, so the waves one CU runs at once share a segment's rows in L2.
// ---------------------------------------------------------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));
// the wave list T (one register) merged with a batch of 64 keys, one copy of the network
__device__ __attribute__((noinline)) u64 merge_tile_keys(u64 T, u64 x) {
    u64 t[1] = {T};
    topk_merge<1>(t, x);
    return t[0];
}
template <int NG, int QW, typename E>
__global__ __launch_bounds__(256) void k_direct_rows(DirectTileArgs a) {
    static_assert(QW % 2 == 0, "queries go in pairs");
    constexpr int QP = QW / 2;
    const int lane = lane_id();
    const int64_t u = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int qg = (int)(u % a.n_qblocks);
    const int seg = (int)(u / a.n_qblocks);
    if (seg >= a.nseg) return;  // (wave-uniform: the grid's last block may be partial)
    const int64_t row_begin = (int64_t)seg * a.seg_len;
    const int64_t row_end = min(a.nt, row_begin + a.seg_len);
    const E* __restrict__ train = reinterpret_cast<const E*>(a.train);
    const E* __restrict__ test = reinterpret_cast<const E*>(a.test);
    const int d = a.d, k = a.k;
    const int rem = d - 4 * (NG - 1);  // features in the last group, 1..4

    int64_t qi[QW];
    f2v qv[QP][4 * NG];  // query pair p, feature c: (q_2p[c], q_2p+1[c]); zero past d
#pragma unroll
    for (int i = 0; i < QW; i++) qi[i] = (int64_t)qg * QW + i;
#pragma unroll
    for (int p = 0; p < QP; p++) {
        const E* r0 = test + min(qi[2 * p], a.nq - 1) * (int64_t)a.ld_q;
        const E* r1 = test + min(qi[2 * p + 1], a.nq - 1) * (int64_t)a.ld_q;
#pragma unroll
        for (int g = 0; g < NG; g++) {
            const float4 x = load4(r0 + 4 * g), y = load4(r1 + 4 * g);
            qv[p][4 * g + 0] = f2v{x.x, y.x};
            qv[p][4 * g + 1] = f2v{x.y, y.y};
            qv[p][4 * g + 2] = f2v{x.z, y.z};
            qv[p][4 * g + 3] = f2v{x.w, y.w};
        }
    }
    u64 T[QW][1];
    float thr[QW];
#pragma unroll
    for (int i = 0; i < QW; i++) {
        T[i][0] = KEY_NONE;
        thr[i] = FLT_MAX;  // main.cpp:33: the FLT_MAX sentinel
    }
    const int64_t nrows = row_end > row_begin ? row_end - row_begin : 0;
    const int ntiles = (int)((nrows + 63) >> 6);
    auto load_row = [&](int t, float4 (&x)[NG]) __attribute__((always_inline)) {
        const int64_t r = min(row_begin + 64 * (int64_t)t + lane, row_end - 1);
#pragma unroll
        for (int g = 0; g < NG; g++) x[g] = load4(train + r * a.ld_t + 4 * g);
    };
    float4 buf[3][NG];  // rows of tiles t, t+1, t+2 (loads two tiles ahead)
    if (ntiles > 0) load_row(0, buf[0]);
    if (ntiles > 1) load_row(1, buf[1]);
    auto dist = [&](const float4 (&x)[NG], f2v (&acc)[QP]) __attribute__((always_inline)) {
#pragma unroll
        for (int p = 0; p < QP; p++) acc[p] = f2v{0.0f, 0.0f};
#pragma unroll
        for (int g = 0; g < NG; g++) {
#pragma unroll
            for (int c = 0; c < 4; c++) {
                if (g == NG - 1 && c >= rem) break;  // (wave-uniform)
                const float tv = f4get(x[g], c);
#pragma unroll
                for (int p = 0; p < QP; p++) {
                    const f2v df = qv[p][4 * g + c] - f2v{tv, tv};
                    acc[p] = acc[p] + df * df;
                }
            }
        }
    };
    // tile 0 of the segment: every row passes the FLT_MAX sentinel, so each list starts as the
    // sorted tile (one bitonic sort, KEY_NONE for rows past the segment) -- after it the lists
    // are full and every later tile goes through the lane shift, one passing row at a time
    // (a tile with many passing rows, rare past tile 0, just takes more rounds)
    auto first = [&](const float4 (&x)[NG]) __attribute__((always_inline)) {
        f2v acc[QP];
        dist(x, acc);
        const int64_t row = row_begin + lane;
        const bool valid = row < row_end;
#pragma unroll
        for (int i = 0; i < QW; i++) {
            const float di = (i & 1) ? acc[i >> 1].y : acc[i >> 1].x;
            T[i][0] = sort64(valid ? make_key(di, (uint32_t)row) : KEY_NONE, /*descending=*/false);
            thr[i] = kth_dist(T[i][0], k);
        }
    };
    auto tile = [&](int t, const float4 (&x)[NG]) __attribute__((always_inline)) {
        f2v acc[QP];
        dist(x, acc);
        const int64_t row = row_begin + 64 * (int64_t)t + lane;
        const bool valid = row < row_end;
        const uint32_t row0 = (uint32_t)(row - lane);
#pragma unroll
        for (int i = 0; i < QW; i++) {
            const float di = (i & 1) ? acc[i >> 1].y : acc[i >> 1].x;
            const bool pass = valid && di < thr[i];
            u64 m = __ballot(pass);
            if (__popcll(m) > DT_SHIFT_MAX) {
                // many passing rows (train rows in decreasing distance order, e.g. sorted or
                // clustered data): one bitonic merge of the tile instead of up to 64 serial lane
                // shifts -- k_direct_tile's SH guard.  Same result: the merge keeps the
                // k smallest (distance, index) keys, the shifts insert in row order.  Out of line:
                // inlined in the loop's six tile copies it cost config L 17 % (r06i); out of line
                // 7 % (0.083 -> 0.089 ms, 61 -> 65 VGPRs; bounding the kernel to 64 VGPRs spilled:
                // 0.115 ms, r06l), while train rows in decreasing distance ran 16x slower than
                // uniform rows without it and 6x with it (scripts/diag_direct_rows_adversarial.py)
                T[i][0] = merge_tile_keys(T[i][0], pass ? make_key(di, (uint32_t)row) : KEY_NONE);
                thr[i] = kth_dist(T[i][0], k);
                m = 0;
            }
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                const float x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(di), b));
                if (x < thr[i]) {  // (re-tested against the threshold the earlier rows left)
                    shift_insert(T[i][0], ((u64)__float_as_uint(x) << 32) | (u64)(row0 + (uint32_t)b), lane < k);
                    thr[i] = kth_dist(T[i][0], k);
                }
            }
        }
    };
    if (ntiles > 2) load_row(2, buf[2]);
    if (ntiles > 0) first(buf[0]);
    // tiles 1, 2, ...: loads two tiles ahead into three static buffer places (no register copies)
    int t = 1;
    for (; t + 3 <= ntiles; t += 3) {
        if (t + 2 < ntiles) load_row(t + 2, buf[0]);
        tile(t, buf[1]);
        if (t + 3 < ntiles) load_row(t + 3, buf[1]);
        tile(t + 1, buf[2]);
        if (t + 4 < ntiles) load_row(t + 4, buf[2]);
        tile(t + 2, buf[0]);
    }
    if (t < ntiles) {
        if (t + 2 < ntiles) load_row(t + 2, buf[0]);
        tile(t, buf[1]);
        if (t + 1 < ntiles) tile(t + 1, buf[2]);
    }
    if (a.nseg == 1) {
#pragma unroll
        for (int i = 0; i < QW; i++)
            if (qi[i] < a.nq) finish_query<1>(T[i], k, a.C, a.labels, nullptr, qi[i], a.out, a.status);
        return;
    }
    // Fused merge (round 6, a.arrive): the last of the query group's nseg waves to finish merges
    // every segment's records into its own list -- by (distance, row): the reference's
    // lower-index tie rule across segments, as k_merge_vote -- and votes, in this launch.  The
    // records cross CUs (and XCDs, whose L2s are not coherent with each other) inside the
    // kernel, so they go through device-scope (sc1) stores and loads, which the XCD L2s do not
    // hold stale; `s_waitcnt vmcnt(0)` retires this wave's record stores before lane 0's
    // device-scope arrival, and the last arriver reads the others' records only after it saw
    // the count.  (An agent-scope release / acquire fence would add an L2 write-back and
    // invalidate per wave: buffer_wbl2 / buffer_inv sc1.)  The merging wave resets the
    // group's counter: zero between calls.
    const bool fused = a.arrive != nullptr;
    auto put = [&](int32_t* p, int32_t v) __attribute__((always_inline)) {
        if (fused) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *p = v;
    };
#pragma unroll
    for (int i = 0; i < QW; i++) {
        if (qi[i] >= a.nq) continue;
        int32_t* rec = a.rec + ((int64_t)seg * a.nq + qi[i]) * 3 * (int64_t)k;
        if (lane < k) {
            const u64 key = T[i][0];
            const bool none = key == KEY_NONE;
            const int32_t idx = (int32_t)(uint32_t)(key & 0xffffffffull);
            put(rec + lane, none ? (int32_t)__float_as_uint(FLT_MAX) : (int32_t)(uint32_t)(key >> 32));
            put(rec + k + lane, none ? -1 : idx);
            put(rec + 2 * k + lane, none ? -1 : a.labels[idx]);
        }
    }
    if (!fused) return;  // (k_merge_vote merges the segments)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(&a.arrive[qg], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old != a.nseg - 1) return;
    if (lane == 0) __hip_atomic_store(&a.arrive[qg], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int i = 0; i < QW; i++) {
        if (qi[i] >= a.nq) continue;
        u64 kth = list_at(T[i], k - 1);
        for (int s = 0; s < a.nseg; s++) {
            if (s == seg) continue;  // (this wave's own list is T[i] already)
            const int32_t* rec = a.rec + ((int64_t)s * a.nq + qi[i]) * 3 * (int64_t)k;
            u64 key = KEY_NONE;
            if (lane < k) {
                const int32_t ix = __hip_atomic_load(rec + k + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int32_t db = __hip_atomic_load(rec + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (ix >= 0) key = make_key(__int_as_float(db), (uint32_t)ix);
            }
            // a segment's list ascends: the keys below the current k-th are its prefix
            const bool pass = key < kth;
            if (!__ballot(pass)) continue;
            topk_merge_sorted<1>(T[i], pass ? key : KEY_NONE);
            kth = list_at(T[i], k - 1);
        }
        finish_query<1>(T[i], k, a.C, a.labels, nullptr, qi[i], a.out, a.status);
    }
}
#pragma clang fp contract(on)


// ---------------------------------------------------------------------------------
// k_row_norms: out[r] = sum_i x[r][i]^2 (fp32).  Flags rows whose norm is too large
// for the GEMM form's error certificate (>= 2^125) so the host falls back, and keeps
// the maximum norm (ordered bits, atomicMax) for the filter's conservative fast test.
// For the fused bf16 filter it also bounds the operand rounding (DESIGN.md
// "Certificate"): with rx = rn_bf16(oscale x) / oscale, sqrt-of-sum upper bounds of
// ||x - rx|| and ||rx|| (x - rx is exact in fp32): per query row (qstat) or per 64-row
// tile maximum (tstat).
// ---------------------------------------------------------------------------------
// sqrt of an fmaf sum of d squares, rounded up: the sum errs by <= d u (relative), the
// squares below 2^-150 that flushed add <= d 2^-149; the factor covers d <= 8000
__device__ __forceinline__ float norm_ub(float s, int d) {
    return sqrtf(fmaf((float)d, 0x1p-149f, s)) * (1.0f + 0x1p-12f);
}
template <typename E>
__global__ __launch_bounds__(256) void k_row_norms(const E* __restrict__ x, int64_t n, int ld,
                                                   int d, float* __restrict__ out,
                                                   int32_t* __restrict__ status,
                                                   uint32_t* __restrict__ maxo,
                                                   float* __restrict__ outp, float c1,
                                                   float4* __restrict__ tstat, const int32_t* __restrict__ gate,
                                                   float2* __restrict__ qstat, float oscale) {
    if (gate && *gate == 0) return;  // a gated stage (AUTO's re-run) that is not taken
    // rows [n, n + 64) of out/outp get +inf: the GEMM filter's tile tail reads them
    const int lane = threadIdx.x & 63;
    const int64_t r0 = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63);  // the wave's 64 rows
    const int64_t r = r0 + lane;
    const bool rstat = tstat || qstat;
    const float inv = 1.0f / oscale;  // 1 or -0.5: exact
    // 16 lanes per row, 4 rows at a time (coalesced 256-byte reads); lane r0 + l ends with
    // row l's sums.  The fp32 sum order differs from a serial chain: the certificate's bound
    // on a norm (d u relative) holds for any order.
    float s = 0.0f, se = 0.0f, sr = 0.0f;
    const int g = lane >> 4, l16 = lane & 15;
    float a, ae, ar;
    auto acc = [&](float v) __attribute__((always_inline)) {
        a = fmaf(v, v, a);
        if (rstat) {
            const float rv = __uint_as_float(bf16_rne(oscale * v) << 16) * inv;
            const float e = v - rv;
            ae = fmaf(e, e, ae);
            ar = fmaf(rv, rv, ar);
        }
    };
    // the round's sums to their rows: lane l takes row l = 4 r4 + (l & 3) from lane 16 (l & 3)
    auto finish_round = [&](int r4) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 8; j > 0; j >>= 1) {
            a += __shfl_xor(a, j);
            if (rstat) { ae += __shfl_xor(ae, j); ar += __shfl_xor(ar, j); }
        }
        const float va = __shfl(a, 16 * (lane & 3));
        const float vae = rstat ? __shfl(ae, 16 * (lane & 3)) : 0.0f;
        const float var = rstat ? __shfl(ar, 16 * (lane & 3)) : 0.0f;
        if ((lane >> 2) == r4) { s = va; se = vae; sr = var; }
    };
    if (d % 4 == 0 && d <= 256) {
        // four rounds' loads (up to 16 float4 per lane) in flight before their sums, instead of
        // one load per round trip; the zero padding adds exact zeros, so the sums are the
        // loop's below bit for bit
        for (int r4 = 0; r4 < 16; r4 += 4) {
            float4 v[4][4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int64_t row = r0 + 4 * (r4 + u) + g;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const int i = 4 * l16 + 64 * c;
                    v[u][c] = (row < n && i + 4 <= d) ? load4(x + row * ld + i) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                a = 0.0f; ae = 0.0f; ar = 0.0f;
#pragma unroll
                for (int c = 0; c < 4; c++) { acc(v[u][c].x); acc(v[u][c].y); acc(v[u][c].z); acc(v[u][c].w); }
                finish_round(r4 + u);
            }
        }
    } else {
        for (int r4 = 0; r4 < 16; r4++) {
            const int64_t row = r0 + 4 * r4 + g;
            a = 0.0f; ae = 0.0f; ar = 0.0f;
            if (row < n) {
                const E* xr = x + row * ld;
                int i = 4 * l16;
                for (; i + 4 <= d; i += 64) {
                    const float4 v = load4(xr + i);
                    acc(v.x); acc(v.y); acc(v.z); acc(v.w);
                }
                for (int t = (d & ~3) + l16; t < d; t += 16) acc(widen(xr[t]));  // the d % 4 tail
            }
            finish_round(r4);
        }
    }
    if (r < n) {
        out[r] = s;
        if (qstat) qstat[r] = make_float2(norm_ub(s, d), norm_ub(se, d));
        if (outp) outp[r] = c1 * s;
        if (!(s < 0x1p125f)) atomicOr(status, KNN_STATUS_GEMM_UNSAFE);
    } else if (outp && r < n + 64) {
        out[r] = __uint_as_float(0x7f800000u);
        outp[r] = __uint_as_float(0x7f800000u);
    }
    if (maxo || tstat) {
        // the wave's 64 rows are one 64-row tile of the fused filter (rows >= n count as 0)
        float m = s, me = r < n ? norm_ub(se, d) : 0.0f, mr = r < n ? norm_ub(sr, d) : 0.0f;
#pragma unroll
        for (int j = 32; j > 0; j >>= 1) {
            m = fmaxf(m, __shfl_xor(m, j));
            me = fmaxf(me, __shfl_xor(me, j));
            mr = fmaxf(mr, __shfl_xor(mr, j));
        }
        if ((threadIdx.x & 63) == 0) {
            // one word for the whole launch: the atomic only when it can raise the maximum (a
            // stale read is never above the stored value, so nothing larger is skipped)
            if (maxo) {
                const uint32_t mo = f2o(m);
                if (mo > __hip_atomic_load(maxo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(maxo, mo);
            }
            if (tstat && r < n) tstat[r >> 6] = make_float4(m, me, mr, 0.0f);
        }
    }
}

// ---------------------------------------------------------------------------------
// k_split_rows: fp32 rows -> bf16 [hi | lo] rows for the split filter (ELEM_SPLIT).
// hi = rn(x); x - hi is exact in fp32 (Sterbenz: hi is within 2^-8 |x| of x, or 0 when
// |x| < 2^-134); lo = rn(x - hi).  |x - hi - lo| <= 2^-16 |x| + 2^-134.  One thread per
// 4 elements (coalesced float4 in, two 8-byte bf16 quads out).
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_split_rows(const float* __restrict__ x, int64_t n, int ld, int d,
                                                    bf16_t* __restrict__ out, const int32_t* __restrict__ gate) {
    if (gate && *gate == 0) return;
    const int per_row = d >> 2;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n * per_row; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / per_row;
    const int c = (int)(i - r * per_row) * 4;
    const float4 v = *reinterpret_cast<const float4*>(x + r * ld + c);
    const float e[4] = {v.x, v.y, v.z, v.w};
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        hi[t] = bf16_rne(e[t]);
        lo[t] = bf16_rne(e[t] - __uint_as_float(hi[t] << 16));
    }
    bf16_t* o = out + r * (int64_t)(2 * d) + c;
    *reinterpret_cast<uint2*>(o) = make_uint2(hi[0] | (hi[1] << 16), hi[2] | (hi[3] << 16));
    *reinterpret_cast<uint2*>(o + d) = make_uint2(lo[0] | (lo[1] << 16), lo[2] | (lo[3] << 16));
    }
}

// ---------------------------------------------------------------------------------
// k_round_rows: fp32 rows -> bf16 rows rn(x) for the rounded filter (ELEM_ROUND, d
// elements per row): |x - rn(x)| <= 2^-8 |x| + 2^-134.  The filter runs the bf16 kernel
// on them; the certificate (knn_capi.cpp) carries the rounding.  One thread per 4
// elements (coalesced float4 in, one 8-byte bf16 quad out).
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_round_rows(const float* __restrict__ x, int64_t n, int ld, int d,
                                                    bf16_t* __restrict__ out, const int32_t* __restrict__ gate) {
    if (gate && *gate == 0) return;
    const int per_row = d >> 2;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n * per_row; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / per_row;
        const int c = (int)(i - r * per_row) * 4;
        const float4 v = *reinterpret_cast<const float4*>(x + r * ld + c);
        *reinterpret_cast<uint2*>(out + r * (int64_t)d + c) =
            make_uint2(bf16_rne(v.x) | (bf16_rne(v.y) << 16), bf16_rne(v.z) | (bf16_rne(v.w) << 16));
    }
}

// ---------------------------------------------------------------------------------
// k_gemm_filter<E, RB, MINB, NBUF, QG>: GEMM-form candidate filter on MFMA.
//   E = float (RB/4-d rows, v_mfma_f32_32x32x2_f32, exact fp32) or bf16 (RB/2-d rows,
//   v_mfma_f32_32x32x16_bf16) or split_t (fp32 data as RB/4-d [hi | lo] bf16 rows: three
//   32x32x16 bf16 MFMAs per 16 features); RB = bytes per row (128, 256, 512).
//
// Block = 256 threads = 4 waves; each wave owns QG groups of 32 queries (BM = 128 QG
// per block); a train tile holds BN = 32 RG rows with RG = 2 / QG, so every wave runs
// two 32x32 accumulators per tile either way: (rows 0-31, rows 32-63) x its 32 queries
// for QG = 1 (fp32: MFMA-bound, fewer heaps), or rows 0-31 x (queries 0-31, 32-63) for
// QG = 2 (bf16: a 32x32x16 MFMA moves 16x the FLOP of the fp32 one, so the train bytes
// per FLOP must halve -- twice the queries per staged byte -- to stay under what L2 ->
// LDS delivers per CU, and each A fragment read feeds two MFMAs).
// Each lane keeps 16 bytes of its query rows per k-step s (bytes [32s+16h, 32s+16h+16),
// h = lane>>5) as B-operand fragments, in VGPRs for the whole scan.  Train tiles are
// copied global -> LDS by LDS-DMA (global_load_lds_dwordx4, no staging registers), NBUF
// buffers deep with one barrier per tile.  Rows keep natural k order and are padded to
// RB+16 bytes (the pad slot of each row receives a harmless duplicate) so the A-operand
// ds_read_b128 is conflict-free; lane (j,h) reads the same 16 bytes of train row j (and
// 32+j) as its query fragment: fp32 feeds 4 k-steps of 32x32x2 (k = 8s+4h+jj), bf16 one
// 32x32x16 (k = 16s+8h+jj, the gfx950 A/B lane map).  Per tile each wave issues the
// tile's MFMAs into accumulator set X while the certified test of the PREVIOUS tile
// (set Y) runs in between (software pipelining).  Accumulator a of a lane l holds
// query group qg(a), train row 32 rg(a) + (reg&3) + 8(reg>>2) + 4(l>>5), column l&31.
//
// Certificate: with s = qn+tn, G = fma(-2, q.t, s), Delta = coef*s+eta,
// L = G - Delta <= D <= U = G + Delta for the reference's direct-form distance D
// (coef/eta per element type, set by the host).
// A row is kept for query q iff L <= thr_q, thr_q = the k-th smallest U among rows
// this block kept (the root of a per-query max-heap of the k smallest U, in LDS) or a
// smaller bound published by another segment (gthr).  Every row of the exact top-k
// has L <= D <= D_(k) <= thr_q.  The per-value fast test y = fma(-2, q.t, (1-coef) tn)
// <= tf_q is a conservative superset of L <= thr_q (tf_q adds 2^-16 (|thr|+qn+max tn)
// > the rounding gap of the two formulas); a wave re-checks exactly only when some lane
// passes (slow path).  Kept rows go to this segment's slice of the query's candidate
// list (LDS counter).
// ---------------------------------------------------------------------------------
// constants of the filter (measured against their alternatives in rounds 1-2)
static constexpr int FILTER_PF = 6;            // A-fragment prefetch depth in MFMAs (bf16)
static constexpr int FILTER_RQ = 4;            // deferred-queue depth per lane (8-wave shape)
static constexpr int FILTER_DEFER_EVERY = 64;  // tiles between flushes of the deferred queues

template <typename E, int RB, int MINW, int NBUF, int NW, int QG, int RG>
__global__ __launch_bounds__(64 * NW, MINW) void k_gemm_filter(GemmFilterArgs a) {
    if ((a.gate && *a.gate == 0) || (*a.status & KNN_STATUS_GEMM_UNSAFE)) return;  // not taken / exact path
    typedef FilterTile<RB, NW, QG, RG> FT;
    constexpr bool BF = sizeof(E) == 2;
    constexpr bool SPLIT = std::is_same<E, split_t>::value;  // [hi | lo] rows of fp32 data
    constexpr int NACC = FT::NACC, BN = FT::BN, BM = FT::BM, STRIDE = FT::STRIDE, SLOTS = FT::SLOTS;
    constexpr int DMA_INS = FT::DMA_INS, TILE = FT::TILE;
    constexpr int NT = 64 * NW;                    // threads per block
    constexpr int DMA_PER_WAVE = (DMA_INS + NW - 1) / NW;
    constexpr int NS = RB / 32;                    // k-steps: 16 B per lane half per step
    constexpr int NV = 16 * NACC;                  // fast-test values per lane per tile
    constexpr int VPS = 16 / NS;                   // values per accumulator per k-step
    constexpr int NR = NBUF + 1;                   // norm ring slots: tiles it-1 .. it+NBUF-1
    static_assert(16 % NS == 0 && (NACC == 1 || NACC == 2) && (QG == 1 || RG == 1), "tile geometry");
    static_assert(NBUF == 2, "tile buffers");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* tiles = smem;                                     // [NBUF][TILE]
    float* ring = reinterpret_cast<float*>(smem + NBUF * TILE);      // [NR][2][BN]: (1-c) tn, tn
    const int hs = heap_stride(a.k);
    float* topU = ring + NR * 2 * BN;                                // [BM][hs] max-heaps of U
    const int cap_sub = a.cap_seg / 2;  // candidate sub-slice of one lane half (h) of a query

    const int lane = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // scalar: uniform DMA branches
    const int j = lane & 31;
    const int h = lane >> 5;
    const int qt = blockIdx.x % a.n_qtiles;
    const int seg = blockIdx.x / a.n_qtiles;
    const int64_t row_begin = (int64_t)seg * a.seg_len;
    const int64_t row_end = min(a.nt, row_begin + a.seg_len);
    const int k = a.k;
    const float INF = __uint_as_float(0x7f800000u);
    const float coef = a.coef, eta = a.eta, c1 = 1.0f - a.coef;
    const float tnmax = o2f(*a.tnmax);
    const int64_t ldb = (int64_t)a.ld_t * sizeof(E);  // train row pitch, bytes
    const unsigned char* trainb = reinterpret_cast<const unsigned char*>(a.train);

    for (int i = threadIdx.x; i < BM * hs; i += NT) {
        const int e = i % hs;
        topU[i] = (e == hs - 1 || e <= k - 2) ? INF : -INF;  // root, nodes 1..k-1: +inf
    }
    for (int i = threadIdx.x; i < NR * 2 * BN; i += NT) ring[i] = INF;

    // per query group g: this lane's query (local jl[g], global q[g]) and its state
    int jl[QG];
    int64_t q[QG];
    bool qvalid[QG];
    float qn[QG], thr[QG], published[QG], tf[QG];
    float root[QG];    // this query's heap root (k-th smallest U kept so far), mirrored in both lanes
    int ccnt[QG];      // candidates this lane half kept (its sub-slice fill)
    auto make_tf = [&](int g, float th) -> float {
        if (!qvalid[g]) return -INF;
        const float m = 0x1p-16f * (fabsf(th) + qn[g] + tnmax);
        return ((th - c1 * qn[g]) + eta) + m;
    };
    uint4 qf[QG][NS];
#pragma unroll
    for (int g = 0; g < QG; g++) {
        jl[g] = wave * 32 * QG + 32 * g + j;
        q[g] = (int64_t)qt * BM + jl[g];
        qvalid[g] = q[g] < a.nq;
        const unsigned char* qrow = reinterpret_cast<const unsigned char*>(a.test) +
                                    (qvalid[g] ? q[g] : 0) * (int64_t)a.ld_q * (int64_t)sizeof(E);
#pragma unroll
        for (int s = 0; s < NS; s++)
            qf[g][s] = qvalid[g] ? *reinterpret_cast<const uint4*>(qrow + 32 * s + 16 * h)
                                 : make_uint4(0u, 0u, 0u, 0u);
        qn[g] = qvalid[g] ? a.qnorm[q[g]] : 0.0f;
        thr[g] = qvalid[g] ? o2f(a.gthr[q[g]]) : -INF;
        published[g] = thr[g];
        tf[g] = make_tf(g, thr[g]);
        root[g] = INF;
        ccnt[g] = 0;
    }

    // LDS-DMA of one tile: slot P (16 B) of the padded image -> row P / SLOTS, slot P % SLOTS;
    // the pad slot (SLOTS-1) gets a duplicate of slot 0.  The last instruction may be
    // partial (LAST_LANES active; each buffer has room for a whole one).  Rows past nt are
    // the operand's pad rows; their ring entries are +inf (tnorm/tnp are padded with +inf):
    // never pass.
    uint32_t doff[DMA_PER_WAVE];  // per-lane byte offsets of this wave's DMA slots in a tile
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; i++) {
        const int P = (wave + NW * i) * 64 + lane;
        const int row = min(P / SLOTS, BN - 1), sl = P % SLOTS;
        doff[i] = (uint32_t)(row * ldb + 16 * (sl == SLOTS - 1 ? 0 : sl));
    }
    // DMA piece i < DMA_PER_WAVE: this wave's i-th 1 KiB instruction of the tile; piece
    // DMA_PER_WAVE: the tile's norm terms (two waves).  The step issues the pieces spread
    // between its MFMAs: issued as one burst after the barrier, every wave queued behind
    // the CU's whole tile of DMA issue (measured ~550 clocks per tile) with its MFMAs idle.
    constexpr int NPIECE = DMA_PER_WAVE + 1;
    // LDS byte offsets as plain 32-bit SGPR values (one generic -> LDS conversion, here)
    const uint32_t lds_tiles = __builtin_amdgcn_readfirstlane(lds_addr(tiles));
    const uint32_t lds_ring = __builtin_amdgcn_readfirstlane(lds_addr(ring));
    // one tile's DMA: uniform source row pointer, LDS buffer / ring offsets.  Every tile is
    // whole: the operand rows cover the 64-row tile grid (run_gemm pads them), so a piece is
    // always the scalar tile base + this lane's fixed offset
    struct DmaTile { const unsigned char* src; uint32_t lds, lring; int64_t r0; };
    auto dma_desc = [&](int buf, int slot, int64_t r0) -> DmaTile {
        return DmaTile{trainb + r0 * ldb, lds_tiles + (uint32_t)(buf * TILE),
                       lds_ring + (uint32_t)(slot * 2 * BN * 4), r0};
    };
    auto dma_piece = [&](int i, const DmaTile& d) __attribute__((always_inline)) {
        if (i < DMA_PER_WAVE) {
            const int ins = wave + NW * i;
            if (ins < DMA_INS) {
                if (i == DMA_PER_WAVE - 1 && ins == DMA_INS - 1 && lane >= FT::LAST_LANES) return;
                dma16s(doff[i], d.src, d.lds + (uint32_t)ins * 1024u);
            }
        } else if (lane < BN) {
            if (wave == NW - 2)
                dma4s(4u * lane, a.tnp + d.r0, d.lring);
            else if (wave == NW - 1)
                dma4s(4u * lane, a.tnorm + d.r0, d.lring + BN * 4);
        }
    };
    auto dma_tile = [&](int buf, int slot, int64_t r0) __attribute__((always_inline)) {
        const DmaTile d = dma_desc(buf, slot, r0);
#pragma unroll
        for (int i = 0; i < NPIECE; i++) dma_piece(i, d);
    };
    // pieces issued at k-step s of a step, spread evenly over the tile's MFMAs
    auto dma_at = [&](int s, bool on, const DmaTile& d) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NPIECE; i++)
            if (on && (i * NS) / NPIECE == s) dma_piece(i, d);
    };

    // accumulator a <-> (row group, query group)
    auto rg_of = [](int acc) { return RG == 2 ? acc : 0; };
    auto qg_of = [](int acc) { return QG == 2 ? acc : 0; };

    // MFMAs of one tile into X, interleaved with the fast test of the previous tile (Y)
    auto step = [&](floatx16 (&X)[NACC], floatx16 (&Y)[NACC], int buf, int slotY, bool dma_on,
                    const DmaTile& dd) -> bool {
        const unsigned char* tile = tiles + buf * TILE;
        const unsigned char* a0p = tile + j * STRIDE + 16 * h;
        const unsigned char* a1p = tile + ((RG == 2 ? 32 : 0) + j) * STRIDE + 16 * h;
        const float* tnpY = ring + slotY * 2 * BN;
#pragma unroll
        for (int c = 0; c < NACC; c++) X[c] = floatx16{};
        float4 t4[RG];  // norm terms of the rows in use, per row group
#pragma unroll
        for (int r = 0; r < RG; r++) t4[r] = make_float4(0.f, 0.f, 0.f, 0.f);
        float mn[NACC];  // min over this lane's fast-test values per accumulator
#pragma unroll
        for (int c = 0; c < NACC; c++) mn[c] = INF;
        // fast-test values v = 16 acc + reg; QG = 2: both accumulators share the rows
        auto epi_y = [&](int v) -> float {
            const int acc = v >> 4, reg = v & 15, ta = rg_of(acc);
            if ((reg & 3) == 0 && (RG == 2 || acc == 0))
                t4[ta] = *reinterpret_cast<const float4*>(tnpY + 32 * ta + 8 * (reg >> 2) + 4 * h);
            return fmaf(-2.0f, Y[acc][reg], f4get(t4[ta], reg & 3));
        };
        if constexpr (BF) {
            // one 32x32x16 MFMA per 16-B fragment: prefetch the A fragments PF k-steps ahead
            // and interleave the previous tile's fast test between the MFMAs
            constexpr int PF = FILTER_PF / NACC;  // covers ~FILTER_PF x 32 MFMA cycles of LDS latency
            uint4 xa[NS], xb[NS];
#pragma unroll
            for (int s = 0; s < PF && s < NS; s++) {
                xa[s] = *reinterpret_cast<const uint4*>(a0p + 32 * s);
                if (RG == 2) xb[s] = *reinterpret_cast<const uint4*>(a1p + 32 * s);
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
                    if constexpr (SPLIT) {
                        // rows are [hi | lo]: steps s < NS/2 read t_hi (x q_hi, then x q_lo),
                        // steps s >= NS/2 read t_lo (x q_hi); lo x lo is left out (certificate)
                        constexpr int H2 = NS / 2;
                        const int sq = s < H2 ? s : s - H2;
                        X[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                            A, __builtin_bit_cast(bf16x8, qf[qg_of(c)][sq]), X[c], 0, 0, 0);
                        if (s < H2)
                            X[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                A, __builtin_bit_cast(bf16x8, qf[qg_of(c)][s + H2]), X[c], 0, 0, 0);
                    } else {
                        const bf16x8 B = __builtin_bit_cast(bf16x8, qf[qg_of(c)][s]);
                        X[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, X[c], 0, 0, 0);
                    }
#pragma unroll
                    for (int vv = 0; vv < VPS; vv++) {
                        if (!KNN_STUDY_NO_EPI) {
                            const float y = epi_y(16 * c + s * VPS + vv);
                            asm volatile("" ::"v"(y));  // computed here, beside this MFMA
                            mn[c] = fminf(mn[c], y);
                        } else {
                            asm volatile("" ::"v"(Y[c][(s * VPS + vv) & 15]));
                        }
                    }
                }
                __builtin_amdgcn_sched_barrier(0);  // keep this k-step's order (prefetch, MFMA, VALU)
            }
        } else {
#pragma unroll
            for (int s = 0; s < NS; s++) {
                dma_at(s, dma_on, dd);
                const uint4 x0 = *reinterpret_cast<const uint4*>(a0p + 32 * s);
                const uint4 x1 = RG == 2 ? *reinterpret_cast<const uint4*>(a1p + 32 * s) : x0;
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
#pragma unroll
                    for (int c = 0; c < NACC; c++)
                        X[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(u4getf((RG == 2 && c) ? x1 : x0, jj),
                                                                    u4getf(qf[qg_of(c)][s], jj), X[c], 0, 0, 0);
                }
#pragma unroll
                for (int c = 0; c < NACC; c++)
#pragma unroll
                    for (int vv = 0; vv < VPS; vv++) {
                        if (!KNN_STUDY_NO_EPI) mn[c] = fminf(mn[c], epi_y(16 * c + s * VPS + vv));
                        else asm volatile("" ::"v"(Y[c][(s * VPS + vv) & 15]));
                    }
            }
        }
        bool any = false;
#pragma unroll
        for (int c = 0; c < NACC; c++) any |= mn[c] <= tf[qg_of(c)];
        return __ballot(any) != 0ull;
    };

    // exact re-check of tile tp (accumulators Y) for the values whose fast test passed:
    // a bit-mask pass, then a wave-uniform loop over the set bits (the value is picked by
    // a select chain, so the accumulators are never indexed dynamically)
    // keep candidate (L, U) of global row t for query group g of this lane: the exact test
    // against the current threshold, the candidate store into this lane half's sub-slice,
    // and, if U beats the heap root, a sift-down of the 4-ary max-heap (node n >= 1 in
    // H[n-1], the root in H[hs-1]: the four children 4i+1..4i+4 of node i are one aligned
    // 16-byte read at H[4i]).  Only one lane of a query may run it at a time.
    auto accept = [&](float L, float U, int64_t t, bool g1) __attribute__((always_inline)) {
        float& th = g1 ? thr[QG - 1] : thr[0];
        if (!(L <= th)) return;
        int& slot = g1 ? ccnt[QG - 1] : ccnt[0];
        if (slot < cap_sub) {
            const int64_t qq = g1 ? q[QG - 1] : q[0];
            const int64_t o = qq * (int64_t)a.cap + (int64_t)(2 * seg + h) * cap_sub + slot;
            a.cand[o] = CandRec{(int32_t)t, L, U};
        }
        slot++;
        float& rt = g1 ? root[QG - 1] : root[0];
        if (U < rt) {
            float* H = topU + (g1 ? jl[QG - 1] : jl[0]) * hs;
            int i = 0;
            float newroot = U;
            for (;;) {
                if (4 * i + 1 > k - 1) break;
                const float4 cc = *reinterpret_cast<const float4*>(H + 4 * i);
                const float m01 = fmaxf(cc.x, cc.y), m23 = fmaxf(cc.z, cc.w);
                const float cm = fmaxf(m01, m23);
                if (cm <= U) break;
                const int ci = cm == cc.x ? 0 : cm == cc.y ? 1 : cm == cc.z ? 2 : 3;
                H[i == 0 ? hs - 1 : i - 1] = cm;
                if (i == 0) newroot = cm;
                i = 4 * i + 1 + ci;
            }
            H[i == 0 ? hs - 1 : i - 1] = U;
            rt = newroot;
            th = fminf(th, rt);
        }
    };
    // after a round of accepts: the partner lane takes the root, thresholds tighten
    auto sync_roots = [&](int hh) __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < QG; g++) {
            const float other = __shfl_xor(root[g], 32);
            if (h != hh) root[g] = other;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    };
    auto publish = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < QG; g++) {
            if (qvalid[g]) {
                thr[g] = fminf(thr[g], root[g]);
                // publish for the other segments of this query (single segment: nobody reads it)
                if (a.nseg > 1 && h == 0 && thr[g] < published[g]) {
                    atomicMin(&a.gthr[q[g]], f2o(thr[g]));
                    published[g] = thr[g];
                }
                tf[g] = make_tf(g, thr[g]);
            }
        }
    };
    // fast-test pass bits of tile tp's accumulators Y (bit v = value v)
    auto pass_mask = [&](floatx16 (&Y)[NACC], int tp) -> uint32_t {
        const float* tnpY = ring + (tp % NR) * 2 * BN;
        uint32_t m = 0;  // built high to low with shift-or (no literals)
#pragma unroll
        for (int v4 = NV / 4 - 1; v4 >= 0; v4--) {
            const int acc = v4 >> 2, rq = v4 & 3;
            const float4 t4 = *reinterpret_cast<const float4*>(tnpY + 32 * rg_of(acc) + 8 * rq + 4 * h);
            const float tfa = tf[qg_of(acc)];
#pragma unroll
            for (int e = 3; e >= 0; e--)
                m = (m << 1) | (uint32_t)(fmaf(-2.0f, Y[acc][4 * rq + e], f4get(t4, e)) <= tfa);
        }
        return m;
    };
    // exact (L, U, row) of value b of tile tp (a select tree on the bits of b: the
    // accumulators are never indexed dynamically)
    auto value_lu = [&](floatx16 (&Y)[NACC], int tp, int b, float& L, float& U, int64_t& t, bool& g1) {
        float lv[NV];
#pragma unroll
        for (int v = 0; v < NV; v++) lv[v] = Y[v >> 4][v & 15];
#pragma unroll
        for (int lvl = 0; (NV >> (lvl + 1)) >= 1; lvl++) {
            const bool hi = (b >> lvl) & 1;
#pragma unroll
            for (int v = 0; v < (NV >> (lvl + 1)); v++) lv[v] = hi ? lv[2 * v + 1] : lv[2 * v];
        }
        const int reg = b & 15;
        const int row = 32 * rg_of(b >> 4) + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        g1 = QG == 2 && qg_of(b >> 4);
        const float s = (g1 ? qn[QG - 1] : qn[0]) + ring[(tp % NR) * 2 * BN + BN + row];
        const float G = fmaf(-2.0f, lv[0], s);
        const float dl = fmaf(coef, s, eta);
        L = G - dl;
        U = G + dl;
        const int64_t tt = row_begin + (int64_t)tp * BN + row;
        t = tt < row_end ? tt : -1;
    };

    // immediate slow path: every passing value of tile tp is accepted now
    auto slow = [&](floatx16 (&Y)[NACC], int tp) {
        const uint32_t m = pass_mask(Y, tp);
        // the two lanes of a query take turns, so each heap has one writer at a time; the
        // candidate slot counters are per lane (each lane half owns a sub-slice)
        for (int hh = 0; hh < 2; hh++) {
            uint32_t mm = (h == hh) ? m : 0u;
            while (__ballot(mm != 0u)) {
                if (mm != 0u) {
                    const int b = __builtin_ctz(mm);
                    mm &= mm - 1u;
                    float L, U;
                    int64_t t;
                    bool g1;
                    value_lu(Y, tp, b, L, U, t, g1);
                    if (t >= 0) accept(L, U, t, g1);
                }
            }
            sync_roots(hh);
        }
        publish();
    };

    // deferred slow path (8-wave shape): passing values are only recorded -- exact (L, U,
    // row) into a small per-lane register queue, no LDS chain, no global stores -- and the
    // queue is flushed through accept() every DEFER_EVERY tiles by every wave at the same
    // tile (one wave's heap work then no longer holds the other seven at each barrier),
    // or at once when some lane's queue is full.  A threshold that waits for the flush is
    // stale but still valid (it only ever tightens).
    constexpr int RQ = FILTER_RQ;
    float qL[RQ], qU[RQ];
    int qT[RQ];
    bool qG[RQ];
    int qcnt = 0;
#pragma unroll
    for (int i = 0; i < RQ; i++) { qL[i] = qU[i] = 0.f; qT[i] = 0; qG[i] = false; }
    auto flush = [&]() __attribute__((always_inline)) {
        for (int hh = 0; hh < 2; hh++) {
#pragma unroll
            for (int i = 0; i < RQ; i++) {
                const bool mine = h == hh && i < qcnt;
                if (__ballot(mine) && mine) accept(qL[i], qU[i], (int64_t)qT[i], qG[i]);
            }
            sync_roots(hh);
        }
        qcnt = 0;
        publish();
    };
    auto record = [&](floatx16 (&Y)[NACC], int tp) {
        uint32_t mm = pass_mask(Y, tp);
        while (__ballot(mm != 0u)) {
            if (__ballot(qcnt >= RQ && mm != 0u)) flush();
            if (mm != 0u) {
                const int b = __builtin_ctz(mm);
                mm &= mm - 1u;
                float L, U;
                int64_t t;
                bool g1;
                value_lu(Y, tp, b, L, U, t, g1);
                if (t >= 0 && L <= (g1 ? thr[QG - 1] : thr[0])) {
#pragma unroll
                    for (int i = 0; i < RQ; i++)
                        if (i == qcnt) { qL[i] = L; qU[i] = U; qT[i] = (int)t; qG[i] = g1; }
                    qcnt++;
                }
            }
        }
    };

    const int ntiles = (row_end > row_begin) ? (int)((row_end - row_begin + BN - 1) / BN) : 0;
    floatx16 accA[NACC], accB[NACC];
#pragma unroll
    for (int c = 0; c < NACC; c++) accA[c] = accB[c] = floatx16{};
    __syncthreads();  // LDS init above is complete before any DMA lands
#pragma unroll
    for (int p = 0; p < NBUF - 1; p++)
        if (p < ntiles) dma_tile(p, p, row_begin + (int64_t)p * BN);
    // the step issues the next tile's DMA between its MFMAs: it must land by the next barrier
    constexpr bool DEFER = NW == 8;  // deferred slow path (see record())
    constexpr int DEFER_EVERY = FILTER_DEFER_EVERY;
    auto iter = [&](floatx16 (&X)[NACC], floatx16 (&Y)[NACC], int it) {
        const int64_t r0 = row_begin + (int64_t)it * BN;
        if ((it & 63) == 63 && a.nseg > 1) {
            // pick up thresholds published by other segments (the value is waited on here)
#pragma unroll
            for (int g = 0; g < QG; g++) {
                if (qvalid[g]) {
                    const float gv = o2f(__hip_atomic_load(&a.gthr[q[g]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    if (gv < thr[g]) { thr[g] = gv; tf[g] = make_tf(g, thr[g]); }
                }
            }
        }
        // tile it landed; every wave is done with the buffer / ring slot the next DMA
        // overwrites (tile it-1's, read last iteration)
        wait_dma_barrier();
        const bool dma_on = !KNN_STUDY_NO_DMA && it + NBUF - 1 < ntiles;
        const DmaTile dd = dma_desc((it + NBUF - 1) % NBUF, (it + NBUF - 1) % NR, r0 + (int64_t)(NBUF - 1) * BN);
        const bool any = step(X, Y, it % NBUF, (it + NR - 1) % NR, dma_on, dd);
        if (!KNN_STUDY_NO_SLOW) {
            if constexpr (DEFER) {
                if (any && it > 0) record(Y, it - 1);
                if ((it & (DEFER_EVERY - 1)) == DEFER_EVERY - 1 && __ballot(qcnt > 0)) flush();
            } else if (any && it > 0) {
                slow(Y, it - 1);
            }
        } else if (any) {
            asm volatile("" ::"v"(Y[0][0]), "v"(Y[NACC - 1][3]));
        }
    };
    for (int it = 0; it < ntiles; it += 2) {
        iter(accA, accB, it);
        if (it + 1 < ntiles) iter(accB, accA, it + 1);
    }
    if (ntiles > 0) {
        // drain: the last tile's accumulators are in accA (ntiles odd) or accB (even)
        const int last = ntiles - 1;
        // one static binding per branch: a runtime-selected reference to a register array
        // would put both accumulator sets in scratch memory
        auto drain = [&](floatx16 (&L)[NACC]) {
            bool any = false;
            const float* tnpL = ring + (last % NR) * 2 * BN;
#pragma unroll
            for (int v = 0; v < NV; v++) {
                const int acc = v >> 4, reg = v & 15;
                const int row = 32 * rg_of(acc) + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                any |= fmaf(-2.0f, L[acc][reg], tnpL[row]) <= tf[qg_of(acc)];
            }
            if (__ballot(any)) {
                if constexpr (DEFER) record(L, last);
                else slow(L, last);
            }
        };
        if (last & 1) drain(accB);
        else drain(accA);
    }
    if constexpr (DEFER) {
        if (__ballot(qcnt > 0)) flush();
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < QG; g++)
        if (qvalid[g]) a.cnt[(int64_t)(2 * seg + h) * a.nq + q[g]] = ccnt[g];
}

// ---------------------------------------------------------------------------------
// k_rescore<R, CAPW, E>: one wave per query.  Final threshold = the k-th smallest U among
// the query's candidates; candidates with L <= threshold are rescored with the exact
// direct form and selected by key.  Queries whose list overflowed (or holds < k entries)
// go to the exact fallback list.
//  * The candidates sit in a.nseg (<= 64) sub-slices of cap_seg entries; compact entry e
//    maps to (slice, offset) through the slices' prefix sums.  Their ordered U bits are
//    staged in LDS (su, <= 64 CAPW words), so the bisection reads only the entries that
//    exist, in ceil(total / 64) ballots per round, and between the wave's smallest and
//    largest U instead of over all 2^32 values.
//  * The survivors (L <= threshold) reuse su as their compact index list.
// LDS per wave: q row [ld_pad] f32 | counts [C] i32 (C <= KNN_VOTE_LDS_MAX_C) | su [su_cap]
// ---------------------------------------------------------------------------------
#if KNN_FUSED_STAMPS
// study build (KNN_STUDY_STAMPS): per-query phase cycles of k_rescore, written (plain vector
// stores, no shared counter) into a caller's [nq][10] u64 buffer -- [0] fill counts, [1]
// records staged, [2] bisection, [3] compaction, [4] survivor distances, [5] selection + vote,
// [6] 1, [7] survivors, [8] record batches, [9] bisection rounds
__device__ unsigned long long* g_knn_rst_buf;
__device__ long long g_knn_rst_n;
extern "C" int knn_debug_rescore_stamps_buffer(void* buf, long long n) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_knn_rst_buf), &buf, sizeof(buf)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_knn_rst_n), &n, sizeof(n)) == hipSuccess ? 0 : -1;
}
#endif

template <int R, int CAPW, typename E>
__device__ __forceinline__ void rescore_query(const RescoreArgs& a, const int64_t q, unsigned char* my) {
    [[maybe_unused]] uint64_t rst[7] = {};
    [[maybe_unused]] int rounds = 0;
    auto rstamp = [&](int i) __attribute__((always_inline)) {
        if constexpr (KNN_FUSED_STAMPS) rst[i] = __builtin_amdgcn_s_memtime();
    };
    rstamp(0);
    const int lane = lane_id();
    float* qs = reinterpret_cast<float*>(my);
    int* counts = a.c_lds_bytes ? reinterpret_cast<int*>(my + a.q_lds_bytes) : nullptr;  // NULL: vote_ballot
    uint32_t* su = reinterpret_cast<uint32_t*>(my + a.q_lds_bytes + a.c_lds_bytes);
    // sub-slice fills: lane sg < nseg (<= 64) holds slice sg's; inclusive prefix over the wave.
    // Read before the gate and status words (allocated either way), so the three loads
    // share one round trip.
    const int cs = lane < a.nseg ? a.cnt[(int64_t)lane * a.nq + q] : 0;
    // the filter's final bound for this query (ordered bits; the same round trip as the fills)
    const uint32_t tbits = a.gthr ? a.gthr[__builtin_amdgcn_readfirstlane((int)q)] : 0u;  // (scalar load)
    if (a.gate && *a.gate == 0) return;  // a gated stage (AUTO's re-run) that is not taken
    if (*a.status & KNN_STATUS_GEMM_UNSAFE) {
        // a norm too large for the certificate: every query takes the exact scan
        if (lane == 0) a.fb_list[atomicAdd(a.fb_count, 1)] = (int32_t)q;
        return;
    }
    const int k = a.k;
    const E* train = reinterpret_cast<const E*>(a.train);
    const E* test = reinterpret_cast<const E*>(a.test);
    const bool overflow = __ballot(cs > a.cap_seg) != 0ull;
    int incl = cs;
#pragma unroll
    for (int j = 1; j < 64; j <<= 1) {
        const int o = __shfl_up(incl, j);
        if (lane >= j) incl += o;
    }
    const int total = __shfl(incl, 63);
    rstamp(1);
    if (overflow || total < k) {
        if (lane == 0) a.fb_list[atomicAdd(a.fb_count, 1)] = (int32_t)q;
        return;
    }
    // the query row into LDS now: its loads overlap the candidate reads below
    for (int i = lane; i < a.d; i += 64) qs[i] = widen(test[q * a.ld_q + i]);
    const int excl = incl - cs;
    const int64_t qbase = q * (int64_t)a.cap;
    // candidate position of compact entry e: slice = last sg with excl[sg] <= e
    auto position = [&](int e) __attribute__((always_inline)) -> int64_t {
        int sg = 0, base = 0;
        for (int s2 = 1; s2 < a.nseg; s2++) {  // uniform loop, <= 63 steps
            const int ex = __builtin_amdgcn_readlane(excl, s2);
            if (e >= ex) { sg = s2; base = ex; }
        }
        return qbase + (int64_t)sg * a.cap_seg + (e - base);
    };
    const int nreg = (total + 63) >> 6;  // <= CAPW (total <= nseg * cap_seg <= cap)
    // entries e < su_cap are staged in LDS; a longer list (rare: su_cap is sized ~3x the
    // expected count) re-reads the rest from the candidate arrays in each bisection round
    const int su_cap = a.su_cap;
    int m = 0;
    [[maybe_unused]] auto rstamps_flush = [&]() __attribute__((always_inline)) {
#if KNN_FUSED_STAMPS
        rstamp(6);
        unsigned long long* o = g_knn_rst_buf;
        if (o && q < g_knn_rst_n && lane < 10) {
            const unsigned long long v = lane < 6 ? (unsigned long long)(rst[lane + 1] - rst[lane])
                                       : lane == 6 ? 1ull : lane == 7 ? (unsigned long long)m
                                       : lane == 8 ? (unsigned long long)nreg : (unsigned long long)rounds;
            o[q * 10 + lane] = v;
        }
#endif
    };
    // survivors' indices in su[0, m): exact distances, selection, vote
    auto finish_selection = [&](const int m) __attribute__((always_inline)) {
        u64 T[R];
#pragma unroll
        for (int r = 0; r < R; r++) T[r] = KEY_NONE;
        if (m <= 64) {
            // one batch (the common case): each survivor's rank among the m keys by a scalar
            // broadcast loop, then one permute puts key r in lane r -- the sorted list without the
            // bitonic network's 40-odd cross-lane shuffles.  Keys are distinct (the index breaks
            // ties); an infinite distance gets the key ~0 << 32 | idx (after every finite key,
            // distinct) and reads KEY_NONE again after the permute.
            const uint32_t t = lane < m ? su[lane] : 0u;
            // the survivor's label now: its load lands under the distance's row loads (no
            // dependent label read after the selection)
            const int lab = lane < m ? a.labels[t] : -1;
            u64 key = KEY_NONE;
            // few survivors: G = d / 32 lanes per row, each row read in one round trip
            const int G = a.d >> 5;
            const bool mis = lane < m && ((uintptr_t)(train + (int64_t)t * a.ld_t) & (4 * sizeof(E) - 1)) != 0;
            // (k <= 32 implies R == 1: the larger lists' instances do not carry its registers)
            if (R == 1 && (a.d & 31) == 0 && G >= 2 && m * G <= 64 && !__ballot(mis)) {
                const int r = lane / G, p = lane - r * G;
                const uint32_t tr = (uint32_t)__shfl((int)t, r < m ? r : 0);
                const float part = direct_dist_grouped(qs, train + (int64_t)tr * a.ld_t, r < m, p, G);
                const float dist = __shfl(part, (lane < m ? lane : 0) * G + G - 1);
                if (lane < m) key = make_key(dist, t);
            } else if (lane < m) {
                key = make_key(direct_dist_batched(qs, train + (int64_t)t * a.ld_t, a.d), t);
            }
            if (lane < m && key == KEY_NONE) key = 0xffffffff00000000ull | t;
            if constexpr (KNN_FUSED_STAMPS) {
                (void)__ballot(key != 0ull);  // (the distances are in registers before the stamp)
                rstamp(5);
            }
            int rank = 0;
            for (int jj = 0; jj < m; jj++) {
                const u64 kj = ((u64)__builtin_amdgcn_readlane((uint32_t)(key >> 32), jj) << 32) |
                               (u64)__builtin_amdgcn_readlane((uint32_t)key, jj);
                rank += kj < key ? 1 : 0;
            }
            const int dst = 4 * (lane < m ? rank : lane);
            const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)key);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)(key >> 32));
            T[0] = hi == 0xffffffffu ? KEY_NONE : (((u64)hi << 32) | lo);
            const int labp = __builtin_amdgcn_ds_permute(dst, lab);
            finish_query<R>(T, k, a.C, a.labels, counts, q, a.out, a.status, &labp);
            rstamps_flush();
            return;
        } else {
            rstamp(5);
            u64 kth = KEY_NONE;
            for (int b = 0; b < m; b += 64) {
                u64 key = KEY_NONE;
                if (b + lane < m) {
                    const int32_t t = (int32_t)su[b + lane];
                    key = make_key(direct_dist_batched(qs, train + (int64_t)t * a.ld_t, a.d), (uint32_t)t);
                }
                const bool pass = key < kth;
                if (__ballot(pass)) {
                    topk_merge<R>(T, pass ? key : KEY_NONE);
                    kth = list_at(T, k - 1);
                }
            }
        }
        finish_query<R>(T, k, a.C, a.labels, counts, q, a.out, a.status);
        rstamps_flush();
    };
    // Staged selection (the fused filter: a.gthr).  tb = the filter's final bound for this
    // query, >= the k-th smallest U of all its candidates; a candidate with L > tb cannot
    // survive (a true neighbour has L <= D <= D_(k) <= tb), and every candidate with U <= the
    // k-th smallest U has L <= tb, so the k-th smallest U of the staged set is the same value.
    // One pass over the records stages {U, L, idx} of those (B: ~90 of ~550) in LDS; the
    // bisection and the survivors then work on at most 4 register batches of them.  More than
    // CS staged: the general path below (every candidate's U in su).
    const int CS = min(4 * 64, (su_cap / 3) & ~63);
    bool staged = false;
    if (a.gthr && CS >= 64) {
        const float tb = o2f(tbits);
        uint32_t* cu = su;
        float* cl = reinterpret_cast<float*>(su + CS);
        int32_t* ci = reinterpret_cast<int32_t*>(su + 2 * CS);
        int nc = 0;
        constexpr int RS = 4;  // record batches in flight per chunk
        for (int i0 = 0; i0 < nreg; i0 += RS) {
            CandRec rc[RS];
#pragma unroll
            for (int jj = 0; jj < RS; jj++) {
                const int e = lane + 64 * (i0 + jj);
                const int64_t o = i0 + jj < nreg ? position(e) : 0;  // (uniform: every lane calls it)
                rc[jj] = (i0 + jj < nreg && e < total) ? a.cand[o] : CandRec{0, 0.0f, 0.0f};
            }
#pragma unroll
            for (int jj = 0; jj < RS; jj++) {
                if (i0 + jj >= nreg) break;
                const int e = lane + 64 * (i0 + jj);
                const bool pass = e < total && rc[jj].L <= tb;
                const u64 bal = __ballot(pass);
                const int slot = nc + __popcll(bal & ((1ull << lane) - 1ull));
                if (pass && slot < CS) {
                    cu[slot] = f2o(rc[jj].U);
                    cl[slot] = rc[jj].L;
                    ci[slot] = rc[jj].idx;
                }
                nc += __popcll(bal);
            }
        }
        if (nc <= CS && nc >= k) {
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const int nbc = (nc + 63) >> 6;
            uint32_t ub[4];
            float lb[4];
            int32_t ib[4];
            uint32_t cmin = 0xffffffffu, cmax = 0u;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int e = lane + 64 * b;
                const bool v = b < nbc && e < nc;
                ub[b] = v ? cu[e] : 0xffffffffu;
                lb[b] = v ? cl[e] : __uint_as_float(0x7f800000u);
                ib[b] = v ? ci[e] : 0;
                cmin = min(cmin, ub[b]);
                cmax = v ? max(cmax, ub[b]) : cmax;
            }
#pragma unroll
            for (int j = 32; j > 0; j >>= 1) {
                cmin = min(cmin, (uint32_t)__shfl_xor((int)cmin, j));
                cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, j));
            }
            rstamp(2);
            uint32_t lo = cmin, hi = cmax;
            while (hi - lo > 1024u) {
                const uint32_t mid = lo + ((hi - lo) >> 1);
                int c = 0;
#pragma unroll
                for (int b = 0; b < 4; b++)
                    if (b < nbc) c += __popcll(__ballot(ub[b] <= mid));
                if (c >= k) hi = mid; else lo = mid + 1;
                if constexpr (KNN_FUSED_STAMPS) rounds++;
            }
            const float thr = o2f(hi);
            rstamp(3);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();  // every staged entry is in registers: su is free
            m = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                if (b >= nbc) break;
                const bool sv = lb[b] <= thr;
                const u64 bal = __ballot(sv);
                const int slot = m + __popcll(bal & ((1ull << lane) - 1ull));
                if (sv) su[slot] = (uint32_t)ib[b];
                m += __popcll(bal);
            }
            staged = true;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();  // (su is rewritten below)
    }
    // General path: every candidate's U staged in su (entries past su_cap re-read), the
    // bisection over all of them, then the survivors.
    if (!staged) {
        uint32_t umin = 0xffffffffu, umax = 0u;
        // the first RC batches of records stay in registers: all their loads are issued before
        // the first use, and the compaction below reads L and idx from them, not memory
        constexpr int RC = 4;
        CandRec cr[RC];
#pragma unroll
        for (int i = 0; i < RC; i++) {
            const int e = lane + 64 * i;
            const int64_t o = position(e);
            cr[i] = CandRec{0, 0.0f, 0.0f};
            if (i < nreg && e < total) cr[i] = a.cand[o];
        }
#pragma unroll
        for (int i = 0; i < RC; i++) {
            const int e = lane + 64 * i;
            if (i < nreg && e < total) {
                const uint32_t u = f2o(cr[i].U);
                if (e < su_cap) su[e] = u;
                umin = min(umin, u);
                umax = max(umax, u);
            }
        }
        // batches past RC: their U values in chunks of RCH loads in flight (one round trip per
        // chunk instead of one per batch: B's 552 rows per query are 9 batches)
        constexpr int RCH = 4;
        for (int i0 = RC; i0 < nreg; i0 += RCH) {
            uint32_t uc[RCH];
#pragma unroll
            for (int jj = 0; jj < RCH; jj++) {
                const int e = lane + 64 * (i0 + jj);
                const int64_t o = i0 + jj < nreg ? position(e) : 0;  // (uniform: every lane calls it)
                uc[jj] = (i0 + jj < nreg && e < total) ? f2o(a.cand[o].U) : 0u;
            }
#pragma unroll
            for (int jj = 0; jj < RCH; jj++) {
                const int e = lane + 64 * (i0 + jj);
                if (i0 + jj < nreg && e < total) {
                    if (e < su_cap) su[e] = uc[jj];
                    umin = min(umin, uc[jj]);
                    umax = max(umax, uc[jj]);
                }
            }
        }
#pragma unroll
        for (int j = 32; j > 0; j >>= 1) {
            umin = min(umin, (uint32_t)__shfl_xor((int)umin, j));
            umax = max(umax, (uint32_t)__shfl_xor((int)umax, j));
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        rstamp(2);
        // the threshold: the smallest x with #{U <= x} >= k, or any x above it -- every x >= it
        // is a valid bound (it only admits more survivors) -- so the bisection stops at 2^10
        // ordered-float steps (2^-13 relative), far inside the certificate's band
        // the register-resident batches count from their own U bits (no LDS round trip per round)
        uint32_t ur[RC];
#pragma unroll
        for (int i = 0; i < RC; i++) ur[i] = (i < nreg && lane + 64 * i < total) ? f2o(cr[i].U) : 0xffffffffu;
        uint32_t lo = umin, hi = umax;
        while (hi - lo > 1024u) {
            const uint32_t mid = lo + ((hi - lo) >> 1);
            int c = 0;
#pragma unroll
            for (int i = 0; i < RC; i++)
                if (i < nreg) c += __popcll(__ballot(lane + 64 * i < total && ur[i] <= mid));
            for (int i = RC; i < nreg; i++) {
                const int e = lane + 64 * i;
                // position() shuffles across the wave: every lane calls it (wave-uniform branch)
                const int64_t o = 64 * i + 63 >= su_cap ? position(e) : 0;
                uint32_t u = 0xffffffffu;
                if (e < total) u = e < su_cap ? su[e] : f2o(a.cand[o].U);
                c += __popcll(__ballot(e < total && u <= mid));
            }
            if (c >= k) hi = mid; else lo = mid + 1;
            if constexpr (KNN_FUSED_STAMPS) rounds++;
        }
        const float thr = o2f(hi);
        rstamp(3);
        // compact survivors L <= thr into su (a write never overtakes an unread entry; more
        // survivors than su holds -- pathological ties -- send the query to the exact scan)
        m = 0;
        auto compact = [&](int i, const CandRec& r) __attribute__((always_inline)) {
            const int e = lane + 64 * i;
            const bool sv = e < total && r.L <= thr;
            const int32_t t = sv ? r.idx : 0;
            const u64 bal = __ballot(sv);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const int slot = m + __popcll(bal & ((1ull << lane) - 1ull));
            if (sv && slot < su_cap) su[slot] = (uint32_t)t;
            m += __popcll(bal);
        };
#pragma unroll
        for (int i = 0; i < RC; i++)  // static indices: the records stay in registers
            if (i < nreg) compact(i, cr[i]);
        for (int i0 = RC; i0 < nreg; i0 += RCH) {  // (chunks of RCH record loads in flight)
            CandRec rc[RCH];
#pragma unroll
            for (int jj = 0; jj < RCH; jj++) {
                const int e = lane + 64 * (i0 + jj);
                const int64_t o = i0 + jj < nreg ? position(e) : 0;
                rc[jj] = (i0 + jj < nreg && e < total) ? a.cand[o] : CandRec{0, 0.0f, 0.0f};
            }
#pragma unroll
            for (int jj = 0; jj < RCH; jj++)
                if (i0 + jj < nreg) compact(i0 + jj, rc[jj]);
        }
        if (m > su_cap) {
            if (lane == 0) a.fb_list[atomicAdd(a.fb_count, 1)] = (int32_t)q;
            return;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    rstamp(4);
    finish_selection(m);
}

// GATED (AUTO's re-run, a.gate set): a bounded grid strides over the queries, so a re-run not
// taken costs a few thousand empty waves, not nq / 4 blocks.  The ungated instance keeps one
// query per wave and no loop (the loop in the hot instance cost A 0.26 -> 0.37 ms, r04j).
// (6 waves per SIMD for the k <= 512 instances: the staged selection left the f32 k <= 64
// instance at 81 VGPRs, one over the 6-wave budget)
template <int R, int CAPW, typename E, bool GATED>
__global__ __launch_bounds__(256, (R <= 8 && !GATED) ? 6 : 1) void k_rescore(RescoreArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    unsigned char* my = smem + (size_t)wave * a.wave_lds_bytes;
    if constexpr (GATED) {
        if (*a.gate == 0) return;
        for (int64_t q = (int64_t)blockIdx.x * 4 + wave; q < a.nq; q += (int64_t)gridDim.x * 4)
            rescore_query<R, CAPW, E>(a, q, my);
    } else {
        const int64_t q = (int64_t)blockIdx.x * 4 + wave;
        if (q < a.nq) rescore_query<R, CAPW, E>(a, q, my);
    }
}


// ---------------------------------------------------------------------------------
// k_merge_vote<R>: train-sharded runs.  Each of nsrc train shards gives
// every query its exact k nearest rows as (dist bits, global idx, label), ascending.
// One wave per query merges the nsrc*k keys with the same wave list, so ties keep the
// lower GLOBAL index exactly like the reference's serial scan over the whole train set,
// then votes over the k winners: a shard's winners are a prefix of its list, found by
// key <= the k-th key.  LDS per wave: counts [C] i32.  A source list must ascend by (dist,
// idx) (the merge reads it in sorted runs and stops at the first batch that cannot pass):
// every batch it reads is checked (adjacent lanes, and its first key against the previous
// batch's last) and a descent sets KNN_STATUS_UNSORTED (knn_merge_vote_device: KNN_EINVAL).
// ---------------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(256) void k_merge_vote(MergeArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    // per-wave LDS: class counts [Cpad] (C <= KNN_VOTE_LDS_MAX_C), else the k winners'
    // labels [k] + an append counter (vote_ballot)
    const bool lds_counts = a.C <= KNN_VOTE_LDS_MAX_C;
    int* counts = reinterpret_cast<int*>(smem) + wave * merge_wave_words(a.C, a.k);
    const int64_t q = (int64_t)blockIdx.x * 4 + wave;
    if (q >= a.nq) return;
    const int k = a.k;
    u64 T[R];
#pragma unroll
    for (int r = 0; r < R; r++) T[r] = KEY_NONE;
    u64 kth = KEY_NONE;
    bool unsorted = false;
    for (int s = 0; s < a.nsrc; s++) {
        const int32_t* rec = a.rec + ((int64_t)s * a.nq + q) * 3 * k;
        u64 last = 0;  // the previous batch's last key
        for (int e0 = 0; e0 < k; e0 += 64) {
            const int e = e0 + lane;
            u64 key = KEY_NONE;
            if (e < k) {
                const int32_t ix = rec[k + e];
                if (ix >= 0) key = make_key(__int_as_float(rec[e]), (uint32_t)ix);
            }
            {
                const int pl = lane == 0 ? 0 : lane - 1;
                const u64 prev = lane == 0 ? last
                                           : (((u64)(uint32_t)__shfl((int)(uint32_t)(key >> 32), pl) << 32) |
                                              (u64)(uint32_t)__shfl((int)(uint32_t)key, pl));
                if (__ballot(key < prev)) unsorted = true;
                last = (((u64)(uint32_t)__shfl((int)(uint32_t)(key >> 32), 63) << 32) |
                        (u64)(uint32_t)__shfl((int)(uint32_t)key, 63));
            }
            // a source list ascends by key (a shard's exact top-k, or a segment's), so a batch
            // is a sorted run: passing keys are its prefix, none past the first that fails
            const bool pass = key < kth;
            if (!__ballot(pass)) break;
            topk_merge_sorted<R>(T, pass ? key : KEY_NONE);
            kth = list_at(T, k - 1);
        }
    }
    if (unsorted && lane == 0) atomicOr(a.status, KNN_STATUS_UNSORTED);
    if (a.labels) {
        // segments of one train set (k_direct_tile): indices are local rows of a.labels
        finish_query<R>(T, k, a.C, a.labels, lds_counts ? counts : nullptr, q, a.out, a.status);
        return;
    }
    const bool bad = (kth == KEY_NONE);
    const QueryOut& o = a.out;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int e = 64 * r + lane;
        if (e < k) {
            const int64_t off = q * o.stride + e;
            const u64 key = T[r];
            if (o.dist) o.dist[off] = key == KEY_NONE ? FLT_MAX : __uint_as_float((uint32_t)(key >> 32));
            if (o.idx) o.idx[off] = key == KEY_NONE ? -1 : (int32_t)(o.idx_base + (uint32_t)(key & 0xffffffffull));
        }
    }
    if (!o.pred) return;
    if (lds_counts) {
        for (int c = lane; c < a.C; c += 64) counts[c] = 0;
    } else if (lane == 0) {
        counts[k] = 0;  // append counter of the winners' labels
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int s = 0; s < a.nsrc; s++) {
        const int32_t* rec = a.rec + ((int64_t)s * a.nq + q) * 3 * k;
        for (int e = lane; e < k; e += 64) {
            const int32_t ix = rec[k + e];
            if (ix < 0) continue;
            const u64 key = make_key(__int_as_float(rec[e]), (uint32_t)ix);
            if (key <= kth && key != KEY_NONE) {
                const int lab = rec[2 * k + e];
                if (lab >= 0 && lab < a.C) {
                    if (lds_counts) atomicAdd(&counts[lab], 1);
                    else counts[atomicAdd(&counts[k], 1)] = lab;
                } else {
                    atomicOr(a.status, KNN_STATUS_BAD_LABEL);
                }
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    u64 best = 0;
    if (lds_counts) {
        for (int c = lane; c < a.C; c += 64) {
            u64 v = ((u64)(uint32_t)counts[c] << 32) | (u64)(0xffffffffu - (uint32_t)c);
            best = umax64(best, v);
        }
#pragma unroll
        for (int j = 32; j > 0; j >>= 1) best = umax64(best, __shfl_xor(best, j));
    } else {
        const int nw = counts[k];
        int labr[R];
#pragma unroll
        for (int r = 0; r < R; r++) labr[r] = (64 * r + lane < nw) ? counts[64 * r + lane] : -1;
        best = vote_ballot<R>(labr, k);
    }
    if (lane == 0) {
        o.pred[q] = bad ? 0 : (int32_t)(0xffffffffu - (uint32_t)(best & 0xffffffffull));
        if (bad && !KNN_STUDY_RESULTS_INVALID) atomicOr(a.status, KNN_STATUS_TOO_FEW);
    }
}

// ---------------------------------------------------------------------------------
// k_mfma_probe: the bf16 filter's MFMA chain on caller data, for the self-test of the
// certificate's hardware assumption (knn_capi.cpp certificate(): bf16 x bf16 products
// exact, the MFMA's internal sums no worse than 2u per addition, denormals possibly
// flushed).  One wave computes out[i][j] = sum_k a[i][k] b[j][k] (a, b: [32][K] bf16
// bits, K % 16 == 0) exactly as k_gemm_filter does: per 16-wide k-step one
// v_mfma_f32_32x32x16_bf16 accumulating into the same registers, lane l feeding row
// l & 31 / column l & 31 with elements [16s + 8(l >> 5), +8); register r of lane l is
// out[(r & 3) + 8 (r >> 2) + 4 (l >> 5)][l & 31].
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_mfma_probe(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                                   int K, float* __restrict__ out) {
    const int lane = lane_id();
    const int j = lane & 31, h = lane >> 5;
    floatx16 acc = floatx16{};
    for (int s = 0; s < K / 16; s++) {
        const uint4 fa = *reinterpret_cast<const uint4*>(a + (int64_t)j * K + 16 * s + 8 * h);
        const uint4 fb = *reinterpret_cast<const uint4*>(b + (int64_t)j * K + 16 * s + 8 * h);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, fa), __builtin_bit_cast(bf16x8, fb),
                                                      acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; r++) out[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + j] = acc[r];
}

hipError_t knn_launch_mfma_probe(const uint16_t* a, const uint16_t* b, int K, float* out, hipStream_t st) {
    if (K <= 0 || K % 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_mfma_probe, dim3(1), dim3(64), 0, st, a, b, K, out);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

// ---------------------------------------------------------------------------------
// k_generate: the synthetic rows of SURVEY.md 8d (same hash as oracle/knn_oracle.c)
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t gen_hash(uint64_t seed, uint32_t stream, uint64_t row, uint32_t col) {
    uint64_t x = (seed * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)stream * 0xD1B54A32D192ED03ull);
    x += row * 0xA0761D6478BD642Full + (uint64_t)col * 0xE7037ED1A0B428DBull;
    return mix64(x);
}

// kinds 2 / 3 (SURVEY.md 8d's clustered variant): the class centroids' stream, as in
// oracle/knn_oracle.c
#define GEN_CENTROID_STREAM 0xC3u
__device__ __forceinline__ float grid_value(uint32_t u) { return (float)(int32_t)(u >> 8) * (1.0f / 8388608.0f) - 1.0f; }

__global__ __launch_bounds__(256) void k_generate(GenerateArgs a) {
    const int64_t total = a.n * a.ld;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total || i < a.n; i += (int64_t)gridDim.x * 256) {
    if (i < total) {
        int64_t r = i / a.ld;
        int c = (int)(i % a.ld);
        float v = 0.0f;
        if (c < a.d) {
            const uint64_t row = (uint64_t)(a.row0 + r);
            uint32_t u = (uint32_t)(gen_hash(a.seed, a.stream, row, (uint32_t)c) >> 32);
            if (a.kind == 1) {
                v = (float)((int32_t)(u >> 24) - 128) * (1.0f / 128.0f);
            } else if (a.kind >= 2) {
                // clustered: the row's class centroid (stream GEN_CENTROID_STREAM, row = class)
                // plus noise -- kind 2: grid centroid + 0.5 x grid value (exact product, one
                // rounded add, no contraction: pragma below); kind 3: bf16-exact (k1 + k2)/128
                const uint32_t cls = (uint32_t)(gen_hash(a.seed, a.stream, row, 0xFFFFu) >> 32) % (uint32_t)a.C;
                const uint32_t m = (uint32_t)(gen_hash(a.seed, GEN_CENTROID_STREAM, cls, (uint32_t)c) >> 32);
                if (a.kind == 3)
                    v = (float)(((int32_t)(m >> 24) - 128) + ((int32_t)(u >> 26) - 32)) * (1.0f / 128.0f);
                else
                    v = grid_value(m) + 0.5f * grid_value(u);
            } else {
                v = grid_value(u);
            }
        }
        if (a.bf16_out)
            reinterpret_cast<uint16_t*>(a.out)[i] = (uint16_t)(__float_as_uint(v) >> 16);  // exact for kinds 1, 3
        else
            reinterpret_cast<float*>(a.out)[i] = v;
    }
    if (a.labels && i < a.n) {
        uint32_t u = (uint32_t)(gen_hash(a.seed, a.stream, (uint64_t)(a.row0 + i), 0xFFFFu) >> 32);
        a.labels[i] = (int32_t)(u % (uint32_t)a.C);
    }
    }
}

// ---------------------------------------------------------------------------------
// k_confusion: cm[label][pred] += 1 (main.cpp:87-100) and the trace (main.cpp:102-112).
// Integer counts: blocks privatise a C x C matrix in LDS when it fits (C <= 64), so the
// global atomics are one per cell per block; labels / predictions outside [0, C) set
// KNN_STATUS_BAD_LABEL instead of writing out of bounds.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_confusion(const int32_t* __restrict__ pred,
                                                   const int32_t* __restrict__ labels, int64_t n, int C,
                                                   int32_t* __restrict__ cm,
                                                   unsigned long long* __restrict__ correct,
                                                   int32_t* __restrict__ status) {
    __shared__ int32_t lcm[64 * 64];
    const bool priv = C <= 64;
    if (priv)
        for (int i = threadIdx.x; i < C * C; i += 256) lcm[i] = 0;
    __syncthreads();
    unsigned long long ok = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int t = labels[i], p = pred[i];
        if (t < 0 || t >= C || p < 0 || p >= C) { atomicOr(status, KNN_STATUS_BAD_LABEL); continue; }
        ok += (t == p);
        if (priv) atomicAdd(&lcm[t * C + p], 1);
        else atomicAdd(&cm[(int64_t)t * C + p], 1);
    }
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) ok += __shfl_xor(ok, j);
    if ((threadIdx.x & 63) == 0 && ok) atomicAdd(correct, ok);
    __syncthreads();
    if (priv)
        for (int i = threadIdx.x; i < C * C; i += 256)
            if (lcm[i]) atomicAdd(&cm[i], lcm[i]);
}

// ---------------------------------------------------------------------------------
// Device-side control of a predict call (no host round trip inside a call):
//   k_fill_u32     p[0..n) = v when the gate is open (a gated stage's threshold reset)
//   k_rerun_decide AUTO's re-run of the rounded filter as split: open the gate when the
//                  call is not on the exact path and more than `limit` queries fell back,
//                  and reset the fallback list the split run rebuilds
// ctrl: [0] status bits, [1] fallback count, [2] ordered max train norm, [3] re-run gate
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fill_u32(uint32_t* __restrict__ p, int64_t n, uint32_t v,
                                                  const int32_t* __restrict__ gate) {
    if (gate && *gate == 0) return;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}

__global__ void k_rerun_decide(int32_t* ctrl, int64_t limit) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int open = !(ctrl[0] & KNN_STATUS_GEMM_UNSAFE) && (int64_t)ctrl[1] > limit;
    ctrl[3] = open;
    if (open) ctrl[1] = 0;
}

// The end of a call: the status words go straight to the host's mapped (fine-grained) copy and
// are reset for the next call -- one tiny kernel instead of a device-to-host copy (a DMA-engine
// round trip) plus the next call's memset of the words.  Then host[n] = seq, after a system-
// scope release: the host waits for that word (finish_call) instead of the stream's completion
// signal.  Every earlier kernel of the stream has completed, its end-of-kernel release included,
// before this one starts (in-order stream: barrier bit set).
__global__ __launch_bounds__(64) void k_finish(int32_t* __restrict__ ctrl, int32_t* __restrict__ host, int n,
                                               uint32_t seq) {
    const int i = threadIdx.x;
    if (i < n) {
        host[i] = ctrl[i];
        ctrl[i] = 0;
    }
    __syncthreads();
    if (i == 0) {
        __threadfence_system();
        __hip_atomic_store(host + n, (int32_t)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t knn_launch_finish(int32_t* ctrl, int32_t* host_mapped, int n, uint32_t seq, hipStream_t st) {
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(64), 0, st, ctrl, host_mapped, n, seq);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t knn_launch_fill_u32(uint32_t* p, int64_t n, uint32_t v, const int32_t* gate, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_fill_u32, dim3(grid), dim3(256), 0, st, p, n, v, gate);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t knn_launch_rerun_decide(int32_t* ctrl, int64_t limit, hipStream_t st) {
    hipLaunchKernelGGL(k_rerun_decide, dim3(1), dim3(64), 0, st, ctrl, limit);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

// ---------------------------------------------------------------------------------
// Launchers (host side)
// ---------------------------------------------------------------------------------
static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// k <= 64R selects the wave-list register count R
static int list_regs(int k) { return k <= 64 ? 1 : k <= 128 ? 2 : k <= 256 ? 4 : k <= 512 ? 8 : 16; }

template <int R, typename E>
static hipError_t launch_exact_r(const ExactScanArgs& a0, int grid, hipStream_t st) {
    ExactScanArgs a = a0;
    a.q_lds_bytes = (int)align16((size_t)a.d * sizeof(float));
    size_t lds = a.q_lds_bytes + 4 * 64 * R * sizeof(u64) +
                 (a.C <= KNN_VOTE_LDS_MAX_C ? align16((size_t)a.C * sizeof(int)) : 0);
    hipLaunchKernelGGL((k_exact_scan<R, E>), dim3(grid), dim3(256), lds, st, a);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

template <typename E>
static hipError_t launch_exact_e(const ExactScanArgs& a, int grid, hipStream_t st) {
    switch (list_regs(a.k)) {
        case 1: return launch_exact_r<1, E>(a, grid, st);
        case 2: return launch_exact_r<2, E>(a, grid, st);
        case 4: return launch_exact_r<4, E>(a, grid, st);
        case 8: return launch_exact_r<8, E>(a, grid, st);
        default: return launch_exact_r<16, E>(a, grid, st);
    }
}

hipError_t knn_launch_exact_scan(const ExactScanArgs& a, int grid, hipStream_t st) {
    return a.elem == ELEM_BF16 ? launch_exact_e<bf16_t>(a, grid, st) : launch_exact_e<float>(a, grid, st);
}

size_t knn_exact_scan_lds(int d, int k, int C) {
    return align16((size_t)d * 4) + 4 * 64 * (size_t)list_regs(k) * 8 +
           (C <= KNN_VOTE_LDS_MAX_C ? align16((size_t)C * 4) : 0);
}

// ---- k_direct_tile ----
// QW queries per wave: 8 / list registers (the wave lists T[QW][R] stay at 16 VGPRs)
static int direct_qw(int k) { return std::max(1, 8 / list_regs(k)); }
int knn_direct_tile_qb(int k) { return DT_NW * direct_qw(k); }

// dims per staged chunk and the padded LDS row stride (an odd number of 16-B slots)
static void direct_tile_geom(int d, int* dc, int* stride) {
    const int dpad = (d + 3) & ~3;
    *dc = std::min(dpad, DT_MAX_DC);
    int slots = *dc / 4;
    if ((slots & 1) == 0) slots++;
    *stride = 4 * slots;
}

size_t knn_direct_tile_lds(int d, int C) {
    int dc, stride;
    direct_tile_geom(d, &dc, &stride);
    return 2 * 64 * (size_t)stride * 4 + (C <= KNN_VOTE_LDS_MAX_C ? (size_t)DT_NW * ((C + 3) & ~3) * 4 : 0);
}

template <int QW, int R, typename E, bool SH = false>
static const void* direct_tile_fn() { return reinterpret_cast<const void*>(&k_direct_tile<QW, R, E, SH>); }

template <typename E>
static const void* direct_tile_fn_e(int k) {
    switch (list_regs(k)) {
        case 1: return k <= 16 ? direct_tile_fn<8, 1, E, true>() : direct_tile_fn<8, 1, E>();
        case 2: return direct_tile_fn<4, 2, E>();
        case 4: return direct_tile_fn<2, 4, E>();
        case 8: return direct_tile_fn<1, 8, E>();
        default: return direct_tile_fn<1, 16, E>();
    }
}
static const void* direct_tile_ptr(int k, int elem) {
    return elem == ELEM_BF16 ? direct_tile_fn_e<bf16_t>(k) : direct_tile_fn_e<float>(k);
}

// k_direct_rows (d <= 16, k <= 16): DR_QW queries per wave (their features stay in scalar
// registers), a wave per work unit
// (one query pair per wave: more waves, each with fewer inserts in flight; config L, same box,
// direct + merge stages: 4 queries per wave 0.097 ms at its best segment count, 2 queries 0.089,
// 8 queries 0.136 -- r05y)
#ifndef KNN_DR_QW
#define KNN_DR_QW 2  // (a study build may set 4 or 8)
#endif
static constexpr int DR_QW = KNN_DR_QW;
static bool direct_rows(int k, int d) { return d <= 16 && k <= 16; }
bool knn_direct_rows_shape(int k, int d) { return direct_rows(k, d); }
int64_t knn_direct_rows_groups(int64_t nq) { return (nq + DR_QW - 1) / DR_QW; }
template <typename E>
static const void* direct_rows_fn(int d) {
    switch ((d + 3) / 4) {
        case 1: return reinterpret_cast<const void*>(&k_direct_rows<1, DR_QW, E>);
        case 2: return reinterpret_cast<const void*>(&k_direct_rows<2, DR_QW, E>);
        case 3: return reinterpret_cast<const void*>(&k_direct_rows<3, DR_QW, E>);
        default: return reinterpret_cast<const void*>(&k_direct_rows<4, DR_QW, E>);
    }
}
static const void* direct_rows_ptr(int d, int elem) {
    return elem == ELEM_BF16 ? direct_rows_fn<bf16_t>(d) : direct_rows_fn<float>(d);
}

hipError_t knn_direct_tile_occupancy(int k, int elem, int d, int C, int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, direct_tile_ptr(k, elem), 64 * DT_NW,
                                                        knn_direct_tile_lds(d, C));
}

hipError_t knn_direct_units(int k, int elem, int d, int C, int* queries_per_unit, int* units_per_cu) {
    int occ = 1;
    hipError_t e;
    if (direct_rows(k, d)) {
        *queries_per_unit = DR_QW;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, direct_rows_ptr(d, elem), 256, 0);
        *units_per_cu = 4 * std::max(occ, 1);
    } else {
        *queries_per_unit = knn_direct_tile_qb(k);
        e = knn_direct_tile_occupancy(k, elem, d, C, &occ);
        *units_per_cu = std::max(occ, 1);
    }
    return e;
}

hipError_t knn_launch_direct_tile(DirectTileArgs a, hipStream_t st) {
    if (a.nq <= 0) return hipSuccess;
    if (a.nseg < 1 || (a.nseg > 1 && !a.rec) || a.d < 1 || a.k < 1 || a.k > 1024) return hipErrorInvalidValue;
    if (direct_rows(a.k, a.d)) {
        // the wave-per-unit shape: n_qblocks query groups of DR_QW, 4 units per block
        a.n_qblocks = (int)((a.nq + DR_QW - 1) / DR_QW);
        const int64_t units = (int64_t)a.n_qblocks * a.nseg;
        void* args[] = {&a};
        hipError_t e = hipLaunchKernel(direct_rows_ptr(a.d, a.elem), dim3((unsigned)((units + 3) / 4)), dim3(256), args,
                                       0, st);
        if (e != hipSuccess) return e;
        KNN_LAUNCH_CHECK();
        return hipSuccess;
    }
    direct_tile_geom(a.d, &a.dc, &a.stride);
    a.vote_lds = a.C <= KNN_VOTE_LDS_MAX_C;
    const int qb = knn_direct_tile_qb(a.k);
    a.n_qblocks = (int)((a.nq + qb - 1) / qb);
    const dim3 grid((unsigned)((int64_t)a.n_qblocks * a.nseg));
    void* args[] = {&a};
    hipError_t e = hipLaunchKernel(direct_tile_ptr(a.k, a.elem), grid, dim3(64 * DT_NW), args,
                                   knn_direct_tile_lds(a.d, a.C), st);
    if (e != hipSuccess) return e;
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t knn_launch_row_norms(const void* x, int elem, int64_t n, int ld, int d, float* out,
                                int32_t* status, uint32_t* maxo, float* outp, float c1, hipStream_t st,
                                float4* tstat, const int32_t* gate, float2* qstat, float oscale) {
    if (n <= 0) return hipSuccess;
    const int64_t rows = n + (outp ? 64 : 0);
    dim3 grid((unsigned)((rows + 255) / 256));
    if (elem == ELEM_BF16)
        hipLaunchKernelGGL(k_row_norms<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, n, ld, d, out,
                           status, maxo, outp, c1, tstat, gate, qstat, oscale);
    else
        hipLaunchKernelGGL(k_row_norms<float>, grid, dim3(256), 0, st, (const float*)x, n, ld, d, out,
                           status, maxo, outp, c1, tstat, gate, qstat, oscale);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

// LDS of one filter block (mirrors FilterTile + the kernel's carve-up)
static size_t gemm_filter_lds_of(int row_bytes, int k, int nw, int qg, int rg, int nbuf) {
    const int bn = 32 * rg, bm = 32 * qg * nw;
    const int ins = (bn * (row_bytes / 16 + 1) + 63) / 64;
    return (size_t)nbuf * ins * 1024 + ((size_t)(nbuf + 1) * 2 * bn + (size_t)bm * heap_stride(k)) * sizeof(float);
}

// Filter plan per (element type, row bytes, k).
//  fp32 (MFMA-bound, 16x the cycles per FLOP of bf16): 4 waves x 32 queries, 64-row tiles;
//    two blocks per CU with double-buffered tiles when the LDS allows (one block's barrier /
//    DMA phase hides under the other's MFMAs), else one block triple-buffered.
//  bf16 / split: 8 waves x 32 queries (two waves per SIMD hide each other's fast test, slow
//    path and waits): 256 queries share every staged train byte, so the L2 -> LDS bytes per
//    FLOP halve.  64-row tiles (two accumulators per wave, double-buffered) when the LDS
//    allows, else 32-row tiles, triple-buffered when the LDS allows (large k: big heaps).
//    Larger k that does not fit falls back to the fp32 shape.
//  bf16 rows of 128 bytes (64 features): 4 waves x 32 queries, 64-row tiles, two blocks per CU.
FilterPlan knn_gemm_filter_plan(int elem, int row_bytes, int k) {
    const size_t cap = 160 * 1024;
    auto fits = [&](int nw, int qg, int rg, int nbuf, size_t limit) {
        return gemm_filter_lds_of(row_bytes, k, nw, qg, rg, nbuf) <= limit;
    };
    auto make = [&](int nw, int qg, int rg, int minw, int nbuf) {
        FilterPlan f{nw, qg, rg, minw, nbuf, 32 * qg * nw, gemm_filter_lds_of(row_bytes, k, nw, qg, rg, nbuf)};
        return f;
    };
    if (elem != ELEM_F32) {
        // short rows (64 bf16 features: 4 MFMAs per 32x32 block and tile): the per-tile
        // barrier and fast test outweigh the MFMAs, so two 4-wave blocks per CU hide each
        // other's synchronisation (B, rounded bf16, k=32: 880 ms vs 1062 ms for 8 waves)
        if (row_bytes == 128 && fits(4, 1, 2, 2, cap / 2)) return make(4, 1, 2, 2, 2);
        // 8 waves x 32 queries over 64-row tiles (two accumulators per wave): half the
        // barriers, waits and DMA-issue rounds per MFMA of the 32-row shape; 32-row tiles
        // when the heaps of a large k leave no room
        if (fits(8, 1, 2, 2, cap)) return make(8, 1, 2, 2, 2);
        if (fits(8, 1, 1, 2, cap)) return make(8, 1, 1, 2, 2);
    }
    if (fits(4, 1, 2, 2, cap / 2)) return make(4, 1, 2, 2, 2);
    return make(4, 1, 2, 1, 2);
}

size_t knn_gemm_filter_lds(int elem, int row_bytes, int k) {
    return knn_gemm_filter_plan(elem, row_bytes, k).lds;
}

bool knn_gemm_filter_supported(int elem, int row_bytes) {
    (void)elem;
    return row_bytes == 128 || row_bytes == 256 || row_bytes == 512;
}

template <typename E, int RB>
static const void* gemm_filter_fn(const FilterPlan& f) {
#define KNN_FILTER_FN(MINW, NW, RG) reinterpret_cast<const void*>(&k_gemm_filter<E, RB, MINW, 2, NW, 1, RG>)
    if constexpr (sizeof(E) == 2) {
        if (f.nw == 8) return f.rg == 2 ? KNN_FILTER_FN(2, 8, 2) : KNN_FILTER_FN(2, 8, 1);
    }
    return f.minw == 2 ? KNN_FILTER_FN(2, 4, 2) : KNN_FILTER_FN(1, 4, 2);
#undef KNN_FILTER_FN
}

static const void* gemm_filter_ptr(int elem, int row_bytes, const FilterPlan& f) {
    if (elem == ELEM_SPLIT)
        return row_bytes == 128 ? gemm_filter_fn<split_t, 128>(f)
             : row_bytes == 256 ? gemm_filter_fn<split_t, 256>(f) : gemm_filter_fn<split_t, 512>(f);
    if (elem == ELEM_BF16 || elem == ELEM_ROUND)
        return row_bytes == 128 ? gemm_filter_fn<bf16_t, 128>(f)
             : row_bytes == 256 ? gemm_filter_fn<bf16_t, 256>(f) : gemm_filter_fn<bf16_t, 512>(f);
    return row_bytes == 128 ? gemm_filter_fn<float, 128>(f)
         : row_bytes == 256 ? gemm_filter_fn<float, 256>(f) : gemm_filter_fn<float, 512>(f);
}

hipError_t knn_gemm_filter_occupancy(int elem, int row_bytes, int k, int* blocks_per_cu) {
    if (!knn_gemm_filter_supported(elem, row_bytes)) return hipErrorInvalidValue;
    const FilterPlan f = knn_gemm_filter_plan(elem, row_bytes, k);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, gemm_filter_ptr(elem, row_bytes, f),
                                                        64 * f.nw, f.lds);
}

hipError_t knn_launch_gemm_filter(const GemmFilterArgs& a, int elem, int row_bytes, hipStream_t st) {
    if (!knn_gemm_filter_supported(elem, row_bytes)) return hipErrorInvalidValue;
    const FilterPlan f = knn_gemm_filter_plan(elem, row_bytes, a.k);
    const void* fn = gemm_filter_ptr(elem, row_bytes, f);
    void* args[] = {const_cast<GemmFilterArgs*>(&a)};
    const dim3 grid((unsigned)(a.n_qtiles * a.nseg));
    hipError_t e = hipLaunchKernel(fn, grid, dim3(64 * f.nw), args, f.lds, st);
    if (e != hipSuccess) return e;
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

template <int R, typename E>
static hipError_t launch_rescore_r(const RescoreArgs& a0, hipStream_t st) {
    RescoreArgs a = a0;
    a.q_lds_bytes = (int)align16((size_t)a.d * 4);
    a.c_lds_bytes = a.C <= KNN_VOTE_LDS_MAX_C ? (int)align16((size_t)a.C * 4) : 0;
    a.su_cap = std::max(64, std::min(64 * KNN_RESCORE_CAPW, (a.su_cap + 63) / 64 * 64));
    a.wave_lds_bytes = a.q_lds_bytes + a.c_lds_bytes + a.su_cap * 4;
    size_t lds = 4 * (size_t)a.wave_lds_bytes;
    unsigned grid = (unsigned)((a.nq + 3) / 4);
    if (grid == 0) return hipSuccess;
    if (a.gate)
        hipLaunchKernelGGL((k_rescore<R, KNN_RESCORE_CAPW, E, true>), dim3(gated_grid(grid, a.gate)), dim3(256), lds, st, a);
    else
        hipLaunchKernelGGL((k_rescore<R, KNN_RESCORE_CAPW, E, false>), dim3(grid), dim3(256), lds, st, a);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

template <typename E>
static hipError_t launch_rescore_e(const RescoreArgs& a, hipStream_t st) {
    switch (list_regs(a.k)) {
        case 1: return launch_rescore_r<1, E>(a, st);
        case 2: return launch_rescore_r<2, E>(a, st);
        case 4: return launch_rescore_r<4, E>(a, st);
        case 8: return launch_rescore_r<8, E>(a, st);
        default: return launch_rescore_r<16, E>(a, st);
    }
}

hipError_t knn_launch_rescore(const RescoreArgs& a, hipStream_t st) {
    return a.elem == ELEM_BF16 ? launch_rescore_e<bf16_t>(a, st) : launch_rescore_e<float>(a, st);
}


template <int R>
static hipError_t launch_merge_r(const MergeArgs& a, hipStream_t st) {
    const unsigned grid = (unsigned)((a.nq + 3) / 4);
    if (grid == 0) return hipSuccess;
    const size_t lds = 4 * (size_t)merge_wave_words(a.C, a.k) * sizeof(int);
    hipLaunchKernelGGL(k_merge_vote<R>, dim3(grid), dim3(256), lds, st, a);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t knn_launch_merge(const MergeArgs& a, hipStream_t st) {
    switch (list_regs(a.k)) {
        case 1: return launch_merge_r<1>(a, st);
        case 2: return launch_merge_r<2>(a, st);
        case 4: return launch_merge_r<4>(a, st);
        case 8: return launch_merge_r<8>(a, st);
        default: return launch_merge_r<16>(a, st);
    }
}

hipError_t knn_launch_confusion(const int32_t* pred, const int32_t* labels, int64_t n, int C, int32_t* cm,
                                unsigned long long* correct, int32_t* status, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_confusion, dim3(grid), dim3(256), 0, st, pred, labels, n, C, cm, correct, status);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t knn_launch_split_rows(const float* x, int64_t n, int ld, int d, uint16_t* out, hipStream_t st,
                                 const int32_t* gate) {
    const int64_t total = n * (d / 4);
    if (total <= 0) return hipSuccess;
    if (d % 4 || ld % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_split_rows, dim3(gated_grid(elementwise_grid(total), gate)), dim3(256), 0, st, x, n, ld, d, out, gate);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t knn_launch_round_rows(const float* x, int64_t n, int ld, int d, uint16_t* out, hipStream_t st,
                                 const int32_t* gate) {
    const int64_t total = n * (d / 4);
    if (total <= 0) return hipSuccess;
    if (d % 4 || ld % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_round_rows, dim3(gated_grid(elementwise_grid(total), gate)), dim3(256), 0, st, x, n, ld, d, out, gate);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t knn_launch_generate(const GenerateArgs& a, hipStream_t st) {
    int64_t total = a.n * a.ld;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_generate, dim3(elementwise_grid(std::max(total, a.n))), dim3(256), 0, st, a);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}
