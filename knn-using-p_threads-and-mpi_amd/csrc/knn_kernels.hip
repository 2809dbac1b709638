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
// Kernels
//   k_exact_scan   fused direct-form distance + wave-resident top-k + vote (low d,
//                  ARFF inputs, and the per-query fallback of the GEMM path)
//   k_row_norms    ||x||^2 per row (for the GEMM form)
//   k_gemm_filter  q.t on FP32 MFMA (v_mfma_f32_32x32x2_f32), certified candidate
//                  filter with a running per-query threshold
//   k_rescore      exact direct-form rescore of the surviving candidates + top-k + vote
//   k_generate     counter-based synthetic rows (same formula as oracle/knn_oracle.c)
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "knn_kernels.h"

typedef unsigned long long u64;
static constexpr u64 KEY_NONE = ~0ull;
typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------------
// Keys and wave-level bitonic networks (64 lanes, one element per lane per register)
// ---------------------------------------------------------------------------------
__device__ __forceinline__ u64 make_key(float dist, uint32_t idx) {
    if (!(dist < FLT_MAX)) return KEY_NONE;  // main.cpp:47 against the FLT_MAX sentinel
    return ((u64)__float_as_uint(dist) << 32) | (u64)idx;
}

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ u64 umin64(u64 a, u64 b) { return a < b ? a : b; }
__device__ __forceinline__ u64 umax64(u64 a, u64 b) { return a < b ? b : a; }

// compare-exchange with lane ^ j; keep the smaller key if keep_min
__device__ __forceinline__ u64 cx(u64 v, int j, bool keep_min) {
    u64 o = __shfl_xor(v, j);
    return keep_min ? umin64(v, o) : umax64(v, o);
}

// full bitonic sort of 64 keys across the wave
__device__ __forceinline__ u64 sort64(u64 v, bool descending) {
    const int lane = lane_id();
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int j = size >> 1; j > 0; j >>= 1) {
            bool up = ((lane & size) == 0) != descending;
            bool lower = (lane & j) == 0;
            v = cx(v, j, lower == up);
        }
    }
    return v;
}

// bitonic merge of a bitonic 64-sequence
__device__ __forceinline__ u64 merge64(u64 v, bool ascending) {
    const int lane = lane_id();
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) v = cx(v, j, ((lane & j) == 0) == ascending);
    return v;
}

// Wave-resident sorted list of the 64*R smallest keys: element e = 64*r + lane lives in
// T[r] of lane (e & 63).  Merge one batch of 64 new keys (one per lane).
template <int R>
__device__ __forceinline__ void topk_merge(u64 (&T)[R], u64 x) {
    x = sort64(x, /*descending=*/true);
    u64 y = umin64(T[R - 1], x);  // half-cleaner: the 64 smallest of T[R-1] u x, bitonic
    if constexpr (R == 1) {
        T[0] = merge64(y, true);
    } else {
        // [T0..T(R-2) ascending, T(R-1) descending] is bitonic over 64R elements
        T[R - 1] = merge64(y, false);
#pragma unroll
        for (int s = R / 2; s >= 1; s >>= 1) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                if ((r & s) == 0) {
                    u64 a = T[r], b = T[r + s];
                    T[r] = umin64(a, b);
                    T[r + s] = umax64(a, b);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) T[r] = merge64(T[r], true);
    }
}

// element e of the wave list, broadcast to every lane
template <int R>
__device__ __forceinline__ u64 list_at(const u64 (&T)[R], int e) {
    u64 v = T[0];
#pragma unroll
    for (int r = 1; r < R; r++)
        if (r == (e >> 6)) v = T[r];
    return __shfl(v, e & 63);
}

// ---------------------------------------------------------------------------------
// Direct-form distance, restated from main.cpp:14-23 with contraction disabled so
// every diff*diff and += rounds to fp32 exactly like the reference.
// ---------------------------------------------------------------------------------
#pragma clang fp contract(off)
template <typename QP>
__device__ __forceinline__ float direct_dist(QP q, const float* __restrict__ t, int d) {
    float sum = 0.0f;
    int i = 0;
    if ((((uintptr_t)t) & 15) == 0) {
        for (; i + 4 <= d; i += 4) {
            float4 v = *reinterpret_cast<const float4*>(t + i);
            float d0 = q[i + 0] - v.x; sum = sum + d0 * d0;
            float d1 = q[i + 1] - v.y; sum = sum + d1 * d1;
            float d2 = q[i + 2] - v.z; sum = sum + d2 * d2;
            float d3 = q[i + 3] - v.w; sum = sum + d3 * d3;
        }
    }
    for (; i < d; i++) {
        float df = q[i] - t[i];
        sum = sum + df * df;
    }
    return sum;
}
#pragma clang fp contract(on)

// ---------------------------------------------------------------------------------
// Vote + outputs for one query from a finished wave list (main.cpp:64-78).
// counts: wave-private LDS array of C ints.  Runs on one wave.
// ---------------------------------------------------------------------------------
template <int R>
__device__ void finish_query(const u64 (&T)[R], int k, int C, const int32_t* __restrict__ labels,
                             int* counts, int64_t q, int32_t* __restrict__ pred,
                             float* __restrict__ topk_dist, int32_t* __restrict__ topk_idx,
                             int32_t* __restrict__ status) {
    const int lane = lane_id();
    for (int c = lane; c < C; c += 64) counts[c] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    u64 kth = list_at(T, k - 1);
    bool bad = (kth == KEY_NONE);
#pragma unroll
    for (int r = 0; r < R; r++) {
        int e = 64 * r + lane;
        if (e < k) {
            u64 key = T[r];
            if (key != KEY_NONE) {
                int32_t idx = (int32_t)(uint32_t)(key & 0xffffffffull);
                if (topk_dist) topk_dist[q * k + e] = __uint_as_float((uint32_t)(key >> 32));
                if (topk_idx) topk_idx[q * k + e] = idx;
                int lab = labels[idx];
                if (lab >= 0 && lab < C) atomicAdd(&counts[lab], 1);
                else atomicOr(status, KNN_STATUS_BAD_LABEL);
            } else {
                if (topk_dist) topk_dist[q * k + e] = FLT_MAX;
                if (topk_idx) topk_idx[q * k + e] = -1;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // argmax, strict '>' scanning 0..C-1 == max count, smallest label on ties
    u64 best = 0;
    for (int c = lane; c < C; c += 64) {
        u64 v = ((u64)(uint32_t)counts[c] << 32) | (u64)(0xffffffffu - (uint32_t)c);
        best = umax64(best, v);
    }
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) best = umax64(best, __shfl_xor(best, j));
    if (lane == 0) {
        pred[q] = bad ? 0 : (int32_t)(0xffffffffu - (uint32_t)(best & 0xffffffffull));
        if (bad) atomicOr(status, KNN_STATUS_TOO_FEW);
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
template <int R>
__global__ __launch_bounds__(256) void k_exact_scan(ExactScanArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* qs = reinterpret_cast<float*>(smem);
    u64* lists = reinterpret_cast<u64*>(smem + a.q_lds_bytes);
    int* counts = reinterpret_cast<int*>(smem + a.q_lds_bytes + 4 * 64 * R * sizeof(u64));
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const int64_t n_work = a.qlist ? (int64_t)(*a.qcount) : a.nq;

    for (int64_t w = blockIdx.x; w < n_work; w += gridDim.x) {
        const int64_t q = a.qlist ? (int64_t)a.qlist[w] : w;
        __syncthreads();
        for (int i = threadIdx.x; i < a.d; i += 256) qs[i] = a.test[q * a.ld_q + i];
        __syncthreads();

        u64 T[R];
#pragma unroll
        for (int r = 0; r < R; r++) T[r] = KEY_NONE;
        u64 thr = KEY_NONE;
        for (int64_t base = (int64_t)wave * 64; base < a.nt; base += 256) {
            const int64_t t = base + lane;
            u64 key = KEY_NONE;
            if (t < a.nt) key = make_key(direct_dist(qs, a.train + t * a.ld_t, a.d), (uint32_t)t);
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
            finish_query<R>(T, a.k, a.C, a.labels, counts, q, a.pred, a.topk_dist, a.topk_idx,
                            a.status);
        }
    }
}

// ---------------------------------------------------------------------------------
// k_row_norms: out[r] = sum_i x[r][i]^2 (fp32).  Flags rows whose norm is too large
// for the GEMM form's error certificate (>= 2^125) so the host falls back.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_row_norms(const float* __restrict__ x, int64_t n, int ld,
                                                   int d, float* __restrict__ out,
                                                   int32_t* __restrict__ status) {
    int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const float* row = x + r * ld;
    float s = 0.0f;
    int i = 0;
    for (; i + 4 <= d; i += 4) {
        float4 v = *reinterpret_cast<const float4*>(row + i);
        s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
    }
    for (; i < d; i++) s = fmaf(row[i], row[i], s);
    out[r] = s;
    if (!(s < 0x1p125f)) atomicOr(status, KNN_STATUS_GEMM_UNSAFE);
}

// ordered uint <-> float (monotone for all non-NaN floats)
__device__ __forceinline__ uint32_t f2o(float f) {
    uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// ---------------------------------------------------------------------------------
// k_gemm_filter<DK>: GEMM-form candidate filter on FP32 MFMA.
//
// Block = 256 threads = 4 waves; query tile BM = 128 (32 per wave) whose B-operand
// fragments stay in VGPRs for the whole scan; train tile BN = 64 rows staged in LDS
// (register prefetch of tile t+1 while tile t is multiplied).  Per wave and tile:
// 2 x (DK/2) v_mfma_f32_32x32x2_f32 give a 64(train) x 32(query) block; lane l holds
// query j = l&31 and train rows (reg&3) + 8(reg>>2) + 4(l>>5) (+32 for the 2nd block).
//
// Certificate (DESIGN.md "GEMM-form certificate"): with s = qn+tn,
// G = s - 2 q.t, Delta = coef*s + eta, L = G - Delta <= D <= U = G + Delta for the
// reference's direct-form D.  A train row is kept for query q iff L <= thr_q, where
// thr_q is the k-th smallest U among kept rows (kept in LDS, sorted) or a smaller
// threshold published by another segment of the same query (gthr, atomicMin).
// Every row of the exact top-k satisfies L <= D <= D_(k) <= thr_q, so is kept.
// ---------------------------------------------------------------------------------
static constexpr int GF_BM = 128;
static constexpr int GF_BN = 64;

template <int DK>
__global__ __launch_bounds__(256, 2) void k_gemm_filter(GemmFilterArgs a) {
    constexpr int STRIDE = DK + 4;          // floats per LDS tile row (pad: conflict-free b128)
    constexpr int GROUPS = GF_BN * DK / 8;  // 8-float groups per tile
    constexpr int GPT = GROUPS / 256;       // groups per thread
    static_assert(GROUPS % 256 == 0, "tile groups must divide the block");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* tile = reinterpret_cast<float*>(smem);                 // [BN][STRIDE]
    float* tn_s = tile + GF_BN * STRIDE;                          // [BN]
    float* spill = tn_s + GF_BN;                                  // [4 waves][32][64]
    float* topU = spill + 4 * 32 * 64;                            // [BM][k]

    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const int j = lane & 31;
    const int h = lane >> 5;
    const int qt = blockIdx.x % a.n_qtiles;
    const int seg = blockIdx.x / a.n_qtiles;
    const int jl = wave * 32 + j;                     // query within the tile
    const int64_t q = (int64_t)qt * GF_BM + jl;
    const bool qvalid = q < a.nq;
    const int64_t row_begin = (int64_t)seg * a.seg_len;
    const int64_t row_end = min(a.nt, row_begin + a.seg_len);
    const int k = a.k;

    // topU lists start at +inf
    for (int i = threadIdx.x; i < GF_BM * k; i += 256) topU[i] = __uint_as_float(0x7f800000u);

    // query fragments: qf[s] = Q[q][2s + h]
    float qf[DK / 2];
    {
        const float* qrow = a.test + (qvalid ? q : 0) * a.ld_q;
#pragma unroll
        for (int s = 0; s < DK / 2; s++) {
            int c = 2 * s + h;
            qf[s] = (qvalid && c < a.d) ? qrow[c] : 0.0f;
        }
    }
    const float qn = qvalid ? a.qnorm[q] : __uint_as_float(0x7f800000u);
    float thr = qvalid ? o2f(a.gthr[q]) : -__uint_as_float(0x7f800000u);
    float published = thr;
    const float coef = a.coef, eta = a.eta;

    // register prefetch of one tile: GPT groups of 8 floats per thread
    float4 pre[GPT][2];
    auto load_tile = [&](int64_t r0) {
#pragma unroll
        for (int i = 0; i < GPT; i++) {
            int gi = threadIdx.x + 256 * i;
            int row = gi / (DK / 8);
            int g = gi % (DK / 8);
            int64_t t = r0 + row;
            float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
            if (t < row_end) {
                const float* src = a.train + t * a.ld_t + 8 * g;
                if (8 * g + 8 <= a.d) {
                    v0 = *reinterpret_cast<const float4*>(src);
                    v1 = *reinterpret_cast<const float4*>(src + 4);
                } else {
                    float tmp[8];
#pragma unroll
                    for (int e = 0; e < 8; e++) tmp[e] = (8 * g + e < a.d) ? src[e] : 0.0f;
                    v0 = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
                    v1 = make_float4(tmp[4], tmp[5], tmp[6], tmp[7]);
                }
            }
            pre[i][0] = v0;
            pre[i][1] = v1;
        }
    };
    // permuted store: within each 8-group, position 4h + jj holds k = 2jj + h
    auto store_tile = [&](int64_t r0) {
#pragma unroll
        for (int i = 0; i < GPT; i++) {
            int gi = threadIdx.x + 256 * i;
            int row = gi / (DK / 8);
            int g = gi % (DK / 8);
            float4 v0 = pre[i][0], v1 = pre[i][1];
            float* dst = tile + row * STRIDE + 8 * g;
            *reinterpret_cast<float4*>(dst) = make_float4(v0.x, v0.z, v1.x, v1.z);
            *reinterpret_cast<float4*>(dst + 4) = make_float4(v0.y, v0.w, v1.y, v1.w);
        }
        if (threadIdx.x < GF_BN) {
            int64_t t = r0 + threadIdx.x;
            tn_s[threadIdx.x] = (t < row_end) ? a.tnorm[t] : __uint_as_float(0x7f800000u);
        }
    };

    const int64_t ntiles = (row_end > row_begin) ? (row_end - row_begin + GF_BN - 1) / GF_BN : 0;
    if (ntiles > 0) load_tile(row_begin);
    for (int64_t it = 0; it < ntiles; it++) {
        const int64_t r0 = row_begin + it * GF_BN;
        __syncthreads();  // every wave has finished reading the previous tile
        store_tile(r0);
        __syncthreads();
        if (it + 1 < ntiles) load_tile(r0 + GF_BN);

        floatx16 acc0 = {}, acc1 = {};
        const float* a0p = tile + j * STRIDE + 4 * h;
        const float* a1p = tile + (32 + j) * STRIDE + 4 * h;
#pragma unroll
        for (int g = 0; g < DK / 8; g++) {
            float4 x0 = *reinterpret_cast<const float4*>(a0p + 8 * g);
            float4 x1 = *reinterpret_cast<const float4*>(a1p + 8 * g);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0.x, qf[4 * g + 0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1.x, qf[4 * g + 0], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0.y, qf[4 * g + 1], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1.y, qf[4 * g + 1], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0.z, qf[4 * g + 2], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1.z, qf[4 * g + 2], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0.w, qf[4 * g + 3], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1.w, qf[4 * g + 3], acc1, 0, 0, 0);
        }

        // epilogue: certified filter, one bit per (block, reg)
        uint32_t mask = 0;
#pragma unroll
        for (int rb = 0; rb < 4; rb++) {
            float4 tA = *reinterpret_cast<const float4*>(tn_s + 8 * rb + 4 * h);
            float4 tB = *reinterpret_cast<const float4*>(tn_s + 32 + 8 * rb + 4 * h);
            float tnA[4] = {tA.x, tA.y, tA.z, tA.w};
            float tnB[4] = {tB.x, tB.y, tB.z, tB.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int reg = 4 * rb + e;
                float sA = qn + tnA[e];
                float GA = fmaf(-2.0f, acc0[reg], sA);
                float LA = GA - fmaf(coef, sA, eta);
                float sB = qn + tnB[e];
                float GB = fmaf(-2.0f, acc1[reg], sB);
                float LB = GB - fmaf(coef, sB, eta);
                mask |= (uint32_t)(LA <= thr) << reg;
                mask |= (uint32_t)(LB <= thr) << (16 + reg);
            }
        }

        if (__ballot(mask != 0)) {
            // slow path (rare after warm-up): spill the raw dot products, then the two
            // lanes of each query take turns appending candidates and inserting U
            float* sp = spill + wave * 32 * 64;
#pragma unroll
            for (int reg = 0; reg < 16; reg++) {
                sp[reg * 64 + lane] = acc0[reg];
                sp[(16 + reg) * 64 + lane] = acc1[reg];
            }
            float* myU = topU + jl * k;
            for (int hh = 0; hh < 2; hh++) {
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (h == hh) {
                    uint32_t mm = mask;
                    while (mm) {
                        const int b = __builtin_ctz(mm);
                        mm &= mm - 1;
                        const int reg = b & 15;
                        const int row = 32 * (b >> 4) + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                        const float s = qn + tn_s[row];
                        const float G = fmaf(-2.0f, sp[b * 64 + lane], s);
                        const float dl = fmaf(coef, s, eta);
                        const float L = G - dl;
                        if (!(L <= thr)) continue;  // threshold moved since the mask was taken
                        const float U = G + dl;
                        const int32_t t = (int32_t)(r0 + row);
                        const int slot = atomicAdd(&a.cnt[q], 1);
                        if (slot < a.cap) {
                            const int64_t o = q * (int64_t)a.cap + slot;
                            a.cand_idx[o] = t;
                            a.cand_L[o] = L;
                            a.cand_U[o] = U;
                        }
                        if (U < myU[k - 1]) {
                            int p = k - 1;
                            while (p > 0 && myU[p - 1] > U) {
                                myU[p] = myU[p - 1];
                                p--;
                            }
                            myU[p] = U;
                            thr = fminf(thr, myU[k - 1]);
                        }
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (qvalid) thr = fminf(thr, myU[k - 1]);
            thr = fminf(thr, __shfl_xor(thr, 32));
            if (qvalid && h == 0 && thr < published) {
                atomicMin(&a.gthr[q], f2o(thr));
                published = thr;
            }
        }
        // pick up thresholds published by other segments of the same queries
        if ((it & 15) == 15 && qvalid) thr = fminf(thr, o2f(__hip_atomic_load(&a.gthr[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
    }
}

// ---------------------------------------------------------------------------------
// k_rescore<R, CAPW>: one wave per query.  Final threshold = k-th smallest U among the
// query's candidates (found by bisection over ordered float bits); candidates with
// L <= threshold are rescored with the exact direct form and selected by key.
// Queries whose list overflowed (or holds < k entries) go to the exact fallback list.
// LDS per wave: q row [ld_pad] f32 | counts [C] i32 | survivors [64*CAPW] i32
// ---------------------------------------------------------------------------------
template <int R, int CAPW>
__global__ __launch_bounds__(256) void k_rescore(RescoreArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    unsigned char* my = smem + (size_t)wave * a.wave_lds_bytes;
    float* qs = reinterpret_cast<float*>(my);
    int* counts = reinterpret_cast<int*>(my + a.q_lds_bytes);
    int32_t* surv = reinterpret_cast<int32_t*>(my + a.q_lds_bytes + a.c_lds_bytes);
    const int64_t q = (int64_t)blockIdx.x * 4 + wave;
    if (q >= a.nq) return;
    const int n = a.cnt[q];
    const int k = a.k;
    if (n > a.cap || n < k) {
        if (lane == 0) a.fb_list[atomicAdd(a.fb_count, 1)] = (int32_t)q;
        return;
    }
    // load candidates (ordered-uint U, float L)
    uint32_t uo[CAPW];
    float lv[CAPW];
#pragma unroll
    for (int i = 0; i < CAPW; i++) {
        int e = lane + 64 * i;
        bool v = e < n;
        int64_t o = q * (int64_t)a.cap + e;
        uo[i] = v ? f2o(a.cand_U[o]) : 0xffffffffu;
        lv[i] = v ? a.cand_L[o] : __uint_as_float(0x7f800000u);
    }
    // smallest x with #{U <= x} >= k
    uint32_t lo = 0u, hi = 0xfffffffeu;
    while (lo < hi) {
        uint32_t mid = lo + ((hi - lo) >> 1);
        int c = 0;
#pragma unroll
        for (int i = 0; i < CAPW; i++) c += __popcll(__ballot(uo[i] <= mid));
        if (c >= k) hi = mid; else lo = mid + 1;
    }
    const float thr = o2f(lo);
    // compact survivors L <= thr
    int m = 0;
#pragma unroll
    for (int i = 0; i < CAPW; i++) {
        bool s = lv[i] <= thr;
        u64 bal = __ballot(s);
        if (s) {
            int pos = m + __popcll(bal & ((1ull << lane) - 1ull));
            surv[pos] = a.cand_idx[q * (int64_t)a.cap + lane + 64 * i];
        }
        m += __popcll(bal);
    }
    for (int i = lane; i < a.d; i += 64) qs[i] = a.test[q * a.ld_q + i];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();

    u64 T[R];
#pragma unroll
    for (int r = 0; r < R; r++) T[r] = KEY_NONE;
    u64 kth = KEY_NONE;
    for (int b = 0; b < m; b += 64) {
        u64 key = KEY_NONE;
        if (b + lane < m) {
            int32_t t = surv[b + lane];
            key = make_key(direct_dist(qs, a.train + (int64_t)t * a.ld_t, a.d), (uint32_t)t);
        }
        bool pass = key < kth;
        if (__ballot(pass)) {
            topk_merge<R>(T, pass ? key : KEY_NONE);
            kth = list_at(T, k - 1);
        }
    }
    finish_query<R>(T, k, a.C, a.labels, counts, q, a.pred, a.topk_dist, a.topk_idx, a.status);
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

__global__ __launch_bounds__(256) void k_generate(GenerateArgs a) {
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    int64_t total = a.n * a.ld;
    if (i < total) {
        int64_t r = i / a.ld;
        int c = (int)(i % a.ld);
        float v = 0.0f;
        if (c < a.d) {
            uint32_t u = (uint32_t)(gen_hash(a.seed, a.stream, (uint64_t)(a.row0 + r), (uint32_t)c) >> 32);
            v = (a.kind == 1) ? (float)((int32_t)(u >> 24) - 128) * (1.0f / 128.0f)
                              : (float)(int32_t)(u >> 8) * (1.0f / 8388608.0f) - 1.0f;
        }
        if (a.bf16_out)
            reinterpret_cast<uint16_t*>(a.out)[i] = (uint16_t)(__float_as_uint(v) >> 16);  // exact for kind 1
        else
            reinterpret_cast<float*>(a.out)[i] = v;
    }
    if (a.labels && i < a.n) {
        uint32_t u = (uint32_t)(gen_hash(a.seed, a.stream, (uint64_t)(a.row0 + i), 0xFFFFu) >> 32);
        a.labels[i] = (int32_t)(u % (uint32_t)a.C);
    }
}

// ---------------------------------------------------------------------------------
// Launchers (host side)
// ---------------------------------------------------------------------------------
#define KNN_LAUNCH_CHECK() do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return e_; } while (0)

static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

template <int R>
static hipError_t launch_exact_r(const ExactScanArgs& a0, int grid, hipStream_t st) {
    ExactScanArgs a = a0;
    a.q_lds_bytes = (int)align16((size_t)a.d * sizeof(float));
    size_t lds = a.q_lds_bytes + 4 * 64 * R * sizeof(u64) + align16((size_t)a.C * sizeof(int));
    hipLaunchKernelGGL(k_exact_scan<R>, dim3(grid), dim3(256), lds, st, a);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t knn_launch_exact_scan(const ExactScanArgs& a, int grid, hipStream_t st) {
    if (a.k <= 64) return launch_exact_r<1>(a, grid, st);
    if (a.k <= 128) return launch_exact_r<2>(a, grid, st);
    if (a.k <= 256) return launch_exact_r<4>(a, grid, st);
    if (a.k <= 512) return launch_exact_r<8>(a, grid, st);
    return launch_exact_r<16>(a, grid, st);
}

size_t knn_exact_scan_lds(int d, int k, int C) {
    int R = k <= 64 ? 1 : k <= 128 ? 2 : k <= 256 ? 4 : k <= 512 ? 8 : 16;
    return align16((size_t)d * 4) + 4 * 64 * (size_t)R * 8 + align16((size_t)C * 4);
}

hipError_t knn_launch_row_norms(const float* x, int64_t n, int ld, int d, float* out,
                                int32_t* status, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_row_norms, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n, ld, d,
                       out, status);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

size_t knn_gemm_filter_lds(int dk, int k) {
    return ((size_t)GF_BN * (dk + 4) + GF_BN + 4 * 32 * 64 + (size_t)GF_BM * k) * sizeof(float);
}

template <int DK>
static const void* gemm_filter_fn() { return reinterpret_cast<const void*>(&k_gemm_filter<DK>); }

hipError_t knn_gemm_filter_occupancy(int dk, int k, int* blocks_per_cu) {
    size_t lds = knn_gemm_filter_lds(dk, k);
    const void* fn = dk == 32 ? gemm_filter_fn<32>()
                   : dk == 64 ? gemm_filter_fn<64>() : gemm_filter_fn<128>();
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, 256, lds);
}

hipError_t knn_launch_gemm_filter(const GemmFilterArgs& a, int dk, hipStream_t st) {
    size_t lds = knn_gemm_filter_lds(dk, a.k);
    dim3 grid((unsigned)(a.n_qtiles * a.nseg));
    switch (dk) {
        case 32: hipLaunchKernelGGL(k_gemm_filter<32>, grid, dim3(256), lds, st, a); break;
        case 64: hipLaunchKernelGGL(k_gemm_filter<64>, grid, dim3(256), lds, st, a); break;
        case 128: hipLaunchKernelGGL(k_gemm_filter<128>, grid, dim3(256), lds, st, a); break;
        default: return hipErrorInvalidValue;
    }
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

template <int R>
static hipError_t launch_rescore_r(const RescoreArgs& a0, hipStream_t st) {
    RescoreArgs a = a0;
    a.q_lds_bytes = (int)align16((size_t)a.d * 4);
    a.c_lds_bytes = (int)align16((size_t)a.C * 4);
    a.wave_lds_bytes = a.q_lds_bytes + a.c_lds_bytes + 64 * KNN_RESCORE_CAPW * 4;
    size_t lds = 4 * (size_t)a.wave_lds_bytes;
    unsigned grid = (unsigned)((a.nq + 3) / 4);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((k_rescore<R, KNN_RESCORE_CAPW>), dim3(grid), dim3(256), lds, st, a);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t knn_launch_rescore(const RescoreArgs& a, hipStream_t st) {
    if (a.k <= 64) return launch_rescore_r<1>(a, st);
    if (a.k <= 128) return launch_rescore_r<2>(a, st);
    if (a.k <= 256) return launch_rescore_r<4>(a, st);
    if (a.k <= 512) return launch_rescore_r<8>(a, st);
    return launch_rescore_r<16>(a, st);
}

hipError_t knn_launch_generate(const GenerateArgs& a, hipStream_t st) {
    int64_t total = a.n * a.ld;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_generate, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
    KNN_LAUNCH_CHECK();
    return hipSuccess;
}
