// knn_device.h -- device helpers shared by the kernel translation units of libknn_amd
// (knn_kernels.hip, knn_fused.hip): keys and wave bitonic networks, bf16 helpers,
// ordered-float bits, LDS-DMA issue and the GEMM filter tile geometry.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <float.h>
#include <stdint.h>

#include "knn_kernels.h"

typedef unsigned long long u64;

// Grid of a grid-stride elementwise kernel over `total` items (256 threads per block): at most
// 2^20 blocks.  A dispatch's size is a 32-bit count of work-items, so one thread per item
// would wrap for more than 2^32 items (a 32M x 256 generator fill has 8.2e9) and leave the
// tail untouched.
static inline unsigned elementwise_grid(int64_t total) {
    return (unsigned)std::min<int64_t>((total + 255) / 256, (int64_t)1 << 20);
}
// a gated stage (AUTO's re-run, rarely taken) launches at most 2048 blocks of a grid-stride
// kernel: a re-run not taken then costs a few thousand empty waves, not one per 256 elements
static inline unsigned gated_grid(unsigned grid, const void* gate) {
    return gate ? std::min(grid, 2048u) : grid;
}
#define KNN_LAUNCH_CHECK() do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return e_; } while (0)
static constexpr u64 KEY_NONE = ~0ull;
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
#ifndef KNN_FILTER_PK
#define KNN_FILTER_PK 0
#endif

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

// The word of lane ^ j (j a power of two <= 32, a constant once the networks below are
// unrolled), without ds_bpermute: j = 1, 2 by a DPP quad permutation, j = 4, 8 by two DPP
// row shifts (row_shl / row_shr: the partner sits j lanes up or down inside its row of 16)
// and a select, j = 16 by ds_swizzle's xor mode (no address operand), j = 32 by
// v_permlane32_swap (one of its two results is the other half's word).  All but j = 16 are
// VALU instructions, so a compare-exchange stage waits on no LDS round trip.
__device__ __forceinline__ uint32_t lane_xor(uint32_t v, int j) {
    const int lane = lane_id();
    switch (j) {
        case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
        case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
        case 4: {
            const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xF, 0xF, false);  // row_shl:4
            const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
            return (lane & 4) ? dn : up;
        }
        case 8: {
            const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x108, 0xF, 0xF, false);  // row_shl:8
            const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
            return (lane & 8) ? dn : up;
        }
        case 16: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (16 << 10) | 0x1F);  // xor_mask 16, and_mask 31
        default: {
            const auto sw = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            return (lane & 32) ? sw[0] : sw[1];
        }
    }
}
__device__ __forceinline__ u64 lane_xor64(u64 v, int j) {
    return ((u64)lane_xor((uint32_t)(v >> 32), j) << 32) | (u64)lane_xor((uint32_t)v, j);
}

// compare-exchange with lane ^ j; keep the smaller key if keep_min
__device__ __forceinline__ u64 cx(u64 v, int j, bool keep_min) {
    const u64 o = lane_xor64(v, j);
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

// topk_merge for a batch that is already ascending across the lanes (a prefix of a sorted
// list, KEY_NONE padding at the end): reversed by one lane permutation instead of sorted
template <int R>
__device__ __forceinline__ void topk_merge_sorted(u64 (&T)[R], u64 x) {
    const int src = 4 * (63 - lane_id());
    const u64 rev = ((u64)(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(x >> 32)) << 32) |
                    (u64)(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)x);
    u64 y = umin64(T[R - 1], rev);  // half-cleaner: the 64 smallest of T[R-1] u x, bitonic
    if constexpr (R == 1) {
        T[0] = merge64(y, true);
    } else {
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
// Feature elements: fp32, or bf16 bits widened exactly (bf16 -> fp32 is a 16-bit shift)
// ---------------------------------------------------------------------------------
typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
// filter operand tag for ELEM_SPLIT rows (bf16 bits [hi(d) | lo(d)] of fp32 data)
struct split_t { uint16_t v; };

// fp32 -> bf16 bits, round to nearest even (finite inputs)
__device__ __forceinline__ uint32_t bf16_rne(float x) {
    const uint32_t b = __float_as_uint(x);
    return (b + 0x7fffu + ((b >> 16) & 1u)) >> 16;
}

__device__ __forceinline__ float widen(float v) { return v; }
__device__ __forceinline__ float widen(bf16_t v) { return __uint_as_float((uint32_t)v << 16); }

// four consecutive elements as fp32 (p aligned to 4 elements)
__device__ __forceinline__ float4 load4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 load4(const bf16_t* p) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                       __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u));
}

// ordered uint <-> float (monotone for all non-NaN floats)
__device__ __forceinline__ uint32_t f2o(float f) {
    uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// min / max of two non-NaN floats as one v_med3 (fminf/fmaxf add two canonicalising v_max in
// IEEE mode): the middle of {a, b, -inf} is min(a, b), of {a, b, +inf} max(a, b)
__device__ __forceinline__ float fmin_fast(float a, float b) {
    return __builtin_amdgcn_fmed3f(a, b, __uint_as_float(0xff800000u));
}
__device__ __forceinline__ float fmax_fast(float a, float b) {
    return __builtin_amdgcn_fmed3f(a, b, __uint_as_float(0x7f800000u));
}

__device__ __forceinline__ float f4get(const float4& v, int i) {
    return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}
__device__ __forceinline__ float u4getf(const uint4& v, int i) {
    return __uint_as_float(i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w);
}

// LDS-DMA issued by inline asm: the compiler does not see these as LDS writes, so it
// does not put a vmcnt(0) in front of the next LDS read (which would serialise every
// tile's compute behind the DMA of the tile after it); the kernel orders them itself
// with waits + s_barrier (wait_dma_barrier).  M0 = the LDS destination (wave-uniform),
// written in the same statement that reads it (the compiler reserves M0 and does not
// preserve it around the statement: the statement saves and restores it).  Wait states
// inside the string, which the compiler does not pad: the SALU write of M0 needs 1 before
// the load reads it (s_nop 0); the scalar base may come straight from v_readfirstlane (a
// VALU write of an SGPR), which needs 5 before a vector-memory instruction reads it as its
// base -- s_nop 2 (3) and the two M0 moves (2) open the string.  Every
// operand is a value fixed before the statement (scalar tile base, the lane's constant
// offset VGPR): no per-tile address arithmetic feeds a DMA.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// a wave-uniform value the compiler may have kept in VGPRs, as SGPRs
__device__ __forceinline__ const void* sgpr_ptr(const void* p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
// scalar base + 32-bit per-lane offset (no per-lane 64-bit address math in the loop)
__device__ __forceinline__ void dma16s(uint32_t voff, const void* sbase, uint32_t lds) {
    sbase = sgpr_ptr(sbase);
    lds = __builtin_amdgcn_readfirstlane(lds);
    uint32_t keep;
    asm volatile("s_nop 2\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds)
                 : "memory");
}
__device__ __forceinline__ void dma4s(uint32_t voff, const void* sbase, uint32_t lds) {
    sbase = sgpr_ptr(sbase);
    lds = __builtin_amdgcn_readfirstlane(lds);
    uint32_t keep;
    asm volatile("s_nop 2\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds)
                 : "memory");
}
// The tile barrier of the LDS-DMA filters: this wave's tile DMAs have landed (vmcnt(0): its
// pieces of the tiles about to be read) AND every LDS read it issued has returned its data
// (lgkmcnt(0)), then s_barrier.  Both halves are needed:
//  * RAW -- after the barrier every wave's pieces of the next tiles are in LDS;
//  * WAR -- a ds_read is asynchronous, and s_barrier does not wait for it.  The DMAs issued
//    after this barrier overwrite the buffers the previous tiles used; a read of such a buffer
//    still in flight at the barrier (its MFMA scheduled after it) would return the NEW bytes.
//    With lgkmcnt(0) here no read of any earlier tile outlives the barrier, whatever order
//    the compiler gives the k-steps (without it the filter was correct only while a
//    per-k-step sched_barrier kept each tile's reads and MFMAs ahead of the barrier).
__device__ __forceinline__ void wait_dma_barrier() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// per-query 4-ary heap stride in floats: node n >= 1 in slot n-1, the root in the last slot;
// slots of nodes >= k hold -inf up to the last child group a parent < k reads (slot k+1)
__host__ __device__ __forceinline__ int heap_stride(int k) { return (k + 3 + 3) & ~3; }

// tile geometry shared by the kernel and the host's LDS sizing: NW waves per block,
// QG 32-query groups per wave, RG 32-row groups per tile; NACC = QG * RG accumulators;
// HS header slots of 16 B after the rows (the fused filter's per-tile norms and statistics)
template <int RB, int NW, int QG, int RG, int HS = 0>
struct FilterTile {
    static constexpr int NACC = QG * RG;             // 32x32 accumulators per wave per tile
    static constexpr int BN = 32 * RG;               // train rows per tile
    static constexpr int BM = 32 * QG * NW;          // queries per block
    static constexpr int STRIDE = RB + 16;           // LDS bytes per tile row
    static constexpr int SLOTS = RB / 16 + 1;        // 16-B slots per padded row
    static constexpr int DMA_INS = (BN * SLOTS + HS + 63) / 64;     // 1 KiB DMA instructions per tile
    static constexpr int LAST_LANES = BN * SLOTS + HS - 64 * (DMA_INS - 1);  // active lanes of the last
    static constexpr int TILE = DMA_INS * 1024;      // LDS bytes per buffer (>= BN * STRIDE + 16 HS)
    static constexpr int HDR = BN * STRIDE;          // LDS offset of the header
};
