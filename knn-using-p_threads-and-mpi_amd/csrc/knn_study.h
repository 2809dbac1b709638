// knn_study.h -- hooks of the kernel-study builds (`make ablate`, build/ablate/*.so).
// The product library defines none of the KNN_ABLATE_* macros, so every hook below is a
// constant that removes nothing there; the studies themselves are documented in DESIGN.md.
#pragma once

// Ablation builds time the GEMM filters with one part of their work removed (results invalid):
//   KNN_ABLATE_NO_SLOW  no slow path (passing values are not visited)
//   KNN_ABLATE_NO_EPI   no fast test between the MFMAs
//   KNN_ABLATE_NO_DMA   no tile copies (the MFMAs read whatever the LDS holds)
#ifdef KNN_ABLATE_NO_SLOW
#define KNN_STUDY_NO_SLOW 1
#else
#define KNN_STUDY_NO_SLOW 0
#endif
#ifdef KNN_ABLATE_NO_EPI
#define KNN_STUDY_NO_EPI 1
#else
#define KNN_STUDY_NO_EPI 0
#endif
#ifdef KNN_ABLATE_NO_DMA
#define KNN_STUDY_NO_DMA 1
#else
#define KNN_STUDY_NO_DMA 0
#endif

// KNN_ABLATE_NO_NORM: the fused filter's accumulators start from zero instead of the tile
// header's norms (no norm ds_read_b128; results invalid) -- prices the norm reads of the
// 32-query shape (round 6).
#ifdef KNN_ABLATE_NO_NORM
#define KNN_STUDY_NO_NORM 1
#else
#define KNN_STUDY_NO_NORM 0
#endif

// KNN_ABLATE_NO_BARRIER: the fused filter's tile barrier keeps its waits but drops the s_barrier
// (results invalid: waves may read tiles other waves' DMAs have not landed) -- prices the
// cross-wave synchronisation.
#ifdef KNN_ABLATE_NO_BARRIER
#define KNN_STUDY_NO_BARRIER 1
#else
#define KNN_STUDY_NO_BARRIER 0
#endif

#if KNN_STUDY_NO_SLOW || KNN_STUDY_NO_EPI || KNN_STUDY_NO_DMA || KNN_STUDY_NO_BARRIER || KNN_STUDY_NO_NORM
// the fallback scan is skipped (results invalid) ...
#define KNN_STUDY_SKIP_FALLBACK(qlist) \
    do {                               \
        if (qlist) return;             \
    } while (0)
// ... and a query left with fewer than k rows is not an error there
#define KNN_STUDY_RESULTS_INVALID 1
#else
#define KNN_STUDY_RESULTS_INVALID 0
#define KNN_STUDY_SKIP_FALLBACK(qlist) \
    do {                               \
    } while (0)
#endif

// The fused filter's instruction order inside a k-step (knn_fused.hip, step()): the compiler
// schedules across the k-steps (round 4, octets: A 21.33 -> 21.08 ms, B equal, r04ae).  The
// order is a performance choice only: correctness rests on the tile barrier retiring every LDS
// read (wait_dma_barrier).  KNN_FUSED_STRICT_SCHEDULE (study) puts a full scheduling barrier
// after every k-step (each step's A-fragment prefetch, DMA piece, MFMAs and fast-test VALU
// kept together: the round-2/3 default).
#ifdef KNN_FUSED_STRICT_SCHEDULE
#define KNN_FUSED_KSTEP_ORDER() __builtin_amdgcn_sched_barrier(0)
#else
#define KNN_FUSED_KSTEP_ORDER() \
    do {                        \
    } while (0)
#endif

// KNN_STUDY_STAMPS: per-wave shader-clock stamps of the fused filter's loop (barrier wait, step,
// slow path), summed over the launch into a device array (knn_debug_stamps).  Timing study only.
#ifdef KNN_STUDY_STAMPS
#define KNN_FUSED_STAMPS 1
#else
#define KNN_FUSED_STAMPS 0
#endif

// KNN_STUDY_AUG64: d = 64 keeps the norm in an augmented k-step (2d + 32 bytes per row) instead
// of starting its accumulators from the tile header's norms (knn_fused_row_bytes).
#ifdef KNN_STUDY_AUG64
#define KNN_FUSED_AUG64 1
#else
#define KNN_FUSED_AUG64 0
#endif

