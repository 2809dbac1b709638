// knn_study.h -- hooks of the kernel-study builds (`make ablate`, build/ablate/*.so).
// The product library defines none of the KNN_ABLATE_* macros, so every hook below is
// empty there; the studies themselves are documented in DESIGN.md.
#pragma once

#if defined(KNN_ABLATE_NO_SLOW) || defined(KNN_ABLATE_NO_EPI) || defined(KNN_ABLATE_NO_DMA)
// ablation builds time the GEMM filter alone: the fallback scan is skipped (results invalid)
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

// The fused filter's per-k-step scheduling barrier (knn_fused.hip, step()).  Product: a full
// sched_barrier after every k-step.  Study builds (DESIGN.md "Filter studies", all of them
// give WRONG results today): KNN_FUSED_NO_SCHED_BARRIER (none), KNN_FUSED_SB_MASK (the
// instruction classes let through), KNN_FUSED_SB_STEPS (only the first k-steps closed),
// KNN_FUSED_RELAX (none, plus wait states at the head of each step).
#ifndef KNN_FUSED_SB_MASK
#define KNN_FUSED_SB_MASK 0
#endif
#ifndef KNN_FUSED_SB_STEPS
#define KNN_FUSED_SB_STEPS 64
#endif
#if defined(KNN_FUSED_NO_SCHED_BARRIER) || (defined(KNN_FUSED_RELAX) && KNN_FUSED_RELAX)
#define KNN_STUDY_KSTEP_BARRIER(s) \
    do {                           \
    } while (0)
#else
#define KNN_STUDY_KSTEP_BARRIER(s)                                               \
    do {                                                                         \
        if ((s) < KNN_FUSED_SB_STEPS) __builtin_amdgcn_sched_barrier(KNN_FUSED_SB_MASK); \
    } while (0)
#endif
#if defined(KNN_FUSED_RELAX) && KNN_FUSED_RELAX
#define KNN_STUDY_STEP_HEAD()                                  \
    do {                                                       \
        __builtin_amdgcn_sched_barrier(0);                     \
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7");      \
        __builtin_amdgcn_sched_barrier(0);                     \
    } while (0)
#else
#define KNN_STUDY_STEP_HEAD() \
    do {                      \
    } while (0)
#endif
