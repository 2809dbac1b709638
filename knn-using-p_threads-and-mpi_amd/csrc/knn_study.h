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
