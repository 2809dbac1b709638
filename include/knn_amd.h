/*
 * knn_amd.h -- C ABI of the MI355X-native KNN classifier (libknn_amd.so).
 *
 * Plain pointers and sizes only; no exceptions cross this boundary.  Every
 * entry point below names the reference interface it replaces
 * (srna99/KNN-using-p_threads-and-MPI, file:line).  The C++ surface that keeps
 * the reference's own names (ArffParser / ArffData / KNN / computeConfusionMatrix
 * / computeAccuracy) lives in knn_arff.hpp and is implemented on top of this ABI.
 *
 * Semantics (all paths, bit-exact with the reference serial KNN, main.cpp:25-85):
 *   distance  = sum_{i<d} (q_i - t_i)^2, fp32, i ascending, no FMA (main.cpp:14-23)
 *   neighbours= the k smallest (distance, train index) pairs -- the reference's
 *               strict-'<' insertion queue keeps the lower index on ties
 *               (main.cpp:45-61); distances >= FLT_MAX or NaN never qualify
 *   vote      = bincount of the k labels, argmax with ties to the smallest label
 *               (main.cpp:64-78)
 * Data layout: row-major features [n][ld] (ld >= d elements, rows 16-B aligned
 * for the device entry points), int32 labels in [0, num_classes).  Features are fp32
 * or bf16 (KNN_BF16: raw bf16 bits; distances are the fp32 direct form on the exactly
 * widened values, i.e. what the reference computes on those values as floats).
 */
#ifndef KNN_AMD_H
#define KNN_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: KNN_OPT_CACHE_TRAIN no longer reuses operands derived from a caller's DEVICE train buffer;
 *    that is the separate opt-in KNN_OPT_CACHE_TRAIN_DEVICE (ABI 2 did it under the one flag) */
#define KNN_AMD_ABI_VERSION 3

typedef enum {
    KNN_OK = 0,
    KNN_EINVAL = 1,   /* bad argument: k > n_train, d mismatch, label outside [0,C), ... */
    KNN_ENOMEM = 2,   /* host or device allocation failed */
    KNN_EHIP = 3,     /* a HIP runtime call failed */
    KNN_ERANGE = 4,   /* fewer than k neighbours with a finite distance (< FLT_MAX) */
    KNN_ENODEV = 5,   /* no usable gfx950 device */
    KNN_EIO = 6,      /* file could not be opened / parsed (ARFF loader) */
    KNN_ERCCL = 7     /* an RCCL call failed (train-sharded exchange) */
} knn_status;

typedef enum { KNN_F32 = 0, KNN_BF16 = 1 } knn_dtype;

typedef enum {
    KNN_ALGO_AUTO = 0,    /* direct form for low d / small problems, MFMA GEMM form otherwise */
    KNN_ALGO_DIRECT = 1,  /* direct form, tiled (k_direct_tile: LDS-staged train tiles shared by
                             the queries of a block, scalar query operands, wave top-k + vote) */
    KNN_ALGO_GEMM = 2,    /* ||q||^2+||t||^2-2q.t on MFMA (fp32 data: fp32 MFMA, bf16 data: bf16
                             MFMA) + certified exact rescore */
    KNN_ALGO_GEMM_SPLIT = 3, /* GEMM form with fp32 data split into bf16 hi + lo (q.t = hi.hi +
                               hi.lo + lo.hi on the bf16 MFMA, fp32-grade certificate) + the
                               same exact fp32 rescore; bf16 data: as KNN_ALGO_GEMM */
    KNN_ALGO_GEMM_BF16 = 4, /* GEMM form with fp32 data rounded to bf16 for the filter only (one
                               bf16 MFMA per 16 features, certificate widened by the rounding
                               error, 2^-7 (|q|^2+|t|^2)) + the same exact fp32 rescore; AUTO
                               runs it first and re-runs a call as KNN_ALGO_GEMM_SPLIT when
                               more than 1/16 of its queries overflow their candidate lists.
                               bf16 data: as KNN_ALGO_GEMM */
    KNN_ALGO_DIRECT_SCAN = 5 /* direct form, one block per query (k_exact_scan, the GEMM path's
                                per-query fallback) */
} knn_algo;

/* knn_opts.flags */
#define KNN_OPT_CACHE_TRAIN 1  /* knn_predict keeps the device copy of train across calls, keyed
                                  by (feat, labels, n, d, ld, dtype) and the generation set by
                                  knn_set_generation, together with the train-side operands of
                                  the bf16 MFMA filter derived from that copy (train norms, tile
                                  statistics, bf16 tile blocks) */
#define KNN_OPT_CACHE_TRAIN_DEVICE 2  /* (with KNN_OPT_CACHE_TRAIN) the device entry points
                                  (knn_predict_device, knn_shard_topk_device,
                                  knn_predict_train_sharded) also keep the filter operands derived
                                  from the CALLER's device train buffer, keyed by (feat, n, d, ld,
                                  dtype, filter tile height) and the generation.  The library
                                  cannot see writes to that buffer: a caller that rewrites it in
                                  place (hipMemcpy, its own kernels) or frees it and reuses the
                                  address must bump the generation (knn_set_generation) before
                                  the next call, or it gets results for the old rows.  Without
                                  this flag every device call rebuilds them (A: ~0.3 ms) */

/* Context options.  One context drives one device (a compute stream and a copy stream). */
typedef struct {
    int32_t device;        /* HIP device ordinal */
    int32_t algo;          /* knn_algo */
    int32_t train_splits;  /* GEMM path: train segments per query tile (0 = auto) */
    int32_t profile;       /* 1 = record per-stage HIP events (knn_stage_times); 2 = also count the
                              filter's candidates (an extra read of the counts per call); 3 = events
                              around the dominant stages only (filter, rescore, direct form, exact
                              scan, exchange, merge): a few microseconds less per stage skipped */
    int32_t flags;         /* KNN_OPT_* */
} knn_opts;

/* A dataset view.  feat: row-major [n][ld] of dtype; labels: int32 [n] (train only). */
typedef struct {
    const void* feat;
    const int32_t* labels;
    int64_t n;
    int32_t d;
    int32_t ld;
    int32_t dtype;         /* knn_dtype */
} knn_dataset;

typedef struct knn_ctx knn_ctx;

/* Library / ABI version (KNN_AMD_ABI_VERSION). */
int32_t knn_version(void);

/* Source hash of the tree this library was built from (16 hex digits; computed by
 * knn-using-p_threads-and-mpi_amd/build_id.py over the package's Makefile, csrc/ and
 * include/).  Tests compare it with the sources beside the library they load. */
const char* knn_build_id(void);

/* Create / destroy a context (replaces the per-run setup in main.cpp:114-131,
 * multi-thread.cpp:133-160 and mpi.cpp:119-149).  A context serves one call at a time:
 * threads that share one serialise their calls (the C++ KNN() does, per device), or each
 * creates its own. */
knn_status knn_create(knn_ctx** out, const knn_opts* opts);
void knn_destroy(knn_ctx* ctx);

/* Text of the last error on this context ("" if none). */
const char* knn_last_error(const knn_ctx* ctx);

/* Invalidates cached train uploads and cached train-side filter operands
 * (KNN_OPT_CACHE_TRAIN): both cache keys include this generation.  The reference has no counterpart (every KNN() call re-reads ArffData,
 * main.cpp:40-43). */
knn_status knn_set_generation(knn_ctx* ctx, uint64_t generation);

/* Page-locked host memory for datasets and outputs of knn_predict: copies from/to it run
 * as asynchronous DMA, overlapping the device's compute (pageable buffers work too, at
 * the runtime's staged rate). */
knn_status knn_alloc_pinned(size_t bytes, void** out);
void knn_free_pinned(void* p);

/*
 * Host-buffer entry point.  Replaces `int* KNN(ArffData* train, ArffData* test, int k)`
 * (main.cpp:25) for queries [0, test->n) and the MPI variant
 * `int* KNN(train, test, k, start, end)` (mpi.cpp:26) / pthreads thread body
 * `void* KNN(void*)` (multi-thread.cpp:37) for a [q_begin, q_end) slice.
 * out_pred: caller-allocated int32[q_end - q_begin].
 * out_topk_dist / out_topk_idx: optional (NULL) [q_end-q_begin][k], ascending.
 * k must satisfy 1 <= k <= train->n (the reference crashes for k > n_train and
 * returns all-zero predictions for k <= 0; the C++ KNN() wrapper reproduces the
 * latter, the ABI reports KNN_EINVAL).
 * Data movement: train is uploaded once per call, or once per context with
 * KNN_OPT_CACHE_TRAIN; queries stream through two device slots in batches -- batch b+1
 * uploads on the context's copy stream while batch b computes, and batch b's results
 * download while b+1 computes.  knn_last_stats()[6] / [7] report the train / query bytes
 * this call moved host -> device.
 */
knn_status knn_predict(knn_ctx* ctx, const knn_dataset* train, const knn_dataset* test,
                       int32_t k, int32_t num_classes, int64_t q_begin, int64_t q_end,
                       int32_t* out_pred, float* out_topk_dist, int32_t* out_topk_idx);

/*
 * Device-buffer entry point (inputs already resident in HBM): all pointers in the
 * datasets and outputs are device pointers on ctx's device; work is enqueued on
 * `hip_stream` (a hipStream_t; NULL = the context's own stream, a blocking stream: ordered
 * after work issued earlier on the legacy null stream).  Returns after
 * the stream has drained and the device-side status word was checked.
 */
knn_status knn_predict_device(knn_ctx* ctx, const knn_dataset* train, const knn_dataset* test,
                              int32_t k, int32_t num_classes, int32_t* d_pred,
                              float* d_topk_dist, int32_t* d_topk_idx, void* hip_stream);

/*
 * Train-sharded runs (the reference has only test-sharded drivers,
 * multi-thread.cpp:154-192 / mpi.cpp:141-186, so these two calls replace the inner
 * loop of `KNN` main.cpp:40-62 split over train shards, and its vote main.cpp:64-78).
 *
 * knn_shard_topk_device: the exact k nearest rows of ONE train shard for every query,
 * written as packed int32 records d_rec[nq][3][k]: k distance bits (fp32, the
 * reference's direct form), k global indices (idx_base + local row; -1 = none) and
 * k labels, ascending by (distance, index).  k may exceed the shard's rows (missing
 * entries are -1).  Device pointers; work on `hip_stream` (NULL = context stream).
 *
 * knn_merge_vote_device: merges nsrc such record blocks, d_rec[nsrc][nq][3][k] (e.g.
 * after an all-to-all over the ranks that own the shards), into each query's k nearest
 * by (distance, global index) -- the reference's tie rule over the whole train set --
 * and votes (smallest label on ties).  d_dist / d_idx (optional) receive [nq][k].
 * Each source list must ascend by (distance, index) with -1 padding last, as
 * knn_shard_topk_device writes it: the merge reads a list in sorted runs and stops at the
 * first run that cannot enter the top k.  A descent inside what it reads gives KNN_EINVAL.
 * KNN_ERANGE if some query has fewer than k neighbours over all shards.
 */
knn_status knn_shard_topk_device(knn_ctx* ctx, const knn_dataset* train_shard, const knn_dataset* test,
                                 int32_t k, int32_t num_classes, int64_t idx_base, int32_t* d_rec,
                                 void* hip_stream);
knn_status knn_merge_vote_device(knn_ctx* ctx, int32_t nsrc, int64_t nq, int32_t k, int32_t num_classes,
                                 const int32_t* d_rec, int32_t* d_pred, float* d_dist, int32_t* d_idx,
                                 void* hip_stream);

/*
 * Train-sharded KNN over ranks, one process per GPU (replaces the MPI
 * collective pattern of mpi.cpp:130-201 -- MPI_Init / Scatter / Gatherv -- for a train set
 * sharded instead of replicated).  The communicator is RCCL (over xGMI on one node),
 * loaded at knn_comm_create.
 *   knn_comm_unique_id: 128 opaque bytes made on one rank and handed to every rank by the
 *     caller's own bootstrap (MPI_Bcast, torch.distributed, a file).
 *   knn_comm_create: ncclCommInitRank on ctx's device; collective over the nranks ranks.
 *   knn_predict_train_sharded: rank r holds train rows [idx_base, idx_base + shard->n) and
 *     every query (test, device buffers); it computes its shard's exact top-k of every query
 *     (knn_shard_topk_device), one grouped send/recv all-to-all hands each rank the lists of
 *     the queries it owns, shard_range(test->n, nranks, rank), and k_merge_vote merges them
 *     by (distance, global index) -- the reference's lower-index tie rule over the whole
 *     train set -- and votes.  d_pred (and optional d_dist / d_idx [owned][k]) receive the
 *     owned queries' results.  Collective: every rank calls it with the same test set and k.
 *     A failure local to one rank (memory, its shard's arguments, a HIP error that leaves the
 *     device usable) is voted on by every rank (one max-allreduce of a preset device word)
 *     before the exchange: the failing rank returns its own status, its peers KNN_ERCCL, and
 *     no rank is left waiting inside the exchange.  A failure of a collective itself (e.g. after
 *     a device fault) aborts the communicator (ncclCommAbort): that rank returns KNN_ERCCL,
 *     every later call on the communicator fails, and peers inside the collective are released
 *     by their own RCCL / watchdog timeout.  With profile = 1 the
 *     context's stage times hold the shard's stages, "exchange" and "merge_vote".
 *   knn_shard_range: the reference's contiguous split with the remainder on the last worker
 *     (multi-thread.cpp:154-158, mpi.cpp:141-170).
 *   knn_exchange_layout: element offsets / counts of the all-to-all for `rank` (int32
 *     records [nq][3][k] sent, [world][owned][3][k] received); arrays of `world` entries.
 */
#define KNN_COMM_ID_BYTES 128
typedef struct knn_comm knn_comm;
knn_status knn_comm_unique_id(void* id_out);
knn_status knn_comm_create(knn_ctx* ctx, const void* id, int32_t nranks, int32_t rank, knn_comm** out);
void knn_comm_destroy(knn_comm* comm);
/* the number of ranks the RCCL communicator spans (ncclCommCount) */
knn_status knn_comm_count(const knn_comm* comm, int32_t* nranks);
/* *broken = 1 once a collective on this communicator failed and it was aborted: every later
 * knn_predict_train_sharded on it returns KNN_ERCCL at once (no shard pass, no collective), so
 * a caller that sees KNN_ERCCL can tell "a peer's shard failed, the communicator is fine" (0)
 * from "tear down every rank and build a new communicator" (1). */
knn_status knn_comm_broken(const knn_comm* comm, int32_t* broken);
/* The exchange's message plan (round 6).  Every RCCL send / recv of knn_predict_train_sharded
 * carries at most chunk_elems int32 (<= 0: the default, 64 Mi elements = 256 MiB); with
 * self_via_rccl = 0 (the default) the rank's own block is a device copy, with 1 it goes through
 * the same grouped ncclSend / ncclRecv loop as the peers' blocks -- so a one-rank communicator
 * executes the multi-rank loop's chunk offsets and counts (the GPU test of that loop; a one-GPU
 * box cannot hold two RCCL ranks).  Not collective; call it alike on every rank. */
knn_status knn_comm_set_exchange(knn_comm* comm, int64_t chunk_elems, int32_t self_via_rccl);
knn_status knn_predict_train_sharded(knn_ctx* ctx, knn_comm* comm, const knn_dataset* train_shard, int64_t idx_base,
                                     const knn_dataset* test, int32_t k, int32_t num_classes, int32_t* d_pred,
                                     float* d_dist, int32_t* d_idx, void* hip_stream);
knn_status knn_shard_range(int64_t n, int32_t world, int32_t rank, int64_t* begin, int64_t* end);
/* The partition of a `world`-GPU run (north_star "Partitioning"; the reference only splits the
 * test set, multi-thread.cpp:154-158 / mpi.cpp:141-170): *policy = KNN_SHARD_TEST (queries split
 * by knn_shard_range, train replicated, no collective on the data path) while one copy of train
 * and its bf16 filter operands fits half of `hbm_bytes` (<= 0: 288 GiB), else KNN_SHARD_TRAIN
 * (knn_predict_train_sharded).  The C++ KNN() (KNN_AMD_SHARD=auto), knn_cli --shard=auto and
 * bench.py --shard auto ask it; every caller may force either partition. */
typedef enum { KNN_SHARD_TEST = 0, KNN_SHARD_TRAIN = 1 } knn_shard_kind;
knn_status knn_shard_policy(int64_t n_train, int64_t n_query, int32_t d, int32_t dtype, int32_t world,
                            int64_t hbm_bytes, int32_t* policy);
knn_status knn_exchange_layout(int64_t nq, int32_t k, int32_t world, int32_t rank, int64_t* send_off,
                               int64_t* send_cnt, int64_t* recv_off, int64_t* recv_cnt);

/* Per-stage device times (ms) of the last predict call when opts.profile >= 1.
 * names: optional array of n const char* to receive stage names. Returns the
 * number of stages recorded (<= n). */
int32_t knn_stage_times(const knn_ctx* ctx, const char** names, float* ms, int32_t n);

/* Counters of the last predict call: [0] GEMM candidates kept, [1] queries sent to
 * the exact fallback, [2] train segments used, [3] filter operand type (-1 = no GEMM
 * filter ran, 0 = fp32, 1 = bf16, 2 = bf16 hi/lo split of fp32, 3 = bf16 rounding of
 * fp32), [4] 1 when AUTO re-ran the call with the split filter, [5] 1 when the filter
 * ran with the train norm folded into the MFMA (the fused-norm bf16 filter), [6] train
 * bytes and [7] query bytes a knn_predict call copied host -> device, [8] 1 when the
 * filter's train-side operands came from the KNN_OPT_CACHE_TRAIN cache (no train norm or
 * tile-block pass ran), [9] the fused filter's MFMA shape (32: v_mfma_f32_32x32x16_bf16,
 * 16: v_mfma_f32_16x16x32_bf16, 0: no fused filter ran), [10] the fused filter's queries per
 * wave (32 or 64, knn_fused_plan's rule; 0: no fused filter ran).  Returns the number
 * written (<= 11). */
int32_t knn_last_stats(const knn_ctx* ctx, int64_t* out, int32_t n);

/*
 * Synthetic generator, device side: fills rows [row0, row0+n) of a
 * row-major [n][ld] device buffer (pad columns zeroed) and optional labels,
 * from the counter-based hash keyed by (seed, stream, row, col).
 * kind: 0 = fp32 on the 2^-23 grid in [-1,1), 1 = bf16-exact k/128; 2 / 3 = the same two
 *       clustered: the row's class centroid + noise, so labels carry signal
 *       (needs num_classes >= 1; bf16 output: kinds 1 and 3).
 * out dtype follows `dtype` (KNN_BF16 stores bf16 bits).
 */
knn_status knn_generate(knn_ctx* ctx, void* d_feat, int32_t* d_labels, int64_t row0, int64_t n,
                        int32_t d, int32_t ld, int32_t dtype, int32_t kind, uint64_t seed,
                        uint32_t stream, int32_t num_classes, void* hip_stream);

/* Evaluation, host side.  computeConfusionMatrix (main.cpp:87-100): cm is
 * caller-allocated int32[C*C], row = true class, col = predicted. */
knn_status knn_confusion_matrix(const int32_t* pred, const int32_t* labels, int64_t n,
                                int32_t num_classes, int32_t* cm);
/* computeAccuracy (main.cpp:102-112): trace(cm) / n as float. */
float knn_accuracy(const int32_t* cm, int32_t num_classes, int64_t n);

/* On-device computeConfusionMatrix (main.cpp:87-100) for predictions that stay in HBM:
 * d_cm (device int32[C*C], overwritten) += 1 at [label][pred] for every query; d_correct
 * (optional device int64[1]) receives trace(cm), so accuracy = *d_correct / (float)n as in
 * computeAccuracy (main.cpp:102-112).  KNN_EINVAL if a label or prediction is outside
 * [0, C) (the reference writes out of bounds there). */
knn_status knn_confusion_matrix_device(knn_ctx* ctx, const int32_t* d_pred, const int32_t* d_labels,
                                       int64_t n, int32_t num_classes, int32_t* d_cm,
                                       int64_t* d_correct, void* hip_stream);

/* Self-test of the hardware assumption behind the bf16 GEMM-form certificate (no
 * reference counterpart; DESIGN.md "Certificate"): runs the bf16 filter's MFMA chain
 * (v_mfma_f32_32x32x16_bf16 over K/16 k-steps, the filter's lane map) on device
 * operands a, b = [32][K] bf16 bits (K % 16 == 0) and writes d_out[i][j] =
 * sum_k a[i][k] b[j][k] as the MFMA accumulates it (device float [32][32]). */
knn_status knn_mfma_probe_bf16(knn_ctx* ctx, const uint16_t* d_a, const uint16_t* d_b, int32_t K,
                               float* d_out, void* hip_stream);

/* ARFF loader (replaces ArffParser::parse, libarff/arff_parser.cpp:23, for the
 * read path): NUMERIC attributes parsed with libarff's istringstream>>float rules.
 * The class is the last attribute. */
typedef struct knn_arff knn_arff;
knn_status knn_arff_open(const char* path, knn_arff** out, char* err, int32_t err_len);
void knn_arff_shape(const knn_arff* h, int64_t* n_instances, int32_t* n_attributes,
                    int32_t* num_classes);
/* Copies features [n][ld] (pad zeroed) and (int)(float) labels of the last attribute. */
knn_status knn_arff_copy(const knn_arff* h, float* feat, int32_t ld, int32_t* labels);
void knn_arff_close(knn_arff* h);

#ifdef __cplusplus
}
#endif
#endif /* KNN_AMD_H */
