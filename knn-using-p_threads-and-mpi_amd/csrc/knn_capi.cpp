// knn_capi.cpp -- the C ABI (include/knn_amd.h): contexts, workspace, stage launches.
//
// Replaces the reference's drivers: the serial loop of main.cpp:25-85, the pthreads
// fan-out of multi-thread.cpp:154-192 and the MPI scatter/gather of mpi.cpp:141-186
// become one device pipeline per context:
//   DIRECT:  k_exact_scan                                  (fused distance/top-k/vote)
//   GEMM:    k_row_norms x2 -> k_gemm_filter -> k_rescore -> k_exact_scan(fallback list)
// Train-sharded runs use the same pipeline per shard with the vote
// replaced by a packed (dist, global idx, label) neighbour list, then k_merge_vote.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/knn_amd.h"
#include "knn_kernels.h"

namespace {

struct DBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n) {
        if (n <= bytes && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, n ? n : 16);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T> T* as() const { return reinterpret_cast<T*>(p); }
};

struct Stage {
    const char* name;
    hipEvent_t a, b;
};

}  // namespace

struct knn_ctx {
    int device = 0;
    int algo = KNN_ALGO_AUTO;
    int train_splits = 0;
    int profile = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // device workspace
    DBuf tnorm, tnp, qnorm, gthr, cnt, cand, fb_list, ctrl, scratch;
    DBuf split_t, split_q;  // KNN_ALGO_GEMM_SPLIT / _BF16: bf16 [hi | lo] / rn copies of fp32 rows
    DBuf pad_t;             // KNN_ALGO_GEMM, n_train not a multiple of 64: the rows padded to the tile grid
    DBuf seg_rec;           // k_direct_tile segment records [nseg][nq][3][k]
    DBuf tmax;              // fused filter: per-64-row train stats {max tn, max |t - rt|, max |rt|, 0}
    DBuf tsmax;             // fused filter: their maxima over all tiles (k_tile_stat_max; cached with tmax)
    DBuf cursor;            // fused filter: per-XCD scan cursors (64-row units; performance hint only)
    DBuf lshare;            // fused filter: per (query, piece) threshold lists shared between pieces
    DBuf qstat;             // fused filter: per-query {|q|, |q - rq|} upper bounds
    DBuf tblk;              // fused filter: train tile blocks [bn rows rn(t) | bn norms | tile stats]
    DBuf tctrl;             // the train norms' share of the status word: [unsafe bits, 0, max norm, 0]
    // train-side operands of the fused filter (tnorm, tnp, tmax, tblk, tctrl) kept across calls
    // under KNN_OPT_CACHE_TRAIN, keyed by the train view, the tile height and the generation;
    // epoch = the upload count of knn_predict's own train buffer (its pointer does not change)
    struct { const void* feat; int64_t n; int d, ld, dtype, bn; uint64_t gen, epoch; bool valid; }
        tprep{nullptr, 0, 0, 0, 0, 0, 0, 0, false};
    uint64_t train_epoch = 0;
    // the same for the non-fused GEMM paths' train copy padded to the 64-row grid (pad_t)
    struct { const void* feat; int64_t n; int d, ld, dtype; uint64_t gen, epoch; bool valid; }
        tpad{nullptr, 0, 0, 0, 0, 0, 0, false};
    int rescore_su = 0;  // test hook KNN_RESCORE_SU: the rescore's LDS staging size (0 = sized)
    // study overrides of the fused filter's plan (KNN_FUSED_QG / _NBUF / _HEAPS), read once at
    // knn_create: a call never reads the environment, and one pass uses one plan throughout
    FusedForce fforce;
    // the device entry points reuse derived train operands across calls only under
    // KNN_OPT_CACHE_TRAIN_DEVICE (the caller's device buffer may change behind the library)
    int cache_train_device = 0;
    // study switches of run_gemm, read once at knn_create
    bool no_lshare = false, no_cursor = false, rescore_all = false;
    // host-API staging (device copies of host inputs / outputs)
    DBuf h_train, h_labels, h_test, h_pred, h_dist, h_idx;
    int32_t* ctrl_host = nullptr;  // pinned, mapped, fine-grained: [0] status, [1] fallback count,
                                   // [4] the sequence number of the last k_finish
    uint32_t finish_seq = 0;
    int32_t* ctrl_host_dev = nullptr;  // its device address (k_finish writes it)
    bool ctrl_clean = false;  // the status words are zero (the last call ended in k_finish)
    DBuf arrive;              // k_direct_rows' fused merge: per query group, segments finished
    bool arrive_clean = false;  // arrive is all zero (the last launch ran to completion)
    bool merge_kernel = false;  // study switch KNN_DIRECT_MERGE_KERNEL=1: k_direct_rows' segments via k_merge_vote
    // host-buffer calls (knn_predict): cached train upload, two query slots streamed on a copy stream
    int cache_train = 0;
    uint64_t generation = 0;
    struct { const void* feat; const int32_t* labels; int64_t n; int d, ld, dtype, ldd; uint64_t gen; bool valid; }
        tcache{nullptr, nullptr, 0, 0, 0, 0, 0, 0, false};
    hipStream_t cstream = nullptr;
    hipEvent_t ev_up[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr}, ev_down[2] = {nullptr, nullptr};
    DBuf q_slot[2], pred_slot[2], dist_slot[2], idx_slot[2];
    std::vector<int32_t*> ctrl_slots;  // pinned copies of the status word, one per batch
    int64_t batch_rows = 131072;       // queries per streamed batch of a host-buffer call
    int64_t ws_queries = 1 << 22;      // GEMM-path queries per pass (candidate workspace budget)
    int64_t h2d_train = 0, h2d_query = 0;
    // profiling
    std::vector<hipEvent_t> events;
    std::vector<Stage> stages;
    bool stage_open = false;  // the last stage_begin recorded an event (profile = 3 skips some)
    std::vector<float> stage_ms;
    std::vector<const char*> stage_names;
    int64_t stats[11] = {0, 0, 0, -1, 0, 0, 0, 0, 0, 0, 0};  // candidates, fallback queries, segments, filter
                                                      // operand type, rerun, fused, train / query H2D
                                                      // bytes, train-side filter operands from the cache
    int subs = 2;                           // candidate sub-slices per segment of the last GEMM pass
    int64_t rerun_stats[3] = {0, -1, 0};    // segments, operand type, fused of AUTO's gated split re-run
    int num_cus = 256;
};

namespace {

knn_status fail(knn_ctx* c, knn_status s, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
knn_status fail(knn_ctx* c, knn_status s, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return s;
}

#define HIP_OR_FAIL(ctx, expr)                                                                  \
    do {                                                                                        \
        hipError_t e__ = (expr);                                                                \
        if (e__ != hipSuccess)                                                                  \
            return fail(ctx, e__ == hipErrorOutOfMemory ? KNN_ENOMEM : KNN_EHIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(e__), __FILE__, __LINE__);                    \
    } while (0)

// HIP_OR_FAIL inside knn_predict's enqueue phase: drain and invalidate first (abort_call)
#define HIP_OR_ABORT(expr)                                                                     \
    do {                                                                                        \
        hipError_t e__ = (expr);                                                                \
        if (e__ != hipSuccess)                                                                  \
            return abort_call(fail(c, e__ == hipErrorOutOfMemory ? KNN_ENOMEM : KNN_EHIP,       \
                                   "%s: %s (%s:%d)", #expr, hipGetErrorString(e__), __FILE__, __LINE__)); \
    } while (0)

// profiling helpers: events are created lazily and reused across calls
// profile = 3: events only around the dominant kernels' stages.  Each event costs the
// stream a few microseconds: with every stage timed, A's 8-GPU share (12,500 queries) ran
// 3.44 -> 3.56 ms per step, A 22.58 -> 22.73 (scripts/event_overhead.py, profiles/r04n).
static bool hot_stage(const char* n) {
    static const char* const hot[] = {"gemm_filter", "rescore", "direct_tile", "exact_scan", "merge_vote", "exchange"};
    for (const char* h : hot)
        if (!strcmp(n, h)) return true;
    return false;
}
void stage_begin(knn_ctx* c, hipStream_t st, const char* name) {
    c->stage_open = false;
    if (!c->profile || (c->profile == 3 && !hot_stage(name))) return;
    size_t i = c->stages.size();
    while (c->events.size() < 2 * (i + 1)) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        c->events.push_back(e);
    }
    Stage s{name, c->events[2 * i], c->events[2 * i + 1]};
    c->stages.push_back(s);
    (void)hipEventRecord(s.a, st);
    c->stage_open = true;
}
void stage_end(knn_ctx* c, hipStream_t st) {
    if (!c->profile || c->stages.empty() || !c->stage_open) return;
    c->stage_open = false;
    (void)hipEventRecord(c->stages.back().b, st);
}

int elem_size(int dtype) { return dtype == KNN_BF16 ? 2 : 4; }

knn_status check_dataset(knn_ctx* c, const knn_dataset* x, const char* what, bool need_labels) {
    if (!x) return fail(c, KNN_EINVAL, "%s dataset is NULL", what);
    if (x->n < 0) return fail(c, KNN_EINVAL, "%s: n < 0", what);
    if (x->d <= 0) return fail(c, KNN_EINVAL, "%s: d must be > 0", what);
    if (x->ld < x->d) return fail(c, KNN_EINVAL, "%s: ld < d", what);
    if (x->dtype != KNN_F32 && x->dtype != KNN_BF16)
        return fail(c, KNN_EINVAL, "%s: dtype must be KNN_F32 or KNN_BF16", what);
    if (x->n > 0 && !x->feat) return fail(c, KNN_EINVAL, "%s: feat is NULL", what);
    if (need_labels && x->n > 0 && !x->labels) return fail(c, KNN_EINVAL, "%s: labels are NULL", what);
    return KNN_OK;
}

// filter operand type of a GEMM-path call: fp32 data runs split (ELEM_SPLIT, bf16 hi/lo
// rows of 4d bytes) under KNN_ALGO_GEMM_SPLIT, rounded (ELEM_ROUND, bf16 rows of 2d bytes)
// under KNN_ALGO_GEMM_BF16, else the data's own type
int filter_elem(int algo, int dtype) {
    if (dtype != KNN_F32) return dtype;
    return algo == KNN_ALGO_GEMM_SPLIT ? ELEM_SPLIT : algo == KNN_ALGO_GEMM_BF16 ? ELEM_ROUND : dtype;
}
int filter_row_bytes(int felem, int d) {
    return felem == ELEM_SPLIT ? 4 * d : felem == ELEM_ROUND ? 2 * d : d * elem_size(felem);
}
bool is_gemm(int algo) {
    return algo == KNN_ALGO_GEMM || algo == KNN_ALGO_GEMM_SPLIT || algo == KNN_ALGO_GEMM_BF16;
}

int choose_algo(const knn_ctx* c, int64_t nt, int64_t nq, int d, int k, int dtype) {
    if (c->algo == KNN_ALGO_DIRECT || c->algo == KNN_ALGO_DIRECT_SCAN) return c->algo;
    // the LDS-DMA filter stages whole rows: a row must be one of its tile widths
    // (128, 256 or 512 bytes: fp32 d = 32/64/128 (fp32 or split), bf16 d = 64/128/256)
    auto gemm_ok = [&](int algo) {
        const int fe = filter_elem(algo, dtype), rb = filter_row_bytes(fe, d);
        return knn_gemm_filter_supported(fe, rb) && k <= 128 && k <= nt &&
               knn_gemm_filter_lds(fe, rb, k) <= 160 * 1024;
    };
    if (is_gemm(c->algo))
        return gemm_ok(c->algo) ? c->algo : KNN_ALGO_DIRECT;
    // AUTO: the direct form wins at low d (3 VALU ops per dim, no rescore) and on small jobs;
    // above that the rounded bf16 filter (one MFMA per 16 features), re-run as split when
    // its wider certificate overflows the candidate lists (predict_core).  For the fused
    // filter's widths (d = 64, 128, 256) "small" now means under 16k rows (round 6, with the
    // small-set pieces): same box, ms per call direct -> filter, d = 128 (rows x queries): 1M x 1
    // 11.7 -> 0.78, 1M x 64 13.0 -> 0.87, 100k x 100 1.07 -> 0.27, 30k x 300 0.41 -> 0.26, 100k x
    // 1000 1.38 -> 0.35, 1M x 500 8.72 -> 1.07; d = 64, k = 32: 50k x 200 0.61 -> 0.37, 100k x
    // 2000 2.51 -> 0.49; 20k x 150 0.29 either way; at 10k rows the two are equal (0.21-0.26)
    // and the direct form wins at d = 64, k = 32 (0.25 vs 0.31; profiles/r06_studies/r06au).
    // Other widths keep the 10^9-pair rule.
    const double pairs = (double)nt * (double)nq;
    if (d >= 32 && nt >= 8192 && (pairs >= 1e9 || (knn_fused_supported(d) && nt >= 16384))) {
        if (gemm_ok(KNN_ALGO_GEMM_BF16)) return KNN_ALGO_GEMM_BF16;
        if (gemm_ok(KNN_ALGO_GEMM_SPLIT)) return KNN_ALGO_GEMM_SPLIT;
        if (gemm_ok(KNN_ALGO_GEMM)) return KNN_ALGO_GEMM;
    }
    return KNN_ALGO_DIRECT;
}

// per-stage times of the drained stream (profile mode)
void collect_stages(knn_ctx* c) {
    if (!c->profile) return;
    c->stage_ms.clear();
    c->stage_names.clear();
    for (auto& s : c->stages) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, s.a, s.b);
        c->stage_ms.push_back(ms);
        c->stage_names.push_back(s.name);
    }
}

knn_status check_status(knn_ctx* c, const int32_t* ctrl) {
    const int32_t status = ctrl[0];
    if (status & KNN_STATUS_BAD_LABEL) return fail(c, KNN_EINVAL, "a train label is outside [0, num_classes)");
    if (status & KNN_STATUS_UNSORTED)
        return fail(c, KNN_EINVAL, "merge: a source neighbour list is not ascending by (distance, index)");
    if (status & KNN_STATUS_TOO_FEW) return fail(c, KNN_ERANGE, "fewer than k train rows have a finite distance (< FLT_MAX)");
    return KNN_OK;
}

// the one host synchronisation of a call: k_finish writes the status words to the host's
// mapped copy and zeroes them for the next call, then the stream drains.  The host first spins
// (up to 200 us) on the sequence word k_finish writes last: a short call returns ~6 us sooner
// than through hipStreamSynchronize, whose completion signal costs ~12 us per wait even for a
// finished stream (scripts/diag/sync_latency.hip, profiles/r06_studies/r06sync.log).  Longer
// calls, and profile mode (its events are read through the runtime), end in the stream sync.
knn_status finish_call(knn_ctx* c, hipStream_t st) {
    const uint32_t seq = ++c->finish_seq;
    HIP_OR_FAIL(c, knn_launch_finish(c->ctrl.as<int32_t>(), c->ctrl_host_dev, 4, seq, st));
    bool done = false;
    if (!c->profile) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int spin = 0;; spin++) {
            if ((uint32_t)__atomic_load_n(c->ctrl_host + 4, __ATOMIC_ACQUIRE) == seq) {
                done = true;
                break;
            }
            if ((spin & 63) == 63 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) break;
            __builtin_ia32_pause();  // (x86-64 host: yield the core's pipeline to its sibling thread)
        }
    }
    if (!done) HIP_OR_FAIL(c, hipStreamSynchronize(st));
    c->ctrl_clean = true;
    c->arrive_clean = true;  // every query group's merging wave reset its counter
    collect_stages(c);
    return check_status(c, c->ctrl_host);
}
// a call's first enqueue: the status words start at zero (k_finish left them so, unless the last
// call failed before it ran)
hipError_t reset_ctrl(knn_ctx* c, hipStream_t st) {
    const bool clean = c->ctrl_clean;
    c->ctrl_clean = false;
    return clean ? hipSuccess : hipMemsetAsync(c->ctrl.p, 0, 4 * sizeof(int32_t), st);
}

// k_direct_tile segments: enough (query block, segment) units to fill whole waves of
// resident blocks (more segments only when they raise the filled fraction by > 2 %, each
// one costs a merge pass), at least 4 tiles per segment, records within 2 GB
int choose_direct_segments(const knn_ctx* c, int64_t nt, int64_t nq, int d, int k, int C, int elem) {
    int qb = 1, occ = 1;
    if (knn_direct_units(k, elem, d, C, &qb, &occ) != hipSuccess || occ < 1) occ = 1;
    const int64_t nqb = (nq + qb - 1) / qb;
    const int64_t slots = (int64_t)occ * c->num_cus;
    if (qb < knn_direct_tile_qb(k)) {
        // k_direct_rows (a wave per unit): about one round of resident waves -- its waves need
        // no co-residents to hide a barrier, and every segment adds a sorted first tile and a
        // merge source (config L, 859 query pairs, same box: 4 segments 0.092 ms, 5 0.094, 8
        // 0.089, 12 0.097, 16 0.103, 32 0.131; r05y)
        const int64_t want = (slots + nqb / 2) / nqb;
        int64_t s = std::max<int64_t>(1, std::min<int64_t>(want, 32));
        while (s > 1 && nt / s < 256) s--;
        while (s > 1 && (double)s * (double)nq * 12.0 * k > 2e9) s--;
        return (int)s;
    }
    int best = 1;
    double best_eff = 0.0;
    for (int s = 1; s <= 32; s++) {
        if (s > 1 && nt / s < 256) break;
        if (s > 1 && (double)s * (double)nq * 12.0 * k > 2e9) break;
        const int64_t w = nqb * s;
        const double eff = (double)w / (double)(((w + slots - 1) / slots) * slots);
        if (eff > best_eff + 0.02) { best = s; best_eff = eff; }
    }
    return best;
}

// the direct form over the whole query set: k_direct_tile (+ k_merge_vote of its segments)
knn_status run_direct_tile(knn_ctx* c, const knn_dataset* tr, const knn_dataset* te, int k, int C,
                           const QueryOut& out, hipStream_t st) {
    DirectTileArgs a{};
    a.train = tr->feat; a.labels = tr->labels; a.nt = tr->n; a.ld_t = tr->ld;
    a.test = te->feat; a.ld_q = te->ld; a.nq = te->n;
    a.d = tr->d; a.k = k; a.C = C; a.elem = tr->dtype;
    a.status = c->ctrl.as<int32_t>();
    const int nseg = c->train_splits > 0 ? std::min(32, c->train_splits)
                                         : choose_direct_segments(c, tr->n, te->n, tr->d, k, C, tr->dtype);
    a.nseg = nseg;
    a.seg_len = (tr->n + nseg - 1) / nseg;
    c->stats[2] = nseg;
    if (nseg == 1) {
        a.out = out;
        HIP_OR_FAIL(c, knn_launch_direct_tile(a, st));
        return KNN_OK;
    }
    HIP_OR_FAIL(c, c->seg_rec.ensure(sizeof(int32_t) * 3 * (size_t)k * (size_t)te->n * nseg));
    a.rec = c->seg_rec.as<int32_t>();
    if (knn_direct_rows_shape(k, tr->d) && !c->merge_kernel) {
        // k_direct_rows merges its segments itself (the last wave of a query group to finish):
        // one launch, no k_merge_vote pass (config L: 0.012 ms of merge + a launch, round 6)
        const int64_t groups = knn_direct_rows_groups(te->n);
        const void* before = c->arrive.p;
        HIP_OR_FAIL(c, c->arrive.ensure(sizeof(int32_t) * (size_t)groups));
        if (c->arrive.p != before) c->arrive_clean = false;
        if (!c->arrive_clean) HIP_OR_FAIL(c, hipMemsetAsync(c->arrive.p, 0, c->arrive.bytes, st));
        c->arrive_clean = false;  // (set again when the call's stream synchronises)
        a.arrive = c->arrive.as<int32_t>();
        a.out = out;
        HIP_OR_FAIL(c, knn_launch_direct_tile(a, st));
        return KNN_OK;
    }
    HIP_OR_FAIL(c, knn_launch_direct_tile(a, st));
    // (the merge is its own stage: "direct_tile" times the distance kernel alone)
    stage_end(c, st);
    stage_begin(c, st, "merge_vote");
    MergeArgs m{};
    m.rec = a.rec; m.nsrc = nseg; m.nq = te->n; m.k = k; m.C = C;
    m.out = out; m.status = a.status; m.labels = tr->labels;
    HIP_OR_FAIL(c, knn_launch_merge(m, st));
    return KNN_OK;
}

// one k_exact_scan block per query: KNN_ALGO_DIRECT_SCAN over every query, or the GEMM
// path's fallback over a device-side query list (qlist / qcount)
knn_status run_exact_scan(knn_ctx* c, const knn_dataset* tr, const knn_dataset* te, int k, int C,
                          const QueryOut& out, hipStream_t st, const int32_t* qlist, const int32_t* qcount) {
    ExactScanArgs a{};
    a.train = tr->feat; a.labels = tr->labels; a.nt = tr->n; a.ld_t = tr->ld;
    a.test = te->feat; a.ld_q = te->ld; a.nq = te->n;
    a.d = tr->d; a.k = k; a.C = C; a.elem = tr->dtype;
    a.qlist = qlist; a.qcount = qcount;
    a.out = out; a.status = c->ctrl.as<int32_t>();
    const int grid = qlist ? std::max(1, 2 * c->num_cus) : (int)std::min<int64_t>(te->n, 16384);
    if (grid <= 0) return KNN_OK;
    HIP_OR_FAIL(c, knn_launch_exact_scan(a, grid, st));
    return KNN_OK;
}

// GEMM-form certificate constants: Delta = coef*(qn+tn) + eta, u = 2^-24.
//   fp32 MFMA (an exact fmaf chain):  coef = (4d+32) u, eta = (6d+8) 2^-149
//   bf16 MFMA (products exact; internal sums assumed no worse than 2u per add, and
//   denormal results possibly flushed):  coef = (6d+32) u, eta = (6d+8) 2^-125
//   split (fp32 x = hi + lo + r, |r| <= 2^-16 |x| (+2^-134); q.t ~ hi.hi + hi.lo + lo.hi
//   on the bf16 MFMA): the dropped terms lo.lo, (hi+lo) r_t, r_q (hi+lo) give
//   <= 3.04 2^-16 sum|q_i t_i| <= 1.52 2^-16 N (N = qn + tn), i.e. <= 779 u N in G; the
//   accumulation of 3d exact products at 2u per add gives <= 6.1 d u N in G; the norm
//   and final-rounding terms are the fp32 ones, (3d+32) u N.  Flushed subnormal operands
//   (<= 2^-126 |t_i| each, <= (1+N)/2 2^-126 by |t_i| <= (1+t_i^2)/2) add <= 3.1 d 2^-126
//   (1+N).  coef = (10d + 840) u, eta = (8d+8) 2^-125.
//   rounded (fp32 x -> bf16 rn(x), |rn(x) - x| <= 2^-8 |x| (+2^-134)): each product moves by
//   <= (2^-7 + 2^-16) |q_i t_i|, in sum <= (2^-7 + 2^-16) N/2, i.e. <= 131328 u N in G; the
//   accumulation of d exact products at 2u per add gives <= 2.02 d u N in G; norm and final
//   roundings (3d+32) u N; L/U/Delta roundings and slack within 512 u N.  Flushed or
//   subnormal operands as for split.  coef = (6d + 131840) u, eta = (8d+8) 2^-125.
void certificate(int d, int felem, float* coef, float* eta) {
    if (felem == ELEM_ROUND) {
        *coef = (float)(6 * d + 131840) * 0x1p-24f;
        *eta = (float)(8 * d + 8) * 0x1p-125f;
    } else if (felem == ELEM_SPLIT) {
        *coef = (float)(10 * d + 840) * 0x1p-24f;
        *eta = (float)(8 * d + 8) * 0x1p-125f;
    } else if (felem == KNN_BF16) {
        *coef = (float)(6 * d + 32) * 0x1p-24f;
        *eta = (float)(6 * d + 8) * 0x1p-125f;
    } else {
        *coef = (float)(4 * d + 32) * 0x1p-24f;
        *eta = (float)(6 * d + 8) * 0x1p-149f;
    }
}

// Fused-norm filter (knn_fused.hip): y = fl_mfma(tn + sum -2 rq_i rt_i) -- the fp32 norm from
// the tile block's header is the first MFMA's C operand, every d (the KNN_STUDY_AUG64 build
// splits it over an augmented k-step at d = 64 instead: + tn_hi + tn_mid + tn_lo, the terms
// the coefficient still covers), G = fl(qn + y), Delta = coef (qn +
// tn) + eta; rq, rt = the bf16 operands (q, t themselves for bf16 data, rn(q), rn(t) for fp32
// data).  With N = qn + tn (exact norms):
//   MFMA accumulation of d + 3 terms (d + 1 with the C-operand norm) at <= 2u per add, terms
//   summing to <= 2.01 N: 4.02 (d+3) u N
//   tn split hi + mid + lo (each subtraction exact): <= 2^-24 tn <= u N (0 with the C operand)
//   fp32 norms (fmaf chains): <= 1.01 d u each, 2.02 d u N;  G's rounding: <= 3.01 u N
//   the reference's D vs the exact distance: <= 2 (d+2) u N
// -> (8.04 d + 20.1) u N; the roundings of s, coef s, L and U and slack in 512 u N:
//   coef = (9d + 512) u.
// Rounded fp32 data adds the operand rounding, exactly 2 (q.t - rq.rt) = 2 (q.(t - rt) +
// (q - rq).rt), bounded by Cauchy-Schwarz with the row statistics of k_row_norms:
//   |.| <= 2 (|q| |t - rt| + |q - rq| |rt|)   (rq = rn(-2q) / -2, rt = rn(t))
// -- per (query, 64-row tile) with the tile's maxima, added to Delta by the kernel (tq.y).
// For random rounding errors it is ~2.6x tighter than the worst case (2^-7 + 2^-16) N
// (the round-1 coefficient 131328 u); for bf16 data it is 0.  (The terms of the MFMA
// sum stay <= 2.01 N: |rq_i rt_i| <= (1 + 2^-8)^2 |q_i t_i|.)
// eta (products or partial sums flushed to zero, subnormal operand rounding): (8d + 16) 2^-125.
void certificate_fused(int d, bool /*rounded*/, float* coef, float* eta) {
    *coef = (float)(9 * d + 512) * 0x1p-24f;
    *eta = (float)(8 * d + 16) * 0x1p-125f;
}

// the most train segments (or schedule pieces) per query tile, at most smax, whose expected
// kept rows fit their slice of the candidate list (choose_splits' rule)
int max_splits(int64_t nt, int k, int cap, int smax = 8) {
    int best = 1;
    for (int s = 2; s <= smax; s++) {
        const double rows = (double)nt / s;
        const double expect = k * (1.0 + std::log(std::max(rows / k, 1.0))) + 64.0;
        if (1.5 * (0.5 * expect + 32.0) > (double)(cap / s / 2)) break;
        best = s;
    }
    return best;
}

int choose_splits(const knn_ctx* c, int64_t n_qtiles, int64_t nt, int dtype, int rb, int k, int cap,
                  bool fused = false, int d = 0, const FilterPlan* fplan = nullptr, int smax = 8) {
    if (c->train_splits > 0) return std::min(8, c->train_splits);
    // More segments shrink the partial last wave of blocks (measured on config A:
    // S=3 224 ms, S=5 217 ms, S=8 216 ms), but each segment must fit its rows in its
    // slice of the candidate list: a running k-smallest threshold keeps about
    // k (1 + ln(rows / k)) rows (the expected number of records) plus a 64-row warm-up
    // tile; the slice gets a 1.5x margin.  Overflowing queries still finish exactly,
    // on the slow full-scan fallback.
    int occ = 1;
    const hipError_t oe = fused ? knn_fused_occupancy(d, *fplan, &occ) : knn_gemm_filter_occupancy(dtype, rb, k, &occ);
    if (oe != hipSuccess || occ < 1) occ = 1;
    const int64_t slots = (int64_t)occ * c->num_cus;
    int best = 1;
    double best_eff = 0.0;
    for (int s = 1; s <= smax; s++) {
        const double rows = (double)nt / s;
        if (s > 1 && rows < 64 * 64) break;
        const double expect = k * (1.0 + std::log(std::max(rows / k, 1.0))) + 64.0;
        // each lane half of a query fills its own half of the slice with about half the rows
        if (s > 1 && 1.5 * (0.5 * expect + 32.0) > (double)(cap / s / 2)) break;
        const int64_t w = n_qtiles * s;
        const double eff = (double)w / (double)(((w + slots - 1) / slots) * slots);
        if (eff >= best_eff) { best = s; best_eff = eff; }
    }
    return best;
}

// The GEMM pipeline of one filter operand type, enqueued on st with no host round trip:
// norms -> operand rows -> filter -> rescore (queries whose candidate list overflowed, or
// every query when a norm is too large for the certificate, go to the fallback list).
// gate (optional): every stage runs only when *gate != 0 (AUTO's re-run, decided on the
// device by k_rerun_decide).  The fallback scan is enqueued by the caller.
knn_status run_gemm(knn_ctx* c, const knn_dataset* tr, const knn_dataset* te, int k, int C,
                    const QueryOut& out, hipStream_t st, int algo, const int32_t* gate) {
    const int64_t nt = tr->n, nq = te->n;
    const int d = tr->d;
    const int dtype = tr->dtype;
    const int felem = filter_elem(algo, dtype);  // the filter's operand type
    const int rb = filter_row_bytes(felem, d);
    const int kelem = felem == ELEM_ROUND ? ELEM_BF16 : felem;  // ELEM_ROUND runs the bf16 kernel
    // Small query sets (round 6): when the base list's pieces would leave CUs idle (256-query
    // tiles x max_splits pieces under 80 % of the CUs -- a 3,125-query call on A's rows ran 13
    // tiles x 5 pieces on 256 CUs), a candidate list 2-4x as long per query, so the filter may
    // cut each query tile into up to 16 pieces (32 candidate sub-slices; 32 pieces for the tiny
    // sets below, 64 sub-slices, k_rescore's limit).  The
    // workspace stays within 1.5 GiB.  The queries-per-wave choice (knn_fused_plan) still
    // counts the base list's pieces: 64-query waves cut into more than ~5 pieces lost to the
    // 32-query shape (A's rows, 6,250 queries: 2.06 against 1.84 ms, r06bh).  (The 16x16x32
    // study filter's quarter lists: 8 pieces.)
    const size_t per_q = 12 * 64 * (size_t)KNN_RESCORE_CAPW, ws_lim = (size_t)1536 << 20;
    const bool idle = (nq + 255) / 256 * (int64_t)max_splits(nt, k, 64 * KNN_RESCORE_CAPW) * 5 < (int64_t)4 * c->num_cus;
    // (a handful of query tiles, idle even at 16 pieces each -- 1,000 queries: 4 tiles -- gets
    // an 8x list and up to 32 pieces, 64 sub-slices)
    const bool tiny = idle && (nq + 255) / 256 * 16 * 5 < (int64_t)4 * c->num_cus;
    const int capmul = (c->fforce.m16 || !idle) ? 1
                     : tiny && (size_t)nq * per_q * 8 <= ws_lim ? 8
                     : (size_t)nq * per_q * 4 <= ws_lim ? 4
                     : (size_t)nq * per_q * 2 <= ws_lim ? 2 : 1;
    const int cap = 64 * KNN_RESCORE_CAPW * capmul;
    const int smax = capmul == 8 ? 32 : capmul > 1 ? 16 : 8;
    HIP_OR_FAIL(c, c->tnorm.ensure(sizeof(float) * (nt + 64)));
    HIP_OR_FAIL(c, c->tnp.ensure(sizeof(float) * (nt + 64)));
    HIP_OR_FAIL(c, c->qnorm.ensure(sizeof(float) * nq));
    HIP_OR_FAIL(c, c->gthr.ensure(sizeof(uint32_t) * nq));
    HIP_OR_FAIL(c, c->cnt.ensure(sizeof(int32_t) * nq * 64));  // [subs * nseg][nq], subs * nseg <= 64
    HIP_OR_FAIL(c, c->cand.ensure(sizeof(CandRec) * nq * cap));
    HIP_OR_FAIL(c, c->fb_list.ensure(sizeof(int32_t) * nq));

    // bf16 MFMA operands (rounded fp32 rows or bf16 data) run the fused-norm filter
    // the fused filter's plan, computed once: it sizes the tile blocks (bn_f), the occupancy,
    // the schedule and the launch of this pass
    const FilterPlan fplan = knn_fused_supported(d) ? knn_fused_plan(d, k, nq, c->num_cus, c->fforce, max_splits(nt, k, 64 * KNN_RESCORE_CAPW)) : FilterPlan{};
    const bool fused = (felem == ELEM_ROUND || felem == ELEM_BF16) && knn_fused_supported(d) && fplan.nw > 0;
    float coef, eta;
    if (fused) {
        certificate_fused(d, felem == ELEM_ROUND, &coef, &eta);
        HIP_OR_FAIL(c, c->tmax.ensure(sizeof(float4) * ((nt + 63) / 64 + 1)));
        HIP_OR_FAIL(c, c->tsmax.ensure(sizeof(float4)));
        HIP_OR_FAIL(c, c->qstat.ensure(sizeof(float2) * (nq + 1)));
    } else {
        certificate(d, felem, &coef, &eta);
    }
    // train-side operands of the fused filter: norms + tile statistics (k_row_norms) and the
    // tile blocks (k_tn_rows), reused from an earlier call on the same train view when the
    // context caches train (no train pass at all then; main.cpp:40-43 re-reads every train row
    // per query, this is the part of that work that depends on train alone)
    const bool fused_tn = fused && knn_fused_row_bytes(d) == 2 * d;
    const int bn_f = fused ? 32 * fplan.rg : 0;
    const bool own_train = tr->feat == c->h_train.p;  // knn_predict's uploaded copy
    // derived train operands are reused for knn_predict's own upload (KNN_OPT_CACHE_TRAIN), and
    // for a caller's device buffer only under KNN_OPT_CACHE_TRAIN_DEVICE
    const bool may_cache = c->cache_train && (own_train || c->cache_train_device);
    auto& tp = c->tprep;
    const bool prep_hit = fused_tn && !gate && may_cache && tp.valid && tp.feat == tr->feat && tp.n == nt &&
                          tp.d == d && tp.ld == tr->ld && tp.dtype == dtype && tp.bn == bn_f &&
                          tp.gen == c->generation && tp.epoch == (own_train ? c->train_epoch : 0);
    if (fused_tn && !gate) {
        HIP_OR_FAIL(c, c->tctrl.ensure(4 * sizeof(int32_t)));
        tp.valid = false;  // (set again below once this call's train pass is enqueued)
    }
    stage_begin(c, st, gate ? "norms_rerun" : "norms");
    if (fused_tn && !gate) {
        // train norms into their own status words, then into this call's status word
        if (!prep_hit) {
            HIP_OR_FAIL(c, hipMemsetAsync(c->tctrl.p, 0, 4 * sizeof(int32_t), st));
            HIP_OR_FAIL(c, knn_launch_row_norms(tr->feat, dtype, nt, tr->ld, d, c->tnorm.as<float>(),
                                                c->tctrl.as<int32_t>(), c->tctrl.as<uint32_t>() + 2,
                                                c->tnp.as<float>(), 1.0f - coef, st, c->tmax.as<float4>(), nullptr));
            HIP_OR_FAIL(c, knn_launch_tile_stat_max(c->tmax.as<float4>(), (nt + 63) / 64, c->tsmax.as<float4>(), st));
        }
        HIP_OR_FAIL(c, hipMemcpyAsync(c->ctrl.p, c->tctrl.p, 4 * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    } else {
        HIP_OR_FAIL(c, knn_launch_row_norms(tr->feat, dtype, nt, tr->ld, d, c->tnorm.as<float>(),
                                            c->ctrl.as<int32_t>(), c->ctrl.as<uint32_t>() + 2,
                                            c->tnp.as<float>(), 1.0f - coef, st, fused ? c->tmax.as<float4>() : nullptr,
                                            gate));
        if (fused && !gate)
            HIP_OR_FAIL(c, knn_launch_tile_stat_max(c->tmax.as<float4>(), (nt + 63) / 64, c->tsmax.as<float4>(), st));
    }
    // (the fused filter's query operand is rn(-2 q): its rounding is bounded for rn(-2 q) / -2)
    HIP_OR_FAIL(c, knn_launch_row_norms(te->feat, dtype, nq, te->ld, d, c->qnorm.as<float>(),
                                        c->ctrl.as<int32_t>(), nullptr, nullptr, 0.0f, st, nullptr, gate,
                                        fused ? c->qstat.as<float2>() : nullptr, -2.0f));
    stage_end(c, st);
    // (a norm >= 2^125 sets GEMM_UNSAFE in the status word: the filter then skips and the
    // rescore sends every query to the exact fallback scan -- decided on the device)
    stage_begin(c, st, gate ? "filter_init_rerun" : "filter_init");
    HIP_OR_FAIL(c, knn_launch_fill_u32(c->gthr.as<uint32_t>(), nq, 0xFF800000u, gate, st));  // ordered(+inf)
    stage_end(c, st);

    // filter operands: the rows themselves, or their bf16 [hi | lo] split (2d elements per row);
    // train operand rows always cover the 64-row tile grid (ntp rows)
    const int64_t ntp = (nt + 63) / 64 * 64;
    const void* ftrain = tr->feat;
    const void* ftest = te->feat;
    int fld_t = tr->ld, fld_q = te->ld;
    if (fused_tn) {
        // train as tile blocks [bn rows of rn(t) | bn norms | tile statistics] (the
        // filter starts each accumulator from the norms), queries as rn(-2 q) rows; one more
        // tile of pad blocks past the grid (the filter scans tiles in twos, k_gemm_fused).
        // The gated split re-run never takes this branch (the fused filter is the first pass).
        const int64_t ntf = ntp + 256;  // (256 pad rows: a piece's scan may run up to 224 rows past
                                        //  its own -- seven 32-row tiles of an octet, k_gemm_fused)
        const size_t tb = (size_t)bn_f * 2 * d + 4 * bn_f + 16;
        HIP_OR_FAIL(c, c->split_q.ensure(sizeof(uint16_t) * (size_t)d * nq));
        stage_begin(c, st, "aug");
        if (!prep_hit) {
            HIP_OR_FAIL(c, c->tblk.ensure(tb * (size_t)(ntf / bn_f)));
            HIP_OR_FAIL(c, knn_launch_tn_rows(tr->feat, dtype, ntf, nt, tr->ld, d, c->tnorm.as<float>(), 1.0f,
                                              c->tblk.p, c->tmax.as<float4>(), bn_f, st, nullptr));
        }
        HIP_OR_FAIL(c, knn_launch_tn_rows(te->feat, dtype, nq, nq, te->ld, d, nullptr, -2.0f, c->split_q.p, nullptr,
                                          0, st, nullptr));
        stage_end(c, st);
        ftrain = c->tblk.p; ftest = c->split_q.p;
        fld_t = fld_q = d;
        c->stats[8] = prep_hit ? 1 : 0;
        if (may_cache)
            tp = {tr->feat, nt, d, tr->ld, dtype, bn_f, c->generation, own_train ? c->train_epoch : 0, true};
    } else if (fused) {
        // (study build KNN_STUDY_AUG64, d = 64) augmented bf16 rows: train [rn(t) | tn split],
        // queries [-2 rn(q) | 1 1 1]
        // (pad rows: zero features, a huge norm -- they never pass)
        // (pad rows past the grid: the filter scans tiles in twos, k_gemm_fused)
        const int64_t ntf = ntp + 256;
        HIP_OR_FAIL(c, c->split_t.ensure(sizeof(uint16_t) * (size_t)(d + 16) * ntf));
        HIP_OR_FAIL(c, c->split_q.ensure(sizeof(uint16_t) * (size_t)(d + 16) * nq));
        stage_begin(c, st, gate ? "aug_rerun" : "aug");
        HIP_OR_FAIL(c, knn_launch_aug_rows(tr->feat, dtype, ntf, nt, tr->ld, d, c->tnorm.as<float>(), 1.0f,
                                           c->split_t.as<uint16_t>(), c->tmax.as<float4>(), st, gate));
        HIP_OR_FAIL(c, knn_launch_aug_rows(te->feat, dtype, nq, nq, te->ld, d, nullptr, -2.0f,
                                           c->split_q.as<uint16_t>(), nullptr, st, gate));
        stage_end(c, st);
        ftrain = c->split_t.p; ftest = c->split_q.p;
        fld_t = fld_q = d + 16;
    } else if (felem == ELEM_SPLIT) {
        HIP_OR_FAIL(c, c->split_t.ensure(sizeof(uint16_t) * 2 * d * ntp));
        HIP_OR_FAIL(c, c->split_q.ensure(sizeof(uint16_t) * 2 * d * nq));
        stage_begin(c, st, gate ? "split_rerun" : "split");
        HIP_OR_FAIL(c, hipMemsetAsync(c->split_t.as<uint16_t>() + 2 * d * nt, 0, sizeof(uint16_t) * 2 * d * (ntp - nt), st));
        HIP_OR_FAIL(c, knn_launch_split_rows((const float*)tr->feat, nt, tr->ld, d, c->split_t.as<uint16_t>(), st, gate));
        HIP_OR_FAIL(c, knn_launch_split_rows((const float*)te->feat, nq, te->ld, d, c->split_q.as<uint16_t>(), st, gate));
        stage_end(c, st);
        ftrain = c->split_t.p; ftest = c->split_q.p;
        fld_t = fld_q = 2 * d;
    } else if (felem == ELEM_ROUND) {
        HIP_OR_FAIL(c, c->split_t.ensure(sizeof(uint16_t) * d * ntp));
        HIP_OR_FAIL(c, c->split_q.ensure(sizeof(uint16_t) * d * nq));
        stage_begin(c, st, gate ? "round_rerun" : "round");
        HIP_OR_FAIL(c, hipMemsetAsync(c->split_t.as<uint16_t>() + d * nt, 0, sizeof(uint16_t) * d * (ntp - nt), st));
        HIP_OR_FAIL(c, knn_launch_round_rows((const float*)tr->feat, nt, tr->ld, d, c->split_t.as<uint16_t>(), st, gate));
        HIP_OR_FAIL(c, knn_launch_round_rows((const float*)te->feat, nq, te->ld, d, c->split_q.as<uint16_t>(), st, gate));
        stage_end(c, st);
        ftrain = c->split_t.p; ftest = c->split_q.p;
        fld_t = fld_q = d;
    } else if (nt % 64) {
        // the caller's rows, copied onto the 64-row tile grid: every tile the filter copies
        // into LDS is whole (one DMA form, knn_kernels.hip), the pad rows never pass (+inf norms).
        // Kept across calls like the fused operands (KNN_OPT_CACHE_TRAIN, same key).
        const size_t es = (size_t)elem_size(dtype), pitch = es * (size_t)tr->ld;
        auto& pk = c->tpad;
        const uint64_t ep = tr->feat == c->h_train.p ? c->train_epoch : 0;
        const bool hit = may_cache && pk.valid && pk.feat == tr->feat && pk.n == nt && pk.d == d &&
                         pk.ld == tr->ld && pk.dtype == dtype && pk.gen == c->generation && pk.epoch == ep;
        pk.valid = false;
        if (!hit) {
            HIP_OR_FAIL(c, c->pad_t.ensure(pitch * (size_t)ntp));
            HIP_OR_FAIL(c, hipMemcpyAsync(c->pad_t.p, tr->feat, pitch * (size_t)nt, hipMemcpyDeviceToDevice, st));
            HIP_OR_FAIL(c, hipMemsetAsync((unsigned char*)c->pad_t.p + pitch * (size_t)nt, 0, pitch * (size_t)(ntp - nt), st));
        }
        if (may_cache) pk = {tr->feat, nt, d, tr->ld, dtype, c->generation, ep, true};
        ftrain = c->pad_t.p;
    }

    const FilterPlan plan = fused ? fplan : knn_gemm_filter_plan(kelem, rb, k);
    const bool shared = fused && !c->no_lshare && knn_fused_list_share_width(plan) > 0;
    const int64_t n_qtiles = (nq + plan.bm - 1) / plan.bm;
    GemmFilterArgs g{};
    g.nt = nt; g.n_qtiles = (int)n_qtiles;
    // fused filter: the balanced schedule (knn_fused_schedule) when its pieces per query tile
    // fit the candidate list like segments do; else (or with explicit train_splits) segments
    int nseg = 0;
    // (the balanced schedule's ranges span two query tiles, a piece of each, so a block may pay
    // two threshold warm-ups; with the longer lists of small query sets (capmul > 1), whose
    // pieces are many and short, the even segments measured faster: A's rows, 6,250 queries,
    // 2.02 against 1.84 ms, r06bi)
    if (fused && c->train_splits <= 0 && capmul == 1) {
        int occ = 1;
        if (knn_fused_occupancy(d, plan, &occ) != hipSuccess || occ < 1) occ = 1;
        int nb = 1;
        knn_fused_schedule(g, occ * c->num_cus, &nb);
        if (nb <= max_splits(nt, k, cap, smax)) nseg = nb;
    }
    if (nseg == 0) {
        nseg = choose_splits(c, n_qtiles, nt, kelem, rb, k, cap, fused, d, &plan, smax);
        g.g2 = -1;  // segment schedule
    }
    int64_t seg_len = (nt + nseg - 1) / nseg;
    seg_len = (seg_len + 63) / 64 * 64;
    g.train = ftrain; g.nt = nt; g.ld_t = fld_t;
    g.test = ftest; g.nq = nq; g.ld_q = fld_q; g.d = d;
    g.tnorm = c->tnorm.as<float>(); g.tnp = c->tnp.as<float>(); g.qnorm = c->qnorm.as<float>();
    g.tnmax = c->ctrl.as<uint32_t>() + 2;
    g.k = k; g.seg_len = seg_len; g.nseg = nseg;
    g.coef = coef; g.eta = eta;
    g.gthr = c->gthr.as<uint32_t>();
    g.cnt = c->cnt.as<int32_t>(); g.cand = c->cand.as<CandRec>(); g.cap = cap; g.cap_seg = cap / nseg;
    g.qstat = fused ? c->qstat.as<float2>() : nullptr;
    g.tsmax = fused ? c->tsmax.as<float4>() : nullptr;
    // per-XCD scan cursors for the multi-segment schedule (B: filter traffic beyond L2 664 ->
    // 494 GB per launch, time unchanged; with one segment or the balanced schedule they saved
    // nothing: r03s).  KNN_NO_SCAN_CURSOR=1 turns them off (a diagnostic; same results).
    if (fused && !c->no_cursor && g.g2 < 0 && nseg > 1) {
        HIP_OR_FAIL(c, c->cursor.ensure(sizeof(uint32_t) * 8));
        HIP_OR_FAIL(c, hipMemsetAsync(c->cursor.p, 0, sizeof(uint32_t) * 8, st));
        g.cursor = c->cursor.as<uint32_t>();
    }
    // the pieces of a query share their threshold lists, not just their k-th values: the
    // union's k-th smallest U is the bound a single scan would have.  The 32-queries-per-wave
    // shape only -- the small query counts, whose query tiles are cut into many pieces (A's
    // 8-GPU share: 5 pieces, 599 -> 447 kept rows per query, filter 3.38 -> 3.19 ms, r04g; on
    // A and B, 3 and 2 pieces, it measured equal or slower).  KNN_NO_LIST_SHARE=1: off.
    if (shared && nseg > 1) {
        g.lshare_w = knn_fused_list_share_width(plan);
        const int64_t nls = nq * (int64_t)nseg * g.lshare_w;
        HIP_OR_FAIL(c, c->lshare.ensure(sizeof(float) * nls));
        HIP_OR_FAIL(c, knn_launch_fill_u32(c->lshare.as<uint32_t>(), nls, 0x7f800000u, gate, st));  // +inf
        g.lshare = c->lshare.as<float>();
    }
    g.status = c->ctrl.as<int32_t>();
    g.gate = gate;
    // candidate sub-slices per segment: per lane half (32x32 filters), per quarter (k_gemm_fused16)
    const int subs = fused ? knn_fused_subslices(plan) : 2;
    if (fused && g.g2 >= 0 && nseg > 1)  // whole query tiles write only their piece's sub-slices
        HIP_OR_FAIL(c, hipMemsetAsync(c->cnt.p, 0, sizeof(int32_t) * subs * nseg * nq, st));
    stage_begin(c, st, gate ? "gemm_filter_rerun" : "gemm_filter");
    if (fused) HIP_OR_FAIL(c, knn_launch_fused(g, plan, st));
    else HIP_OR_FAIL(c, knn_launch_gemm_filter(g, kelem, rb, st));
    stage_end(c, st);

    RescoreArgs r{};
    r.train = tr->feat; r.labels = tr->labels; r.ld_t = tr->ld;
    r.test = te->feat; r.ld_q = te->ld; r.nq = nq; r.d = d; r.k = k; r.C = C; r.elem = dtype;
    r.cnt = g.cnt; r.cand = g.cand; r.cap = cap;
    r.nseg = subs * nseg; r.cap_seg = g.cap_seg / subs;  // sub-slices: (segment, lane half or quarter)
    r.out = out; r.status = c->ctrl.as<int32_t>();
    r.fb_list = c->fb_list.as<int32_t>(); r.fb_count = c->ctrl.as<int32_t>() + 1;
    r.gate = gate;
    // the fused filter's final thresholds: the selection stages only the candidates that can
    // survive (KNN_RESCORE_ALL=1 stages every candidate: a study switch)
    r.gthr = fused && !c->rescore_all ? g.gthr : nullptr;
    // LDS staging for about twice the expected kept rows -- k (1 + ln(nt / k)) for one scan,
    // +25 % per extra segment (they share thresholds through gthr), measured 238 per query on
    // A and 605 on B -- rounded to 64 by the launcher and capped at the list capacity: a
    // smaller footprint per wave lets more query waves share a CU
    {
        const double expect = k * (1.0 + std::log(std::max((double)nt / k, 1.0))) * (1.0 + 0.25 * (nseg - 1)) + 64.0;
        r.su_cap = c->rescore_su > 0 ? c->rescore_su : (int)std::min<double>(cap, 2.0 * expect);
    }
    stage_begin(c, st, gate ? "rescore_rerun" : "rescore");
    HIP_OR_FAIL(c, knn_launch_rescore(r, st));
    stage_end(c, st);

    if (!gate) {
        c->stats[2] = nseg;
        c->stats[3] = felem;
        c->stats[5] = fused;
        c->stats[9] = fused ? (plan.m16 ? 16 : 32) : 0;
        c->stats[10] = fused ? 32 * plan.qg : 0;
        c->subs = subs;
    } else {
        c->rerun_stats[0] = nseg;
        c->rerun_stats[1] = felem;
        c->rerun_stats[2] = fused;
    }
    return KNN_OK;
}

}  // namespace

extern "C" {

int32_t knn_version(void) { return KNN_AMD_ABI_VERSION; }

knn_status knn_create(knn_ctx** out, const knn_opts* opts) {
    if (!out) return KNN_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return KNN_ENODEV;
    knn_ctx* c = new (std::nothrow) knn_ctx();
    if (!c) return KNN_ENOMEM;
    if (opts) {
        c->device = opts->device;
        c->algo = opts->algo;
        c->train_splits = opts->train_splits;
        c->profile = opts->profile;
        c->cache_train = (opts->flags & KNN_OPT_CACHE_TRAIN) != 0;
        c->cache_train_device = c->cache_train && (opts->flags & KNN_OPT_CACHE_TRAIN_DEVICE) != 0;
    }
    // test hooks and study switches, read here once, never per call
    if (const char* e = getenv("KNN_RESCORE_SU")) c->rescore_su = atoi(e);
    if (const char* e = getenv("KNN_FUSED_QG")) c->fforce.qg = atoi(e);
    if (const char* e = getenv("KNN_FUSED_NBUF")) c->fforce.nbuf = atoi(e);
    c->fforce.heaps = getenv("KNN_FUSED_HEAPS") != nullptr;
    c->fforce.m16 = getenv("KNN_FUSED_MFMA16") != nullptr && std::atoi(getenv("KNN_FUSED_MFMA16")) == 1;
    c->no_lshare = getenv("KNN_NO_LIST_SHARE") != nullptr;
    c->no_cursor = getenv("KNN_NO_SCAN_CURSOR") != nullptr;
    c->rescore_all = getenv("KNN_RESCORE_ALL") != nullptr;
    c->merge_kernel = getenv("KNN_DIRECT_MERGE_KERNEL") != nullptr;
    if (c->device < 0 || c->device >= ndev) { delete c; return KNN_ENODEV; }
    hipDeviceProp_t prop;
    if (hipSetDevice(c->device) != hipSuccess || hipGetDeviceProperties(&prop, c->device) != hipSuccess) {
        delete c;
        return KNN_ENODEV;
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        // kernels are built for gfx950 only
        delete c;
        return KNN_ENODEV;
    }
    c->num_cus = prop.multiProcessorCount;
    // the context's own stream (device calls given no stream) is a BLOCKING stream: ordered after
    // the work the caller issued on the legacy null stream (torch's default stream), as the
    // device entry points promise; the copy stream of the host pipeline stays non-blocking
    if (hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess ||
        hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&c->ctrl_host, 8 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void**)&c->ctrl_host_dev, c->ctrl_host, 0) != hipSuccess ||
        c->ctrl.ensure(4 * sizeof(int32_t)) != hipSuccess) {
        knn_destroy(c);
        return KNN_EHIP;
    }
    for (int i = 0; i < 2; i++)
        if (hipEventCreateWithFlags(&c->ev_up[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_done[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_down[i], hipEventDisableTiming) != hipSuccess) {
            knn_destroy(c);
            return KNN_EHIP;
        }
    // GEMM-path candidate workspace: 12 B x 64 CAPW per query; passes of at most a quarter of
    // the free HBM (KNN_WS_QUERIES / KNN_BATCH_ROWS override, for tests)
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0)
        c->ws_queries = std::max<int64_t>(4096, (int64_t)(free_b / 4) / (12 * 64 * KNN_RESCORE_CAPW + 64));
    if (const char* e = getenv("KNN_WS_QUERIES")) c->ws_queries = std::max<int64_t>(1, atoll(e));
    if (const char* e = getenv("KNN_BATCH_ROWS")) c->batch_rows = std::max<int64_t>(1, atoll(e));
    *out = c;
    return KNN_OK;
}

void knn_destroy(knn_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    for (DBuf* b : {&c->tnorm, &c->tnp, &c->qnorm, &c->gthr, &c->cnt, &c->cand,
                    &c->fb_list, &c->ctrl, &c->scratch, &c->split_t, &c->split_q, &c->pad_t, &c->seg_rec, &c->arrive, &c->tmax, &c->tsmax, &c->qstat, &c->tblk, &c->tctrl, &c->cursor, &c->lshare, &c->h_train, &c->h_labels, &c->h_test, &c->h_pred,
                    &c->h_dist, &c->h_idx})
        b->release();
    for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
    for (int i = 0; i < 2; i++) {
        for (hipEvent_t e : {c->ev_up[i], c->ev_done[i], c->ev_down[i]})
            if (e) (void)hipEventDestroy(e);
        for (DBuf* b : {&c->q_slot[i], &c->pred_slot[i], &c->dist_slot[i], &c->idx_slot[i]}) b->release();
    }
    for (int32_t* p : c->ctrl_slots) (void)hipHostFree(p);
    if (c->ctrl_host) (void)hipHostFree(c->ctrl_host);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    delete c;
}

const char* knn_last_error(const knn_ctx* c) { return c ? c->err.c_str() : "null context"; }

}  // extern "C"

int knn_ctx_device(const knn_ctx* c) { return c->device; }
void* knn_ctx_stream(const knn_ctx* c) { return (void*)c->stream; }
void knn_ctx_stage_begin(knn_ctx* c, void* stream, const char* name);
void knn_ctx_stage_end(knn_ctx* c, void* stream);
knn_status knn_merge_vote_append(knn_ctx* c, int32_t nsrc, int64_t nq, int32_t k, int32_t C, const int32_t* d_rec,
                                 int32_t* d_pred, float* d_dist, int32_t* d_idx, void* hip_stream);

namespace {

// Validation shared by the device entry points.
knn_status validate_call(knn_ctx* c, const knn_dataset* tr, const knn_dataset* te, int32_t k, int32_t C,
                         const QueryOut& out, bool shard) {
    knn_status s;
    if ((s = check_dataset(c, tr, "train", true)) != KNN_OK) return s;
    if ((s = check_dataset(c, te, "test", false)) != KNN_OK) return s;
    if (tr->d != te->d) return fail(c, KNN_EINVAL, "feature count mismatch: train d=%d test d=%d", tr->d, te->d);
    if (tr->dtype != te->dtype) return fail(c, KNN_EINVAL, "train and test dtypes differ");
    if (k < 1 || (!shard && k > tr->n))
        return fail(c, KNN_EINVAL, "k=%d outside [1, n_train=%lld]", k, (long long)tr->n);
    if (k > 1024) return fail(c, KNN_EINVAL, "k=%d exceeds the supported maximum 1024", k);
    if (C < 1 || C > 16384) return fail(c, KNN_EINVAL, "num_classes=%d outside [1, 16384]", C);
    if (tr->n + out.idx_base > 0x7fffffffLL || out.idx_base < 0)
        return fail(c, KNN_EINVAL, "train row indices exceed 2^31-1");
    const int es = elem_size(tr->dtype);
    if (((int64_t)tr->ld * es) % 16 || ((int64_t)te->ld * es) % 16 || (((uintptr_t)tr->feat) & 15) ||
        (((uintptr_t)te->feat) & 15))
        return fail(c, KNN_EINVAL, "device rows must be 16-byte aligned (ld * element size %% 16 == 0)");
    if (te->n > 0 && !shard && !out.pred) return fail(c, KNN_EINVAL, "pred is NULL");
    // the exact scan (KNN_ALGO_DIRECT_SCAN, and every GEMM path's fallback) stages the query
    // row in LDS: bound d by it up front instead of failing at a launch
    if (knn_exact_scan_lds(tr->d, k, C) > 160 * 1024)
        return fail(c, KNN_EINVAL, "d=%d too wide for the exact scan's LDS query row at k=%d, C=%d (d <= ~%d)",
                    tr->d, k, C, (int)((160 * 1024 - knn_exact_scan_lds(0, k, C)) / 4));
    return KNN_OK;
}

// One pass of the pipeline over a query set, enqueued on st with no host synchronisation;
// the status word is copied to ctrl_copy (pinned host, optional) at the end.
knn_status predict_enqueue(knn_ctx* c, const knn_dataset* tr, const knn_dataset* te, int32_t k, int32_t C,
                           const QueryOut& out, hipStream_t st, int algo, int32_t* ctrl_copy) {
    knn_status s;
    HIP_OR_FAIL(c, reset_ctrl(c, st));
    if (is_gemm(algo)) {
        // AUTO on fp32 data runs the rounded filter first; when more than 1/16 of the queries
        // (at least 256) overflow its candidate lists, the call is re-run with the split
        // filter (every output is rewritten).  The decision is made on the device
        // (k_rerun_decide): the split stages are enqueued behind a gate, so a call ends in a
        // single stream synchronisation either way.
        const bool adaptive = c->algo == KNN_ALGO_AUTO && filter_elem(algo, tr->dtype) == ELEM_ROUND;
        if ((s = run_gemm(c, tr, te, k, C, out, st, algo, nullptr)) != KNN_OK) return s;
        if (adaptive) {
            const int64_t limit = std::max<int64_t>(256, te->n / 16);
            HIP_OR_FAIL(c, knn_launch_rerun_decide(c->ctrl.as<int32_t>(), limit, st));
            if ((s = run_gemm(c, tr, te, k, C, out, st, KNN_ALGO_GEMM_SPLIT, c->ctrl.as<int32_t>() + 3)) != KNN_OK)
                return s;
        }
        stage_begin(c, st, "fallback_scan");
        if ((s = run_exact_scan(c, tr, te, k, C, out, st, c->fb_list.as<int32_t>(), c->ctrl.as<int32_t>() + 1)) != KNN_OK)
            return s;
        stage_end(c, st);
    } else if (algo == KNN_ALGO_DIRECT_SCAN) {
        stage_begin(c, st, "exact_scan");
        if ((s = run_exact_scan(c, tr, te, k, C, out, st, nullptr, nullptr)) != KNN_OK) return s;
        stage_end(c, st);
    } else {
        stage_begin(c, st, "direct_tile");
        if ((s = run_direct_tile(c, tr, te, k, C, out, st)) != KNN_OK) return s;
        stage_end(c, st);
    }
    if (ctrl_copy) HIP_OR_FAIL(c, hipMemcpyAsync(ctrl_copy, c->ctrl.p, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    return KNN_OK;
}

// stats of a finished pass (status word in ctrl)
void pass_stats(knn_ctx* c, const int32_t* ctrl, bool gemm) {
    c->stats[1] += ctrl[1];
    if (gemm && ctrl[3]) {
        // the split re-run ran: its segments / operand type describe the results
        c->stats[4] = 1;
        c->stats[2] = c->rerun_stats[0];
        c->stats[3] = c->rerun_stats[1];
        c->stats[5] = c->rerun_stats[2];
    }
}

QueryOut offset_out(const QueryOut& o, int64_t q0) {
    QueryOut r = o;
    if (r.pred) r.pred += q0;
    if (r.dist) r.dist += q0 * r.stride;
    if (r.idx) r.idx += q0 * r.stride;
    if (r.label) r.label += q0 * r.stride;
    return r;
}

knn_dataset offset_rows(const knn_dataset& x, int64_t r0, int64_t n) {
    knn_dataset r = x;
    r.feat = (const unsigned char*)x.feat + (size_t)r0 * (size_t)x.ld * (size_t)elem_size(x.dtype);
    r.n = n;
    return r;
}

void reset_stats(knn_ctx* c) {
    c->stages.clear();
    for (int i = 0; i < 11; i++) c->stats[i] = 0;
    c->stats[3] = -1;
}

// Shared pipeline of knn_predict_device / knn_shard_topk_device: the GEMM path runs the
// queries in passes of at most c->ws_queries (the candidate workspace, 24 KB per query, is
// bounded by a quarter of the free HBM), each ending in one synchronisation.
// shard = true: the train set is one shard of a larger one; k may exceed its rows and
// queries with fewer than k neighbours are not an error (the merge decides).
knn_status predict_core(knn_ctx* c, const knn_dataset* tr, const knn_dataset* te, int32_t k, int32_t C,
                        const QueryOut& out, void* hip_stream, bool shard) {
    knn_status s;
    if ((s = validate_call(c, tr, te, k, C, out, shard)) != KNN_OK) return s;
    HIP_OR_FAIL(c, hipSetDevice(c->device));
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
    reset_stats(c);
    if (te->n == 0) return KNN_OK;
    const int algo = choose_algo(c, tr->n, te->n, tr->d, k, tr->dtype);
    const bool gemm = is_gemm(algo);
    const int64_t pass = gemm ? std::max<int64_t>(1, c->ws_queries) : te->n;
    for (int64_t q0 = 0; q0 < te->n; q0 += pass) {
        const knn_dataset tq = offset_rows(*te, q0, std::min(pass, te->n - q0));
        if ((s = predict_enqueue(c, tr, &tq, k, C, offset_out(out, q0), st, algo, nullptr)) != KNN_OK ||
            (s = finish_call(c, st)) != KNN_OK) {
            if (s != KNN_EINVAL && s != KNN_ERANGE) c->tprep.valid = c->tpad.valid = false;  // a HIP failure: the operands may be partial
            return s;
        }
        pass_stats(c, c->ctrl_host, gemm);
    }
    if (c->profile == 2 && gemm) {
        // diagnostic only: total candidates kept by the filter (last pass)
        std::vector<int32_t> h(std::min(pass, te->n) * c->subs * c->stats[2]);
        if (hipMemcpy(h.data(), c->cnt.p, sizeof(int32_t) * h.size(), hipMemcpyDeviceToHost) == hipSuccess) {
            int64_t tot = 0;
            for (int32_t v : h) tot += v;
            c->stats[0] = tot;
        }
    }
    return KNN_OK;
}

// The train set of a host-buffer call on the device: reused across calls when the context
// caches train uploads (KNN_OPT_CACHE_TRAIN) and the buffer, shape and generation match.
knn_status train_device(knn_ctx* c, const knn_dataset* tr, hipStream_t st, knn_dataset* dtr) {
    const size_t es = (size_t)elem_size(tr->dtype);
    const int per16 = (int)(16 / es);
    const int ldd = (tr->d + per16 - 1) / per16 * per16;  // device rows padded to 16 B
    auto& tc = c->tcache;
    const bool hit = c->cache_train && tc.valid && tc.feat == tr->feat && tc.labels == tr->labels && tc.n == tr->n &&
                     tc.d == tr->d && tc.ld == tr->ld && tc.dtype == tr->dtype && tc.gen == c->generation;
    if (!hit) {
        tc.valid = false;
        c->train_epoch++;  // the uploaded copy changes: the train-side filter operands of it are stale
        HIP_OR_FAIL(c, c->h_train.ensure(es * (size_t)ldd * tr->n));
        HIP_OR_FAIL(c, c->h_labels.ensure(sizeof(int32_t) * tr->n));
        HIP_OR_FAIL(c, hipMemcpy2DAsync(c->h_train.p, es * ldd, tr->feat, es * tr->ld, es * tr->d, tr->n,
                                        hipMemcpyHostToDevice, st));
        HIP_OR_FAIL(c, hipMemcpyAsync(c->h_labels.p, tr->labels, sizeof(int32_t) * tr->n, hipMemcpyHostToDevice, st));
        c->stats[6] += (int64_t)(es * tr->d * tr->n + sizeof(int32_t) * tr->n);
        if (c->cache_train) {
            tc = {tr->feat, tr->labels, tr->n, tr->d, tr->ld, tr->dtype, ldd, c->generation, true};
        }
    }
    *dtr = knn_dataset{c->h_train.p, c->h_labels.as<int32_t>(), tr->n, tr->d, ldd, tr->dtype};
    return KNN_OK;
}

}  // namespace

extern "C" {

knn_status knn_predict_device(knn_ctx* c, const knn_dataset* tr, const knn_dataset* te, int32_t k,
                              int32_t C, int32_t* pred, float* dist, int32_t* idx, void* hip_stream) {
    if (!c) return KNN_EINVAL;
    c->err.clear();
    QueryOut out{pred, dist, idx, nullptr, k, 0};
    return predict_core(c, tr, te, k, C, out, hip_stream, false);
}

knn_status knn_shard_topk_device(knn_ctx* c, const knn_dataset* shard, const knn_dataset* te, int32_t k,
                                 int32_t C, int64_t idx_base, int32_t* d_rec, void* hip_stream) {
    if (!c) return KNN_EINVAL;
    c->err.clear();
    if (te && te->n > 0 && !d_rec) return fail(c, KNN_EINVAL, "d_rec is NULL");
    QueryOut out{nullptr, reinterpret_cast<float*>(d_rec), d_rec ? d_rec + k : nullptr,
                 d_rec ? d_rec + 2 * (int64_t)k : nullptr, 3 * (int64_t)k, idx_base};
    return predict_core(c, shard, te, k, C, out, hip_stream, true);
}

knn_status knn_merge_vote_device(knn_ctx* c, int32_t nsrc, int64_t nq, int32_t k, int32_t C,
                                 const int32_t* d_rec, int32_t* d_pred, float* d_dist, int32_t* d_idx,
                                 void* hip_stream) {
    if (!c) return KNN_EINVAL;
    c->err.clear();
    c->stages.clear();
    return knn_merge_vote_append(c, nsrc, nq, k, C, d_rec, d_pred, d_dist, d_idx, hip_stream);
}

}  // extern "C"

// the merge, with its stage appended to the context's profile (knn_predict_train_sharded
// keeps the shard's filter / rescore stages and the exchange beside it)
knn_status knn_merge_vote_append(knn_ctx* c, int32_t nsrc, int64_t nq, int32_t k, int32_t C, const int32_t* d_rec,
                                 int32_t* d_pred, float* d_dist, int32_t* d_idx, void* hip_stream) {
    if (nsrc < 1 || nq < 0 || k < 1 || k > 1024 || C < 1 || C > 16384)
        return fail(c, KNN_EINVAL, "merge: bad nsrc=%d nq=%lld k=%d C=%d", nsrc, (long long)nq, k, C);
    if (nq > 0 && (!d_rec || !d_pred)) return fail(c, KNN_EINVAL, "merge: d_rec / d_pred is NULL");
    HIP_OR_FAIL(c, hipSetDevice(c->device));
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
    if (nq == 0) return KNN_OK;
    HIP_OR_FAIL(c, reset_ctrl(c, st));
    MergeArgs m{};
    m.rec = d_rec; m.nsrc = nsrc; m.nq = nq; m.k = k; m.C = C;
    m.out = QueryOut{d_pred, d_dist, d_idx, nullptr, k, 0};
    m.status = c->ctrl.as<int32_t>();
    stage_begin(c, st, "merge_vote");
    HIP_OR_FAIL(c, knn_launch_merge(m, st));
    stage_end(c, st);
    return finish_call(c, st);
}

extern "C" {

knn_status knn_predict(knn_ctx* c, const knn_dataset* tr, const knn_dataset* te, int32_t k, int32_t C,
                       int64_t q_begin, int64_t q_end, int32_t* out_pred, float* out_dist,
                       int32_t* out_idx) {
    if (!c) return KNN_EINVAL;
    c->err.clear();
    knn_status s;
    if ((s = check_dataset(c, tr, "train", true)) != KNN_OK) return s;
    if ((s = check_dataset(c, te, "test", false)) != KNN_OK) return s;
    if (q_begin < 0 || q_end < q_begin || q_end > te->n)
        return fail(c, KNN_EINVAL, "query range [%lld, %lld) outside [0, %lld)", (long long)q_begin,
                    (long long)q_end, (long long)te->n);
    if (tr->d != te->d) return fail(c, KNN_EINVAL, "feature count mismatch: train d=%d test d=%d", tr->d, te->d);
    if (tr->dtype != te->dtype) return fail(c, KNN_EINVAL, "train and test dtypes differ");
    if (k < 1 || k > tr->n) return fail(c, KNN_EINVAL, "k=%d outside [1, n_train=%lld]", k, (long long)tr->n);
    const int64_t nq = q_end - q_begin;
    reset_stats(c);
    if (nq == 0) return KNN_OK;
    if (!out_pred) return fail(c, KNN_EINVAL, "out_pred is NULL");
    HIP_OR_FAIL(c, hipSetDevice(c->device));
    hipStream_t st = c->stream, cs = c->cstream;
    const int d = tr->d;
    const size_t es = (size_t)elem_size(tr->dtype);
    const int ldd = (int)((d + (int)(16 / es) - 1) / (int)(16 / es) * (int)(16 / es));  // device rows padded to 16 B
    const int algo = choose_algo(c, tr->n, nq, d, k, tr->dtype);
    const bool gemm = is_gemm(algo);
    // queries stream through two device slots: batch b+1 uploads (copy stream) while batch b
    // computes, and batch b's outputs download while b+1 computes
    int64_t B = std::min<int64_t>(nq, c->batch_rows);
    if (gemm) B = std::min<int64_t>(B, c->ws_queries);
    const int64_t nb = (nq + B - 1) / B;
    {
        // the device call's checks on the shapes it will see, before anything is enqueued: no
        // early return may leave a copy to or from the caller's buffers in flight
        const knn_dataset vtr{(const void*)(uintptr_t)256, tr->labels, tr->n, d, ldd, tr->dtype};
        const knn_dataset vq{(const void*)(uintptr_t)256, nullptr, B, d, ldd, te->dtype};
        const QueryOut vo{out_pred, out_dist, out_idx, nullptr, k, 0};
        if ((s = validate_call(c, &vtr, &vq, k, C, vo, false)) != KNN_OK) return s;
    }
    // from here on every error drains both streams (no DMA outlives the call) and drops the
    // train cache entry (its upload may not have run)
    auto abort_call = [&](knn_status e) {
        (void)hipStreamSynchronize(cs);
        (void)hipStreamSynchronize(st);
        c->tcache.valid = false;
        c->tprep.valid = c->tpad.valid = false;
        return e;
    };
    knn_dataset dtr;
    if ((s = train_device(c, tr, st, &dtr)) != KNN_OK) return abort_call(s);
    for (int i = 0; i < 2 && i < nb; i++) {
        HIP_OR_ABORT(c->q_slot[i].ensure(es * (size_t)ldd * B));
        HIP_OR_ABORT(c->pred_slot[i].ensure(sizeof(int32_t) * B));
        if (out_dist) HIP_OR_ABORT(c->dist_slot[i].ensure(sizeof(float) * B * k));
        if (out_idx) HIP_OR_ABORT(c->idx_slot[i].ensure(sizeof(int32_t) * B * k));
    }
    if (nb == 1) {
        // one batch (a call of config L's size): one stream and no events -- the upload, the pass,
        // k_finish's status hand-off (finish_call: the spin on its sequence word), then the
        // downloads.  The pipelined form below pays three cross-stream event waits and a status
        // copy per batch, which only pay off when batches overlap.
        const unsigned char* src = (const unsigned char*)te->feat + es * (size_t)q_begin * (size_t)te->ld;
        HIP_OR_ABORT(hipMemcpy2DAsync(c->q_slot[0].p, es * ldd, src, es * te->ld, es * d, nq, hipMemcpyHostToDevice, st));
        c->stats[7] += (int64_t)(es * d * nq);
        const knn_dataset dq{c->q_slot[0].p, nullptr, nq, d, ldd, te->dtype};
        const QueryOut o{c->pred_slot[0].as<int32_t>(), out_dist ? c->dist_slot[0].as<float>() : nullptr,
                         out_idx ? c->idx_slot[0].as<int32_t>() : nullptr, nullptr, k, 0};
        if ((s = predict_enqueue(c, &dtr, &dq, k, C, o, st, algo, nullptr)) != KNN_OK) return abort_call(s);
        if ((s = finish_call(c, st)) != KNN_OK) {
            if (s != KNN_EINVAL && s != KNN_ERANGE) return abort_call(s);
            return s;  // (a status error: every kernel of the call has completed)
        }
        // (synchronous copies on the null stream: ordered after the context's blocking stream)
        HIP_OR_ABORT(hipMemcpy(out_pred, c->pred_slot[0].p, sizeof(int32_t) * nq, hipMemcpyDeviceToHost));
        if (out_dist)
            HIP_OR_ABORT(hipMemcpy(out_dist, c->dist_slot[0].p, sizeof(float) * nq * k, hipMemcpyDeviceToHost));
        if (out_idx)
            HIP_OR_ABORT(hipMemcpy(out_idx, c->idx_slot[0].p, sizeof(int32_t) * nq * k, hipMemcpyDeviceToHost));
        pass_stats(c, c->ctrl_host, gemm);
        return KNN_OK;
    }
    while ((int64_t)c->ctrl_slots.size() < nb) {
        int32_t* p = nullptr;
        HIP_OR_ABORT(hipHostMalloc((void**)&p, 4 * sizeof(int32_t), hipHostMallocDefault));
        c->ctrl_slots.push_back(p);
    }
    auto rows = [&](int64_t b) { return std::min(B, nq - b * B); };
    auto upload = [&](int64_t b) -> knn_status {
        const int sl = (int)(b & 1);
        const unsigned char* src = (const unsigned char*)te->feat + es * (size_t)(q_begin + b * B) * (size_t)te->ld;
        HIP_OR_ABORT(hipMemcpy2DAsync(c->q_slot[sl].p, es * ldd, src, es * te->ld, es * d, rows(b),
                                        hipMemcpyHostToDevice, cs));
        HIP_OR_ABORT(hipEventRecord(c->ev_up[sl], cs));
        c->stats[7] += (int64_t)(es * d * rows(b));
        return KNN_OK;
    };
    if ((s = upload(0)) != KNN_OK) return abort_call(s);
    for (int64_t b = 0; b < nb; b++) {
        const int sl = (int)(b & 1);
        HIP_OR_ABORT(hipStreamWaitEvent(st, c->ev_up[sl], 0));
        if (b >= 2) HIP_OR_ABORT(hipStreamWaitEvent(st, c->ev_down[sl], 0));  // output slot downloaded
        const knn_dataset dq{c->q_slot[sl].p, nullptr, rows(b), d, ldd, te->dtype};
        const QueryOut o{c->pred_slot[sl].as<int32_t>(), out_dist ? c->dist_slot[sl].as<float>() : nullptr,
                         out_idx ? c->idx_slot[sl].as<int32_t>() : nullptr, nullptr, k, 0};
        if ((s = predict_enqueue(c, &dtr, &dq, k, C, o, st, algo, c->ctrl_slots[b])) != KNN_OK) return abort_call(s);
        HIP_OR_ABORT(hipEventRecord(c->ev_done[sl], st));
        if (b + 1 < nb) {
            if (b + 1 >= 2) HIP_OR_ABORT(hipStreamWaitEvent(cs, c->ev_done[(b + 1) & 1], 0));  // slot free
            if ((s = upload(b + 1)) != KNN_OK) return abort_call(s);
        }
        HIP_OR_ABORT(hipStreamWaitEvent(cs, c->ev_done[sl], 0));
        const int64_t q0 = b * B;
        HIP_OR_ABORT(hipMemcpyAsync(out_pred + q0, c->pred_slot[sl].p, sizeof(int32_t) * rows(b),
                                      hipMemcpyDeviceToHost, cs));
        if (out_dist)
            HIP_OR_ABORT(hipMemcpyAsync(out_dist + q0 * k, c->dist_slot[sl].p, sizeof(float) * rows(b) * k,
                                          hipMemcpyDeviceToHost, cs));
        if (out_idx)
            HIP_OR_ABORT(hipMemcpyAsync(out_idx + q0 * k, c->idx_slot[sl].p, sizeof(int32_t) * rows(b) * k,
                                          hipMemcpyDeviceToHost, cs));
        HIP_OR_ABORT(hipEventRecord(c->ev_down[sl], cs));
    }
    HIP_OR_ABORT(hipStreamSynchronize(cs));
    HIP_OR_ABORT(hipStreamSynchronize(st));
    collect_stages(c);
    for (int64_t b = 0; b < nb; b++) {
        if ((s = check_status(c, c->ctrl_slots[b])) != KNN_OK) return s;
        pass_stats(c, c->ctrl_slots[b], gemm);
    }
    return KNN_OK;
}

knn_status knn_set_generation(knn_ctx* c, uint64_t generation) {
    if (!c) return KNN_EINVAL;
    c->generation = generation;
    return KNN_OK;
}

knn_status knn_alloc_pinned(size_t bytes, void** out) {
    if (!out) return KNN_EINVAL;
    *out = nullptr;
    if (bytes == 0) return KNN_OK;
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return KNN_ENOMEM;
    }
    return KNN_OK;
}

void knn_free_pinned(void* p) {
    if (p) (void)hipHostFree(p);
}

int32_t knn_stage_times(const knn_ctx* c, const char** names, float* ms, int32_t n) {
    if (!c) return 0;
    int32_t m = (int32_t)std::min<size_t>((size_t)std::max(n, 0), c->stage_ms.size());
    for (int32_t i = 0; i < m; i++) {
        if (names) names[i] = c->stage_names[i];
        if (ms) ms[i] = c->stage_ms[i];
    }
    return m;
}

int32_t knn_last_stats(const knn_ctx* c, int64_t* out, int32_t n) {
    if (!c || !out) return 0;
    int32_t m = std::min(n, 11);
    for (int32_t i = 0; i < m; i++) out[i] = c->stats[i];
    return m;
}

knn_status knn_generate(knn_ctx* c, void* d_feat, int32_t* d_labels, int64_t row0, int64_t n, int32_t d,
                        int32_t ld, int32_t dtype, int32_t kind, uint64_t seed, uint32_t stream,
                        int32_t C, void* hip_stream) {
    if (!c) return KNN_EINVAL;
    if (n < 0 || d <= 0 || ld < d || (d_labels && C < 1) || (n > 0 && !d_feat) || kind < 0 || kind > 3 ||
        (dtype != KNN_F32 && dtype != KNN_BF16))
        return fail(c, KNN_EINVAL, "knn_generate: bad arguments");
    if (dtype == KNN_BF16 && kind != 1 && kind != 3)
        return fail(c, KNN_EINVAL, "bf16 output needs kind 1 or 3 (bf16-exact values)");
    if (kind >= 2 && C < 1) return fail(c, KNN_EINVAL, "clustered kinds need num_classes >= 1");
    HIP_OR_FAIL(c, hipSetDevice(c->device));
    GenerateArgs a{d_feat, d_labels, row0, n, d, ld, dtype == KNN_BF16, kind, seed, stream, C};
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
    HIP_OR_FAIL(c, knn_launch_generate(a, st));
    HIP_OR_FAIL(c, hipStreamSynchronize(st));
    return KNN_OK;
}

knn_status knn_mfma_probe_bf16(knn_ctx* c, const uint16_t* d_a, const uint16_t* d_b, int32_t K, float* d_out,
                               void* hip_stream) {
    if (!c) return KNN_EINVAL;
    c->err.clear();
    if (K <= 0 || K % 16 || !d_a || !d_b || !d_out) return fail(c, KNN_EINVAL, "mfma probe: K must be a positive multiple of 16");
    HIP_OR_FAIL(c, hipSetDevice(c->device));
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
    HIP_OR_FAIL(c, knn_launch_mfma_probe(d_a, d_b, K, d_out, st));
    HIP_OR_FAIL(c, hipStreamSynchronize(st));
    return KNN_OK;
}

knn_status knn_confusion_matrix_device(knn_ctx* c, const int32_t* d_pred, const int32_t* d_labels, int64_t n,
                                       int32_t C, int32_t* d_cm, int64_t* d_correct, void* hip_stream) {
    if (!c) return KNN_EINVAL;
    c->err.clear();
    if (C < 1 || C > 16384 || n < 0 || !d_cm || (n > 0 && (!d_pred || !d_labels)))
        return fail(c, KNN_EINVAL, "confusion: bad arguments (n=%lld, C=%d)", (long long)n, C);
    HIP_OR_FAIL(c, hipSetDevice(c->device));
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
    c->stages.clear();
    HIP_OR_FAIL(c, reset_ctrl(c, st));
    HIP_OR_FAIL(c, hipMemsetAsync(d_cm, 0, sizeof(int32_t) * (size_t)C * (size_t)C, st));
    unsigned long long* corr = reinterpret_cast<unsigned long long*>(d_correct);
    if (!corr) {
        HIP_OR_FAIL(c, c->scratch.ensure(sizeof(unsigned long long)));  // scratch word
        corr = c->scratch.as<unsigned long long>();
    }
    HIP_OR_FAIL(c, hipMemsetAsync(corr, 0, sizeof(unsigned long long), st));
    stage_begin(c, st, "confusion");
    HIP_OR_FAIL(c, knn_launch_confusion(d_pred, d_labels, n, C, d_cm, corr, c->ctrl.as<int32_t>(), st));
    stage_end(c, st);
    knn_status s = finish_call(c, st);
    if (s == KNN_EINVAL) return fail(c, KNN_EINVAL, "a label or prediction is outside [0, num_classes)");
    return s;
}

knn_status knn_confusion_matrix(const int32_t* pred, const int32_t* labels, int64_t n, int32_t C, int32_t* cm) {
    if (!cm || C < 1 || n < 0 || (n > 0 && (!pred || !labels))) return KNN_EINVAL;
    std::memset(cm, 0, sizeof(int32_t) * (size_t)C * (size_t)C);
    for (int64_t i = 0; i < n; i++) {
        int32_t t = labels[i], p = pred[i];
        if (t < 0 || t >= C || p < 0 || p >= C) return KNN_EINVAL;  // the reference writes out of bounds here
        cm[(int64_t)t * C + p]++;
    }
    return KNN_OK;
}

float knn_accuracy(const int32_t* cm, int32_t C, int64_t n) {
    int ok = 0;
    for (int32_t i = 0; i < C; i++) ok += cm[(int64_t)i * C + i];
    return ok / (float)n;
}

}  // extern "C"

void knn_ctx_stage_begin(knn_ctx* c, void* stream, const char* name) { stage_begin(c, (hipStream_t)stream, name); }
void knn_ctx_stage_end(knn_ctx* c, void* stream) { stage_end(c, (hipStream_t)stream); }
