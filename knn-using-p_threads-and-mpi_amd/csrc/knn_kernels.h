// knn_kernels.h -- kernel argument blocks and host launchers (internal to libknn_amd).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// device status word bits (one int32 per predict call)
#define KNN_STATUS_TOO_FEW 1       // a query has fewer than k finite distances
#define KNN_STATUS_BAD_LABEL 2     // a neighbour's label is outside [0, C)
#define KNN_STATUS_GEMM_UNSAFE 4   // a row norm is too large for the GEMM certificate
#define KNN_STATUS_UNSORTED 8      // k_merge_vote: a source list read was not ascending by (dist, idx)

// candidate-list capacity per query on the GEMM path (entries = 64 * CAPW)
#define KNN_RESCORE_CAPW 32

// feature element types (knn_dtype): rows are fp32 or bf16 bits; every distance is the
// reference's fp32 direct form on the (exactly) widened values
enum { ELEM_F32 = 0, ELEM_BF16 = 1 };
// filter-only operand type: fp32 rows split into bf16 [hi(d) | lo(d)] (k_split_rows), so
// q.t ~ hi.hi + hi.lo + lo.hi runs on the bf16 MFMA with an fp32-grade error bound
enum { ELEM_SPLIT = 2 };
// filter-only operand type: fp32 rows rounded to bf16 (k_round_rows, d elements per row);
// the filter runs the bf16 kernel on them under a certificate widened by the rounding
enum { ELEM_ROUND = 3 };

// Where a finished query's neighbours go.  pred may be NULL (train-shard mode: no vote);
// dist/idx/label may be NULL; entry e of query q is at [q * stride + e]; idx is reported
// as idx_base + local train row (train shards carry their global offset).
struct QueryOut {
    int32_t* pred; float* dist; int32_t* idx; int32_t* label;
    int64_t stride; int64_t idx_base;
};

struct ExactScanArgs {
    const void* train; const int32_t* labels; int64_t nt; int ld_t;
    const void* test; int ld_q; int64_t nq;
    int d; int k; int C; int elem;
    const int32_t* qlist; const int32_t* qcount;  // optional query list (device count)
    QueryOut out; int32_t* status;
    int q_lds_bytes;                              // set by the launcher
};

// one kept candidate of the GEMM filters: its train row and certified bounds L <= D <= U
// (one 12-byte store per kept row)
struct CandRec { int32_t idx; float L; float U; };

struct GemmFilterArgs {
    const void* train; int64_t nt; int ld_t;      // ld in elements
    const void* test; int64_t nq; int ld_q; int d;
    const float* tnorm; const float* tnp; const float* qnorm;  // tnorm/tnp padded with +inf to nt+64
    const uint32_t* tnmax;  // ordered bits of max tnorm
    int k; int64_t seg_len; int nseg; int n_qtiles;
    float coef; float eta;
    uint32_t* gthr;
    int32_t* cnt;  // [nseg][nq] kept rows per (segment, query)
    CandRec* cand; int cap; int cap_seg;  // [nq][cap] candidate records
    const float2* qstat;  // fused filter, per query: {|q|, |q - rq|} upper bounds (rq: the operand / -2)
    // fused filter schedule (knn_fused_schedule): p1_blocks whole query tiles, then g2 blocks
    // over the remaining w2 (query tile, 64-row unit) pairs; tiles64 units per query tile
    int p1_blocks; int g2; int64_t w2; int64_t tiles64;
    uint32_t* cursor;       // fused filter, optional: per XCD, the 64-row unit its blocks scan now
    // fused filter, register-list shapes with nseg > 1 (optional): each piece's threshold list
    // [nq][nseg][lshare_w] (U values, +inf where empty), shared between a query's pieces
    float* lshare; int lshare_w;
    // fused filter: the maxima over all 64-row tiles of the tile statistics {max tn, max |t - rt|,
    // max |rt|, 0} (k_tile_stat_max): the fast test's tile term, one per query group and piece
    const float4* tsmax;
    const int32_t* status;  // the call's status word: a set GEMM_UNSAFE bit skips the filter
    const int32_t* gate;    // optional: the filter runs only when *gate != 0 (AUTO's re-run)
};

struct RescoreArgs {
    const void* train; const int32_t* labels; int ld_t;
    const void* test; int ld_q; int64_t nq; int d; int k; int C; int elem;
    const int32_t* cnt; const CandRec* cand; int cap;
    int nseg; int cap_seg;
    QueryOut out; int32_t* status;
    int32_t* fb_list; int32_t* fb_count;
    const int32_t* gate;  // optional: runs only when *gate != 0 (AUTO's re-run)
    int su_cap;           // candidates staged in LDS per query (host: ~3x the expected count)
    // optional (the fused filter): per query, an upper bound on the k-th smallest U of its
    // candidates (ordered float bits, the filter's final thresholds): only candidates with
    // L <= it can survive, so the selection stages those alone
    const uint32_t* gthr;
    int q_lds_bytes; int c_lds_bytes; int wave_lds_bytes;  // set by the launcher
};

// Merge of per-shard neighbour lists.  rec: [nsrc][nq][3][k] int32 records (k dist bits,
// k global indices (-1 = none), k labels), each list ascending by (dist, idx).
// labels != NULL: the sources are segments of ONE train set (k_direct_tile): indices are
// its local rows, the vote and out.label read labels[idx] (finish_query).
struct MergeArgs {
    const int32_t* rec; int nsrc; int64_t nq; int k; int C;
    QueryOut out; int32_t* status;
    const int32_t* labels;
};

// class counts up to this many live in a per-wave LDS table; above it the vote runs
// table-free (vote_ballot), so every path accepts any num_classes
#define KNN_VOTE_LDS_MAX_C 1024
// per-wave LDS words of k_merge_vote: class counts, or the k winners' labels + a counter
__host__ __device__ inline int merge_wave_words(int C, int k) {
    return C <= KNN_VOTE_LDS_MAX_C ? ((C + 3) & ~3) : ((k + 1 + 3) & ~3);
}

// k_direct_tile: DT_NW waves per block, 64 train rows per tile, rows staged in chunks of
// dc <= DT_MAX_DC dims (DT_MAXP 16-B staging registers per thread)
#define DT_NW 8
#define DT_MAX_DC 128
#define DT_MAXP (64 * (DT_MAX_DC / 4) / (64 * DT_NW))
struct DirectTileArgs {
    const void* train; const int32_t* labels; int64_t nt; int ld_t;
    const void* test; int ld_q; int64_t nq;
    int d; int k; int C; int elem;
    int64_t seg_len; int nseg; int n_qblocks;
    int dc; int stride;        // dims per staged chunk (multiple of 4), LDS row stride (floats)
    int vote_lds;              // per-wave LDS class counts (C <= KNN_VOTE_LDS_MAX_C)
    QueryOut out; int32_t* status;
    int32_t* rec;              // nseg > 1: segment records [nseg][nq][3][k] (local rows)
    // k_direct_rows with nseg > 1 (optional): per query group, the segments that finished
    // (zero between calls); the last wave of a group merges every segment's records and votes
    // in the same launch (no k_merge_vote pass)
    int32_t* arrive;
};
// queries per k_direct_tile block for k (8 * QW, QW = max(1, 8 / list registers))
int knn_direct_tile_qb(int k);
// launch geometry: LDS bytes per block and blocks per CU at that LDS
size_t knn_direct_tile_lds(int d, int C);
hipError_t knn_direct_tile_occupancy(int k, int elem, int d, int C, int* blocks_per_cu);
// work units of the direct form for (k, d): queries per unit and units resident per CU --
// k_direct_tile: a block of 8 waves; k_direct_rows (d <= 16, k <= 16): one wave
hipError_t knn_direct_units(int k, int elem, int d, int C, int* queries_per_unit, int* units_per_cu);
// fills dc / stride / vote_lds / n_qblocks from d, C, nq and launches nseg units per query
// unit (k_direct_tile: blocks; k_direct_rows for d <= 16, k <= 16: waves, four per block)
hipError_t knn_launch_direct_tile(DirectTileArgs a, hipStream_t st);
// whether (k, d) runs k_direct_rows (d <= 16, k <= 16), and its query groups for nq queries
bool knn_direct_rows_shape(int k, int d);
int64_t knn_direct_rows_groups(int64_t nq);

struct GenerateArgs {
    void* out; int32_t* labels; int64_t row0; int64_t n; int d; int ld;
    int bf16_out; int kind; uint64_t seed; uint32_t stream; int C;
};

hipError_t knn_launch_exact_scan(const ExactScanArgs& a, int grid, hipStream_t st);
size_t knn_exact_scan_lds(int d, int k, int C);
// tstat (optional, train rows of the fused filter): per 64-row tile [ceil(n / 64)]
//   {max ||x||^2, max ||x - rx||, max ||rx||, 0}, rx = rn_bf16(x) (upper bounds)
// qstat (optional, query rows of the fused filter): per row {||x||, ||x - rx||} upper bounds,
//   rx = rn_bf16(oscale x) / oscale (the operand the filter multiplies, unscaled)
// gate (optional): the stage runs only when *gate != 0 (device-side control of AUTO's re-run)
hipError_t knn_launch_row_norms(const void* x, int elem, int64_t n, int ld, int d, float* out,
                                int32_t* status, uint32_t* maxo, float* outp, float c1, hipStream_t st,
                                float4* tstat = nullptr, const int32_t* gate = nullptr,
                                float2* qstat = nullptr, float oscale = 1.0f);
// row_bytes = d * element size: 128, 256 or 512
bool knn_gemm_filter_supported(int elem, int row_bytes);
// block shape of the filter for (element type, row bytes, k): waves per block, query
// groups per wave, row groups per tile, min waves per SIMD (launch bounds), tile buffers,
// queries per block, LDS bytes per block
struct FilterPlan {
    int nw, qg, rg, minw, nbuf, bm;
    size_t lds;
    int kr = 0;  // fused: register-list shape (16, 32, 104; 0 = LDS heaps)
    int ls = 0;  // fused: the kernel exchanges threshold lists between a query's pieces
    int m16 = 0;  // fused: the v_mfma_f32_16x16x32_bf16 form of the shape (k_gemm_fused16)
};
FilterPlan knn_gemm_filter_plan(int elem, int row_bytes, int k);
hipError_t knn_launch_gemm_filter(const GemmFilterArgs& a, int elem, int row_bytes, hipStream_t st);
size_t knn_gemm_filter_lds(int elem, int row_bytes, int k);
hipError_t knn_gemm_filter_occupancy(int elem, int row_bytes, int k, int* blocks_per_cu);
// fp32 rows [n][ld] (d % 4 == 0) -> bf16 rows [n][2d]: hi = rn(x), lo = rn(x - hi)
hipError_t knn_launch_split_rows(const float* x, int64_t n, int ld, int d, uint16_t* out, hipStream_t st,
                                 const int32_t* gate = nullptr);
hipError_t knn_launch_round_rows(const float* x, int64_t n, int ld, int d, uint16_t* out, hipStream_t st,
                                 const int32_t* gate = nullptr);
hipError_t knn_launch_fill_u32(uint32_t* p, int64_t n, uint32_t v, const int32_t* gate, hipStream_t st);
// host_mapped[0..n) = ctrl[0..n) (a mapped pinned host buffer), then ctrl[0..n) = 0
hipError_t knn_launch_finish(int32_t* ctrl, int32_t* host_mapped, int n, uint32_t seq, hipStream_t st);
// AUTO's re-run decision on the device: ctrl[3] = !unsafe && ctrl[1] > limit (and ctrl[1] = 0 then)
hipError_t knn_launch_rerun_decide(int32_t* ctrl, int64_t limit, hipStream_t st);
hipError_t knn_launch_rescore(const RescoreArgs& a, hipStream_t st);
// fused-norm filter (knn_fused.hip), d in {64, 128, 256}: train as tile blocks [bn rows rn(t) |
// bn fp32 norms | tile statistics] (k_tn_rows), each accumulator starting from the norms
bool knn_fused_supported(int d);
// Study overrides of the fused plan (the product plan is knn_fused_plan's rule; a context
// snapshots these once, at knn_create, from KNN_FUSED_QG / KNN_FUSED_NBUF / KNN_FUSED_HEAPS so
// the tests can run every shape): qg 1|2 forces the queries per wave, nbuf 4|8|16 the tile
// group, heaps the LDS-heap shape for 32 < k <= 104 at d = 256.  0 / false: the rule.
struct FusedForce {
    int qg = 0;
    int nbuf = 0;
    bool heaps = false;
    bool m16 = false;  // KNN_FUSED_MFMA16=1: the 16x16x32 form of the register-list shapes (k_gemm_fused16)
};
// nw == 0: k too large.  nq, num_cus and max_pieces (the most pieces a query's candidate list
// allows) pick the queries per wave (register-list shapes): 64 on 32-row tiles when the
// 512-query blocks, at most max_pieces per query tile, fill 80 % of a round of CUs, else 32 on
// 64-row tiles (fewer pieces per query tile).  run_gemm computes the plan once per pass and sizes the
// operands, the occupancy, the schedule and the launch from that one plan.
FilterPlan knn_fused_plan(int d, int k, int64_t nq, int num_cus, const FusedForce& force, int max_pieces);
hipError_t knn_fused_occupancy(int d, const FilterPlan& f, int* blocks_per_cu);
// out = component maxima of n tile statistics (the fused filter's a.tsmax)
hipError_t knn_launch_tile_stat_max(const float4* tstat, int64_t n, float4* out, hipStream_t st);
// k_gemm_fused16's kernel for plan f (f.m16; knn_fused16.hip), nullptr if f has no 16x16x32 form
const void* knn_fused16_ptr(int d, const FilterPlan& f);
// candidate sub-slices per segment (piece) of plan f: one per lane half (32x32), per quarter (16x16)
inline int knn_fused_subslices(const FilterPlan& f) { return f.m16 ? 4 : 2; }
// whether plan f's kernel exchanges threshold lists between a query's pieces (a.lshare, lshare_w floats per piece)
int knn_fused_list_share_width(const FilterPlan& f);
// fills a.p1_blocks / g2 / w2 / tiles64 for the balanced schedule over `slots` resident
// blocks; returns the grid, *nseg = the most pieces one query tile gets.  (a.g2 = -1 and
// a.seg_len / nseg instead: the segment schedule, n_qtiles * nseg blocks.)
int knn_fused_schedule(GemmFilterArgs& a, int slots, int* nseg);
// f: the plan run_gemm sized the grid and operands with (knn_fused_plan)
hipError_t knn_launch_fused(const GemmFilterArgs& a, const FilterPlan& f, hipStream_t st);
// (study build KNN_STUDY_AUG64 only, d = 64) x [n_valid][ld] (fp32 or bf16) -> bf16 [n][d + 16]:
// rn(scale * x) | split of norms[r] (or 1 1 1) | 0,
// and (tstat != NULL, train) the 64-row tile statistics in columns d+8..d+10 of rows 32i;
// rows n_valid .. n-1 (train: padding to the 64-row tile grid) never pass the filter
hipError_t knn_launch_aug_rows(const void* x, int elem, int64_t n, int64_t n_valid, int ld, int d, const float* norms,
                               float scale, uint16_t* out, const float4* tstat, hipStream_t st,
                               const int32_t* gate = nullptr);
// knn_fused_row_bytes(d) == 2d: x -> queries [n][d] bf16 rn(scale x) (norms == NULL),
// or train blocks of bn rows [bn][d] bf16 | bn fp32 norms | tstat of the enclosing 64-row tile
hipError_t knn_launch_tn_rows(const void* x, int elem, int64_t n, int64_t n_valid, int ld, int d, const float* norms,
                              float scale, void* out, const float4* tstat, int bn, hipStream_t st,
                              const int32_t* gate = nullptr);
// bytes per operand row of the fused filter's tile image: 2d (2d + 32 in the KNN_STUDY_AUG64 build)
int knn_fused_row_bytes(int d);
hipError_t knn_launch_merge(const MergeArgs& a, hipStream_t st);
hipError_t knn_launch_generate(const GenerateArgs& a, hipStream_t st);
// the bf16 filter's MFMA chain on [32][K] bf16 operands (certificate self-test)
hipError_t knn_launch_mfma_probe(const uint16_t* a, const uint16_t* b, int K, float* out, hipStream_t st);
hipError_t knn_launch_confusion(const int32_t* pred, const int32_t* labels, int64_t n, int C, int32_t* cm,
                                unsigned long long* correct, int32_t* status, hipStream_t st);
