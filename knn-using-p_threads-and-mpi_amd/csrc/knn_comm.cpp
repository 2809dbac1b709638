// knn_comm.cpp -- train-sharded KNN over ranks behind the C ABI: an RCCL
// communicator (one process per GPU, xGMI on one node) and the exchange of per-shard
// neighbour lists.
//
// The reference shards only the test set (mpi.cpp:141-186: MPI_Scatter of [start, end)
// ranges, MPI_Gatherv of int predictions).  Here a rank may own a contiguous shard of the
// TRAIN set instead (config C: 32M rows do not need to be replicated): every rank computes
// its shard's exact top-k for every query (knn_shard_topk_device), one grouped
// ncclSend/ncclRecv all-to-all hands rank b the lists of the queries it owns
// (shard_range(nq, world, b), the reference's split), and k_merge_vote merges them by
// (distance, global index) -- the reference's lower-index tie rule over the whole train
// set -- and votes.
//
// RCCL is loaded with dlopen when the first communicator is created: the library has no
// link-time dependency on it, and a process that already holds an RCCL (PyTorch's, same
// SONAME librccl.so.1) shares that one.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/knn_amd.h"

// context internals (knn_capi.cpp)
int knn_ctx_device(const knn_ctx* c);
void* knn_ctx_stream(const knn_ctx* c);
void knn_ctx_stage_begin(knn_ctx* c, void* stream, const char* name);
void knn_ctx_stage_end(knn_ctx* c, void* stream);
knn_status knn_merge_vote_append(knn_ctx* c, int32_t nsrc, int64_t nq, int32_t k, int32_t C, const int32_t* d_rec,
                                 int32_t* d_pred, float* d_dist, int32_t* d_idx, void* hip_stream);

namespace {

struct Rccl {
    void* h = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclCommCount) comm_count = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string err;
};

Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
            r.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (r.h) break;
        }
        if (!r.h) {
            r.err = std::string("RCCL not found: ") + dlerror();
            return;
        }
#define KNN_RCCL_SYM(field, sym) r.field = reinterpret_cast<decltype(r.field)>(dlsym(r.h, sym))
        KNN_RCCL_SYM(get_unique_id, "ncclGetUniqueId");
        KNN_RCCL_SYM(init_rank, "ncclCommInitRank");
        KNN_RCCL_SYM(destroy, "ncclCommDestroy");
        KNN_RCCL_SYM(abort, "ncclCommAbort");
        KNN_RCCL_SYM(group_start, "ncclGroupStart");
        KNN_RCCL_SYM(group_end, "ncclGroupEnd");
        KNN_RCCL_SYM(send, "ncclSend");
        KNN_RCCL_SYM(recv, "ncclRecv");
        KNN_RCCL_SYM(all_reduce, "ncclAllReduce");
        KNN_RCCL_SYM(comm_count, "ncclCommCount");
        KNN_RCCL_SYM(error_string, "ncclGetErrorString");
#undef KNN_RCCL_SYM
        if (!r.get_unique_id || !r.init_rank || !r.destroy || !r.group_start || !r.group_end || !r.send || !r.recv ||
            !r.all_reduce || !r.comm_count)
            r.err = "RCCL lacks a required symbol";
    });
    return r;
}

bool rccl_ok() {
    Rccl& r = rccl();
    return r.h && r.err.empty();
}

}  // namespace

// int32 elements per RCCL send / recv of the exchange (knn_comm_set_exchange overrides it per
// communicator): 64 Mi = 256 MiB
#ifndef KNN_XCHG_CHUNK
#define KNN_XCHG_CHUNK ((int64_t)64 << 20)
#endif

struct knn_comm {
    ncclComm_t comm = nullptr;
    int32_t nranks = 0, rank = 0, device = 0;
    // exchange workspace: this rank's shard records for all queries, and the lists of its
    // owned queries from every rank
    void* rec = nullptr;
    size_t rec_bytes = 0;
    void* lists = nullptr;
    size_t lists_bytes = 0;
    // the per-call failure vote, allocated at create: flag[0] receives the max-allreduce of
    // flag[1] (= 0, this rank succeeded) or flag[2] (= 1, it failed) -- constants written once,
    // so taking part in the vote needs no copy that could itself fail
    int32_t* flag = nullptr;
    int32_t* flag_host = nullptr;  // pinned copy of the vote's result
    bool broken = false;           // aborted after a failed collective: every later call fails
    // the exchange's message plan (knn_comm_set_exchange): int32 elements per RCCL message, and
    // whether the own block takes the RCCL loop too (else a device copy)
    int64_t chunk = KNN_XCHG_CHUNK;
    bool self_rccl = false;
    std::string err;
};

namespace {

hipError_t grow(void** p, size_t* have, size_t need) {
    if (*p && *have >= need) return hipSuccess;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    hipError_t e = hipMalloc(p, need ? need : 16);
    if (e == hipSuccess) *have = need;
    return e;
}

}  // namespace

extern "C" {

knn_status knn_shard_range(int64_t n, int32_t world, int32_t rank, int64_t* begin, int64_t* end) {
    if (n < 0 || world < 1 || rank < 0 || rank >= world || !begin || !end) return KNN_EINVAL;
    // multi-thread.cpp:154-158 / mpi.cpp:141-170: worker w < world-1 gets [w*(n/world),
    // (w+1)*(n/world)); the last worker also takes the remainder
    const int64_t per = n / world;
    *begin = (int64_t)rank * per;
    *end = *begin + per + (rank == world - 1 ? n % world : 0);
    return KNN_OK;
}

knn_status knn_shard_policy(int64_t n_train, int64_t n_query, int32_t d, int32_t dtype, int32_t world,
                            int64_t hbm_bytes, int32_t* policy) {
    if (n_train < 0 || n_query < 0 || d < 1 || world < 1 || !policy || (dtype != KNN_F32 && dtype != KNN_BF16))
        return KNN_EINVAL;
    // north_star's rule: replicate train (test-sharded, no collective on the data path) while a
    // full copy fits one GPU's HBM with room for the filter's derived operands (bf16 tile blocks:
    // half an fp32 copy; one bf16 copy) and the per-query workspace (candidate lists, 24 KB per
    // query of a pass, bounded separately); else shard train and exchange per-shard top-k lists
    const double esz = dtype == KNN_BF16 ? 2.0 : 4.0;
    const double train_b = (double)n_train * d * esz + (double)n_train * d * 2.0;
    const double budget = 0.5 * (double)(hbm_bytes > 0 ? hbm_bytes : (int64_t)288 << 30);
    *policy = (world > 1 && train_b > budget) ? KNN_SHARD_TRAIN : KNN_SHARD_TEST;
    return KNN_OK;
}

knn_status knn_exchange_layout(int64_t nq, int32_t k, int32_t world, int32_t rank, int64_t* send_off,
                               int64_t* send_cnt, int64_t* recv_off, int64_t* recv_cnt) {
    if (nq < 0 || k < 1 || world < 1 || rank < 0 || rank >= world || !send_off || !send_cnt || !recv_off || !recv_cnt)
        return KNN_EINVAL;
    // records are int32 [nq][3][k]; rank b owns queries shard_range(nq, world, b): it receives
    // from every rank a the rows of its own queries, into lists [a][my_nq][3][k]
    const int64_t row = 3 * (int64_t)k;
    int64_t m0, m1;
    knn_shard_range(nq, world, rank, &m0, &m1);
    for (int32_t b = 0; b < world; b++) {
        int64_t b0, b1;
        knn_shard_range(nq, world, b, &b0, &b1);
        send_off[b] = b0 * row;
        send_cnt[b] = (b1 - b0) * row;
        recv_off[b] = (int64_t)b * (m1 - m0) * row;
        recv_cnt[b] = (m1 - m0) * row;
    }
    return KNN_OK;
}

knn_status knn_comm_unique_id(void* id_out) {
    if (!id_out) return KNN_EINVAL;
    if (!rccl_ok()) return KNN_ENODEV;
    ncclUniqueId id;
    if (rccl().get_unique_id(&id) != ncclSuccess) return KNN_ERCCL;
    std::memcpy(id_out, &id, sizeof(id));
    return KNN_OK;
}

knn_status knn_comm_create(knn_ctx* ctx, const void* id, int32_t nranks, int32_t rank, knn_comm** out) {
    if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return KNN_EINVAL;
    *out = nullptr;
    if (!rccl_ok()) return KNN_ENODEV;
    knn_comm* c = new (std::nothrow) knn_comm();
    if (!c) return KNN_ENOMEM;
    c->nranks = nranks;
    c->rank = rank;
    c->device = knn_ctx_device(ctx);
    if (hipSetDevice(c->device) != hipSuccess) {
        delete c;
        return KNN_EHIP;
    }
    // the failure vote's words exist before any call, so a call never fails to take part in it
    static const int32_t words[3] = {0, 0, 1};
    if (hipMalloc((void**)&c->flag, sizeof(words)) != hipSuccess ||
        hipHostMalloc((void**)&c->flag_host, sizeof(int32_t), hipHostMallocDefault) != hipSuccess) {
        knn_comm_destroy(c);
        return KNN_ENOMEM;
    }
    if (hipMemcpy(c->flag, words, sizeof(words), hipMemcpyHostToDevice) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {  // (landed before any stream of the comm reads it)
        knn_comm_destroy(c);
        return KNN_EHIP;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    if (rccl().init_rank(&c->comm, nranks, uid, rank) != ncclSuccess) {
        c->comm = nullptr;
        knn_comm_destroy(c);
        return KNN_ERCCL;
    }
    *out = c;
    return KNN_OK;
}

knn_status knn_comm_count(const knn_comm* c, int32_t* nranks) {
    if (!c || !nranks || !c->comm) return KNN_EINVAL;
    int n = 0;
    if (rccl().comm_count(c->comm, &n) != ncclSuccess) return KNN_ERCCL;
    *nranks = n;
    return KNN_OK;
}

knn_status knn_comm_broken(const knn_comm* c, int32_t* broken) {
    if (!c || !broken) return KNN_EINVAL;
    *broken = c->broken ? 1 : 0;
    return KNN_OK;
}

knn_status knn_comm_set_exchange(knn_comm* c, int64_t chunk_elems, int32_t self_via_rccl) {
    if (!c || (self_via_rccl != 0 && self_via_rccl != 1)) return KNN_EINVAL;
    c->chunk = chunk_elems > 0 ? chunk_elems : KNN_XCHG_CHUNK;
    c->self_rccl = self_via_rccl == 1;
    return KNN_OK;
}

void knn_comm_destroy(knn_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->comm && rccl_ok()) {
        if (c->broken && rccl().abort) (void)rccl().abort(c->comm);
        else (void)rccl().destroy(c->comm);
    }
    if (c->rec) (void)hipFree(c->rec);
    if (c->lists) (void)hipFree(c->lists);
    if (c->flag) (void)hipFree(c->flag);
    if (c->flag_host) (void)hipHostFree(c->flag_host);
    delete c;
}

knn_status knn_predict_train_sharded(knn_ctx* ctx, knn_comm* comm, const knn_dataset* shard, int64_t idx_base,
                                     const knn_dataset* test, int32_t k, int32_t num_classes, int32_t* d_pred,
                                     float* d_dist, int32_t* d_idx, void* hip_stream) {
    // arguments every rank passes alike (collective contract): a bad one fails on every rank
    // before any collective
    if (!ctx || !comm || !shard || !test) return KNN_EINVAL;
    if (k < 1 || k > 1024 || comm->nranks > 1024) return KNN_EINVAL;
    const int64_t nq = test->n;
    int64_t m0, m1;
    knn_shard_range(nq, comm->nranks, comm->rank, &m0, &m1);
    // an aborted communicator (an earlier collective failed) can reach no peer: fail at once,
    // before paying for a shard pass (knn_comm_broken lets the caller tear every rank down)
    if (comm->broken) return KNN_ERCCL;
    if (hipSetDevice(comm->device) != hipSuccess) return KNN_EHIP;
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : (hipStream_t)knn_ctx_stream(ctx);
    const size_t row = 3 * (size_t)k * sizeof(int32_t);
    // 1. this rank's shard: exact top-k of every query, records with global indices.  A
    //    failure here is local (memory, this rank's arguments): it is not returned yet
    knn_status s = KNN_OK;
    if (m1 > m0 && !d_pred) s = KNN_EINVAL;
    if (s == KNN_OK && (grow(&comm->rec, &comm->rec_bytes, row * (size_t)std::max<int64_t>(nq, 1)) != hipSuccess ||
                        grow(&comm->lists, &comm->lists_bytes,
                             row * (size_t)std::max<int64_t>(m1 - m0, 1) * comm->nranks) != hipSuccess))
        s = KNN_ENOMEM;
    if (s == KNN_OK) s = knn_shard_topk_device(ctx, shard, test, k, num_classes, idx_base, (int32_t*)comm->rec, st);
    // 2. every rank votes on whether all shards succeeded (a max-allreduce of one word), so a
    //    rank that failed locally still meets its peers here and all of them return instead of
    //    one leaving the others blocked inside the exchange.  The vote reads a preset device
    //    word (flag[1] or flag[2]): no copy precedes it.  What the vote cannot cover is a
    //    failure of the collective itself (e.g. a sticky device fault from step 1 makes RCCL's
    //    own launch fail): then the communicator is aborted (ncclCommAbort), this rank returns
    //    KNN_ERCCL, and the communicator fails every later call; peers already inside the
    //    all-reduce are released only by their own RCCL timeout (NCCL_COMM_BLOCKING /
    //    the caller's watchdog), since no signal reaches them from a faulted device.
    Rccl& r = rccl();
    auto give_up = [&]() {
        if (!comm->broken && r.abort) (void)r.abort(comm->comm);
        comm->broken = true;
        return KNN_ERCCL;
    };
    const int32_t* vote_src = comm->flag + (s == KNN_OK ? 1 : 2);
    if (r.all_reduce(vote_src, comm->flag, 1, ncclInt32, ncclMax, comm->comm, st) != ncclSuccess) return give_up();
    if (hipMemcpyAsync(comm->flag_host, comm->flag, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return give_up();
    if (s != KNN_OK) return s;
    if (*comm->flag_host != 0) return KNN_ERCCL;  // a peer's shard failed
    // 3. all-to-all of the records: rank b receives the rows of its own queries from everyone
    //    (a failure inside the group still closes it, then aborts: peers must not wait on a
    //    half-posted exchange)
    int64_t so[1024], sc[1024], ro[1024], rc[1024];
    knn_exchange_layout(nq, k, comm->nranks, comm->rank, so, sc, ro, rc);
    knn_ctx_stage_begin(ctx, st, "exchange");
    // this rank's own block is a device copy (unless comm->self_rccl); the other blocks go
    // through one group of RCCL sends / receives, each of at most comm->chunk elements.
    // (Round 5: a one-rank communicator's grouped self send/recv of config C1's 1.2 GB of records
    // delivered only its first half -- the queries past ~500k got wrong neighbour lists, r05i --
    // so no transfer relies on a single multi-GB RCCL message; DESIGN.md "Multi-GPU" has what
    // round 6 measured of that failure.)
    const int64_t chunk = comm->chunk;
    const bool self_copy = !comm->self_rccl;
    if (self_copy && sc[comm->rank] > 0 &&
        hipMemcpyAsync((int32_t*)comm->lists + ro[comm->rank], (const int32_t*)comm->rec + so[comm->rank],
                       sizeof(int32_t) * (size_t)sc[comm->rank], hipMemcpyDeviceToDevice, st) != hipSuccess)
        return give_up();  // (every rank takes this branch alike; a failure here is local -- see give_up)
    if (comm->nranks > 1 || !self_copy) {
        if (r.group_start() != ncclSuccess) return give_up();
        bool ok = true;
        for (int32_t b = 0; b < comm->nranks && ok; b++) {
            if (b == comm->rank && self_copy) continue;
            for (int64_t o = 0; ok && o < sc[b]; o += chunk)
                ok = r.send((const int32_t*)comm->rec + so[b] + o, (size_t)std::min<int64_t>(chunk, sc[b] - o),
                            ncclInt32, b, comm->comm, st) == ncclSuccess;
            for (int64_t o = 0; ok && o < rc[b]; o += chunk)
                ok = r.recv((int32_t*)comm->lists + ro[b] + o, (size_t)std::min<int64_t>(chunk, rc[b] - o),
                            ncclInt32, b, comm->comm, st) == ncclSuccess;
        }
        if (r.group_end() != ncclSuccess || !ok) return give_up();
    }
    knn_ctx_stage_end(ctx, st);
    // 4. merge + vote of the owned queries (ordered by distance, then global index); the
    //    shard's stage times stay in the context's profile beside the exchange and the merge
    if (m1 == m0) return hipStreamSynchronize(st) == hipSuccess ? KNN_OK : KNN_EHIP;
    return knn_merge_vote_append(ctx, comm->nranks, m1 - m0, k, num_classes, (const int32_t*)comm->lists, d_pred,
                                 d_dist, d_idx, st);
}

}  // extern "C"
