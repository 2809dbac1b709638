"""Throughput bench of the KNN hot path (BASELINE.json metric: distance pairs/s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config A|B|C|C1|L] [--no-cpu-baseline]

One process per GPU (torchrun for N > 1).  Workload A (default, BASELINE configs[2]):
1,000,000 train x 100,000 query rows x 128-d fp32, k = 10, 10 classes, synthetic rows from
the counter-based generator generated directly in HBM.  The path partitions by
query (north_star: test-sharded, train replicated, no data-path collective; the reference's
MPI_Gatherv of predictions, mpi.cpp:186, is not part of the timed region), so on N GPUs the
fixed 100k-query set BASELINE names is split by the reference's rule (rank r owns
shard_range(100k, N, r), multi-thread.cpp:154-158 / mpi.cpp:141-170): strong scaling, the
reference's own fixed-problem speed-up, "scaling": "strong".  --weak (a study option, never the
driver's line) gives every rank 100,000 queries of its own instead (global rows [r*100k,
(r+1)*100k)).  A "step" is one KNN(train, test, k) pass over the resident inputs: norms -> MFMA
filter -> exact rescore/vote -> fallback.  B (configs[3]) is the same split of its fixed 1M
queries over a 4M-row train set.

Config C (BASELINE configs[4]) is train-sharded: 32M bf16 train rows x 1M queries x
256-d, k = 100; rank r owns train rows shard_range(32M, N, r) and every query, computes
the exact per-shard top-k (bf16 MFMA filter + exact fp32 rescore), the lists go through
one all-to-all (RCCL over xGMI) to the rank that owns each query, which merges + votes.
C1 is one rank's share of C on 8 GPUs (4M train rows x 1M queries), runnable on 1 GPU
through the same code path.

Config L (BASELINE configs[1]) is the reference's own large ARFF pair (tests/data,
30,803 train x 1,718 test x 11-d, k = 5) parsed by the boundary's reader, resident in
HBM, classified by the direct-form path (k_exact_scan); its predictions are compared
with the golden file captured from the reference (accuracy bit-match), and the CPU
baseline is the reference's own multi-thread binary (and serial main) on the same files.

Rank 0 prints one JSON line.  roofline: the dominant kernel (k_gemm_fused, the fused-norm
bf16 filter; k_gemm_filter for the fp32 / split operands) timed with
HIP events on its own stream; cpu_baseline: the reference's pthreads KNN (oracle/_ref,
built -O0 as shipped) on a bounded sample, else the C restatement labelled "port".
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CONFIGS = {
    # name: (n_train, n_query (total; per GPU under --weak), d, k, classes, seed, scaling, dtype, sharding)
    "A": (1_000_000, 100_000, 128, 10, 10, 1, "strong", "f32", "test"),
    "B": (4_000_000, 1_000_000, 64, 32, 10, 2, "strong", "f32", "test"),
    "C": (32_000_000, 1_000_000, 256, 100, 10, 3, "strong", "bf16", "train"),
    "C1": (4_000_000, 1_000_000, 256, 100, 10, 3, "strong", "bf16", "train"),
    "L": (30_803, 1_718, 11, 5, 10, 0, "strong", "f32", "arff"),
}
DEFAULT_STEPS = {"A": 200, "B": 10, "C": 2, "C1": 3, "L": 300}  # (L: 0.1 ms calls; 300 average out the clock ramp)
ARFF_L = ("tests/data/large-train.arff", "tests/data/large-test.arff", "tests/golden/pred_large_k5.txt")
METRIC = "distance pairs/sec + queries/sec at 1/2/4/8 GPUs; accuracy bit-match"
MFMA_PEAK_TFLOPS = {  # MI355X_MICROARCH.md, dense
    "f32": 157.3,    # v_mfma_f32_32x32x2_f32
    "bf16": 2500.0,  # v_mfma_f32_32x32x16_bf16 (~2.5 PF dense)
}
# filter operand type (ctx.stats()["filter_operands"]) -> (peak of one algorithmic FLOP,
# MFMA FLOP issued per algorithmic FLOP).  The split filter runs an fp32 dot as three bf16
# MFMA products (hi.hi + hi.lo + lo.hi), so its roof is the bf16 dense peak / 3.
FILTER_ROOF = {"f32": (157.3, 1), "bf16": (2500.0, 1), "bf16x3 split": (2500.0 / 3, 3),
               "bf16 rounded": (2500.0, 1)}
# pmc summary key suffix per filter operand type on fp32 data
PMC_SUFFIX = {"bf16x3 split": "/split", "bf16 rounded": "/bf16r"}


MPIEXEC = os.environ.get("KNN_MPIEXEC", "/opt/conda/bin/mpiexec")


def _ref_exe(name):
    return os.path.join(REPO, "oracle", "_ref", name)


def cpu_baseline(d, k, C, seed, kind=0, nt_cfg=1_000_000):
    """Reference pthreads KNN (multi-thread.cpp:37) on a bounded sample of the workload,
    beside it the same sample through the reference's -O2 build (ref_bench_O2) and the
    reference's MPI path (mpi.cpp:141-186, ref_bench_mpi under mpiexec, as many ranks as
    threads).  Sample: the full train set up to 1M rows x 8 T queries (T
    threads, a multiple of T so the remainder rule does not skew); the MPI leg, whose every
    rank builds its own libarff copy of train (~10 GB per 1M x 128 rows), uses 100k train
    rows x 64 T queries."""
    threads = int(os.environ.get("KNN_BENCH_CPU_THREADS", min(16, os.cpu_count() or 1)))
    nt_s, nq_s = min(nt_cfg, 1_000_000), 8 * threads
    exe = _ref_exe("ref_bench")
    sample = f"{nq_s} queries x {nt_s} train rows (d={d}, k={k}) of the same generator"
    argv = [str(kind), str(seed), str(nt_s), str(nq_s), str(d), str(k), str(C)]
    nt_m, nq_m = 100_000 * 128 // max(d, 128), 64 * threads
    argv_m = [str(kind), str(seed), str(nt_m), str(nq_m), str(d), str(k), str(C)]

    def run(cmd):
        out = subprocess.run(cmd, capture_output=True, text=True, check=True, timeout=900)
        return json.loads(out.stdout.strip().splitlines()[-1])

    if os.path.exists(exe):
        r = run([exe] + argv + [str(threads)])
        rec = {"value": r["pairs_per_s"], "unit": "pairs/s", "cores": threads, "kind": "reference",
               "sample": sample + "; reference multi-thread.cpp KNN built -O0 as shipped",
               "queries_per_s": r["queries_per_s"]}
        if os.path.exists(_ref_exe("ref_bench_O2")):
            r2 = run([_ref_exe("ref_bench_O2")] + argv + [str(threads)])
            rec["O2"] = {"value": r2["pairs_per_s"], "unit": "pairs/s", "cores": threads,
                         "queries_per_s": r2["queries_per_s"],
                         "note": "the same sample through multi-thread.cpp built -O2"}
        if os.path.exists(_ref_exe("ref_bench_mpi")) and os.path.exists(MPIEXEC):
            r3 = run([MPIEXEC, "-n", str(threads), _ref_exe("ref_bench_mpi")] + argv_m)
            rec["mpi"] = {"value": r3["pairs_per_s"], "unit": "pairs/s", "cores": threads,
                          "queries_per_s": r3["queries_per_s"],
                          "note": f"{nq_m} queries x {nt_m} train rows through mpi.cpp's KNN + Scatter/Gatherv, "
                                  f"-O0, MPICH, mpiexec -n {threads} (every rank holds its own train copy)"}
        else:
            rec["mpi"] = "absent"
        return rec
    # fallback: the C restatement (same algorithm, -O2), labelled as a port
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import Oracle
    o = Oracle()
    tr, tl = o.gen(seed, 0, 0, nt_s, d, kind=kind, C=C)
    te, _ = o.gen(seed, 1, 0, nq_s, d, kind=kind, C=C)
    t0 = time.perf_counter()
    o.knn(tr, tl, te, k, C, threads=threads, topk=False)
    dt = time.perf_counter() - t0
    return {"value": nt_s * nq_s / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": sample + "; oracle/knn_oracle.c -O2", "queries_per_s": nq_s / dt, "mpi": "absent"}


def cpu_baseline_arff(k, threads=None):
    """The reference binaries themselves (oracle/_ref, -O0 as shipped) on the large ARFF
    pair: multi-thread.cpp with T threads and serial main.cpp.  They print whole
    milliseconds of KNN() time (parse excluded, multi-thread.cpp:160-199); median of 3."""
    import re
    threads = threads or int(os.environ.get("KNN_BENCH_CPU_THREADS", min(16, os.cpu_count() or 1)))
    tr, te = (os.path.join(REPO, p) for p in ARFF_L[:2])
    exe_mt = os.path.join(REPO, "oracle", "_ref", "multi-thread")
    exe_se = os.path.join(REPO, "oracle", "_ref", "main")
    if not (os.path.exists(exe_mt) and os.path.exists(exe_se)):
        return None

    def run(cmd):
        out = subprocess.run(cmd, capture_output=True, text=True, check=True, timeout=600).stdout
        return int(re.search(r"required (\d+) ms", out).group(1))

    mt = sorted(run([exe_mt, tr, te, str(k), str(threads)]) for _ in range(3))[1]
    se = run([exe_se, tr, te, str(k)])
    pairs = 30_803 * 1_718
    rec = {"value": pairs / (mt * 1e-3), "unit": "pairs/s", "cores": threads, "kind": "reference",
           "sample": f"the whole workload (large ARFF pair, k={k}); reference multi-thread.cpp with "
                     f"{threads} threads, -O0 as shipped, median of 3 (ms resolution)",
           "ms": mt, "serial_main_ms": se, "serial_main_pairs_per_s": pairs / (se * 1e-3)}
    if os.path.exists(_ref_exe("mpi")) and os.path.exists(MPIEXEC):
        mp = sorted(run([MPIEXEC, "-n", str(threads), _ref_exe("mpi"), tr, te, str(k)]) for _ in range(3))[1]
        rec["mpi"] = {"value": pairs / (mp * 1e-3), "unit": "pairs/s", "cores": threads, "ms": mp,
                      "note": f"reference mpi.cpp (-O0, MPICH), mpiexec -n {threads}, median of 3"}
    else:
        rec["mpi"] = "absent"
    return rec


def oracle_bit_match(seed, kind, nt, d, k, C, q_rows, got_pred, threads=None, chunk=1 << 20):
    """The bench run proves its own result (metric: "...; accuracy bit-match"): the
    predictions the timed steps produced for a spread sample of global query rows q_rows
    against the C oracle (oracle/knn_oracle.c, main.cpp:25-85) over the WHOLE train set,
    regenerated on the host from the same counter-based generator in chunks of `chunk` rows:
    each chunk's exact top-k (the oracle's stable insertion), merged by (distance bits,
    global index) -- the reference's lower-index tie rule -- then the vote (smallest label on
    ties).  Runs after the timed region; the oracle is the checker only."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import Oracle
    o = Oracle()
    threads = threads or int(os.environ.get("KNN_BENCH_CPU_THREADS", min(16, os.cpu_count() or 1)))
    t0 = time.perf_counter()
    te = np.concatenate([o.gen(seed, 1, int(q), 1, d, kind=kind, C=C)[0] for q in q_rows])
    nq = len(q_rows)
    best_d = np.zeros((nq, 0), np.uint32)
    best_i = np.zeros((nq, 0), np.int64)
    best_l = np.zeros((nq, 0), np.int32)
    for r0 in range(0, nt, chunk):
        n = min(chunk, nt - r0)
        tr, tl = o.gen(seed, 0, r0, n, d, kind=kind, C=C)
        bad, _, dist, idx = o.knn(tr, tl, te, min(k, n), C, threads=threads)
        ok = idx >= 0
        lab = np.where(ok, tl[np.clip(idx, 0, n - 1)], -1)
        best_d = np.concatenate([best_d, dist.view(np.uint32)], axis=1)
        best_i = np.concatenate([best_i, np.where(ok, idx.astype(np.int64) + r0, -1)], axis=1)
        best_l = np.concatenate([best_l, lab], axis=1)
        keep_d, keep_i, keep_l = [], [], []
        for q in range(nq):
            v = best_i[q] >= 0
            order = np.lexsort((best_i[q][v], best_d[q][v]))[:k]
            keep_d.append(best_d[q][v][order]); keep_i.append(best_i[q][v][order]); keep_l.append(best_l[q][v][order])
        best_d, best_i, best_l = np.stack(keep_d), np.stack(keep_i), np.stack(keep_l)
        del tr, tl
    want = np.array([int(np.argmax(np.bincount(best_l[q], minlength=C))) for q in range(nq)], np.int32)
    got = np.asarray(got_pred, np.int32)
    bad = np.nonzero(got != want)[0]
    return {"predictions_equal_oracle": bool(np.array_equal(got, want)), "queries_checked": int(nq),
            "mismatches": int(len(bad)), "mismatch_rows": [int(q_rows[i]) for i in bad[:8]],
            "query_rows": [int(q) for q in q_rows[:4]] + ["..."],
            "checker": "oracle/knn_oracle.c over the whole train set (host-regenerated, chunked, merged)",
            "check_s": round(time.perf_counter() - t0, 1)}


def bench_arff(args, knn, torch, local):
    """configs[1]: the reference's large ARFF pair, k = 5, inputs resident in HBM."""
    nt, nq, d, k, C = CONFIGS["L"][:5]
    tf, tl, _ = knn.read_arff(os.path.join(REPO, ARFF_L[0]))
    qf, ql, _ = knn.read_arff(os.path.join(REPO, ARFF_L[1]))
    assert tf.shape == (nt, d) and qf.shape == (nq, d), (tf.shape, qf.shape)
    C = int(tl.max()) + 1  # train->num_classes() (main.cpp:35)
    dev = torch.device("cuda", local)
    # the timed calls run without events (each timed event pair costs a call ~6 us of its 0.1 ms:
    # scripts/diag/sync_latency.hip); a second context with events around the dominant stage
    # only then repeats the same steps for the kernel's time (stages_ms, roofline)
    ctx = knn.Context(local, algo=args.algo, train_splits=args.splits)
    pctx = knn.Context(local, algo=args.algo, train_splits=args.splits, profile=3)
    # device rows are 16-B aligned: [n][ld] with ld = 12 for d = 11 (the pad column is never read)
    ld = (d + 3) // 4 * 4
    train = torch.zeros((nt, ld), dtype=torch.float32, device=dev)
    test = torch.zeros((nq, ld), dtype=torch.float32, device=dev)
    train[:, :d] = torch.from_numpy(tf).to(dev)
    test[:, :d] = torch.from_numpy(qf).to(dev)
    labels = torch.from_numpy(tl).to(dev)
    pred = torch.empty(nq, dtype=torch.int32, device=dev)
    for _ in range(args.warmup):
        ctx.predict_device(train, labels, test, k, C, pred, d=d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.predict_device(train, labels, test, k, C, pred, d=d)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    got = pred.cpu().numpy()
    stage_sum = {}
    ppred = torch.empty_like(pred)
    for step in range(args.warmup + args.steps):
        pctx.predict_device(train, labels, test, k, C, ppred, d=d)
        if step >= args.warmup:
            for name, ms in pctx.stage_times().items():
                stage_sum[name] = stage_sum.get(name, 0.0) + ms
    pctx.close()
    assert torch.equal(ppred, pred)
    want = np.loadtxt(os.path.join(REPO, ARFF_L[2]), dtype=np.int32)
    # host buffers in, predictions out (knn_predict: uploads inside the call, PCIe-inclusive):
    # cold = first call on a caching context (train uploaded), warm = the next one
    hctx = knn.Context(local, algo=args.algo, cache_train=True)
    host_ms = {}
    for phase in ("cold", "warm"):
        t1 = time.perf_counter()
        host_pred = hctx.predict(tf, tl, qf, k, C)
        host_ms[phase] = round(1e3 * (time.perf_counter() - t1), 3)
    hctx.close()
    cm = knn.computeConfusionMatrix(got, ql, C)
    pairs = float(nt) * nq * args.steps
    stages = {n: v / args.steps for n, v in stage_sum.items()}
    # the dominant kernel: AUTO picks the direct form here -- k_direct_rows for d <= 16, k <= 16
    # (config L: its segments merged by its own last wave per query group, round 6), else
    # k_direct_tile -- its segments merged by k_merge_vote (stage "merge_vote")
    kname = "direct_tile" if "direct_tile" in stages else "exact_scan"
    scan = stages.get(kname)
    roof = None
    if scan:
        ops = 3.0 * d * nt * nq  # sub, mul, add per dimension per pair (unfused: the reference's bits)
        kernel = ("k_direct_rows" if d <= 16 and k <= 16 else "k_direct_tile") if kname == "direct_tile" \
            else "k_exact_scan"
        roof = {"bound": "valu", "achieved": round(ops / (scan * 1e-3) / 1e12, 3), "peak": 78.6,
                "unit": "Tops/s", "frac": round(ops / (scan * 1e-3) / 1e12 / 78.6, 4),
                "traffic": pmc_traffic("L")[0] if kernel == "k_direct_rows" else None,
                "traffic_source": (pmc_traffic("L")[1] and f"profiles/{pmc_traffic('L')[1]}_pmc_traffic.json")
                if kernel == "k_direct_rows" else None,
                "kernel": kernel, "avg_launch_ms": round(scan, 4),
                "peak_basis": "fp32 VALU: 256 CUs x 4 SIMDs x 32 lanes/clk at 2.4 GHz, packed fp32 "
                              "(v_pk_add/mul_f32: two ops per lane) -- MI355X_MICROARCH.md: 157.3 TFLOP/s "
                              "counting an FMA as 2",
                "merge_ms": round(stages.get("merge_vote", 0.0), 4),
                "merge": ("fused: each query group's last segment wave merges + votes (round 6)"
                          if kernel == "k_direct_rows" else "k_merge_vote"),
                "note": "launch/latency bound: 52.9 M pairs is ~22 us of VALU at peak"}
    out = {
        "metric": METRIC, "value": pairs / elapsed, "unit": "pairs/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "the reference's large ARFF pair (tests/data), parsed by the boundary's reader",
        "config": {"workload": f"L: large-train.arff x large-test.arff ({nt} x {nq} x {d}-d), k={k}",
                   "n_train": nt, "n_query_total": nq, "d": d, "k": k, "classes": C,
                   "parallelism": "single GPU, direct form"},
        "queries_per_s": nq * args.steps / elapsed,
        "stages_ms": {n: round(v, 4) for n, v in stages.items()},
        "stages_source": "a second run of the same steps with HIP events around the dominant stage",
        "bit_match": {"predictions_equal_reference": bool(np.array_equal(got, want)),
                      "host_path_equal": bool(np.array_equal(host_pred, want)),
                      "accuracy": float(np.float32(np.trace(cm)) / np.float32(nq))},
        "host_buffers_ms": host_ms,
        "roofline": roof,
        "cpu_baseline": None if args.no_cpu_baseline else cpu_baseline_arff(k),
    }
    print(json.dumps(out), flush=True)
    ctx.close()


def host_buffer_times(knn, local, algo, train, labels, test, k, C, pred_dev):
    """PCIe-inclusive rates (never `value`): the same KNN call from host buffers through
    knn_predict (main.cpp:25's KNN on host data).  cold = first call on a context with the
    train cache (train + queries uploaded), warm = the next call (train cached, queries
    streamed in batches through two slots overlapping compute), for pageable numpy arrays
    and for page-locked buffers (knn_alloc_pinned).  Predictions must equal the resident
    run's."""
    import torch
    tr, tl, te = train.cpu().numpy(), labels.cpu().numpy(), test.cpu().numpy()
    want = pred_dev.cpu().numpy()
    out = {"note": "knn_predict on host buffers, PCIe-inclusive (H2D of train when cold, of the "
                   "queries always, D2H of predictions); the headline value keeps inputs in HBM"}
    nt, nq = tr.shape[0], te.shape[0]
    pinned = []
    for kind in ("pageable", "pinned"):
        if kind == "pinned":
            ptr, pte = knn.PinnedArray(tr.shape, np.float32), knn.PinnedArray(te.shape, np.float32)
            ptr.array[:] = tr
            pte.array[:] = te
            pinned = [ptr, pte]
            a_tr, a_te = ptr.array, pte.array
        else:
            a_tr, a_te = tr, te
        ctx = knn.Context(local, algo=algo, cache_train=True)
        rec = {}
        for phase in ("cold", "warm"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            got = ctx.predict(a_tr, tl, a_te, k, C)
            ms = 1e3 * (time.perf_counter() - t0)
            st = ctx.stats()
            rec[phase + "_ms"] = round(ms, 2)
            rec[phase + "_pairs_per_s"] = nt * nq / (ms * 1e-3)
            rec[phase + "_h2d_bytes"] = st["h2d_train_bytes"] + st["h2d_query_bytes"]
            rec[phase + "_equal_resident"] = bool(np.array_equal(got, want))
        ctx.close()
        out[kind] = rec
    for p in pinned:
        p.free()
    return out


def pmc_traffic(key):
    """HBM bytes per filter launch from the newest committed rocprofv3 --pmc summary of this
    exact workload: profiles/pmc_latest.json maps the bench's pmc_key (config, filter operands,
    any --nt/--nq override) to the summary scripts/summarize_profile.py wrote last for it.
    Returns (bytes, source tag) or (None, None)."""
    try:
        with open(os.path.join(REPO, "profiles", "pmc_latest.json")) as f:
            rec = json.load(f).get(key)
    except (OSError, ValueError):
        rec = None
    if not rec:
        return None, None
    return rec.get("gemm_filter_bytes_per_launch"), rec.get("tag")


XCHECK_LIMIT_S = 180  # the exchange check's watchdog (a hung collective ends the run, line printed)
XCHECK_TIMEOUT_EXIT = 3  # exit status of a run whose exchange check hung (the line is still printed)


def run_with_watchdog(fn, limit_s, line, rank, exit_fn=os._exit):
    """fn() under a watchdog: if it has not returned after limit_s seconds (a hung RCCL
    collective cannot be interrupted), rank 0's line is printed with the check's status
    "timeout" and the process ends with XCHECK_TIMEOUT_EXIT -- a failure torchrun and the driver
    see, not a success with the hang hidden inside the JSON."""
    def expired():
        if line is not None:
            line["rccl_exchange_check"] = {"status": "timeout", "limit_s": limit_s}
            print(json.dumps(line), flush=True)
        print(f"[bench rank {rank}] exchange check timed out", file=sys.stderr, flush=True)
        sys.stderr.flush()
        exit_fn(XCHECK_TIMEOUT_EXIT)
    wd = threading.Timer(limit_s, expired)
    wd.daemon = True
    wd.start()
    try:
        return fn()
    finally:
        wd.cancel()


def rccl_exchange_check(knn, torch, dist, local, world, rank, share, seed):
    """The C-ABI train-sharded path over a real multi-rank RCCL communicator, checked: every rank
    holds shard_range(NT, world, rank) of a small synthetic train set and all NQ queries,
    knn_predict_train_sharded (shard top-k -> grouped ncclSend/Recv -> merge + vote) gives the
    owned queries' neighbour lists, and the same queries against the WHOLE train set on the
    rank's own GPU (knn_predict_device, the test-sharded path the parity suite pins to the
    oracle) must give the same predictions, global indices and distance bits (mpi.cpp:173-186:
    the gather the exchange replaces).  Runs after the timed region of a multi-rank line, so the
    driver's N = 2/4/8 runs exercise the exchange on xGMI; returns the summary for the line."""
    nt_s, nq_s, d_s, k_s, c_s = 262_144, 8_192, 64, 16, 10
    out = {"n_train": nt_s, "n_query": nq_s, "d": d_s, "k": k_s, "ranks": world, "status": "ok"}
    dev = torch.device("cuda", local)
    bad, ok = 0, 1
    t0 = time.perf_counter()
    ctx = comm = None
    try:
        ctx = knn.Context(local, profile=3)
        uid = [knn.comm_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        comm = knn.Comm(ctx, uid[0], world, rank)
        out["rccl_comm_ranks"] = comm.count()
        a0, a1 = knn.shard_range(nt_s, world, rank)
        m0, m1 = knn.shard_range(nq_s, world, rank)
        shard = torch.empty((a1 - a0, d_s), dtype=torch.float32, device=dev)
        slab = torch.empty(a1 - a0, dtype=torch.int32, device=dev)
        test = torch.empty((nq_s, d_s), dtype=torch.float32, device=dev)
        ctx.generate(shard, slab, a0, d_s, 0, seed, 0, c_s)
        ctx.generate(test, None, 0, d_s, 0, seed, 1, c_s)
        pred = torch.empty(m1 - m0, dtype=torch.int32, device=dev)
        dd = torch.empty((m1 - m0, k_s), dtype=torch.float32, device=dev)
        ii = torch.empty((m1 - m0, k_s), dtype=torch.int32, device=dev)
        comm.predict_train_sharded(shard, slab, a0, test, k_s, c_s, pred, dist=dd, idx=ii)
        torch.cuda.synchronize(dev)
        out["exchange_ms"] = round(ctx.stage_times().get("exchange", float("nan")), 3)
        full = torch.empty((nt_s, d_s), dtype=torch.float32, device=dev)
        flab = torch.empty(nt_s, dtype=torch.int32, device=dev)
        ctx.generate(full, flab, 0, d_s, 0, seed, 0, c_s)
        rp = torch.empty_like(pred)
        rd = torch.empty_like(dd)
        ri = torch.empty_like(ii)
        if m1 > m0:
            ctx.predict_device(full, flab, test[m0:m1], k_s, c_s, rp, dist=rd, idx=ri)
        torch.cuda.synchronize(dev)
        rows = (pred != rp) | (ii != ri).any(dim=1) | (dd.view(torch.int32) != rd.view(torch.int32)).any(dim=1)
        bad = int(rows.sum().item())
    except Exception as e:  # reported on the line; the ranks still meet at the all-reduce below
        ok = 0
        out["status"] = "error"
        out["error"] = f"rank {rank}: {e!r}"[:300]
    finally:
        if comm is not None:
            comm.close()
        if ctx is not None:
            ctx.close()
    v = torch.tensor([bad, 1 - ok], dtype=torch.int64, device="cpu" if share else dev)
    if world > 1:
        dist.all_reduce(v)
    out["mismatched_queries"] = int(v[0].item())
    if int(v[1].item()) and out["status"] == "ok":
        out["status"] = "error on another rank"
    out["equal_to_whole_train_path"] = out["status"] == "ok" and out["mismatched_queries"] == 0
    out["check_s"] = round(time.perf_counter() - t0, 2)
    return out


def resolve_scaling(sharding, strong=False, weak=False):
    """The line's scaling.  Default: strong -- BASELINE's fixed problem (A's 100k / B's 1M
    queries; C's 32M train rows) split over the ranks by the reference's rule, so a --gpus N
    value is that one problem's throughput (mpi.cpp:141-186).  --weak (test-sharded configs
    only, a study option) gives every rank a full query set of its own."""
    if strong and weak:
        raise SystemExit("--strong and --weak exclude each other")
    return "weak" if (sharding == "test" and weak) else "strong"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default K per workload: a timed region of about 5 s (A's step is ~25 ms), long enough for
    # an outside sampler of GPU activity to see the run
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: per config)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default: per config)")
    ap.add_argument("--config", default="A", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--strong", action="store_true",
                    help="(the default) test-sharded configs: split BASELINE's fixed n_query set by the "
                         "reference's rule (shard_range)")
    ap.add_argument("--weak", action="store_true",
                    help="study option, test-sharded configs: every rank gets n_query rows of its own "
                         "(weak scaling) instead of a share of the fixed set")
    ap.add_argument("--exchange", default="rccl", choices=["rccl", "torch"],
                    help="train-sharded configs: C-ABI RCCL communicator or torch.distributed all-to-all")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-buffer calls")
    ap.add_argument("--algo", default="auto", choices=["auto", "gemm", "gemm_split", "gemm_bf16", "direct"])
    ap.add_argument("--splits", type=int, default=0, help="train segments per query tile (0 = auto)")
    ap.add_argument("--nt", type=int, default=0, help="override train rows (kernel studies)")
    ap.add_argument("--nq", type=int, default=0, help="override query rows (kernel studies)")
    ap.add_argument("--no-train-cache", action="store_true",
                    help="recompute the train-side filter operands (norms, tile blocks) in every step")
    ap.add_argument("--shard", default=None, choices=["test", "train", "auto"],
                    help="partition over ranks: test-sharded (train replicated), train-sharded (RCCL "
                         "exchange + merge) or auto (knn_shard_policy); default: the config's own")
    ap.add_argument("--no-uncached", action="store_true",
                    help="skip the extra steps that time a context without the train-operand cache")
    ap.add_argument("--data", default="uniform", choices=["uniform", "clustered"],
                    help="synthetic rows: uniform (SURVEY.md 8d, labels independent of the rows) or "
                         "clustered (class centroid + noise: the labels carry signal, accuracy is non-trivial)")
    ap.add_argument("--no-bit-match", action="store_true",
                    help="skip the oracle check of a sample of this run's predictions")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = DEFAULT_STEPS[args.config]
    if args.warmup is None:
        args.warmup = {"A": 3, "L": 20}.get(args.config, 1)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # KNN_BENCH_SHARE_GPU=1 rehearses N ranks on fewer GPUs (device = local % count, gloo);
    # the real multi-GPU run uses one GPU per rank and RCCL ("nccl").
    share = os.environ.get("KNN_BENCH_SHARE_GPU") == "1"
    if share:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from importlib.util import module_from_spec, spec_from_file_location
    spec = spec_from_file_location("knn_amd", os.path.join(REPO, "knn-using-p_threads-and-mpi_amd", "__init__.py"))
    knn = module_from_spec(spec)
    spec.loader.exec_module(knn)
    if args.config == "L":
        if world > 1:
            raise SystemExit("config L is a single-GPU line (52.9 M pairs)")
        return bench_arff(args, knn, torch, local)

    nt, nq_cfg, d, k, C, seed, scaling, dtype, sharding = CONFIGS[args.config]
    nt, nq_cfg = args.nt or nt, args.nq or nq_cfg
    # the partition: the config's own (BASELINE configs: A/B test-sharded, C train-sharded), or
    # --shard test|train, or --shard auto = knn_shard_policy (north_star's rule: replicate train
    # while it fits one GPU, else shard it)
    shard_req = args.shard or sharding
    if args.shard == "auto":
        sharding = knn.shard_policy(nt, nq_cfg, d, dtype, world,
                                    torch.cuda.get_device_properties(local).total_memory)
    elif args.shard:
        sharding = args.shard
    scaling = resolve_scaling(sharding, args.strong, args.weak)
    kind = 1 if dtype == "bf16" else 0                  # bf16-exact generator values for bf16
    if args.data == "clustered":
        kind += 2                                       # the clustered variants (kinds 2 / 3)
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    dev = torch.device("cuda", local)
    # the train set is resident and unchanged across steps (a serving process): the context
    # keeps its filter-side operands (KNN_OPT_CACHE_TRAIN); the first (warmup) step builds them
    # profile=3: HIP events around the dominant stages only (filter, rescore, exchange, merge) in
    # the timed steps -- every stage timed costs A's 8-GPU share 3 % (scripts/event_overhead.py);
    # the other stages' times come from the untimed diagnostic steps below
    ctx = knn.Context(local, algo=args.algo, train_splits=args.splits, profile=3,
                      cache_train=not args.no_train_cache)
    if sharding == "test":
        # test-sharded: train replicated on every rank, this rank's query rows
        q0, nq = knn.rank_queries(nq_cfg, world, rank, scaling)
        t0_row, nt_local = 0, nt
    else:
        # train-sharded: this rank's train rows, every query (owned queries after the exchange)
        q0, nq = 0, nq_cfg
        t0_row, t1_row = knn.shard_range(nt, world, rank)
        nt_local = t1_row - t0_row
    train = torch.empty((nt_local, d), dtype=tdt, device=dev)
    labels = torch.empty(nt_local, dtype=torch.int32, device=dev)
    test = torch.empty((nq, d), dtype=tdt, device=dev)
    ctx.generate(train, labels, t0_row, d, kind, seed, 0, C)
    truth = torch.empty(nq, dtype=torch.int32, device=dev)  # the generator's labels of the query rows
    ctx.generate(test, truth, q0, d, kind, seed, 1, C)
    if sharding == "test":
        pred = torch.empty(nq, dtype=torch.int32, device=dev)
    else:
        rec = torch.empty((nq, 3, k), dtype=torch.int32, device=dev)
        own0, own1 = knn.shard_range(nq, world, rank)
        pred = torch.empty(own1 - own0, dtype=torch.int32, device=dev)
    cur = torch.cuda.current_stream(dev).cuda_stream
    # train-sharded exchange: the C ABI's RCCL communicator (knn_predict_train_sharded) by
    # default; "torch" = exchange_shard_lists over torch.distributed (the only choice when
    # ranks share a GPU: RCCL wants one rank per device)
    exchange = args.exchange if not share else "torch"
    comm = None
    rccl_ranks = None
    if sharding == "train" and exchange == "rccl":
        uid = [knn.comm_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        comm = knn.Comm(ctx, uid[0], world, rank)
        rccl_ranks = comm.count()  # ncclCommCount: the ranks RCCL itself sees

    def step():
        if sharding == "test":
            ctx.predict_device(train, labels, test, k, C, pred)
            return ctx.stage_times()
        if comm is not None:
            # shard top-k -> grouped ncclSend/Recv -> merge + vote, one stream, one C call
            t_x = time.perf_counter()
            comm.predict_train_sharded(train, labels, t0_row, test, k, C, pred, stream=cur)
            torch.cuda.current_stream(dev).synchronize()
            times = ctx.stage_times()
            times["train_sharded_wall"] = 1e3 * (time.perf_counter() - t_x)
            return times
        # per-shard exact top-k -> all-to-all (torch.distributed) -> merge + vote, on one stream
        ctx.shard_topk_device(train, labels, test, k, C, t0_row, rec, stream=cur)
        times = ctx.stage_times()
        t_x = time.perf_counter()
        lists, _ = knn.exchange_shard_lists(rec, nq, world, rank)
        torch.cuda.current_stream(dev).synchronize()
        times["exchange_wall"] = 1e3 * (time.perf_counter() - t_x)
        ctx.merge_vote_device(lists, k, C, pred, stream=cur)
        times.update(ctx.stage_times())
        return times

    for i in range(args.warmup):
        step()
        print(f"[bench rank {rank}] warmup {i + 1}/{args.warmup} done", file=sys.stderr, flush=True)
    stage_sum = {}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        for name, ms in step().items():
            stage_sum[name] = stage_sum.get(name, 0.0) + ms
        if rank == 0:
            print(f"[bench] step {i + 1}/{args.steps}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if share else dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    stats = ctx.stats()
    pred_timed = pred.clone()  # the timed steps' predictions (bit_match below checks these)
    # select stage (k_rescore): one untimed diagnostic pass counts the filter's candidates,
    # giving the rescore's algorithmic bytes (select stage vs HBM)
    select = None
    # untimed diagnostic steps (every rank: a train-sharded step is collective) on a context
    # with every stage timed and the filter's candidates counted (profile=2); the first builds
    # its train operand cache like the warmup did, the second is the one reported
    ctx.close()
    ctx = knn.Context(local, algo=args.algo, train_splits=args.splits, profile=2,
                      cache_train=not args.no_train_cache)
    if comm is not None:
        comm.ctx = ctx  # the communicator is bound to a device, the context per call
    step()
    diag_stages = step()
    if "rescore" in stage_sum:
        cand = ctx.stats()["candidates"]
        stats["candidates"] = cand  # the timed steps do not count them (profile=2 pass only)
        esz = 2 if dtype == "bf16" else 4
        nseg = max(1, stats["train_segments"])
        resc_ms = stage_sum["rescore"] / args.steps
        # cnt words + (idx, L, U) per candidate + the query row + k exact rows (a lower
        # bound on the survivors) + k labels + the prediction
        byts = 4 * nseg * nq + 12 * cand + nq * d * esz + nq * k * (d * esz + 4) + 4 * nq
        select = {"kernel": "k_rescore", "bound": "hbm", "avg_launch_ms": round(resc_ms, 3),
                  "candidates_per_query": round(cand / nq, 1), "algorithmic_bytes": byts,
                  "achieved": round(byts / (resc_ms * 1e-3) / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                  "frac": round(byts / (resc_ms * 1e-3) / 1e9 / 8000.0, 4)}
    # the same step with the train-side operands rebuilt in every step (a context without
    # KNN_OPT_CACHE_TRAIN: the reference's one-shot KNN(train, test, k) pays this pass,
    # main.cpp:25-43) -- reported beside value, never as it
    uncached_ms = None
    if not args.no_train_cache and not args.no_uncached:
        ctx.close()
        ctx = knn.Context(local, algo=args.algo, train_splits=args.splits, profile=0, cache_train=False)
        if comm is not None:
            comm.ctx = ctx
        step()  # workspace allocation
        n_unc = 3 if 1e3 * elapsed / args.steps < 100 else 1
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t_u = time.perf_counter()
        for _ in range(n_unc):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tu = torch.tensor([time.perf_counter() - t_u], dtype=torch.float64, device="cpu" if share else dev)
        if world > 1:
            dist.all_reduce(tu, op=dist.ReduceOp.MAX)
        uncached_ms = 1e3 * float(tu.item()) / n_unc
    # bit-match of this run's own predictions (rank 0's queries, a spread sample) against the
    # oracle over the whole train set
    bitm = None
    if rank == 0 and not args.no_bit_match:
        own_q0 = q0 if sharding == "test" else knn.shard_range(nq, world, rank)[0]
        pl = pred_timed.cpu().numpy()
        n_s = 64 if float(nt) * d <= 2.1e9 else 8
        pos = np.unique(np.linspace(0, len(pl) - 1, min(n_s, len(pl))).astype(np.int64))
        bitm = oracle_bit_match(seed, kind, nt, d, k, C, own_q0 + pos, pl[pos])
    # computeAccuracy (main.cpp:102-112) of this rank's predictions against the generator's labels
    # of its query rows (~1/C for uniform rows, whose labels carry no signal)
    own_truth = truth if sharding == "test" else truth[own0:own1]
    accuracy = round(float((pred_timed == own_truth).float().mean().item()), 6) if len(pred_timed) else None
    host = None
    if rank == 0 and world == 1 and sharding == "test" and not args.no_host_path:
        host = host_buffer_times(knn, local, args.algo, train, labels, test, k, C, pred)
    total_q = nq_cfg * world if scaling == "weak" else nq_cfg
    gathered = None
    if world > 1:  # outside the timed region: rank 0 collects predictions (mpi.cpp:186)
        p0 = q0 if sharding == "test" else own0
        full = knn.gather_predictions(pred.cpu().numpy(), p0, total_q, world, rank)
        if rank == 0:
            gathered = int((full >= 0).sum())

    line = None
    if rank == 0:
        pairs = float(total_q) * nt * args.steps
        stages = {n: v / args.steps for n, v in stage_sum.items()}
        stages.update({n: v for n, v in diag_stages.items() if n not in stages})
        filt_ms = stages.get("gemm_filter")
        operands = stats.get("filter_operands") or dtype
        # the workload key of the PMC summaries (scripts/summarize_profile.py reads it back)
        pmc_key = (args.config + ("" if operands == dtype else PMC_SUFFIX.get(operands, "/" + operands))
                   + ("/clustered" if args.data == "clustered" else "")
                   + (f"/nt{args.nt}" if args.nt else "") + (f"/nq{args.nq}" if args.nq else ""))
        roof = None
        if filt_ms:
            peak, issued = FILTER_ROOF[operands]
            flops = 2.0 * d * nq * nt_local  # algorithmic: 2d FLOP per (query, train) pair, one launch
            ach = flops / (filt_ms * 1e-3) / 1e12
            traffic, traffic_tag = pmc_traffic(pmc_key)
            roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": round(peak, 1),
                    "unit": "TFLOP/s", "frac": round(ach / peak, 4),
                    "traffic": traffic, "traffic_source": traffic_tag and f"profiles/{traffic_tag}_pmc_traffic.json",
                    "kernel": "k_gemm_fused" if stats.get("fused_norm") else "k_gemm_filter",
                    "filter_operands": operands,
                    "algorithmic_flops_per_launch": flops, "avg_launch_ms": round(filt_ms, 3)}
            if issued > 1:
                roof["peak_basis"] = (f"bf16 dense {MFMA_PEAK_TFLOPS['bf16']} TFLOP/s / {issued}: "
                                      f"{issued} bf16 MFMA products per fp32 product (hi.hi + hi.lo + lo.hi)")
                roof["mfma_flops_issued_per_launch"] = issued * flops
                roof["x_fp32_mfma_peak"] = round(ach / MFMA_PEAK_TFLOPS["f32"], 3)
            elif operands == "bf16 rounded":
                roof["peak_basis"] = (f"bf16 dense {MFMA_PEAK_TFLOPS['bf16']} TFLOP/s: fp32 rows rounded to bf16 "
                                      "for the filter only (one bf16 MFMA product per fp32 product); "
                                      "distances re-scored exactly in fp32")
                roof["x_fp32_mfma_peak"] = round(ach / MFMA_PEAK_TFLOPS["f32"], 3)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(d, k, C, seed, kind, nt)
        par = (f"test-sharded dp{world}, train replicated" if sharding == "test" else
               f"train-sharded x{world} (shard_range of train rows), all-to-all of per-shard top-k "
               f"({'RCCL via knn_predict_train_sharded' if comm is not None else 'torch.distributed'}), merge")
        out = {
            "metric": METRIC, "value": pairs / elapsed, "unit": "pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": dtype,
            "data": (f"synthetic{' clustered (class centroid + noise)' if args.data == 'clustered' else ''} "
                     "(counter-based generator, SURVEY.md 8d), generated in HBM"),
            "accuracy_vs_generator_labels": accuracy,
            "config": {"workload": f"{args.config}: synthetic{' clustered' if args.data == 'clustered' else ''} "
                                   f"{nt} train x {nq_cfg} query"
                                   f"{'/GPU' if scaling == 'weak' else ''} x {d}-d {dtype}, k={k}",
                       "n_train": nt, "n_query_total": total_q, "d": d, "k": k, "classes": C,
                       "parallelism": par, "shard": {"requested": shard_req, "used": sharding}},
            "queries_per_s": total_q * args.steps / elapsed,
            "stages_ms": {n: round(v, 3) for n, v in stages.items()},
            "stages_source": ("timed steps for " + ", ".join(sorted(stage_sum)) +
                              "; one untimed profiled step for the rest"),
            "gemm_stats": stats,
            "predictions_gathered": gathered,
            "rccl_comm_ranks": rccl_ranks,
            "pmc_key": pmc_key,
            "ms_per_step_uncached": None if uncached_ms is None else round(uncached_ms, 3),
            "value_uncached": None if uncached_ms is None else pairs / args.steps / (uncached_ms * 1e-3),
            "bit_match": bitm,
            "train_operands": ("cached across steps (KNN_OPT_CACHE_TRAIN: norms, tile statistics and bf16 "
                               "tile blocks built in the warmup step)" if stats.get("train_operands_cached")
                               else "rebuilt every step"),
            "roofline": roof,
            "cpu_baseline": cpu,
            "select_stage": select,
            "host_buffers": host,
        }
        line = out
    # multi-rank lines: the train-sharded C-ABI path over a real RCCL communicator of all ranks,
    # checked against the whole-train path (KNN_BENCH_XCHECK=1 runs it at one rank too)
    if (world > 1 and not share) or os.environ.get("KNN_BENCH_XCHECK") == "1":
        xc = run_with_watchdog(lambda: rccl_exchange_check(knn, torch, dist, local, world, rank, share, seed),
                               XCHECK_LIMIT_S, line, rank)
        if line is not None:
            line["rccl_exchange_check"] = xc
    if line is not None:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
