"""Host-buffer calls (knn_predict, the replacement of main.cpp:25's KNN on ArffData): the
cached train upload (KNN_OPT_CACHE_TRAIN, keyed by buffer + shape + generation), query
batches streamed through two device slots on a copy stream, GEMM-path passes bounded by
the candidate workspace, and page-locked buffers (knn_alloc_pinned).  Every variant must
give the oracle's results bit for bit (main.cpp:40-82); the byte counters
(knn_last_stats [6], [7]) show what moved host -> device.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data(oracle, nt=30000, nq=2500, d=64, seed=61):
    tr, tl = oracle.gen(seed, 0, 0, nt, d)
    te, _ = oracle.gen(seed, 1, 0, nq, d)
    return tr, tl, te


def _same(a, b):
    return all(np.array_equal(x.view(np.uint32) if x.dtype == np.float32 else x,
                              y.view(np.uint32) if y.dtype == np.float32 else y) for x, y in zip(a, b))


def test_train_cache_second_call_uploads_no_train(knn, oracle):
    tr, tl, te = _data(oracle)
    k = 10
    bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
    ctx = knn.Context(0, cache_train=True)
    try:
        first = ctx.predict(tr, tl, te, k, 10, topk=True)
        s1 = ctx.stats()
        second = ctx.predict(tr, tl, te, k, 10, topk=True)
        s2 = ctx.stats()
        assert s1["h2d_train_bytes"] == tr.nbytes + tl.nbytes
        assert s2["h2d_train_bytes"] == 0          # the cached upload is reused
        assert s2["h2d_query_bytes"] == te.nbytes  # queries always move
        assert _same(first, second) and _same(first, (opred, odist, oidx))
        # a new generation (the caller rewrote the buffer in place) uploads again
        tr[:100] = tr[100:200]
        ctx.set_generation(1)
        third = ctx.predict(tr, tl, te, k, 10, topk=True)
        assert ctx.stats()["h2d_train_bytes"] == tr.nbytes + tl.nbytes
        bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
        assert _same(third, (opred, odist, oidx))
        # another train buffer with the same shape is a miss
        tr2 = tr.copy()
        ctx.predict(tr2, tl, te, k, 10)
        assert ctx.stats()["h2d_train_bytes"] > 0
    finally:
        ctx.close()


def test_no_cache_uploads_every_call(knn, oracle):
    tr, tl, te = _data(oracle, nt=5000, nq=100)
    ctx = knn.Context(0)
    try:
        for _ in range(2):
            ctx.predict(tr, tl, te, 5, 10)
            assert ctx.stats()["h2d_train_bytes"] == tr.nbytes + tl.nbytes
    finally:
        ctx.close()


@pytest.mark.parametrize("algo", ["auto", "direct", "gemm_bf16"])
def test_streamed_query_batches(knn, oracle, monkeypatch, algo):
    """Small batches (KNN_BATCH_ROWS) exercise the two-slot pipeline: upload of batch b+1
    and download of batch b-1 overlap batch b; a query range (mpi.cpp:26 slices) too."""
    tr, tl, te = _data(oracle, nt=40000, nq=3001, d=128)
    k = 7
    bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
    monkeypatch.setenv("KNN_BATCH_ROWS", "700")
    ctx = knn.Context(0, algo=algo)
    try:
        got = ctx.predict(tr, tl, te, k, 10, topk=True)
        assert _same(got, (opred, odist, oidx))
        assert ctx.stats()["h2d_query_bytes"] == te.nbytes
        part = ctx.predict(tr, tl, te, k, 10, q_begin=123, q_end=2345, topk=True)
        assert _same(part, (opred[123:2345], odist[123:2345], oidx[123:2345]))
    finally:
        ctx.close()


def test_gemm_workspace_passes(knn, oracle, monkeypatch):
    """The GEMM path runs the queries in passes bounded by the candidate workspace
    (KNN_WS_QUERIES here, a quarter of the free HBM by default): same results."""
    import torch
    tr, tl, te = _data(oracle, nt=60000, nq=2000, d=128, seed=67)
    k = 10
    bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
    monkeypatch.setenv("KNN_WS_QUERIES", "333")
    ctx = knn.Context(0, algo="gemm_bf16")
    try:
        dev = "cuda:0"
        dtr, dtl, dte = (torch.from_numpy(x).to(dev) for x in (tr, tl, te))
        pred = torch.empty(len(te), dtype=torch.int32, device=dev)
        dist = torch.empty((len(te), k), dtype=torch.float32, device=dev)
        idx = torch.empty((len(te), k), dtype=torch.int32, device=dev)
        ctx.predict_device(dtr, dtl, dte, k, 10, pred, dist, idx)
        assert ctx.stats()["train_segments"] >= 1
        assert _same((pred.cpu().numpy(), dist.cpu().numpy(), idx.cpu().numpy()), (opred, odist, oidx))
    finally:
        ctx.close()


def test_pinned_buffers(knn, oracle):
    tr, tl, te = _data(oracle, nt=20000, nq=1500)
    k = 9
    bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
    ptr = knn.PinnedArray(tr.shape, np.float32)
    pte = knn.PinnedArray(te.shape, np.float32)
    ptr.array[:] = tr
    pte.array[:] = te
    ctx = knn.Context(0, cache_train=True)
    try:
        got = ctx.predict(ptr.array, tl, pte.array, k, 10, topk=True)
        assert _same(got, (opred, odist, oidx))
    finally:
        ctx.close()
        ptr.free()
        pte.free()


def test_loaded_library_is_this_trees(knn):
    """The libknn_amd.so these GPU tests load was built from the sources beside it
    (knn_build_id() == build_id.py's hash of the tree)."""
    built, tree = knn.build_id()
    assert built == tree


def test_cache_survives_reused_temporaries(knn, oracle):
    """cache_train with inputs _dataset must convert (float64 features, int64 labels): each
    call's temporaries are new arrays that the allocator may place at a freed temporary's
    address; the results must still be each call's own (the Context holds the keyed arrays)."""
    ctx = knn.Context(0, cache_train=True)
    try:
        for seed in (71, 72, 73):
            tr, tl, te = _data(oracle, nt=6000, nq=300, d=64, seed=seed)
            bad, opred, odist, oidx = oracle.knn(tr, tl, te, 5, 10)
            got = ctx.predict(tr.astype(np.float64), tl.astype(np.int64), te.astype(np.float64), 5, 10, topk=True)
            assert _same(got, (opred, odist, oidx)), seed
    finally:
        ctx.close()


def test_cpp_cache_keyed_by_flat_view(knn, oracle, tmp_path):
    """The C++ KNN() contexts cache train uploads: datasets of one shape parsed, classified
    and freed in turn (their pinned buffers reused at the same address) must each give their
    own predictions (tests/cpp/flat_cache_check.cpp)."""
    import os
    import subprocess
    from conftest import PKG_DIR
    exe = os.path.join(PKG_DIR, "build", "flat_cache_check")
    if not os.path.exists(exe):
        pytest.skip("build/flat_cache_check not built (make -C knn-using-p_threads-and-mpi_amd)")
    args, want = [], []
    for seed in (81, 82, 83):
        tr, tl, te = _data(oracle, nt=3000, nq=200, d=16, seed=seed)
        paths = []
        for name, f, lab in (("train", tr, tl), ("test", te, np.zeros(len(te), np.int32))):
            p = tmp_path / f"{name}{seed}.arff"
            with open(p, "w") as fh:
                fh.write("@relation r\n" + "".join(f"@attribute a{i} numeric\n" for i in range(16)))
                fh.write("@attribute class numeric\n@data\n")
                for r in range(len(f)):
                    fh.write(",".join(f"{v:.9g}" for v in f[r]) + f",{lab[r]}\n")
            paths.append(str(p))
        args += paths
        want.append(oracle.knn(tr, tl, te, 5, 10)[1])
    r = subprocess.run([exe, "5"] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 3
    for line, w in zip(lines, want):
        assert np.array_equal(np.array(line.split(), np.int32), w)
