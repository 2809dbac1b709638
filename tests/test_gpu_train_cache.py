"""Round-4 boundary behaviour on the device.

* The train-side operands of the bf16 MFMA filter (train norms, 64-row tile statistics, bf16
  tile blocks) are kept across calls under KNN_OPT_CACHE_TRAIN (knn_last_stats()[8]): a
  second call on the same train view runs no train pass and gives the same bits; an in-place
  write seen by torch, knn_set_generation or another tensor recomputes them.  The reference
  re-reads every train row for every query (main.cpp:40-43); what is cached is the part of
  that work that depends on train alone.
* knn_merge_vote_device rejects source lists that are not ascending (KNN_EINVAL).
* knn_predict_train_sharded's failure vote reads preset device words: a local failure on a
  one-rank communicator returns that failure and leaves the communicator usable.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _rows(knn, nt, nq, d, seed, dtype="f32"):
    import torch
    kind = 1 if dtype == "bf16" else 0
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    g = knn.Context(0)
    train = torch.empty((nt, d), dtype=tdt, device=DEV)
    labels = torch.empty(nt, dtype=torch.int32, device=DEV)
    test = torch.empty((nq, d), dtype=tdt, device=DEV)
    g.generate(train, labels, 0, d, kind, seed, 0, 10)
    g.generate(test, None, 0, d, kind, seed, 1, 10)
    torch.cuda.synchronize()
    g.close()
    return train, labels, test


def _call(ctx, train, labels, test, k):
    import torch
    nq = test.shape[0]
    pred = torch.empty(nq, dtype=torch.int32, device=DEV)
    dist = torch.empty((nq, k), dtype=torch.float32, device=DEV)
    idx = torch.empty((nq, k), dtype=torch.int32, device=DEV)
    ctx.predict_device(train, labels, test, k, 10, pred, dist, idx)
    torch.cuda.synchronize()
    return pred.cpu().numpy(), dist.cpu().numpy().view(np.uint32), idx.cpu().numpy(), ctx.stats()


def _same(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a[:3], b[:3]))


@pytest.mark.parametrize("dtype,d,k", [("f32", 128, 10), ("f32", 64, 32), ("bf16", 256, 100)])
def test_train_operands_cached_across_calls(knn, oracle, dtype, d, k):
    import torch
    nt, nq = 40_000, 1_500
    train, labels, test = _rows(knn, nt, nq, d, 71, dtype)
    # (gemm_bf16: the MFMA filter at a size AUTO would give to the direct form)
    ctx = knn.Context(0, algo="gemm_bf16", profile=True, cache_train=True)
    ref = knn.Context(0, algo="gemm_bf16")  # no cache: every call prepares train itself
    try:
        want = _call(ref, train, labels, test, k)
        first = _call(ctx, train, labels, test, k)
        assert first[3]["fused_norm"] and not first[3]["train_operands_cached"], first[3]
        assert _same(first, want)
        second = _call(ctx, train, labels, test, k)
        assert second[3]["train_operands_cached"], second[3]
        assert _same(second, want)
        # other queries against the cached train: still the oracle's bits
        test2 = test.flip(0).contiguous()
        third = _call(ctx, train, labels, test2, k)
        assert third[3]["train_operands_cached"]
        qs = np.linspace(0, nq - 1, 6).astype(np.int64)
        bad, opred, odist, oidx = oracle.knn(train.float().cpu().numpy(), labels.cpu().numpy(),
                                             test2.float().cpu().numpy()[qs], k, 10)
        assert bad == 0 and np.array_equal(third[2][qs], oidx) and np.array_equal(third[0][qs], opred)
        # an in-place write through torch bumps the generation: recomputed, and the new rows count
        train[:2000] = train[2000:4000]
        fourth = _call(ctx, train, labels, test, k)
        assert not fourth[3]["train_operands_cached"]
        assert _same(fourth, _call(ref, train, labels, test, k))
        # an explicit generation recomputes too; a different tensor of the same shape is a miss
        ctx.set_generation(1234)
        assert not _call(ctx, train, labels, test, k)[3]["train_operands_cached"]
        other = train.clone()
        assert not _call(ctx, other, labels, test, k)[3]["train_operands_cached"]
        assert _call(ctx, other, labels, test, k)[3]["train_operands_cached"]
        # a context without cache_train never reuses
        assert not _call(ref, train, labels, test, k)[3]["train_operands_cached"]
    finally:
        ctx.close()
        ref.close()


def test_generate_into_slice_invalidates_cache(knn):
    """Context.generate writes through the C ABI, behind torch's version counter: a write into a
    slice of a cached train tensor, from this context or from another one, must drop the cached
    operands (the next call recomputes them and matches an uncached context bit for bit)."""
    import torch
    train, labels, test = _rows(knn, 30_000, 1_000, 128, 91)
    ctx = knn.Context(0, algo="gemm_bf16", cache_train=True)
    ref = knn.Context(0, algo="gemm_bf16")
    other = knn.Context(0)
    try:
        _call(ctx, train, labels, test, 10)
        assert _call(ctx, train, labels, test, 10)[3]["train_operands_cached"]
        for writer, seed in ((ctx, 5), (other, 6)):
            part = train[7_000:9_000]            # a view: another tensor object, same storage
            writer.generate(part, None, 7_000, 128, 0, seed, 0, 10)
            torch.cuda.synchronize()
            got = _call(ctx, train, labels, test, 10)
            assert not got[3]["train_operands_cached"], writer
            assert _same(got, _call(ref, train, labels, test, 10))
            assert _call(ctx, train, labels, test, 10)[3]["train_operands_cached"]
        # a write elsewhere (another tensor) leaves the cache alone
        spare = torch.empty_like(train[:100])
        other.generate(spare, None, 0, 128, 0, 7, 0, 10)
        torch.cuda.synchronize()
        assert _call(ctx, train, labels, test, 10)[3]["train_operands_cached"]
    finally:
        ctx.close()
        ref.close()
        other.close()


def test_cache_train_without_device_flag(knn):
    """ABI 3: KNN_OPT_CACHE_TRAIN alone never reuses operands derived from a caller's device
    buffer (only knn_predict's own upload); KNN_OPT_CACHE_TRAIN_DEVICE opts in."""
    import ctypes
    import torch
    train, labels, test = _rows(knn, 30_000, 800, 128, 93)
    lib = knn.load_library()
    h = ctypes.c_void_p()
    opts = knn.knn_opts(0, knn.ALGOS["gemm_bf16"], 0, 0, knn.KNN_OPT_CACHE_TRAIN)
    assert lib.knn_create(ctypes.byref(h), ctypes.byref(opts)) == knn.KNN_OK
    try:
        tr = knn._device_dataset(train, labels)
        te = knn._device_dataset(test)
        pred = torch.empty(800, dtype=torch.int32, device=DEV)
        st = torch.cuda.current_stream().cuda_stream
        v = (ctypes.c_int64 * 9)()
        for _ in range(2):
            assert lib.knn_predict_device(h, ctypes.byref(tr), ctypes.byref(te), 10, 10, pred.data_ptr(),
                                          None, None, ctypes.c_void_p(st)) == knn.KNN_OK
            lib.knn_last_stats(h, v, 9)
            assert v[5] == 1 and v[8] == 0  # fused filter ran, train operands rebuilt
    finally:
        lib.knn_destroy(h)


def test_train_operands_cached_host_path(knn, oracle):
    """knn_predict with KNN_OPT_CACHE_TRAIN: a hit on the uploaded copy is also a hit on its
    filter operands; a new upload (generation) recomputes them."""
    tr, tl = oracle.gen(81, 0, 0, 40_000, 128)
    te, _ = oracle.gen(81, 1, 0, 800, 128)
    bad, opred, odist, oidx = oracle.knn(tr, tl, te, 10, 10)
    ctx = knn.Context(0, algo="gemm_bf16", cache_train=True)
    try:
        a = ctx.predict(tr, tl, te, 10, 10, topk=True)
        assert not ctx.stats()["train_operands_cached"]
        b = ctx.predict(tr, tl, te, 10, 10, topk=True)
        s = ctx.stats()
        assert s["h2d_train_bytes"] == 0 and s["train_operands_cached"], s
        for got in (a, b):
            assert np.array_equal(got[0], opred) and np.array_equal(got[2], oidx)
            assert np.array_equal(got[1].view(np.uint32), odist.view(np.uint32))
        tr[:50] = tr[50:100]
        ctx.set_generation(7)
        c = ctx.predict(tr, tl, te, 10, 10, topk=True)
        assert not ctx.stats()["train_operands_cached"]
        bad, opred, odist, oidx = oracle.knn(tr, tl, te, 10, 10)
        assert np.array_equal(c[0], opred) and np.array_equal(c[2], oidx)
    finally:
        ctx.close()


@pytest.mark.parametrize("dtype,d,k", [("f32", 64, 32), ("f32", 128, 10), ("f32", 128, 16), ("bf16", 256, 5),
                                       ("bf16", 64, 24)])
def test_fused_queries_per_wave_shapes(knn, oracle, dtype, d, k, monkeypatch):
    """The register-list filter with 32 queries per wave on 64-row tiles (QG = 1) and with 64
    per wave on 32-row tiles (QG = 2, picked for large query counts): both give the oracle's
    top-k and predictions bit for bit (main.cpp:40-82), ragged sizes included."""
    nt, nq = 21_000 + 37, 1_500 + 11
    train, labels, test = _rows(knn, nt, nq, d, 23, dtype)
    trf, lab, tef = train.float().cpu().numpy(), labels.cpu().numpy(), test.float().cpu().numpy()
    qs = np.linspace(0, nq - 1, 40).astype(np.int64)
    bad, opred, odist, oidx = oracle.knn(trf, lab, tef[qs], k, 10)
    assert bad == 0
    out = {}
    for qg in ("1", "2"):
        monkeypatch.setenv("KNN_FUSED_QG", qg)
        c = knn.Context(0, algo="gemm_bf16")
        out[qg] = _call(c, train, labels, test, k)
        c.close()
        assert out[qg][3]["fused_norm"]
        assert np.array_equal(out[qg][2][qs], oidx) and np.array_equal(out[qg][0][qs], opred)
        assert np.array_equal(out[qg][1][qs], odist.view(np.uint32))
    assert _same(out["1"], out["2"])


@pytest.mark.parametrize("k", [33, 64, 100, 104])
def test_fused_long_register_lists_vs_heaps(knn, oracle, k, monkeypatch):
    """d = 256, 32 < k <= 104: the filter keeps per-half 52-entry register lists (32-row tiles
    in quads) instead of LDS heaps; both shapes give the oracle's top-k and predictions bit for
    bit (main.cpp:40-82), and each other's.  k = 104 fills the lists (no pad entries)."""
    nt, nq = 20_000 + 53, 1_200 + 7
    train, labels, test = _rows(knn, nt, nq, 256, 29, "bf16")
    trf, lab, tef = train.float().cpu().numpy(), labels.cpu().numpy(), test.float().cpu().numpy()
    qs = np.linspace(0, nq - 1, 24).astype(np.int64)
    bad, opred, odist, oidx = oracle.knn(trf, lab, tef[qs], k, 10)
    assert bad == 0
    out = {}
    for heaps in (False, True):
        if heaps:
            monkeypatch.setenv("KNN_FUSED_HEAPS", "1")
        c = knn.Context(0, algo="gemm_bf16")
        out[heaps] = _call(c, train, labels, test, k)
        c.close()
        assert out[heaps][3]["fused_norm"] and out[heaps][3]["fallback_queries"] == 0
        assert np.array_equal(out[heaps][2][qs], oidx) and np.array_equal(out[heaps][0][qs], opred)
        assert np.array_equal(out[heaps][1][qs], odist.view(np.uint32))
    assert _same(out[False], out[True])


def test_profile_hot_stages_only(knn):
    """profile = 3 times only the dominant stages (the filter and the rescore here); profile = 1
    times every stage; results are the same."""
    train, labels, test = _rows(knn, 30_000, 2_000, 128, 5)
    res, names = {}, {}
    for prof in (1, 3):
        c = knn.Context(0, algo="gemm_bf16", profile=prof)
        res[prof] = _call(c, train, labels, test, 10)
        names[prof] = set(c.stage_times())
        c.close()
    assert _same(res[1], res[3])
    assert {"norms", "gemm_filter", "rescore"} <= names[1]
    assert names[3] == {"gemm_filter", "rescore"}


def test_merge_rejects_unsorted_lists(knn):
    import torch
    c = knn.Context(0)
    try:
        k, nq = 70, 5
        rec = torch.zeros((2, nq, 3, k), dtype=torch.int32, device=DEV)
        d = torch.arange(k, dtype=torch.float32, device=DEV).view(torch.int32)
        for s in range(2):
            rec[s, :, 0, :] = d
            rec[s, :, 1, :] = torch.arange(k, dtype=torch.int32, device=DEV) + 1000 * s
        pred = torch.empty(nq, dtype=torch.int32, device=DEV)
        c.merge_vote_device(rec, k, 10, pred)  # sorted: fine
        bad = rec.clone()
        bad[0, 3, 0, 5], bad[0, 3, 0, 6] = bad[0, 3, 0, 6].item(), bad[0, 3, 0, 5].item()  # a descent in batch 0
        with pytest.raises(knn.KnnError) as e:
            c.merge_vote_device(bad, k, 10, pred)
        assert e.value.status == knn.KNN_EINVAL
        bad = rec.clone()
        bad[1, 0, 0, 64] = 0  # batch 1 starts below batch 0's last key
        bad[1, 0, 1, 64] = 0
        with pytest.raises(knn.KnnError):
            c.merge_vote_device(bad, k, 10, pred)
    finally:
        c.close()


def test_comm_local_failure_vote_single_rank(knn, oracle):
    """A local failure (an argument only this rank passes: pred NULL) goes through the vote
    and comes back as itself; the communicator stays usable."""
    import torch
    trf, tl = oracle.gen(17, 0, 0, 9000, 64)
    tef, _ = oracle.gen(17, 1, 0, 300, 64)
    bad, opred, _, _ = oracle.knn(trf, tl, tef, 5, 10)
    train = torch.from_numpy(trf).to(DEV)
    test = torch.from_numpy(tef).to(DEV)
    labels = torch.from_numpy(tl).to(DEV)
    ctx = knn.Context(0)
    comm = knn.Comm(ctx, knn.comm_unique_id(), 1, 0)
    try:
        import ctypes
        tr = knn._device_dataset(train, labels, None)
        te = knn._device_dataset(test, None, None)
        st = ctx.lib.knn_predict_train_sharded(ctx.h, comm.h, ctypes.byref(tr), 0, ctypes.byref(te), 5, 10,
                                               None, None, None, None)
        assert st == knn.KNN_EINVAL
        assert not comm.broken()  # a voted local failure leaves the communicator healthy
        pred = torch.empty(300, dtype=torch.int32, device=DEV)
        comm.predict_train_sharded(train, labels, 0, test, 5, 10, pred)
        torch.cuda.synchronize()
        assert np.array_equal(pred.cpu().numpy(), opred)
    finally:
        comm.close()
        ctx.close()


def test_stream_device_mismatch_rejected(knn):
    import torch
    if torch.cuda.device_count() > 1:
        pytest.skip("needs one visible device (the check is exercised with a fake index)")
    c = knn.Context(0)
    try:
        c.device = 1  # pretend the context lives on another device
        x = torch.zeros((4, 64), dtype=torch.float32, device=DEV)
        lab = torch.zeros(4, dtype=torch.int32, device=DEV)
        pred = torch.empty(4, dtype=torch.int32, device=DEV)
        with pytest.raises(knn.KnnError):
            c.predict_device(x, lab, x, 1, 2, pred)
    finally:
        c.device = 0
        c.close()


@pytest.mark.parametrize("dtype,d,k", [("f32", 64, 32), ("f32", 128, 10), ("f32", 128, 16), ("bf16", 64, 24),
                                       ("f32", 128, 32)])
def test_fused16_shapes_vs_oracle(knn, oracle, dtype, d, k, monkeypatch):
    """k_gemm_fused16 (KNN_FUSED_MFMA16=1, round 6): the register-list filter on
    v_mfma_f32_16x16x32_bf16 -- quarter lists, swizzled LDS rows -- in both query shapes
    (32 queries per wave on 64-row tiles, 64 on 32-row tiles) gives the oracle's top-k and
    predictions bit for bit (main.cpp:40-82), the same as the 32x32 filter, and reports its
    MFMA shape.  Pieces (several per query tile) run the quarter-list exchange."""
    nt, nq = 21_000 + 37, 1_500 + 11
    train, labels, test = _rows(knn, nt, nq, d, 31, dtype)
    trf, lab, tef = train.float().cpu().numpy(), labels.cpu().numpy(), test.float().cpu().numpy()
    qs = np.linspace(0, nq - 1, 40).astype(np.int64)
    bad, opred, odist, oidx = oracle.knn(trf, lab, tef[qs], k, 10)
    assert bad == 0
    c = knn.Context(0, algo="gemm_bf16")
    ref = _call(c, train, labels, test, k)
    c.close()
    assert ref[3]["filter_mfma"] == 32
    monkeypatch.setenv("KNN_FUSED_MFMA16", "1")
    for qg in ("1", "2"):
        monkeypatch.setenv("KNN_FUSED_QG", qg)
        c = knn.Context(0, algo="gemm_bf16")
        got = _call(c, train, labels, test, k)
        c.close()
        assert got[3]["fused_norm"] and got[3]["filter_mfma"] == 16, got[3]
        assert np.array_equal(got[2][qs], oidx) and np.array_equal(got[0][qs], opred)
        assert np.array_equal(got[1][qs], odist.view(np.uint32))
        assert _same(got, ref)


def test_fused_query_shape_fill_rule(knn, oracle, monkeypatch):
    """knn_fused_plan's round-6 rule: 64 queries per wave (QG = 2) once its 512-query blocks,
    at most max_splits pieces per query tile (the candidate lists' capacity), fill 80 % of the
    CUs -- below that, 32 per wave.  Both sizes give the oracle's top-k and predictions on a
    sample (main.cpp:40-82) and, on every query, the same results as the forced other shape;
    knn_last_stats()[10] reports the shape."""
    import math
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    nt, d, k = 200_000 + 13, 128, 10

    def max_pieces():  # knn_capi.cpp max_splits, cap = 64 * KNN_RESCORE_CAPW (32)
        best, cap = 1, 64 * 32
        for s in range(2, 9):
            e = k * (1.0 + math.log(max(nt / s / k, 1.0))) + 64.0
            if 1.5 * (0.5 * e + 32.0) > cap // s // 2:
                break
            best = s
        return best

    tiles_needed = -(-4 * cus // (5 * max_pieces()))  # query tiles of 512 for an 80 % fill
    for nq in (max(512 * (tiles_needed - 8), 1_000) + 7, 512 * (tiles_needed + 4) + 7):
        want = 64 if (nq + 511) // 512 * max_pieces() * 5 >= 4 * cus or nq >= 384 * cus else 32
        train, labels, test = _rows(knn, nt, nq, d, 37, "f32")
        trf, lab, tef = train.float().cpu().numpy(), labels.cpu().numpy(), test.float().cpu().numpy()
        qs = np.linspace(0, nq - 1, 24).astype(np.int64)
        bad, opred, odist, oidx = oracle.knn(trf, lab, tef[qs], k, 10)
        assert bad == 0
        monkeypatch.delenv("KNN_FUSED_QG", raising=False)
        c = knn.Context(0, algo="gemm_bf16")
        got = _call(c, train, labels, test, k)
        c.close()
        assert got[3]["fused_norm"] and got[3]["queries_per_wave"] == want, (nq, got[3])
        assert np.array_equal(got[2][qs], oidx) and np.array_equal(got[0][qs], opred)
        assert np.array_equal(got[1][qs], odist.view(np.uint32))
        monkeypatch.setenv("KNN_FUSED_QG", "1" if want == 64 else "2")
        c = knn.Context(0, algo="gemm_bf16")
        other = _call(c, train, labels, test, k)
        c.close()
        assert other[3]["queries_per_wave"] == 96 - want
        assert _same(got, other)


def test_device_calls_use_torch_current_stream(knn):
    """A device call with no stream argument is enqueued on torch's current stream of the
    tensor's device (_stream_arg: the raw handle), also under a `torch.cuda.stream` context, so
    it is ordered after the torch work that made its inputs; results equal the default stream's."""
    import torch
    x = torch.zeros((8, 16), device=DEV)
    # (torch's default stream is the legacy null stream, handle 0: the call then runs on the
    # context's own stream, which is a blocking stream -- ordered after null-stream work)
    assert (knn._stream_arg(None, x).value or 0) == torch.cuda.current_stream().cuda_stream
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        assert knn._stream_arg(None, x).value == s.cuda_stream
    train, labels, test = _rows(knn, 5_000, 300, 16, 41)
    c = knn.Context(0)
    try:
        ref = _call(c, train, labels, test, 5)
        with torch.cuda.stream(s):
            t2 = test * 1.0  # made on s: the call must be ordered after it
            got = _call(c, train, labels, t2, 5)
        assert _same(ref, got)
        t3 = test * 1.0  # made on the null stream, no synchronisation before the call
        assert _same(ref, _call(c, train, labels, t3, 5))
    finally:
        c.close()


@pytest.mark.parametrize("dtype,d,k", [("f32", 128, 10), ("f32", 64, 32), ("bf16", 256, 100)])
def test_small_query_sets_many_pieces(knn, oracle, dtype, d, k):
    """Round 6: a small query set gets a 2-4x candidate list per query, so the filter cuts each
    query tile into up to 16 pieces (32 candidate sub-slices in k_rescore) to fill the CUs.  The
    results equal the oracle's on a sample (main.cpp:40-82) and the exact scan's on every
    query, ties and all."""
    nt, nq = 300_000 + 29, 1_200 + 5
    train, labels, test = _rows(knn, nt, nq, d, 43, dtype)
    trf, lab, tef = train.float().cpu().numpy(), labels.cpu().numpy(), test.float().cpu().numpy()
    qs = np.linspace(0, nq - 1, 16).astype(np.int64)
    bad, opred, odist, oidx = oracle.knn(trf, lab, tef[qs], k, 10)
    assert bad == 0
    c = knn.Context(0, algo="gemm_bf16")
    got = _call(c, train, labels, test, k)
    c.close()
    assert got[3]["fused_norm"] and got[3]["fallback_queries"] == 0, got[3]
    # more pieces than a list of the base length allows (k = 100: 6 against 1)
    assert got[3]["train_segments"] > (8 if k <= 32 else 1), got[3]
    assert np.array_equal(got[2][qs], oidx) and np.array_equal(got[0][qs], opred)
    assert np.array_equal(got[1][qs], odist.view(np.uint32))
    c = knn.Context(0, algo="direct_scan")
    ref = _call(c, train, labels, test, k)
    c.close()
    assert _same(got, ref)


@pytest.mark.parametrize("nq", [1, 7, 33])
def test_few_queries_idle_waves(knn, oracle, nq):
    """A few-query call: one query tile whose other waves hold no valid query (they run only
    the block's barriers and their tile-DMA pieces) cut into up to 32 pieces; every query
    equals the oracle (main.cpp:40-82), for both query shapes."""
    import os
    nt, d, k = 100_000 + 17, 128, 10
    train, labels, test = _rows(knn, nt, nq, d, 47, "f32")
    trf, lab, tef = train.float().cpu().numpy(), labels.cpu().numpy(), test.float().cpu().numpy()
    bad, opred, odist, oidx = oracle.knn(trf, lab, tef, k, 10)
    assert bad == 0
    for qg in ("1", "2"):
        os.environ["KNN_FUSED_QG"] = qg
        try:
            c = knn.Context(0, algo="gemm_bf16")
        finally:
            del os.environ["KNN_FUSED_QG"]
        got = _call(c, train, labels, test, k)
        c.close()
        assert got[3]["fused_norm"] and got[3]["queries_per_wave"] == 32 * int(qg), got[3]
        assert np.array_equal(got[2], oidx) and np.array_equal(got[0], opred)
        assert np.array_equal(got[1], odist.view(np.uint32))
