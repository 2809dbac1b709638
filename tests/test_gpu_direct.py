"""GPU parity of the tiled direct-form kernel (k_direct_tile, KNN_ALGO_DIRECT) and of the
table-free vote (num_classes above the per-wave LDS table, KNN_VOTE_LDS_MAX_C).

Bar: bit-exact predictions, top-k indices and top-k distance bits against the oracle
(oracle/knn_oracle.c, itself pinned to the reference's fixtures), i.e. the reference's
sequential unfused fp32 distance (main.cpp:14-23), its strict-'<' insertion queue
(main.cpp:45-61) and its smallest-label vote (main.cpp:64-78).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(ctx, oracle, tr, tl, te, k, C, feats=None):
    """Run ctx on (tr, tl, te) and compare with the oracle on the fp32 values `feats`
    (the widened bf16 values for bf16 inputs)."""
    ftr, fte = feats if feats is not None else (tr, te)
    bad, opred, odist, oidx = oracle.knn(ftr, tl, fte, k, C)
    assert bad == 0
    pred, dist, idx = ctx.predict(tr, tl, te, k, C, topk=True)
    assert np.array_equal(idx, oidx)
    assert np.array_equal(dist.view(np.uint32), odist.view(np.uint32))
    assert np.array_equal(pred, opred)
    return ctx.stats()


# (d, k, nt, nq): d not a multiple of 4, rows staged in several 128-dim chunks, every list
# register count (k <= 64 .. 1024: 8, 4, 2, 1, 1 queries per wave), ragged query counts
DIRECT_CASES = [(7, 3, 5000, 300), (13, 10, 20000, 257), (129, 7, 6000, 130), (300, 10, 4000, 65),
                (64, 100, 8000, 70), (32, 300, 5000, 50), (16, 1024, 3000, 20), (128, 1, 9000, 1),
                (5, 4, 3, 17)]


@pytest.mark.parametrize("d,k,nt,nq", DIRECT_CASES)
def test_direct_tile_vs_oracle(knn, oracle, d, k, nt, nq):
    tr, tl = oracle.gen(17, 0, 0, nt, d)
    te, _ = oracle.gen(17, 1, 0, nq, d)
    if k > nt:
        k = nt
    ctx = knn.Context(0, algo="direct")
    try:
        _check(ctx, oracle, tr, tl, te, k, 10)
    finally:
        ctx.close()


@pytest.mark.parametrize("splits", [1, 3, 7, 32])
def test_direct_tile_segments(knn, oracle, splits):
    """Forced train segments: per-segment exact top-k records merged by k_merge_vote (the
    lower-index tie rule must survive the merge: duplicated rows straddle segments)."""
    tr, tl = oracle.gen(19, 0, 0, 20000, 40)
    te, _ = oracle.gen(19, 1, 0, 300, 40)
    tr[5000:10000] = tr[:5000]      # exact duplicates in other segments
    tr[15000:20000] = tr[:5000]
    ctx = knn.Context(0, algo="direct", train_splits=splits)
    try:
        for k in (1, 10, 64, 65):
            st = _check(ctx, oracle, tr, tl, te, k, 10)
            assert st["train_segments"] == splits
    finally:
        ctx.close()


def test_direct_tile_bf16(knn, oracle):
    tr, tl = oracle.gen(23, 0, 0, 12000, 256, kind=1)
    te, _ = oracle.gen(23, 1, 0, 200, 256, kind=1)
    btr, bte = knn.to_bf16_bits(tr), knn.to_bf16_bits(te)
    ctx = knn.Context(0, algo="direct")
    try:
        for k in (5, 100):
            _check(ctx, oracle, btr, tl, bte, k, 10, feats=(tr, te))
    finally:
        ctx.close()


@pytest.mark.parametrize("case", ["subnormal", "wide_range", "ties"])
def test_direct_tile_numerics(knn, oracle, case):
    """Subnormal differences and squares (fp32 denormals preserved), huge dynamic range,
    and many exactly equal distances (the packed v_pk_add/mul_f32 the compiler emits must
    round every op like the reference's scalar x86 sequence)."""
    rng = np.random.default_rng({"subnormal": 31, "wide_range": 32, "ties": 33}[case])
    nt, nq, d = 9000, 90, 24
    if case == "subnormal":
        tr = (rng.standard_normal((nt, d)) * 2.0 ** -140).astype(np.float32)
        te = (rng.standard_normal((nq, d)) * 2.0 ** -140).astype(np.float32)
        tr[:, : d // 3] *= np.float32(2.0 ** 70)
        te[:, : d // 3] *= np.float32(2.0 ** 70)
    elif case == "wide_range":
        sc = np.float32(2.0) ** rng.integers(-60, 60, size=(1, d)).astype(np.float32)
        tr = (rng.standard_normal((nt, d)).astype(np.float32) * sc).astype(np.float32)
        te = (rng.standard_normal((nq, d)).astype(np.float32) * sc).astype(np.float32)
    else:
        tr = rng.integers(-2, 3, size=(nt, d)).astype(np.float32)
        te = rng.integers(-2, 3, size=(nq, d)).astype(np.float32)
    tl = rng.integers(0, 10, size=nt).astype(np.int32)
    ctx = knn.Context(0, algo="direct")
    try:
        for k in (1, 9, 40):
            bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
            if bad:
                continue
            pred, dist, idx = ctx.predict(tr, tl, te, k, 10, topk=True)
            assert np.array_equal(idx, oidx), (case, k)
            assert np.array_equal(dist.view(np.uint32), odist.view(np.uint32)), (case, k)
            assert np.array_equal(pred, opred), (case, k)
    finally:
        ctx.close()


@pytest.mark.parametrize("algo", ["direct", "direct_scan", "gemm", "gemm_bf16"])
def test_large_num_classes(knn, oracle, algo):
    """num_classes far above the LDS vote table (C = 5000 and 16384): the table-free vote
    (vote_ballot) must give the reference's argmax, smallest label on ties; the train-
    sharded merge vote is covered in test_gpu_bf16_shard."""
    tr, _ = oracle.gen(29, 0, 0, 20000, 64)
    te, _ = oracle.gen(29, 1, 0, 150, 64)
    rng = np.random.default_rng(29)
    ctx = knn.Context(0, algo=algo)
    try:
        for C in (5000, 16384):
            tl = rng.integers(0, C, size=len(tr)).astype(np.int32)
            tl[::3] = C - 1 - (np.arange(len(tl[::3])) % 7)  # frequent high labels: vote ties
            for k in (1, 12, 70):
                st = _check(ctx, oracle, tr, tl, te, k, C)
                if algo.startswith("gemm"):
                    assert st["train_segments"] >= 1
    finally:
        ctx.close()


def test_device_dataset_validation(knn):
    """Views are read with their row stride; wrong dtypes are rejected (no silent
    reinterpretation of int64 labels or float64 outputs)."""
    import torch
    dev = "cuda:0"
    ctx = knn.Context(0, algo="direct")
    try:
        g = torch.Generator().manual_seed(5)
        wide = torch.rand((3000, 48), generator=g).to(dev)
        test = torch.rand((40, 48), generator=g).to(dev)
        lab = torch.randint(0, 10, (3000,), generator=g, dtype=torch.int32).to(dev)
        pred_v = torch.empty(40, dtype=torch.int32, device=dev)
        pred_c = torch.empty(40, dtype=torch.int32, device=dev)
        # a column view x[:, :32] of a 48-wide tensor (ld = 48) == its contiguous copy
        ctx.predict_device(wide[:, :32], lab, test[:, :32], 5, 10, pred_v)
        ctx.predict_device(wide[:, :32].contiguous(), lab, test[:, :32].contiguous(), 5, 10, pred_c)
        assert torch.equal(pred_v, pred_c)
        with pytest.raises(knn.KnnError):
            ctx.predict_device(wide, lab.to(torch.int64), test, 5, 10, pred_v)
        with pytest.raises(knn.KnnError):
            ctx.predict_device(wide, lab, test, 5, 10, pred_v.to(torch.int64))
        with pytest.raises(knn.KnnError):
            ctx.predict_device(wide[:, ::2], lab, test[:, ::2], 5, 10, pred_v)
    finally:
        ctx.close()


# k_direct_rows (d <= 16, k <= 16): every feature-group count NG = 1..4 with every remainder,
# ragged query counts (query groups of 4), train sets shorter than a tile, forced segments
ROWS_CASES = [(1, 1, 700, 9), (2, 5, 3000, 33), (3, 16, 5000, 7), (4, 2, 63, 5), (5, 3, 65, 13),
              (6, 7, 9000, 64), (7, 16, 2000, 3), (8, 4, 4100, 101), (9, 9, 130, 40), (10, 1, 8000, 1),
              (11, 5, 30803 // 4, 1718 // 8), (12, 12, 6000, 66), (13, 6, 129, 17), (14, 15, 7000, 50),
              (15, 8, 3333, 31), (16, 16, 16, 4)]


@pytest.mark.parametrize("d,k,nt,nq", ROWS_CASES)
def test_direct_rows_vs_oracle(knn, oracle, d, k, nt, nq):
    """k_direct_rows: per-lane row loads, packed fp32 query pairs (v_pk_add/mul_f32), the sorted
    first tile and the lane-shift inserts give the oracle's top-k bits and predictions."""
    tr, tl = oracle.gen(41 + d, 0, 0, nt, d)
    te, _ = oracle.gen(41 + d, 1, 0, nq, d)
    ctx = knn.Context(0, algo="direct")
    try:
        _check(ctx, oracle, tr, tl, te, min(k, nt), 10)
    finally:
        ctx.close()


@pytest.mark.parametrize("splits", [1, 3, 17])
def test_direct_rows_segments_ties_bf16(knn, oracle, splits):
    """Forced segments with exact duplicates straddling them (the lower-index tie rule through
    k_merge_vote), integer-valued features (many equal distances), bf16 rows, subnormal
    differences, and a class count above the LDS vote table (table-free ballot vote)."""
    rng = np.random.default_rng(splits)
    nt, nq, d = 12000, 70, 11
    tr = rng.integers(-2, 3, size=(nt, d)).astype(np.float32)
    tr[4000:8000] = tr[:4000]
    te = rng.integers(-2, 3, size=(nq, d)).astype(np.float32)
    tl = rng.integers(0, 10, size=nt).astype(np.int32)
    ctx = knn.Context(0, algo="direct", train_splits=splits)
    try:
        for k in (1, 5, 16):
            st = _check(ctx, oracle, tr, tl, te, k, 10)
            assert st["train_segments"] == splits
        sub_tr = (rng.standard_normal((nt, d)) * 2.0 ** -140).astype(np.float32)
        sub_te = (rng.standard_normal((nq, d)) * 2.0 ** -140).astype(np.float32)
        _check(ctx, oracle, sub_tr, tl, sub_te, 7, 10)
        big = rng.integers(0, 3000, size=nt).astype(np.int32)
        _check(ctx, oracle, tr, big, te, 9, 3000)
        btr, bl = oracle.gen(47, 0, 0, nt, 16, kind=1)
        bte, _ = oracle.gen(47, 1, 0, nq, 16, kind=1)
        _check(ctx, oracle, knn.to_bf16_bits(btr), bl, knn.to_bf16_bits(bte), 10, 10, feats=(btr, bte))
    finally:
        ctx.close()


@pytest.mark.parametrize("splits", [0, 1, 5])
def test_direct_rows_descending_distance(knn, oracle, splits):
    """Train rows in DEcreasing distance from every query (rows scaled toward the queries'
    centre): every row of every tile passes the running k-th distance, so each tile takes
    k_direct_rows' many-pass guard (one bitonic merge instead of up to 64 serial lane shifts,
    ADVICE r5).  Bit-exact against the oracle; duplicates keep the lower index."""
    rng = np.random.default_rng(77 + splits)
    nt, nq, d = 9000, 40, 11
    v = rng.standard_normal((nt, d)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    tr = (v * np.linspace(50.0, 1.0, nt, dtype=np.float32)[:, None]).astype(np.float32)
    tr[6000:6500] = tr[5500:6000]  # equal distances at different indices
    te = (rng.standard_normal((nq, d)) * 0.01).astype(np.float32)
    tl = rng.integers(0, 10, size=nt).astype(np.int32)
    ctx = knn.Context(0, algo="direct", train_splits=splits)
    try:
        for k in (1, 5, 16):
            _check(ctx, oracle, tr, tl, te, k, 10)
    finally:
        ctx.close()
