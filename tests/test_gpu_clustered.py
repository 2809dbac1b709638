"""GPU parity on the clustered synthetic rows (SURVEY.md 8d's "clustered" variant: the row's
class centroid + noise, generator kinds 2 / 3).  Uniform rows put every neighbour list far from
the query; clustered rows give close same-class neighbours, so the thresholds converge early
and the labels carry signal -- another regime for the filter's certificate and the vote.

Bar (main.cpp:40-82): every query bit-exact (indices, distance bits, prediction) against the
direct form (KNN_ALGO_DIRECT, pinned to the oracle by test_gpu_fullsize.py), and a few queries
against the C oracle itself; accuracy against the generator's labels well above 1/C.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPES = [  # (d, k, nt, nq, kind, force_qg): the fused filter's shapes A / B / C at test size
    # (nt x nq >= 1e9: AUTO's rule for the MFMA filter, knn_capi.cpp choose_algo)
    (128, 10, 250_000, 4096, 2, None),
    (128, 10, 250_000, 4096, 2, "2"),
    (64, 32, 250_000, 4096, 2, None),
    (64, 32, 250_000, 4096, 2, "2"),
    (256, 100, 200_000, 5000, 3, None),
    (128, 16, 250_000, 4096, 3, None),
]


@pytest.mark.parametrize("d,k,nt,nq,kind,qg", SHAPES)
def test_clustered_fused_vs_direct_and_oracle(knn, oracle, monkeypatch, d, k, nt, nq, kind, qg):
    import torch
    if qg:
        monkeypatch.setenv("KNN_FUSED_QG", qg)  # snapshot at knn_create: both query shapes
    dev = "cuda:0"
    C, seed = 10, 11
    tdt = torch.bfloat16 if kind == 3 else torch.float32
    auto = knn.Context(0, algo="auto")
    direct = knn.Context(0, algo="direct")
    try:
        train = torch.empty((nt, d), dtype=tdt, device=dev)
        labels = torch.empty(nt, dtype=torch.int32, device=dev)
        test = torch.empty((nq, d), dtype=tdt, device=dev)
        truth = torch.empty(nq, dtype=torch.int32, device=dev)
        auto.generate(train, labels, 0, d, kind, seed, 0, C)
        auto.generate(test, truth, 0, d, kind, seed, 1, C)
        out = {}
        for name, c in (("auto", auto), ("direct", direct)):
            p = torch.empty(nq, dtype=torch.int32, device=dev)
            dd = torch.empty((nq, k), dtype=torch.float32, device=dev)
            ii = torch.empty((nq, k), dtype=torch.int32, device=dev)
            c.predict_device(train, labels, test, k, C, p, dist=dd, idx=ii)
            torch.cuda.synchronize()
            out[name] = (p.cpu().numpy(), dd.cpu().numpy(), ii.cpu().numpy())
        st = auto.stats()
        assert st["fused_norm"], st  # the MFMA filter ran, not a fallback
        pa, da, ia = out["auto"]
        pd, dd_, id_ = out["direct"]
        assert np.array_equal(ia, id_)
        assert np.array_equal(da.view(np.uint32), dd_.view(np.uint32))
        assert np.array_equal(pa, pd)
        # a spread sample against the C oracle over the whole train set
        trf, tl = oracle.gen(seed, 0, 0, nt, d, kind=kind, C=C)
        qs = np.linspace(0, nq - 1, 6).astype(np.int64)
        tef = np.concatenate([oracle.gen(seed, 1, int(q), 1, d, kind=kind, C=C)[0] for q in qs])
        bad, op, od, oi = oracle.knn(trf, tl, tef, k, C)
        assert bad == 0
        assert np.array_equal(oi, ia[qs]) and np.array_equal(od.view(np.uint32), da[qs].view(np.uint32))
        assert np.array_equal(op, pa[qs])
        # the labels carry signal: accuracy against the generator's labels of the queries
        assert np.mean(pa == truth.cpu().numpy()) > 0.5
    finally:
        auto.close()
        direct.close()


def test_nonfinite_train_rows_at_filter_size(knn, oracle):
    """NaN / inf features in a few train rows at a size where AUTO runs the MFMA filter: such a
    row's norm fails the certificate's range check (k_row_norms: !(norm < 2^125)), the call
    takes the exact path, and -- like main.cpp:47's strict '<' -- the rows never become
    neighbours.  Every query equal to the direct form; a sample equal to the oracle."""
    import torch
    dev = "cuda:0"
    nt, nq, d, k, C = 262_144, 4096, 128, 10, 10
    auto = knn.Context(0, algo="auto")
    direct = knn.Context(0, algo="direct")
    try:
        train = torch.empty((nt, d), dtype=torch.float32, device=dev)
        labels = torch.empty(nt, dtype=torch.int32, device=dev)
        test = torch.empty((nq, d), dtype=torch.float32, device=dev)
        auto.generate(train, labels, 0, d, 2, 21, 0, C)
        auto.generate(test, None, 0, d, 2, 21, 1, C)
        train[5, 3] = float("nan")
        train[77_777, 0] = float("inf")
        train[200_000, 127] = float("-inf")
        out = {}
        for name, c in (("auto", auto), ("direct", direct)):
            p = torch.empty(nq, dtype=torch.int32, device=dev)
            dd = torch.empty((nq, k), dtype=torch.float32, device=dev)
            ii = torch.empty((nq, k), dtype=torch.int32, device=dev)
            c.predict_device(train, labels, test, k, C, p, dist=dd, idx=ii)
            torch.cuda.synchronize()
            out[name] = (p.cpu().numpy(), dd.cpu().numpy(), ii.cpu().numpy())
        pa, da, ia = out["auto"]
        pd, dd_, id_ = out["direct"]
        assert np.array_equal(ia, id_) and np.array_equal(da.view(np.uint32), dd_.view(np.uint32))
        assert np.array_equal(pa, pd)
        assert not np.isin(ia, [5, 77_777, 200_000]).any()
        qs = np.array([0, 1234, 4095])
        bad, op, od, oi = oracle.knn(train.cpu().numpy(), labels.cpu().numpy(), test.cpu().numpy()[qs], k, C)
        assert bad == 0
        assert np.array_equal(oi, ia[qs]) and np.array_equal(op, pa[qs])
    finally:
        auto.close()
        direct.close()
