"""GPU parity: the HIP path through the C ABI vs the reference's fixtures and the oracle.

Bar: bit-exact predictions, top-k train indices and top-k distance bits (the reference's
direct-form fp32 distance, main.cpp:14-23), on every device algorithm: the direct scan,
the GEMM form on the fp32 MFMA and the GEMM form on the bf16 MFMA with fp32 rows split
into bf16 hi + lo (gemm_split), and the GEMM form on the bf16 MFMA with fp32 rows rounded
to bf16 for the filter only (gemm_bf16; AUTO re-runs it as split when its candidate lists
overflow).
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import (DATA, DATASETS, KS, PKG_DIR, golden_cm, golden_manifest, golden_topk,
                      pred_sha)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs(knn):
    out = {a: knn.Context(0, algo=a) for a in ("direct", "gemm", "gemm_split", "gemm_bf16", "auto")}
    yield out
    for c in out.values():
        c.close()


@pytest.fixture(scope="module")
def arff(knn):
    return {ds: (knn.read_arff(f"{DATA}/{ds}-train.arff"), knn.read_arff(f"{DATA}/{ds}-test.arff"))
            for ds in DATASETS}


GEMM_OPERANDS = {"gemm": "f32", "gemm_split": "bf16x3 split", "gemm_bf16": "bf16 rounded"}
# feature counts whose filter rows are one of the LDS-DMA tile widths (128/256/512 B)
GEMM_DIMS = {"gemm": (32, 64, 128), "gemm_split": (32, 64, 128), "gemm_bf16": (64, 128, 256)}


@pytest.mark.parametrize("algo", ["direct", "gemm", "gemm_split", "gemm_bf16"])
@pytest.mark.parametrize("ds", DATASETS)
@pytest.mark.parametrize("k", KS)
def test_arff_golden(knn, ctxs, arff, algo, ds, k):
    (tf, tl, C), (qf, ql, Cq) = arff[ds]
    if algo != "direct":
        # zero-pad d=7/11 to the filter's 32-wide tile: the extra (0-0)^2 terms add +0 at the
        # end of the sequential sum, so distances stay bit-identical to the reference
        w = GEMM_DIMS[algo][0]
        tf = np.pad(tf, ((0, 0), (0, w - tf.shape[1])))
        qf = np.pad(qf, ((0, 0), (0, w - qf.shape[1])))
    pred, dist, idx = ctxs[algo].predict(tf, tl, qf, k, C, topk=True)
    if algo != "direct":
        st = ctxs[algo].stats()
        assert st["train_segments"] >= 1  # the MFMA filter path ran
        assert st["filter_operands"] == GEMM_OPERANDS[algo]
    assert pred_sha(pred) == golden_manifest()[f"{ds}_k{k}"]["sha256"]
    gd, gi = golden_topk(ds, k)
    assert np.array_equal(idx, gi)
    assert np.array_equal(dist.view(np.uint32), gd)
    acc, cm = golden_cm(ds, k)
    mycm = knn.computeConfusionMatrix(pred, ql, Cq)
    assert np.array_equal(mycm, cm)
    assert f"{knn.computeAccuracy(mycm, len(pred)):.4f}" == f"{acc:.4f}"


def test_query_range(ctxs, arff):
    """mpi.cpp:26 / multi-thread.cpp:37 slices == the same rows of the full run."""
    (tf, tl, C), (qf, ql, _) = arff["large"]
    full = ctxs["auto"].predict(tf, tl, qf, 5, C)
    for s, e in [(0, 1), (100, 615), (1717, 1718), (0, 1718)]:
        assert np.array_equal(ctxs["direct"].predict(tf, tl, qf, 5, C, s, e), full[s:e])


@pytest.mark.parametrize("d,k,nt,nq", [(128, 10, 20000, 300), (64, 32, 30000, 200), (100, 5, 9000, 257),
                                       (128, 1, 5000, 130), (40, 100, 12000, 64), (128, 128, 8192, 70),
                                       (32, 3, 70001, 129), (64, 100, 20000, 100), (128, 10, 64, 5),
                                       # 16 < k <= 32: the fused filter's per-half register lists
                                       (256, 17, 20000, 96), (128, 31, 30000, 128), (64, 24, 40000, 100)])
def test_synthetic_vs_oracle(knn, oracle, ctxs, d, k, nt, nq):
    tr, tl = oracle.gen(7, 0, 0, nt, d)
    te, _ = oracle.gen(7, 1, 0, nq, d)
    bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
    assert bad == 0
    for algo in ("direct", "gemm", "gemm_split", "gemm_bf16"):
        pred, dist, idx = ctxs[algo].predict(tr, tl, te, k, 10, topk=True)
        if algo != "direct" and d in GEMM_DIMS[algo]:
            st = ctxs[algo].stats()
            assert st["train_segments"] >= 1 and st["filter_operands"] == GEMM_OPERANDS[algo]
        assert np.array_equal(idx, oidx), algo
        assert np.array_equal(dist.view(np.uint32), odist.view(np.uint32)), algo
        assert np.array_equal(pred, opred), algo


def test_gemm_duplicates_and_ties(knn, oracle, ctxs):
    """Heavy exact ties (as in large-train: rows repeated up to 56x) through the GEMM path."""
    rng = np.random.default_rng(3)
    base = rng.integers(-3, 4, size=(50, 64)).astype(np.float32)
    tr = base[rng.integers(0, 50, size=12000)]
    tl = rng.integers(0, 10, size=12000).astype(np.int32)
    te = base[rng.integers(0, 50, size=100)] + 0.5 * rng.integers(0, 2, size=(100, 64)).astype(np.float32)
    for k in (1, 7, 64):
        bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
        for algo in ("gemm", "gemm_split", "gemm_bf16"):
            pred, dist, idx = ctxs[algo].predict(tr, tl, te, k, 10, topk=True)
            assert ctxs[algo].stats()["train_segments"] >= 1
            assert np.array_equal(idx, oidx) and np.array_equal(pred, opred)


@pytest.mark.parametrize("su", [64, 128])
def test_rescore_small_staging(knn, oracle, monkeypatch, su):
    """k_rescore stages about twice the expected candidates per query in LDS; longer lists
    re-read the rest from the candidate arrays in every bisection round, and more survivors
    than the staging holds send the query to the exact scan.  KNN_RESCORE_SU (test hook)
    shrinks the staging so both paths run on most queries: results stay bit-identical."""
    monkeypatch.setenv("KNN_RESCORE_SU", str(su))
    for d, k, nt, nq in ((128, 10, 20000, 300), (64, 32, 30000, 200), (128, 100, 9000, 70)):
        tr, tl = oracle.gen(17, 0, 0, nt, d)
        te, _ = oracle.gen(17, 1, 0, nq, d)
        tr[1::5] = tr[0]  # exact ties: long candidate lists, many survivors
        bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
        assert bad == 0
        for algo in ("gemm", "gemm_bf16", "auto"):
            ctx = knn.Context(0, algo=algo)
            try:
                pred, dist, idx = ctx.predict(tr, tl, te, k, 10, topk=True)
            finally:
                ctx.close()
            assert np.array_equal(idx, oidx), (algo, d, k)
            assert np.array_equal(dist.view(np.uint32), odist.view(np.uint32)), (algo, d, k)
            assert np.array_equal(pred, opred), (algo, d, k)


@pytest.mark.parametrize("algo", ["gemm_split", "gemm_bf16"])
@pytest.mark.parametrize("case", ["near_ties", "wide_range", "subnormal", "large"])
def test_split_operands_stress(knn, oracle, ctxs, case, algo):
    """Inputs where a bf16 rounding of the rows alone would reorder neighbours: the split
    filter's certificate (hi.hi + hi.lo + lo.hi) must still keep every true
    neighbour, so results stay bit-identical to the reference's fp32 direct form."""
    rng = np.random.default_rng({"near_ties": 11, "wide_range": 12, "subnormal": 13, "large": 14}[case])
    nt, nq, d = 20000, 96, 64
    if case == "near_ties":
        # all rows within a few fp32 ulps of 1: every distance differs only below bf16 precision
        base = np.ones((1, d), np.float32)
        tr = base + rng.integers(-64, 65, size=(nt, d)).astype(np.float32) * np.float32(2.0 ** -23)
        te = base + rng.integers(-64, 65, size=(nq, d)).astype(np.float32) * np.float32(2.0 ** -23)
    elif case == "wide_range":
        sc = np.float32(2.0) ** rng.integers(-40, 20, size=(1, d)).astype(np.float32)
        tr = (rng.standard_normal((nt, d)).astype(np.float32) * sc).astype(np.float32)
        te = (rng.standard_normal((nq, d)).astype(np.float32) * sc).astype(np.float32)
    elif case == "subnormal":
        tr = (rng.standard_normal((nt, d)) * 2.0 ** -135).astype(np.float32)
        te = (rng.standard_normal((nq, d)) * 2.0 ** -135).astype(np.float32)
        # half the columns normal (squares ~2^-120), half subnormal (2^-135)
        tr[:, : d // 2] *= np.float32(2.0 ** 75)
        te[:, : d // 2] *= np.float32(2.0 ** 75)
    else:
        tr = (rng.standard_normal((nt, d)) * 2.0 ** 55).astype(np.float32)
        te = (rng.standard_normal((nq, d)) * 2.0 ** 55).astype(np.float32)
    tl = rng.integers(0, 10, size=nt).astype(np.int32)
    for k in (1, 10, 33):
        bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
        if bad:
            continue
        pred, dist, idx = ctxs[algo].predict(tr, tl, te, k, 10, topk=True)
        assert ctxs[algo].stats()["filter_operands"] == GEMM_OPERANDS[algo]
        assert np.array_equal(idx, oidx), (case, k)
        assert np.array_equal(dist.view(np.uint32), odist.view(np.uint32)), (case, k)
        assert np.array_equal(pred, opred), (case, k)


@pytest.mark.parametrize("d", [64, 128, 256])
def test_rounded_filter_aligned_rounding(knn, oracle, ctxs, d):
    """The worst case of the rounded filter's operand-rounding term (DESIGN.md
    "Certificate"): every element sits just below a bf16 rounding midpoint, so every
    rounding error has the same sign and q.(t - rt) reaches the Cauchy-Schwarz bound
    |q| |t - rt| the certificate charges -- while the coarse bf16 grid under the elements
    keeps the distances spread, so the band (not an overflow) decides which rows are kept.
    Every true neighbour must survive: results bit-identical to the oracle."""
    rng = np.random.default_rng(31 + d)
    nt, nq = 20000, 96

    def rows(n):
        s = 2.0 ** rng.integers(0, 4, size=(n, d))                # binades [1, 16): spread distances
        m = 1.0 + rng.integers(0, 128, size=(n, d)) / 128.0      # bf16-exact grid in [1, 2)
        delta = rng.integers(1, 64, size=(n, d)) * 2.0 ** -22     # stay below the midpoint
        return ((m + 2.0 ** -8 - delta) * s).astype(np.float32)   # rounds down to m s

    tr, te = rows(nt), rows(nq)
    tl = rng.integers(0, 10, size=nt).astype(np.int32)
    for k in (1, 10, 33):
        bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
        assert bad == 0
        pred, dist, idx = ctxs["gemm_bf16"].predict(tr, tl, te, k, 10, topk=True)
        st = ctxs["gemm_bf16"].stats()
        assert st["filter_operands"] == GEMM_OPERANDS["gemm_bf16"] and st["fused_norm"], st
        assert st["fallback_queries"] < nq // 4, st  # the band, not the fallback, decides
        assert np.array_equal(idx, oidx), (d, k)
        assert np.array_equal(dist.view(np.uint32), odist.view(np.uint32)), (d, k)
        assert np.array_equal(pred, opred), (d, k)


@pytest.mark.parametrize("case", ["near_ties", "uniform"])
def test_auto_rounded_filter_rerun(knn, oracle, ctxs, case):
    """AUTO on fp32 data runs the rounded bf16 filter; when its wider certificate overflows
    more than 1/16 of the candidate lists (rows within a few ulps of 1: every row passes)
    the call is re-run with the split filter.  Either way the results are the exact
    direct-form scan's (GPU direct path, itself checked against the oracle above)."""
    rng = np.random.default_rng(21)
    nt, nq, d = 160000, 6400, 64  # nt * nq >= 1e9: AUTO takes the GEMM path
    if case == "near_ties":
        tr = 1 + rng.integers(-64, 65, size=(nt, d)).astype(np.float32) * np.float32(2.0 ** -23)
        te = 1 + rng.integers(-64, 65, size=(nq, d)).astype(np.float32) * np.float32(2.0 ** -23)
        tr, te = tr.astype(np.float32), te.astype(np.float32)
        tl = rng.integers(0, 10, size=nt).astype(np.int32)
    else:
        tr, tl = oracle.gen(9, 0, 0, nt, d)
        te, _ = oracle.gen(9, 1, 0, nq, d)
    k = 10
    pred, dist, idx = ctxs["auto"].predict(tr, tl, te, k, 10, topk=True)
    st = ctxs["auto"].stats()
    assert st["rerun_split"] == (case == "near_ties"), st
    assert st["filter_operands"] == ("bf16x3 split" if case == "near_ties" else "bf16 rounded"), st
    dpred, ddist, didx = ctxs["direct"].predict(tr, tl, te, k, 10, topk=True)
    assert np.array_equal(idx, didx)
    assert np.array_equal(dist.view(np.uint32), ddist.view(np.uint32))
    assert np.array_equal(pred, dpred)


@pytest.mark.parametrize("algo", ["gemm", "gemm_split", "gemm_bf16", "auto"])
def test_gemm_norm_guard(knn, oracle, ctxs, algo):
    """Rows whose squared norm reaches 2^125 are outside the GEMM certificate: the filter
    skips on the device (status bit) and every query takes the exact fallback scan --
    same results, and no host round trip inside the call."""
    rng = np.random.default_rng(51)
    nt, nq, d = 20000, 70, 64
    tr = rng.standard_normal((nt, d)).astype(np.float32)
    te = rng.standard_normal((nq, d)).astype(np.float32)
    tr[123] *= np.float32(2.0 ** 62)  # ||t||^2 ~ 2^130
    tl = rng.integers(0, 10, size=nt).astype(np.int32)
    if algo == "auto":
        tr = np.tile(tr, (3, 1))[: 3 * nt]   # nt * nq >= 1e9 is not needed: AUTO picks by size,
        tl = np.tile(tl, 3)                 # so force the GEMM path through the filter algos
    for k in (1, 10):
        bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
        assert bad == 0
        pred, dist, idx = ctxs[algo].predict(tr, tl, te, k, 10, topk=True)
        assert np.array_equal(idx, oidx) and np.array_equal(pred, opred), (algo, k)
        assert np.array_equal(dist.view(np.uint32), odist.view(np.uint32)), (algo, k)
        if algo != "auto":
            assert ctxs[algo].stats()["fallback_queries"] == nq


def test_edge_cases(knn, ctxs):
    tr = np.arange(12, dtype=np.float32).reshape(6, 2)
    tl = np.array([0, 1, 2, 1, 0, 1], np.int32)
    te = np.array([[0.5, 1.5], [10, 11]], np.float32)
    c = ctxs["auto"]
    # k == n_train works (main.cpp accepts it)
    p = c.predict(tr, tl, te, 6, 3)
    assert list(p) == [1, 1]
    # k > n_train: the reference segfaults; the ABI reports EINVAL
    with pytest.raises(knn.KnnError) as e:
        c.predict(tr, tl, te, 7, 3)
    assert e.value.status == knn.KNN_EINVAL
    # label outside [0, C)
    with pytest.raises(knn.KnnError) as e:
        c.predict(tr, np.array([0, 1, 5, 1, 0, 1], np.int32), te, 3, 3)
    assert e.value.status == knn.KNN_EINVAL
    # non-finite distances never qualify (main.cpp:47): fewer than k finite -> ERANGE
    bad = tr.copy()
    bad[1:, 0] = np.inf
    with pytest.raises(knn.KnnError) as e:
        c.predict(bad, tl, te, 2, 3)
    assert e.value.status == knn.KNN_ERANGE
    assert list(c.predict(bad, tl, te, 1, 3)) == [0, 0]
    # empty query set
    assert c.predict(tr, tl, te[:0], 3, 3).shape == (0,)
    # rows too wide for the exact scan's LDS query row (the fallback of every path): EINVAL
    # up front, not a failed launch
    import torch
    wide = torch.zeros((70, 45000), dtype=torch.float32, device="cuda:0")
    wl = torch.zeros(70, dtype=torch.int32, device="cuda:0")
    wp = torch.empty(3, dtype=torch.int32, device="cuda:0")
    with pytest.raises(knn.KnnError) as e:
        c.predict_device(wide, wl, wide[:3], 3, 3, wp)
    assert e.value.status == knn.KNN_EINVAL and "too wide" in str(e.value)
    # k <= 0: all-zero predictions at the Python/C++ surface (reference quirk)
    assert list(knn.KNN((tr, tl), te, 0)) == [0, 0]


def test_generator_matches_oracle(knn, oracle):
    import torch
    c = knn.Context(0)
    for kind, d, ld in ((0, 128, 128), (0, 11, 16), (1, 256, 256), (2, 128, 128), (2, 11, 16), (3, 64, 64)):
        feat = torch.empty((777, ld), dtype=torch.float32, device="cuda:0")
        lab = torch.empty(777, dtype=torch.int32, device="cuda:0")
        c.generate(feat, lab, 1000, d, kind, 5, 1, 10)
        of, ol = oracle.gen(5, 1, 1000, 777, d, ld, kind)
        assert np.array_equal(feat.cpu().numpy().view(np.uint32), of.view(np.uint32))
        assert np.array_equal(lab.cpu().numpy(), ol)
    c.close()


def test_cli_large_k5():
    """The C++ drop-in (knn_cli, include/knn_arff.hpp) prints the reference's line."""
    out_file = "/tmp/knn_cli_pred_large_k5.txt"
    env = dict(os.environ, KNN_CLI_PRED_OUT=out_file)
    r = subprocess.run([os.path.join(PKG_DIR, "knn_cli"), f"{DATA}/large-train.arff",
                        f"{DATA}/large-test.arff", "5"], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    line = r.stdout.strip()
    assert line.startswith("The 5-NN classifier for 1718 test instances on 30803 train instances required ")
    assert line.endswith("ms CPU time. Accuracy was 0.9948")
    with open(out_file) as f:
        assert pred_sha([int(x) for x in f.read().split()]) == golden_manifest()["large_k5"]["sha256"]


@pytest.mark.parametrize("ds,k,workers,shard", [("large", 5, 3, "train"), ("medium", 100, 4, "train"),
                                                 ("large", 32, 2, "auto"), ("small", 3, 3, "test")])
def test_cli_shard_policies(ds, k, workers, shard):
    """knn_cli --shard=...: the C++ KNN() split over `workers` device contexts (rehearsed on one
    GPU: KNN_AMD_SHARE_GPU=1), test-sharded by the reference's rule or train-sharded (each
    worker's shard top-k, merged on worker 0 by (distance, global index)): the golden
    predictions of the reference's serial KNN either way (main.cpp:25-85)."""
    out_file = f"/tmp/knn_cli_pred_{ds}_k{k}_{shard}.txt"
    env = dict(os.environ, KNN_CLI_PRED_OUT=out_file, KNN_AMD_SHARE_GPU="1")
    r = subprocess.run([os.path.join(PKG_DIR, "knn_cli"), f"{DATA}/{ds}-train.arff", f"{DATA}/{ds}-test.arff",
                        str(k), str(workers), f"--shard={shard}"], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert "-NN classifier for" in r.stdout
    with open(out_file) as f:
        assert pred_sha([int(x) for x in f.read().split()]) == golden_manifest()[f"{ds}_k{k}"]["sha256"]


def test_full_size_config_a_sampled(knn, oracle):
    """BASELINE config A at full size (1M x 100k x 128, k=10) on device; 48 sampled queries
    checked bit-exactly against the oracle on the full train set."""
    import torch
    nt, nq, d, k = 1_000_000, 100_000, 128, 10
    c = knn.Context(0, algo="auto", profile=True)
    train = torch.empty((nt, d), dtype=torch.float32, device="cuda:0")
    labels = torch.empty(nt, dtype=torch.int32, device="cuda:0")
    test = torch.empty((nq, d), dtype=torch.float32, device="cuda:0")
    c.generate(train, labels, 0, d, 0, 1, 0, 10)
    c.generate(test, None, 0, d, 0, 1, 1, 10)
    pred = torch.empty(nq, dtype=torch.int32, device="cuda:0")
    dist = torch.empty((nq, k), dtype=torch.float32, device="cuda:0")
    idx = torch.empty((nq, k), dtype=torch.int32, device="cuda:0")
    c.predict_device(train, labels, test, k, 10, pred, dist, idx)
    st = c.stats()
    assert st["train_segments"] >= 1  # GEMM path taken
    p, dd, ii = pred.cpu().numpy(), dist.cpu().numpy(), idx.cpu().numpy()
    # size-independent properties: sorted neighbour lists, valid classes
    assert np.all(np.diff(dd.view(np.uint32).astype(np.int64), axis=1) >= 0)
    assert p.min() >= 0 and p.max() < 10
    qs = np.linspace(0, nq - 1, 48).astype(np.int64)
    tr_h = train.cpu().numpy()
    lab_h = labels.cpu().numpy()
    te_h = test.cpu().numpy()[qs]
    bad, opred, odist, oidx = oracle.knn(tr_h, lab_h, te_h, k, 10)
    assert np.array_equal(ii[qs], oidx)
    assert np.array_equal(dd[qs].view(np.uint32), odist.view(np.uint32))
    assert np.array_equal(p[qs], opred)
    c.close()


def test_confusion_matrix_device(knn, ctxs, arff):
    """computeConfusionMatrix / computeAccuracy (main.cpp:87-112) on device == the host
    version and the reference's fixtures (large k=5), plus a 1M-query random case."""
    import torch
    (tf, tl, C), (qf, ql, Cq) = arff["large"]
    c = ctxs["auto"]
    pred = c.predict(tf, tl, qf, 5, C)
    dp = torch.from_numpy(pred).to("cuda:0")
    dl = torch.from_numpy(ql).to("cuda:0")
    cm, acc = c.confusion_matrix_device(dp, dl, Cq)
    gacc, gcm = golden_cm("large", 5)
    assert np.array_equal(cm.cpu().numpy(), gcm)
    assert f"{acc:.4f}" == f"{gacc:.4f}"
    rng = np.random.default_rng(1)
    for CC in (10, 300):  # LDS-privatised and global-atomic variants
        p = rng.integers(0, CC, 1_000_000).astype(np.int32)
        t = rng.integers(0, CC, 1_000_000).astype(np.int32)
        cm, acc = c.confusion_matrix_device(torch.from_numpy(p).cuda(), torch.from_numpy(t).cuda(), CC)
        host = knn.computeConfusionMatrix(p, t, CC)
        assert np.array_equal(cm.cpu().numpy(), host)
        assert acc == knn.computeAccuracy(host, len(p))
    bad = torch.tensor([0, 1, 10], dtype=torch.int32, device="cuda:0")
    with pytest.raises(knn.KnnError) as e:
        c.confusion_matrix_device(bad, torch.zeros(3, dtype=torch.int32, device="cuda:0"), 10)
    assert e.value.status == knn.KNN_EINVAL
