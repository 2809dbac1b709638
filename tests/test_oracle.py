"""Pin the CPU oracle against the reference's golden fixtures (no GPU needed).

The fixtures in tests/golden/ were captured from the reference itself
(oracle/ref_capture.cpp around /root/reference/main.cpp; tests/golden/make_golden.py).
"""
import json
import os

import numpy as np
import pytest

from conftest import (ORACLE_DIR, DATA, DATASETS, KS, golden_cm, golden_manifest, golden_pred, golden_topk,
                      pred_sha)

SURVEY_SHA = {  # SURVEY.md 8c, captured independently by the survey
    ("small", 1): "4bdb894a6ac2a3cf3dd63fc6e4895afa5ce7229542f8ce6933cbd4938621ba34",
    ("small", 3): "4bdb894a6ac2a3cf3dd63fc6e4895afa5ce7229542f8ce6933cbd4938621ba34",
    ("small", 5): "ba5cccdce3e49a58687bccbd54330ac778f052174f963c35f0b349d34741836b",
    ("medium", 1): "8ae4dfa098c94417a0fdff2381552bcb7cedb28c44091c99b39e93a953b694b8",
    ("medium", 3): "c1498c4261e1cb6f4f846e35165c96d7a3852779cd368b6894b51a94aaa708ed",
    ("medium", 5): "02698225cb205c8514bd99391eae92178d8008d3002e46a18de9ffc56df185b4",
    ("large", 1): "64d8b3c6003641ec2467d99887a35a4fd21994499b43ecf994a85f44669a4eae",
    ("large", 3): "fce352df8a4e2d2ed87c4b6ae5fd5dd76290652808dcd38a2e77e3b6318eb4da",
    ("large", 5): "fce352df8a4e2d2ed87c4b6ae5fd5dd76290652808dcd38a2e77e3b6318eb4da",
    ("large", 10): "31ec143cec2c4a4981931f16b59cb30f303a5a6e9859d8e34bf997aec5073274",
    ("large", 32): "d909b4be6eb48f78c2a826f3f633bf7c60556394562580626fb20e3dd1896eb3",
    ("large", 100): "25f15e3c9ce04d7b31da5b3aee4e486e6f0bfa5ba96003f5a7a885c5c56b8102",
}


def test_manifest_matches_survey():
    man = golden_manifest()
    for (ds, k), sha in SURVEY_SHA.items():
        assert man[f"{ds}_k{k}"]["sha256"] == sha
    for key, ent in man.items():
        assert pred_sha(golden_pred(ent["dataset"], ent["k"])) == ent["sha256"]


@pytest.fixture(scope="module")
def arff(oracle):
    out = {}
    for ds in DATASETS:
        tr, tl, d = oracle.read_arff(f"{DATA}/{ds}-train.arff")
        te, ql, _ = oracle.read_arff(f"{DATA}/{ds}-test.arff")
        out[ds] = (tr, tl, te, ql, d)
    return out


@pytest.mark.parametrize("ds", DATASETS)
@pytest.mark.parametrize("k", KS)
def test_oracle_matches_reference(oracle, arff, ds, k):
    tr, tl, te, ql, d = arff[ds]
    C = int(tl.max()) + 1
    bad, pred, dist, idx = oracle.knn(tr, tl, te, k, C)
    assert bad == 0
    assert pred_sha(pred) == golden_manifest()[f"{ds}_k{k}"]["sha256"]
    gd, gi = golden_topk(ds, k)
    assert np.array_equal(dist.view(np.uint32), gd)
    assert np.array_equal(idx, gi)
    # confusion matrix / accuracy (main.cpp:87-112)
    acc, cm = golden_cm(ds, k)
    Ct = int(ql.max()) + 1
    mycm = np.zeros((Ct, Ct), np.int32)
    oracle.lib.oracle_confusion_matrix(oracle.p(pred), oracle.p(ql), len(pred), Ct, oracle.p(mycm))
    assert np.array_equal(mycm, cm)
    assert f"{oracle.lib.oracle_accuracy(oracle.p(mycm), Ct, len(pred)):.4f}" == f"{acc:.4f}"


def test_oracle_topk_is_stable_sort(oracle):
    """Restatement check: insertion queue == first k of a stable sort by distance."""
    rng = np.random.default_rng(0)
    tr = rng.integers(0, 4, size=(300, 3)).astype(np.float32)  # many exact ties
    te = rng.integers(0, 4, size=(20, 3)).astype(np.float32)
    lab = rng.integers(0, 5, size=300).astype(np.int32)
    k = 17
    bad, pred, dist, idx = oracle.knn(tr, lab, te, k, 5)
    assert bad == 0
    for q in range(len(te)):
        qrow = np.ascontiguousarray(te[q])
        dd = np.array([oracle.lib.oracle_distance(oracle.p(qrow), oracle.p(tr[t]), 3)
                       for t in range(len(tr))], np.float32)
        order = np.argsort(dd, kind="stable")[:k]
        assert np.array_equal(idx[q], order)
        counts = np.bincount(lab[order], minlength=5)
        assert pred[q] == int(np.argmax(counts))  # argmax: first max == smallest label


def test_oracle_generator_values(oracle):
    f, lab = oracle.gen(1, 0, 0, 64, 128)
    assert f.min() >= -1.0 and f.max() < 1.0
    # every value is on the 2^-23 grid
    assert np.all((f.astype(np.float64) * 2 ** 23) == np.round(f.astype(np.float64) * 2 ** 23))
    assert set(np.unique(lab)) <= set(range(10))
    f2, _ = oracle.gen(1, 0, 32, 32, 128)
    assert np.array_equal(f[32:], f2)  # counter-based: rows are independent of the block
    fb, _ = oracle.gen(3, 0, 0, 16, 256, kind=1)
    assert np.all(fb * 128 == np.round(fb * 128)) and fb.min() >= -1 and fb.max() < 1


def test_oracle_clustered_generator(oracle):
    """SURVEY.md 8d's clustered variant (kinds 2 / 3): value = the row's class centroid +
    noise, exact on its grid, rows independent of the block, and labels that carry signal."""
    f, lab = oracle.gen(4, 0, 0, 400, 64, kind=2)
    g = f.astype(np.float64) * 2 ** 24  # centroid (2^-23 grid) + half a grid value: 2^-24 grid
    assert np.all(g == np.round(g)) and np.abs(f).max() < 1.5
    f2, _ = oracle.gen(4, 0, 200, 200, 64, kind=2)
    assert np.array_equal(f[200:], f2)
    t, tl = oracle.gen(4, 1, 0, 50, 64, kind=2)  # test rows: same centroids, their own noise
    _, pred, _, _ = oracle.knn(f, lab, t, 3, 10)
    assert np.mean(pred == tl) > 0.9  # uniform data gives ~0.1
    fb, lb = oracle.gen(5, 0, 0, 300, 32, kind=3)
    assert np.all(fb * 128 == np.round(fb * 128)) and np.abs(fb * 128).max() <= 160
    # bf16-exact: the top 16 bits hold the whole value
    assert np.array_equal(fb.view(np.uint32) & 0xFFFF, np.zeros_like(fb.view(np.uint32)))
    # kinds 0 / 1 unchanged by the class count
    assert np.array_equal(oracle.gen(1, 0, 0, 8, 16, kind=0, C=3)[0], oracle.gen(1, 0, 0, 8, 16, kind=0, C=10)[0])


def test_oracle_k_above_n_flags(oracle):
    tr = np.zeros((3, 2), np.float32)
    bad, *_ = oracle.knn(tr, np.zeros(3, np.int32), tr, 4, 1)
    assert bad == 1


# --- the reference's MPI path (cpu_baseline "mpi" leg) ----------------------------------
def _ref_mpi(name):
    p = os.path.join(ORACLE_DIR, "_ref", name)
    if not (os.path.exists(p) and os.path.exists("/opt/conda/bin/mpiexec")):
        pytest.skip("reference MPI build absent")
    return p


def test_reference_mpi_bench_matches_pthreads_and_oracle(oracle, tmp_path):
    """ref_bench_mpi (mpi.cpp's KNN + Scatter/Gatherv under mpiexec) and ref_bench
    (multi-thread.cpp's KNN) give the oracle's predictions on the same generated sample."""
    import subprocess
    argv = ["0", "7", "3000", "61", "32", "5", "10"]
    r = subprocess.run(["/opt/conda/bin/mpiexec", "-n", "3", _ref_mpi("ref_bench_mpi")] + argv +
                       [str(tmp_path / "mpi.txt")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["ranks"] == 3 and rec["nq"] == 61
    r = subprocess.run([_ref_mpi("ref_bench")] + argv + ["2", str(tmp_path / "mt.txt")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    mpi = np.loadtxt(tmp_path / "mpi.txt", dtype=np.int32)
    mt = np.loadtxt(tmp_path / "mt.txt", dtype=np.int32)
    tr, tl = oracle.gen(7, 0, 0, 3000, 32)
    te, _ = oracle.gen(7, 1, 0, 61, 32)
    _, opred, _, _ = oracle.knn(tr, tl, te, 5, 10)
    assert np.array_equal(mpi, opred) and np.array_equal(mt, opred)


def test_reference_clustered_matches_oracle(oracle, tmp_path):
    """The reference's own pthreads KNN (ref_bench: multi-thread.cpp compiled from
    /root/reference) on clustered rows (kind 2, built through libarff's API) gives the oracle's
    predictions: the clustered generator's values are pinned by the reference itself."""
    import subprocess
    argv = ["2", "9", "4000", "64", "24", "7", "10"]
    r = subprocess.run([_ref_mpi("ref_bench")] + argv + ["4", str(tmp_path / "mt.txt")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    mt = np.loadtxt(tmp_path / "mt.txt", dtype=np.int32)
    tr, tl = oracle.gen(9, 0, 0, 4000, 24, kind=2)
    te, truth = oracle.gen(9, 1, 0, 64, 24, kind=2)
    _, opred, _, _ = oracle.knn(tr, tl, te, 7, 10)
    assert np.array_equal(mt, opred)
    assert np.mean(opred == truth) > 0.8


def test_reference_mpi_binary_line():
    """The reference's own mpi binary (mpi.cpp built with MPICH) on the small pair: its
    line carries the golden accuracy (the line the drop-in driver must reproduce)."""
    import re
    import subprocess
    r = subprocess.run(["/opt/conda/bin/mpiexec", "-n", "2", _ref_mpi("mpi"), f"{DATA}/small-train.arff",
                        f"{DATA}/small-test.arff", "3"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    m = re.search(r"Accuracy was (\d\.\d{4})", r.stdout)
    assert m and m.group(1) == f"{golden_manifest()['small_k3']['accuracy']:.4f}"
