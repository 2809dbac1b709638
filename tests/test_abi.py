"""CPU-side checks of the boundary: the C-ABI library loads and exports every symbol
include/knn_amd.h declares; host-side evaluation and the ARFF loader match the oracle and
libarff's observable behaviour.  No compute calls need a GPU here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import DATA, DATASETS, ORACLE_DIR, PKG_DIR, REPO


def header_symbols():
    with open(os.path.join(REPO, "include", "knn_amd.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(knn_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_header_symbol(knn):
    lib = knn.load_library()
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s
    assert lib.knn_version() == 3


def test_library_built_from_this_tree(knn):
    """knn_build_id() (baked in by the Makefile) equals the hash of the sources beside the
    library: the .so the tests load is the one these sources build."""
    built, tree = knn.build_id()
    assert built == tree


def test_cpp_surface_symbols_exported():
    out = subprocess.run(["nm", "-DC", "--defined-only", os.path.join(PKG_DIR, "libknn_amd.so")],
                         capture_output=True, text=True, check=True).stdout
    for sig in ["KNN(ArffData*, ArffData*, int)", "KNN(ArffData*, ArffData*, int, int, int)",
                "KNN(void*)", "computeConfusionMatrix(int*, ArffData*)",
                "computeAccuracy(int*, ArffData*)", "ArffParser::parse()",
                "ArffData::num_classes()", "ArffInstance::get(int) const",
                "ArffValue::operator float() const"]:
        assert sig in out, sig


def test_create_without_gpu_is_loud(knn):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    with pytest.raises(knn.KnnError) as e:
        knn.Context(0)
    assert e.value.status == knn.KNN_ENODEV


def test_confusion_and_accuracy_match_oracle(knn, oracle):
    rng = np.random.default_rng(1)
    pred = rng.integers(0, 7, 500).astype(np.int32)
    lab = rng.integers(0, 7, 500).astype(np.int32)
    cm = knn.computeConfusionMatrix(pred, lab, 7)
    ocm = np.zeros((7, 7), np.int32)
    oracle.lib.oracle_confusion_matrix(oracle.p(pred), oracle.p(lab), 500, 7, oracle.p(ocm))
    assert np.array_equal(cm, ocm)
    assert knn.computeAccuracy(cm, 500) == oracle.lib.oracle_accuracy(oracle.p(ocm), 7, 500)
    with pytest.raises(knn.KnnError):
        knn.computeConfusionMatrix(np.array([9], np.int32), np.array([0], np.int32), 7)


@pytest.mark.parametrize("ds", DATASETS)
@pytest.mark.parametrize("part", ["train", "test"])
def test_arff_loader_matches_oracle(knn, oracle, ds, part):
    path = f"{DATA}/{ds}-{part}.arff"
    f, lab, C = knn.read_arff(path)
    of, olab, d = oracle.read_arff(path)
    assert f.shape == of.shape
    assert np.array_equal(f.view(np.uint32), of.view(np.uint32))
    assert np.array_equal(lab, olab)
    assert C == int(olab.max()) + 1


NUMERIC_CASES = [("1.5x", True), ("0x10", True), ("+2", True), (".5", True), ("1.", True),
                 ("1e-40", True), ("-0", True), ("1e5x", True), ("1.2.3", True), ("7", True),
                 ("nan", False), ("inf", False), ("3.4e39", False), ("1e", False), ("abc", False),
                 ("-", False), (".", False), ("e5", False)]


def _write_arff(path, values):
    with open(path, "w") as f:
        f.write("@relation t\n@attribute a NUMERIC\n@attribute class NUMERIC\n@data\n")
        for v in values:
            f.write(f"{v},0\n")


@pytest.mark.parametrize("text,ok", NUMERIC_CASES)
def test_arff_numeric_rules(knn, tmp_path, text, ok):
    """istringstream>>float rules (libarff/arff_utils.h:56-63): prefix parse via strtof,
    overflow and non-numbers rejected."""
    p = str(tmp_path / "x.arff")
    _write_arff(p, [text])
    if ok:
        f, lab, C = knn.read_arff(p)
        libc = ctypes.CDLL(None)
        libc.strtof.restype = ctypes.c_float
        libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
        m = re.match(r"[+-]?(\d*\.?\d*)([eE][+-]?\d+)?", text)
        expect = np.float32(libc.strtof(m.group(0).encode(), None))
        assert f[0, 0].view(np.uint32) == expect.view(np.uint32)
    else:
        with pytest.raises(knn.KnnError):
            knn.read_arff(p)


@pytest.mark.parametrize("text,ok", NUMERIC_CASES)
def test_arff_numeric_rules_agree_with_reference(tmp_path, text, ok):
    """Same cases through the REFERENCE's own parser (oracle/_ref/ref_capture), when built."""
    exe = os.path.join(ORACLE_DIR, "_ref", "ref_capture")
    if not os.path.exists(exe):
        pytest.skip("reference capture binary not built here")
    p = str(tmp_path / "x.arff")
    _write_arff(p, [text])
    r = subprocess.run([exe, p, p, "1", str(tmp_path / "pred.txt")], capture_output=True, timeout=30)
    assert (r.returncode == 0) == ok


def test_arff_structure(knn, tmp_path):
    p = str(tmp_path / "s.arff")
    with open(p, "w") as f:
        f.write("% comment\n@RELATION r\n@Attribute x real\n@attribute y numeric\n"
                "@attribute class NUMERIC\n@DATA\n% another\n1,2,3\n4 5 6\n7,\t8,2.9\n")
    feat, lab, C = knn.read_arff(p)
    assert feat.tolist() == [[1, 2], [4, 5], [7, 8]]
    assert lab.tolist() == [3, 6, 2]  # (int)(float) truncation, main.cpp:66
    assert C == 7
    with pytest.raises(knn.KnnError):
        knn.read_arff(str(tmp_path / "missing.arff"))
    bad = str(tmp_path / "b.arff")
    with open(bad, "w") as f:
        f.write("@relation r\n@attribute x integer\n@data\n1\n")
    with pytest.raises(knn.KnnError):
        knn.read_arff(bad)


def test_cli_usage():
    exe = os.path.join(PKG_DIR, "knn_cli")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0 and r.stdout.startswith("Usage:")


def test_shard_range_rule(knn):
    # multi-thread.cpp:154-158: contiguous, remainder on the last worker
    assert [knn.shard_range(10, 3, r) for r in range(3)] == [(0, 3), (3, 6), (6, 10)]
    for n in (0, 1, 7, 100, 1718):
        for w in (1, 2, 4, 8):
            rs = [knn.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))


def test_c_shard_range_and_exchange_layout(knn):
    """knn_shard_range / knn_exchange_layout (the C ABI's train-sharded exchange plan,
    knn_comm.cpp) agree with shard_range and exchange_shard_lists' all-to-all split."""
    for n in (0, 1, 7, 100, 1718, 1_000_003):
        for w in (1, 2, 3, 8):
            for r in range(w):
                assert knn.shard_range_c(n, w, r) == knn.shard_range(n, w, r)
    for nq, k, w in ((100, 10, 1), (1000, 7, 3), (5, 3, 8), (1_000_000, 100, 8)):
        spans = [knn.shard_range(nq, w, r) for r in range(w)]
        for r in range(w):
            so, sc, ro, rc = knn.exchange_layout(nq, k, w, r)
            mine = (spans[r][1] - spans[r][0]) * 3 * k
            assert list(sc) == [(b - a) * 3 * k for a, b in spans]
            assert list(so) == list(np.concatenate([[0], np.cumsum(sc)[:-1]]))
            assert list(rc) == [mine] * w and list(ro) == [b * mine for b in range(w)]
    with pytest.raises(knn.KnnError):
        knn.exchange_layout(10, 0, 2, 0)
    with pytest.raises(knn.KnnError):
        knn.shard_range_c(10, 2, 2)


def test_shard_policy_rule(knn):
    """knn_shard_policy (north_star "Partitioning"): test-sharded while train and its bf16 filter
    operands fit half of one GPU's HBM, train-sharded beyond; one GPU is always test-sharded."""
    G = 288 << 30
    assert knn.shard_policy(1_000_000, 100_000, 128, "f32", 8) == "test"      # A: 0.77 GB
    assert knn.shard_policy(4_000_000, 1_000_000, 64, "f32", 8) == "test"     # B
    assert knn.shard_policy(32_000_000, 1_000_000, 256, "bf16", 8) == "test"  # C fits (32 GB)
    assert knn.shard_policy(400_000_000, 1_000_000, 256, "bf16", 8) == "train"  # 409 GB
    assert knn.shard_policy(400_000_000, 1_000_000, 256, "bf16", 1) == "test"
    assert knn.shard_policy(32_000_000, 1_000, 256, "bf16", 8, hbm_bytes=16 << 30) == "train"
    assert knn.shard_policy(32_000_000, 1_000, 256, "bf16", 8, hbm_bytes=G) == "test"
    with pytest.raises(knn.KnnError):
        knn.shard_policy(10, 10, 0, "f32", 2)


# --- multi-threaded ingestion ------------------------------------
def _read_with_threads(knn, path, threads):
    old = os.environ.get("KNN_ARFF_THREADS")
    os.environ["KNN_ARFF_THREADS"] = str(threads)
    try:
        return knn.read_arff(path)
    except knn.KnnError as e:
        return ("error", str(e))
    finally:
        if old is None:
            del os.environ["KNN_ARFF_THREADS"]
        else:
            os.environ["KNN_ARFF_THREADS"] = old


def _same(a, b):
    if isinstance(a[0], str) or isinstance(b[0], str):
        return isinstance(a[0], str) and isinstance(b[0], str) and a == b
    return (a[0].view(np.uint32).tobytes() == b[0].view(np.uint32).tobytes()
            and np.array_equal(a[1], b[1]) and a[2] == b[2])


@pytest.mark.parametrize("ds", ["small", "medium", "large"])
def test_parallel_ingestion_matches_serial_on_datasets(knn, ds):
    for part in ("train", "test"):
        path = f"{DATA}/{ds}-{part}.arff"
        serial = _read_with_threads(knn, path, 1)
        for t in (2, 3, 7, 16):
            assert _same(_read_with_threads(knn, path, t), serial), (ds, part, t)


@pytest.mark.parametrize("body", [
    "1,2,0\n3.5,4e2,1\n",                 # plain
    "1,2,0\r\n3,4,1\r\n",                 # CRLF: '\r' stays in the token (libarff)
    "1 2 0 3 4 1\n5 6",                   # whitespace separators, partial last instance
    "1.5x,2,0\n+3,-.5,1\n",               # istream prefix rules
    "1,2,0\n3,,4,1\n",                    # ',,' -> libarff stops at the empty token
    "1,2,0\n 3 , 4,1\n",                  # ' ,' -> empty token
    "1,?,0\n3,4,1\n",                     # missing value
    "1,2,0\n% comment\n3,4,1\n",          # comment line
    "1,2,0\n3,'4',1\n",                   # quoted numeric field
    "1,2,0\n3,abc,1\n",                   # non-numeric field -> error
    "1,2,0\n3,real,1\n",                  # keyword token in data -> error
    "1e40,2,0\n3,4,1\n",                  # overflow -> error
    "\n\n1,2,0\n\n3,4,1",                 # blank lines, no final newline
])
def test_parallel_ingestion_matches_serial_on_edge_cases(knn, tmp_path, body):
    head = "@relation r\n@attribute a numeric\n@attribute b numeric\n@attribute class numeric\n@data\n"
    p = tmp_path / "x.arff"
    p.write_text(head + body * 40)
    serial = _read_with_threads(knn, str(p), 1)
    for t in (2, 5, 16):
        assert _same(_read_with_threads(knn, str(p), t), serial), t


def test_parallel_ingestion_large_synthetic(knn, oracle, tmp_path):
    """A 20k x 33 synthetic file in %.9g (round-trips bit-exactly through strtof)."""
    f, lab = oracle.gen(9, 0, 0, 20000, 32)
    p = tmp_path / "big.arff"
    with open(p, "w") as fh:
        fh.write("@relation big\n" + "".join(f"@attribute a{i} numeric\n" for i in range(32)))
        fh.write("@attribute class numeric\n@data\n")
        for r in range(len(f)):
            fh.write(",".join(f"{v:.9g}" for v in f[r]) + f",{lab[r]}\n")
    got = _read_with_threads(knn, str(p), 8)
    assert got[0].view(np.uint32).tobytes() == f.view(np.uint32).tobytes()
    assert np.array_equal(got[1], lab)
    assert _same(got, _read_with_threads(knn, str(p), 1))
