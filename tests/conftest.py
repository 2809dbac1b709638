"""Shared fixtures.  The oracle (oracle/liboracle.so) is used only as the checker."""
import ctypes
import hashlib
import importlib.util
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "knn-using-p_threads-and-mpi_amd")
DATA = os.path.join(REPO, "tests", "data")
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_DIR = os.path.join(REPO, "oracle")
DATASETS = ["small", "medium", "large"]
KS = [1, 3, 5, 10, 32, 100]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu)")


def load_pkg():
    if "knn_amd" in sys.modules:
        return sys.modules["knn_amd"]
    spec = importlib.util.spec_from_file_location("knn_amd", os.path.join(PKG_DIR, "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["knn_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def knn():
    return load_pkg()


def _build_oracle():
    so = os.path.join(ORACLE_DIR, "liboracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", ORACLE_DIR, "liboracle.so"], check=True, capture_output=True)
    return so


class Oracle:
    """ctypes wrapper over the C restatement (test infrastructure only)."""

    def __init__(self):
        lib = ctypes.CDLL(_build_oracle())
        P, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        lib.oracle_knn.argtypes = [P, P, I64, P, I64, I64, I32, I64, I32, I32, P, P, P, I32]
        lib.oracle_knn.restype = I32
        lib.oracle_arff_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(I64), ctypes.POINTER(I32),
                                         I64, P, P]
        lib.oracle_arff_read.restype = I32
        lib.oracle_gen_block.argtypes = [ctypes.c_uint64, ctypes.c_uint32, I64, I64, I32, I64, I32,
                                         P, P, I32]
        lib.oracle_gen_block.restype = None
        lib.oracle_confusion_matrix.argtypes = [P, P, I64, I32, P]
        lib.oracle_accuracy.argtypes = [P, I32, I64]
        lib.oracle_accuracy.restype = ctypes.c_float
        lib.oracle_distance.argtypes = [P, P, I32]
        lib.oracle_distance.restype = ctypes.c_float
        self.lib = lib

    @staticmethod
    def p(a):
        return None if a is None else ctypes.c_void_p(a.ctypes.data)

    def read_arff(self, path, ld=None):
        n, na = ctypes.c_int64(), ctypes.c_int()
        assert self.lib.oracle_arff_read(path.encode(), ctypes.byref(n), ctypes.byref(na), 1, None, None) == 0
        d = na.value - 1
        ld = d if ld is None else ld
        f = np.zeros((n.value, ld), np.float32)
        lab = np.zeros(n.value, np.int32)
        assert self.lib.oracle_arff_read(path.encode(), ctypes.byref(n), ctypes.byref(na), ld,
                                         self.p(f), self.p(lab)) == 0
        return f, lab, d

    def knn(self, train, labels, test, k, C, d=None, q0=0, q1=None, threads=None, topk=True):
        train = np.ascontiguousarray(train, np.float32)
        test = np.ascontiguousarray(test, np.float32)
        labels = np.ascontiguousarray(labels, np.int32)
        ld = train.shape[1]
        assert test.shape[1] == ld
        d = ld if d is None else d
        q1 = len(test) if q1 is None else q1
        pred = np.zeros(len(test), np.int32)
        dist = np.zeros((len(test), k), np.float32) if topk else None
        idx = np.zeros((len(test), k), np.int32) if topk else None
        threads = threads or min(16, os.cpu_count() or 1)
        bad = self.lib.oracle_knn(self.p(train), self.p(labels), len(train), self.p(test), q0, q1, d, ld,
                                  k, C, self.p(pred), self.p(dist), self.p(idx), threads)
        sl = slice(q0, q1)
        return bad, pred[sl], (dist[sl] if topk else None), (idx[sl] if topk else None)

    def gen(self, seed, stream, row0, n, d, ld=None, kind=0, C=10):
        ld = d if ld is None else ld
        f = np.zeros((n, ld), np.float32)
        lab = np.zeros(n, np.int32)
        self.lib.oracle_gen_block(seed, stream, row0, n, d, ld, kind, self.p(f), self.p(lab), C)
        return f, lab


@pytest.fixture(scope="session")
def oracle():
    return Oracle()


def golden_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_pred(ds, k):
    with open(os.path.join(GOLDEN, f"pred_{ds}_k{k}.txt")) as f:
        return np.array([int(x) for x in f.read().split()], np.int32)


def golden_topk(ds, k):
    raw = np.fromfile(os.path.join(GOLDEN, f"topk_{ds}_k{k}.bin"), np.int32)
    nq, kk = raw[0], raw[1]
    rec = raw[2:].reshape(nq, kk, 2)
    return rec[:, :, 0].view(np.uint32).copy(), rec[:, :, 1].copy()


def golden_cm(ds, k):
    with open(os.path.join(GOLDEN, f"cm_{ds}_k{k}.txt")) as f:
        lines = f.read().strip().split("\n")
    acc = float(lines[0].split()[1])
    cm = np.array([[int(x) for x in ln.split()] for ln in lines[1:]], np.int32)
    return acc, cm


def pred_sha(pred):
    return hashlib.sha256("".join(f"{int(p)}\n" for p in pred).encode()).hexdigest()


def merge_lists_reference(rec, k, C):
    """Host restatement of k_merge_vote (test infrastructure): rec [nsrc][nq][3][k] int32
    per-shard lists (dist bits, global idx or -1, label) -> (pred, dist, idx) of the k
    smallest (dist, idx) over all shards, vote = bincount argmax (smallest label on ties,
    main.cpp:64-78)."""
    rec = np.asarray(rec)
    nsrc, nq = rec.shape[0], rec.shape[1]
    pred = np.zeros(nq, np.int32)
    dist = np.full((nq, k), np.finfo(np.float32).max, np.float32)
    idx = np.full((nq, k), -1, np.int32)
    for q in range(nq):
        r = rec[:, q]                                   # [nsrc][3][k]
        d = r[:, 0, :].reshape(-1).view(np.uint32)
        i = r[:, 1, :].reshape(-1)
        lab = r[:, 2, :].reshape(-1)
        ok = i >= 0
        d, i, lab = d[ok], i[ok], lab[ok]
        order = np.lexsort((i, d))[:k]
        n = len(order)
        dist[q, :n] = d[order].view(np.float32)
        idx[q, :n] = i[order]
        pred[q] = int(np.argmax(np.bincount(lab[order], minlength=C))) if n == k else 0
    return pred, dist, idx
