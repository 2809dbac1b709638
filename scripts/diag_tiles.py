"""Study build check (KNN_AMD_LIB=.../libknn_amd_{check,freecheck}.so): run the synthetic cases
the free schedule fails, compare with the oracle, and read the tile-integrity counters
(knn_fused.hip, KNN_FUSED_CHECK_TILES)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from conftest import Oracle, load_pkg  # noqa: E402

knn = load_pkg()
oracle = Oracle()
lib = knn.load_library()
lib.knn_debug_tile_check.argtypes = [ctypes.c_void_p, ctypes.c_int]
cnt = (ctypes.c_uint32 * 8)()
lib.knn_debug_tile_check(cnt, 1)
ctx = knn.Context(0, algo="gemm_bf16")
for d, k, nt, nq in [(128, 10, 20000, 300), (128, 1, 5000, 130), (64, 24, 40000, 100), (128, 10, 100000, 3000)]:
    tr, tl = oracle.gen(21, 0, 0, nt, d)
    te, _ = oracle.gen(21, 1, 0, nq, d)
    bad, opred, odist, oidx = oracle.knn(tr, tl, te, k, 10)
    pred, dist, idx = ctx.predict(tr, tl, te, k, 10, topk=True)
    ok = np.array_equal(idx, oidx) and np.array_equal(pred, opred)
    lib.knn_debug_tile_check(cnt, 1)
    nbad = int((idx != oidx).any(axis=1).sum())
    print(f"d={d} k={k} nt={nt} nq={nq}: equal={ok} queries_off={nbad} stats={ctx.stats()['train_segments']} "
          f"tile_mismatch={cnt[0]} checks={cnt[1]} first=(block {cnt[2]}, it {cnt[3]}, buf {cnt[4]}, slot {cnt[5]}, "
          f"wave {cnt[6]}, lane {cnt[7]})", flush=True)
