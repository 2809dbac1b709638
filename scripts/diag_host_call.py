"""Per-call time of the host-buffer entry (knn_predict: host arrays in, predictions out, the
train upload cached) on config L's ARFF pair -- the path the reference's own KNN() callers
take.  Diagnostic for DESIGN.md's config-L notes; KNN_AMD_LIB selects another build."""
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
import importlib
knn = importlib.import_module("knn-using-p_threads-and-mpi_amd")

tf, tl, _ = knn.read_arff(os.path.join(REPO, "tests/data/large-train.arff"))
qf, ql, _ = knn.read_arff(os.path.join(REPO, "tests/data/large-test.arff"))
want = np.loadtxt(os.path.join(REPO, "tests/golden/pred_large_k5.txt"), dtype=np.int32)
C = int(tl.max()) + 1
ctx = knn.Context(0, cache_train=True)
for _ in range(20):
    p = ctx.predict(tf, tl, qf, 5, C)
assert np.array_equal(p, want)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
t = time.perf_counter()
for _ in range(n):
    p = ctx.predict(tf, tl, qf, 5, C)
ms = 1e3 * (time.perf_counter() - t) / n
assert np.array_equal(p, want)
print(f"host-buffer call (L, train cached): {ms:.4f} ms per call over {n} calls; predictions equal the reference's")
ctx.close()
