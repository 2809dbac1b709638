"""Timing study (KNN_AMD_LIB=.../build/study/libknn_amd_<v>.so from `KERNELS=1
scripts/build_variant.sh <v> . -DKNN_STUDY_STAMPS`): where a k_rescore wave's cycles go on
configs A and B -- fill counts, record staging, bisection, compaction, survivor distances,
selection + vote -- from the per-wave shader-clock stamps (knn_kernels.hip).  One line per
config: cycles per query in each phase, survivors, record batches and bisection rounds."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from conftest import load_pkg  # noqa: E402

knn = load_pkg()
lib = knn.load_library()
lib.knn_debug_rescore_stamps_buffer.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
dev = torch.device("cuda", 0)
names = ["counts", "records", "bisection", "compaction", "distances", "select+vote"]
for name, nt, nq, d, k, seed in [("A", 1_000_000, 100_000, 128, 10, 1), ("B", 4_000_000, 1_000_000, 64, 32, 2)]:
    ctx = knn.Context(0, algo="auto", profile=True, cache_train=True)
    train = torch.empty((nt, d), dtype=torch.float32, device=dev)
    labels = torch.empty(nt, dtype=torch.int32, device=dev)
    test = torch.empty((nq, d), dtype=torch.float32, device=dev)
    ctx.generate(train, labels, 0, d, 0, seed, 0, 10)
    ctx.generate(test, None, 0, d, 0, seed, 1, 10)
    pred = torch.empty(nq, dtype=torch.int32, device=dev)
    ctx.predict_device(train, labels, test, k, 10, pred)
    torch.cuda.synchronize()
    buf = torch.zeros((nq, 10), dtype=torch.int64, device=dev)
    lib.knn_debug_rescore_stamps_buffer(buf.data_ptr(), nq)
    ctx.predict_device(train, labels, test, k, 10, pred)
    torch.cuda.synchronize()
    st = ctx.stage_times()
    lib.knn_debug_rescore_stamps_buffer(None, 0)
    v = [int(x) for x in buf.sum(0).cpu()]
    n = max(v[6], 1)
    phases = ", ".join(f"{nm} {v[i] / n:.0f}" for i, nm in enumerate(names))
    print(f"{name}: rescore {st.get('rescore', 0):.3f} ms; {v[6]} queries; cycles per query-wave (mean): {phases}; "
          f"total {sum(v[:6]) / n:.0f}; survivors {v[7] / n:.1f}, record batches {v[8] / n:.2f}, "
          f"bisection rounds {v[9] / n:.1f}", flush=True)
    ctx.close()
    del train, labels, test, pred
