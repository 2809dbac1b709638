"""Timing study (KNN_AMD_LIB=.../build/ablate/libknn_amd_stamps.so): where a fused-filter
wave's cycles go on configs A and B -- barrier wait, step (MFMAs + fast test + DMA issue),
slow path -- from the per-wave shader-clock stamps of the KNN_STUDY_STAMPS build
(knn_fused.hip).  Prints one line per config."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from conftest import load_pkg  # noqa: E402

knn = load_pkg()
lib = knn.load_library()
lib.knn_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 8)()
dev = torch.device("cuda", 0)
# (C1s: config C1's shard shape -- 4M bf16 rows x 256-d, k = 100 -- on 65,536 queries)
# (As: A's 8-GPU share, 12,500 queries; STAMPS_CONFIGS=A,As selects)
ALL = [("A", 1_000_000, 100_000, 128, 10, 1, 0), ("As", 1_000_000, 12_500, 128, 10, 1, 0),
       ("B", 4_000_000, 1_000_000, 64, 32, 2, 0), ("C1s", 4_000_000, 65_536, 256, 100, 3, 1)]
pick = os.environ.get("STAMPS_CONFIGS")
for name, nt, nq, d, k, seed, bf in [c for c in ALL if not pick or c[0] in pick.split(",")]:
    ctx = knn.Context(0, algo="auto", profile=True)
    dt = torch.bfloat16 if bf else torch.float32
    train = torch.empty((nt, d), dtype=dt, device=dev)
    labels = torch.empty(nt, dtype=torch.int32, device=dev)
    test = torch.empty((nq, d), dtype=dt, device=dev)
    ctx.generate(train, labels, 0, d, bf, seed, 0, 10)
    ctx.generate(test, None, 0, d, bf, seed, 1, 10)
    pred = torch.empty(nq, dtype=torch.int32, device=dev)
    ctx.predict_device(train, labels, test, k, 10, pred)
    torch.cuda.synchronize()
    lib.knn_debug_stamps(buf, 1)
    ctx.predict_device(train, labels, test, k, 10, pred)
    torch.cuda.synchronize()
    st = ctx.stage_times()
    lib.knn_debug_stamps(buf, 1)
    bar, step, slow, piece, slow_tiles, tiles, waves = (int(buf[i]) for i in range(7))
    print(f"{name}: filter {st.get('gemm_filter', 0):.2f} ms; per wave-piece sums over {waves} wave-pieces: "
          f"barrier {bar / piece:.3f}, step {step / piece:.3f}, slow {slow / piece:.3f} of the piece cycles; "
          f"tiles with a slow path {slow_tiles / tiles:.3f}; slow cycles per such tile {slow / max(slow_tiles, 1):.0f}; "
          f"step cycles per tile {step / tiles:.0f}; barrier cycles per tile {bar / tiles:.0f}; "
          f"other (exchanges, piece set-up, drain) {(piece - bar - step - slow) / piece:.3f}", flush=True)
    ctx.close()
    del train, labels, test, pred
