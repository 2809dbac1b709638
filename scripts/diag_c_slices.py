"""Diagnostic: one config-C shard (DIAG_SHARD, 4M x 256 bf16, k = 100) against all 1M queries
in slices of DIAG_SLICE queries, one shard_topk call per slice: time, candidates and
fallback queries per slice (which slice stalls, if one does)."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402
from conftest import load_pkg  # noqa: E402

knn = load_pkg()
stop = False


def beat():
    t0 = time.time()
    while not stop:
        time.sleep(15)
        print(f"  ... {time.time() - t0:.0f} s", flush=True)


threading.Thread(target=beat, daemon=True).start()
NT, NQ, D, K, C, S = 32_000_000, 1_000_000, 256, 100, 10, 8
r = int(os.environ.get("DIAG_SHARD", "3"))
SL = int(os.environ.get("DIAG_SLICE", "65536"))
ctx = knn.Context(0, algo="auto", profile=2)
test = torch.empty((NQ, D), dtype=torch.bfloat16, device="cuda:0")
ctx.generate(test, None, 0, D, 1, 3, 1, C)
a, b = knn.shard_range(NT, S, r)
train = torch.empty((b - a, D), dtype=torch.bfloat16, device="cuda:0")
labels = torch.empty(b - a, dtype=torch.int32, device="cuda:0")
ctx.generate(train, labels, a, D, 1, 3, 0, C)
rec = torch.empty((NQ, 3, K), dtype=torch.int32, device="cuda:0")
for q0 in range(0, NQ, SL):
    q1 = min(NQ, q0 + SL)
    t = time.time()
    ctx.shard_topk_device(train, labels, test[q0:q1], K, C, a, rec[q0:q1])
    st = ctx.stats()
    print(f"shard {r} queries [{q0}, {q1}): {time.time() - t:.2f} s, cand/q {st['candidates'] / (q1 - q0):.0f}, "
          f"fallback {st['fallback_queries']}, stages { {n: round(v, 1) for n, v in ctx.stage_times().items()} }",
          flush=True)
stop = True
