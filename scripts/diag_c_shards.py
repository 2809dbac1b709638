"""Diagnostic: config C's eight 4M-row shards (32M x 256 bf16, k = 100) against the first
NQ queries, one shard at a time: stage times, candidates and fallback queries per shard."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402
from conftest import load_pkg  # noqa: E402

NQ = int(os.environ.get("DIAG_NQ", "65536"))
knn = load_pkg()
stop = False


def beat():
    t0 = time.time()
    while not stop:
        time.sleep(20)
        print(f"  ... {time.time() - t0:.0f} s", flush=True)


threading.Thread(target=beat, daemon=True).start()
ctx = knn.Context(0, algo="auto", profile=2)
NT, D, K, C, S = 32_000_000, 256, 100, 10, 8
test = torch.empty((NQ, D), dtype=torch.bfloat16, device="cuda:0")
ctx.generate(test, None, 0, D, 1, 3, 1, C)
for r in [int(x) for x in os.environ.get("DIAG_SHARDS", "3,0,1,2,4,5,6,7").split(",")]:
    a, b = knn.shard_range(NT, S, r)
    train = torch.empty((b - a, D), dtype=torch.bfloat16, device="cuda:0")
    labels = torch.empty(b - a, dtype=torch.int32, device="cuda:0")
    ctx.generate(train, labels, a, D, 1, 3, 0, C)
    rec = torch.empty((NQ, 3, K), dtype=torch.int32, device="cuda:0")
    t = time.time()
    ctx.shard_topk_device(train, labels, test, K, C, a, rec)
    st = ctx.stats()
    print(f"shard {r}: {time.time() - t:.2f} s, stats {st}, stages "
          f"{ {n: round(v, 2) for n, v in ctx.stage_times().items()} }", flush=True)
    del train, labels, rec
stop = True
