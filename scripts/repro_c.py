"""Config C's eight shards exactly as tests/test_gpu_config_c.py runs them (views of one 32M-row
tensor, 1M queries), one line per shard, a heartbeat every 15 s (DIAG_ORDER sets the order)."""
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
dev = "cuda:0"
ctx = knn.Context(0, algo="auto", profile=True)
train = torch.empty((NT, D), dtype=torch.bfloat16, device=dev)
labels = torch.empty(NT, dtype=torch.int32, device=dev)
test = torch.empty((NQ, D), dtype=torch.bfloat16, device=dev)
ctx.generate(train, labels, 0, D, 1, 3, 0, C)
ctx.generate(test, None, 0, D, 1, 3, 1, C)
rec = torch.empty((S, NQ, 3, K), dtype=torch.int32, device=dev)
print("generated", flush=True)
for r in [int(x) for x in os.environ.get("DIAG_ORDER", "3,0,1,2,4,5,6,7").split(",")]:
    a, b = knn.shard_range(NT, S, r)
    t = time.time()
    ctx.shard_topk_device(train[a:b], labels[a:b], test, K, C, a, rec[r])
    print(f"shard {r}: {time.time() - t:.2f} s, {ctx.stats()}, "
          f"{ {n: round(v, 1) for n, v in ctx.stage_times().items()} }", flush=True)
stop = True
