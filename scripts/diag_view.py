"""Which path stalls on config C's shard 3 as a view of the 32M-row tensor?  DIAG_CASE:
direct (k_direct_tile on the view), auto (the fused filter pipeline on the view), clone (the
same pipeline on a copy of the shard), rec (own shard tensor, output into a view of a
9.6 GB record tensor at shard 3's offset)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402
from conftest import load_pkg  # noqa: E402

knn = load_pkg()
NT, D, K, C, S = 32_000_000, 256, 100, 10, 8
NQ = int(os.environ.get("DIAG_NQ", "4096"))
case = os.environ.get("DIAG_CASE", "auto")
r = int(os.environ.get("DIAG_SHARD", "3"))
dev = "cuda:0"
a, b = knn.shard_range(NT, S, r)
ctx = knn.Context(0, algo="direct" if case == "direct" else "auto", profile=2)
test = torch.empty((NQ, D), dtype=torch.bfloat16, device=dev)
ctx.generate(test, None, 0, D, 1, 3, 1, C)
if case == "rec":
    train = torch.empty((b - a, D), dtype=torch.bfloat16, device=dev)
    labels = torch.empty(b - a, dtype=torch.int32, device=dev)
    ctx.generate(train, labels, a, D, 1, 3, 0, C)
    big = torch.empty((S, NQ, 3, K), dtype=torch.int32, device=dev)
    rec = big[r]
else:
    full = torch.empty((NT, D), dtype=torch.bfloat16, device=dev)
    flab = torch.empty(NT, dtype=torch.int32, device=dev)
    ctx.generate(full[a:b], flab[a:b], a, D, 1, 3, 0, C)
    train, labels = full[a:b], flab[a:b]
    if case == "clone":
        train, labels = train.clone(), labels.clone()
    rec = torch.empty((NQ, 3, K), dtype=torch.int32, device=dev)
print(f"case {case}: train at {train.data_ptr():#x} (+{train.data_ptr() - (full.data_ptr() if case in ('auto', 'direct') else train.data_ptr()):#x}), "
      f"rec at {rec.data_ptr():#x}", flush=True)
t = time.time()
ctx.shard_topk_device(train, labels, test, K, C, a, rec)
print(f"case {case}: {time.time() - t:.2f} s {ctx.stats()} {ctx.stage_times()}", flush=True)
