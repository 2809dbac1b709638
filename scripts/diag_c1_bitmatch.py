"""Diagnostic: config C1 (4M bf16 train rows x 1M queries x 256-d, k = 100) predictions of
three paths for 64 spread queries against the oracle over the whole train set: the
train-sharded C-ABI call (knn_predict_train_sharded, one-rank RCCL communicator), the
shard top-k + merge from Python, and the plain device call (knn_predict_device).
NT / NQ environment variables shrink the problem."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_pkg  # noqa: E402
import bench  # noqa: E402

knn = load_pkg()
nt = int(os.environ.get("NT", 4_000_000))
nq = int(os.environ.get("NQ", 1_000_000))
d, k, C, seed, kind = 256, 100, 10, 3, 1
dev = torch.device("cuda", 0)
ctx = knn.Context(0, algo="auto")
train = torch.empty((nt, d), dtype=torch.bfloat16, device=dev)
labels = torch.empty(nt, dtype=torch.int32, device=dev)
test = torch.empty((nq, d), dtype=torch.bfloat16, device=dev)
ctx.generate(train, labels, 0, d, kind, seed, 0, C)
ctx.generate(test, None, 0, d, kind, seed, 1, C)
torch.cuda.synchronize()
pos = np.unique(np.linspace(0, nq - 1, 64).astype(np.int64))
res = {}
comm = knn.Comm(ctx, knn.comm_unique_id(), 1, 0)
pred = torch.empty(nq, dtype=torch.int32, device=dev)
comm.predict_train_sharded(train, labels, 0, test, k, C, pred)
torch.cuda.synchronize()
res["rccl"] = pred.cpu().numpy()[pos]
print("rccl stats", ctx.stats(), flush=True)
rec = torch.empty((nq, 3, k), dtype=torch.int32, device=dev)
ctx.shard_topk_device(train, labels, test, k, C, 0, rec)
torch.cuda.synchronize()
pred2 = torch.empty(nq, dtype=torch.int32, device=dev)
ctx.merge_vote_device(rec.view(1, nq, 3, k), k, C, pred2)
torch.cuda.synchronize()
res["topk+merge"] = pred2.cpu().numpy()[pos]
recs = rec.cpu().numpy()[pos]
# the bench's context: train-side operands cached across calls (KNN_OPT_CACHE_TRAIN_DEVICE)
cctx = knn.Context(0, algo="auto", cache_train=True)
ccomm = knn.Comm(cctx, knn.comm_unique_id(), 1, 0)
for rep in range(2):
    predc = torch.empty(nq, dtype=torch.int32, device=dev)
    ccomm.predict_train_sharded(train, labels, 0, test, k, C, predc)
    torch.cuda.synchronize()
    res[f"rccl_cached_call{rep}"] = predc.cpu().numpy()[pos]
    print("cached call", rep, cctx.stats(), flush=True)
ccomm.close()
cctx.close()
pred3 = torch.empty(nq, dtype=torch.int32, device=dev)
ctx.predict_device(train, labels, test, k, C, pred3)
torch.cuda.synchronize()
res["device"] = pred3.cpu().numpy()[pos]
print("device stats", ctx.stats(), flush=True)
for name, p in res.items():
    r = bench.oracle_bit_match(seed, kind, nt, d, k, C, pos, p)
    print(name, r["predictions_equal_oracle"], r["mismatches"], r["mismatch_rows"], flush=True)
# the first sampled query in detail: shard record list vs oracle top-k
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import Oracle  # noqa: E402
o = Oracle()
q = int(pos[1])
te1, _ = o.gen(seed, 1, q, 1, d, kind=kind, C=C)
best = []
for r0 in range(0, nt, 1 << 20):
    n = min(1 << 20, nt - r0)
    tr, tl = o.gen(seed, 0, r0, n, d, kind=kind, C=C)
    bad, _, dist, idx = o.knn(tr, tl, te1, k, C)
    best += [(int(dist.view(np.uint32)[0, i]), int(idx[0, i]) + r0, int(tl[idx[0, i]])) for i in range(k)]
best.sort()
want = best[:k]
got = list(zip(recs[1, 0].view(np.uint32).tolist(), recs[1, 1].tolist(), recs[1, 2].tolist()))
diff = [i for i in range(k) if want[i] != tuple(got[i])]
print("query", q, "first differing list positions", diff[:10], flush=True)
if diff:
    i = diff[0]
    print("want", want[i:i + 3], "got", got[i:i + 3])
