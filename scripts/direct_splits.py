"""Study: config L (the reference's large ARFF pair, k = 5) through k_direct_tile at several
segment counts (knn_opts.train_splits), ms per call from HIP events (profile=3)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from conftest import load_pkg  # noqa: E402

knn = load_pkg()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tf, tl, _ = knn.read_arff(os.path.join(REPO, "tests", "data", "large-train.arff"))
qf, ql, _ = knn.read_arff(os.path.join(REPO, "tests", "data", "large-test.arff"))
dev = torch.device("cuda", 0)
nt, d = tf.shape
nq = qf.shape[0]
ld = (d + 3) // 4 * 4
train = torch.zeros((nt, ld), dtype=torch.float32, device=dev)
test = torch.zeros((nq, ld), dtype=torch.float32, device=dev)
train[:, :d] = torch.from_numpy(tf).to(dev)
test[:, :d] = torch.from_numpy(qf).to(dev)
labels = torch.from_numpy(tl).to(dev)
C = int(tl.max()) + 1
ref = None
for splits in (0, 4, 8, 12, 16, 24, 32):
    ctx = knn.Context(0, algo="direct", train_splits=splits, profile=3)
    pred = torch.empty(nq, dtype=torch.int32, device=dev)
    for _ in range(3):
        ctx.predict_device(train, labels, test, 5, C, pred, d=d)
    torch.cuda.synchronize()
    ms = []
    for _ in range(20):
        ctx.predict_device(train, labels, test, 5, C, pred, d=d)
        ms.append(sum(ctx.stage_times().values()))
    got = pred.cpu().numpy()
    ref = got if ref is None else ref
    print(f"splits {splits}: {np.median(ms):.4f} ms, stats segments {ctx.stats()['train_segments']}, "
          f"same predictions {bool(np.array_equal(got, ref))}", flush=True)
    ctx.close()
