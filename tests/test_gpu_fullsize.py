"""Full-size parity of BASELINE configs A and B on the device.

Every query's top-k indices, top-k distance bits and prediction from the default path
(AUTO: the rounded-bf16 MFMA filter + exact fp32 rescore, with the train segments, slice
sizes and block shape the plan picks at these sizes) are compared with the tiled direct
form (KNN_ALGO_DIRECT, k_direct_tile: oracle- and golden-pinned in test_gpu_direct.py /
test_gpu_parity.py), and a spread sample of queries with the oracle itself on the full
train set.  Anchor: main.cpp:40-82 (the per-query loop) at the configs' sizes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run_full(knn, oracle, nt, nq, d, k, seed, n_sample, expect_segments_min, q0=0):
    import torch
    dev = "cuda:0"
    gen = knn.Context(0)
    train = torch.empty((nt, d), dtype=torch.float32, device=dev)
    labels = torch.empty(nt, dtype=torch.int32, device=dev)
    test = torch.empty((nq, d), dtype=torch.float32, device=dev)
    gen.generate(train, labels, 0, d, 0, seed, 0, 10)
    gen.generate(test, None, q0, d, 0, seed, 1, 10)
    gen.close()
    out = {}
    for algo in ("auto", "direct"):
        c = knn.Context(0, algo=algo)
        pred = torch.empty(nq, dtype=torch.int32, device=dev)
        dist = torch.empty((nq, k), dtype=torch.float32, device=dev)
        idx = torch.empty((nq, k), dtype=torch.int32, device=dev)
        c.predict_device(train, labels, test, k, 10, pred, dist, idx)
        torch.cuda.synchronize()
        out[algo] = (pred, dist, idx, c.stats())
        c.close()
    pa, da, ia, st = out["auto"]
    pd, dd, idd, _ = out["direct"]
    assert st["filter_operands"] == "bf16 rounded" and st["train_segments"] >= expect_segments_min, st
    # every query, bit for bit (compared on the device: no multi-GB host copies)
    assert torch.equal(ia, idd), int((ia != idd).any(dim=1).sum())
    assert torch.equal(da.view(torch.int32), dd.view(torch.int32))
    assert torch.equal(pa, pd)
    # size-independent properties: ascending lists, valid classes, distinct neighbours
    assert bool((da[:, 1:] >= da[:, :-1]).all())
    assert int(pa.min()) >= 0 and int(pa.max()) < 10
    # a spread sample against the oracle on the whole train set
    qs = np.linspace(0, nq - 1, n_sample).astype(np.int64)
    bad, opred, odist, oidx = oracle.knn(train.cpu().numpy(), labels.cpu().numpy(),
                                         test[torch.from_numpy(qs).to(dev)].cpu().numpy(), k, 10)
    assert bad == 0
    assert np.array_equal(ia.cpu().numpy()[qs], oidx)
    assert np.array_equal(da.cpu().numpy()[qs].view(np.uint32), odist.view(np.uint32))
    assert np.array_equal(pa.cpu().numpy()[qs], opred)
    return st


def test_full_size_config_a(knn, oracle):
    """Config A: 1M train x 100k query x 128-d fp32, k=10 -- all 100,000 queries."""
    _run_full(knn, oracle, 1_000_000, 100_000, 128, 10, 1, 48, 1)


def test_full_size_config_b(knn, oracle):
    """Config B: 4M train x 1M query x 64-d fp32, k=32 -- all 1,000,000 queries (B's plan:
    the two-block 4-wave shape for 128-byte bf16 rows, several train segments)."""
    st = _run_full(knn, oracle, 4_000_000, 1_000_000, 64, 32, 2, 16, 2)
    assert st["fallback_queries"] < 1_000_000 // 16, st


def test_config_a_rank_share(knn, oracle):
    """Config A's per-rank share at 8 GPUs under the fixed-problem split (bench --strong): the
    last rank's 12,500 query rows (knn_rank_queries, mpi.cpp:141-170) against the whole 1M
    train set -- the partition knn_shard_policy picks for A (test-sharded), in the plan's
    share-size shape (32 queries per wave, each query tile cut into pieces that exchange
    thresholds and lists).  Every query bit-exact against the direct form."""
    q0, nq = knn.rank_queries(100_000, 8, 7, "strong")
    assert (q0, nq) == (87_500, 12_500)
    assert knn.shard_policy(1_000_000, 100_000, 128, "f32", 8, 288 << 30) == "test"
    st = _run_full(knn, oracle, 1_000_000, nq, 128, 10, 1, 24, 1, q0=q0)
    assert st["fused_norm"], st
