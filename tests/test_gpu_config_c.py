"""Config C at its BASELINE size on one GPU (BASELINE.json configs[4]): 32M
bf16 train rows x 1M queries x 256-d, k = 100, train-sharded into 8 contiguous shards run one
after another ("emulate N shards on fewer GPUs by running shards
sequentially"), each an exact per-shard top-k with global indices (knn_shard_topk_device,
the bf16 MFMA filter + exact rescore), then k_merge_vote over the [8][1M][3][100] records --
the same kernels an 8-rank run executes around its RCCL all-to-all.

Checks (the reference's loop main.cpp:40-82 over all 32M rows; the split mpi.cpp:141-186):
  * every query: ascending (dist, idx), distinct in-range indices, labels = labels[idx],
    predictions in [0, C), the vote of the merged list;
  * 4096 spread queries: bit-exact (idx, dist bits, pred) against KNN_ALGO_DIRECT (the
    oracle-pinned direct form, tests/test_gpu_fullsize.py) over all 32M rows;
  * 8 queries: bit-exact against the C oracle, run shard by shard and merged on the host
    by (dist, global idx) (conftest.merge_lists_reference).
"""
import numpy as np
import pytest

from conftest import merge_lists_reference

pytestmark = pytest.mark.gpu

NT, NQ, D, K, C, S = 32_000_000, 1_000_000, 256, 100, 10, 8
SEED = 3  # config C uses seed 3 (train stream 0, queries stream 1)


def _progress(msg):
    """A line per stage (the run takes a minute or two): appended to gpurun_out/ when that
    scratch directory exists (pytest captures the test's own stderr), else to stderr."""
    import os
    import sys
    import time
    line = f"[config C {time.strftime('%H:%M:%S')}] {msg}\n"
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, "config_c_progress.log"), "a") as f:
            f.write(line)
    else:
        sys.__stderr__.write(line)
        sys.__stderr__.flush()


@pytest.fixture(scope="module")
def config_c(knn):
    _progress("start")
    import torch
    dev = "cuda:0"
    ctx = knn.Context(0, algo="auto", profile=True)
    train = torch.empty((NT, D), dtype=torch.bfloat16, device=dev)
    labels = torch.empty(NT, dtype=torch.int32, device=dev)
    test = torch.empty((NQ, D), dtype=torch.bfloat16, device=dev)
    ctx.generate(train, labels, 0, D, 1, SEED, 0, C)
    ctx.generate(test, None, 0, D, 1, SEED, 1, C)
    rec = torch.empty((S, NQ, 3, K), dtype=torch.int32, device=dev)
    segs = []
    _progress("data generated")
    for r in range(S):
        a, b = knn.shard_range(NT, S, r)
        ctx.shard_topk_device(train[a:b], labels[a:b], test, K, C, a, rec[r])
        segs.append(ctx.stats()["train_segments"])
        _progress(f"shard {r} [{a}, {b}): {ctx.stage_times()}")
    pred = torch.empty(NQ, dtype=torch.int32, device=dev)
    dist = torch.empty((NQ, K), dtype=torch.float32, device=dev)
    idx = torch.empty((NQ, K), dtype=torch.int32, device=dev)
    ctx.merge_vote_device(rec, K, C, pred, dist, idx)
    torch.cuda.synchronize()
    _progress(f"merged: {ctx.stage_times()}")
    out = dict(ctx=ctx, train=train, labels=labels, test=test, rec=rec, pred=pred, dist=dist, idx=idx, segs=segs)
    yield out
    ctx.close()
    out.clear()
    torch.cuda.empty_cache()


def test_config_c_properties_every_query(knn, config_c):
    import torch
    assert all(s >= 1 for s in config_c["segs"]), "bf16 MFMA filter did not run"
    idx, dist, pred = config_c["idx"], config_c["dist"], config_c["pred"]
    labels = config_c["labels"]
    assert int(idx.min()) >= 0 and int(idx.max()) < NT
    db = dist.view(torch.int32)                     # distances >= 0: bits order like values
    assert bool((db[:, 1:] >= db[:, :-1]).all())
    tie = db[:, 1:] == db[:, :-1]
    assert bool((idx[:, 1:] > idx[:, :-1])[tie].all())      # equal distance: ascending index
    srt, _ = torch.sort(idx, dim=1)
    assert bool((srt[:, 1:] != srt[:, :-1]).all())           # distinct neighbours
    assert int(pred.min()) >= 0 and int(pred.max()) < C
    # the vote of the merged list: bincount argmax, ties to the smallest label (main.cpp:64-78)
    lab = labels[idx.long()]
    counts = torch.zeros((NQ, C), dtype=torch.int32, device=idx.device)
    counts.scatter_add_(1, lab.long(), torch.ones_like(lab))
    assert bool((pred == torch.argmax(counts * C + (C - 1 - torch.arange(C, device=idx.device)), dim=1)).all())
    # each shard's list is sorted, in its shard's index range, and labelled by labels[idx]
    rec = config_c["rec"]
    for r in range(S):
        a, b = knn.shard_range(NT, S, r)
        ri = rec[r, :, 1, :]
        assert int(ri.min()) >= a and int(ri.max()) < b
        rb = rec[r, :, 0, :]
        assert bool((rb[:, 1:] >= rb[:, :-1]).all())
        assert bool((rec[r, :, 2, :] == labels[ri.long()]).all())


def test_config_c_vs_direct_4096(knn, config_c):
    import torch
    qs = torch.linspace(0, NQ - 1, 4096, device="cuda:0").round().long()
    test = config_c["test"][qs].contiguous()
    d = knn.Context(0, algo="direct")
    try:
        pred = torch.empty(len(qs), dtype=torch.int32, device="cuda:0")
        dist = torch.empty((len(qs), K), dtype=torch.float32, device="cuda:0")
        idx = torch.empty((len(qs), K), dtype=torch.int32, device="cuda:0")
        _progress("direct form over 32M rows, 4096 queries")
        d.predict_device(config_c["train"], config_c["labels"], test, K, C, pred, dist, idx)
        torch.cuda.synchronize()
        _progress("direct done")
        assert torch.equal(idx, config_c["idx"][qs])
        assert torch.equal(dist.view(torch.int32), config_c["dist"][qs].view(torch.int32))
        assert torch.equal(pred, config_c["pred"][qs])
    finally:
        d.close()


def test_config_c_vs_oracle_8(knn, oracle, config_c):
    """The C oracle over all 32M rows for 8 queries, one shard at a time (4 GB of fp32 rows on
    the host per shard), merged by (distance, global index)."""
    import torch
    qs = np.linspace(0, NQ - 1, 8).round().astype(np.int64)
    tef = config_c["test"][torch.from_numpy(qs).cuda()].float().cpu().numpy()
    rec = np.zeros((S, len(qs), 3, K), np.int32)
    lab_all = config_c["labels"]
    for r in range(S):
        a, b = knn.shard_range(NT, S, r)
        trf = config_c["train"][a:b].float().cpu().numpy()
        lab = lab_all[a:b].cpu().numpy()
        bad, _, odist, oidx = oracle.knn(trf, lab, tef, K, C)
        assert bad == 0
        _progress(f"oracle shard {r} done")
        rec[r, :, 0, :] = odist.view(np.int32)
        rec[r, :, 1, :] = oidx + a
        rec[r, :, 2, :] = lab[oidx]
        del trf
    opred, odist, oidx = merge_lists_reference(rec, K, C)
    got_idx = config_c["idx"][torch.from_numpy(qs).cuda()].cpu().numpy()
    got_dist = config_c["dist"][torch.from_numpy(qs).cuda()].cpu().numpy()
    got_pred = config_c["pred"][torch.from_numpy(qs).cuda()].cpu().numpy()
    assert np.array_equal(got_idx, oidx)
    assert np.array_equal(got_dist.view(np.uint32), odist.view(np.uint32))
    assert np.array_equal(got_pred, opred)
