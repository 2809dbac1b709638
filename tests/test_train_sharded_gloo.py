"""Train-sharded path on CPU: world_size-2 gloo runs of the
exchange that bench.py --config C and knn_amd.train_sharded_predict use.  Each rank
owns a contiguous train shard; its per-shard top-k for EVERY query comes from the
oracle here (the GPU path's call is knn_shard_topk_device), packed as the device
records [nq][3][k]; exchange_shard_lists (all_to_all_single) delivers each rank the lists
of the queries it owns (the reference's split, mpi.cpp:141-170); the host merge
restatement then must equal the oracle's serial KNN over the whole train set."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _pack(dist, idx, base, labels):
    """oracle per-shard top-k -> device record layout [nq][3][k] (global idx, label)."""
    nq, k = idx.shape
    rec = np.empty((nq, 3, k), np.int32)
    rec[:, 0, :] = dist.view(np.int32)
    ok = idx >= 0
    rec[:, 1, :] = np.where(ok, idx + base, -1)
    rec[:, 2, :] = np.where(ok, labels[np.clip(idx, 0, None)], -1)
    return rec


def _worker(rank, world, port, nt, nq, d, k, kind, out_q):
    import torch
    import torch.distributed as dist
    from conftest import Oracle, load_pkg, merge_lists_reference
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    knn = load_pkg()
    o = Oracle()
    tr, tl = o.gen(5, 0, 0, nt, d, kind=kind)
    te, _ = o.gen(5, 1, 0, nq, d, kind=kind)
    a, b = knn.shard_range(nt, world, rank)            # this rank's train shard
    _, _, sd, si = o.knn(tr[a:b], tl[a:b], te, k, 10, threads=2)
    rec = torch.from_numpy(_pack(sd, si, a, tl[a:b]))
    lists, (q0, q1) = knn.exchange_shard_lists(rec, nq, world, rank)
    assert tuple(lists.shape) == (world, q1 - q0, 3, k)
    pred, dd, ii = merge_lists_reference(lists.numpy(), k, 10)
    _, opred, odist, oidx = o.knn(tr, tl, te[q0:q1], k, 10, threads=2)
    ok = (np.array_equal(pred, opred) and np.array_equal(ii, oidx)
          and np.array_equal(dd.view(np.uint32), odist.view(np.uint32)))
    full = knn.gather_predictions(pred, q0, nq, world, rank)     # MPI_Gatherv analogue
    if rank == 0:
        _, allpred, _, _ = o.knn(tr, tl, te, k, 10, threads=2, topk=False)
        out_q.put((bool(np.array_equal(full, allpred)),))
    out_q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("nt,nq,d,k,kind", [(3001, 77, 64, 10, 0), (2000, 40, 256, 100, 1), (90, 13, 16, 60, 0)])
def test_two_rank_train_sharded(nt, nq, d, k, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, nt, nq, d, k, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs)
    res = [q.get(timeout=10) for _ in range(3)]
    gathered = [r for r in res if len(r) == 1]
    per_rank = sorted(r for r in res if len(r) == 2)
    assert gathered == [(True,)]
    assert per_rank == [(0, True), (1, True)]


def test_exchange_single_rank_is_identity():
    import torch
    from conftest import load_pkg
    knn = load_pkg()
    rec = torch.arange(5 * 3 * 4, dtype=torch.int32).view(5, 3, 4)
    out, (q0, q1) = knn.exchange_shard_lists(rec, 5, 1, 0)
    assert (q0, q1) == (0, 5) and torch.equal(out[0], rec)
