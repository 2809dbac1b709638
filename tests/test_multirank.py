"""N > 1 path on CPU: world_size-2 gloo runs of the rank logic bench.py uses (query
ownership per rank, barrier + max-over-ranks timing, MPI_Gatherv-style gather of
predictions to rank 0).  The per-rank compute is the oracle here (no GPU); the GPU
path's per-rank call is knn_predict_device on the same [q0, q0+nq) rows."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import DATA


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, scaling, nq_cfg, out_q):
    import torch
    import torch.distributed as dist
    from conftest import Oracle, load_pkg
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    knn = load_pkg()
    o = Oracle()
    tr, tl, d = o.read_arff(f"{DATA}/medium-train.arff")
    te_all, _, _ = o.read_arff(f"{DATA}/medium-test.arff")
    n_total = nq_cfg * world if scaling == "weak" else nq_cfg
    te_all = np.concatenate([te_all] * (n_total // len(te_all) + 1))[:n_total]
    q0, nq = knn.rank_queries(nq_cfg, world, rank, scaling)
    _, pred, _, _ = o.knn(tr, tl, te_all[q0:q0 + nq], 5, 10, threads=2, topk=False)
    dist.barrier()
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)          # bench.py's max-over-ranks time
    full = knn.gather_predictions(pred, q0, n_total, world, rank)
    if rank == 0:
        _, ref, _, _ = o.knn(tr, tl, te_all, 5, 10, threads=2, topk=False)
        out_q.put((float(t.item()), bool(np.array_equal(full, ref)), int(n_total)))
    dist.destroy_process_group()


@pytest.mark.parametrize("scaling,nq_cfg", [("strong", 370), ("strong", 101), ("weak", 150)])
def test_two_rank_gloo(scaling, nq_cfg):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, scaling, nq_cfg, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs)
    tmax, match, n_total = q.get(timeout=10)
    assert tmax == 2.0 and match and n_total == (nq_cfg * 2 if scaling == "weak" else nq_cfg)


def test_rank_queries_cover_everything():
    from conftest import load_pkg
    knn = load_pkg()
    for world in (1, 2, 4, 8):
        spans = [knn.rank_queries(1718, world, r, "strong") for r in range(world)]
        covered = np.concatenate([np.arange(q0, q0 + n) for q0, n in spans])
        assert np.array_equal(covered, np.arange(1718))
        weak = [knn.rank_queries(100, world, r, "weak") for r in range(world)]
        assert [w[0] for w in weak] == [100 * r for r in range(world)]
