"""The reference's MPI driver contract (mpi.cpp:118-206) on the MI355X path.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        knn-using-p_threads-and-mpi_amd/mpi_driver.py train.arff test.arff k

(or plain `python mpi_driver.py ...` for one rank).  Like mpi.cpp every rank parses both
files; rank 0 cuts the test set with the reference's rule (dataPerProcess = n / N, the
last rank also takes n % N) and scatters the [start, end) pairs (MPI_Scatter,
mpi.cpp:170); every rank classifies its slice on its own GPU (KNN(train, test, k, start,
end), mpi.cpp:172, here knn_predict on device LOCAL_RANK); rank 0 gathers the slices at
displacement rank * dataPerProcess (MPI_Gatherv, mpi.cpp:174-186), computes the confusion
matrix and accuracy and prints the reference's line.  The timed region is the
reference's: from before the scatter to after the gather (CLOCK_MONOTONIC_RAW, ms
truncated).  Control messages (two ints per rank, the int predictions) travel over
torch.distributed's gloo backend, the analogue of the reference's MPI on host memory.
"""
import importlib.util
import os
import sys
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))

USAGE = "Usage: mpiexec -np numProcesses ./mpi datasets/train.arff datasets/test.arff k"


def _pkg():
    if "knn_amd" in sys.modules:
        return sys.modules["knn_amd"]
    spec = importlib.util.spec_from_file_location("knn_amd", os.path.join(_HERE, "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["knn_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def _c_strtol(s):
    """strtol(argv[3], NULL, 10): leading whitespace, sign, digits; 0 if none."""
    s = s.lstrip()
    i = 1 if s[:1] in "+-" else 0
    j = i
    while j < len(s) and s[j].isdigit():
        j += 1
    return int(s[:j]) if j > i else 0


def gpu_context():
    """This rank's context on device LOCAL_RANK (mod the visible devices).  Created before
    the timed region, as mpi.cpp:119-125's MPI_Init / rank setup is."""
    knn = _pkg()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    try:
        import torch
        ndev = max(1, torch.cuda.device_count())
    except ImportError:
        ndev = 1
    return knn.Context(local % ndev, cache_train=True)


def gpu_slice(ctx):
    """The rank's KNN(train, test, k, start, end) (mpi.cpp:26) on its GPU context."""
    knn = _pkg()

    def compute(train, test, k, start, end):
        return knn.KNN_range(train, test, k, start, end, ctx=ctx)
    return compute


def run(argv, compute=None, out=sys.stdout):
    """mpi.cpp main(); `compute` is the per-rank slice classifier (default: the GPU path on
    a context made before the timed region).  With KNN_PRED_OUT set, rank 0 also writes the
    gathered int32 predictions there (a test hook; the reference prints only its line)."""
    if len(argv) != 4:
        print(USAGE, file=out)
        return 0
    import torch.distributed as dist
    knn = _pkg()
    k = _c_strtol(argv[3])
    own_group = not dist.is_initialized()
    if own_group:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        dist.init_process_group("gloo", rank=int(os.environ.get("RANK", "0")),
                                world_size=int(os.environ.get("WORLD_SIZE", "1")))
    rank, world = dist.get_rank(), dist.get_world_size()
    ctx = None
    if compute is None:
        ctx = gpu_context()
        compute = gpu_slice(ctx)
    try:
        tf, tl, C = knn.read_arff(argv[1])
        qf, ql, Cq = knn.read_arff(argv[2])
        n = len(qf)
        per, left = divmod(n, world)
        if rank == 0:
            t0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC_RAW)
            spans, s = [], 0
            for i in range(world):
                e = s + per + (left if i == world - 1 else 0)
                spans.append((s, e))
                s = e
        else:
            spans = None
        mine = [None]
        dist.scatter_object_list(mine, spans, src=0)
        start, end = mine[0]
        sub = np.asarray(compute((tf, tl), (qf, ql), k, start, end), np.int32)
        full = knn.gather_predictions(sub, start, n, world, rank)
        if rank == 0:
            t1 = time.clock_gettime_ns(time.CLOCK_MONOTONIC_RAW)
            cm = knn.computeConfusionMatrix(full, ql, Cq)
            acc = knn.computeAccuracy(cm, n)
            ms = (t1 - t0) // 1_000_000
            print(f"The {k}-NN classifier for {n} test instances on {len(tf)} train instances "
                  f"required {ms} ms CPU time. Accuracy was {acc:.4f}", file=out, flush=True)
            if os.environ.get("KNN_PRED_OUT"):
                np.asarray(full, np.int32).tofile(os.environ["KNN_PRED_OUT"])
            return full
        return None
    finally:
        if ctx is not None:
            ctx.close()
        if own_group:
            dist.destroy_process_group()


if __name__ == "__main__":
    # import torch before libknn_amd so one HIP runtime serves the process
    import torch  # noqa: F401
    run(sys.argv)
