"""Study: what the per-stage HIP events (Context(profile=True), bench.py's stage breakdown) and
the per-call host synchronisation cost per step, on config A's shapes (full and the 8-GPU
share).  Prints ms per step with stage events on and off, same process, same inputs.

    python scripts/event_overhead.py [--nq 12500 100000] [--steps 50]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import importlib  # noqa: E402

knn = importlib.import_module("knn-using-p_threads-and-mpi_amd")


def run(nq, steps, profile, nt=1_000_000, d=128, k=10, C=10):
    dev = torch.device("cuda", 0)
    ctx = knn.Context(0, profile=profile, cache_train=True)
    train = torch.empty((nt, d), dtype=torch.float32, device=dev)
    labels = torch.empty(nt, dtype=torch.int32, device=dev)
    test = torch.empty((nq, d), dtype=torch.float32, device=dev)
    ctx.generate(train, labels, 0, d, 0, 1234, 0, C)
    ctx.generate(test, None, 0, d, 0, 1234, 1, C)
    pred = torch.empty(nq, dtype=torch.int32, device=dev)
    for _ in range(3):
        ctx.predict_device(train, labels, test, k, C, pred)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.predict_device(train, labels, test, k, C, pred)
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    stages = ctx.stage_times() if profile else {}
    ctx.close()
    return ms, stages


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", type=int, nargs="+", default=[12500, 100000])
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    for nq in a.nq:
        for rep in range(2):
            off, _ = run(nq, a.steps, False)
            on, st = run(nq, a.steps, True)
            print(f"nq {nq} rep {rep}: events off {off:.3f} ms/step, on {on:.3f} ms/step, "
                  f"stage sum {sum(st.values()):.3f}, filter {st.get('gemm_filter', 0):.3f}", flush=True)


if __name__ == "__main__":
    main()
