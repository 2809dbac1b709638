"""Host-side cost of one knn_predict_device call from Python (config L's shape): the
wrapper's pieces timed alone, then whole calls.  Diagnostic for DESIGN.md's config-L notes."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import importlib
knn = importlib.import_module("knn-using-p_threads-and-mpi_amd")


def per_call_us(fn, n=20000):
    for _ in range(100):
        fn()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    return round(1e6 * (time.perf_counter() - t) / n, 2)


dev = torch.device("cuda", 0)
x = torch.zeros((30803, 12), device=dev)
q = torch.zeros((1718, 12), device=dev)
lab = torch.zeros(30803, dtype=torch.int32, device=dev)
pred = torch.empty(1718, dtype=torch.int32, device=dev)
ctx = knn.Context(0, profile=3)
print("current_stream", per_call_us(lambda: torch.cuda.current_stream(dev).cuda_stream))
if hasattr(torch._C, "_cuda_getCurrentRawStream"):
    print("raw_stream", per_call_us(lambda: torch._C._cuda_getCurrentRawStream(0)))
print("_device_dataset", per_call_us(lambda: knn._device_dataset(x, lab, 11)))
print("_outputs", per_call_us(lambda: knn._outputs(1718, 5, pred)))
print("stage_times", per_call_us(lambda: ctx.stage_times()))
print("stats", per_call_us(lambda: ctx.stats()))
print("version", per_call_us(lambda: knn.load_library().knn_version()))
for prof in (3, 0):
    c = knn.Context(0, profile=prof)
    for _ in range(20):
        c.predict_device(x, lab, q, 5, 10, pred, d=11)
    torch.cuda.synchronize()
    n = 2000
    t = time.perf_counter()
    for _ in range(n):
        c.predict_device(x, lab, q, 5, 10, pred, d=11)
    torch.cuda.synchronize()
    print(f"predict_device profile={prof}", round(1e6 * (time.perf_counter() - t) / n, 2), "us per call (zero rows)")
    c.close()
ctx.close()
