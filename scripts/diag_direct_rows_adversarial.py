"""Diagnostic (round 6): k_direct_rows on train rows in decreasing distance from every query
(each tile's rows all pass the running k-th distance: the lane-shift insert's worst case) against
uniform rows of the same shape (config L's: 30,803 x 1,718 x 11, k = 5).  Prints ms per call for
the library KNN_AMD_LIB selects."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from importlib.util import module_from_spec, spec_from_file_location

spec = spec_from_file_location("knn_amd", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                       "knn-using-p_threads-and-mpi_amd", "__init__.py"))
knn = module_from_spec(spec)
spec.loader.exec_module(knn)
nt, nq, d, k = 30_803, 1_718, 11, 5
rng = np.random.default_rng(5)
v = rng.standard_normal((nt, d)).astype(np.float32)
v /= np.linalg.norm(v, axis=1, keepdims=True)
desc = (v * np.linspace(50.0, 1.0, nt, dtype=np.float32)[:, None]).astype(np.float32)
unif = rng.uniform(-1, 1, (nt, d)).astype(np.float32)
te = (rng.standard_normal((nq, d)) * 0.01).astype(np.float32)
lab = rng.integers(0, 10, nt).astype(np.int32)
ctx = knn.Context(0, algo="direct")
ld = 12
out = {}
for name, tr in (("descending", desc), ("uniform", unif)):
    t_tr = torch.zeros((nt, ld), dtype=torch.float32, device="cuda")
    t_te = torch.zeros((nq, ld), dtype=torch.float32, device="cuda")
    t_tr[:, :d] = torch.from_numpy(tr).cuda()
    t_te[:, :d] = torch.from_numpy(te).cuda()
    t_lab = torch.from_numpy(lab).cuda()
    pred = torch.empty(nq, dtype=torch.int32, device="cuda")
    for _ in range(10):
        ctx.predict_device(t_tr, t_lab, t_te, k, 10, pred, d=d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        ctx.predict_device(t_tr, t_lab, t_te, k, 10, pred, d=d)
    torch.cuda.synchronize()
    out[name] = round(1e3 * (time.perf_counter() - t0) / 100, 4)
print(json.dumps({"lib": os.environ.get("KNN_AMD_LIB", "product"), "ms_per_call": out}))
