#!/bin/bash
# round 3, pass f: config C at size (fixed generator grid), the GPU suite, then the free
# schedule (no per-k-step sched_barrier) for correctness, then same-box filter times:
# base = commit 98d12ae, product = + pinned fast test + LDS-carried tile stats, free.
set -o pipefail
mkdir -p gpurun_out
L=knn-using-p_threads-and-mpi_amd/build/exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_config_c.py -m gpu -v -s --timeout 500 --timeout-method thread --durations=5 > gpurun_out/r03f_config_c.log 2>&1
rc=$?; echo "config C rc=$rc"; grep -E 'PASSED|FAILED|ERROR|passed|failed' gpurun_out/r03f_config_c.log | tail -5
[ $rc -gt 1 ] && exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread --durations=15 \
  --deselect tests/test_gpu_config_c.py > gpurun_out/r03f_pytest_gpu.log 2>&1
rc=$?
echo "product suite rc=$rc :: $(tail -1 gpurun_out/r03f_pytest_gpu.log)"; grep -E '^FAILED|^ERROR' gpurun_out/r03f_pytest_gpu.log | head
[ $rc -gt 1 ] && exit 1
K="bf16_grid or bf16_random or synthetic_vs or aligned_rounding or duplicates or train_sharded_matches"
KNN_AMD_LIB=$L/free.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py -v \
  --timeout 200 --timeout-method thread -k "$K" > gpurun_out/r03f_pytest_free.log 2>&1
rc=$?
echo "free rc=$rc :: $(tail -1 gpurun_out/r03f_pytest_free.log)"; grep '^FAILED' gpurun_out/r03f_pytest_free.log | head
[ $rc -gt 1 ] && exit 1
KNN_AMD_LIB=$L/free.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -v -x --timeout 300 --timeout-method thread > gpurun_out/r03f_full_free.log 2>&1
rc=$?
echo "fullsize free rc=$rc :: $(tail -1 gpurun_out/r03f_full_free.log)"
[ $rc -gt 1 ] && exit 1
PREFIX=r03f STEPS=3 RUNS="A_base A KNN_AMD_LIB=$L/base.so; A_prod A; A_free A KNN_AMD_LIB=$L/free.so; B_base B KNN_AMD_LIB=$L/base.so; B_prod B; B_free B KNN_AMD_LIB=$L/free.so; A_prod2 A" bash scripts/study.sh
