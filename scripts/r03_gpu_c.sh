#!/bin/bash
# round 3, pass c: config C's shards as the test runs them (stall hunt), the GPU suite on the
# cleaned build (padded operand rows, one DMA form with M0 saved, DPP/swizzle lane exchanges),
# then the free schedule (no per-k-step sched_barrier) for correctness and same-box filter time.
set -o pipefail
mkdir -p gpurun_out
L=knn-using-p_threads-and-mpi_amd/build/exp
timeout -k 10 300 python -u scripts/repro_c.py > gpurun_out/r03c_repro.log 2>&1
rc=$?; echo "repro rc=$rc"; tail -12 gpurun_out/r03c_repro.log | cut -c1-300
[ $rc -ne 0 ] && exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread --durations=15 \
  --deselect tests/test_gpu_config_c.py > gpurun_out/r03c_pytest_gpu.log 2>&1
rc=$?
echo "product suite rc=$rc :: $(tail -1 gpurun_out/r03c_pytest_gpu.log)"; grep -E '^FAILED|^ERROR' gpurun_out/r03c_pytest_gpu.log | head
[ $rc -gt 1 ] && exit 1
K="bf16_grid or bf16_random or synthetic_vs or aligned_rounding or duplicates or train_sharded_matches"
KNN_AMD_LIB=$L/free.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py -v \
  --timeout 200 --timeout-method thread -k "$K" > gpurun_out/r03c_pytest_free.log 2>&1
rc=$?
echo "free rc=$rc :: $(tail -1 gpurun_out/r03c_pytest_free.log)"; grep '^FAILED' gpurun_out/r03c_pytest_free.log | head
[ $rc -gt 1 ] && exit 1
KNN_AMD_LIB=$L/free.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -v -x --timeout 300 --timeout-method thread > gpurun_out/r03c_full_free.log 2>&1
rc=$?
echo "fullsize free rc=$rc :: $(tail -1 gpurun_out/r03c_full_free.log)"
[ $rc -gt 1 ] && exit 1
PREFIX=r03c STEPS=3 RUNS="A_strict A; A_free A KNN_AMD_LIB=$L/free.so; B_strict B; B_free B KNN_AMD_LIB=$L/free.so; A_strict2 A" bash scripts/study.sh
