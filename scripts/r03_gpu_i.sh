#!/bin/bash
# round 3, pass i: product = even tile count per piece (no accumulator copies at the loop's back
# edge) + a tile barrier that also retires the wave's LDS reads (lgkmcnt(0)); the whole GPU suite;
# then the free schedule (no per-k-step sched_barrier) on that barrier -- the cases that failed
# in round 2 and full-size A/B parity; then same-box filter times: base (HEAD 0dba8dc), product,
# free.
set -o pipefail
mkdir -p gpurun_out
P=r03i
L=knn-using-p_threads-and-mpi_amd/build/exp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread --durations=15 \
  > gpurun_out/${P}_pytest_gpu.log 2>&1
rc=$?
echo "suite rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_gpu.log)"; grep -E '^FAILED|^ERROR' gpurun_out/${P}_pytest_gpu.log | head
[ $rc -gt 1 ] && exit 1
K="bf16_grid or bf16_random or synthetic_vs or aligned_rounding or duplicates or train_sharded_matches"
KNN_AMD_LIB=$L/free.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py -v \
  --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${P}_pytest_free.log 2>&1
rc=$?
echo "free rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_free.log)"; grep '^FAILED' gpurun_out/${P}_pytest_free.log | head
[ $rc -gt 1 ] && exit 1
KNN_AMD_LIB=$L/free.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -v -x --timeout 300 --timeout-method thread > gpurun_out/${P}_full_free.log 2>&1
rc=$?
echo "fullsize free rc=$rc :: $(tail -1 gpurun_out/${P}_full_free.log)"
[ $rc -gt 1 ] && exit 1
PREFIX=$P STEPS=3 RUNS="A_base A KNN_AMD_LIB=$L/base.so; A_prod A; A_free A KNN_AMD_LIB=$L/free.so; B_base B KNN_AMD_LIB=$L/base.so; B_prod B; B_free B KNN_AMD_LIB=$L/free.so; A_prod2 A" bash scripts/study.sh
