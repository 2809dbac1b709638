#!/bin/bash
# round 3, pass o: accumulators started from the tile header's norms (no augmented k-step) for
# d >= 128 -- the whole GPU suite, then same-box filter times vs the lane-parallel product
# (prod.so), then the C1 bench line.
set -o pipefail
mkdir -p gpurun_out
P=r03o
L=knn-using-p_threads-and-mpi_amd/build
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 500 --timeout-method thread --durations=10 \
  > gpurun_out/${P}_pytest_gpu.log 2>&1
rc=$?
echo "suite rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_gpu.log)"; grep -E '^FAILED|^ERROR' gpurun_out/${P}_pytest_gpu.log | head
[ $rc -gt 1 ] && exit 1
PREFIX=$P STEPS=3 RUNS="A_prev A KNN_AMD_LIB=$L/exp/prod.so; A_tn A; B_prev B KNN_AMD_LIB=$L/exp/prod.so; B_tn B; A_prev2 A KNN_AMD_LIB=$L/exp/prod.so; A_tn2 A" bash scripts/study.sh || exit 1
timeout -k 10 500 python -u bench.py --config C1 --steps 2 --warmup 1 > gpurun_out/${P}_bench_C1.log 2>&1 || { echo "bench C1 failed"; tail -5 gpurun_out/${P}_bench_C1.log; exit 1; }
echo "C1: $(tail -1 gpurun_out/${P}_bench_C1.log | cut -c1-700)"
