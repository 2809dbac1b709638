#!/bin/bash
# round 3, pass k: (1) issue cost of the K = 8 bf16 MFMA (the augmented k-step needs 3 of 16
# columns); (2) tile quads (eight buffers, one barrier per four tiles) vs pairs, same box, and
# quads' parity subset; (3) rocprofv3 trace + PMC passes of the C1 workload (train-sharded
# path, 4M x 1M x 256 bf16, k = 100).
set -o pipefail
mkdir -p gpurun_out
P=r03k
L=knn-using-p_threads-and-mpi_amd/build/ablate
timeout -k 10 60 ./build_tools/mfma_cycles > gpurun_out/${P}_mfma_cycles.log 2>&1 || { echo "mfma_cycles failed"; exit 1; }
cat gpurun_out/${P}_mfma_cycles.log
PREFIX=$P STEPS=3 RUNS="A_prod A; A_quads A KNN_AMD_LIB=$L/libknn_amd_quads.so; B_prod B; B_quads B KNN_AMD_LIB=$L/libknn_amd_quads.so; A_prod2 A; A_quads2 A KNN_AMD_LIB=$L/libknn_amd_quads.so" bash scripts/study.sh || exit 1
K="bf16_grid or bf16_random or synthetic_vs or aligned_rounding or duplicates or train_sharded_matches"
KNN_AMD_LIB=$L/libknn_amd_quads.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py -q \
  --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${P}_pytest_quads.log 2>&1
rc=$?
echo "quads parity rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_quads.log)"
[ $rc -gt 1 ] && exit 1
STEPS=1 BENCH_ARGS="--config C1" bash scripts/profile_bench.sh || exit 1
echo done
