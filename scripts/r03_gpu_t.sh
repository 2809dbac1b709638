#!/bin/bash
# round 3, pass t: the step's DMA pieces in its first k-steps (earlydma) vs spread over the step
# (product), same box, A / B / C1 (131k queries); earlydma's parity subset.
set -o pipefail
mkdir -p gpurun_out
P=r03t
A=knn-using-p_threads-and-mpi_amd/build/ablate
K="bf16 or synthetic or aligned_rounding or duplicates or shard or golden or stress"
KNN_AMD_LIB=$A/libknn_amd_earlydma.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py -q \
  --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${P}_pytest_early.log 2>&1
rc=$?
echo "earlydma subset rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_early.log)"
[ $rc -gt 1 ] && exit 1
PREFIX=$P STEPS=3 RUNS="A_prod A; A_early A KNN_AMD_LIB=$A/libknn_amd_earlydma.so; B_prod B; B_early B KNN_AMD_LIB=$A/libknn_amd_earlydma.so; C1_prod C1 --nq=131072; C1_early C1 --nq=131072 KNN_AMD_LIB=$A/libknn_amd_earlydma.so; A_prod2 A; A_early2 A KNN_AMD_LIB=$A/libknn_amd_earlydma.so" bash scripts/study.sh || exit 1
