#!/bin/bash
# round 3, pass n: six-buffer pairs with the DMA two pairs ahead (deep) -- parity subset, then
# same-box filter times vs the product, and the slow-path / fast-test ablation bounds of the
# product with the lane-parallel slow path.
set -o pipefail
mkdir -p gpurun_out
P=r03n
L=knn-using-p_threads-and-mpi_amd/build/ablate
K="bf16 or synthetic or aligned_rounding or duplicates or shard or golden or stress"
KNN_AMD_LIB=$L/libknn_amd_deep.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py -q \
  --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${P}_pytest_deep.log 2>&1
rc=$?
echo "deep subset rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_deep.log)"; grep '^FAILED' gpurun_out/${P}_pytest_deep.log | head
[ $rc -gt 1 ] && exit 1
PREFIX=$P STEPS=3 RUNS="A_prod A; A_deep A KNN_AMD_LIB=$L/libknn_amd_deep.so; A_noslow A KNN_AMD_LIB=$L/libknn_amd_noslow.so; A_noepi A KNN_AMD_LIB=$L/libknn_amd_noepi.so; B_prod B; B_deep B KNN_AMD_LIB=$L/libknn_amd_deep.so; B_noslow B KNN_AMD_LIB=$L/libknn_amd_noslow.so; A_prod2 A; A_deep2 A KNN_AMD_LIB=$L/libknn_amd_deep.so" bash scripts/study.sh || exit 1
