#!/bin/bash
# round 3, pass p: config C1's filter (heap shapes, k = 100, d = 256) same box on 131,072
# queries: before the lane-parallel slow path (old), lane-parallel (prod), + norm-initialised
# accumulators (tn), + single-instruction min in the list updates (product); A for the last
# two; the product's parity subset and build identity.
set -o pipefail
mkdir -p gpurun_out
P=r03p
L=knn-using-p_threads-and-mpi_amd/build/exp
A=knn-using-p_threads-and-mpi_amd/build/ablate
K="bf16 or synthetic or aligned_rounding or duplicates or shard or golden or stress or this_trees"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py tests/test_gpu_host_path.py -q \
  --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${P}_pytest_subset.log 2>&1
rc=$?
echo "subset rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_subset.log)"; grep '^FAILED' gpurun_out/${P}_pytest_subset.log | head
[ $rc -gt 1 ] && exit 1
PREFIX=$P STEPS=2 RUNS="C1_old C1 --nq=131072 KNN_AMD_LIB=$L/old.so; C1_prod C1 --nq=131072 KNN_AMD_LIB=$L/prod.so; C1_tn C1 --nq=131072 KNN_AMD_LIB=$L/tn.so; C1_cur C1 --nq=131072; A_tn A KNN_AMD_LIB=$L/tn.so; A_cur A; C1_old2 C1 --nq=131072 KNN_AMD_LIB=$L/old.so; C1_cur2 C1 --nq=131072; A_nobar A KNN_AMD_LIB=$A/libknn_amd_nobar.so; A_noslow A KNN_AMD_LIB=$A/libknn_amd_noslow.so; B_cur B; B_nobar B KNN_AMD_LIB=$A/libknn_amd_nobar.so; A_cur2 A" bash scripts/study.sh || exit 1
