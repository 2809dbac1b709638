#!/bin/bash
# round 3, pass q: product = heap shapes back on wave-wide visits + remainder DMA pieces rotated
# between even and odd tiles + round 1 of the lane scan by group minima.  Same box: C1 vs the
# pre-lane-parallel build (old), A/B vs rotation only (rot), d = 64 with norm-initialised
# accumulators (tn64, rotation only); parity subsets of the product and tn64.
set -o pipefail
mkdir -p gpurun_out
P=r03q
L=knn-using-p_threads-and-mpi_amd/build/exp
A=knn-using-p_threads-and-mpi_amd/build/ablate
K="bf16 or synthetic or aligned_rounding or duplicates or shard or golden or stress or this_trees"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py tests/test_gpu_host_path.py -q \
  --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${P}_pytest_subset.log 2>&1
rc=$?
echo "subset rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_subset.log)"; grep '^FAILED' gpurun_out/${P}_pytest_subset.log | head
[ $rc -gt 1 ] && exit 1
K2="bf16 or synthetic or aligned_rounding or duplicates or shard or golden or stress"
KNN_AMD_LIB=$A/libknn_amd_tn64.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py -q \
  --timeout 300 --timeout-method thread -k "$K2" > gpurun_out/${P}_pytest_tn64.log 2>&1
rc=$?
echo "tn64 subset rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_tn64.log)"; grep '^FAILED' gpurun_out/${P}_pytest_tn64.log | head
[ $rc -gt 1 ] && exit 1
PREFIX=$P STEPS=2 RUNS="C1_old C1 --nq=131072 KNN_AMD_LIB=$L/old.so; C1_cur C1 --nq=131072; A_rot A KNN_AMD_LIB=$L/rot.so; A_cur A; B_rot B KNN_AMD_LIB=$L/rot.so; B_tn64 B KNN_AMD_LIB=$A/libknn_amd_tn64.so; B_cur B; A_rot2 A KNN_AMD_LIB=$L/rot.so; A_cur2 A; C1_old2 C1 --nq=131072 KNN_AMD_LIB=$L/old.so; C1_cur2 C1 --nq=131072" bash scripts/study.sh || exit 1
