#!/bin/bash
# round 3, pass r: product candidate (d = 64 norm-initialised too, 16-value lane scan, remainder
# DMA pieces rotated between even and odd tiles): parity subset + full-size A/B, then same box
# vs the same build without the rotation (norot), A, B and C1 (131k queries).
set -o pipefail
mkdir -p gpurun_out
P=r03r
A=knn-using-p_threads-and-mpi_amd/build/ablate
K="bf16 or synthetic or aligned_rounding or duplicates or shard or golden or stress or this_trees"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py tests/test_gpu_host_path.py -q \
  --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${P}_pytest_subset.log 2>&1
rc=$?
echo "subset rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_subset.log)"; grep '^FAILED' gpurun_out/${P}_pytest_subset.log | head
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -q -x --timeout 300 --timeout-method thread > gpurun_out/${P}_full.log 2>&1
rc=$?
echo "fullsize rc=$rc :: $(tail -1 gpurun_out/${P}_full.log)"
[ $rc -ne 0 ] && exit 1
PREFIX=$P STEPS=3 RUNS="A_cand A; A_norot A KNN_AMD_LIB=$A/libknn_amd_norot.so; B_cand B; B_norot B KNN_AMD_LIB=$A/libknn_amd_norot.so; C1_cand C1 --nq=131072; C1_norot C1 --nq=131072 KNN_AMD_LIB=$A/libknn_amd_norot.so; A_cand2 A; A_norot2 A KNN_AMD_LIB=$A/libknn_amd_norot.so" bash scripts/study.sh || exit 1
