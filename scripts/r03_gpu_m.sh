#!/bin/bash
# round 3, pass m: lane-parallel slow path of the register-list shapes -- parity first (the
# bf16/synthetic subset, then full-size A/B), then same-box filter times vs the previous
# product (prev.so), the stamps split, and the LDS broadcast-read micro-benchmark.
set -o pipefail
mkdir -p gpurun_out
P=r03m
L=knn-using-p_threads-and-mpi_amd/build
K="bf16 or synthetic or aligned_rounding or duplicates or shard or golden or stress"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py -q \
  --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${P}_pytest_subset.log 2>&1
rc=$?
echo "subset rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_subset.log)"; grep '^FAILED' gpurun_out/${P}_pytest_subset.log | head
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -q -x --timeout 300 --timeout-method thread > gpurun_out/${P}_full.log 2>&1
rc=$?
echo "fullsize rc=$rc :: $(tail -1 gpurun_out/${P}_full.log)"
[ $rc -ne 0 ] && exit 1
PREFIX=$P STEPS=3 RUNS="A_prev A KNN_AMD_LIB=$L/exp/prev.so; A_new A; B_prev B KNN_AMD_LIB=$L/exp/prev.so; B_new B; A_new2 A" bash scripts/study.sh || exit 1
KNN_AMD_LIB=$L/ablate/libknn_amd_stamps.so timeout -k 10 240 python -u scripts/stamps.py > gpurun_out/${P}_stamps.log 2>&1 || { echo "stamps failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/${P}_stamps.log
timeout -k 10 60 ./build_tools/lds_bcast > gpurun_out/${P}_lds_bcast.log 2>&1 || { echo "lds_bcast failed"; exit 1; }
cat gpurun_out/${P}_lds_bcast.log
