#!/bin/bash
# round 2, pass e: fused filter with the pass set built in the step; shapes; parity
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout-method thread"
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
A=knn-using-p_threads-and-mpi_amd/build/ablate
run() {  # name env... -- config
  local name=$1; shift; local cfg=$1; shift
  env "$@" timeout -k 10 300 $B --config $cfg > gpurun_out/r02e_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/r02e_$name.log; exit 1; }
  echo "$name $(grep -o '"gemm_filter": [0-9.]*' gpurun_out/r02e_$name.log) $(grep -o '"candidates": [0-9]*' gpurun_out/r02e_$name.log | tail -1) $(grep -m1 'knn filter timing' gpurun_out/r02e_$name.log)"
}
run A_fused A X=1

run A_timing A KNN_AMD_LIB=$PWD/$A/libknn_amd_timing.so KNN_FILTER_TIMING=1
run B_fused B X=1

run B_timing B KNN_AMD_LIB=$PWD/$A/libknn_amd_timing.so KNN_FILTER_TIMING=1
timeout -k 10 600 $T --timeout 240 tests/test_gpu_parity.py tests/test_gpu_mfma_cert.py tests/test_gpu_bf16_shard.py > gpurun_out/r02e_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r02e_pytest.log; exit 1; }
tail -1 gpurun_out/r02e_pytest.log
timeout -k 10 400 $T --timeout 300 tests/test_gpu_fullsize.py > gpurun_out/r02e_full.log 2>&1 || { echo "fullsize failed"; tail -30 gpurun_out/r02e_full.log; exit 1; }
tail -1 gpurun_out/r02e_full.log
