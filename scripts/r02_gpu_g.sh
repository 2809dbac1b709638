#!/bin/bash
# round 2, pass g: soft-barrier fused filter: parity first, then same-box timing
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout-method thread"
KNN_FILTER_NBUF=5 timeout -k 10 300 $T --timeout 120 tests/test_gpu_parity.py -k "synthetic or gemm_duplicates or stress or golden" > gpurun_out/r02g_pytest_soft.log 2>&1 || { echo "soft parity failed"; tail -30 gpurun_out/r02g_pytest_soft.log; exit 1; }
tail -1 gpurun_out/r02g_pytest_soft.log
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
run() {
  local name=$1; shift; local cfg=$1; shift
  env "$@" timeout -k 10 200 $B --config $cfg > gpurun_out/r02g_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/r02g_$name.log; exit 1; }
  echo "$name $(grep -o '"gemm_filter": [0-9.]*' gpurun_out/r02g_$name.log) $(grep -o '"candidates": [0-9]*' gpurun_out/r02g_$name.log | tail -1) $(grep -m1 'knn filter timing' gpurun_out/r02g_$name.log)"
}
A=knn-using-p_threads-and-mpi_amd/build/ablate
run A_base A X=1
run A_nb4 A KNN_FILTER_NBUF=4
run A_nb5 A KNN_FILTER_NBUF=5
run A_nb5_timing A KNN_FILTER_NBUF=5 KNN_AMD_LIB=$PWD/$A/libknn_amd_timing.so KNN_FILTER_TIMING=1
run B_base B X=1
run B_nb5 B KNN_FILTER_NBUF=5
run A_base2 A X=1
run A_nb5_2 A KNN_FILTER_NBUF=5
KNN_FILTER_NBUF=5 timeout -k 10 400 $T --timeout 300 tests/test_gpu_fullsize.py > gpurun_out/r02g_full_soft.log 2>&1 || { echo "fullsize soft failed"; tail -30 gpurun_out/r02g_full_soft.log; exit 1; }
tail -1 gpurun_out/r02g_full_soft.log
