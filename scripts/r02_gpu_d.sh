#!/bin/bash
# round 2, pass d: fused filter phase clocks (record / flush counts) and triple buffering
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
A=knn-using-p_threads-and-mpi_amd/build/ablate
for cfg in A B; do
  for nb in 2 3; do
    env KNN_FILTER_NBUF=$nb timeout -k 10 300 $B --config $cfg > gpurun_out/r02d_bench_${cfg}_nb$nb.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r02d_bench_${cfg}_nb$nb.log; exit 1; }
    echo "$cfg nbuf=$nb $(grep -o '"gemm_filter": [0-9.]*' gpurun_out/r02d_bench_${cfg}_nb$nb.log)"
    env KNN_AMD_LIB=$PWD/$A/libknn_amd_timing.so KNN_FILTER_TIMING=1 KNN_FILTER_NBUF=$nb timeout -k 10 300 $B --config $cfg > gpurun_out/r02d_tim_${cfg}_nb$nb.log 2>&1 || { echo "timing failed"; exit 1; }
    echo "   timing $(grep -o '"gemm_filter": [0-9.]*' gpurun_out/r02d_tim_${cfg}_nb$nb.log) $(grep -m1 'knn filter timing' gpurun_out/r02d_tim_${cfg}_nb$nb.log)"
  done
done
