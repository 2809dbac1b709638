#!/bin/bash
# ablation study of the split filter on config A (run via gpurun); KNN_FILTER_TIMING=1
# prints the per-phase clocks of the timing builds
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --config ${CFG:-A} --algo ${ALGO:-gemm_split} --steps 2 --warmup 1 --no-cpu-baseline"
for v in ${VARIANTS:-base noslow noepi nodma timing tnoslow}; do
  if [ $v = base ]; then L=""; else L="KNN_AMD_LIB=$PWD/knn-using-p_threads-and-mpi_amd/build/ablate/libknn_amd_$v.so"; fi
  case $v in t*) L="$L KNN_FILTER_TIMING=1";; esac
  env $L timeout -k 10 200 $B > gpurun_out/abl_$v.log 2>&1 || { echo "fail $v"; tail -3 gpurun_out/abl_$v.log; exit 1; }
  echo "$v $(grep -o '"gemm_filter": [0-9.]*' gpurun_out/abl_$v.log) $(grep -m1 'knn filter timing' gpurun_out/abl_$v.log)"
done
