#!/bin/bash
# filter shape study for the split / bf16 filters (run via gpurun):
# parity of the forced shape on the synthetic + stress cases, then filter times
set -o pipefail
mkdir -p gpurun_out
KNN_FILTER_SHAPE=${PSHAPE:-w4r1} timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "synthetic or stress or duplicates or golden" > gpurun_out/sh_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/sh_pytest.log; exit 1; }
tail -1 gpurun_out/sh_pytest.log
for run in ${RUNS:-A:w8:3:base A:w4r1:3:base A:w4r1:2:base A:w4r1:3:w4defer B:w8:3:base B:w4r1:3:base}; do
  IFS=: read cfg shape nb lib <<< "$run"
  L=""; [ $lib != base ] && L="KNN_AMD_LIB=$PWD/knn-using-p_threads-and-mpi_amd/build/ablate/libknn_amd_$lib.so"
  case $lib in t*) L="$L KNN_FILTER_TIMING=1";; esac
  env $L KNN_FILTER_SHAPE=$shape KNN_FILTER_NBUF=$nb timeout -k 10 300 python -u bench.py --config $cfg --algo ${ALGO:-gemm_split} \
      --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sh_$cfg.log 2>&1 || { echo "fail $run"; tail -3 gpurun_out/sh_$cfg.log; exit 1; }
  echo "$run $(grep -o '"gemm_filter": [0-9.]*' gpurun_out/sh_$cfg.log) $(grep -m1 'knn filter timing' gpurun_out/sh_$cfg.log)"
done
