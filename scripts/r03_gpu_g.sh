#!/bin/bash
# round 3, pass g: tile-integrity check of the free schedule (and the strict one as control)
mkdir -p gpurun_out
L=knn-using-p_threads-and-mpi_amd/build/exp
for v in check freecheck; do
  KNN_AMD_LIB=$L/$v.so timeout -k 5 120 python -u scripts/diag_tiles.py > gpurun_out/r03g_$v.log 2>&1
  echo "$v rc=$?"; grep -v amdgpu.ids gpurun_out/r03g_$v.log | tail -6 | cut -c1-300
done
exit 0
