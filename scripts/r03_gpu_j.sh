#!/bin/bash
# round 3, pass j: where the fused filter's time goes after the copy fix -- same-box ablation
# bounds (no slow path / no fast test / no DMA / neither) and the per-half 8-entry lists for
# k <= 16, on A and B; then two PMC passes of the A filter (stall classes, instruction mix);
# then the C1 bench line (train-sharded path, one rank) with its CPU baseline.
set -o pipefail
mkdir -p gpurun_out
P=r03j
L=knn-using-p_threads-and-mpi_amd/build/ablate
PREFIX=$P STEPS=3 RUNS="A_prod A; A_noslow A KNN_AMD_LIB=$L/libknn_amd_noslow.so; A_noepi A KNN_AMD_LIB=$L/libknn_amd_noepi.so; A_nodma A KNN_AMD_LIB=$L/libknn_amd_nodma.so; A_noepidma A KNN_AMD_LIB=$L/libknn_amd_noepidma.so; A_half8 A KNN_AMD_LIB=$L/libknn_amd_half8.so; B_prod B; B_noslow B KNN_AMD_LIB=$L/libknn_amd_noslow.so; B_noepi B KNN_AMD_LIB=$L/libknn_amd_noepi.so; B_nodma B KNN_AMD_LIB=$L/libknn_amd_nodma.so; A_prod2 A" bash scripts/study.sh || exit 1
R=$(pwd)
(cd /tmp && export TMPDIR=/tmp
 i=0
 while read -r SET; do
   i=$((i+1))
   timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $R/gpurun_out/${P}_pmc_$i -o run -- python3 $R/bench.py --config A --steps 1 --warmup 0 --no-cpu-baseline --no-host-path \
       > $R/gpurun_out/${P}_pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
   echo "pmc pass $i ok"
 done <<< "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT") || exit 1
timeout -k 10 500 python -u bench.py --config C1 --steps 2 --warmup 1 > gpurun_out/${P}_bench_C1.log 2>&1 || { echo "bench C1 failed"; tail -5 gpurun_out/${P}_bench_C1.log; exit 1; }
echo "C1: $(tail -1 gpurun_out/${P}_bench_C1.log | cut -c1-600)"
