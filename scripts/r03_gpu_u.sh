#!/bin/bash
# round 3, pass u: knobs on the final kernel, same box -- free schedule (no per-k-step
# sched_barrier), A-fragment prefetch depth 4 / 8 MFMAs (product 6); A, B, C1 (131k queries).
set -o pipefail
mkdir -p gpurun_out
P=r03u
A=knn-using-p_threads-and-mpi_amd/build/ablate
PREFIX=$P STEPS=3 RUNS="A_prod A; A_free A KNN_AMD_LIB=$A/libknn_amd_free.so; A_pf4 A KNN_AMD_LIB=$A/libknn_amd_pf4.so; A_pf8 A KNN_AMD_LIB=$A/libknn_amd_pf8.so; B_prod B; B_free B KNN_AMD_LIB=$A/libknn_amd_free.so; B_pf4 B KNN_AMD_LIB=$A/libknn_amd_pf4.so; B_pf8 B KNN_AMD_LIB=$A/libknn_amd_pf8.so; C1_prod C1 --nq=131072; C1_free C1 --nq=131072 KNN_AMD_LIB=$A/libknn_amd_free.so; A_prod2 A; A_free2 A KNN_AMD_LIB=$A/libknn_amd_free.so" bash scripts/study.sh || exit 1
