#!/bin/bash
# round 3, pass v: the rescore's grouped row reads (G = d/32 lanes per survivor row when
# m * G <= 64) vs the committed per-lane rows (libknn_amd_base.so), same box; then the GPU
# suite on the new product (parity of the grouped path).
set -o pipefail
mkdir -p gpurun_out
P=r03v
A=knn-using-p_threads-and-mpi_amd/build/ablate
PREFIX=$P STEPS=3 RUNS="A_grp A; A_base A KNN_AMD_LIB=$A/libknn_amd_base.so; B_grp B; B_base B KNN_AMD_LIB=$A/libknn_amd_base.so; A_grp2 A; A_base2 A KNN_AMD_LIB=$A/libknn_amd_base.so" PYTEST_ENV="KNN_STUDY_TAG=v" bash scripts/study.sh || exit 1
