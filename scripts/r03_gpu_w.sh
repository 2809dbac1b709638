#!/bin/bash
# round 3, pass w: register-list shapes in 4-wave blocks, two per CU (KNN_STUDY_NW4), vs the
# product's 8-wave blocks, same box; then the GPU suite on the study library (parity).
set -o pipefail
mkdir -p gpurun_out
P=r03w
A=knn-using-p_threads-and-mpi_amd/build/ablate
PREFIX=$P STEPS=3 RUNS="A_prod A; A_nw4 A KNN_AMD_LIB=$A/libknn_amd_nw4.so; B_prod B; B_nw4 B KNN_AMD_LIB=$A/libknn_amd_nw4.so; A_prod2 A; A_nw4_2 A KNN_AMD_LIB=$A/libknn_amd_nw4.so" PYTEST_ENV="KNN_AMD_LIB=$A/libknn_amd_nw4.so" PYTEST_ARGS="--deselect tests/test_gpu_host_path.py::test_loaded_library_is_this_trees" bash scripts/study.sh || exit 1
