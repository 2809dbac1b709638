#!/bin/bash
# round 3, pass x: k_row_norms with four rounds' loads in flight and the maximum-norm atomic only when it raises the maximum (vs libknn_amd_base.so, the
# previous commit), same box; then the GPU suite on the product.
set -o pipefail
mkdir -p gpurun_out
P=${PREFIX:-r03x}
A=knn-using-p_threads-and-mpi_amd/build/ablate
PREFIX=$P STEPS=3 RUNS="A_new A; A_base A KNN_AMD_LIB=$A/libknn_amd_base.so; B_new B; B_base B KNN_AMD_LIB=$A/libknn_amd_base.so" PYTEST_ENV="KNN_STUDY_TAG=x" bash scripts/study.sh || exit 1
for f in gpurun_out/${P}_A_new.log gpurun_out/${P}_A_base.log gpurun_out/${P}_B_new.log gpurun_out/${P}_B_base.log; do python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], d['stages_ms'].get('norms'), d['stages_ms'].get('aug'))" $f; done
