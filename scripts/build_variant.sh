#!/bin/bash
# Same-box A/B studies of the filter kernel: a library whose knn_fused.hip comes from a git
# revision (or the working tree, "."), compiled with extra flags, linked with the current
# objects of everything else.  Select it with KNN_AMD_LIB=<path> (the package's loader).
#   bash scripts/build_variant.sh base HEAD              -> build/study/libknn_amd_base.so
#   bash scripts/build_variant.sh stamps . -DKNN_STUDY_STAMPS
# F16=1: knn_fused16.hip from the same revision with the same flags too.
# KERNELS=1: knn_kernels.hip (rescore, direct form, ...) from the same revision with the same
# flags too (e.g. the rescore's phase stamps, knn_debug_rescore_stamps).
set -e
NAME=$1; REV=$2; shift 2
P=$(cd "$(dirname "$0")/../knn-using-p_threads-and-mpi_amd" && pwd)
cd "$P"
make -s libknn_amd.so
mkdir -p build/study
SRC=csrc/.variant_${NAME}.hip
if [ "$REV" = "." ]; then cp csrc/knn_fused.hip $SRC; else git show "$REV:knn-using-p_threads-and-mpi_amd/csrc/knn_fused.hip" > $SRC; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -fno-slp-vectorize "$@" -c -o build/study/knn_fused_$NAME.o $SRC
rm -f $SRC
F16OBJ=build/knn_fused16.o
if [ "$F16" = 1 ]; then  # knn_fused16.hip (the 16x16x32 filter) from the same revision with the same flags
  FSRC=csrc/.variant_f16_${NAME}.hip
  if [ "$REV" = "." ]; then cp csrc/knn_fused16.hip $FSRC; else git show "$REV:knn-using-p_threads-and-mpi_amd/csrc/knn_fused16.hip" > $FSRC; fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -fno-slp-vectorize "$@" -c -o build/study/knn_fused16_$NAME.o $FSRC
  rm -f $FSRC
  F16OBJ=build/study/knn_fused16_$NAME.o
fi
KOBJ=build/knn_kernels.o
if [ "$KERNELS" = 1 ]; then
  KSRC=csrc/.variant_k_${NAME}.hip
  if [ "$REV" = "." ]; then cp csrc/knn_kernels.hip $KSRC; else git show "$REV:knn-using-p_threads-and-mpi_amd/csrc/knn_kernels.hip" > $KSRC; fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -c -o build/study/knn_kernels_$NAME.o $KSRC
  rm -f $KSRC
  KOBJ=build/study/knn_kernels_$NAME.o
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/study/libknn_amd_$NAME.so $KOBJ \
    build/study/knn_fused_$NAME.o $F16OBJ build/knn_capi.o build/knn_comm.o build/knn_arff.o build/knn_build_id.o -ldl
echo "built build/study/libknn_amd_$NAME.so"
