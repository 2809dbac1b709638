set -o pipefail
B="python -u bench.py --config C1 --nq 250000 --steps 1 --warmup 1 --no-cpu-baseline"
for v in ${VARIANTS:-base noslow noepi nodma}; do
  if [ $v = base ]; then L=""; else L="KNN_AMD_LIB=$PWD/knn-using-p_threads-and-mpi_amd/build/ablate/libknn_amd_$v.so"; fi
  env $L timeout -k 10 200 $B > gpurun_out/abl_$v.log 2>&1 || { echo "fail $v"; exit 1; }
  echo "$v $(grep -o '"stages_ms": {[^}]*}' gpurun_out/abl_$v.log)"
done
