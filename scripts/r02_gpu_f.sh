#!/bin/bash
# round 2, pass f: same-box comparison of filter variants on A and B
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
run() {
  local name=$1; shift; local cfg=$1; shift
  env "$@" timeout -k 10 300 $B --config $cfg > gpurun_out/r02f_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/r02f_$name.log; exit 1; }
  echo "$name $(grep -o '"gemm_filter": [0-9.]*' gpurun_out/r02f_$name.log) $(grep -o '"candidates": [0-9]*' gpurun_out/r02f_$name.log | tail -1)"
}
for rep in 1 2; do
run A_pstep1_$rep A KNN_FILTER_PSTEP=1
run A_pstep0_$rep A KNN_FILTER_PSTEP=0
run A_old_$rep A KNN_FILTER_FUSED=0
run B_pstep0_$rep B KNN_FILTER_PSTEP=0
run B_pstep1_$rep B KNN_FILTER_PSTEP=1
run B_old_$rep B KNN_FILTER_FUSED=0
done
