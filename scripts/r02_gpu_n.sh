#!/bin/bash
# round 2, pass n: filter phase timing (KNN_FILTER_TIMING build) and the no-slow-path bound, A and B
set -o pipefail
mkdir -p gpurun_out
L=knn-using-p_threads-and-mpi_amd/build/ablate
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);s=d['stages_ms'];g=d['gemm_stats']
print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'filter', s.get('gemm_filter'), 'cand/q', (d['select_stage'] or {}).get('candidates_per_query'))" $1; grep -m2 "filter timing" $1 || true; }
run() { local tag=$1 cfg=$2; shift 2; env "$@" timeout -k 10 300 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/r02n_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r02n_$tag.log; exit 1; }; summ gpurun_out/r02n_$tag.log; }
run B_heap_t B KNN_FILTER_KR=0 KNN_FILTER_TIMING=1 KNN_AMD_LIB=$L/libknn_amd_timing.so
run B_rl_t B KNN_FILTER_TIMING=1 KNN_AMD_LIB=$L/libknn_amd_timing.so
run B_noslow B KNN_FILTER_KR=0 KNN_AMD_LIB=$L/libknn_amd_noslow.so
run A_heap_t A KNN_FILTER_KR=0 KNN_FILTER_TIMING=1 KNN_AMD_LIB=$L/libknn_amd_timing.so
run A_rl_t A KNN_FILTER_TIMING=1 KNN_AMD_LIB=$L/libknn_amd_timing.so
run A_noslow A KNN_AMD_LIB=$L/libknn_amd_noslow.so
