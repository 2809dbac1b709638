#!/bin/bash
# round 2, pass v: where the fused filter's time goes on A (and B): ablation builds
#   noslow (fast test, no slow path), noepi (no fast test: MFMA + DMA + barrier only),
#   nodma (no tile DMA: stale LDS, timing only), noepidma (MFMA + LDS reads + barrier)
set -o pipefail
mkdir -p gpurun_out
L=knn-using-p_threads-and-mpi_amd/build/ablate
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);s=d['stages_ms']
print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'filter', s.get('gemm_filter'), 'cand/q', (d['select_stage'] or {}).get('candidates_per_query'))" $1; grep -m1 "filter timing" $1 || true; }
run() { local tag=$1 cfg=$2; shift 2; env "$@" timeout -k 10 300 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/r02v_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r02v_$tag.log; exit 1; }; summ gpurun_out/r02v_$tag.log; }
run A_nodma A KNN_AMD_LIB=$L/libknn_amd_nodma.so
run A_noepidma A KNN_AMD_LIB=$L/libknn_amd_noepidma.so
run A_timing A KNN_FILTER_TIMING=1 KNN_AMD_LIB=$L/libknn_amd_timing.so
run B_default B
run B_noepi B KNN_AMD_LIB=$L/libknn_amd_noepi.so
run B_noepidma B KNN_AMD_LIB=$L/libknn_amd_noepidma.so
echo done
