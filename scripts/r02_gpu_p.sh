#!/bin/bash
# round 2, pass p: two query groups per wave (knn_fused2.hip) -- parity, then A/B vs the one-group kernel
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 600 $T --timeout 240 tests/test_gpu_parity.py tests/test_gpu_bf16_shard.py tests/test_gpu_mfma_cert.py > gpurun_out/r02p_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|Error" gpurun_out/r02p_pytest.log | head; tail -30 gpurun_out/r02p_pytest.log; exit 1; }
tail -1 gpurun_out/r02p_pytest.log
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);s=d['stages_ms'];g=d['gemm_stats']
print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'filter', s.get('gemm_filter'), 'rescore', s.get('rescore'), 'cand/q', (d['select_stage'] or {}).get('candidates_per_query'), 'fb', g['fallback_queries'], 'segs', g['train_segments'], 'qg', g['fused_query_groups'])" $1; }
run() { local tag=$1 cfg=$2; shift 2; env KNN_FILTER_ROTATE=0 "$@" timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/r02p_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r02p_$tag.log; exit 1; }; summ gpurun_out/r02p_$tag.log; }
run A_qg2 A
run A_qg1_rl A KNN_FILTER_QG=1
run B_qg2 B
run B_qg1_heap B KNN_FILTER_QG=1 KNN_FILTER_KR=0
run A_qg2_p0 A KNN_FILTER_PSTEP=0
run B_qg2_p1 B KNN_FILTER_PSTEP=1
