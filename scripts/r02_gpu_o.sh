#!/bin/bash
# round 2, pass o: config B -- one train segment vs two, 8-wave vs 4-wave blocks (heap thresholds)
set -o pipefail
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);s=d['stages_ms'];g=d['gemm_stats']
print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'filter', s.get('gemm_filter'), 'rescore', s.get('rescore'), 'cand/q', (d['select_stage'] or {}).get('candidates_per_query'), 'fb', g['fallback_queries'], 'segs', g['train_segments'])" $1; }
run() { local tag=$1; shift; env KNN_FILTER_KR=0 "$@" timeout -k 10 200 python -u bench.py --config B --steps 2 --warmup 1 --no-cpu-baseline --no-host-path $EXTRA > gpurun_out/r02o_$tag.log 2>&1 || { echo "bench $tag failed"; tail -3 gpurun_out/r02o_$tag.log; exit 1; }; summ gpurun_out/r02o_$tag.log; }
EXTRA="--splits 1" run s1
EXTRA="" run w8 KNN_FILTER_SHAPE=w8
EXTRA="--splits 1" run w8s1 KNN_FILTER_SHAPE=w8
