#!/bin/bash
# round 2, pass l: config B filter vs segment count (MALL-sized segments), block shape and
# tile rotation (heap thresholds: KNN_FILTER_KR=0 throughout)
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --config B --steps 2 --warmup 1 --no-cpu-baseline --no-host-path"
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);s=d['stages_ms'];g=d['gemm_stats']
print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'filter', s.get('gemm_filter'), 'rescore', s.get('rescore'), 'cand/q', (d['select_stage'] or {}).get('candidates_per_query'), 'fb', g['fallback_queries'], 'segs', g['train_segments'], 'rerun', g['rerun_split'])" $1; }
export KNN_FILTER_KR=0
run() { local tag=$1; shift; env "$@" timeout -k 10 300 $B $EXTRA > gpurun_out/r02l_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r02l_$tag.log; exit 1; }; summ gpurun_out/r02l_$tag.log; }
EXTRA="" run s2 KNN_FILTER_ROTATE=0
EXTRA="--splits 3" run s3 KNN_FILTER_ROTATE=0
EXTRA="--splits 4" run s4 KNN_FILTER_ROTATE=0
EXTRA="--splits 4" run s4rot KNN_FILTER_ROTATE=1
EXTRA="--splits 6" run s6 KNN_FILTER_ROTATE=0
EXTRA="" run w8s2 KNN_FILTER_ROTATE=0 KNN_FILTER_SHAPE=w8
EXTRA="--splits 4" run w8s4 KNN_FILTER_ROTATE=0 KNN_FILTER_SHAPE=w8
