#!/bin/bash
# round 2, pass s: L2-sized segments with carried thresholds and one candidate list per query
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 600 $T --timeout 240 tests/test_gpu_parity.py tests/test_gpu_bf16_shard.py tests/test_gpu_host_path.py > gpurun_out/r02s_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|Error" gpurun_out/r02s_pytest.log | head; tail -30 gpurun_out/r02s_pytest.log; exit 1; }
tail -1 gpurun_out/r02s_pytest.log
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);s=d['stages_ms'];g=d['gemm_stats']
print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'filter', s.get('gemm_filter'), 'rescore', s.get('rescore'), 'cand/q', (d['select_stage'] or {}).get('candidates_per_query'), 'fb', g['fallback_queries'], 'segs', g['train_segments'])" $1; }
run() { local tag=$1 cfg=$2; shift 2; env "$@" timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/r02s_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/r02s_$tag.log; exit 1; }; summ gpurun_out/r02s_$tag.log; }
run A_2m A
run B_2m B
run A_1m A KNN_SEG_BYTES=1048576
run B_1m B KNN_SEG_BYTES=1048576
run A_8m A KNN_SEG_BYTES=8388608
run B_8m B KNN_SEG_BYTES=8388608
run B_64m B KNN_SEG_BYTES=67108864
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r02s_fetch_B -o run -- python3 $R/bench.py --config B --steps 1 --warmup 0 --no-cpu-baseline --no-host-path > $R/gpurun_out/r02s_fetch_B.log 2>&1 || { echo "fetch B failed"; exit 1; }
echo "fetch B ok"
cd $R && timeout -k 10 900 $T --timeout 600 tests/test_gpu_fullsize.py > gpurun_out/r02s_fullsize.log 2>&1 || { echo "fullsize failed"; tail -30 gpurun_out/r02s_fullsize.log; exit 1; }
tail -1 gpurun_out/r02s_fullsize.log
