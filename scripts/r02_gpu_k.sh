#!/bin/bash
# round 2, pass k: register-list thresholds (KR) + tile rotation in the fused filter:
# parity first, then A/B same-box comparisons (default vs KR=0 vs ROTATE=0), then full size
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 600 $T --timeout 240 tests/test_gpu_parity.py tests/test_gpu_bf16_shard.py tests/test_gpu_host_path.py tests/test_gpu_mfma_cert.py > gpurun_out/r02k_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|Error" gpurun_out/r02k_pytest.log | head; tail -30 gpurun_out/r02k_pytest.log; exit 1; }
tail -1 gpurun_out/r02k_pytest.log
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path"
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);s=d['stages_ms'];g=d['gemm_stats']
print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'filter', s.get('gemm_filter'), 'rescore', s.get('rescore'), 'cand/q', (d['select_stage'] or {}).get('candidates_per_query'), 'fb', g['fallback_queries'], 'segs', g['train_segments'])" $1; }
for cfg in A B; do
  for v in default kr0 rot0; do
    case $v in default) E="";; kr0) E="KNN_FILTER_KR=0";; rot0) E="KNN_FILTER_ROTATE=0";; esac
    env $E timeout -k 10 300 $B --config $cfg > gpurun_out/r02k_bench_${cfg}_$v.log 2>&1 || { echo "bench $cfg $v failed"; tail -5 gpurun_out/r02k_bench_${cfg}_$v.log; exit 1; }
    summ gpurun_out/r02k_bench_${cfg}_$v.log
  done
done
timeout -k 10 900 $T --timeout 600 tests/test_gpu_fullsize.py > gpurun_out/r02k_fullsize.log 2>&1 || { echo "fullsize failed"; tail -30 gpurun_out/r02k_fullsize.log; exit 1; }
tail -1 gpurun_out/r02k_fullsize.log
