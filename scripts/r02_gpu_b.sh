#!/bin/bash
# round 2, pass b: MFMA certificate probe + bf16 stress, full parity with the fused filter,
# fused vs old bf16 filter on A and B (same box)
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout-method thread"
timeout -k 10 600 $T --timeout 240 tests/test_gpu_mfma_cert.py tests/test_gpu_parity.py tests/test_gpu_direct.py tests/test_gpu_bf16_shard.py -s > gpurun_out/r02b_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/r02b_pytest.log | head -20; tail -30 gpurun_out/r02b_pytest.log; exit 1; }
tail -3 gpurun_out/r02b_pytest.log
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for cfg in A B; do
  timeout -k 10 300 $B --config $cfg > gpurun_out/r02b_bench_${cfg}_fused.log 2>&1 || { echo "bench $cfg failed"; tail -20 gpurun_out/r02b_bench_${cfg}_fused.log; exit 1; }
  KNN_FILTER_FUSED=0 timeout -k 10 300 $B --config $cfg > gpurun_out/r02b_bench_${cfg}_old.log 2>&1 || { echo "bench $cfg old failed"; exit 1; }
  for v in fused old; do python3 -c "
import json,sys;d=json.loads(open('gpurun_out/r02b_bench_${cfg}_$v.log').read().strip().splitlines()[-1]);r=d['roofline'] or {}
print('$cfg $v', round(d['ms_per_step'],2), d['stages_ms'], r.get('frac'), d['gemm_stats'])"; done
done
timeout -k 10 400 $T --timeout 300 tests/test_gpu_fullsize.py > gpurun_out/r02b_full.log 2>&1 || { echo "fullsize failed"; tail -30 gpurun_out/r02b_full.log; exit 1; }
tail -3 gpurun_out/r02b_full.log
