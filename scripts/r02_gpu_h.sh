#!/bin/bash
# round 2, pass h: device-side gates (no in-call host syncs) + compacted rescore
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 600 $T --timeout 240 tests/test_gpu_parity.py tests/test_gpu_direct.py tests/test_gpu_bf16_shard.py tests/test_gpu_mfma_cert.py > gpurun_out/r02h_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|Error" gpurun_out/r02h_pytest.log | head; tail -30 gpurun_out/r02h_pytest.log; exit 1; }
tail -1 gpurun_out/r02h_pytest.log
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for cfg in A B; do
  timeout -k 10 300 $B --config $cfg > gpurun_out/r02h_bench_$cfg.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/r02h_bench_$cfg.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/r02h_bench_$cfg.log').read().strip().splitlines()[-1]);print('$cfg', round(d['ms_per_step'],2), d['stages_ms'], (d['select_stage'] or {}).get('frac'), d['roofline']['frac'])"
done
timeout -k 10 400 $T --timeout 300 tests/test_gpu_fullsize.py > gpurun_out/r02h_full.log 2>&1 || { echo "fullsize failed"; tail -30 gpurun_out/r02h_full.log; exit 1; }
tail -1 gpurun_out/r02h_full.log
