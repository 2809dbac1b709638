#!/bin/bash
# round 2, pass i: host-buffer path (cache, streamed batches, workspace passes, pinned) + parity
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 300 $T --timeout 120 tests/test_gpu_host_path.py > gpurun_out/r02i_host.log 2>&1 || { echo "host path failed"; tail -40 gpurun_out/r02i_host.log; exit 1; }
tail -1 gpurun_out/r02i_host.log
timeout -k 10 600 $T --timeout 240 tests/test_gpu_parity.py tests/test_gpu_direct.py tests/test_gpu_bf16_shard.py tests/test_gpu_mfma_cert.py tests/test_mpi_driver.py > gpurun_out/r02i_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|Error" gpurun_out/r02i_pytest.log | head; tail -30 gpurun_out/r02i_pytest.log; exit 1; }
tail -1 gpurun_out/r02i_pytest.log
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for cfg in A B; do
  timeout -k 10 300 $B --config $cfg > gpurun_out/r02i_bench_$cfg.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/r02i_bench_$cfg.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/r02i_bench_$cfg.log').read().strip().splitlines()[-1]);print('$cfg', round(d['ms_per_step'],2), d['stages_ms'].get('gemm_filter'), d['stages_ms'].get('rescore'), (d['select_stage'] or {}).get('frac'), d['roofline']['frac'])"
done
