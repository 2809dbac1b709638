#!/bin/bash
# round 2, pass c: fused filter vs the previous bf16 filter on A and B, phase clocks, parity
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout-method thread"
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
A=knn-using-p_threads-and-mpi_amd/build/ablate
for cfg in A B; do
  for v in fused old; do
    if [ $v = old ]; then E="KNN_FILTER_FUSED=0"; else E=""; fi
    env $E timeout -k 10 300 $B --config $cfg > gpurun_out/r02c_bench_${cfg}_$v.log 2>&1 || { echo "bench $cfg $v failed"; tail -20 gpurun_out/r02c_bench_${cfg}_$v.log; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/r02c_bench_${cfg}_$v.log').read().strip().splitlines()[-1]);r=d['roofline'] or {}
print('$cfg $v', round(d['ms_per_step'],2), d['stages_ms'].get('gemm_filter'), r.get('frac'), d['gemm_stats']['candidates'], d['gemm_stats']['train_segments'])"
  done
done
for v in timing noslow; do
  env KNN_AMD_LIB=$PWD/$A/libknn_amd_$v.so KNN_FILTER_TIMING=1 timeout -k 10 300 $B --config A > gpurun_out/r02c_abl_A_$v.log 2>&1 || { echo "abl $v failed"; tail -5 gpurun_out/r02c_abl_A_$v.log; exit 1; }
  echo "A $v $(grep -o '"gemm_filter": [0-9.]*' gpurun_out/r02c_abl_A_$v.log) $(grep -m1 'knn filter timing' gpurun_out/r02c_abl_A_$v.log)"
done
timeout -k 10 600 $T --timeout 240 tests/test_gpu_parity.py tests/test_gpu_mfma_cert.py tests/test_gpu_bf16_shard.py > gpurun_out/r02c_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r02c_pytest.log; exit 1; }
tail -2 gpurun_out/r02c_pytest.log
timeout -k 10 400 $T --timeout 300 tests/test_gpu_fullsize.py > gpurun_out/r02c_full.log 2>&1 || { echo "fullsize failed"; tail -30 gpurun_out/r02c_full.log; exit 1; }
tail -2 gpurun_out/r02c_full.log
