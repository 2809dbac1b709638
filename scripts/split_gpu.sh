#!/bin/bash
# split-filter iteration: parity (gpu tests of test_gpu_parity.py) + A/B bench lines for
# both GEMM operand types (run via gpurun)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/s_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/s_pytest.log; exit 1; }
tail -1 gpurun_out/s_pytest.log
for run in ${BENCHES:-A:gemm A:gemm_split B:gemm B:gemm_split}; do
  cfg=${run%%:*}; algo=${run##*:}
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps ${STEPS:-3} --warmup 1 --config $cfg --algo $algo \
      > gpurun_out/s_bench_${cfg}_${algo}.log 2>&1 || { echo "bench failed $run"; tail -5 gpurun_out/s_bench_${cfg}_${algo}.log; exit 1; }
  echo "$run :: $(tail -1 gpurun_out/s_bench_${cfg}_${algo}.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print("%.4g" % r["value"], r["stages_ms"], r["roofline"]["frac"], r["gemm_stats"], r["select_stage"]["candidates_per_query"])')"
done
