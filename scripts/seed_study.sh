#!/bin/bash
# GPU tests, then the filter with and without the seeded thresholds on one box (run via gpurun)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/seed_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/seed_pytest.log; exit 1; }
tail -1 gpurun_out/seed_pytest.log
for run in ${RUNS:-A:1 A:0 B:1 B:0 C1:1 C1:0 A:1 A:0}; do
  IFS=: read cfg sd <<< "$run"
  extra=""; [ "$cfg" = C1 ] && extra="--nq 250000"
  KNN_FILTER_SEED=$sd timeout -k 10 300 python -u bench.py --config $cfg $extra --steps 2 --warmup 1 --no-cpu-baseline \
      > gpurun_out/seed_$cfg.log 2>&1 || { echo "fail $run"; tail -3 gpurun_out/seed_$cfg.log; exit 1; }
  echo "$run $(tail -1 gpurun_out/seed_$cfg.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print("%.4g" % r["value"], r["stages_ms"], r["gemm_stats"]["candidates"], r["gemm_stats"]["fallback_queries"])')"
done
