#!/bin/bash
# quick GPU iteration: parity subset + bench lines (run via gpurun)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "${PYTEST_K:-bf16 or synthetic or shard or duplicates}" > gpurun_out/q_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -1 gpurun_out/q_pytest.log
for cfg in ${BENCHES:---config=A}; do
  [ "$cfg" = none ] && continue
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 $cfg > gpurun_out/q_bench.log 2>&1 || { echo "bench failed $cfg"; tail -5 gpurun_out/q_bench.log; exit 1; }
  echo "$cfg :: $(tail -1 gpurun_out/q_bench.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["stages_ms"], r["roofline"]["frac"])')"
done
