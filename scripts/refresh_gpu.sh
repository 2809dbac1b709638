#!/bin/bash
# Full GPU refresh (run on the GPU box via gpurun): the whole -m gpu suite, then the bench
# lines (A default with the CPU baseline, L = large ARFF, optional extra configs).
# Each step under its own limit; the chain stops at the first failure.
set -o pipefail
TAG=${TAG:-r01h}
[ "$SKIP_TESTS" = 1 ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
[ "$SKIP_TESTS" = 1 ] || tail -1 gpurun_out/${TAG}_pytest_gpu.log
for cfg in ${BENCHES:-A L}; do
  extra=""; [ "$cfg" = B ] && extra="--steps 1 --no-cpu-baseline"; [ "$cfg" = L ] && extra="--steps 50 --warmup 5"
  timeout -k 10 400 python -u bench.py --config $cfg $extra > gpurun_out/${TAG}_bench_$cfg.log 2>&1 \
      || { echo "bench $cfg failed"; tail -5 gpurun_out/${TAG}_bench_$cfg.log; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/${TAG}_bench_$cfg.log | cut -c1-400)"
done
