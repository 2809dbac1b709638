#!/bin/bash
# round 3, final pass 1: the product as committed -- the whole GPU suite, smoke(), and the bench
# lines: A as the driver runs it (20 steps, 5 warmup, CPU baseline, host-buffer path), B, C1
# (with its CPU baseline at d = 256, k = 100).
set -o pipefail
mkdir -p gpurun_out
P=${PREFIX:-r03z}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread --durations=15 \
  > gpurun_out/${P}_pytest_gpu.log 2>&1
rc=$?
echo "suite rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_gpu.log)"; grep -E '^FAILED|^ERROR' gpurun_out/${P}_pytest_gpu.log | head
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/${P}_smoke.log; exit 1; }
tail -1 gpurun_out/${P}_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${P}_bench_A.log 2>&1 || { echo "bench A failed"; tail -5 gpurun_out/${P}_bench_A.log; exit 1; }
echo "A: $(tail -1 gpurun_out/${P}_bench_A.log | cut -c1-400)"
timeout -k 10 400 python -u bench.py --config B --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/${P}_bench_B.log 2>&1 || { echo "bench B failed"; tail -5 gpurun_out/${P}_bench_B.log; exit 1; }
echo "B: $(tail -1 gpurun_out/${P}_bench_B.log | cut -c1-400)"
timeout -k 10 500 python -u bench.py --config C1 --steps 2 --warmup 1 > gpurun_out/${P}_bench_C1.log 2>&1 || { echo "bench C1 failed"; tail -5 gpurun_out/${P}_bench_C1.log; exit 1; }
echo "C1: $(tail -1 gpurun_out/${P}_bench_C1.log | cut -c1-400)"
