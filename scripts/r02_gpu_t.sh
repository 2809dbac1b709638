#!/bin/bash
# round 2, pass t: the whole -m gpu suite, then the default bench (A, with CPU baselines and
# host-buffer rates) and B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r02t_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|Error" gpurun_out/r02t_pytest_gpu.log | head; tail -30 gpurun_out/r02t_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r02t_pytest_gpu.log
timeout -k 10 500 python -u bench.py > gpurun_out/r02t_bench_A.log 2>&1 || { echo "bench A failed"; tail -5 gpurun_out/r02t_bench_A.log; exit 1; }
tail -1 gpurun_out/r02t_bench_A.log
timeout -k 10 400 python -u bench.py --config B --steps 3 --no-cpu-baseline > gpurun_out/r02t_bench_B.log 2>&1 || { echo "bench B failed"; tail -5 gpurun_out/r02t_bench_B.log; exit 1; }
tail -1 gpurun_out/r02t_bench_B.log
