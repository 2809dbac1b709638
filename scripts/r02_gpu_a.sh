#!/bin/bash
# round 2, first GPU pass: tiled direct path parity + full-size A/B parity + direct bench
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout-method thread"
timeout -k 10 500 $T --timeout 240 tests/test_gpu_direct.py tests/test_gpu_parity.py > gpurun_out/r02a_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r02a_pytest.log; exit 1; }
tail -3 gpurun_out/r02a_pytest.log
timeout -k 10 200 python -u bench.py --algo direct --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02a_bench_direct.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r02a_bench_direct.log; exit 1; }
tail -1 gpurun_out/r02a_bench_direct.log | cut -c1-600
timeout -k 10 400 $T --timeout 300 tests/test_gpu_fullsize.py > gpurun_out/r02a_full.log 2>&1 || { echo "fullsize failed"; tail -30 gpurun_out/r02a_full.log; exit 1; }
tail -5 gpurun_out/r02a_full.log
