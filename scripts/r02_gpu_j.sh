#!/bin/bash
# round 2, pass j: RCCL comm (nranks=1), drop-in reference drivers, mpi_driver sha, build id;
# then bench A with the full CPU baseline (pthreads -O0, -O2, MPI)
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout-method thread"
timeout -k 10 600 $T --timeout 240 tests/test_gpu_bf16_shard.py tests/test_dropin.py tests/test_mpi_driver.py tests/test_gpu_host_path.py -m gpu > gpurun_out/r02j_pytest.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|Error" gpurun_out/r02j_pytest.log | head; tail -30 gpurun_out/r02j_pytest.log; exit 1; }
tail -1 gpurun_out/r02j_pytest.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/r02j_bench_A.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r02j_bench_A.log; exit 1; }
tail -1 gpurun_out/r02j_bench_A.log
