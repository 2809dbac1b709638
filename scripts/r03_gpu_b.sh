#!/bin/bash
# round 3, pass b: config C at size first (progress on stderr), then the rest of the GPU
# suite verbosely, then the relaxed-schedule study on the padded tree.
set -o pipefail
mkdir -p gpurun_out
L=knn-using-p_threads-and-mpi_amd/build/exp
timeout -k 10 300 python -u -c "import time; t=time.time(); import torch; print('torch import', round(time.time()-t,1), 's', torch.cuda.is_available(), flush=True)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_config_c.py -m gpu -v --timeout 500 --timeout-method thread -s --durations=5 > gpurun_out/r03b_config_c.log 2>&1
rc=$?
echo "config C rc=$rc"; tail -12 gpurun_out/r03b_config_c.log
[ $rc -gt 1 ] && exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread --durations=15 --deselect tests/test_gpu_config_c.py > gpurun_out/r03b_pytest_gpu.log 2>&1
rc=$?
echo "product suite rc=$rc :: $(tail -1 gpurun_out/r03b_pytest_gpu.log)"; grep -E '^FAILED|^ERROR' gpurun_out/r03b_pytest_gpu.log | head
[ $rc -gt 1 ] && exit 1
K="bf16_grid or bf16_random or synthetic_vs or aligned_rounding or duplicates or train_sharded_matches"
KNN_AMD_LIB=$L/nosb_pad.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py -v \
  --timeout 200 --timeout-method thread -k "$K" > gpurun_out/r03b_pytest_nosb_pad.log 2>&1
rc=$?
echo "nosb_pad rc=$rc :: $(tail -1 gpurun_out/r03b_pytest_nosb_pad.log)"; grep '^FAILED' gpurun_out/r03b_pytest_nosb_pad.log | head
[ $rc -gt 1 ] && exit 1
KNN_AMD_LIB=$L/nosb_pad.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -v -x --timeout 300 --timeout-method thread > gpurun_out/r03b_full_nosb_pad.log 2>&1
rc=$?
echo "fullsize nosb_pad rc=$rc :: $(tail -1 gpurun_out/r03b_full_nosb_pad.log)"
[ $rc -gt 1 ] && exit 1
PREFIX=r03b STEPS=3 RUNS="A_strict A; A_relax A KNN_AMD_LIB=$L/nosb_pad.so; B_strict B; B_relax B KNN_AMD_LIB=$L/nosb_pad.so; A_strict2 A" bash scripts/study.sh
