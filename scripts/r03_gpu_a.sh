#!/bin/bash
# round 3, pass a: the product's GPU suite (padded train tiles, DPP/swizzle lane exchanges,
# sorted-run merges, config C at size), then the in-step LDS-DMA hazard: the relaxed schedule
# (no per-k-step sched_barrier) on the padded tree, and same-box filter times strict vs relaxed.
set -o pipefail
mkdir -p gpurun_out
L=knn-using-p_threads-and-mpi_amd/build/exp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread --durations=15 > gpurun_out/r03a_pytest_gpu.log 2>&1
rc=$?
echo "product suite rc=$rc :: $(tail -1 gpurun_out/r03a_pytest_gpu.log)"; grep -E '^FAILED|^ERROR' gpurun_out/r03a_pytest_gpu.log | head
[ $rc -gt 1 ] && exit 1
K="bf16_grid or bf16_random or synthetic_vs or aligned_rounding or duplicates or train_sharded_matches"
KNN_AMD_LIB=$L/nosb_pad.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py -q \
  --timeout 200 --timeout-method thread -k "$K" > gpurun_out/r03a_pytest_nosb_pad.log 2>&1
rc=$?
echo "nosb_pad rc=$rc :: $(tail -1 gpurun_out/r03a_pytest_nosb_pad.log)"; grep '^FAILED' gpurun_out/r03a_pytest_nosb_pad.log | head
[ $rc -gt 1 ] && exit 1
KNN_AMD_LIB=$L/nosb_pad.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r03a_full_nosb_pad.log 2>&1
rc=$?
echo "fullsize nosb_pad rc=$rc :: $(tail -1 gpurun_out/r03a_full_nosb_pad.log)"
[ $rc -gt 1 ] && exit 1
PREFIX=r03a STEPS=3 RUNS="A_strict A; A_relax A KNN_AMD_LIB=$L/nosb_pad.so; B_strict B; B_relax B KNN_AMD_LIB=$L/nosb_pad.so; A_strict2 A" bash scripts/study.sh
