#!/bin/bash
# round 3, pass s: per-XCD scan cursor (co-resident blocks start their piece where the XCD's other
# blocks are; the rotation broadcast to the block through LDS), scalar pass-twice detection in the
# lane scan, 12-entry lists for k <= 12 -- parity subset + full-size A/B, same-box filter times vs
# the committed product (nocursor.so) and vs the same build with the cursor off
# (KNN_NO_SCAN_CURSOR=1), and FETCH_SIZE of the B and A filters with the cursor on and off.
set -o pipefail
mkdir -p gpurun_out
P=r03s
L=knn-using-p_threads-and-mpi_amd/build/exp
R=$(pwd)
K="bf16 or synthetic or aligned_rounding or duplicates or shard or golden or stress or this_trees"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_shard.py tests/test_gpu_parity.py tests/test_gpu_host_path.py -q \
  --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${P}_pytest_subset.log 2>&1
rc=$?
echo "subset rc=$rc :: $(tail -1 gpurun_out/${P}_pytest_subset.log)"; grep '^FAILED' gpurun_out/${P}_pytest_subset.log | head
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -q -x --timeout 300 --timeout-method thread > gpurun_out/${P}_full.log 2>&1
rc=$?
echo "fullsize rc=$rc :: $(tail -1 gpurun_out/${P}_full.log)"
[ $rc -ne 0 ] && exit 1
PREFIX=$P STEPS=3 RUNS="A_cur A; A_off A KNN_NO_SCAN_CURSOR=1; A_prev A KNN_AMD_LIB=$L/nocursor.so; B_cur B; B_off B KNN_NO_SCAN_CURSOR=1; B_prev B KNN_AMD_LIB=$L/nocursor.so; C1_cur C1 --nq=131072; C1_prev C1 --nq=131072 KNN_AMD_LIB=$L/nocursor.so; A_cur2 A; A_prev2 A KNN_AMD_LIB=$L/nocursor.so" bash scripts/study.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for v in cur nocur; do
  for cfg in B A; do
    if [ $v = nocur ]; then export KNN_NO_SCAN_CURSOR=1; else unset KNN_NO_SCAN_CURSOR; fi
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${P}_fetch_${cfg}_$v -o run \
      -- python3 $R/bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-host-path > $R/gpurun_out/${P}_fetch_${cfg}_$v.log 2>&1 \
      || { echo "fetch $cfg $v failed"; exit 1; }
    echo "fetch $cfg $v ok"
  done
done
