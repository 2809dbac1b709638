#!/bin/bash
# PMC study of k_gemm_filter on one workload (run on the GPU box via gpurun):
#   BENCH_ARGS="--config C1 --nq 64000" bash scripts/pmc_filter.sh
# Each counter set is its own rocprofv3 pass (per-block hardware limits) under its own
# time limit; the chain stops at the first failure.  Outputs: gpurun_out/pmc_<n>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out
ARGS=${BENCH_ARGS:-"--config C1 --nq 64000"}
BENCH="$R/bench.py $ARGS --steps 1 --warmup 0 --no-cpu-baseline"
if [ -n "$LIST" ]; then timeout -s KILL 60 rocprofv3 -L > $OUT/pmc_list.txt 2>&1; fi
i=0
while read -r SET; do
  [ -z "$SET" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/pmc_$i -o run -- python3 $BENCH \
      > $OUT/pmc_$i.log 2>&1 || { echo "pass $i failed: $SET"; exit 1; }
  echo "pass $i ok: $SET"
done <<< "${SETS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
TCC_HIT_sum TCC_MISS_sum}"
