#!/bin/bash
# round 2, pass q: counters of the fused filter on A (one query group, register lists) and B (heaps)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT"
i=0
for cfg in A B; do
  for SET in "$P1" "$P2" "$P3" "FETCH_SIZE"; do
    i=$((i+1))
    E="KNN_FILTER_QG=1 KNN_FILTER_ROTATE=0"; [ $cfg = B ] && E="$E KNN_FILTER_KR=0"
    env $E timeout -s KILL 150 rocprofv3 --pmc $SET --output-format csv -d $R/gpurun_out/r02q_pmc_${cfg}_$i -o run -- python3 $R/bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-host-path > $R/gpurun_out/r02q_pmc_${cfg}_$i.log 2>&1 || { echo "pass $cfg $i failed: $SET"; tail -3 $R/gpurun_out/r02q_pmc_${cfg}_$i.log; exit 1; }
    echo "pass $cfg $i ok"
  done
done
