#!/bin/bash
# Profile bench.py (workload A, or BENCH_ARGS="--config C1 ...") on one MI355X (run on the GPU box via gpurun):
#   1. rocprofv3 --kernel-trace --stats           -> per-kernel average durations
#   2. rocprofv3 --pmc FETCH_SIZE                 -> HBM read bytes   (own pass)
#   3. rocprofv3 --pmc WRITE_SIZE                 -> HBM write bytes  (own pass)
#   4. rocprofv3 --pmc SQ_* / GRBM_GUI_ACTIVE     -> MFMA busy, waits, clock (own pass)
#   5. rocprofv3 --pmc SQ_*LDS* ...               -> LDS instructions, array-busy cycles (own pass)
# Outputs land in gpurun_out/prof_*; scripts/summarize_profile.py turns them into
# profiles/<tag>_*.{csv,json}.  Every pass runs under its own time limit and the chain
# stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
STEPS=${STEPS:-2}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out
PT=${PROF_TAG:-prof}   # output dirs $OUT/${PT}_{trace,fetch,write,sq}
BENCH="$R/bench.py --steps $STEPS --warmup 1 --no-cpu-baseline --no-host-path --no-bit-match --no-uncached ${BENCH_ARGS:-}"

# (the trace pass runs TRACE_STEPS timed steps: a 2-step run averages the first launches, whose clock
# differs -- A: 20.15 ms over 2 steps, 19.19 ms over 100 against the bench's 19.2-19.5 by events, r06x)
TBENCH="$R/bench.py --steps ${TRACE_STEPS:-$STEPS} --warmup 1 --no-cpu-baseline --no-host-path --no-bit-match --no-uncached ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${PT}_trace -o run \
    -- python3 $TBENCH > $OUT/${PT}_trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
echo "trace pass ok"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${PT}_fetch -o run \
    -- python3 $BENCH > $OUT/${PT}_fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
echo "fetch pass ok"
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${PT}_write -o run \
    -- python3 $BENCH > $OUT/${PT}_write.log 2>&1 || { echo "write pass failed"; exit 1; }
echo "write pass ok"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/${PT}_sq -o run \
    -- python3 $BENCH > $OUT/${PT}_sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
echo "sq pass ok"
# LDS / instruction-mix pass (the filter's LDS load: reads per MFMA, array-busy cycles, waits)
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/${PT}_lds -o run \
    -- python3 $BENCH > $OUT/${PT}_lds.log 2>&1 || { echo "lds pass failed"; exit 1; }
echo "lds pass ok"
