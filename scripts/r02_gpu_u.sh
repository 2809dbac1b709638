#!/bin/bash
# round 2, pass u: rocprofv3 summaries of the default bench (A and B) + smoke
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02u_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r02u_smoke.log; exit 1; }
tail -1 gpurun_out/r02u_smoke.log
STEPS=3 bash scripts/profile_bench.sh || exit 1
mkdir -p gpurun_out/r02u_A && mv gpurun_out/prof_* gpurun_out/r02u_A/
STEPS=2 BENCH_ARGS="--config B" bash scripts/profile_bench.sh || exit 1
mkdir -p gpurun_out/r02u_B && mv gpurun_out/prof_* gpurun_out/r02u_B/
echo done
