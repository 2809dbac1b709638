#!/bin/bash
# round 2, pass z: smoke, the whole -m gpu suite, the default bench (A, with CPU baselines and
# host-buffer rates) and B, then rocprofv3 summaries (trace + FETCH/WRITE/SQ passes) of A and B
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r02z}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|Error" gpurun_out/${T}_pytest_gpu.log | head; tail -30 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.log
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench_A.log 2>&1 || { echo "bench A failed"; tail -5 gpurun_out/${T}_bench_A.log; exit 1; }
tail -1 gpurun_out/${T}_bench_A.log | cut -c1-400
timeout -k 10 400 python -u bench.py --config B --steps 3 --no-cpu-baseline > gpurun_out/${T}_bench_B.log 2>&1 || { echo "bench B failed"; tail -5 gpurun_out/${T}_bench_B.log; exit 1; }
tail -1 gpurun_out/${T}_bench_B.log | cut -c1-300
STEPS=3 bash scripts/profile_bench.sh || exit 1
rm -rf gpurun_out/${T}_A && mkdir -p gpurun_out/${T}_A && mv gpurun_out/prof_* gpurun_out/${T}_A/
STEPS=2 BENCH_ARGS="--config B" bash scripts/profile_bench.sh || exit 1
rm -rf gpurun_out/${T}_B && mkdir -p gpurun_out/${T}_B && mv gpurun_out/prof_* gpurun_out/${T}_B/
echo done
