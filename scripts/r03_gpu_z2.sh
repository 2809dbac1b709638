#!/bin/bash
# round 3, final pass 2: rocprofv3 kernel trace + PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) of the
# A, B and C1 bench workloads (scripts/profile_bench.sh; summaries by summarize_profile.py).
set -o pipefail
mkdir -p gpurun_out
P=${PREFIX:-r03z}
STEPS=2 PROF_TAG=${P}_A BENCH_ARGS="--config A" bash scripts/profile_bench.sh || exit 1
STEPS=1 PROF_TAG=${P}_B BENCH_ARGS="--config B" bash scripts/profile_bench.sh || exit 1
STEPS=1 PROF_TAG=${P}_C1 BENCH_ARGS="--config C1" bash scripts/profile_bench.sh || exit 1
echo done
