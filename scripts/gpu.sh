#!/bin/bash
# The one GPU-box driver (run through gpurun).  Steps, in this order, each optional, each under
# its own time limit; the chain stops at the first failure (no GPU step after a failed one):
#
#   RUNS="tag cfg [VAR=v ...] [--flag=v ...]; ..."
#                      same-box bench lines: one bench.py run per spec, its summary printed
#                      (step, filter, rescore, candidates per query); STEPS / WARMUP per run
#   STAMPS=<variant>   scripts/stamps.py on build/study/libknn_amd_<variant>.so (a -DKNN_STUDY_STAMPS build)
#   TESTS=1            the whole -m gpu suite (PYTEST_K narrows it, PYTEST_ENV="VAR=v ..." sets env;
#                      TESTS_ALT_ENV="VAR=v ..." runs it a second time under that env)
#   BENCHES="A L B"    full bench lines (default steps, CPU baselines on) -> gpurun_out/${TAG}_bench_<cfg>.log
#   PROFILE="A B C1"   rocprofv3 trace + FETCH/WRITE/SQ passes per workload (scripts/profile_bench.sh),
#                      outputs gpurun_out/${TAG}_<cfg>_{trace,fetch,write,sq}
#   SMOKE=1            __graft_entry__.smoke()
#
#   TAG=r04a RUNS="A0 A KNN_SEED_ROWS=0; A1 A KNN_SEED_ROWS=1024" TESTS=1 bash scripts/gpu.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-run}
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);s=d['stages_ms']
sel=d.get('select_stage') or {}
print(sys.argv[1].split('/')[-1], 'value %.4g'%d['value'], 'step', round(d['ms_per_step'],3), 'filter', s.get('gemm_filter'), 'rescore', s.get('rescore'),
      'norms', s.get('norms'), 'aug', s.get('aug'), 'init', s.get('filter_init'), 'cand/q', sel.get('candidates_per_query'),
      'fb', d['gemm_stats'].get('fallback_queries'), 'seg', d['gemm_stats'].get('train_segments'), 'frac', (d.get('roofline') or {}).get('frac'), 'sel_frac', sel.get('frac'))" $1; }

IFS=';' read -ra SPECS <<< "$RUNS"
for spec in "${SPECS[@]}"; do
  read -ra W <<< "$spec"
  [ ${#W[@]} -lt 2 ] && continue
  tag=${W[0]}; cfg=${W[1]}
  EV=(); AR=()
  for w in "${W[@]:2}"; do if [[ $w == --* ]]; then AR+=("$w"); else EV+=("$w"); fi; done
  env "${EV[@]}" timeout -k 10 400 python -u bench.py --config $cfg --steps ${STEPS:-3} --warmup ${WARMUP:-1} \
      --no-cpu-baseline --no-host-path --no-bit-match --no-uncached "${AR[@]}" > gpurun_out/${TAG}_$tag.log 2>&1 \
      || { echo "bench $tag failed"; tail -5 gpurun_out/${TAG}_$tag.log; exit 1; }
  summ gpurun_out/${TAG}_$tag.log
done

if [ -n "$STAMPS" ]; then  # per-wave cycle split of the filter (study build, scripts/build_variant.sh)
  KNN_AMD_LIB=$R/knn-using-p_threads-and-mpi_amd/build/study/libknn_amd_$STAMPS.so timeout -k 10 400 \
      python -u scripts/stamps.py > gpurun_out/${TAG}_stamps.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/${TAG}_stamps.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${TAG}_stamps.log
fi

if [ "$TESTS" = 1 ]; then
  env $PYTEST_ENV timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
      || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest_gpu.log
  if [ -n "$TESTS_ALT_ENV" ]; then  # the suite once more under another study switch
    env $TESTS_ALT_ENV timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_pytest_gpu_alt.log 2>&1 \
        || { echo "pytest (alt) failed"; tail -30 gpurun_out/${TAG}_pytest_gpu_alt.log; exit 1; }
    tail -1 gpurun_out/${TAG}_pytest_gpu_alt.log
  fi
fi

for cfg in $BENCHES; do
  extra=""
  timeout -k 10 600 python -u bench.py --config $cfg $extra > gpurun_out/${TAG}_bench_$cfg.log 2>&1 \
      || { echo "bench $cfg failed"; tail -5 gpurun_out/${TAG}_bench_$cfg.log; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/${TAG}_bench_$cfg.log | cut -c1-300)"
done

for cfg in $PROFILE; do
  st=2; [ "$cfg" != A ] && st=1; [ "$cfg" = L ] && st=50
  tst=$st; [ "$cfg" = A ] && tst=100; [ "$cfg" = B ] && tst=5; [ "$cfg" = L ] && tst=300
  TRACE_STEPS=$tst STEPS=$st PROF_TAG=${TAG}_$cfg BENCH_ARGS="--config $cfg ${PROFILE_ARGS:-}" bash scripts/profile_bench.sh || exit 1
done

if [ "$SMOKE" = 1 ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
      || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -2 gpurun_out/${TAG}_smoke.log
fi
echo done
