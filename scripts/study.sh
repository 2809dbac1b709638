#!/bin/bash
# Same-box filter study (run via gpurun): bench lines for "tag config [VAR=value ...]" specs
# separated by ';' in $RUNS, then, if $PYTEST_ENV is set, the GPU suite under that env.
#   RUNS="A2 A; A4 A KNN_FILTER_NBUF=4" PYTEST_ENV="KNN_FILTER_NBUF=4" bash scripts/study.sh
set -o pipefail
mkdir -p gpurun_out
P=${PREFIX:-study}
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);s=d['stages_ms']
print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'filter', s.get('gemm_filter'), 'rescore', s.get('rescore'), 'cand/q', (d['select_stage'] or {}).get('candidates_per_query'), 'fb', d['gemm_stats'].get('fallback_queries'))" $1; grep -m1 "filter timing" $1 || true; }
IFS=';' read -ra SPECS <<< "$RUNS"
for spec in "${SPECS[@]}"; do
  read -ra W <<< "$spec"
  [ ${#W[@]} -lt 2 ] && continue
  tag=${W[0]}; cfg=${W[1]}
  EV=(); AR=()
  for w in "${W[@]:2}"; do if [[ $w == --* ]]; then AR+=("$w"); else EV+=("$w"); fi; done
  env "${EV[@]}" timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-host-path "${AR[@]}" > gpurun_out/${P}_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/${P}_$tag.log; exit 1; }
  summ gpurun_out/${P}_$tag.log
done
if [ -n "$PYTEST_ENV" ]; then
  env $PYTEST_ENV timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${P}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${P}_pytest.log; exit 1; }
  tail -1 gpurun_out/${P}_pytest.log
fi
echo done
