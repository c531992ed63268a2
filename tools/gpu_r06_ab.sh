#!/bin/bash
# Round-6 A/B: optional first tests, then C2 bench lines for each env variant
# (VARIANTS: ';'-separated env assignment lists, e.g. "GI_EVAL_ORDER=0;GI_EVAL_ORDER=1"),
# no CPU baseline / parity leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06ab}
if [ -n "${FIRST:-}" ]; then
  timeout -k 10 400 python -u -m pytest $FIRST ${FIRST_K:+-k "$FIRST_K"} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_first.log 2>&1 || { tail -40 gpurun_out/${TAG}_first.log; exit 1; }
  tail -1 gpurun_out/${TAG}_first.log
fi
IFS=';' read -ra VS <<< "${VARIANTS:-}"
i=0
for envs in "${VS[@]}"; do
  i=$((i+1))
  for c in ${CONFIGS:-c2}; do
    echo "== v$i ($envs) $c $(date +%T)"
    env $envs timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --e2e-iters 0 ${BENCH_ARGS:-} > gpurun_out/${TAG}_v${i}_${c}.json 2> gpurun_out/${TAG}_v${i}_${c}.err || { tail -20 gpurun_out/${TAG}_v${i}_${c}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_v${i}_${c}.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items() if v['ms'] > 0.3})"
  done
done
