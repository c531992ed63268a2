#!/bin/bash
# Round-6 A/B: optional first tests, then C2 bench lines with env settings A and B
# (AB_A / AB_B: env assignments, e.g. "GI_EVAL_ORDER=0"), no CPU baseline / parity leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06ab}
if [ -n "${FIRST:-}" ]; then
  timeout -k 10 400 python -u -m pytest $FIRST ${FIRST_K:+-k "$FIRST_K"} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_first.log 2>&1 || { tail -40 gpurun_out/${TAG}_first.log; exit 1; }
  tail -1 gpurun_out/${TAG}_first.log
fi
for v in A B; do
  envs=$([ $v = A ] && echo "${AB_A:-}" || echo "${AB_B:-}")
  for c in ${CONFIGS:-c2}; do
    echo "== $v ($envs) $c $(date +%T)"
    env $envs timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --e2e-iters 0 > gpurun_out/${TAG}_${v}_${c}.json 2> gpurun_out/${TAG}_${v}_${c}.err || { tail -20 gpurun_out/${TAG}_${v}_${c}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${v}_${c}.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items() if v['ms'] > 0.3})"
  done
done
