#!/bin/bash
# Sweep of the gate's first-stage budget (GI_PREFIX_BUDGET) on C4 and C3
# (bench without the CPU baseline), plus GI_GATE=0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05d}
for c in ${CONFIGS:-c4 c3}; do
  for b in ${BUDGETS:-0 4 16 64}; do
    echo "== $c budget $b $(date +%T)"
    GI_PREFIX_BUDGET=$b timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --e2e-iters 0 --no-cpu-baseline > gpurun_out/${TAG}_${c}_b${b}.json 2> gpurun_out/${TAG}_${c}_b${b}.err || { tail -20 gpurun_out/${TAG}_${c}_b${b}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${c}_b${b}.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items() if v['ms'] > 10})"
  done
done
echo done
