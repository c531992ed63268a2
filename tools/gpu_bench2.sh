#!/bin/bash
# C2 bench twice in one call (box-to-box variance check), plus an optional test subset first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-b2}
if [ -n "${FIRST:-}" ]; then
  timeout -k 10 300 python -u -m pytest $FIRST ${FIRST_K:+-k "$FIRST_K"} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_first.log 2>&1 || { tail -40 gpurun_out/${TAG}_first.log; exit 1; }
  tail -1 gpurun_out/${TAG}_first.log
fi
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-iters 0 > gpurun_out/${TAG}_run$i.json 2> gpurun_out/${TAG}_run$i.err || { tail -20 gpurun_out/${TAG}_run$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_run$i.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items() if v['ms'] > 0.5})"
done
