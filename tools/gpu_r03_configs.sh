#!/bin/bash
# One GPU call: the C3 / C4 / C5 bench lines with their oracle parity samples.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
for c in ${CONFIGS:-c3 c4 c5}; do
  echo "== $c $(date +%T)"
  timeout -k 10 420 python -u bench.py --config $c --steps 3 --warmup 1 --e2e-iters 0 > gpurun_out/${TAG}_${c}_bench.json 2> gpurun_out/${TAG}_${c}.err || { tail -20 gpurun_out/${TAG}_${c}.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${c}_bench.json')); print(d['value'], d['gb_per_s_scanned'], d['ms_per_step'], d['config']['requests_per_gpu'], d['pa_void_requests'], d.get('parity_sample',{}).get('n'), d.get('parity_sample',{}).get('mismatches'))"
done
