#!/bin/bash
# One GPU call: the C3 / C4 / C5 bench lines (no CPU baseline).  TAG names the outputs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-cfg}
for c in c3 c4 c5; do
  echo "== $c $(date +%T)"
  timeout -k 10 500 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_${c}_bench.json 2> gpurun_out/${TAG}_${c}.err || { tail -20 gpurun_out/${TAG}_${c}.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${c}_bench.json')); print(d['value'], d['ms_per_step'], d['gb_per_s_scanned'], d['roofline']['kernel'], d['roofline']['frac'])"
done
