#!/bin/bash
# One GPU call: GI_PROF=1 cycle breakdowns (k_stream per bucket, k_body per
# link, k_eval per request + hottest rule links) on C2 and C4 -- stderr.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-prof}
for c in ${CONFIGS:-c2 c4}; do
  echo "== $c $(date +%T)"
  GI_PROF=1 timeout -k 10 300 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline ${ARGS:-} > gpurun_out/${TAG}_prof_${c}_bench.json 2> gpurun_out/${TAG}_prof_${c}.err || { tail -20 gpurun_out/${TAG}_prof_${c}.err; exit 1; }
  grep GI_PROF -A41 gpurun_out/${TAG}_prof_${c}.err | tail -40
done
