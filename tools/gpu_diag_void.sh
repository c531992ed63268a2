#!/bin/bash
# One GPU call: C3 / C4 benches with GI_DIAG=1 -- which phase-A capacity voids
# requests (void events per cause on stderr).  TAG names gpurun_out/<TAG>_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-void}
for c in ${CONFIGS:-c4 c3}; do
  echo "== $c $(date +%T)"
  GI_DIAG=1 timeout -k 10 300 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline ${ARGS:-} > gpurun_out/${TAG}_${c}_bench.json 2> gpurun_out/${TAG}_${c}.err || { tail -20 gpurun_out/${TAG}_${c}.err; exit 1; }
  grep GI_DIAG gpurun_out/${TAG}_${c}.err | tail -3
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${c}_bench.json')); print(d['value'], d['ms_per_step'], d['pa_void_requests'], {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items()})"
done
