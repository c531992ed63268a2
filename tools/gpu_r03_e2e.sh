#!/bin/bash
# One GPU call: GPU parity tests, the tally fixture (tools/record_tally.py),
# the default bench (with the pipelined e2e leg).  TAG names gpurun_out/<TAG>_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-e2e}
step() { echo "== $1 $(date +%T)"; }
if [ "${TESTS:-1}" = "1" ]; then
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
fi
step tally
timeout -k 10 300 python -u tools/record_tally.py --out gpurun_out/tally_crs_pl1_world2.json > gpurun_out/${TAG}_tally.log 2>&1 || { tail -20 gpurun_out/${TAG}_tally.log; exit 1; }
tail -1 gpurun_out/${TAG}_tally.log
step bench
timeout -k 10 500 python -u bench.py ${ARGS:-} > gpurun_out/${TAG}_c2_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_bench.json')); print(d['value'], d['ms_per_step'], d.get('parity_sample',{}).get('mismatches'), json.dumps(d['e2e']))"
