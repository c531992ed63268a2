#!/bin/bash
# One GPU call per iteration: GPU parity tests, then the C2 bench (with the
# oracle parity sample) and C4 / C3 benches with GI_DIAG=1 (phase-A void
# causes on stderr).  TAG names gpurun_out/<TAG>_*; TESTS=0 skips pytest.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-it}
step() { echo "== $1 $(date +%T)"; }
if [ "${TESTS:-1}" = "1" ]; then
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYARGS:-} > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
fi
for c in ${CONFIGS:-c2 c4 c3}; do
  step $c
  ex="--no-cpu-baseline"; [ "$c" = "c2" ] && ex=""; [ "${PARITY_ALL:-0}" = "1" ] && ex=""
  GI_DIAG=1 timeout -k 10 400 python -u bench.py --config $c --steps ${STEPS:-3} --warmup 1 $ex ${ARGS:-} > gpurun_out/${TAG}_${c}_bench.json 2> gpurun_out/${TAG}_${c}.err || { tail -20 gpurun_out/${TAG}_${c}.err; exit 1; }
  grep GI_DIAG gpurun_out/${TAG}_${c}.err | tail -2
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${c}_bench.json')); print(d['value'], d['ms_per_step'], 'void', d['pa_void_requests'], 'parity', d.get('parity_sample',{}).get('mismatches'), {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items()})"
done
