#!/bin/bash
# Regex stress: GPU parity (tests/test_rxstress.py), the c2x bench line, and the default C2 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05rx}
echo "== parity $(date +%T)"
timeout -k 10 500 python -u -m pytest tests/test_rxstress.py ${EXTRA_TESTS:-} -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_parity.log 2>&1 || { tail -30 gpurun_out/${TAG}_parity.log; exit 1; }
tail -1 gpurun_out/${TAG}_parity.log
echo "== c2x $(date +%T)"
timeout -k 10 400 python -u bench.py --config c2x --steps 5 --warmup 1 --e2e-iters 0 > gpurun_out/${TAG}_c2x_bench.json 2> gpurun_out/${TAG}_c2x.err || { tail -20 gpurun_out/${TAG}_c2x.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c2x_bench.json')); print(d['value'], d['ms_per_step'], d.get('parity_sample',{}).get('mismatches'), {k: round(v['ms'],2) for k, v in d['roofline']['secondary']['launches'].items() if v['ms'] > 0.5})"
if [ "${C2:-1}" = "1" ]; then
  echo "== c2 $(date +%T)"
  timeout -k 10 400 python -u bench.py --e2e-iters 0 > gpurun_out/${TAG}_c2_bench.json 2> gpurun_out/${TAG}_c2.err || { tail -20 gpurun_out/${TAG}_c2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_bench.json')); print(d['value'], d['ms_per_step'], d.get('parity_sample',{}).get('mismatches'), {k: round(v['ms'],2) for k, v in d['roofline']['secondary']['launches'].items() if v['ms'] > 0.5})"
fi
echo done
