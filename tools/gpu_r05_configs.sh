#!/bin/bash
# Round-5 GPU step: C2 A/B of k_eval variants (tools/ab_build.sh; VARIANTS),
# then C3 / C4 / C5 with the phase-1 gate on (and C3/C4 with GI_GATE=0 when
# NOGATE=1).  TAG names gpurun_out/<TAG>_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05b}
if [ -n "${VARIANTS:-}" ]; then
  VARIANTS="$VARIANTS" STEPS=10 bash tools/ab_bench.sh || exit 1
fi
for c in ${CONFIGS:-c3 c4 c5}; do
  echo "== $c $(date +%T)"
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --e2e-iters 0 > gpurun_out/${TAG}_${c}_bench.json 2> gpurun_out/${TAG}_${c}.err || { tail -20 gpurun_out/${TAG}_${c}.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${c}_bench.json')); print(d['value'], d['ms_per_step'], d.get('gb_per_s_scanned'), d.get('parity_sample',{}).get('mismatches'), {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items() if v['ms'] > 2})"
done
if [ "${NOGATE:-0}" = "1" ]; then
  for c in c3 c4; do
    echo "== $c nogate $(date +%T)"
    GI_GATE=0 timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --e2e-iters 0 --no-cpu-baseline > gpurun_out/${TAG}_${c}_nogate_bench.json 2> gpurun_out/${TAG}_${c}_nogate.err || { tail -20 gpurun_out/${TAG}_${c}_nogate.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${c}_nogate_bench.json')); print(d['value'], d['ms_per_step'], d.get('parity_sample',{}).get('mismatches'))"
  done
fi
echo done
