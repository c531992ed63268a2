#!/bin/bash
# C3/C4 with the adaptive gate, and C4 with lower k_eval_wave field thresholds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05j}
run() {  # name config env...
  local n=$1 c=$2; shift 2
  echo "== $n $(date +%T)"
  env "$@" timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --e2e-iters 0 --no-cpu-baseline > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err || { tail -20 gpurun_out/${TAG}_$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_$n.json')); print(d['value'], d['ms_per_step'], d['gate'], {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items() if v['ms'] > 20})"
}
run c4 c4 GI_DUMMY=1
run c3 c3 GI_DUMMY=1
run c4_wf512 c4 GI_EVAL_WAVE_FIELDS=512
run c4_wf128 c4 GI_EVAL_WAVE_FIELDS=128
run c3_wf512 c3 GI_EVAL_WAVE_FIELDS=512
echo done
