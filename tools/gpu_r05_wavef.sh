#!/bin/bash
# k_eval_wave field threshold A/B (GI_EVAL_WAVE_FIELDS) on C4 and C3 at 50k requests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CFGS:-c4 c3}; do
  for v in ${VALS:-4096 1024 256}; do
    GI_EVAL_WAVE_FIELDS=$v timeout -k 10 300 python -u bench.py --config $c --n-req 50000 --steps 3 --warmup 1 --e2e-iters 0 --no-cpu-baseline > gpurun_out/r05wf_${c}_$v.json 2> gpurun_out/r05wf_${c}_$v.err || { tail -5 gpurun_out/r05wf_${c}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r05wf_${c}_$v.json')); l=d['roofline']['secondary']['launches']; print('$c', '$v', d['value'], d['parity_sample']['mismatches'], {k: round(v['ms'],1) for k, v in l.items() if k.startswith('k_eval')})"
  done
done
