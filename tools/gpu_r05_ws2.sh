#!/bin/bash
# Stage-2 pending requests on k_eval_wave (GI_EVAL_WAVE_STAGE2) A/B on C4 at 50k, then the PL4 C3-mix parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pl4 or gated or wave" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05ws2_parity.log 2>&1 || { tail -20 gpurun_out/r05ws2_parity.log; exit 1; }
tail -1 gpurun_out/r05ws2_parity.log
for v in 0 1; do
  GI_EVAL_WAVE_STAGE2=$v timeout -k 10 300 python -u bench.py --config c4 --n-req 50000 --steps 3 --warmup 1 --e2e-iters 0 > gpurun_out/r05ws2_c4_$v.json 2> gpurun_out/r05ws2_c4_$v.err || { tail -5 gpurun_out/r05ws2_c4_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05ws2_c4_$v.json')); l=d['roofline']['secondary']['launches']; print('$v', d['value'], d.get('parity_sample',{}).get('mismatches'), {k: round(v['ms'],1) for k, v in l.items() if k.startswith('k_eval')})"
done
