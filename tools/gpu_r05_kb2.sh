#!/bin/bash
# k_body split over the gate's stages: parity (PL4 C3 mix, body chunks, SecLang surface), then C4 / C3 at 50k.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_body_chunks.py tests/test_seclang_surface.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05kb2_parity.log 2>&1 || { tail -20 gpurun_out/r05kb2_parity.log; exit 1; }
tail -1 gpurun_out/r05kb2_parity.log
for c in c4 c3; do
  timeout -k 10 300 python -u bench.py --config $c --n-req 50000 --steps 3 --warmup 1 --e2e-iters 0 > gpurun_out/r05kb2_$c.json 2> gpurun_out/r05kb2_$c.err || { tail -5 gpurun_out/r05kb2_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05kb2_$c.json')); l=d['roofline']['secondary']['launches']; print('$c', d['value'], d.get('parity_sample',{}).get('mismatches'), d.get('gate'), {k: round(v['ms'],1) for k, v in l.items() if v['ms'] > 3})"
done
