#!/bin/bash
# k_scan unit order A/B (GI_SCAN_MODE=32: job-major) on C2, then a parity spot check.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in 32 0 32 0; do
  GI_SCAN_MODE=$m timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --e2e-iters 0 --no-cpu-baseline > gpurun_out/r05scan_$m.json 2> gpurun_out/r05scan_$m.err || { tail -5 gpurun_out/r05scan_$m.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05scan_$m.json')); l=d['roofline']['secondary']['launches']; print('mode $m', d['value'], {k: round(v['ms'],2) for k, v in l.items() if k.startswith('k_scan')})"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "crs" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05scan_parity.log 2>&1 || { tail -20 gpurun_out/r05scan_parity.log; exit 1; }
tail -1 gpurun_out/r05scan_parity.log
