#!/bin/bash
# k_eval workgroup size A/B on C2 (GI_EVAL_BS 64 / 128), plus the edge-URI test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "edge_uris or crs_pl1_get" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/evalbs_first.log 2>&1 || { tail -30 gpurun_out/evalbs_first.log; exit 1; }
tail -1 gpurun_out/evalbs_first.log
for bs in 128 64; do
  GI_EVAL_BS=$bs timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-iters 0 > gpurun_out/evalbs_$bs.json 2> gpurun_out/evalbs_$bs.err || { tail -20 gpurun_out/evalbs_$bs.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/evalbs_$bs.json')); print($bs, d['value'], d['ms_per_step'], d['roofline']['secondary']['launches']['k_eval']['ms'])"
done
