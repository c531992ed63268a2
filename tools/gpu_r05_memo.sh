#!/bin/bash
# k_detect memo threshold A/B on C2 (1M) and C3 (50k): GI_DET_MEMO_MIN values, and the memo off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VALS:-0 32 64 off}; do
  if [ "$v" = "off" ]; then E="GI_DET_MEMO=0"; else E="GI_DET_MEMO_MIN=$v"; fi
  for c in c2 c3; do
    N=""; [ "$c" = "c3" ] && N="--n-req 50000"
    env $E timeout -k 10 300 python -u bench.py --config $c $N --steps 3 --warmup 1 --e2e-iters 0 --no-cpu-baseline > gpurun_out/r05memo_${c}_$v.json 2> gpurun_out/r05memo_${c}_$v.err || { tail -5 gpurun_out/r05memo_${c}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r05memo_${c}_$v.json')); l=d['roofline']['secondary']['launches']; print('$v', '$c', d['value'], round(l['k_detect']['ms'],2))"
  done
done
